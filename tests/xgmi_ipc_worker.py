"""Worker for tests/test_xgmi_gpu.py::test_ipc_allreduce_processes: one
rank of XgmiAllReduce. All ranks share cuda:0 (one-GPU box), so this runs
the real multi-process path - HIP IPC handle exchange, peer-mapped buffers,
cross-process release/acquire flags - minus only the xGMI link itself."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LOCAL_RANK"] = "0"          # every rank on cuda:0

import torch  # noqa: E402

from nvidia_terraform_modules_amd.parallel.dist import init, shutdown  # noqa: E402
from nvidia_terraform_modules_amd.parallel.xgmi import XgmiAllReduce  # noqa: E402


def main():
    env = init(backend="gloo", device_type="cuda")
    ar = XgmiAllReduce(env, max_bytes=8 << 20, nblk=16)
    n = env.world_size
    results = []
    for count in (8 * n * 64, 8 * n * 4096 + 8 * n * 5, (8 << 20) // 2):
        i = torch.arange(count, device=env.device)
        t = ((2.0 ** (i % 4)) * (env.rank + 1)).to(torch.bfloat16)
        ar(t)
        torch.cuda.synchronize()
        exp = ((2.0 ** (i % 4)) * (n * (n + 1) / 2)).to(torch.bfloat16)
        results.append({"count": count, "wrong": int((t != exp).sum()),
                        "timeout": ar.timed_out(), "path": "staged"})
    # zero-copy path: payload written straight into the registered buffer,
    # reduced in place; several calls back to back with no host sync between
    for count in (8 * n * 16, 8 * n * 65536, (8 << 20) // 2):
        i = torch.arange(count, device=env.device)
        buf = ar.buffer(count)
        for rep in range(3):
            buf.copy_(((2.0 ** (i % 4)) * (env.rank + 1 + rep)).to(torch.bfloat16))
            ar.run(count)
        torch.cuda.synchronize()
        exp = ((2.0 ** (i % 4)) * (n * (n + 1) / 2 + 2 * n)).to(torch.bfloat16)
        results.append({"count": count, "wrong": int((buf != exp).sum()),
                        "timeout": ar.timed_out(), "path": "in_place"})
    # bench.py's C2 sweep, as it runs at N > 1: all_reduce_sweep with the
    # registered buffer as operand (zero-copy, in place), element check + timing
    from nvidia_terraform_modules_amd.parallel.collectives import all_reduce_sweep
    for r in all_reduce_sweep(env, [512, 2048, 1 << 20], dtype="bf16", iters=3, warmup=1, impl=ar):
        results.append({"count": r.count, "wrong": r.errors, "timeout": ar.timed_out(),
                        "path": "bench_sweep", "busbw_GBps": r.busbw_GBps})
    first = ar.stats()
    ar.close()
    # bench.py's N > 1 C2 block exactly (xgmi.c2_sweep): the knob sweep (nblk x
    # one-shot / two-shot x cutoff) and the main sweep on ONE communicator, each
    # point element-checked; on one GPU only the nblk whose blocks of all ranks
    # are co-resident
    from nvidia_terraform_modules_amd.parallel.xgmi import TUNE_NBLKS, c2_sweep
    nblks = tuple(nb for nb in TUNE_NBLKS if nb * n <= 1024)
    c2, _ = c2_sweep(env, [512, 2048, 1 << 20], 1 << 20, iters=2, warmup=1,
                     tune_kwargs={"sizes": (64 << 10, 1 << 20), "nblks": nblks, "iters": 2,
                                  "warmup": 1})
    tr = c2["xgmi_tune"]
    print(json.dumps({"rank": env.rank, "results": results, "first_comm": first,
                      "c2": {k: v for k, v in c2.items() if k != "xgmi_tune"},
                      "tune": {k: tr[k] for k in ("table", "errors", "timed_out", "best_nblk",
                                                  "shared_communicator")}}), flush=True)
    shutdown(env)


if __name__ == "__main__":
    main()
