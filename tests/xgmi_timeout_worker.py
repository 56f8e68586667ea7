"""Worker for tests/test_xgmi_gpu.py::test_ipc_missing_rank_raises: rank 0
calls XgmiAllReduce with short barrier limits while rank 1 never does, so
rank 0's entry barrier times out; ``check=True`` must raise and the output
rank 0 owns must be NaN (the failure contract of XgmiAllReduce)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LOCAL_RANK"] = "0"          # every rank on cuda:0

import torch  # noqa: E402

from nvidia_terraform_modules_amd.parallel.dist import barrier, init, shutdown  # noqa: E402
from nvidia_terraform_modules_amd.parallel.xgmi import XgmiAllReduce  # noqa: E402


def main():
    env = init(backend="gloo", device_type="cuda")
    # one communicator per algorithm (both set up collectively): the two-shot one
    # with its one-shot cutoff at 0, so the two-shot entry-timeout and poison path
    # really runs (128 KiB is under the default 256 KiB cutoff)
    comms = {False: XgmiAllReduce(env, max_bytes=1 << 20, nblk=8, one_shot_max_bytes=0,
                                  spin_limit=4096, entry_spin_limit=4096),
             True: XgmiAllReduce(env, max_bytes=1 << 20, nblk=8, spin_limit=4096,
                                 entry_spin_limit=4096)}
    rep = {"rank": env.rank}
    if env.rank == 0:
        n = env.world_size
        for one_shot, count in ((False, 8 * n * 4096), (True, 8 * n * 64)):
            ar = comms[one_shot]
            assert (count * 2 <= ar.one_shot_max_bytes) == one_shot
            t = torch.ones(count, dtype=torch.bfloat16, device=env.device)
            try:
                ar(t, check=True)
                rep[f"raised_{int(one_shot)}"] = ""
            except RuntimeError as e:
                rep[f"raised_{int(one_shot)}"] = str(e)
            rep[f"all_nan_{int(one_shot)}"] = bool(torch.isnan(t.float()).all())
        rep["timed_out"] = all(ar.timed_out() for ar in comms.values())
    barrier(env)   # rank 1 never launches; it only waits here
    for ar in comms.values():
        ar.close()
    print(json.dumps(rep), flush=True)
    shutdown(env)


if __name__ == "__main__":
    main()
