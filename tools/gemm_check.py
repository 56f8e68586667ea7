"""K1 numerics + throughput check on one MI355X (developer tool).

    python tools/gemm_check.py [--sizes 4096,8192,6144x6144x8192] [--iters 50] [--variants default,pingpong8o]

For every size: full verification of each variant against the independent
fp32 reference kernel, then interleaved timing rounds of every variant and of
torch.matmul (hipBLASLt) on the same uniform [-1,1) data in ONE process
(playbook rule 24). Prints one JSON line per size.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402


def timed(fn, iters: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="default,pingpong8o")
    args = ap.parse_args()
    variants = args.variants.split(",")
    dev = torch.device("cuda:0")
    print(json.dumps({"device": torch.cuda.get_device_name(0), "lib": ops.version()}), flush=True)
    for s in args.sizes.split(","):
        m, n, k = (int(x) for x in s.split("x")) if "x" in s else (int(s),) * 3
        a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
        b = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
        ops.fill_uniform_(a, seed=1)
        ops.fill_uniform_(b, seed=2)
        atol, rtol = ops.gemm_tolerance(k)
        ref = ops.ref_gemm_f32(a, b)
        res = {"size": int(s) if "x" not in s else s}
        cc = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
        served = []
        for v in variants:
            cc.fill_(float("nan"))
            try:
                ops.gemm_bf16(a, b, cc, variant=v)
            except ValueError as e:  # the variant does not serve this shape (host-side check)
                res[f"unserved_{v}"] = str(e)[:120]
                continue
            served.append(v)
            res[f"verify_{v}"] = ops.verify_bf16(cc, ref, atol, rtol).as_dict()
        del ref
        flops = 2.0 * m * n * k
        times = {v: [] for v in served + ["torch"]}
        for _ in range(args.rounds):
            for v in served:
                times[v].append(timed(lambda: ops.gemm_bf16(a, b, cc, variant=v), args.iters))
            times["torch"].append(timed(lambda: torch.matmul(a, b.T, out=cc), args.iters))
        for v, t in times.items():
            t = sorted(t)
            res[f"{v}_ms_min"] = t[0]
            res[f"{v}_ms_med"] = t[len(t) // 2]
            res[f"{v}_tflops_best"] = flops / t[0] / 1e9
            res[f"{v}_tflops_med"] = flops / t[len(t) // 2] / 1e9
        print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
