"""Split-K check (developer tool): interleaved timing of the masked small tiles
with 1..8 K slices, the default dispatch and hipBLASLt (torch.matmul) on
M x N x K shapes, plus the max error of each split against the unsplit result;
one JSON line per shape.

    python tools/experiments/splitk_check.py --shapes 280x6352x7568 [--splits 1,2,3,4,6,8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvidia_terraform_modules_amd import ops  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="280x6352x7568")
    ap.add_argument("--splits", default="1,2,3,4,6,8")
    ap.add_argument("--tiles", default="tile128,tile256x128,tile160")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    splits = [int(s) for s in args.splits.split(",")]
    for sh in args.shapes.split(","):
        m, n, k = (int(x) for x in sh.split("x"))
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        ref = torch.matmul(a.float(), b.float().T)
        fns = {"default": lambda: ops.gemm_bf16(a, b, c),
               "torch": lambda: torch.matmul(a, b.T, out=c)}
        err = {}
        for v in args.tiles.split(","):
            for s in splits:
                name = f"{v}/s{s}"
                fns[name] = lambda v=v, s=s: ops.gemm_bf16(a, b, c, variant=v, splits=s)
                fns[name]()
                err[name] = float((c.float() - ref).abs().max())
        t = {name: [] for name in fns}
        for _ in range(args.rounds):
            for name, fn in fns.items():
                t[name].append(timed(fn, args.iters))
        fl = 2.0 * m * n * k
        row = {"shape": [m, n, k], "plan": list(ops.kernels.k1_splitk_plan(m, n, k))}
        for name, v in t.items():
            v.sort()
            row[name] = round(fl / v[len(v) // 2] / 1e9, 1)
        row["max_err"] = {k_: round(e, 4) for k_, e in err.items()}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
