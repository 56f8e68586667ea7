"""A/B of K1-fp8's default plan against an explicit earlier plan (developer
tool): "ROWS:TOP:REST" runs rows [0, ROWS) of C on fp8 variant TOP and the rest
on REST (row views of A and C), interleaved with the default and hipBLASLt fp8
in one process; the explicit plan's C is checked bitwise against the default's.

    python tools/fp8_plan_ab.py --cases 6144x6144x6144=5376:pingpong8c:tile160x128
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402


def timed(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", required=True)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    one = torch.ones((), device="cuda")
    ok = True
    for case in args.cases.split(","):
        shape, plan = case.split("=")
        m, n, k = (int(x) for x in shape.split("x"))
        rows, top, rest = plan.split(":")
        rows = int(rows)
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        c2 = torch.empty_like(c)

        def old():
            ops.gemm_fp8(a[:rows], b, c2[:rows], variant=top)
            if rows < m:
                ops.gemm_fp8(a[rows:], b, c2[rows:], variant=rest)

        ops.gemm_fp8(a, b, c)
        old()
        torch.cuda.synchronize()
        same = bool(torch.equal(c.view(torch.int16), c2.view(torch.int16)))
        ok &= same
        fns = {"new": lambda: ops.gemm_fp8(a, b, c), "old": old,
               "hipblaslt": lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                     out_dtype=torch.bfloat16)}
        t = {name: [] for name in fns}
        for _ in range(args.rounds):
            for name, fn in fns.items():
                t[name].append(timed(fn, args.iters))
        fl = 2.0 * m * n * k
        row = {"shape": [m, n, k], "new_plan": list(ops.k1_fp8_plan(m, n, k)), "old_plan": plan,
               "old_bitwise_equal": same}
        for name, v in t.items():
            v.sort()
            row[name] = round(fl / v[len(v) // 2] / 1e9, 1)
        row["new/old"] = round(row["new"] / row["old"], 3)
        print(json.dumps(row), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
