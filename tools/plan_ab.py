"""A/B of a dispatch-plan change (developer tool): for each case, time the
default dispatch (the plan in the built library) against an explicit earlier
plan "ROWS:TOP:REST" (rows [0, ROWS) on TOP, the rest on REST; a variant
"tile128/s4" = split-K in 4 slices) and hipBLASLt, interleaved in one process;
the explicit plan is checked against the default result. One JSON line per case.

    python tools/plan_ab.py --cases 3072x3072x3072=3072:pingpong8c:tile128,...
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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


def run(a, b, c, v):
    v, _, sk = v.partition("/s")
    ops.gemm_bf16(a, b, c, variant=v, splits=int(sk) if sk else 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", required=True)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    ok_all = True
    for case in args.cases.split(","):
        shape, spec = case.split("=")
        m, n, k = (int(x) for x in shape.split("x"))
        rows, top, rest = spec.split(":")
        r = int(rows)
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        ref = ops.gemm_bf16(a, b).float()
        atol, rtol = ops.gemm_tolerance(k)

        def old():
            run(a[:r], b, c[:r], top)
            if r < m:
                run(a[r:], b, c[r:], rest)
        old()
        torch.cuda.synchronize()
        ok = bool(torch.all((c.float() - ref).abs() <= atol + rtol * ref.abs()))
        ok_all &= ok
        fns = {"new": lambda: ops.gemm_bf16(a, b, c), "old": old,
               "torch": lambda: torch.matmul(a, b.T, out=c)}
        t = {x: [] for x in fns}
        for _ in range(args.rounds):
            for x, fn in fns.items():
                t[x].append(timed(fn, args.iters))
        fl = 2.0 * m * n * k
        row = {"shape": [m, n, k], "new_plan": list(ops.kernels.k1_splitk_plan(m, n, k)),
               "old_plan": spec, "old_ok": ok}
        for x, v in t.items():
            v.sort()
            row[x] = round(fl / v[len(v) // 2] / 1e9, 1)
        row["new/old"] = round(row["new"] / row["old"], 3)
        print(json.dumps(row), flush=True)
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
