"""Time manual row splits of C against the default dispatch and hipBLASLt
(developer tool): each split "ROWS:TOPVARIANT:RESTVARIANT" runs rows [0, ROWS)
on TOPVARIANT and the rest on RESTVARIANT (two launches; ROWS = M: one), interleaved rounds,
median TF/s; every split is checked against the default result (fp32 tolerance). A variant
"tile128/s8" runs split-K in 8 K slices.

    python tools/experiments/split_check.py --shape 3200x3200x3200 --splits 1920:tile160:tile128
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="3200x3200x3200")
    ap.add_argument("--splits", default="1920:tile160:tile128")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    m, n, k = (int(x) for x in args.shape.split("x"))
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
    c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
    ref = ops.gemm_bf16(a, b).float()
    atol, rtol = ops.gemm_tolerance(k)
    fns = {"default": lambda: ops.gemm_bf16(a, b, c),
           "torch": lambda: torch.matmul(a, b.T, out=c)}
    ok = {}
    for sp in args.splits.split(","):
        rows, top, rest = sp.split(":")
        r = int(rows)

        def run(x, y, z, v):
            v, _, sk = v.partition("/s")
            ops.gemm_bf16(x, y, z, variant=v, splits=int(sk) if sk else 1)

        def f(r=r, top=top, rest=rest):
            run(a[:r], b, c[:r], top)
            if r < m:
                run(a[r:], b, c[r:], rest)
        f()
        torch.cuda.synchronize()
        ok[sp] = bool(torch.all((c.float() - ref).abs() <= atol + rtol * ref.abs()))
        fns[sp] = f
    for _ in range(200):
        fns["torch"]()
    t = {x: [] for x in fns}
    for _ in range(args.rounds):
        for x, fn in fns.items():
            t[x].append(timed(fn, args.iters))
    fl = 2.0 * m * n * k
    row = {"shape": [m, n, k], "splits_ok": ok}
    for x, v in t.items():
        v.sort()
        row[f"{x}_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
    print(json.dumps(row), flush=True)
    return 0 if all(ok.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
