"""A/B of the K1 plan's split-K rule (developer tool): on a seeded set of
random shapes, the plan under the --old-margin / --old-min-k rule (default:
round 4's margin 1.1 everywhere) and under --margin / --min-k (the margin for
splits whose slices keep >= min-k of K; default: the shipping 1.03 / 1024)
are computed on the host (ops.set_plan_splitk); every shape whose plan
changes is timed both ways as an explicit plan, next to hipBLASLt, interleaved
in one process (median over rounds), and the new plan's result is checked
against the old one's. One JSON line per changed shape, then a summary line.

    python tools/margin_ab.py --n 3000 --seed 6 [--margin 1.03 --min-k 1024] [--max 40]
"""
import argparse
import json
import os
import random
import statistics
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


def runner(plan, a, b, c):
    """An explicit split-K plan (rows, top, rest, splits) as a callable."""
    rows, top, rest, splits = plan
    m = a.shape[0]
    if splits > 1 or top in ops.kernels.SK_VARIANTS or rows >= m:
        return lambda: ops.gemm_bf16(a, b, c, variant=top, splits=splits)

    def two():
        ops.gemm_bf16(a[:rows], b, c[:rows], variant=top)
        ops.gemm_bf16(a[rows:], b, c[rows:], variant=rest)
    return two


def runner_fp8(plan, a, b, c):
    """An explicit K1-fp8 split-K plan (rows, top, rest, splits) as a callable."""
    rows, top, rest, splits = plan
    if splits > 1 or rows >= a.shape[0]:
        return lambda: ops.gemm_fp8(a, b, c, variant=top, splits=splits)

    def two():
        ops.gemm_fp8(a[:rows], b, c[:rows], variant=top)
        ops.gemm_fp8(a[rows:], b, c[rows:], variant=rest)
    return two


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--margin", type=float, default=0.0, help="new rule (0: shipping)")
    ap.add_argument("--min-k", type=int, default=-1, help="new rule (-1: shipping)")
    ap.add_argument("--old-margin", type=float, default=1.1)
    ap.add_argument("--old-min-k", type=int, default=0)
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"),
                    help="fp8: K1-fp8's split-K plan (old rule: 1.1 for fp8 too)")
    ap.add_argument("--ragged", action="store_true",
                    help="A/B the ragged pricing of long-slice split-K alone (old: without it; "
                         "without --ragged both sides run without it)")
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--max", type=int, default=40, help="time at most this many changed shapes")
    ap.add_argument("--shapes", default="", help="MxNxK,... instead of the seeded set")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    if args.shapes:
        shapes = [tuple(int(x) for x in s.split("x")) for s in args.shapes.split(",") if s]
    else:
        rng = random.Random(args.seed)
        step = 16 if args.dtype == "fp8" else 8   # K1-fp8: N % 8, K % 16
        shapes = [tuple(rng.randrange(256, 8193, step) for _ in range(3)) for _ in range(args.n)]
    fp8 = args.dtype == "fp8"
    plan = ops.k1_fp8_splitk_plan if fp8 else ops.k1_splitk_plan
    ops.set_plan_splitk(args.old_margin, args.old_min_k, fp8=False)
    ops._lib.lib().ntm_set_plan_splitk_ragged(0)
    if args.ragged:   # A/B of the ragged pricing alone: old = the margin rule without it
        ops.set_plan_splitk()
    old = {s: tuple(plan(*s)) for s in shapes}
    ops.set_plan_splitk(args.margin, args.min_k)
    ops._lib.lib().ntm_set_plan_splitk_ragged(1 if args.ragged else 0)
    new = {s: tuple(plan(*s)) for s in shapes}
    ops._lib.lib().ntm_set_plan_splitk_ragged(1)   # the shipping plan
    ops.set_plan_splitk()
    changed = [s for s in shapes if old[s] != new[s]][: args.max]
    ratios, bad = [], 0
    one = torch.ones((), device="cuda")
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    for m, n, k in changed:
        a = ops.fill_uniform_(torch.empty((m, k), dtype=dt, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=dt, device="cuda"), 2)
        c_old = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        c_new = torch.empty_like(c_old)
        c_t = torch.empty_like(c_old)
        if fp8:
            fns = {"old": runner_fp8(old[(m, n, k)], a, b, c_old),
                   "new": runner_fp8(new[(m, n, k)], a, b, c_new),
                   "torch": lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                     out_dtype=torch.bfloat16)}
        else:
            fns = {"old": runner(old[(m, n, k)], a, b, c_old),
                   "new": runner(new[(m, n, k)], a, b, c_new),
                   "torch": lambda: torch.matmul(a, b.T, out=c_t)}
        t = {x: [] for x in fns}
        for _ in range(args.rounds):
            for x, fn in fns.items():
                t[x].append(timed(fn, args.iters))
        torch.cuda.synchronize()
        atol, rtol = ops.gemm_tolerance(k)
        if fp8:   # e4m3 operands: compare the two plans' bf16 outputs loosely
            atol, rtol = 4 * atol, 4 * rtol
        ref = c_old.float()
        ok = bool(torch.all((c_new.float() - ref).abs() <= atol + rtol * ref.abs()))
        bad += not ok
        med = {x: statistics.median(v) * 1e3 for x, v in t.items()}
        ratios.append(med["old"] / med["new"])
        print(json.dumps({"shape": [m, n, k], "old_plan": old[(m, n, k)], "new_plan": new[(m, n, k)],
                          "old_us": round(med["old"], 1), "new_us": round(med["new"], 1),
                          "hipblaslt_us": round(med["torch"], 1), "new_speedup": round(ratios[-1], 3),
                          "new_ok": ok}), flush=True)
    if ratios:
        print(json.dumps({"summary": True, "dtype": args.dtype, "new": [args.margin, args.min_k],
                          "old": [args.old_margin, args.old_min_k], "shapes": len(shapes),
                          "changed": len(changed), "faster": sum(r > 1.0 for r in ratios),
                          "median_speedup": round(statistics.median(ratios), 3),
                          "min": round(min(ratios), 3), "max": round(max(ratios), 3), "bad": bad}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
