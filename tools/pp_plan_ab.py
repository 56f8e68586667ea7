"""A/B of the default K1 plan with and without the 192x256 / 256x192 ping-pong
tiles, or (--split-only) without just their stream-K split mode (developer tool): per shape, the default dispatch with the tiles (new),
without them (old) and hipBLASLt, timed interleaved, median over rounds; the
plans both ways. Shapes: --shapes MxNxK,... or a seeded ragged set
(tools/ragged_sweep.py's generator) or --random (uniform M, N, K).

    python tools/pp_plan_ab.py --shapes 3072x3072x3072,5120x5120x5120 [--rounds 7 --iters 20]
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
from ragged_sweep import ragged_shapes, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--random", action="store_true", help="uniform M, N, K in [256, 8192], multiples of 8")
    ap.add_argument("--changed-only", action="store_true", help="skip shapes whose plan is the same")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--split-only", action="store_true",
                    help="old = the plan without split mode on the 192-wide tiles only")
    args = ap.parse_args()
    old_knob = (True, False) if args.split_only else (False, False)
    if args.shapes:
        shapes = [tuple(int(x) for x in s.split("x")) for s in args.shapes.split(",") if s]
    elif args.random:
        rng = random.Random(args.seed)
        shapes = [tuple(rng.randrange(256, 8193, 8) for _ in range(3)) for _ in range(args.n)]
    else:
        shapes = ragged_shapes(args.n, args.seed)
    rows = []
    for m, n, k in shapes:
        ops.set_plan_pp_tiles(*old_knob)
        old_plan = list(ops.k1_splitk_plan(m, n, k))
        ops.set_plan_pp_tiles(True)
        new_plan = list(ops.k1_splitk_plan(m, n, k))
        if args.changed_only and old_plan == new_plan:
            continue
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")

        def run(knob):
            ops.set_plan_pp_tiles(*knob)
            ops.gemm_bf16(a, b, c)

        fns = {"new": lambda: run((True, True)), "old": lambda: run(old_knob),
               "hipblaslt": lambda: torch.matmul(a, b.T, out=c)}
        t = {name: [] for name in fns}
        for r in range(args.rounds):
            order = list(fns.items())
            for name, fn in (order if r % 2 == 0 else order[::-1]):
                t[name].append(timed(fn, args.iters))
        ops.set_plan_pp_tiles(True)
        med = {name: statistics.median(v) for name, v in t.items()}
        row = {"shape": [m, n, k], "old_plan": old_plan, "new_plan": new_plan}
        row.update({f"{name}_us": round(v * 1e3, 1) for name, v in med.items()})
        row["new_over_old"] = round(med["old"] / med["new"], 3)
        row["new_over_hipblaslt"] = round(med["hipblaslt"] / med["new"], 3)
        row["old_over_hipblaslt"] = round(med["hipblaslt"] / med["old"], 3)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del a, b, c
    if rows:
        nr = [r["new_over_hipblaslt"] for r in rows]
        orr = [r["old_over_hipblaslt"] for r in rows]
        print(json.dumps({"summary": True, "shapes": len(rows),
                          "new_ahead": sum(x > 1.0 for x in nr),
                          "new_below_0.97": sum(x < 0.97 for x in nr),
                          "old_ahead": sum(x > 1.0 for x in orr),
                          "old_below_0.97": sum(x < 0.97 for x in orr),
                          "new_min": min(nr), "new_median": statistics.median(nr),
                          "new_over_old_min": min(r["new_over_old"] for r in rows),
                          "new_over_old_median": statistics.median(r["new_over_old"] for r in rows)}),
              flush=True)


if __name__ == "__main__":
    main()
