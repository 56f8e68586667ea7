"""Ragged one-round K1 sweep (developer tool): a SEEDED set of
shapes whose C fits at most one round of 256x256 tiles with a ragged edge -
the class where the default plan trailed hipBLASLt by 2-16 % in round 4 -
timed interleaved (every callable once per round, median over rounds): the
default dispatch, hipBLASLt (torch.matmul) and every candidate decomposition
that serves the shape. One JSON line per shape, then a summary line.

    python tools/ragged_sweep.py --n 24 --seed 5 [--rounds 7 --iters 20] [--candidates]

The seed picks the shapes; pass a fresh one to validate a plan change on
shapes it was not tuned on.
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

CANDIDATES = ("pingpong8s", "pingpong8cm", "tile128", "tile256x128", "tile160", "tile160x128",
              "tile128x160", "tile128x256", "pp192x256", "pp256x192", "pp224x256",
              "pp192x256s", "pp256x192s")


def ragged_shapes(n: int, seed: int, lo: float = 0.3, hi: float = 1.0) -> list:
    """n shapes: M, N, K % 8, C between lo and hi rounds of 256x256 tiles (256 CUs),
    at least one of M, N not a multiple of 256; K in [1024, 16384]."""
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        m = rng.randrange(256, 8193, 8)
        nn = rng.randrange(256, 8193, 8)
        k = rng.randrange(1024, 16385, 8)
        tiles = ((m + 255) // 256) * ((nn + 255) // 256)
        if not lo * 256 < tiles <= hi * 256 or (m % 256 == 0 and nn % 256 == 0):
            continue
        out.append((m, nn, k))
    return out


def timed(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--shapes", default="", help="MxNxK,... instead of the seeded set")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--candidates", action="store_true",
                    help="also time every candidate variant that serves the shape")
    ap.add_argument("--splitk", default="",
                    help="also time these split-K candidates, e.g. tile160/s2,tile256x128/s3")
    ap.add_argument("--lo", type=float, default=0.3)
    ap.add_argument("--hi", type=float, default=1.0)
    args = ap.parse_args()
    shapes = ([tuple(int(x) for x in s.split("x")) for s in args.shapes.split(",") if s]
              or ragged_shapes(args.n, args.seed, args.lo, args.hi))
    ratios = []
    for m, n, k in shapes:
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        fns = {"default": lambda: ops.gemm_bf16(a, b, c),
               "hipblaslt": lambda: torch.matmul(a, b.T, out=c)}
        if args.candidates:
            for v in CANDIDATES:
                if v == "pingpong8s" and not ops.sk_ws_bytes(m, n, k):
                    continue
                if v in ops.kernels.SKH_VARIANTS and not ops.kernels.skh_ws_bytes(v, m, n, k):
                    continue
                fns[v] = lambda v=v: ops.gemm_bf16(a, b, c, variant=v)
        for spec in (x for x in args.splitk.split(",") if x):
            v, _, sp = spec.partition("/s")
            fns[spec] = lambda v=v, sp=int(sp): ops.gemm_bf16(a, b, c, variant=v, splits=sp)
        t = {name: [] for name in fns}
        for r in range(args.rounds):
            order = list(fns.items())
            for name, fn in (order if r % 2 == 0 else order[::-1]):
                t[name].append(timed(fn, args.iters))
        med = {name: statistics.median(v) for name, v in t.items()}
        fl = 2.0 * m * n * k
        row = {"shape": [m, n, k],
               "tiles256": ((m + 255) // 256) * ((n + 255) // 256),
               "plan": list(ops.k1_splitk_plan(m, n, k))}
        for name, v in med.items():
            row[f"{name}_us"] = round(v * 1e3, 1)
        row["default_over_hipblaslt"] = round(med["hipblaslt"] / med["default"], 3)
        if args.candidates:
            best = min((v, name) for name, v in med.items() if name != "hipblaslt")
            row["best"] = best[1]
            row["best_over_hipblaslt"] = round(med["hipblaslt"] / best[0], 3)
        ratios.append(row["default_over_hipblaslt"])
        print(json.dumps(row), flush=True)
        del a, b, c
    print(json.dumps({"summary": True, "shapes": len(ratios),
                      "ahead": sum(r > 1.0 for r in ratios),
                      "below_0.97": sum(r < 0.97 for r in ratios),
                      "min": min(ratios), "median": statistics.median(ratios)}), flush=True)


if __name__ == "__main__":
    main()
