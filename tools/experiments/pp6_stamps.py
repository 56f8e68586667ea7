"""Where pingpong8o's tile boundary spends its cycles (VERDICT r3 #2 follow-up,
profiles/r3_stores open question): s_memtime stamps of wave 0 at every phase
start from K-tile T-2 of a workgroup's first tile to K-tile 1 of its second
(gemm_bf16_pp6.hpp STAMP 2), on 256 and 128 workgroups, with C stored and
not stored. A diagnostic build: read its SHARES, not its run time.

    python tools/experiments/pp6_stamps.py [--size 8192] [--k 8192] [--warm-s 1]

Prints one JSON line per (grid, store) with the median over workgroups of
each phase's cycles (16 phases: T-2 P0..P3, T-1 P0..P3, next tile 0 P0..P3,
1 P0..P3), the window total and its excess over the same window without
stores. Boundary stores go out in T-1 P1..P3 and tile-0 P0.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

PHASES = [f"{kt}P{p}" for kt in ("T-2", "T-1", "n0", "n1") for p in range(4)]


def main() -> int:
    import torch

    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle

    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--warm-s", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grids", default="256,128")
    ap.add_argument("--modes", default="1,0",
                    help="1 stored, 0 not stored, 2 stored + spread (the shipping build)")
    args = ap.parse_args()
    m = n = args.size
    k = args.k
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
    c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
    L = lib_experimental()
    base = {}
    modes = [int(x) for x in args.modes.split(",")]
    for grid in (int(g) for g in args.grids.split(",")):
        for store in modes:
            st = torch.zeros((grid, 17), dtype=torch.int64, device="cuda")

            def run():
                check(L.ntm_gemm_bf16_pp6_stamp(grid, store, a.data_ptr(), b.data_ptr(),
                                                c.data_ptr(), m, n, k, k, k, n, st.data_ptr(),
                                                stream_handle()), "ntm_gemm_bf16_pp6_stamp")

            t0 = time.perf_counter()
            while time.perf_counter() - t0 < args.warm_s:
                run()
            torch.cuda.synchronize()
            per = []
            for _ in range(args.reps):
                run()
                torch.cuda.synchronize()
                per.append((st[:, 1:] - st[:, :-1]).double())
            d = torch.cat(per)                                     # (reps*grid, 16)
            med = d.median(dim=0).values.tolist()
            tot = float(d.sum(dim=1).median())
            row = {"grid": grid, "store": store, "phase_cycles_median": dict(zip(PHASES, [
                round(x) for x in med])), "window_cycles_median": round(tot)}
            base[(store, grid)] = (med, tot)
            print(json.dumps(row), flush=True)
        for a_, b_ in ((1, 0), (2, 0)):
            if (a_, grid) in base and (b_, grid) in base:
                (ms, ts), (mn, tn) = base[(a_, grid)], base[(b_, grid)]
                print(json.dumps({"grid": grid, "modes": [a_, b_], "minus_cycles": dict(zip(
                    PHASES, [round(x - y) for x, y in zip(ms, mn)])),
                    "window_delta_cycles": round(ts - tn)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
