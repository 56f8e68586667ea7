"""LDS-DMA access-pattern probe (developer tool, profiles/r5_h192/): the 256x256
ping-pong's loads without MFMAs, on rows whose pitch is 128-B aligned or only
16-B aligned (K % 16 == 8), in three patterns (validation/include/ntm/dma_probe.hpp):

  0  the kernel's pattern as is
  1  misaligned rows re-based to whole 64-B quads (2 L1 accesses per row per
     K-tile, each line still fetched by two K-tiles)
  2  misaligned rows re-based down to their aligned line (the aligned pattern)

Prints per-CU GB/s of staged bytes, interleaved rounds, median. --depths 0,1,2,3
repeats it with 5 / 8 / 12 / 16 halves in flight (counted vmcnt 10 / 16 / 24 / 32).

    python tools/experiments/dma_probe.py [--k 4096 --grid 256 --reps 20 --rounds 7]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--depths", default="0", help="in-flight depths: 0..3 = vmcnt 10 / 16 / 24 / 32")
    ap.add_argument("--policies", default="", help="cache policies 1..5 = sc0 / nt / sc0 nt / sc1 / "
                    "sc1 nt (at depth 0)")
    args = ap.parse_args()
    L = lib_experimental()
    T = args.k // 64 - 2
    cases = {}
    for d in (int(x) for x in args.depths.split(",")):
        sfx = "" if d == 0 else f"@vm{(10, 16, 24, 32)[d]}"
        cases.update({"aligned/0" + sfx: (10 * d, args.k), "misaligned/0" + sfx: (10 * d, args.k + 8),
                      "misaligned/1" + sfx: (10 * d + 1, args.k + 8),
                      "misaligned/2" + sfx: (10 * d + 2, args.k + 8)})
    for a in (int(x) for x in args.policies.split(",") if x):
        sfx = "@" + ("sc0", "nt", "sc0nt", "sc1", "sc1nt")[a - 1]
        cases.update({"aligned/0" + sfx: (100 * a, args.k), "misaligned/0" + sfx: (100 * a, args.k + 8)})
    bufs = {p: torch.zeros(513 * p, dtype=torch.bfloat16, device="cuda") for p in {args.k, args.k + 8}}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(mode, pitch):
        check(L.ntm_dma_probe(mode, bufs[pitch].data_ptr(), pitch, T, args.reps, args.grid,
                              stream_handle()), "ntm_dma_probe")

    times = {c: [] for c in cases}
    for name, (mode, pitch) in cases.items():
        run(mode, pitch)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for name, (mode, pitch) in (list(cases.items()) if r % 2 == 0 else list(cases.items())[::-1]):
            e0.record()
            run(mode, pitch)
            e1.record()
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e-3)
    staged = args.reps * T * 512 * 128          # bytes staged per workgroup
    out = {"k": args.k, "grid": args.grid, "reps": args.reps, "ktiles": T}
    for name, ts in times.items():
        s = statistics.median(ts)
        out[name] = {"ms": round(s * 1e3, 3), "GBps_per_wg": round(staged / s / 1e9, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
