"""Per-XCD balance of K1's persistent build (developer tool): after a settle,
``ops.gemm_clock_ghz`` launches of the shipping pingpong8o clock build, and per
XCD (real XCC_ID) the median workgroup clock and the time its last workgroup
ended. Every XCD gets the same tiles, so the slowest XCD sets the launch time
and ``xcc_finish_spread_us`` is how long the others idle at its end.

    python tools/experiments/xcd_balance.py [--shapes 8192x8192x8192,8192x8192x4096] [--launches 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvidia_terraform_modules_amd import ops  # noqa: E402

KEYS = ("bound_GHz", "launch_GHz", "xcc_clock_spread_pct", "per_xcc_median_GHz",
        "per_xcc_finish_us", "xcc_finish_spread_us", "ms_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8192x8192x8192,8192x8192x4096")
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--settle", type=int, default=600, help="plain launches before the stamped ones")
    args = ap.parse_args()
    for sh in args.shapes.split(","):
        m, n, k = (int(x) for x in sh.split("x"))
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        for _ in range(args.settle):   # queued: the stamped launches follow with no idle gap
            ops.gemm_bf16(a, b, c)
        r = ops.gemm_clock_ghz(a, b, c, steps=args.launches)
        print(json.dumps({"shape": [m, n, k], **{key: r[key] for key in KEYS}}), flush=True)


if __name__ == "__main__":
    main()
