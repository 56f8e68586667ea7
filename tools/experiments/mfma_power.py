"""Sustained matrix-core load vs power (developer diagnostic, round 5): each
MFMA form alone (operands in registers, one wave per SIMD on every CU) for
about --seconds of back-to-back launches, with the AMD SMI power / throttle
window around them (ops/smi.py) and the in-kernel clock. Tells how much of
the GEMM's power-capped budget the matrix cores alone draw.

    python tools/experiments/mfma_power.py [--seconds 1.5]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd.ops import smi  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

FORMS = (("bf16_16x16x32", 0, 2 * 16 * 16 * 32, 8),
         ("bf16_32x32x16", 2, 2 * 32 * 32 * 16, 8),
         ("fp8_16x16x128", 1, 2 * 16 * 16 * 128, 8),
         ("fp8_32x32x64", 3, 2 * 32 * 32 * 64, 8))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--grid", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = torch.zeros(args.grid * 4 * 2, dtype=torch.int64, device=dev)
    sink = torch.zeros(1, device=dev)
    L = lib_experimental()
    for name, mode, flop, per_iter in FORMS:
        def launch():
            check(L.ntm_mfma_rate(mode, args.grid, args.iters, out.data_ptr(), sink.data_ptr(),
                                  stream_handle()), "ntm_mfma_rate")
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        before = smi.sample(dev)
        while time.perf_counter() - t0 < args.seconds:
            for _ in range(4):
                launch()
            n += 4
            torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        after = smi.sample(dev)
        o = out.view(-1, 2).cpu().double()
        clk = float((o[:, 0] / (o[:, 1] / 100e6)).median()) / 1e9
        tflops = n * args.grid * 4 * args.iters * per_iter * flop / wall / 1e12
        w = smi.window(before, after)
        print(json.dumps({"form": name, "launches": n, "wall_s": round(wall, 3),
                          "tflops": round(tflops, 1), "clock_GHz": round(clk, 3),
                          "avg_power_W": w.get("avg_power_W"), "ppt_pct": w.get("ppt_pct"),
                          "thermal_pct": w.get("thermal_pct"),
                          "gfxclk_mhz": w.get("gfxclk_mhz")}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
