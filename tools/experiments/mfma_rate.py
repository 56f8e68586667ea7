"""Matrix-core issue rate on MI355X (developer diagnostic): cycles per MFMA and
in-kernel clock for v_mfma_f32_16x16x32_bf16 vs v_mfma_scale_f32_16x16x128_f8f6f4
(e4m3), operands in registers, one wave per SIMD on every CU, random bits.

    python tools/experiments/mfma_rate.py [--iters 20000]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--grid", type=int, default=256)
    args = ap.parse_args()
    out = torch.zeros(args.grid * 4 * 2, dtype=torch.int64, device="cuda")
    sink = torch.zeros(1, device="cuda")
    res = {}
    for name, f8, k in (("bf16_16x16x32", 0, 32), ("fp8_16x16x128_scaled", 1, 128)):
        for _ in range(3):   # warm the clock
            check(lib_experimental().ntm_mfma_rate(f8, args.grid, args.iters, out.data_ptr(), sink.data_ptr(),
                                      stream_handle()), "ntm_mfma_rate")
        torch.cuda.synchronize()
        o = out.view(-1, 2).cpu().double()
        cyc = float(o[:, 0].median())
        clk = float((o[:, 0] / (o[:, 1] / 100e6)).median())
        n_mfma = args.iters * 8
        flop = 2 * 16 * 16 * k
        res[name] = {"cycles_per_mfma": round(cyc / n_mfma, 2), "clock_GHz": round(clk / 1e9, 3),
                     "flop_per_cycle_per_cu": round(4 * flop / (cyc / n_mfma), 1),
                     "chip_TFLOPs_at_clock": round(256 * 4 * flop / (cyc / n_mfma) * clk / 1e12, 1)}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
