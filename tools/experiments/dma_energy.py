"""Energy per staged byte of two LDS-DMA patterns (developer diagnostic, round 6).

profiles/r6_edec: at 8192^3, removing K1's LDS-DMA lowers the chip's power per
GHz far more than removing its fragment reads. K1 stages each 128-B line with
two instructions (16 rows x 64 B each); hipBLASLt's TA is ~9 % less busy. This
replays the 256x256 kernel's loads without MFMAs (dma_probe.hpp) in the shipping
pattern (mode 0) and in whole-line form (mode 3: 8 rows x 128 B per
instruction, the same bytes and instruction count) on random operands, and
reports per pattern: GB/s staged (all CUs), average package power in an AMD SMI
window of back-to-back launches, and picojoules per staged byte above the idle
floor.

    python tools/experiments/dma_energy.py [--k 4096 --reps 20 --window-s 0.6]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops import smi  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

PATTERNS = {"split_lines_16x64B": 0, "whole_lines_8x128B": 3}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--window-s", type=float, default=0.6)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    L = lib_experimental()
    T = args.k // 64 - 2
    buf = ops.fill_uniform_(torch.empty(513 * args.k, dtype=torch.bfloat16, device=dev), 7)

    def fn(mode):
        return lambda: check(L.ntm_dma_probe(mode, buf.data_ptr(), args.k, T, args.reps, args.grid,
                                             stream_handle()), "ntm_dma_probe")

    fns = {k: fn(m) for k, m in PATTERNS.items()}

    def sync():
        torch.cuda.synchronize(dev)

    sync()
    time.sleep(0.5)
    i0 = smi.sample(dev)
    time.sleep(1.0)
    idle_w = smi.window(i0, smi.sample(dev)).get("avg_power_W")
    bench.prewarm_settle(fns["split_lines_16x64B"], sync, 0.5)
    timing = bench.interleaved_compare(fns, dev, rounds=args.rounds, launches=4)
    power = {k: [] for k in fns}
    for k in list(fns) + list(fns)[::-1]:
        bench.prewarm_settle(fns[k], sync, 0.2)
        b, a, _ = bench.power_window(fns[k], sync, lambda: smi.sample(dev), args.window_s, chunk=16)
        power[k].append(smi.window(b, a))
    staged = args.reps * T * 512 * 128 * args.grid
    out = {"k": args.k, "grid": args.grid, "bytes_per_launch": staged, "idle_W": idle_w}
    for k in fns:
        s = timing[k]["median_s"]
        ws = [w.get("avg_power_W") for w in power[k] if w.get("avg_power_W") is not None]
        pw = statistics.mean(ws) if ws else None
        gbps = staged / s / 1e9
        out[k] = {"ms": round(s * 1e3, 3), "GBps": round(gbps, 1), "avg_power_W": pw and round(pw, 1),
                  "pJ_per_byte_above_idle": round((pw - idle_w) / gbps * 1e3, 2) if pw and idle_w else None,
                  "gfxclk_mhz_end": [(w.get("gfxclk_mhz") or [None, None])[1] for w in power[k]],
                  "ppt_pct": [w.get("ppt_pct") for w in power[k]]}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
