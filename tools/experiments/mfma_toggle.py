"""Operand-toggle energy of the bf16 matrix cores (developer diagnostic, round 6).

mfma_power.py's probe issues the same two operand registers on every MFMA.
This one (gemm_fp8_diag.hpp mfma_toggle_kernel) issues a pp6 quadrant's 16
v_mfma_f32_16x16x32_bf16 per iteration in seven forms (fixed, zero,
one operand changing, both changing, mma_q's order, snake order, mma_q's
order with VGPR instead of AGPR accumulators) and reports,
for each, the sustained TF/s, clock, package power and joules per TFLOP under
the power limit. Rounds interleave the patterns so that drift hits all alike.

    python tools/experiments/mfma_toggle.py [--seconds 1.0] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd.ops import smi  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

PATTERNS = ("fixed", "zero", "one_changes", "both_change", "mma_q_order", "snake_order",
            "mma_q_order_vgpr_acc")
FLOP_PER_ITER = 16 * 2 * 16 * 16 * 32


def run(L, pat, grid, iters, seconds, out, sink, dev):
    def launch():
        check(L.ntm_mfma_toggle(pat, grid, iters, out.data_ptr(), sink.data_ptr(),
                                stream_handle()), "ntm_mfma_toggle")
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    before = smi.sample(dev)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(4):
            launch()
        n += 4
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    after = smi.sample(dev)
    o = out.view(-1, 2).cpu().double()
    clk = float((o[:, 0] / (o[:, 1] / 100e6)).median()) / 1e9
    tflops = n * grid * 4 * iters * FLOP_PER_ITER / wall / 1e12
    w = smi.window(before, after)
    p = w.get("avg_power_W")
    return {"pattern": PATTERNS[pat], "tflops": round(tflops, 1), "clock_GHz": round(clk, 3),
            "avg_power_W": p, "ppt_pct": w.get("ppt_pct"),
            "j_per_tflop": round(p / tflops, 4) if p and tflops else None}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--patterns", default="", help="comma-separated subset of the names")
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--grid", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = torch.zeros(args.grid * 4 * 2, dtype=torch.int64, device=dev)
    sink = torch.zeros(1, device=dev)
    L = lib_experimental()
    rows = {name: [] for name in PATTERNS}
    for r in range(args.rounds):
        pats = [PATTERNS.index(p) for p in args.patterns.split(",")] if args.patterns else list(range(len(PATTERNS)))
        order = pats if r % 2 == 0 else pats[::-1]
        for pat in order:
            row = run(L, pat, args.grid, args.iters, args.seconds, out, sink, dev)
            row["round"] = r
            rows[row["pattern"]].append(row)
            print(json.dumps(row), flush=True)
    summary = {}
    for name, rs in rows.items():
        if not rs:
            continue
        summary[name] = {k: statistics.median([x[k] for x in rs if x[k] is not None] or [0])
                         for k in ("tflops", "clock_GHz", "avg_power_W", "j_per_tflop")}
    print(json.dumps({"summary": summary}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
