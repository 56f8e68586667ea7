"""Ablation timing of the K1 default kernel (developer diagnostic).

Times four builds of pingpong8c (validation/include/ntm/gemm_bf16_pp3_stamp.hpp)
interleaved in one process on random data, after >= 2 s of back-to-back
launches (MI355X_MICROARCH.md 'DVFS give-back' item 6):
  real      the kernel as shipped (+ 2 stamps per wave),
  no_lds    fragment reads + LDS-DMA removed (MFMA + barriers),
  no_mfma   MFMAs removed (reads + DMA + barriers),
  mfma_only MFMAs only (no barriers, no loads),
  reads_no_dma / dma_no_reads  one half of no_lds's removal each,
and reports each one's wall time, in-kernel clock (s_memtime over
s_memrealtime, median over waves) and cycles per K-tile per workgroup.

    python tools/experiments/gemm_stamp.py [--size 8192] [--warm-s 2] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

SLOTS = 8
START, END, RT0, RT1, HWID, XCCID, RL0, RL1 = range(8)
MODES = {"real": 0, "no_lds": 1, "no_mfma": 2, "mfma_only": 3, "reads_no_dma": 4,
         "dma_no_reads": 5}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--warm-s", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    n = args.size
    dev = torch.device("cuda:0")
    a = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device=dev), 1)
    b = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device=dev), 2)
    c = torch.empty((n, n), dtype=torch.bfloat16, device=dev)
    nwg = (n // 256) ** 2
    st = {m: torch.zeros(nwg * 8 * SLOTS, dtype=torch.int64, device=dev) for m in MODES}

    def run(m):
        rc = lib_experimental().ntm_gemm_bf16_stamp(MODES[m], a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                       n, n, n, n, n, n, st[m].data_ptr(), stream_handle())
        check(rc, "ntm_gemm_bf16_stamp")

    t_end = time.time() + args.warm_s
    while time.time() < t_end:
        for _ in range(args.iters):
            run("real")
        torch.cuda.synchronize()
    times = {m: [] for m in MODES}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(args.rounds):
        for m in MODES:
            ev[0].record()
            for _ in range(args.iters):
                run(m)
            ev[1].record()
            torch.cuda.synchronize()
            times[m].append(ev[0].elapsed_time(ev[1]) / args.iters)
    run("real")
    ref = ops.ref_gemm_f32(a, b)
    atol, rtol = ops.gemm_tolerance(n)
    ok = ops.verify_bf16(c, ref, atol, rtol).ok
    T = n // 64
    tiles_per_cu = nwg / 256
    out = {"size": n, "real_verified": ok}
    for m in MODES:
        s = st[m].view(nwg, 8, SLOTS).cpu().double()
        span = s[:, :, END] - s[:, :, START]
        rt = (s[:, :, RT1] - s[:, :, RT0]) / 100e6
        ms = sorted(times[m])[len(times[m]) // 2]
        clk = float((span / rt).median()) / 1e9
        out[m] = {"ms": round(ms, 4), "tflops": round(2 * n ** 3 / ms / 1e9, 1),
                  "clock_GHz": round(clk, 3),
                  "wg_span_cycles_per_ktile": round(float(span.median()) / T, 1),
                  "kernel_cycles_per_ktile_per_cu": round(ms * 1e-3 * clk * 1e9 / (T * tiles_per_cu), 1)}
    # per-CU timeline of the real kernel (last launch): workgroups that ran on the
    # same CU (HW_ID cu/sh/se fields + XCC id) in start order; gap = next start -
    # this end (s_memrealtime, 10 ns ticks), lead = first start - launch's first start.
    s = st["real"].view(nwg, 8, SLOTS).cpu()
    w0 = s[:, 0, :]
    hw = w0[:, HWID]
    cu_key = (w0[:, XCCID] & 0xF) * 4096 + ((hw >> 8) & 0xF) * 256 + ((hw >> 12) & 0x1) * 16 + \
        ((hw >> 13) & 0x7)
    rt0, rt1 = w0[:, RT0].double(), w0[:, RT1].double()
    t0 = float(rt0.min())
    gaps, leads, tails, per_cu = [], [], [], []
    for key in torch.unique(cu_key):
        idx = (cu_key == key).nonzero().flatten()
        order = idx[torch.argsort(rt0[idx])]
        per_cu.append(len(order))
        leads.append(float(rt0[order[0]]) - t0)
        tails.append(float(rt1.max() - rt1[order[-1]]))
        for i in range(len(order) - 1):
            gaps.append(float(rt0[order[i + 1]] - rt1[order[i]]))
    g = torch.tensor(gaps) * 10e-3 if gaps else torch.zeros(1)
    out["timeline_real"] = {
        "cus_seen": len(per_cu), "wgs_per_cu_max": max(per_cu), "wgs_per_cu_min": min(per_cu),
        "wg_gap_us_median": round(float(g.median()), 3), "wg_gap_us_p90": round(float(g.quantile(0.9)), 3),
        "first_start_spread_us_p90": round(float(torch.tensor(leads).quantile(0.9)) * 10e-3, 3),
        "end_spread_us_p90": round(float(torch.tensor(tails).quantile(0.9)) * 10e-3, 3),
        "wg_span_us_median": round(float((rt1 - rt0).median()) * 10e-3, 2),
        "launch_span_us": round(float(rt1.max() - rt0.min()) * 10e-3, 2)}
    # per-workgroup phase split (wave 0; 10 ns ticks): start -> loop entry (prologue:
    # address setup + the first LDS-DMA round trip), the K loop, loop end -> done
    # (drain + LDS-staged epilogue + stores issued). Split by the WG's round on its CU.
    rl0, rl1 = w0[:, RL0].double(), w0[:, RL1].double()
    rounds = {}
    for key in torch.unique(cu_key):
        idx = (cu_key == key).nonzero().flatten()
        order = idx[torch.argsort(rt0[idx])]
        for r, i in enumerate(order.tolist()):
            rounds.setdefault(r, []).append(i)
    def med(x):
        return round(float(x.median()) * 10e-3, 3)
    out["phase_split_real_us"] = {
        f"round{r}": {"prologue": med(rl0[ix] - rt0[ix]), "loop": med(rl1[ix] - rl0[ix]),
                      "epilogue": med(rt1[ix] - rl1[ix]), "n": len(ix)}
        for r, ix in sorted(rounds.items())}
    xcc = (w0[:, XCCID] & 0xF)
    out["per_xcd_real"] = {
        int(x): {"wg_span_us_mean": round(float((rt1 - rt0)[xcc == x].mean()) * 10e-3, 2),
                 "last_end_us": round(float(rt1[xcc == x].max() - t0) * 10e-3, 2),
                 "median_cu_end_us": round(float(rt1[xcc == x].median() - t0) * 10e-3, 2),
                 "clock_GHz": round(float(((s[:, 0, END] - s[:, 0, START]).double() /
                                          ((rt1 - rt0) / 100e6))[xcc == x].median()) / 1e9, 3)}
        for x in torch.unique(xcc)}
    # matrix floor: 2 waves/SIMD x 64 v_mfma_f32_16x16x32_bf16 x 16 cycles per K-tile
    out["mfma_floor_cycles_per_ktile"] = 2048
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
