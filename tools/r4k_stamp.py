"""Cycle budget of the 4-wave one-barrier-per-K-tile K1 build ("dma4k",
developer diagnostic; validation/include/ntm/gemm_r4k_stamp.hpp).

--dtype fp8: the same kernel on e4m3 (one f8f6f4 MFMA per slot, K-tile = 128
e4m3); --temporal: plain C stores instead of nontemporal ones.
Per mode (real / no_dma / no_reads / no_barrier / mfma_only), interleaved in
one process on random data after >= 2 s of back-to-back launches: wall time,
TF/s, in-kernel clock (s_memtime over s_memrealtime, median over waves), and
per K-tile step the median cycles a wave spends in the [lgkmcnt(0) + vmcnt(0)]
wait and in the s_barrier, against the 2048-cycle MFMA floor of a step.

    python tools/r4k_stamp.py [--size 8192] [--warm-s 2] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

SLOTS = 10
MODES = {"real": 0, "no_dma": 1, "no_reads": 2, "no_barrier": 3, "mfma_only": 4}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--warm-s", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--temporal", action="store_true", help="plain (not nontemporal) C stores")
    args = ap.parse_args()
    n = args.size
    dev = torch.device("cuda:0")
    f8 = args.dtype == "fp8"
    dt = torch.float8_e4m3fn if f8 else torch.bfloat16
    a = ops.fill_uniform_(torch.empty((n, n), dtype=dt, device=dev), 1)
    b = ops.fill_uniform_(torch.empty((n, n), dtype=dt, device=dev), 2)
    modes = {m: MODES[m] + (16 if f8 else 0) + (8 if args.temporal else 0)
             for m in args.modes.split(",")}
    c = torch.empty((n, n), dtype=torch.bfloat16, device=dev)
    nwg = (n // 256) ** 2
    steps = n // (128 if f8 else 64)
    st = {m: torch.zeros(nwg * 4 * SLOTS, dtype=torch.int64, device=dev) for m in modes}

    def run(m):
        rc = lib_experimental().ntm_gemm_r4k_stamp(modes[m], a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                                   n, n, n, n, n, n, st[m].data_ptr(), stream_handle())
        check(rc, "ntm_gemm_r4k_stamp")

    t_end = time.time() + args.warm_s
    while time.time() < t_end:
        for _ in range(args.iters):
            run(next(iter(modes)))
        torch.cuda.synchronize()
    times = {m: [] for m in modes}
    for _ in range(args.rounds):
        for m in modes:
            run(m)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run(m)
            e1.record()
            torch.cuda.synchronize()
            times[m].append(e0.elapsed_time(e1) / args.iters)
    for m in modes:
        s = st[m].view(nwg * 4, SLOTS).cpu().tolist()
        span = [r[1] - r[0] for r in s]
        rt = [(r[5] - r[4]) for r in s]
        clk = [sp / (r * 10.0) for sp, r in zip(span, rt) if r > 0]  # s_memrealtime is 100 MHz
        loop = [(r[9] - r[8]) / steps for r in s]
        pro = [r[8] - r[0] for r in s]
        epi = [r[1] - r[9] for r in s]
        wait = [r[2] / steps for r in s]
        bar = [r[3] / steps for r in s]
        ms = statistics.median(times[m])
        # per-XCD view of the last launch: end of the XCD's last wave after the
        # kernel's first wave started (s_memrealtime is one 100 MHz clock), and
        # the XCD's median in-kernel clock
        t0 = min(r[4] for r in s)
        xcd_end, xcd_clk = {}, {}
        for r, cl in zip(s, [sp / (max(r[5] - r[4], 1) * 10.0) for sp, r in zip(span, s)]):
            x = r[7] & 0xF
            xcd_end[x] = max(xcd_end.get(x, 0), r[5] - t0)
            xcd_clk.setdefault(x, []).append(cl)
        ends = [xcd_end[x] / 100.0 for x in sorted(xcd_end)]  # us
        clks = [round(statistics.median(xcd_clk[x]), 3) for x in sorted(xcd_clk)]
        print(json.dumps({
            "mode": m, "ms": round(ms, 4), "tflops": round(2 * n ** 3 / ms / 1e9, 1),
            "clock_GHz": round(statistics.median(clk), 3),
            "wave_cycles_per_step": round(statistics.median(span) / steps, 1),
            "loop_cycles_per_step": round(statistics.median(loop), 1),
            "prologue_cycles": round(statistics.median(pro)),
            "epilogue_cycles": round(statistics.median(epi)),
            "wait_per_step": round(statistics.median(wait), 1),
            "wait_p90": round(sorted(wait)[int(0.9 * len(wait))], 1),
            "barrier_per_step": round(statistics.median(bar), 1),
            "barrier_p90": round(sorted(bar)[int(0.9 * len(bar))], 1),
            "mfma_floor_per_step": 2048,
            "xcd_end_us": [round(e, 1) for e in ends], "xcd_end_spread_us": round(max(ends) - min(ends), 1),
            "xcd_clock_GHz": clks, "dtype": args.dtype,
            "c_stores": "temporal" if args.temporal else "nontemporal"}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
