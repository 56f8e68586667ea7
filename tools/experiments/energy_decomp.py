"""Where K1's joules go at 8192^3 (developer diagnostic, round 6).

K1 bf16 is power-bound at 8192^3, so its speed is set by its energy per launch.
This runs the ablation builds of pingpong8c (gemm_bf16_pp3_stamp.hpp modes
0-5: real, no LDS traffic, no MFMA, MFMA only, fragment reads without LDS-DMA,
LDS-DMA without fragment reads) plus the shipping pingpong8o and its no-C-store
build, each for an AMD SMI energy window of back-to-back launches, and reports
per build: microseconds per launch (HIP events, interleaved rounds), the
in-kernel clock (stamp builds), average package power, millijoules per launch,
and the same above the idle floor (a window with the GPU idle).

The builds run at different clocks and so at different voltages: differences of
millijoules between them are an approximate split, not an exact one.

    python tools/experiments/energy_decomp.py [--window-s 0.6] [--rounds 5]
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

STAMP_MODES = {"pp8c_real": 0, "pp8c_no_lds": 1, "pp8c_no_mfma": 2, "pp8c_mfma_only": 3,
               "pp8c_reads_no_dma": 4, "pp8c_dma_no_reads": 5}
PP6 = {"pp8o_shipping": "pingpong8o", "pp8o_nostore": "pp8o_nostore"}
SLOTS, START, END, RT0, RT1 = 8, 0, 1, 2, 3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--window-s", type=float, default=0.6)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()
    n = args.size
    dev = torch.device("cuda:0")
    a = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device=dev), 1)
    b = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device=dev), 2)
    c = torch.empty((n, n), dtype=torch.bfloat16, device=dev)
    nwg = (n // 256) ** 2
    st = {m: torch.zeros(nwg * 8 * SLOTS, dtype=torch.int64, device=dev) for m in STAMP_MODES}
    L = lib_experimental()

    def stamp_fn(m):
        def f():
            check(L.ntm_gemm_bf16_stamp(STAMP_MODES[m], a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                        n, n, n, n, n, n, st[m].data_ptr(), stream_handle()),
                  "ntm_gemm_bf16_stamp")
        return f

    fns = {m: stamp_fn(m) for m in STAMP_MODES}
    for k, v in PP6.items():
        fns[k] = (lambda v=v: ops.gemm_bf16(a, b, c, variant=v))

    def sync():
        torch.cuda.synchronize(dev)

    # idle floor: the same SMI window with nothing queued
    sync()
    time.sleep(0.5)
    i0 = smi.sample(dev)
    time.sleep(1.0)
    i1 = smi.sample(dev)
    idle = smi.window(i0, i1)
    idle_w = idle.get("avg_power_W")
    print(json.dumps({"idle": {"avg_power_W": idle_w, "seconds": idle.get("seconds")}}), flush=True)

    bench.prewarm_settle(fns["pp8o_shipping"], sync, 1.0)
    timing = bench.interleaved_compare(fns, dev, rounds=args.rounds, launches=args.launches)
    names = list(fns)
    power = {k: [] for k in names}
    for r in range(2):   # two energy windows per build, the order reversed in the second pass
        for k in (names if r == 0 else names[::-1]):
            bench.prewarm_settle(fns[k], sync, 0.2)
            bw, aw, _ = bench.power_window(fns[k], sync, lambda: smi.sample(dev), args.window_s,
                                           chunk=bench.POWER_WINDOW_CHUNK)
            w = smi.window(bw, aw)
            power[k].append(w)
            print(json.dumps({"window": k, "pass": r, "avg_power_W": w.get("avg_power_W"),
                              "ppt_pct": w.get("ppt_pct"), "gfxclk_mhz": w.get("gfxclk_mhz")}),
                  flush=True)
    rows = {}
    for k in names:
        s_per = timing[k]["median_s"]
        ws = [w.get("avg_power_W") for w in power[k] if w.get("avg_power_W") is not None]
        pw = statistics.mean(ws) if ws else None
        clk = None
        if k in st:
            s = st[k].view(nwg, 8, SLOTS).cpu().double()
            clk = round(float(((s[:, :, END] - s[:, :, START]) /
                               ((s[:, :, RT1] - s[:, :, RT0]) / 100e6)).median()) / 1e9, 3)
        rows[k] = {"us_per_launch": round(s_per * 1e6, 1),
                   "tflops": round(2 * n ** 3 / s_per / 1e12, 1), "clock_GHz": clk,
                   "avg_power_W": round(pw, 1) if pw else None,
                   "mJ_per_launch": round(pw * s_per * 1e3, 1) if pw else None,
                   "mJ_above_idle": round((pw - idle_w) * s_per * 1e3, 1) if pw and idle_w else None,
                   "ppt_pct": [w.get("ppt_pct") for w in power[k]],
                   "gfxclk_mhz_end": [(w.get("gfxclk_mhz") or [None, None])[1] for w in power[k]]}
    print(json.dumps({"size": n, "idle_W": idle_w, "rows": rows}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
