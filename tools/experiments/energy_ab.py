"""Joules per TFLOP of K1 builds against hipBLASLt, bf16 and fp8 (developer
diagnostic, profiles/r6_fp8): the shipping default, one alternative build
(bf16 variant / fp8 knob) and hipBLASLt on the same operands. Throughput is
the interleaved median (bench.interleaved_compare); energy comes from AMD SMI
windows of >= --window-s of one kernel each, in palindromic order (A B C C B A)
so no kernel always runs on the warmer chip; J/TFLOP = mean window power / TF/s.

    python tools/experiments/energy_ab.py [--bf16-alt dma4k_d3[,OTHER,...]] [--fp8-knob 12]
    (--fp8-knob 0 skips the fp8 comparison)
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

import bench  # noqa: E402
from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops import smi  # noqa: E402


def measure(fns: dict, flops: float, dev, rounds: int, iters: int, window_s: float) -> dict:
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    bench.prewarm_settle(next(iter(fns.values())), sync, 0.3)
    cmp_ = bench.interleaved_compare(fns, dev, rounds, iters)
    tf = {k: flops / v["median_s"] / 1e12 for k, v in cmp_.items()}
    names = list(fns)
    order = names + names[::-1]
    win: dict = {k: [] for k in names}
    for k in order:
        bench.prewarm_settle(fns[k], sync, 0.2)
        b, a, _ = bench.power_window(fns[k], sync, lambda: smi.sample(dev), window_s,
                                     chunk=bench.POWER_WINDOW_CHUNK)
        win[k].append(smi.window(b, a))
    out = {}
    for k in names:
        ws = [w.get("avg_power_W") for w in win[k] if w.get("avg_power_W")]
        p = statistics.mean(ws) if ws else None
        out[k] = {"tflops": round(tf[k], 1), "avg_power_W": round(p, 1) if p else None,
                  "joules_per_tflop": round(p / tf[k], 4) if p else None,
                  "ppt_pct": [w.get("ppt_pct") for w in win[k]],
                  "gfxclk_mhz": [(w.get("gfxclk_mhz") or [None, None])[1] for w in win[k]]}
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--bf16-alt", default="dma4k_d3")
    ap.add_argument("--fp8-knob", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--window-s", type=float, default=0.6)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    smi.sample(dev)
    n = args.size
    fl = 2.0 * n ** 3
    a = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device=dev), 1)
    b = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device=dev), 2)
    c = torch.empty((n, n), dtype=torch.bfloat16, device=dev)
    ref = ops.gemm_bf16(a, b)
    alts = [v for v in args.bf16_alt.split(",") if v]
    ok = {}
    for v in alts:
        alt = ops.gemm_bf16(a, b, variant=v)
        ok[v] = bool(torch.equal(alt, ref)) or bool(
            ((alt.float() - ref.float()).abs() <= 1e-2 * (1 + ref.float().abs())).all())
    fns = {"default": lambda: ops.gemm_bf16(a, b, c)}
    for v in alts:
        fns[v] = (lambda v=v: ops.gemm_bf16(a, b, c, variant=v))
    fns["hipblaslt"] = lambda: torch.matmul(a, b.T, out=c)
    res = measure(fns, fl, dev, args.rounds, args.iters, args.window_s)
    print(json.dumps({"dtype": "bf16", "size": n, "alt_ok": ok, **res}), flush=True)
    del a, b, ref
    if not args.fp8_knob:
        return 0
    a8 = ops.fill_uniform_(torch.empty((n, n), dtype=torch.float8_e4m3fn, device=dev), 3)
    b8 = ops.fill_uniform_(torch.empty((n, n), dtype=torch.float8_e4m3fn, device=dev), 4)
    ref = ops.gemm_fp8(a8, b8)
    alt = ops.gemm_fp8(a8, b8, knob=args.fp8_knob)
    ok = bool(((alt.float() - ref.float()).abs() <= 1e-2 * (1 + ref.float().abs())).all())
    one = torch.ones((), device=dev)
    res = measure({"default": lambda: ops.gemm_fp8(a8, b8, c),
                   f"knob{args.fp8_knob}": lambda: ops.gemm_fp8(a8, b8, c, knob=args.fp8_knob),
                   "hipblaslt": lambda: torch._scaled_mm(a8, b8.T, scale_a=one, scale_b=one,
                                                         out_dtype=torch.bfloat16)},
                  fl, dev, args.rounds, args.iters, args.window_s)
    print(json.dumps({"dtype": "fp8", "size": n, "alt_ok": ok, **res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
