"""K1-fp8 numerics + throughput on one MI355X (developer tool).

For every size: verification of ops.gemm_fp8 against an fp32 matmul of the
same e4m3 values, then interleaved timing rounds of K1-fp8, K1-bf16 (same
shape) and, when this PyTorch build supports it on the device, hipBLASLt's
fp8 GEMM through torch._scaled_mm (unit scales, bf16 out). One JSON line per
size.

    python tools/gemm_fp8_check.py [--sizes 4096,8192,6144x8192x4096] [--iters 50] [--rounds 7]
        [--knobs 31] [--variants tile256x128,tile128x256] [--no-bf16]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402


def timed(fn, iters: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--knobs", default="", help="comma list of experimental fp8 knobs to time too")
    ap.add_argument("--no-bf16", action="store_true", help="skip the bf16 K1 / hipBLASLt timings")
    ap.add_argument("--variants", default="",
                    help="comma list of K1-fp8 variants (ops.FP8_VARIANTS) to time next to the "
                         "default plan, each verified bitwise-equal-or-within-tolerance first")
    args = ap.parse_args()
    knobs = [int(x) for x in args.knobs.split(",") if x]
    variants = [v for v in args.variants.split(",") if v]
    dev = torch.device("cuda:0")
    ok_all = True
    for size in args.sizes.split(","):
        m, n, k = (int(x) for x in size.split("x")) if "x" in size else (int(size),) * 3
        s = int(size) if "x" not in size else size
        g = torch.Generator(device=dev).manual_seed(m * 7 + n * 3 + k)
        a = (torch.rand((m, k), generator=g, device=dev) * 2 - 1).to(torch.float8_e4m3fn)
        b = (torch.rand((n, k), generator=g, device=dev) * 2 - 1).to(torch.float8_e4m3fn)
        c = ops.gemm_fp8(a, b)
        ref = a.float() @ b.float().T
        atol, rtol = ops.gemm_tolerance(k)
        err = (c.float() - ref).abs()
        bad = int((err > atol + rtol * ref.abs()).sum())
        del ref, err
        ok_all &= bad == 0
        fns = {"ours_fp8": lambda: ops.gemm_fp8(a, b, c)}
        if not args.no_bf16:
            ab = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=dev), 1)
            bb = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=dev), 2)
            cb = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
            fns["ours_bf16"] = lambda: ops.gemm_bf16(ab, bb, cb)
        for kn in knobs:
            ck = ops.gemm_fp8(a, b, knob=kn)
            kbad = int(((ck.float() - c.float()).abs() > 1e-2 * (1 + c.float().abs())).sum())
            ok_all &= kbad == 0
            print(json.dumps({"size": s, "knob": kn, "mismatch_vs_default": kbad}), flush=True)
            fns[f"knob{kn}_fp8"] = (lambda kn=kn: ops.gemm_fp8(a, b, c, knob=kn))
        for v in variants:
            cv = ops.gemm_fp8(a, b, variant=v)
            vbad = int(((cv.float() - c.float()).abs() > 1e-2 * (1 + c.float().abs())).sum())
            ok_all &= vbad == 0
            print(json.dumps({"size": s, "variant": v, "mismatch_vs_default": vbad}), flush=True)
            fns[f"{v}_fp8"] = (lambda v=v: ops.gemm_fp8(a, b, c, variant=v))
        one = torch.ones((), device=dev)
        try:
            torch._scaled_mm(a, b.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            fns["hipblaslt_fp8"] = lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                            out_dtype=torch.bfloat16)
            hb_note = "torch._scaled_mm"
        except Exception as exc:  # not every build/device pairs support e4m3fn
            hb_note = f"unavailable: {type(exc).__name__}: {str(exc)[:120]}"
        if not args.no_bf16:
            fns["hipblaslt_bf16"] = lambda: torch.matmul(ab, bb.T, out=cb)
        times = {k: [] for k in fns}
        for _ in range(args.rounds):
            for name, fn in fns.items():
                times[name].append(timed(fn, args.iters))
        flops = 2.0 * m * n * k
        res = {"size": s, "fp8_bad": bad, "hipblaslt_fp8": hb_note}
        for name, t in times.items():
            t = sorted(t)
            res[f"{name}_tflops_med"] = round(flops / t[len(t) // 2] / 1e9, 1)
        print(json.dumps(res), flush=True)
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
