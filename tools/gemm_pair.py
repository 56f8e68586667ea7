"""Run our K1 GEMM and torch.matmul (hipBLASLt) back to back on the same
random operands - a profiling target for rocprofv3 (developer tool).

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/gemm_pair.py --size 8192 --iters 20
    (--variant A --versus B: two K1 variants instead of K1 vs hipBLASLt)
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--shape", default="", help="MxNxK instead of --size (e.g. 8192x8192x4096)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--which", default="both", choices=["both", "ours", "torch", "all"])
    ap.add_argument("--variant", default="default")
    ap.add_argument("--versus", default="",
                    help="a second K1 variant to run in place of torch.matmul (e.g. tile256x128w4)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--knob", type=int, default=0,
                    help="fp8: experimental K1-fp8 schedule knob for 'ours' (--which all adds the default)")
    ap.add_argument("--warm-iters", type=int, default=40,
                    help="untimed pairs first, so most profiled dispatches run on a settled chip")
    args = ap.parse_args()
    args.iters += args.warm_iters
    m, n, k = (int(x) for x in args.shape.split("x")) if args.shape else (args.size,) * 3
    if args.dtype == "fp8":
        return fp8_pair((m, n, k), args.iters, args.which, args.knob)
    a = torch.empty((m, k), dtype=torch.bfloat16, device="cuda")
    b = torch.empty((n, k), dtype=torch.bfloat16, device="cuda")
    c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
    ops.fill_uniform_(a, 1)
    ops.fill_uniform_(b, 2)
    for _ in range(args.iters):
        if args.which in ("both", "ours", "all"):
            ops.gemm_bf16(a, b, c, variant=args.variant)
        if args.which == "all":
            ops.gemm_bf16(a, b, c, variant="pingpong8")
        if args.which in ("both", "torch", "all"):
            if args.versus:
                ops.gemm_bf16(a, b, c, variant=args.versus)
            else:
                torch.matmul(a, b.T, out=c)
    torch.cuda.synchronize()
    return 0


def fp8_pair(shape, iters: int, which: str, knob: int = 0) -> int:
    """K1-fp8 vs hipBLASLt's fp8 GEMM (torch._scaled_mm, unit scales, bf16 out)."""
    m, n, k = shape
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 1)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 2)
    c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
    one = torch.ones((), device="cuda")
    for _ in range(iters):
        if which in ("both", "ours", "all"):
            ops.gemm_fp8(a, b, c, knob=knob)
        if which == "all" and knob:
            ops.gemm_fp8(a, b, c)
        if which in ("both", "torch", "all"):
            torch._scaled_mm(a, b.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
