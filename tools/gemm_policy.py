"""Default-variant policy check (developer tool): interleaved timing of the
256x256 kernel (pingpong8c), the 128x128 / 256x128 kernels (tile128,
tile256x128), the default
dispatch and hipBLASLt (torch.matmul) on M x N x K shapes; one JSON line each.

    python tools/gemm_policy.py --shapes 2048x2048x2048,4096x2048x4096 [--rounds 7]
    python tools/gemm_policy.py --dtype fp8 --random 40   # K1-fp8 default vs hipBLASLt fp8
    python tools/gemm_policy.py --shapes 4672x1472x6696 --variants tile256x128,tile128x256

--dtype fp8 times the K1-fp8 default dispatch, its 256x256 kernel alone
("pingpong8c") and hipBLASLt's fp8 GEMM (torch._scaled_mm, unit scales, bf16
out) on e4m3 operands; random shapes then use K % 16.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nvidia_terraform_modules_amd import ops  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="2048x2048x2048")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only-default", action="store_true",
                    help="time the default dispatch and hipBLASLt only (shape sweeps)")
    ap.add_argument("--random", type=int, default=0,
                    help="append N random shapes (M, N, K multiples of 8 in [256, 8192], seeded)")
    ap.add_argument("--seed", type=int, default=20261016, help="seed of the --random draws")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"))
    ap.add_argument("--variants", default="",
                    help="time exactly these variants (masked tiles on any shape) besides "
                         "the default and hipBLASLt")
    args = ap.parse_args()
    shapes = [tuple(int(x) for x in sh.split("x")) for sh in args.shapes.split(",") if sh]
    if args.random:
        import random
        rng = random.Random(args.seed)
        shapes += [tuple(rng.randrange(256, 8193, 8) for _ in range(3)) for _ in range(args.random)]
        if args.dtype == "fp8":   # same draws; N, K rounded up to 16 (torch._scaled_mm's rule)
            shapes = [(m, (n + 15) // 16 * 16, (k + 15) // 16 * 16) for m, n, k in shapes]
    if args.dtype == "fp8":
        return fp8_sweep(shapes, args)
    for m, n, k in shapes:
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        fns = {"default": lambda: ops.gemm_bf16(a, b, c),
               "torch": lambda: torch.matmul(a, b.T, out=c)}
        exact_k = k % 128 == 0
        if args.variants:
            for v in args.variants.split(","):
                if v.startswith("pingpong8s") and not ops.sk_ws_bytes(m, n, k):
                    continue  # stream-K serves only a partial round past the first
                fns[v] = lambda v=v: ops.gemm_bf16(a, b, c, variant=v)
        elif not args.only_default:
            if m % 128 == 0 and n % 128 == 0:
                fns["tile128"] = lambda: ops.gemm_bf16(a, b, c, variant="tile128")
            if m % 256 == 0 and n % 256 == 0 and exact_k:
                fns["pingpong8c"] = lambda: ops.gemm_bf16(a, b, c, variant="pingpong8c")
            for v, (tm, tn) in ops.kernels.TILE_SHAPES.items():
                if v != "tile128" and m % tm == 0 and n % tn == 0 and (
                        exact_k or v in ops.kernels.MASKED_TILES):
                    fns[v] = lambda v=v: ops.gemm_bf16(a, b, c, variant=v)
        t = {name: [] for name in fns}
        for _ in range(args.rounds):
            for name, fn in fns.items():
                t[name].append(timed(fn, args.iters))
        fl = 2.0 * m * n * k
        row = {"shape": [m, n, k], "tiles256": (m // 256) * (n // 256),
               "plan": list(ops.kernels.k1_splitk_plan(m, n, k))}
        for name, v in t.items():
            v.sort()
            row[f"{name}_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
        print(json.dumps(row), flush=True)


def fp8_sweep(shapes, args):
    one = torch.ones((), device="cuda")
    for m, n, k in shapes:
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        fns = {"default": lambda: ops.gemm_fp8(a, b, c),
               "pingpong8c": lambda: ops.gemm_fp8(a, b, c, variant="pingpong8c"),
               "hipblaslt": lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                     out_dtype=torch.bfloat16)}
        if args.variants:
            for v in args.variants.split(","):
                fns[v] = lambda v=v: ops.gemm_fp8(a, b, c, variant=v)
        elif not args.only_default:   # every fp8 tile alone (wave-specialised, masked edges)
            for v in ("tile256x128", "tile160", "tile128", "tile160x128", "tile128x160",
                      "tile128x256"):
                fns[v] = lambda v=v: ops.gemm_fp8(a, b, c, variant=v)
        t = {name: [] for name in fns}
        for _ in range(args.rounds):
            for name, fn in fns.items():
                t[name].append(timed(fn, args.iters))
        fl = 2.0 * m * n * k
        row = {"dtype": "fp8", "shape": [m, n, k], "plan": list(ops.k1_fp8_splitk_plan(m, n, k))}
        for name, v in t.items():
            v.sort()
            row[f"{name}_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
        row["default_over_hipblaslt"] = round(row["default_tflops"] / row["hipblaslt_tflops"], 3)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    main()
