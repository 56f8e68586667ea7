"""Row-stride sensitivity of K1 vs hipBLASLt: C[M x N] = A B^T at M = N = --mn
for each K, with the operand rows padded by 0 / 64 / 128 / ... elements (the
tensor is a K-wide view of a (K + pad)-wide buffer, so lda = ldb = K + pad).
A power-of-two row pitch maps the same K column of every row to one memory
channel; padding spreads it. Interleaved rounds, median, CUDA events.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mn", type=int, default=8192)
    ap.add_argument("--ks", default="8192,16384")
    ap.add_argument("--pads", default="0,64")
    ap.add_argument("--variants", default="default")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--knobs", default="0", help="fp8: K1-fp8 knobs to time")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    fp8 = args.dtype == "fp8"
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    one = torch.ones((), device="cuda")
    mn = args.mn
    names = ([f"knob{k}" for k in args.knobs.split(",")] if fp8 else args.variants.split(","))
    for k in [int(x) for x in args.ks.split(",")]:
        for pad in [int(x) for x in args.pads.split(",")]:
            abuf = ops.fill_uniform_(torch.empty((mn, k + pad), dtype=dt, device="cuda"), 1)
            bbuf = ops.fill_uniform_(torch.empty((mn, k + pad), dtype=dt, device="cuda"), 2)
            a, b = abuf[:, :k], bbuf[:, :k]
            c = torch.empty((mn, mn), dtype=torch.bfloat16, device="cuda")
            fns = {}
            for nm in names:
                if fp8:
                    kn = int(nm[4:])
                    fns[nm] = lambda kn=kn: ops.gemm_fp8(a, b, c, knob=kn)
                else:
                    fns[nm] = lambda nm=nm: ops.gemm_bf16(a, b, c, variant=nm)
            if fp8:
                fns["torch"] = lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                        out_dtype=torch.bfloat16)
            else:
                fns["torch"] = lambda: torch.matmul(a, b.T, out=c)
            res = {nm: [] for nm in fns}
            for _ in range(args.rounds):
                for nm, fn in fns.items():
                    res[nm].append(timed(fn, args.iters))
            out = {"k": k, "pad": pad}
            for nm, ts in res.items():
                med = sorted(ts)[len(ts) // 2]
                out[nm + "_tflops"] = round(2 * mn * mn * k / med / 1e6, 1)
            print(json.dumps(out), flush=True)
            del abuf, bbuf, a, b, c
    return 0


if __name__ == "__main__":
    sys.exit(main())
