"""Split GEMM time into K-loop cost and fixed per-tile overhead: time at
fixed M = N over several K, least-squares fit t = a + b * K, for our K1 and
for torch.matmul (hipBLASLt); --dtype fp8: K1-fp8 vs torch._scaled_mm. Interleaved rounds, CUDA events."""
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
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mn", type=int, default=4096)
    ap.add_argument("--ks", default="1024,2048,4096,8192,16384")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variant", default="default")
    ap.add_argument("--knob", type=int, default=0, help="fp8: experimental K1-fp8 schedule knob")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    args = ap.parse_args()
    fp8 = args.dtype == "fp8"
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    one = torch.ones((), device="cuda")
    mn = args.mn
    ks = [int(k) for k in args.ks.split(",")]
    res = {}
    for k in ks:
        a = ops.fill_uniform_(torch.empty((mn, k), dtype=dt, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((mn, k), dtype=dt, device="cuda"), 2)
        c = torch.empty((mn, mn), dtype=torch.bfloat16, device="cuda")
        ours, theirs = [], []
        for _ in range(args.rounds):
            if fp8:
                ours.append(timed(lambda: ops.gemm_fp8(a, b, c, knob=args.knob), 20))
                theirs.append(timed(lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                             out_dtype=torch.bfloat16), 20))
            else:
                ours.append(timed(lambda: ops.gemm_bf16(a, b, c, variant=args.variant), 20))
                theirs.append(timed(lambda: torch.matmul(a, b.T, out=c), 20))
        res[k] = (sorted(ours)[len(ours) // 2], sorted(theirs)[len(theirs) // 2])
        print(json.dumps({"k": k, "ours_us": res[k][0], "torch_us": res[k][1],
                          "ours_tf": 2 * mn * mn * k / res[k][0] / 1e6,
                          "torch_tf": 2 * mn * mn * k / res[k][1] / 1e6}), flush=True)
    for name, idx in (("ours", 0), ("torch", 1)):
        xs = ks
        ys = [res[k][idx] for k in ks]
        n = len(xs)
        mx, my = sum(xs) / n, sum(ys) / n
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        a = my - b * mx
        loop_tf = 2 * mn * mn / (b * 1e-6) / 1e12
        print(json.dumps({"fit": name, "fixed_us": round(a, 2), "us_per_k": b,
                          "loop_only_tflops": round(loop_tf, 1)}), flush=True)


if __name__ == "__main__":
    main()
