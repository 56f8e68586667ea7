"""Quick K1 numerics + throughput check on one MI355X (developer tool).

    python tools/gemm_check.py [--sizes 4096,8192] [--iters 50]

Prints one JSON line per size with: max error vs the fp32 reference kernel and
vs torch (hipBLASLt) fp32, our TFLOP/s and torch.matmul's TFLOP/s on the same
uniform [-1,1) data (interleaved rounds in one process, playbook rule 24).
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
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    print(json.dumps({"device": torch.cuda.get_device_name(0), "lib": ops.version()}), flush=True)
    for s in [int(x) for x in args.sizes.split(",")]:
        m = n = k = s
        a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
        b = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
        ops.fill_uniform_(a, seed=1)
        ops.fill_uniform_(b, seed=2)
        c = ops.gemm_bf16(a, b)
        torch.cuda.synchronize()
        atol, rtol = ops.gemm_tolerance(k)
        ref = ops.ref_gemm_f32(a, b)
        rep = ops.verify_bf16(c, ref, atol, rtol)
        tref = a.float() @ b.float().T
        err_torch = (c.float() - tref).abs().max().item()
        del tref
        flops = 2.0 * m * n * k
        ours, theirs = [], []
        cc = torch.empty_like(c)
        for _ in range(args.rounds):
            ours.append(timed(lambda: ops.gemm_bf16(a, b, cc), args.iters))
            theirs.append(timed(lambda: torch.matmul(a, b.T, out=cc), args.iters))
        print(json.dumps({
            "size": s, "verify": rep.as_dict(), "max_err_vs_torch_fp32": err_torch,
            "ours_ms": min(ours), "ours_tflops": flops / min(ours) / 1e9,
            "torch_ms": min(theirs), "torch_tflops": flops / min(theirs) / 1e9,
            "ours_all_ms": ours, "torch_all_ms": theirs,
        }), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
