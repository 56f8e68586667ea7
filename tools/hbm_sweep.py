"""Sweep the K2 HBM stream kernels (unroll x cache policy x grid) on one
MI355X and compare with torch's copy_. GB/s counts read + write bytes for
copies (the STREAM convention) and read bytes for reads."""
import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nvidia_terraform_modules_amd import ops


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    nbytes = int(args.gib * 2**30) // 4096 * 4096
    src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda")
    ops.fill_uniform_(src, seed=7)
    dst = torch.empty_like(src)
    sink = torch.zeros(1 << 16, dtype=torch.float32, device="cuda")
    rows = []

    def rec(kind, cfg, t, mult):
        gbps = mult * nbytes / t / 1e9
        rows.append({"kind": kind, "cfg": cfg, "ms": round(t * 1e3, 3), "GBps": round(gbps, 1)})
        print(json.dumps(rows[-1]), flush=True)

    rec("copy", "torch.copy_", timed(lambda: dst.copy_(src), args.iters), 2)
    rec("copy", "legacy", timed(lambda: ops.stream_copy(src, dst, config=None), args.iters), 2)
    rec("read", "legacy", timed(lambda: ops.stream_read(src, sink, config=None), args.iters), 1)
    for u, pol, grid in itertools.product((2, 4, 8), (1, 3, 5, 7), (0, 256, 512, 1024, 2048, 4096)):
        cfg = (u, pol, grid)
        rec("copy", list(cfg), timed(lambda: ops.stream_copy(src, dst, config=cfg), args.iters), 2)
    for u, pol, grid in itertools.product((2, 4, 8, 16), (0, 1), (0, 1024, 2048, 4096)):
        cfg = (u, pol, grid)
        rec("read", list(cfg), timed(lambda: ops.stream_read(src, sink, config=cfg), args.iters), 1)
    # correctness of the best copy
    best = max((r for r in rows if r["kind"] == "copy" and isinstance(r["cfg"], list)),
               key=lambda r: r["GBps"])
    dst.zero_()
    ops.stream_copy(src, dst, config=tuple(best["cfg"]))
    assert torch.equal(src, dst), "tuned copy mismatch"
    bestr = max((r for r in rows if r["kind"] == "read" and isinstance(r["cfg"], list)),
                key=lambda r: r["GBps"])
    print("BEST", json.dumps({"copy": best, "read": bestr}))


if __name__ == "__main__":
    main()
