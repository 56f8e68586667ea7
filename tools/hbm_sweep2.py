"""K2 copy sweep, round 2: the chunked kernel (policy 8-11: contiguous span per
block, one-tile-ahead pipeline; bit 0 nontemporal loads, bit 1 nontemporal
stores) against the current default (4, 7, 256), interleaved rounds in one
process on 4 GiB. GB/s counts read + write bytes (STREAM convention)."""
import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nvidia_terraform_modules_amd import ops  # noqa: E402


def timed(fn, iters):
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    nbytes = int(args.gib * 2**30) // 4096 * 4096
    src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda")
    ops.fill_uniform_(src, seed=7)
    dst = torch.empty_like(src)
    cfgs = [(4, 7, 256), (4, 7, 512), (8, 7, 256), (2, 7, 1024)]
    cfgs += list(itertools.product((2, 4, 8), (8, 9, 10, 11), (256, 512, 1024, 2048)))
    res = {c: [] for c in cfgs}
    res["torch"] = []
    for c in cfgs:   # warm + correctness
        dst.zero_()
        ops.stream_copy(src, dst, config=c)
        torch.cuda.synchronize()
        assert torch.equal(src, dst), f"copy mismatch {c}"
    for _ in range(args.rounds):
        for c in cfgs:
            res[c].append(timed(lambda: ops.stream_copy(src, dst, config=c), args.iters))
        res["torch"].append(timed(lambda: dst.copy_(src), args.iters))
    rows = []
    for c, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        rows.append({"cfg": list(c) if c != "torch" else c, "GBps": round(2 * nbytes / t / 1e9, 1)})
        print(json.dumps(rows[-1]), flush=True)
    print("BEST", json.dumps(max(rows, key=lambda r: r["GBps"])))


if __name__ == "__main__":
    main()
