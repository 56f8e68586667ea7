"""Sweep the K2 HBM stream kernels (unroll x cache policy x grid x buffer
size) on one MI355X against torch's copy_, in INTERLEAVED rounds (median and
best per config, one process - cdna_hip_programming.md §5.4 rule 24), and
check every copy config bytewise. GB/s counts read + write bytes for copies
(the STREAM convention) and read bytes for reads."""
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
    ap.add_argument("--gib", default="1,2", help="comma list of buffer sizes (GiB each)")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5, help="interleaved rounds (median reported)")
    ap.add_argument("--grids", default="256,384,512,768,1024",
                    help="comma list; 'tiles' = one block per tile (no grid-stride loop)")
    ap.add_argument("--unrolls", default="2,4,8")
    ap.add_argument("--policies", default="3,7,11",
                    help="copy policy ids (bit0 nt load, bit1 nt store, bit2 pipelined, 8+ chunked)")
    ap.add_argument("--no-read", action="store_true", help="copies only")
    args = ap.parse_args()
    import statistics

    grids = args.grids.split(",")
    unrolls = [int(u) for u in args.unrolls.split(",")]
    policies = [int(p) for p in args.policies.split(",")]
    for gib in [float(x) for x in args.gib.split(",")]:
        nbytes = int(gib * 2**30) // 65536 * 65536
        src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda")
        ops.fill_uniform_(src, seed=7)
        dst = torch.empty_like(src)
        sink = torch.zeros(1 << 16, dtype=torch.float32, device="cuda")
        copies = {"torch.copy_": lambda: dst.copy_(src),
                  "tuned-default": lambda: ops.stream_copy(src, dst),
                  "copy 1,0,0 (grid-stride baseline)": lambda: ops.stream_copy(src, dst, config=None)}
        for u, pol, g in itertools.product(unrolls, policies, grids):
            grid = nbytes // 16 // (256 * u) if g == "tiles" else int(g)
            copies[f"copy {u},{pol},{g}"] = lambda c=(u, pol, grid): ops.stream_copy(src, dst, config=c)
        reads = {"tuned-default": lambda: ops.stream_read(src, sink)}
        for u, pol, grid in itertools.product((4, 8, 16), (1,), (0, 512, 1024, 2048)):
            reads[f"read {u},{pol},{grid}"] = lambda c=(u, pol, grid): ops.stream_read(src, sink, config=c)
        kinds = (("copy", copies, 2),) if args.no_read else (("copy", copies, 2), ("read", reads, 1))
        for kind, cands, mult in kinds:
            ts = {k: [] for k in cands}
            for _ in range(args.rounds):
                for k, fn in cands.items():
                    ts[k].append(timed(fn, args.iters))
            rows = sorted(({"gib": gib, "kind": kind, "cfg": k,
                            "GBps_median": round(mult * nbytes / statistics.median(v) / 1e9, 1),
                            "GBps_best": round(mult * nbytes / min(v) / 1e9, 1)}
                           for k, v in ts.items()), key=lambda r: -r["GBps_median"])
            for r in rows:
                print(json.dumps(r), flush=True)
        for k, fn in copies.items():
            dst.zero_()
            fn()
            torch.cuda.synchronize()
            assert torch.equal(src, dst), f"copy mismatch: {k}"
        print(json.dumps({"gib": gib, "all_copies_bytewise_equal": True, "n": len(copies)}),
              flush=True)
        del src, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
