"""K2 copy: does the store cache policy matter? The shipping copy (one-tile-
ahead pipeline, nontemporal loads + nontemporal stores) against the same
kernel with the store's sc0 / sc1 / nt modifiers spelled out in asm
(libntm_experimental.so ntm_stream_copy_spol). Interleaved rounds, median,
every config checked bytewise. GB/s = (read + write) bytes / time."""
import argparse
import ctypes
import itertools
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

SPOL = {0: "none", 1: "nt", 2: "sc1", 3: "sc0 sc1", 4: "nt sc1", 5: "nt sc0 sc1"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", default="1,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    L = lib_experimental()
    fn = L.ntm_stream_copy_spol
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    for gib in [float(x) for x in args.gib.split(",")]:
        nbytes = int(gib * 2**30) // 65536 * 65536
        src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda")
        ops.fill_uniform_(src, seed=7)
        dst = torch.empty_like(src)
        cands = {"shipping (8,7,512)": lambda: ops.stream_copy(src, dst),
                 "torch.copy_": lambda: dst.copy_(src)}
        for u, sp, grid in itertools.product((4, 8), SPOL, (256, 512)):
            cands[f"u{u} store[{SPOL[sp]}] g{grid}"] = (
                lambda a=(u, sp, grid): check(fn(src.data_ptr(), dst.data_ptr(), nbytes, *a,
                                                 stream_handle()), "spol"))
        for k, f in cands.items():
            dst.zero_()
            f()
            torch.cuda.synchronize()
            assert torch.equal(src, dst), f"copy mismatch: {k}"
        ts = {k: [] for k in cands}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(args.rounds):
            for k, f in cands.items():
                f()
                ev[0].record()
                for _ in range(args.iters):
                    f()
                ev[1].record()
                ev[1].synchronize()
                ts[k].append(ev[0].elapsed_time(ev[1]) / args.iters * 1e-3)
        rows = sorted(({"gib": gib, "cfg": k,
                        "GBps_median": round(2 * nbytes / statistics.median(v) / 1e9, 1),
                        "GBps_best": round(2 * nbytes / min(v) / 1e9, 1)} for k, v in ts.items()),
                      key=lambda r: -r["GBps_median"])
        for r in rows:
            print(json.dumps(r), flush=True)
        del src, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
