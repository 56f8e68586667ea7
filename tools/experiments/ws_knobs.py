"""Schedule-knob sweep of the wave-specialised tile kernels (developer tool;
gemm_bf16_t128.hpp kWsBFirst / kWsEarly / kWsPrio): every knob is checked
bitwise against knob 0 (same MFMA order), then timed in interleaved rounds
next to the 4-wave tile kernel (tile*w4) and hipBLASLt (torch.matmul) after a clock
settle; one JSON line per (shape, tile).

    python tools/experiments/ws_knobs.py --shapes 8192x8192x8192 --tiles 1 [--knobs 0,1,2,3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

TILES = {0: ("tile128w4", 128, 128), 1: ("tile256x128w4", 256, 128), 2: ("tile160w4", 160, 160)}


def timed(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8192x8192x8192")
    ap.add_argument("--tiles", default="1")
    ap.add_argument("--knobs", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    L = lib_experimental()
    knobs = [int(x) for x in args.knobs.split(",")]
    for sh in args.shapes.split(","):
        m, n, k = (int(x) for x in sh.split("x"))
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        for tsel in (int(x) for x in args.tiles.split(",")):
            name, tm, tn = TILES[tsel]
            if m % tm or n % tn or k % 128:
                continue

            def ws(knob, out=c, tsel=tsel):
                check(L.ntm_gemm_bf16_ws_knob(tsel, knob, a.data_ptr(), b.data_ptr(),
                                              out.data_ptr(), m, n, k, k, k, n, stream_handle()),
                      "ntm_gemm_bf16_ws_knob")
            base = torch.empty_like(c)
            ws(0, base)
            bitwise = {}
            for kn in knobs:
                o = torch.empty_like(c)
                ws(kn, o)
                bitwise[kn] = bool(torch.equal(o, base))
            fns = {"torch": lambda: torch.matmul(a, b.T, out=c),
                   name: lambda name=name: ops.gemm_bf16(a, b, c, variant=name)}
            for kn in knobs:
                fns[f"ws{kn}"] = lambda kn=kn: ws(kn)
            for _ in range(200):  # clock settle
                fns["torch"]()
            t = {x: [] for x in fns}
            for _ in range(args.rounds):
                for x, fn in fns.items():
                    t[x].append(timed(fn, args.iters))
            fl = 2.0 * m * n * k
            row = {"shape": [m, n, k], "tile": name, "bitwise_vs_knob0": bitwise}
            for x, v in t.items():
                v.sort()
                row[f"{x}_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
