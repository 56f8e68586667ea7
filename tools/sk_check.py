"""Stream-K tile kernels (developer tool; gemm_bf16_sk.hpp): correctness vs an
fp32 reference, repeat stability (every repeat bitwise equal to the first,
with HBM noise on a second stream), then interleaved timing against the
wave-specialised tile kernel, the default dispatch and hipBLASLt; one JSON
line per (shape, tile, grid).

    python tools/sk_check.py --shapes 3200x3200x3200 --tiles 2 [--grids 256]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402

TILES = {0: ("tile128", 128, 128), 1: ("tile256x128", 256, 128), 2: ("tile160", 160, 160)}


class StreamK:
    """Workspace + epoch counter for one (tile, grid)."""

    def __init__(self, tsel: int, grid: int, dev):
        self.L = lib_experimental()
        self.tsel, self.grid, self.epoch = tsel, grid, 0
        self.part = torch.empty(self.L.ntm_gemm_bf16_sk_bytes(tsel, grid, 0) // 4,
                                dtype=torch.float32, device=dev)
        self.flags = torch.zeros(self.L.ntm_gemm_bf16_sk_bytes(tsel, grid, 1) // 4,
                                 dtype=torch.int32, device=dev)

    def __call__(self, a, b, c, diag=0):
        m, k = a.shape
        n = b.shape[0]
        self.epoch += 1
        check(self.L.ntm_gemm_bf16_sk(self.tsel, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k,
                                      k, k, n, self.part.data_ptr(), self.flags.data_ptr(),
                                      self.epoch, self.grid, diag, stream_handle()),
              "ntm_gemm_bf16_sk")
        return c


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
    ap.add_argument("--shapes", default="3200x3200x3200")
    ap.add_argument("--tiles", default="2")
    ap.add_argument("--grids", default="256")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--repeats", type=int, default=20)
    ap.add_argument("--diag", action="store_true", help="also time the no-wait / no-store builds")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    noise_s = torch.cuda.Stream()
    nsrc = torch.empty(128 << 20, dtype=torch.float32, device=dev)
    ndst = torch.empty_like(nsrc)
    ok_all = True
    for sh in args.shapes.split(","):
        m, n, k = (int(x) for x in sh.split("x"))
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=dev), 11)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=dev), 12)
        ref = ops.ref_gemm_f32(a, b)
        atol, rtol = ops.gemm_tolerance(k)
        for tsel in (int(x) for x in args.tiles.split(",")):
            name, tm, tn = TILES[tsel]
            if m % tm or n % tn or k % 128:
                continue
            for g in (int(x) for x in args.grids.split(",")):
                sk = StreamK(tsel, g, dev)
                c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
                try:
                    first = sk(a, b, c).clone()
                except RuntimeError as e:
                    print(json.dumps({"shape": [m, n, k], "tile": name, "grid": g,
                                      "skipped": str(e)}), flush=True)
                    continue
                torch.cuda.synchronize()
                err = (first.float() - ref).abs()
                ref_ok = bool(torch.all(err <= atol + rtol * ref.abs()))
                mism = 0
                for _ in range(args.repeats):
                    with torch.cuda.stream(noise_s):
                        ndst.copy_(nsrc)
                    sk(a, b, c)
                    torch.cuda.synchronize()
                    mism += int(not torch.equal(c, first))
                ok_all &= ref_ok and mism == 0
                fns = {"torch": lambda: torch.matmul(a, b.T, out=c),
                       "default": lambda: ops.gemm_bf16(a, b, c),
                       name: lambda name=name: ops.gemm_bf16(a, b, c, variant=name),
                       "sk": lambda: sk(a, b, c)}
                if args.diag:  # timing only: results of these runs are not checked
                    fns["sk_nowait"] = lambda: sk(a, b, c, 1)
                    fns["sk_nowait_nostore"] = lambda: sk(a, b, c, 3)
                for _ in range(200):
                    fns["torch"]()
                t = {x: [] for x in fns}
                for _ in range(args.rounds):
                    for x, fn in fns.items():
                        t[x].append(timed(fn, args.iters))
                fl = 2.0 * m * n * k
                row = {"shape": [m, n, k], "tile": name, "grid": g, "ref_ok": ref_ok,
                       "max_abs_err": float(err.max()), "repeat_mismatches": mism}
                for x, v in t.items():
                    v.sort()
                    row[f"{x}_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
                print(json.dumps(row), flush=True)
    print(json.dumps({"passed": ok_all}))
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
