"""Does the slow-XCD tail cost launch time under the power cap? (developer
ablation, profiles/r6_xcd): the shipping pingpong8o at 8192^3 against the same
kernel with every odd-XCD workgroup's LAST tile cut by 2c K-tiles
(libntm_experimental.so ntm_gemm_bf16_pp6_oddcut; C is wrong, timing only).
Even XCDs run 2.5-4.5 % faster clocks on every recorded box, so the odd ones
finish last; if cutting their work shortens the launch by about the tail
(~3 %), an XCD-weighted schedule could reclaim it. Interleaved rounds, median
ms per launch, AMD SMI power over each variant's rounds.

    python tools/experiments/xcd_cut_ab.py [--cuts 0,2,4,6,8,10,12,16] [--rounds 9 --iters 30]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--cuts", default="0,2,4,6,8,10,12,16")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    n = args.size
    L = lib_experimental()
    vp, ci = ctypes.c_void_p, ctypes.c_int
    L.ntm_gemm_bf16_pp6_oddcut.argtypes = [ci, vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    L.ntm_gemm_bf16_pp6_oddcut.restype = ci
    a = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device="cuda"), 1)
    b = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device="cuda"), 2)
    c = torch.empty((n, n), dtype=torch.bfloat16, device="cuda")
    assert ops.k1_plan(n, n, n)[1] == "pingpong8o"

    def cut(k):
        return lambda: check(L.ntm_gemm_bf16_pp6_oddcut(k, a.data_ptr(), b.data_ptr(),
                                                         c.data_ptr(), n, n, n, n, n, n,
                                                         stream_handle()), "oddcut")

    fns = {"shipping": lambda: ops.gemm_bf16(a, b, c)}
    for k in (int(x) for x in args.cuts.split(",") if x):
        fns[f"cut{k}"] = cut(k)
    for _ in range(200):      # settle clocks on the same work
        fns["shipping"]()
    torch.cuda.synchronize()
    t = {k: [] for k in fns}
    order = list(fns.items())
    for r in range(args.rounds):
        for name, fn in (order if r % 2 == 0 else order[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            e1.synchronize()
            t[name].append(e0.elapsed_time(e1) / args.iters)
    base = statistics.median(t["shipping"])
    total_ktiles = (n // 256) ** 2 * (n // 64)
    for name, v in t.items():
        med = statistics.median(v)
        k = int(name[3:]) if name.startswith("cut") else 0
        odd_wgs = min(256, (n // 256) ** 2) // 2
        removed = odd_wgs * 2 * k / total_ktiles
        print(json.dumps({"variant": name, "ms_median": round(med, 4),
                          "vs_shipping": round(med / base, 4),
                          "work_removed_pct": round(100 * removed, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
