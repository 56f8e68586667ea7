"""Back-to-back launch gaps: K1 vs hipBLASLt (developer diagnostic). Runs
--iters launches of each kernel back to back on one stream (bf16 8192^3 and
fp8 8192x8192x4096 by default); run it under `rocprofv3 --kernel-trace` and
pass the trace CSV to --analyse for per-kernel duration and the idle gap
between one dispatch's end and the next one's start.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/experiments/launch_gap.py
    python3 tools/experiments/launch_gap.py --analyse OUT/run_kernel_trace.csv
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def run(iters: int) -> None:
    import torch

    from nvidia_terraform_modules_amd import ops

    n = 8192
    a = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device="cuda"), 1)
    b = ops.fill_uniform_(torch.empty((n, n), dtype=torch.bfloat16, device="cuda"), 2)
    c = torch.empty((n, n), dtype=torch.bfloat16, device="cuda")
    a8 = ops.fill_uniform_(torch.empty((n, 4096), dtype=torch.float8_e4m3fn, device="cuda"), 3)
    b8 = ops.fill_uniform_(torch.empty((n, 4096), dtype=torch.float8_e4m3fn, device="cuda"), 4)
    one = torch.ones((), device="cuda")
    fns = [("k1_bf16", lambda: ops.gemm_bf16(a, b, c)),
           ("hipblaslt_bf16", lambda: torch.matmul(a, b.T, out=c)),
           ("k1_fp8", lambda: ops.gemm_fp8(a8, b8, c)),
           ("hipblaslt_fp8", lambda: torch._scaled_mm(a8, b8.T, scale_a=one, scale_b=one,
                                                      out_dtype=torch.bfloat16))]
    for _ in range(3):
        for _, fn in fns:
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()


def analyse(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs: dict = {}
    prev = None
    for r in rows:
        name = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        fam = ("hipblaslt" if "Cijk" in name else "k1") + ("_fp8" if "F8" in name or "true, true" in name else "_bf16")
        if not ("gemm" in name or "Cijk" in name):
            prev = None
            continue
        d = runs.setdefault(fam, {"dur": [], "gap": []})
        d["dur"].append((e - s) / 1e3)
        if prev is not None and prev[0] == name:
            d["gap"].append((s - prev[1]) / 1e3)
        prev = (name, e)
    for fam, d in sorted(runs.items()):
        print(json.dumps({"kernel": fam, "launches": len(d["dur"]),
                          "dur_us_median": round(statistics.median(d["dur"]), 2),
                          "gap_us_median": round(statistics.median(d["gap"]), 2) if d["gap"] else None,
                          "gap_us_p90": round(sorted(d["gap"])[int(0.9 * len(d["gap"]))], 2) if d["gap"] else None,
                          "period_us": round(statistics.median(d["dur"]) + (statistics.median(d["gap"]) if d["gap"] else 0), 2)}))


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--analyse", default="")
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        run(a.iters)
    return 0


if __name__ == "__main__":
    sys.exit(main())
