"""K1-fp8 vs hipBLASLt fp8 under sustained load (developer diagnostic): for
each shape, the interleaved throughput (ABBA rounds of --iters launches) and
bench.energy_compare's AMD SMI windows (>= 0.6 s of one kernel each, ABBA):
average power, PPT residency, joules per TFLOP, and the gfx clock the
firmware reports at the end of each window. Is K1-fp8 power-capped where
it trails?

    python tools/experiments/fp8_energy.py [--shapes 8192x8192x8192,8192x8192x4096]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

import bench  # noqa: E402
from nvidia_terraform_modules_amd import ops  # noqa: E402
from nvidia_terraform_modules_amd.ops import smi  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--shapes", default="8192x8192x8192,8192x8192x4096")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    sample = lambda: smi.sample(dev)  # noqa: E731
    sample()
    one = torch.ones((), device=dev)
    for shp in args.shapes.split(","):
        m, n, k = (int(x) for x in shp.split("x"))
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device=dev), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device=dev), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
        fns = {"k1_fp8": lambda: ops.gemm_fp8(a, b, c),
               "hipblaslt_fp8": lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one,
                                                         out_dtype=torch.bfloat16)}
        bench.prewarm_settle(fns["k1_fp8"], sync, 0.3)
        cmp_ = bench.interleaved_compare(fns, dev, args.rounds, args.iters)
        fl = 2.0 * m * n * k
        tf = {kk: fl / v["median_s"] / 1e12 for kk, v in cmp_.items()}
        en = bench.energy_compare({kk: (fn, tf[kk]) for kk, fn in fns.items()}, sync, sample, smi)
        print(json.dumps({"shape": [m, n, k],
                          "tflops": {kk: round(v, 1) for kk, v in tf.items()},
                          "k1_over_hipblaslt": round(tf["k1_fp8"] / tf["hipblaslt_fp8"], 4),
                          "energy": en}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
