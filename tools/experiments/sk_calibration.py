"""Tabulate the K1 plan's predicted unsplit / stream-K times against measured
gemm_check.py medians (default plan, pingpong8s, hipBLASLt).

Usage: python tools/experiments/sk_calibration.py gpurun_out/<run>/gemm_check.log [...]
Host only: the plan's times come from ntm_k1_plan_times (no GPU needed).
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvidia_terraform_modules_amd.ops import _lib, kernels  # noqa: E402


def main(paths):
    L = _lib.lib()
    for path in paths:
        for line in open(path):
            if not line.startswith('{"size"'):
                continue
            d = json.loads(line)
            m, n, k = map(int, d["size"].split("x"))
            u, s = ctypes.c_double(), ctypes.c_double()
            _lib.check(L.ntm_k1_plan_times(m, n, k, ctypes.byref(u), ctypes.byref(s)), "plan times")
            tiles = ((m + 255) // 256) * ((n + 255) // 256)
            de, sk, hb = (d[f"{v}_ms_med"] * 1e3 for v in ("default", "pingpong8s", "torch"))
            print("%-18s t=%3d %-44s pu=%6.1f ps=%6.1f | def=%6.1f sk=%6.1f hb=%6.1f sk/def=%.3f"
                  % (d["size"], tiles, kernels.k1_splitk_plan(m, n, k), u.value * 1e6,
                     s.value * 1e6, de, sk, hb, de / sk))


if __name__ == "__main__":
    if any(a in ("-h", "--help") for a in sys.argv[1:]):
        print(__doc__)
        sys.exit(0)
    main(sys.argv[1:])
