"""K1 vs hipBLASLt over several boxes (a +-1 % claim is a
distribution over >= 3 boxes, never a best box).

Reads ``tools/gemm_check.py`` logs (one JSON line per size; one log per box /
gpurun call) and prints, per size and variant, the per-box ratio of the
variant's median to torch.matmul's (hipBLASLt, timed interleaved in the same
process) and the median / min / max of those ratios over the boxes.

    python tools/k1_boxes.py gpurun_out/r4_boxA/gemm_check.log gpurun_out/r4_boxB/gemm_check.log ...
"""
from __future__ import annotations

import json
import statistics
import sys


def ratios(paths: list[str]) -> dict:
    """{(size, variant): [ratio per box]} of variant TF/s over hipBLASLt TF/s."""
    out: dict = {}
    for p in paths:
        with open(p) as f:
            for line in f:
                line = line.strip()
                if not line.startswith("{") or '"size"' not in line:
                    continue
                r = json.loads(line)
                hb = r.get("torch_tflops_med")
                if not hb:
                    continue
                for k, v in r.items():
                    if k.endswith("_tflops_med") and not k.startswith("torch"):
                        out.setdefault((str(r["size"]), k[: -len("_tflops_med")]), []).append(v / hb)
    return out


def main(argv: list[str]) -> int:
    if not argv:
        print(__doc__)
        return 2
    res = ratios(argv)
    for (size, var), rs in sorted(res.items()):
        print(json.dumps({"size": size, "variant": var, "boxes": len(rs),
                          "over_hipblaslt_median": round(statistics.median(rs), 4),
                          "min": round(min(rs), 4), "max": round(max(rs), 4),
                          "per_box": [round(x, 4) for x in rs]}))
    return 0


if __name__ == "__main__":
    if any(a in ("-h", "--help") for a in sys.argv[1:]):
        print(__doc__)
        sys.exit(0)
    sys.exit(main(sys.argv[1:]))
