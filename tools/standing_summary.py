"""Round-end standing of the shipping default plans vs hipBLASLt over several
boxes (developer tool). Reads the logs of ``tools/gpu_run.sh <tag> standing``,
one directory per box / gpurun call, and prints one JSON line per row:

* named bf16 shapes (``standing_bf16.log``, tools/gemm_check.py): default /
  hipBLASLt per box, median over boxes;
* fp8 shapes (``standing_fp8.log``): K1-fp8 / hipBLASLt fp8 per box, median;
* each box's seeded ragged one-round set and 48-shape random set: shapes ahead
  of hipBLASLt, below 0.97, min and median, and the K % 16 == 8 shapes among
  those below 0.97.

    python tools/standing_summary.py gpurun_out/r5_standA gpurun_out/r5_standB ...
    python tools/standing_summary.py profiles/r5_standing      (box<X>_*.log per box)
"""
from __future__ import annotations

import glob
import json
import os
import statistics
import sys


def _rows(path: str):
    with open(path) as f:
        for line in f:
            if line.startswith("{"):
                yield json.loads(line)


def _shape(d) -> list[int]:
    sh = d.get("shape") or d.get("size")
    if isinstance(sh, str):
        return [int(x) for x in sh.split("x")]
    if isinstance(sh, int):
        return [sh] * 3
    return list(sh)


def _set_summary(name: str, ratios: list[tuple[list[int], float]]) -> dict:
    r = [x for _, x in ratios]
    low = [(s, x) for s, x in ratios if x < 0.97]
    return {"set": name, "shapes": len(r), "ahead": sum(x > 1 for x in r),
            "below_0.97": len(low), "min": round(min(r), 3), "median": round(statistics.median(r), 3),
            "below_0.97_shapes": ["x".join(map(str, s)) + f" ({x:.3f})" for s, x in low],
            "below_0.97_with_k_mod_16_eq_8": sum(s[2] % 16 == 8 for s, _ in low)}


def _boxes(dirs: list[str]) -> list[tuple[str, str]]:
    """(directory, file prefix) per box: a gpurun_out/<tag> directory holds one
    box's standing_*.log; a profiles directory holds box<X>_*.log for several."""
    out = []
    for d in dirs:
        pre = sorted({os.path.basename(p).split("_", 1)[0]
                      for p in glob.glob(os.path.join(d, "box*_*.log"))})
        out += [(d, p + "_") for p in pre] or [(d, "standing_")]
    return out


def main(dirs: list[str]) -> int:
    if not dirs or any(a in ("-h", "--help") for a in dirs):
        print(__doc__)
        return 0 if dirs else 2
    boxes = _boxes(dirs)
    named: dict = {}
    for d, pre in boxes:
        for path, key_ours, key_hb in (("bf16.log", "default_tflops_med", "torch_tflops_med"),
                                       ("fp8.log", "ours_fp8_tflops_med",
                                        "hipblaslt_fp8_tflops_med")):
            p = os.path.join(d, pre + path)
            if not os.path.exists(p):
                continue
            dtype = "bf16" if "bf16" in path else "fp8"
            for row in _rows(p):
                if row.get(key_ours) and row.get(key_hb):
                    k = (dtype, "x".join(map(str, _shape(row))))
                    named.setdefault(k, []).append(row[key_ours] / row[key_hb])
    for (dtype, shape), rs in named.items():
        print(json.dumps({"dtype": dtype, "shape": shape, "boxes": len(rs),
                          "over_hipblaslt_median": round(statistics.median(rs), 4),
                          "per_box": [round(x, 4) for x in rs]}))
    for d, pre in boxes:
        for p in sorted(glob.glob(os.path.join(d, pre + "ragged_seed*.log"))):
            rat = [(_shape(r), r["default_over_hipblaslt"]) for r in _rows(p)
                   if "default_over_hipblaslt" in r and not r.get("summary")]
            if rat:
                print(json.dumps(_set_summary(os.path.basename(p)[len(pre):-4], rat)))
        for p in sorted(glob.glob(os.path.join(d, pre + "random48_seed*.log"))):
            rat = [(_shape(r), r["default_tflops"] / r["torch_tflops"]) for r in _rows(p)
                   if r.get("torch_tflops")]
            if rat:
                print(json.dumps(_set_summary(os.path.basename(p)[len(pre):-4], rat)))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
