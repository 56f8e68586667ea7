"""Summarise rocprofv3 counter + kernel-trace CSVs of a `rocprofv3 --pmc` pass (tools/gpu_run.sh)
into one JSON (mean per dispatch, per kernel) plus derived rates."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split("(")[0][:90]


def main(root):
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in acc.items():
            for c, v in d.items():
                out[k][c] = sum(v) / len(v)
    for f in glob.glob(os.path.join(root, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            if k in out:
                out[k]["avg_ns"] = float(r["AverageNs"])
    for k, d in out.items():
        if "GRBM_GUI_ACTIVE" in d and "avg_ns" in d:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs
            d["eff_clock_GHz"] = d["GRBM_GUI_ACTIVE"] / 8 / d["avg_ns"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            d["mfma_busy_per_cu_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 256)
    keep = {k: v for k, v in out.items() if "gemm" in k.lower() or "Cijk" in k}
    json.dump(keep, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
