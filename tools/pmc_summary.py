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
    # dispatch geometry from the kernel trace (first dispatch per kernel)
    geo_cols = ("Grid_Size_X", "Grid_Size", "Workgroup_Size_X", "Workgroup_Size", "LDS_Block_Size",
                "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")
    for f in glob.glob(os.path.join(root, "trace", "*kernel_trace.csv")):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k in seen:
                continue
            seen.add(k)
            out[k]["geometry"] = {c: r[c] for c in geo_cols if c in r}
    for f in glob.glob(os.path.join(root, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            if k in out:
                out[k]["avg_ns"] = float(r["AverageNs"])
    for k, d in out.items():
        if "GRBM_GUI_ACTIVE" in d and "avg_ns" in d:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs
            d["eff_clock_GHz"] = d["GRBM_GUI_ACTIVE"] / 8 / d["avg_ns"]
        if "TCC_EA0_WRREQ_sum" in d and "TCC_EA0_WRREQ_64B_sum" in d:
            # write requests: 64-B ones and the rest (32-B partial-line writes)
            d["wrreq_32B"] = d["TCC_EA0_WRREQ_sum"] - d["TCC_EA0_WRREQ_64B_sum"]
            d["write_MB_from_reqs"] = (d["TCC_EA0_WRREQ_64B_sum"] * 64 + d["wrreq_32B"] * 32) / 1e6
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            d["mfma_busy_per_cu_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 256)
    keep = {k: v for k, v in out.items() if "gemm" in k.lower() or "Cijk" in k
            or "Custom" in k}
    json.dump(keep, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
