"""Score the current K1 split-K plan on every shape with measured timings.

It reads gemm_check.py logs (default + forced variants + hipBLASLt per shape)
and prints the geometric mean of chosen-plan time / best measured time, plus
the worst shapes. Caveat: a split-K small-tile plan (splits > 1) is timed only
as "default", so it is credited with the fastest default measured for that
shape, whichever plan ran it. Treat a changed split-K pick as unmeasured.

    python tools/experiments/plan_eval.py [logs...]   (defaults: the round-4 calibration logs)
Host only.
"""
import math
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvidia_terraform_modules_amd.ops import kernels as K  # noqa: E402

LOGS = ["profiles/r4_sks/split_vs_default.log", "profiles/r4_sks/split_sweep.log",
        "profiles/r4_sks/calibrated_plan_check.log", "profiles/r4_tiles/one_round_all_tiles.log",
        "profiles/r4_sks/fresh24_validation.log"]


def main(paths):
    data = {}
    for f in paths:
        for line in open(f):
            if not line.startswith('{"size"'):
                continue
            d = json.loads(line)
            r = data.setdefault(d["size"], {"_def": []})
            for key, v in d.items():
                if key.endswith("_ms_med") and key not in ("torch_ms_med", "default_ms_med"):
                    r.setdefault(key[:-7], []).append(v * 1e3)
            r["_def"].append(d["default_ms_med"] * 1e3)
    rows, unknown = [], []
    for s, r in data.items():
        m, n, k = map(int, s.split("x"))
        p = K.k1_splitk_plan(m, n, k)
        cands = {key: min(v) for key, v in r.items() if key != "_def"}
        best = min(list(cands.values()) + r["_def"])
        t = min(r["_def"]) if p[3] > 1 else cands.get(p[1])
        if t is None:
            unknown.append((s, p))
            continue
        rows.append((best / t, s, p[1] + (f"x{p[3]}" if p[3] > 1 else ""),
                     min(cands, key=cands.get)))
    g = math.exp(sum(math.log(1 / x[0]) for x in rows) / len(rows))
    print(f"shapes {len(rows)}, geomean chosen/best {g:.4f}, unmeasured plans {unknown}")
    for x in sorted(rows)[:10]:
        print("best/chosen %.3f  %-18s plan=%-16s best=%s" % x)


if __name__ == "__main__":
    if any(a in ("-h", "--help") for a in sys.argv[1:]):
        print(__doc__)
        sys.exit(0)
    main(sys.argv[1:] or LOGS)
