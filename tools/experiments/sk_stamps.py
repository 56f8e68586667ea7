"""Where the stream-K kernel (pingpong8s, gemm_bf16_sk.hpp) spends its time:
per-workgroup s_memrealtime stamps (STAMP build, experimental library) at each
stream-K segment's K loop start / end, after its fix-up and after its C store.

    python tools/experiments/sk_stamps.py [--shape 4472x5688x5832] [--reps 5]

Prints one JSON line per shape: medians over workgroups and launches (µs) of
each segment kind's K loop, fix-up and store, the K-loop time per K-tile pair,
and the kernel span (first start to last end) against the median workgroup's.
A diagnostic build: read its shares, not its run time.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main() -> int:
    import torch

    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle

    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4472x5688x5832,4608x4608x1024,6144x6144x6144")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    for shp in args.shape.split(","):
        m, n, k = (int(x) for x in shp.split("x"))
        a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device="cuda"), 1)
        b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device="cuda"), 2)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        wsb = ops.sk_ws_bytes(m, n, k)
        ws = torch.zeros((wsb + 3) // 4, dtype=torch.float32, device="cuda")
        st = torch.zeros((256, 16), dtype=torch.int64, device="cuda")
        L = lib_experimental()
        rows = []
        for r in range(args.reps + 2):
            check(L.ntm_gemm_bf16_sk_stamp(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, k, k, n,
                                           ws.data_ptr(), wsb, st.data_ptr(), stream_handle()),
                  "ntm_gemm_bf16_sk_stamp")
            torch.cuda.synchronize()
            if r >= 2:
                rows.append(st.cpu().clone())
        tp = (k + 127) // 128
        per = {"whole": {"loop": [], "fix": [], "store": [], "pairs": []},
               "head": {"loop": [], "fix": [], "store": [], "pairs": []},
               "tail": {"loop": [], "fix": [], "store": [], "pairs": []}}
        gaps, spans, ends = [], [], []
        for s in rows:
            t0 = int(s[:, 0].min())
            for w in range(s.shape[0]):
                v = s[w].tolist()
                last = v[0]
                for q in range(3):
                    b0, b1, b2, b3 = v[1 + 4 * q: 5 + 4 * q]
                    if b0 == 0 or b3 == 0:
                        continue
                    kind = ("whole", "head", "tail")[int(v[13 + q])]
                    per[kind]["loop"].append((b1 - b0) / 100.0)
                    per[kind]["fix"].append((b2 - b1) / 100.0)
                    per[kind]["store"].append((b3 - b2) / 100.0)
                    gaps.append((b0 - last) / 100.0)
                    last = b3
                spans.append((last - v[0]) / 100.0)
                ends.append((last - t0) / 100.0)
            st.zero_()
        med = lambda x: round(statistics.median(x), 2) if x else None  # noqa: E731
        out = {"shape": shp, "k_tile_pairs_per_tile": tp, "segments": {
            kname: {"n": len(d["loop"]), "loop_us": med(d["loop"]), "fixup_us": med(d["fix"]),
                    "store_us": med(d["store"])} for kname, d in per.items()},
            "gap_before_segment_us": med(gaps), "workgroup_span_us_median": med(spans),
            "last_end_us": round(max(ends), 2), "median_end_us": med(ends)}
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
