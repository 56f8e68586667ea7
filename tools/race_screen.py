"""Race screen for the LDS-DMA GEMM templates (cdna_hip_programming.md: "a
sync-structure edit makes a NEW template: screen it for races over many runs
at several sizes").

The K1 kernels are deterministic (fixed MFMA order, no atomics), so every
repeat must be BITWISE identical to the first run, and the first run must
pass the fp32 reference check. A concurrent HBM copy on a second stream
perturbs DMA/L2 timing so that a read placed too early (RAW) or a restage
placed too early (WAR) shows up as a changed tile.

    python tools/race_screen.py [--variants pingpong8b] [--repeats 200]

Variant ``fp8`` screens K1-fp8's default plan (ops.gemm_fp8, e4m3 operands),
``fp8:<variant>`` one fp8 kernel (``fp8:tile128`` ...; both also on ragged C);
``<tile>/s<S>`` a masked tile with split-K in S slices (skinny long-K shapes).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nvidia_terraform_modules_amd import ops  # noqa: E402

SHAPES = [(256, 256, 128), (256, 512, 256), (512, 768, 384), (2304, 1536, 640),
          (4096, 4352, 512), (4096, 4096, 4096), (8192, 8192, 8192)]
SHAPES_160 = [(160, 160, 128), (1280, 800, 384), (2560, 1600, 640), (2560, 2560, 2560),
              (5120, 5120, 1280)]
# ragged C for the masked (wave-specialised) tiles and the default dispatch
SHAPES_RAGGED = [(1000, 1000, 1024), (1696, 2560, 640), (333, 1004, 384), (2400, 3200, 512),
                 (1000, 1000, 1000), (333, 1004, 200)]  # the last two: partial K-tiles
MASKED = ("tile128", "tile256x128", "tile160", "tile160x128", "tile128x160", "tile128x256", "pingpong8cm",
          "pingpong8om", "pingpong8omd", "pp192x256", "pp256x192", "pp224x256", "default")
# one round of 192-wide ping-pong tiles on ragged C, partial K (the plan's shapes)
SHAPES_PP = [(3904, 2584, 12760), (7288, 1344, 5768), (3072, 3072, 3072), (200, 200, 136),
             (1312, 6304, 5080)]
# skinny C with a long K: the default dispatch splits K here (k1_splitk_plan)
SHAPES_SPLITK = [(280, 6352, 7568), (128, 8192, 8192), (333, 1004, 2056), (256, 2048, 8200)]
# persistent overlap kernel (pingpong8o*, K >= 256): 1-4 tiles per workgroup,
# one- and two-tile workgroups mixed (4608^2), the shortest tile (K = 256)
SHAPES_PERSIST = [(256, 256, 256), (1024, 512, 1024), (4608, 4608, 512), (8192, 8192, 256),
                  (6144, 6144, 2048), (2304, 1792, 768), (8192, 8192, 8192)]
# ... on ragged C with multi-round tiles and partial K (pingpong8om)
SHAPES_PERSIST_RAGGED = [(4472, 5688, 5832), (4608, 4360, 456), (5000, 4104, 768), (1000, 4104, 328)]
# stream-K (pingpong8s / pingpong8s_rev): more 256x256 tiles than CUs, not a
# multiple of them - one and two rounds, ragged C, partial K, one-pair tiles
SHAPES_SK = [(4472, 5688, 5832), (4608, 4608, 1024), (6144, 6144, 2048), (4472, 5688, 200),
             (8192, 2304, 128), (5000, 4104, 4096), (1000, 17000, 384),
             # split mode (at most half a round of tiles)
             (4672, 1472, 6696), (2048, 2048, 4096), (280, 6352, 7568), (1000, 1000, 1000),
             # split mode at S = 2: the head / tail protocol (round 5)
             (4096, 2048, 8192), (2840, 1768, 8904), (256, 256, 256)]
# shapes where the default plan runs stream-K (two-round / split mode) or a
# split-K small tile picked by the ragged-C pricing (profiles/r4_sks)
SHAPES_DEFAULT_SK = [(4672, 1472, 6696), (976, 5712, 9680), (4064, 1312, 5448),
                     (1360, 2216, 6328), (384, 7648, 6744)]
SHAPES_FP8 = [(256, 256, 256), (256, 512, 512), (512, 768, 768), (2304, 1536, 1280),
              (4096, 4352, 1024), (4096, 4096, 4096), (8192, 8192, 8192)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="pingpong8,pingpong8b,pingpong8c")
    ap.add_argument("--repeats", type=int, default=200)
    ap.add_argument("--noise-mib", type=int, default=512)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    noise_s = torch.cuda.Stream()
    nsrc = torch.empty(args.noise_mib << 18, dtype=torch.float32, device=dev)
    ndst = torch.empty_like(nsrc)
    report = {"repeats": args.repeats, "results": []}
    failed = False
    for v in args.variants.split(","):
        v, _, sp = v.partition("/s")
        splits = int(sp) if sp else 1
        fp8 = v == "fp8" or v.startswith("fp8:")
        fv = v.partition(":")[2] or "default"
        dt = torch.float8_e4m3fn if fp8 else torch.bfloat16

        def gemm(a, b, out=None, v=v, fp8=fp8, fv=fv, splits=splits):
            if fp8:
                return ops.gemm_fp8(a, b, out, variant=fv, splits=splits)
            return ops.gemm_bf16(a, b, out, variant=v, splits=splits)

        tm, tn = ops.kernels.TILE_SHAPES.get(v, (0, 0))
        shapes = SHAPES_FP8 + SHAPES_RAGGED if fp8 else SHAPES_160 if tn == 160 else SHAPES
        if v.startswith("pingpong8o"):
            shapes = SHAPES_PERSIST + (SHAPES_PERSIST_RAGGED if v in ("pingpong8om", "pingpong8omd") else [])
        if v in ("pp192x256s", "pp256x192s"):
            shapes = [(4152, 1096, 16056), (2840, 1768, 8904), (1000, 1000, 4096), (1000, 1000, 1000),
                      (192, 256, 256)]
        if v.startswith("pingpong8s"):
            shapes = SHAPES_SK if v == "pingpong8s" else SHAPES_SK[:7]  # REV: two-round mode
        if splits > 1:
            shapes = SHAPES_SPLITK + SHAPES_RAGGED
        elif v in ("pp192x256", "pp256x192", "pp224x256"):
            shapes = SHAPES_PP + SHAPES_RAGGED
        elif v in MASKED:
            shapes = shapes + SHAPES_RAGGED + (SHAPES_SPLITK + SHAPES_DEFAULT_SK if v == "default" else [])
        for (m, n, k) in shapes:
            if fp8 and not ops.gemm_fp8_shape_ok(m, n, k):
                continue
            if tm and m % tm and v not in MASKED:
                continue
            if v in ("pingpong8cm", "pingpong8om", "pingpong8omd", "pp192x256", "pp256x192", "pp224x256") and n % 8:
                continue
            a = ops.fill_uniform_(torch.empty((m, k), dtype=dt, device=dev), 5 + m)
            b = ops.fill_uniform_(torch.empty((n, k), dtype=dt, device=dev), 6 + n)
            first = gemm(a, b)
            ref = ops.ref_gemm_f32(a, b)
            atol, rtol = ops.gemm_tolerance(k)
            ok_ref = ops.verify_bf16(first, ref, atol, rtol).ok
            del ref
            reps = max(20, min(args.repeats, int(args.repeats * 2**31 / (m * n * k))))
            out = torch.empty_like(first)
            mismatches = 0
            for i in range(reps):
                if i % 2 == 0:
                    with torch.cuda.stream(noise_s):
                        ops.stream_copy(nsrc, ndst)
                out.fill_(float("nan"))
                gemm(a, b, out)
                if not torch.equal(out, first):
                    mismatches += 1
            torch.cuda.synchronize()
            row = {"variant": v + (f"/s{splits}" if splits > 1 else ""), "shape": [m, n, k],
                   "repeats": reps, "ref_ok": ok_ref,
                   "bitwise_mismatches": mismatches}
            failed |= (not ok_ref) or mismatches > 0
            report["results"].append(row)
            print(json.dumps(row), flush=True)
    report["passed"] = not failed
    print(json.dumps({"passed": not failed}))
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
