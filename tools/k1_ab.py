"""K1 plan A/B harness (developer tool): one timing loop, one shape generator
and one explicit-plan runner for every dispatch-plan experiment. Each
subcommand times the callables it compares INTERLEAVED (every callable once per
round, order reversed on odd rounds; median over rounds, HIP events) in one
process, next to hipBLASLt, and checks results. One JSON line per shape, then
a summary line.

Subcommands (they replace round 2-5's plan_ab, fp8_plan_ab, pp_plan_ab,
margin_ab and ragged_sweep):

  ragged    the default dispatch vs hipBLASLt on a SEEDED set of ragged
            one-round shapes (the class the plan trailed on in round 4), with
            --candidates every variant that serves the shape, --splitk split-K
            candidates ("tile160/s2,...")
  plan      the default dispatch vs an explicit earlier plan "ROWS:TOP:REST"
            (--cases MxNxK=ROWS:TOP:REST,...; "tile128/s4" = split-K in 4)
  fp8-plan  the same for K1-fp8 (bitwise check against the default)
  pp-tiles  the plan with and without the 192-wide ping-pong tiles
            (--split-only: without just their stream-K split mode)
  margin    the split-K rule: plans under --old-margin/--old-min-k vs
            --margin/--min-k (--ragged: the ragged pricing alone), every changed
            shape timed both ways as explicit plans (--dtype fp8: K1-fp8)

    python tools/k1_ab.py ragged --n 24 --seed 5 [--rounds 7 --iters 20]
    python tools/k1_ab.py plan --cases 3072x3072x3072=3072:pingpong8c:tile128
    python tools/k1_ab.py pp-tiles --random --n 48 --seed 11 --changed-only
    python tools/k1_ab.py margin --n 3000 --seed 6 --max 40

The plan knobs (ops.set_plan_*) are process-wide and clear the dispatch's plan
memos; every subcommand leaves the shipping plan in place when it returns.
"""
from __future__ import annotations

import argparse
import json
import random
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from nvidia_terraform_modules_amd import ops  # noqa: E402

CANDIDATES = ("pingpong8s", "pingpong8cm", "tile128", "tile256x128", "tile160", "tile160x128",
              "tile128x160", "tile128x256", "pp192x256", "pp256x192", "pp224x256",
              "pp192x256s", "pp256x192s")


# ---- shared pieces -------------------------------------------------------------------------
def timed(fn, iters: int) -> float:
    """ms per call of ``fn`` over ``iters`` back-to-back calls (one untimed first)."""
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def interleave(fns: dict, rounds: int, iters: int) -> dict:
    """Median ms per call of each callable, timed in ABBA rounds."""
    t = {name: [] for name in fns}
    order = list(fns.items())
    for r in range(rounds):
        for name, fn in (order if r % 2 == 0 else order[::-1]):
            t[name].append(timed(fn, iters))
    return {name: statistics.median(v) for name, v in t.items()}


def ragged_shapes(n: int, seed: int, lo: float = 0.3, hi: float = 1.0) -> list:
    """n shapes: M, N, K % 8, C between lo and hi rounds of 256x256 tiles (256 CUs),
    at least one of M, N not a multiple of 256; K in [1024, 16384]."""
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        m = rng.randrange(256, 8193, 8)
        nn = rng.randrange(256, 8193, 8)
        k = rng.randrange(1024, 16385, 8)
        tiles = ((m + 255) // 256) * ((nn + 255) // 256)
        if not lo * 256 < tiles <= hi * 256 or (m % 256 == 0 and nn % 256 == 0):
            continue
        out.append((m, nn, k))
    return out


def uniform_shapes(n: int, seed: int, step: int = 8) -> list:
    rng = random.Random(seed)
    return [tuple(rng.randrange(256, 8193, step) for _ in range(3)) for _ in range(n)]


def parse_shapes(text: str) -> list:
    return [tuple(int(x) for x in s.split("x")) for s in text.split(",") if s]


def operands(m: int, n: int, k: int, dtype=torch.bfloat16):
    a = ops.fill_uniform_(torch.empty((m, k), dtype=dtype, device="cuda"), 1)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=dtype, device="cuda"), 2)
    return a, b


def hipblaslt(a, b, c):
    """hipBLASLt's GEMM on the same operands (torch.matmul / _scaled_mm)."""
    if a.dtype == torch.float8_e4m3fn:
        one = torch.ones((), device="cuda")
        return lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
    return lambda: torch.matmul(a, b.T, out=c)


def explicit(plan, a, b, c):
    """An explicit plan (rows, top, rest, splits) as a callable: rows [0, rows)
    of C on ``top`` (split-K in ``splits`` slices), the rest on ``rest``; a
    variant written "tile128/s4" carries its own split count."""
    rows, top, rest, splits = plan
    gemm = ops.gemm_fp8 if a.dtype == torch.float8_e4m3fn else ops.gemm_bf16

    def one(x, y, out, v, sp):
        v, _, s = v.partition("/s")
        gemm(x, y, out, variant=v, splits=int(s) if s else sp)

    m = a.shape[0]
    if splits > 1 or top in ops.kernels.SK_VARIANTS or rows >= m:
        return lambda: one(a, b, c, top, splits)

    def two():
        one(a[:rows], b, c[:rows], top, 1)
        one(a[rows:], b, c[rows:], rest, 1)
    return two


def within(c, ref, k: int, loose: float = 1.0) -> bool:
    atol, rtol = ops.gemm_tolerance(k)
    r = ref.float()
    return bool(torch.all((c.float() - r).abs() <= loose * (atol + rtol * r.abs())))


def emit(row: dict) -> None:
    print(json.dumps(row), flush=True)


def summary(ratios: list, **extra) -> None:
    if ratios:
        emit({"summary": True, "shapes": len(ratios), "ahead": sum(r > 1.0 for r in ratios),
              "below_0.97": sum(r < 0.97 for r in ratios), "min": min(ratios),
              "median": statistics.median(ratios), **extra})


# ---- subcommands ---------------------------------------------------------------------------
def cmd_ragged(args) -> int:
    shapes = parse_shapes(args.shapes) or ragged_shapes(args.n, args.seed, args.lo, args.hi)
    ratios = []
    for m, n, k in shapes:
        a, b = operands(m, n, k)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        fns = {"default": lambda: ops.gemm_bf16(a, b, c), "hipblaslt": hipblaslt(a, b, c)}
        if args.candidates:
            for v in CANDIDATES:
                if v == "pingpong8s" and not ops.sk_ws_bytes(m, n, k):
                    continue
                if v in ops.kernels.SKH_VARIANTS and not ops.kernels.skh_ws_bytes(v, m, n, k):
                    continue
                fns[v] = lambda v=v: ops.gemm_bf16(a, b, c, variant=v)
        for spec in (x for x in args.splitk.split(",") if x):
            fns[spec] = explicit((m, spec, spec, 1), a, b, c)
        med = interleave(fns, args.rounds, args.iters)
        row = {"shape": [m, n, k], "tiles256": ((m + 255) // 256) * ((n + 255) // 256),
               "plan": list(ops.k1_splitk_plan(m, n, k))}
        row.update({f"{name}_us": round(v * 1e3, 1) for name, v in med.items()})
        row["default_over_hipblaslt"] = round(med["hipblaslt"] / med["default"], 3)
        if args.candidates:
            best = min((v, name) for name, v in med.items() if name != "hipblaslt")
            row["best"] = best[1]
            row["best_over_hipblaslt"] = round(med["hipblaslt"] / best[0], 3)
        ratios.append(row["default_over_hipblaslt"])
        emit(row)
        del a, b, c
    summary(ratios)
    return 0


def _cases(text: str):
    for case in text.split(","):
        shape, spec = case.split("=")
        m, n, k = (int(x) for x in shape.split("x"))
        rows, top, rest = spec.split(":")
        yield (m, n, k), (int(rows), top, rest, 1), spec


def cmd_plan(args, fp8: bool = False) -> int:
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    gemm = ops.gemm_fp8 if fp8 else ops.gemm_bf16
    plan_of = ops.k1_fp8_plan if fp8 else ops.kernels.k1_splitk_plan
    ok_all, ratios = True, []
    for (m, n, k), plan, spec in _cases(args.cases):
        a, b = operands(m, n, k, dt)
        c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        c_old = torch.empty_like(c)
        ref = gemm(a, b)
        old = explicit(plan, a, b, c_old)
        old()
        torch.cuda.synchronize()
        # K1-fp8 plans give the same bytes; bf16 plans with other tiles agree to tolerance
        ok = bool(torch.equal(c_old.view(torch.int16), ref.view(torch.int16))) if fp8 \
            else within(c_old, ref, k)
        ok_all &= ok
        med = interleave({"new": lambda: gemm(a, b, c), "old": old,
                          "hipblaslt": hipblaslt(a, b, c)}, args.rounds, args.iters)
        fl = 2.0 * m * n * k
        row = {"shape": [m, n, k], "new_plan": list(plan_of(m, n, k)), "old_plan": spec,
               "old_ok": ok}
        row.update({name: round(fl / v / 1e9, 1) for name, v in med.items()})
        row["new/old"] = round(row["new"] / row["old"], 3)
        ratios.append(row["new"] / row["hipblaslt"])
        emit(row)
    summary(ratios)
    return 0 if ok_all else 1


def cmd_pp_tiles(args) -> int:
    old_knob = (True, False) if args.split_only else (False, False)
    shapes = (parse_shapes(args.shapes) or
              (uniform_shapes(args.n, args.seed) if args.random else ragged_shapes(args.n, args.seed)))
    rows = []
    try:
        for m, n, k in shapes:
            ops.set_plan_pp_tiles(*old_knob)
            old_plan = list(ops.k1_splitk_plan(m, n, k))
            ops.set_plan_pp_tiles(True)
            new_plan = list(ops.k1_splitk_plan(m, n, k))
            if args.changed_only and old_plan == new_plan:
                continue
            a, b = operands(m, n, k)
            c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")

            def run(knob):
                ops.set_plan_pp_tiles(*knob)
                ops.gemm_bf16(a, b, c)

            med = interleave({"new": lambda: run((True, True)), "old": lambda: run(old_knob),
                              "hipblaslt": hipblaslt(a, b, c)}, args.rounds, args.iters)
            ops.set_plan_pp_tiles(True)
            row = {"shape": [m, n, k], "old_plan": old_plan, "new_plan": new_plan}
            row.update({f"{name}_us": round(v * 1e3, 1) for name, v in med.items()})
            row["new_over_old"] = round(med["old"] / med["new"], 3)
            row["new_over_hipblaslt"] = round(med["hipblaslt"] / med["new"], 3)
            row["old_over_hipblaslt"] = round(med["hipblaslt"] / med["old"], 3)
            rows.append(row)
            emit(row)
            del a, b, c
    finally:
        ops.set_plan_pp_tiles(True)
    if rows:
        summary([r["new_over_hipblaslt"] for r in rows],
                old_ahead=sum(r["old_over_hipblaslt"] > 1.0 for r in rows),
                old_below_097=sum(r["old_over_hipblaslt"] < 0.97 for r in rows),
                new_over_old_min=min(r["new_over_old"] for r in rows),
                new_over_old_median=statistics.median(r["new_over_old"] for r in rows))
    return 0


def cmd_margin(args) -> int:
    fp8 = args.dtype == "fp8"
    shapes = parse_shapes(args.shapes) or uniform_shapes(args.n, args.seed, 16 if fp8 else 8)
    plan = ops.k1_fp8_splitk_plan if fp8 else ops.k1_splitk_plan
    try:
        ops.set_plan_splitk(args.old_margin, args.old_min_k, fp8=False)
        ops.set_plan_splitk_ragged(False)
        if args.ragged:   # A/B of the ragged pricing alone: old = the margin rule without it
            ops.set_plan_splitk()
        old = {s: tuple(plan(*s)) for s in shapes}
        ops.set_plan_splitk(args.margin, args.min_k)
        ops.set_plan_splitk_ragged(bool(args.ragged))
        new = {s: tuple(plan(*s)) for s in shapes}
    finally:
        ops.set_plan_splitk_ragged(True)   # the shipping plan
        ops.set_plan_splitk()
    changed = [s for s in shapes if old[s] != new[s]][: args.max]
    speedups, bad = [], 0
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    for m, n, k in changed:
        a, b = operands(m, n, k, dt)
        c_old = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
        c_new, c_t = torch.empty_like(c_old), torch.empty_like(c_old)
        med = interleave({"old": explicit(old[(m, n, k)], a, b, c_old),
                          "new": explicit(new[(m, n, k)], a, b, c_new),
                          "hipblaslt": hipblaslt(a, b, c_t)}, args.rounds, args.iters)
        torch.cuda.synchronize()
        ok = within(c_new, c_old, k, loose=4.0 if fp8 else 1.0)   # e4m3: the two plans loosely
        bad += not ok
        speedups.append(med["old"] / med["new"])
        emit({"shape": [m, n, k], "old_plan": old[(m, n, k)], "new_plan": new[(m, n, k)],
              "old_us": round(med["old"] * 1e3, 1), "new_us": round(med["new"] * 1e3, 1),
              "hipblaslt_us": round(med["hipblaslt"] * 1e3, 1),
              "new_speedup": round(speedups[-1], 3), "new_ok": ok})
    if speedups:
        emit({"summary": True, "dtype": args.dtype, "new": [args.margin, args.min_k],
              "old": [args.old_margin, args.old_min_k], "shapes": len(shapes),
              "changed": len(changed), "faster": sum(r > 1.0 for r in speedups),
              "median_speedup": round(statistics.median(speedups), 3),
              "min": round(min(speedups), 3), "max": round(max(speedups), 3), "bad": bad})
    return 1 if bad else 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p, n=24, seed=5):
        p.add_argument("--rounds", type=int, default=7)
        p.add_argument("--iters", type=int, default=20)
        p.add_argument("--n", type=int, default=n)
        p.add_argument("--seed", type=int, default=seed)
        p.add_argument("--shapes", default="", help="MxNxK,... instead of the seeded set")

    p = sub.add_parser("ragged", help="default vs hipBLASLt on seeded ragged one-round shapes")
    common(p)
    p.add_argument("--candidates", action="store_true")
    p.add_argument("--splitk", default="", help="split-K candidates, e.g. tile160/s2,tile256x128/s3")
    p.add_argument("--lo", type=float, default=0.3)
    p.add_argument("--hi", type=float, default=1.0)
    for name in ("plan", "fp8-plan"):
        p = sub.add_parser(name, help="the default vs an explicit ROWS:TOP:REST plan")
        p.add_argument("--cases", required=True)
        p.add_argument("--rounds", type=int, default=7)
        p.add_argument("--iters", type=int, default=30 if name == "plan" else 20)
    p = sub.add_parser("pp-tiles", help="the plan with / without the 192-wide ping-pong tiles")
    common(p, seed=11)
    p.add_argument("--random", action="store_true", help="uniform M, N, K in [256, 8192]")
    p.add_argument("--changed-only", action="store_true")
    p.add_argument("--split-only", action="store_true")
    p = sub.add_parser("margin", help="the split-K rule, old vs new")
    common(p, n=3000)
    p.add_argument("--margin", type=float, default=0.0, help="new rule (0: shipping)")
    p.add_argument("--min-k", type=int, default=-1, help="new rule (-1: shipping)")
    p.add_argument("--old-margin", type=float, default=1.1)
    p.add_argument("--old-min-k", type=int, default=0)
    p.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"))
    p.add_argument("--ragged", action="store_true")
    p.add_argument("--max", type=int, default=40)
    return ap


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    return {"ragged": cmd_ragged, "plan": cmd_plan,
            "fp8-plan": lambda a: cmd_plan(a, fp8=True), "pp-tiles": cmd_pp_tiles,
            "margin": cmd_margin}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
