#!/usr/bin/env python3
"""Headline benchmark: validation-Job bf16 GEMM TFLOP/s on 1/2/4/8 MI355X.

BASELINE.json metric: "cluster time-to-GPU-ready (s) + validation HIP GEMM
TFLOPS at 1/2/4/8 MI355X". The cloud half (apply -> Job Succeeded) cannot run
without a cloud account; this measures the GPU half on real hardware:

* one process per GPU (``torch.distributed.run``), RCCL over xGMI,
* each step = one hand-written K1 GEMM, M = N = K = 8192 bf16 (fp32 acc) per
  GPU on synthetic uniform[-1,1) operands generated on device (weak scaling),
* an untimed clock-settle pre-warm (``--prewarm-s`` wall seconds of K1,
  reported as ``prewarm_s``), then an untimed choice of the K1 build for this
  box (``select_k1``: the 8-wave pingpong8o and the 4-wave dma4k_d3, both
  hand-written, timed interleaved; ``per_rank_k1_variant``; ``--k1-variant NAME``
  times one build), then W untimed warmup steps, then EXACTLY K
  steps bracketed by barrier + synchronize and timed with HIP events, max over
  ranks; ``value`` = aggregate TFLOP/s over all GPUs,
* after the timed region (never inside it): full-matrix verification against
  an independent fp32 reference, K1 vs hipBLASLt on the same data measured
  INTERLEAVED (ABAB rounds, median of each), K2 HBM
  check, C1 RCCL all-reduce busbw sweep (N > 1; --p2p adds the per-pair
  send/recv link matrix), the validation Job's own binary on the same n
  GPUs (its process-start -> verdict time), and the in-node
  time-to-GPU-ready phases (process start -> HIP init -> verified). All of it
  but the Job child (which has its own time limit) runs under a deadline
  (``--extras-timeout-s``, ExtrasWatchdog): if a hung peer or link blocks a
  collective, rank 0 still prints the line, with ``extras_timed_out`` naming
  the phase.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--size 8192]
For N > 1 the driver launches it under ``torch.distributed.run``; launched
directly with --gpus N > 1 it starts that launcher as a child process.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

from nvidia_terraform_modules_amd.gpu_ready.phases import PhaseClock

_CLOCK = PhaseClock()

# The metric string is BASELINE.json's, verbatim. `value` is its GEMM half (aggregate TFLOP/s);
# the in-node half of time-to-GPU-ready is reported next to it (time_to_gpu_ready_in_node_s).
METRIC = "cluster time-to-GPU-ready (s) + validation HIP GEMM TFLOPS at 1/2/4/8 MI355X"
VALUE_COMPONENT = "validation HIP GEMM TFLOPS, aggregate over n_gpus (K1 bf16 8192^3 per GPU)"
BASELINE_CONFIG = ("EKS 8xMI355X node, amdgpu-dkms DaemonSet + 288 GB HBM sizing, "
                   "full 1/2/4/8-GPU scaling sweep")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=8192, help="M = N = K of the per-GPU GEMM")
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="untimed clock-settle pre-warm before the W warmup steps (wall seconds)")
    ap.add_argument("--compare-rounds", type=int, default=15,
                    help="ABAB rounds of the interleaved K1 vs hipBLASLt comparison")
    ap.add_argument("--no-check", action="store_true", help="skip full-matrix verification")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip hipBLASLt comparison, HBM and all-reduce sweeps")
    ap.add_argument("--allreduce-max-mib", type=int, default=8192,
                    help="largest all-reduce message (capped by free HBM)")
    ap.add_argument("--no-xgmi", action="store_true",
                    help="N > 1: skip the hand-written xGMI all-reduce sweep (C2, HIP IPC, "
                         "zero-copy in place, device-side barriers) that runs next to RCCL")
    ap.add_argument("--p2p", action="store_true",
                    help="N > 1: also measure the send/recv bandwidth of every ordered rank pair "
                         "(one xGMI link each on a fully connected node)")
    ap.add_argument("--no-job", action="store_true",
                    help="skip running the validation Job binary (amdgpu-validate) on the n GPUs "
                         "after the timed region")
    ap.add_argument("--k1-variant", default="auto",
                    help="the K1 build of the timed loop: auto = the faster of the 8-wave plan "
                         "and the 4-wave dma4k_d3 on this box (select_k1); or a build name "
                         "(default, dma4k_d3) to time that one")
    ap.add_argument("--out", default="", help="also write the JSON line to this file")
    ap.add_argument("--extras-timeout-s", type=float, default=300.0,
                    help="deadline for the work after the timed region (verification, "
                         "comparisons, collective sweeps; the Job child has its own limit): past "
                         "it rank 0 prints the "
                         "JSON line with what it has and extras_timed_out = the phase it was in, "
                         "and every rank exits (ExtrasWatchdog)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="CPU/gloo + PyTorch reference ops: rehearses the multi-process "
                         "orchestration and the JSON contract; NOT a measurement (tests only)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="every rank on cuda:0 with a gloo process group: rehearses the N > 1 "
                         "path with the real kernels (C2 over HIP IPC included) on a one-GPU box; "
                         "NOT a measurement (tests only; set GPU_MAX_HW_QUEUES=1)")
    return ap.parse_args(argv)


class StepTimer:
    """Stream-ordered timing of a launch sequence: HIP events on the current
    stream on a GPU, the host clock (after the work returns) on the CPU path."""

    def __init__(self, dev):
        import torch

        self.dev = dev
        self.ev = ([torch.cuda.Event(enable_timing=True) for _ in range(2)]
                   if dev.type == "cuda" else None)
        self.t = [0.0, 0.0]

    def start(self) -> None:
        if self.ev:
            self.ev[0].record()
        else:
            self.t[0] = time.perf_counter()

    def stop(self) -> None:
        if self.ev:
            self.ev[1].record()
        else:
            self.t[1] = time.perf_counter()

    def seconds(self) -> float:
        """Elapsed seconds (synchronises on the end event)."""
        if self.ev:
            self.ev[1].synchronize()
            return self.ev[0].elapsed_time(self.ev[1]) / 1e3
        return self.t[1] - self.t[0]


def prewarm_settle(fn, sync, min_s: float, chunk: int = 16) -> dict:
    """Run ``fn`` untimed for at least ``min_s`` seconds of wall time (whole
    chunks, synchronised), so clocks and power management reach steady state."""
    t0 = time.perf_counter()
    launches = 0
    while True:
        for _ in range(chunk):
            fn()
        launches += chunk
        sync()
        el = time.perf_counter() - t0
        if el >= min_s:
            return {"seconds": round(el, 3), "launches": launches}


# plain K1 launches queued ahead of a host-blocking AMD SMI read (~43 ms at
# 8192^3): the read measured 1-40 ms (smi_sample_ms), and the GPU must not go
# idle under it
POWER_WINDOW_CHUNK = 64
# plain K1 launches queued (no sync) ahead of each stamped clock batch (~27 ms,
# longer than the ~25 ms post-idle transient)
CLOCK_PREQUEUE = 40


def power_window(fn, sync, sample, min_s: float, chunk: int = 16, final_sync: bool = True):
    """Two telemetry samples around at least ``min_s`` s of back-to-back ``fn``
    launches; each is read while ``chunk`` launches are queued, so neither end
    sees an idle GPU. ``final_sync`` False leaves the last chunk running (the
    caller queues more work behind it at once). Returns (before, after, run)
    for ``smi.window``."""
    for _ in range(chunk):
        fn()
    before = sample()
    run = prewarm_settle(fn, sync, min_s, chunk)
    for _ in range(chunk):
        fn()
    after = sample()
    if final_sync:
        sync()
    return before, after, run


ENERGY_WINDOW_S = 0.6


def energy_compare(kernels: dict, sync, sample, smi_mod, window_s: float = ENERGY_WINDOW_S,
                   order: str = "ABBA") -> dict:
    """Joules per TFLOP of each kernel: ``kernels[name] = (launch callable,
    TF/s)``. Each window is >= ``window_s`` of one kernel's back-to-back
    launches (``power_window``, samples read under queued launches, after a
    0.2 s settle on that kernel); the windows run in ``order`` (ABBA: neither
    kernel always runs on the warmer chip) and each kernel's average power is
    the mean over its windows. Never raises: a window without energy data gives
    None."""
    names = list(kernels)
    seq = [names[0], names[1], names[1], names[0]] if order == "ABBA" and len(names) == 2 \
        else names
    per: dict = {k: [] for k in names}
    for k in seq:
        fn = kernels[k][0]
        prewarm_settle(fn, sync, 0.2)
        b, a, run = power_window(fn, sync, sample, window_s, chunk=POWER_WINDOW_CHUNK)
        per[k].append(smi_mod.window(b, a))
    out = {}
    for k in names:
        ws = [w.get("avg_power_W") for w in per[k]]
        ws = [w for w in ws if w is not None]
        avg = sum(ws) / len(ws) if ws else None
        tf = kernels[k][1]
        out[k] = {"avg_power_W": round(avg, 1) if avg is not None else None,
                  "tflops": round(tf, 1),
                  "joules_per_tflop": round(avg / tf, 4) if avg is not None and tf > 0 else None,
                  "windows_W": [w.get("avg_power_W") for w in per[k]],
                  "windows_s": [w.get("seconds") for w in per[k]],
                  "ppt_pct": [w.get("ppt_pct") for w in per[k]],
                  # the firmware's gfx clock at each window's end
                  "gfxclk_mhz": [(w.get("gfxclk_mhz") or [None, None])[1] for w in per[k]]}
    if len(names) == 2 and all(out[k]["joules_per_tflop"] for k in names):
        out[f"{names[0]}_over_{names[1]}_joules_per_tflop"] = round(
            out[names[0]]["joules_per_tflop"] / out[names[1]]["joules_per_tflop"], 4)
    out["order"] = seq
    return out


def interleaved_compare(fns: dict, dev, rounds: int, launches: int) -> dict:
    """ABBA timing: in each round every callable runs ``launches`` times under
    its own events, in the given order on even rounds and reversed on odd ones
    (neither side always follows the other); per-callable median over rounds
    (seconds per launch)."""
    import statistics

    per: dict = {k: [] for k in fns}
    order = list(fns.items())
    for r in range(rounds):
        for k, fn in (order if r % 2 == 0 else order[::-1]):
            tm = StepTimer(dev)
            tm.start()
            for _ in range(launches):
                fn()
            tm.stop()
            per[k].append(tm.seconds() / launches)
    return {k: {"median_s": statistics.median(v), "rounds_s": v} for k, v in per.items()}


def run_validation_job(n: int, timeout_s: float = 240.0) -> dict:
    """Run validation/build/amdgpu-validate on GPUs 0..n-1 as a child process;
    returns a summary of its JSON report (never raises)."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "validation", "build",
                       "amdgpu-validate")
    if not os.path.exists(exe):
        return {"ran": False, "reason": "amdgpu-validate not built"}
    cmd = [exe, "--gpus", str(n), "--size", "8192", "--iters", "10", "--json"]
    env = {k: v for k, v in os.environ.items() if k != "NTM_FAULT_INJECT"}
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired:
        return {"ran": True, "passed": False, "reason": f"timed out after {timeout_s:.0f} s"}
    wall = time.perf_counter() - t0
    try:
        rep = json.loads(p.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"ran": True, "passed": False, "rc": p.returncode, "reason": p.stderr[-300:]}
    gpus = rep.get("gpus", [])
    p2p = rep.get("xgmi_p2p_GBps") or []
    rccl = rep.get("rccl_allreduce") or []
    return {
        "ran": True, "cmd": " ".join(cmd[1:]), "rc": p.returncode, "passed": rep.get("passed"),
        "n_gpus": rep.get("n_gpus"),
        "process_start_to_verdict_s": rep.get("phases_s", {}).get("end"),
        "wall_s": round(wall, 3),
        "phases_s": rep.get("phases_s"),
        "gemm_tflops_aggregate": rep.get("gemm_tflops_aggregate"),
        "gemm_tflops_per_gpu": [g.get("gemm_tflops") for g in gpus],
        "gemm_fp8_tflops_per_gpu": [g.get("gemm_fp8_tflops") for g in gpus],
        "hbm_copy_GBps_per_gpu": [g.get("hbm_copy_GBps") for g in gpus],
        "rccl_peak_busbw_GBps": max((r.get("busbw_GBps") or 0 for r in rccl), default=None),
        "rccl_sizes_checked": len(rccl),
        "rccl_wrong": sum(r.get("wrong") or 0 for r in rccl),
        "xgmi_peak_busbw_GBps": max((r.get("busbw_GBps") or 0
                                     for r in rep.get("xgmi_allreduce_bf16") or []), default=None),
        "xgmi_p2p_min_GBps": rep.get("xgmi_p2p_min_GBps"),
        "xgmi_p2p_GBps": p2p,
        "failures": rep.get("failures", [])[:8],
    }


SK_CHECK_SHAPE = (4152, 1096, 16056)


def sk_product_check(backend, dev) -> dict:
    """One default-dispatch launch of SK_CHECK_SHAPE (stream-K split mode on a
    192-wide tile) under NTM_SK_CHECK=1, verified against the fp32 reference
    kernel. Never raises: a placement violation or a wrong element is reported
    as ok False."""
    import torch

    m, n, k = SK_CHECK_SHAPE
    os.environ["NTM_SK_CHECK"] = "1"
    res: dict = {"shape": [m, n, k]}
    try:
        res["variant"] = backend.k1_splitk_plan(m, n, k)[1]
        a = backend.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=dev), 9101)
        b = backend.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=dev), 9102)
        try:
            c = backend.gemm_bf16(a, b)
            res["sk_xcc_error"] = 0
        except backend.SkPlacementError as e:
            res.update(ok=False, sk_xcc_error=str(e)[:200])
            return res
        atol, rtol = backend.gemm_tolerance(k)
        rep = backend.verify_bf16(c, backend.ref_gemm_f32(a, b), atol, rtol)
        res.update(bad=rep.bad, max_abs_err=rep.max_abs_err, ok=rep.ok)
    except Exception as e:  # noqa: BLE001 - reported
        res.update(ok=False, error=f"{type(e).__name__}: {e}"[:200])
    return res


K1_SELECT_MARGIN = 0.005


def select_k1(wl, backend, dev, sync, rounds: int = 9, launches: int = 20) -> dict | None:
    """Pick the K1 build the timed loop runs on THIS box (untimed, after the
    pre-warm). The shipping 8-wave pingpong8o and the 4-wave dma4k_d3 trade
    places under the power limit: -3 % .. +1.8 % for dma4k_d3 on three boxes
    (profiles/r6_w4kh). Both are timed interleaved, ABAB, each after its own
    short settle; a build other than the default wins only when its median is
    K1_SELECT_MARGIN faster. Sets ``wl.variant``; returns what was measured."""
    cands = backend.k1_candidates(wl.m, wl.n, wl.k)
    if len(cands) < 2:
        return None
    fns = {v: (lambda v=v: backend.gemm_bf16(wl.a, wl.b, wl.c, variant=v)) for v in cands}
    for fn in fns.values():
        prewarm_settle(fn, sync, 0.15)
    cmp_ = interleaved_compare(fns, dev, rounds=rounds, launches=launches)
    med = {v: cmp_[v]["median_s"] for v in cands}
    best = min(cands, key=lambda v: med[v])
    chosen = best if med[best] < med["default"] * (1 - K1_SELECT_MARGIN) else "default"
    wl.variant = chosen
    prewarm_settle(wl.step, sync, 0.2)          # settle on the chosen build
    return {"candidates": cands, "chosen": chosen, "margin": K1_SELECT_MARGIN,
            "tflops_median": {v: round(wl.flops / med[v] / 1e12, 1) for v in cands},
            "rounds": rounds, "launches_per_round": launches}


def node_topology(env, dev) -> dict:
    """What the run ran on, for reading a scaling curve: every rank's device
    (name, PCI bus id, UUID, CUs, HBM), the peer-access matrix over the
    node's visible GPUs (rank 0) and the RCCL version. Never raises."""
    import torch

    from nvidia_terraform_modules_amd.parallel import dist

    mine: dict = {"rank": env.rank, "device": str(dev)}
    if dev.type == "cuda":
        try:
            p = torch.cuda.get_device_properties(dev)
            mine.update(name=p.name, gcn_arch=getattr(p, "gcnArchName", None),
                        cus=p.multi_processor_count,
                        hbm_gb=round(p.total_memory / 1e9, 1),
                        pci_bus_id=getattr(p, "pci_bus_id", None),
                        pci_device_id=getattr(p, "pci_device_id", None),
                        uuid=str(getattr(p, "uuid", "")) or None)
        except Exception as e:  # noqa: BLE001 - diagnostic only
            mine["error"] = f"{type(e).__name__}: {e}"[:200]
    out: dict = {"ranks": dist.all_gather_obj(env, mine)}
    if env.is_main and dev.type == "cuda":
        try:
            k = torch.cuda.device_count()
            out["visible_gpus"] = k
            out["peer_access"] = [[i == j or bool(torch.cuda.can_device_access_peer(i, j))
                                   for j in range(k)] for i in range(k)]
        except Exception as e:  # noqa: BLE001
            out["peer_access_error"] = f"{type(e).__name__}: {e}"[:200]
        try:
            out["rccl_version"] = ".".join(str(x) for x in torch.cuda.nccl.version())
        except Exception:  # noqa: BLE001
            out["rccl_version"] = None
    out["torch"] = torch.__version__
    out["hip"] = getattr(torch.version, "hip", None)
    return out


def pair_busbw(rccl, xgmi) -> list:
    """C2 against RCCL at the message sizes both sweeps ran (bf16, in place,
    same timing loop): one row per shared size with both busbw and the ratio."""
    rccl_at = {r.bytes: r.busbw_GBps for r in rccl}
    return [{"bytes": r.bytes, "rccl_busbw_GBps": round(rccl_at[r.bytes], 1),
             "xgmi_busbw_GBps": round(r.busbw_GBps, 1),
             "xgmi_over_rccl": round(r.busbw_GBps / rccl_at[r.bytes], 3)
             if rccl_at[r.bytes] > 0 else None}
            for r in xgmi if r.bytes in rccl_at]


class ExtrasWatchdog:
    """Deadline for the work after the timed region, on every rank.

    The headline number is final once the per-rank results are gathered. What
    follows (verification, the hipBLASLt comparison, the RCCL and xGMI sweeps)
    runs collectives that a hung peer or link would block forever, and then no
    JSON line would come out. The deadline is disarmed before the Job binary
    runs: that child has its own time limit, and exiting under it would leave
    it running on the GPUs. When the deadline passes,
    rank 0 prints the line from what it has, with ``extras_timed_out`` naming the
    phase it was in, and every rank leaves with ``os._exit`` (a blocked collective
    cannot be unwound). ``phase`` is set by the main thread as it goes.

    ``NTM_BENCH_INJECT_HANG=<phase>:<rank>`` makes that rank stall when it enters
    that phase (tests of this path only)."""

    def __init__(self, seconds: float, rank: int, on_expire, exit_fn=None):
        import threading

        self.phase = "verify"
        self.rank = rank
        self._lock = threading.Lock()
        self._owner = None          # "main" or "deadline": who prints and exits
        self._on_expire = on_expire
        self._exit = exit_fn or os._exit
        self._t = threading.Timer(seconds, self._fire) if seconds > 0 else None
        if self._t is not None:
            self._t.daemon = True
            self._t.start()

    def enter(self, phase: str) -> None:
        self.phase = phase
        if os.environ.get("NTM_BENCH_INJECT_HANG") == f"{phase}:{self.rank}":
            time.sleep(3600)

    def claim(self) -> bool:
        """The main thread is done: True if it still owns the output (the
        deadline has not fired), and the deadline can no longer fire."""
        with self._lock:
            if self._owner is None:
                self._owner = "main"
        if self._t is not None:
            self._t.cancel()
        return self._owner == "main"

    def _fire(self) -> None:
        with self._lock:
            if self._owner is not None:
                return
            self._owner = "deadline"
        code = 0
        try:
            code = self._on_expire(self.phase)
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            self._exit(code)


def relaunch_distributed(args) -> int:
    """Start torch.distributed.run as a CHILD process (never exec) and return its rc."""
    port = os.environ.get("MASTER_PORT", "29531")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def main(argv=None) -> int:
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch_distributed(args)

    import torch

    from nvidia_terraform_modules_amd.models.validation_job import GemmWorkload, hbm_check
    from nvidia_terraform_modules_amd.ops import smi
    from nvidia_terraform_modules_amd.parallel import collectives as coll
    from nvidia_terraform_modules_amd.parallel import dist

    if args.rehearsal:
        from nvidia_terraform_modules_amd.ops import reference as backend
    else:
        from nvidia_terraform_modules_amd import ops as backend

    _CLOCK.mark("runtime_import")
    if args.rehearsal:
        env = dist.init(backend="gloo", device_type="cpu")
    elif args.shared_gpu:
        os.environ["LOCAL_RANK"] = "0"      # every rank on the one GPU
        env = dist.init(backend="gloo", device_type="cuda")
    else:
        env = dist.init()
    if env.world_size != args.gpus and env.is_main:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={env.world_size}; "
              f"using WORLD_SIZE", file=sys.stderr)
    n = env.world_size
    dev = env.device

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    smi_ms: list = []

    def smi_sample():
        """One AMD SMI read, its host time recorded (smi_sample_ms in the JSON): a
        read that outlasts the launches queued behind it leaves the GPU idle."""
        t = time.perf_counter()
        r = smi.sample(dev)
        smi_ms.append(round((time.perf_counter() - t) * 1e3, 3))
        return r

    _ = torch.empty(1, device=dev)
    _CLOCK.mark("hip_init")
    if dev.type == "cuda":
        smi_sample()   # AMD SMI initialises here, not next to the timed loop

    wl = GemmWorkload(args.size, dev, seed=20250117 + env.rank, backend=backend)
    sync()
    _CLOCK.mark("buffers_ready")
    wl.step()
    sync()
    _CLOCK.mark("first_kernel")

    # ---- clock-settle pre-warm (untimed, wall-time based). A cold MI355X runs the
    # first K1 launches at boost clock, overshoots its power limit ~2 ms in and
    # throttles, then takes ~25 ms of sustained load to settle (rocprofv3 trace:
    # 695 -> 950 -> 680 us per 8192^3 launch, profiles/r2_bench/). Without this the
    # timed window of a short run lands on the transient.
    prewarm = prewarm_settle(wl.step, sync, args.prewarm_s)
    # ---- which hand-written K1 build the timed loop runs on this box (untimed)
    k1_sel = None
    if args.k1_variant != "auto":
        wl.variant = args.k1_variant
        prewarm_settle(wl.step, sync, 0.2)
    elif dev.type == "cuda" and hasattr(backend, "k1_candidates"):
        k1_sel = select_k1(wl, backend, dev, sync)

    # ---- warmup (untimed): exactly W steps. The power / throttle sample that opens
    # the telemetry window is read while POWER_WINDOW_CHUNK more pre-warm launches
    # run (counted in prewarm_launches), with the W warmup steps queued behind
    # them: an SMI read longer than W launches no longer leaves the GPU idle (an
    # idle GPU re-boosts and overshoots its power limit) right before the timed loop.
    if dev.type == "cuda":
        for _ in range(POWER_WINDOW_CHUNK):
            wl.step()
        prewarm["launches"] += POWER_WINDOW_CHUNK
    smi_before = smi_sample() if dev.type == "cuda" else None
    for _ in range(args.warmup):
        wl.step()
    sync()

    # ---- timed region: exactly K steps, barrier + sync on both sides; HIP events
    # on the stream bracket the K launches, the host clock brackets the region
    dist.barrier(env)
    sync()
    tmr = StepTimer(dev)
    t0 = time.perf_counter()
    tmr.start()
    for _ in range(args.steps):
        wl.step()
    tmr.stop()
    sync()
    t1 = time.perf_counter()
    smi_after = smi_sample() if dev.type == "cuda" else None
    dist.barrier(env)
    my_seconds = tmr.seconds()
    elapsed = dist.all_reduce_max(env, my_seconds)
    wall_elapsed = dist.all_reduce_max(env, t1 - t0)
    ms_per_step = elapsed / args.steps * 1e3
    total_tflops = n * wl.flops * args.steps / elapsed / 1e12
    # per-rank view (weak-scaling diagnosis; `value` stays the max-over-ranks
    # figure), right after the timed loop, in the power / thermal state it left:
    # each rank's own TF/s, the clock K1 ITSELF runs at (the shipping pingpong8o
    # build with start / end clock stamps per workgroup, gemm_clock_ghz; a few
    # launches on the same operands) and the clock a dense MFMA-only load holds
    # (clock_probe_ghz, ~1 ms). The two differ: the GEMM also drives LDS and HBM.
    # A failure is recorded, never raised: every rank must reach the gather.
    def _probe(name, *a, **kw):
        fn = getattr(backend, name, None)
        if dev.type != "cuda" or fn is None:
            return None
        try:
            return fn(*a, **kw)
        except Exception as e:  # noqa: BLE001 - reported per rank
            return {"median_GHz": None, "error": f"{type(e).__name__}: {e}"[:200]}

    # The stamped launches must run in the steady state the timed loop ran in, not
    # in the boost / overshoot transient an idle GPU starts (~25 ms of load to
    # settle; BENCH_r04: 663 -> 897 -> 711 us per stamped launch, BENCH_r05: 640 ->
    # 861 -> 664 after an AMD SMI read outlasted the launches queued behind it).
    # So no host-blocking call (SMI sample, sync) comes right before them: after
    # the power window, each stamped batch is queued behind CLOCK_PREQUEUE plain
    # launches (~27 ms) with no sync, and a batch whose per-launch windows drift
    # by more than 3 % (max / min) is stamped again, up to 3 batches
    # (kernels.gemm_clock_stable; the JSON says how many it took).
    power_steady = None
    if dev.type == "cuda":
        prewarm_settle(wl.step, sync, 0.3)
        # The firmware metrics behind AMD SMI refresh every few tens of ms, so a
        # short timed loop (20 x 0.67 ms) gets the same counters at both ends. This
        # window covers >= 0.5 s of the same K1 launches in the steady state the
        # timed loop left, and stands in for it where the timed window is stale.
        b, a, run = power_window(wl.step, sync, lambda: smi_sample(), 0.5,
                                 chunk=POWER_WINDOW_CHUNK, final_sync=False)
        power_steady = {**smi.window(b, a), "launches": run["launches"]}
    gclk = _probe("gemm_clock_stable", wl.a, wl.b, wl.c, steps=min(max(args.steps, 1), 20),
                  prequeue=wl.step, prequeue_launches=CLOCK_PREQUEUE)
    clk = _probe("clock_probe_ghz", dev)
    # the clock the TIMED loop ran at: shader cycles per launch are launch-invariant
    # (1.085-1.091 M at 8192^3), so median cycles / this rank's ms per step
    timed_clk = None
    # (only where the timed kernel IS the clock build's: the default plan runs
    # pingpong8o - at 2048^3 it runs a small tile, whose cycles these are not)
    same_kernel = False
    if dev.type == "cuda" and hasattr(backend, "k1_plan") and wl.variant == "default":
        try:
            same_kernel = backend.k1_plan(args.size, args.size, args.size)[1] == "pingpong8o"
        except ValueError:
            same_kernel = False
    if same_kernel and gclk and gclk.get("per_launch_cycles_median"):
        cyc = sorted(gclk["per_launch_cycles_median"])
        timed_clk = round(cyc[len(cyc) // 2] / (my_seconds / args.steps) / 1e9, 4)
        gclk["ms_per_launch_over_ms_per_step"] = round(
            gclk["ms_per_launch"] / (my_seconds / args.steps * 1e3), 4)
        # the stamped batch's clock measured the way the timed loop's is (median
        # cycles / wall ms per launch, dispatch ramp and drain included): the
        # like-for-like partner of per_rank_timed_loop_clock_GHz; bound_GHz counts
        # only the stamp windows (bound_window_fraction of a step)
        gclk["launch_wall_GHz"] = round(cyc[len(cyc) // 2] / (gclk["ms_per_launch"] * 1e-3) / 1e9, 4)
        # the stamped launches ran at the timed loop's pace: otherwise
        # their clock describes a different power state and must not label the rank
        gclk["clock_trusted"] = 0.95 <= gclk["ms_per_launch_over_ms_per_step"] <= 1.05
        # share of a timed step the bounding XCD's workgroups spend between their
        # stamps (the rest: dispatch ramp, drain, launch gap): timed-loop clock =
        # bound clock x this fraction
        if gclk.get("bound_GHz"):
            gclk["bound_window_fraction"] = round(
                cyc[len(cyc) // 2] / (gclk["bound_GHz"] * 1e9) / (my_seconds / args.steps), 4)
    power = smi.window(smi_before, smi_after) if smi_before is not None else None
    # the power / throttle figures reported per rank: the timed loop's own window
    # when it spans >= 0.1 s and its counters advanced, else the steady-state window
    # beside it (a shorter window holds one or no metrics refresh: quantised or stale)
    power_src = None
    if power is not None:
        power_src = ("timed_loop" if power.get("avg_power_W") is not None
                     and (power.get("seconds") or 0) >= 0.1 else "steady_window")
    per_rank = dist.all_gather_obj(env, {"tflops": round(wl.flops * args.steps / my_seconds / 1e12, 2),
                                         "clock": clk, "gemm_clock": gclk,
                                         "timed_loop_clock": timed_clk, "power": power,
                                         "power_steady": power_steady, "power_src": power_src,
                                         "smi_ms": smi_ms, "k1_variant": wl.variant,
                                         "k1_selection": k1_sel})

    make_line = _make_line_factory(args, n, prewarm, wall_elapsed, ms_per_step, total_tflops,
                                   per_rank)

    def emit(line: dict) -> None:
        if env.is_main:
            s = json.dumps(line)
            print(s, flush=True)
            if args.out:
                with open(args.out, "w") as f:
                    f.write(s + "\n")

    # ---- after the timed region: verification + context measurements, under a
    # deadline (ExtrasWatchdog): a hung collective must not swallow the JSON line
    extras: dict = {}
    verified = None

    def on_deadline(phase: str) -> int:
        if env.is_main:
            line = make_line(dict(extras), verified)
            line["extras_timed_out"] = phase
            line["extras_timeout_s"] = args.extras_timeout_s
            emit(line)
            print(f"[bench] extras deadline ({args.extras_timeout_s:.0f} s) passed in phase "
                  f"{phase!r}: JSON line printed, exiting", file=sys.stderr)
        return 0 if verified in (None, True) else 1

    wd = ExtrasWatchdog(args.extras_timeout_s, env.rank, on_deadline)
    wd.enter("topology")
    extras["node_topology"] = node_topology(env, dev)
    wd.enter("verify")
    if not args.no_check:
        rep = wl.verify()
        bad = dist.all_reduce_sum(env, float(rep.bad))
        verified = bad == 0
        extras["verify_rank0"] = rep.as_dict()
        extras["verify_bad_total"] = int(bad)
    _CLOCK.mark("gemm_verified")
    wd.enter("sk_check")
    if not args.no_check and dev.type == "cuda" and hasattr(backend, "sk_check_enabled"):
        # stream-K placement check on the product path: the split-mode
        # shape the default plan runs on a 192-wide tile, through the default
        # dispatch with NTM_SK_CHECK=1 (a placement violation raises there), checked
        # against the fp32 reference; the word is recorded per rank.
        extras["sk_check_rank0"] = sk_product_check(backend, dev)
        extras["sk_xcc_error"] = extras["sk_check_rank0"].get("sk_xcc_error")
        if not extras["sk_check_rank0"].get("ok"):
            verified = False

    gpu_extras = not args.no_extras and not args.rehearsal
    wd.enter("hipblaslt_compare")
    if gpu_extras:
        # K1 vs hipBLASLt on the same operands, INTERLEAVED (ABAB rounds, median of
        # each), after re-settling the clock on hipBLASLt itself: neither side gets
        # the warmer chip.
        cc = torch.empty_like(wl.c)
        blas = lambda: torch.matmul(wl.a, wl.b.T, out=cc)  # noqa: E731
        prewarm_settle(blas, sync, 0.3)
        cmp_ = interleaved_compare({"k1": wl.step, "hipblaslt": blas}, dev,
                                   rounds=args.compare_rounds, launches=20)
        k1_tf = wl.flops / cmp_["k1"]["median_s"] / 1e12
        hb_tf = wl.flops / cmp_["hipblaslt"]["median_s"] / 1e12
        # energy per flop of each kernel (the headline is power-bound,
        # so J/TFLOP is what ranks a bf16 change): AMD SMI energy-counter windows of
        # >= ENERGY_WINDOW_S of back-to-back launches of ONE kernel, in ABBA order,
        # each sample read under queued launches; J/TFLOP = the window's average
        # socket power / that kernel's interleaved median TF/s.
        if dev.type == "cuda":
            extras["energy_rank0"] = energy_compare(
                {"k1": (wl.step, k1_tf), "hipblaslt": (blas, hb_tf)}, sync, smi_sample, smi)
            for k in ("k1", "hipblaslt"):
                extras[f"{k}_joules_per_tflop"] = extras["energy_rank0"][k]["joules_per_tflop"]
        del cc
        extras["interleaved_compare_rank0"] = {
            "rounds": args.compare_rounds, "launches_per_round": 20,
            "k1_tflops_median": round(k1_tf, 1), "hipblaslt_tflops_median": round(hb_tf, 1),
            "k1_over_hipblaslt": round(k1_tf / hb_tf, 4),
            "k1_tflops_rounds": [round(wl.flops / s / 1e12, 1) for s in cmp_["k1"]["rounds_s"]],
            "hipblaslt_tflops_rounds": [round(wl.flops / s / 1e12, 1)
                                        for s in cmp_["hipblaslt"]["rounds_s"]]}
        extras["hipblaslt_tflops_per_gpu_rank0"] = hb_tf
        extras["k1_over_hipblaslt"] = round(k1_tf / hb_tf, 4)  # rank 0, interleaved medians
        extras["ours_tflops_per_gpu"] = total_tflops / n
        # same K1 with the fused ABFT row-checksum epilogue, then its O(n^2) check
        tm = StepTimer(dev)
        tm.start()
        for _ in range(50):
            wl.step_checked()
        tm.stop()
        sync()
        extras["abft_gemm_tflops_per_gpu_rank0"] = wl.flops / (tm.seconds() / 50) / 1e12
        ab = wl.abft()
        extras["abft_rank0"] = ab.as_dict()
        if not ab.ok:
            verified = False
    del wl
    if dev.type == "cuda":
        torch.cuda.empty_cache()

    wd.enter("hbm")
    if gpu_extras:
        h = hbm_check(dev, 2 << 30, 10)
        extras["hbm_copy_GBps_rank0"] = h["copy_GBps"]
        extras["hbm_read_GBps_rank0"] = h["read_GBps"]
        extras["hbm_capacity_gb"] = h["capacity_total_gb"]
    _CLOCK.mark("hbm_checked")

    wd.enter("rccl_sweep")
    if not args.no_extras and n > 1:
        # nccl-tests style: bf16 from 8 B (latency end) and fp32 from 1 MiB, x4 steps
        max_b = int(dist.all_reduce_max(env, -coll.max_message_bytes(
            env, args.allreduce_max_mib << 20)) * -1)   # the smallest cap over ranks
        sizes = coll.sweep_sizes(1 << 20, max_b, factor=4)
        res = coll.all_reduce_sweep(env, coll.sweep_sizes(8, max_b, 4),
                                    dtype="bf16", iters=10, warmup=3)
        res32 = coll.all_reduce_sweep(env, sizes, dtype="fp32", iters=10, warmup=3)
        for key, rs in (("allreduce_bf16", res), ("allreduce_fp32", res32)):
            extras[key] = [
                {"bytes": r.bytes, "time_us": round(r.time_us, 1),
                 "busbw_GBps": round(r.busbw_GBps, 1), "errors": r.errors} for r in rs]
        extras["allreduce_peak_busbw_GBps"] = coll.peak_busbw(res)
        extras["allreduce_fp32_peak_busbw_GBps"] = coll.peak_busbw(res32)
        if any(r.errors for r in res + res32):
            verified = False
        if args.p2p:
            # per-link check: every ordered pair, one at a time (RCCL send/recv = one xGMI
            # link). Opt-in: the driver's scaling runs keep to the all-reduce sweep.
            pm = coll.p2p_matrix(env, nbytes=(64 << 20) if args.rehearsal else (256 << 20),
                                 iters=3)
            extras["p2p_send_GBps"] = pm.as_dict()
            if pm.errors:
                verified = False
        if not args.no_xgmi and n <= 8:
            # C2 next to RCCL, on ONE communicator for the knob sweep and the main
            # sweep (xgmi.c2_sweep: 3 IPC exports per rank in all, a collective
            # signal reset per blocks-per-rank value). First the knob sweep: blocks
            # per rank (16 .. 256) x one-/two-shot at 6 sizes up to 256 MiB (capped
            # by free HBM), the favoured one-shot cutoff and the best single nblk
            # (~5-10 s at N = 8, bounded by xgmi.TUNE_BUDGET_S); then the RCCL bf16
            # sizes from 512 B to 1 GiB that split into 8-element chunks per rank,
            # in place on the registered buffer, no host sync / barrier / staging
            # per call, in the tuned configuration (the defaults if the tune
            # failed). The rehearsal runs both over torch.distributed to pin the
            # JSON shape and the hand-over.
            from nvidia_terraform_modules_amd.parallel import xgmi as xg

            wd.enter("xgmi")
            xs = [b for b in coll.sweep_sizes(8, max_b, 4)
                  if 512 <= b <= 1 << 30 and (b // 2) % (8 * n) == 0]
            fac = None
            if args.rehearsal:
                fac = lambda nb, mb: xg.ReferenceAllReduce(env, mb, nblk=nb)  # noqa: E731
            c2, xr = xg.c2_sweep(env, xs, max_b, factory=fac)
            if not c2.pop("ok"):
                verified = False
            extras.update(c2)
            if xr:
                extras["xgmi_vs_rccl_bf16"] = pair_busbw(res, xr)
    _CLOCK.mark("collectives_checked")

    if (gpu_extras or args.rehearsal) and not args.no_job:
        # The Kubernetes validation Job's own entrypoint on this node's n GPUs (one
        # process, all GPUs): its process-start -> verdict time is the in-node part
        # of time-to-GPU-ready (it runs C1 RCCL, C2 xGMI and the C3 link matrix
        # when n > 1).
        # Every rank's GPU work is done (barrier); the other ranks then leave, and
        # rank 0 touches no GPU between the child and its print, so whatever the
        # child does, the JSON line still comes out.
        wd.enter("job")
        dist.barrier(env)
        if not env.is_main:
            if not wd.claim():
                time.sleep(3600)   # the deadline's thread is exiting the process
            dist.shutdown(env)
            return 0 if verified in (None, True) else 1
        # the Job child has its own time limit; the deadline stops here, so it never
        # exits this process with the child still running on the GPUs
        if not wd.claim():
            time.sleep(3600)   # the deadline's thread is exiting the process
        extras["validation_job"] = run_validation_job(n)
    wd.enter("report")
    _CLOCK.mark("done")
    line = make_line(extras, verified)
    if not wd.claim():
        time.sleep(3600)       # the deadline's thread printed the line and is exiting
    emit(line)
    dist.shutdown(env)
    return 0 if verified in (None, True) else 1


def _make_line_factory(args, n, prewarm, wall_elapsed, ms_per_step, total_tflops, per_rank):
    def _pw(p: dict, key: str):
        src = p["power"] if p["power_src"] == "timed_loop" else p["power_steady"]
        return (src or {}).get(key)

    def make_line(extras: dict, verified) -> dict:
        return {
            "metric": METRIC,
            "value_component": VALUE_COMPONENT,
            "value": round(total_tflops, 2),
            "unit": "TFLOP/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("REHEARSAL: CPU/gloo + PyTorch reference ops - orchestration test, NOT a "
                     "measurement" if args.rehearsal else
                     "SHARED-GPU REHEARSAL: every rank on cuda:0, gloo group - NOT a measurement"
                     if args.shared_gpu else
                     "synthetic (uniform[-1,1) bf16 operands generated on device, hash RNG)"),
            "config": {
                "model": f"validation-job K1 GEMM C[{args.size}x{args.size}] = A[{args.size}x{args.size}]"
                         f" * B[{args.size}x{args.size}]^T, bf16 in/out, fp32 accumulate",
                "global_batch": n,
                "seq_len": args.size,
                "parallelism": f"dp{n}",
                "baseline_config": BASELINE_CONFIG,
            },
            "verified": verified,
            "timing": "HIP events around the K launches (max over ranks); host clock "
                      "around the barrier+sync-bracketed region in timed_region_wall_s",
            "timed_region_wall_s": round(wall_elapsed, 6),
            "prewarm_s": prewarm["seconds"],
            "prewarm_launches": prewarm["launches"],
            # in-node part of time-to-GPU-ready = the Job binary's process start -> verdict on
            # these n GPUs; the bench process's own (torch import included) is kept beside it
            "time_to_gpu_ready_in_node_s": (
                round(extras["validation_job"]["process_start_to_verdict_s"], 3)
                if (extras.get("validation_job") or {}).get("passed") else None),
            "bench_process_to_verified_s": round(_CLOCK.elapsed("gemm_verified"), 3),
            "in_node_phases_s": {k: round(v, 4) for k, v in _CLOCK.durations().items()},
            "per_rank_tflops": [p["tflops"] for p in per_rank],
            # the hand-written K1 build each rank's timed loop ran (select_k1: the
            # faster of pingpong8o and dma4k_d3 on that box), and what decided it
            "per_rank_k1_variant": [p["k1_variant"] for p in per_rank],
            "per_rank_k1_selection": [p["k1_selection"] for p in per_rank],
            # in-kernel clock: per stamped launch the median workgroup's cycles / window,
            # median over launches (within 2-3 % of the PMC clock, profiles/r4_clock/)
            # the launch-bounding clock: per stamped launch the slowest XCD's median
            # workgroup clock (every XCD gets the same tiles, so it finishes last);
            # the all-workgroup median beside it, and the per-XCD spread
            "per_rank_gemm_clock_GHz": [(p["gemm_clock"] or {}).get("bound_GHz") for p in per_rank],
            # stamped batches it took to get one whose per-launch windows agree within 3 %
            # (kernels.gemm_clock_stable), and whether that batch ran at the timed loop's
            # pace (ms per stamped launch / timed ms per step within 0.95-1.05)
            "per_rank_gemm_launch_wall_clock_GHz": [(p["gemm_clock"] or {}).get("launch_wall_GHz")
                                                    for p in per_rank],
            "per_rank_clock_batches": [(p["gemm_clock"] or {}).get("clock_batches") for p in per_rank],
            "per_rank_clock_trusted": [(p["gemm_clock"] or {}).get("clock_trusted") for p in per_rank],
            # host time of every AMD SMI read per rank (init, window opens / closes), ms
            "per_rank_smi_sample_ms": [p["smi_ms"] for p in per_rank],
            "per_rank_gemm_clock_median_GHz": [(p["gemm_clock"] or {}).get("launch_GHz")
                                               for p in per_rank],
            "per_rank_xcd_clock_spread_pct": [(p["gemm_clock"] or {}).get("xcc_clock_spread_pct")
                                              for p in per_rank],
            "per_rank_gemm_clock_p10_GHz": [(p["gemm_clock"] or {}).get("p10_GHz") for p in per_rank],
            "per_rank_gemm_clock": [p["gemm_clock"] for p in per_rank],
            # median shader cycles per stamped launch / the rank's own timed ms per step
            "per_rank_timed_loop_clock_GHz": [p["timed_loop_clock"] for p in per_rank],
            # AMD SMI per rank: average power (energy counter), PPT (power) and
            # socket-thermal throttle residency in % of firmware iterations, from the
            # window named in per_rank_power_window: "timed_loop" = [last warmup launches
            # .. end of the timed loop]; "steady_window" = >= 0.5 s of the same K1 right
            # after it (the timed window was under 0.1 s or stale). Both
            # raw windows (power / temperature / clock at both ends) are kept.
            "per_rank_avg_power_W": [_pw(p, "avg_power_W") for p in per_rank],
            "per_rank_ppt_throttle_pct": [_pw(p, "ppt_pct") for p in per_rank],
            "per_rank_thermal_throttle_pct": [_pw(p, "thermal_pct") for p in per_rank],
            "per_rank_power_window": [p["power_src"] for p in per_rank],
            "per_rank_power": [p["power"] for p in per_rank],
            "per_rank_power_steady": [p["power_steady"] for p in per_rank],
            "per_rank_clock_GHz": [(p["clock"] or {}).get("median_GHz") for p in per_rank],
            "per_rank_clock_probe": [p["clock"] for p in per_rank],
            "vs_baseline_note": "reference publishes no TFLOP/s or busbw (BASELINE.json published={})",
            **({"rehearsal": True} if args.rehearsal else {}),
            **({"shared_gpu_rehearsal": True} if args.shared_gpu else {}),
            **extras,
        }

    return make_line


if __name__ == "__main__":
    sys.exit(main())
