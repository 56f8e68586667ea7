"""The flagship workload: the post-provision GPU validation Job.

This is what the Kubernetes Job created by ``modules/amd-gpu-stack``
(``kubernetes_job_v1.gpu_validation``) runs on every MI355X it is granted, and
what ``bench.py`` times. It replaces the NVIDIA operator-validator's CUDA
``vectorAdd`` (implicit in /root/reference/eks/main.tf:185-203) with:

* K1 - hand-written bf16 MFMA GEMM (TFLOP/s, fully verified against an
  independent fp32 FMA reference once, then ABFT row-checksummed on every
  checked launch through the fused epilogue - cheap enough to run always),
* K2 - HBM stream bandwidth + capacity check (288 GB class),
* C1 - RCCL all-reduce sweep over xGMI (every element checked),

and fails (non-zero exit / ``passed = False``) on: HIP error, verification
mismatch, TFLOP/s below a floor, HBM below the capacity floor, all-reduce
mismatch. Fault-injection hooks (env ``NTM_FAULT_INJECT``) corrupt one
rank's data to prove the detector fires (failure detection).
"""
from __future__ import annotations

import os
import time
from dataclasses import asdict, dataclass, field

import torch

from ..gpu_ready.phases import PhaseClock
from ..parallel import collectives as coll
from ..parallel.dist import DistEnv, all_reduce_max, all_reduce_sum, barrier

GiB = 1 << 30


@dataclass
class ValidationConfig:
    size: int = 8192                # M = N = K of the K1 GEMM, per GPU
    seed: int = 20250117
    gemm_iters: int = 50            # timed K1 launches for the TFLOP/s figure
    gemm_warmup: int = 5
    check: bool = True              # full-matrix verification vs fp32 reference
    abft_iters: int = 3             # checksum-verified K1 launches (0 = off)
    hbm_bytes: int = 2 * GiB        # K2 copy size (src + dst = 2x this)
    hbm_iters: int = 10
    allreduce_min_bytes: int = 1 << 20
    allreduce_max_bytes: int = 1 << 30
    allreduce_iters: int = 10
    tflops_floor: float = 0.0       # fail below this (0 = report only)
    hbm_floor_GBps: float = 0.0
    min_hbm_capacity_gb: float = 0.0  # 250 on MI355X (288 GB HBM3E per GPU)
    fault_inject: str = field(default_factory=lambda: os.environ.get("NTM_FAULT_INJECT", ""))


class GemmWorkload:
    """Device-resident K1 operands (A: [M,K], B: [N,K], C: [M,N], bf16).

    Operands are generated ON the device by the hash RNG (no host copy), one
    distinct seed per rank so ranks cannot agree by accident.
    """

    def __init__(self, size: int, device: torch.device, seed: int, backend=None):
        from .. import ops  # native; raises if the .so is missing

        self.ops = backend or ops
        self.m = self.n = self.k = size
        if not self.ops.gemm_shape_ok(self.m, self.n, self.k):
            raise ValueError(f"size {size} is not a multiple of 256 (K >= 128)")
        self.device = device
        self.a = torch.empty((self.m, self.k), dtype=torch.bfloat16, device=device)
        self.b = torch.empty((self.n, self.k), dtype=torch.bfloat16, device=device)
        self.c = torch.empty((self.m, self.n), dtype=torch.bfloat16, device=device)
        self.ops.fill_uniform_(self.a, seed=seed * 2 + 1)
        self.ops.fill_uniform_(self.b, seed=seed * 2 + 2)
        self.rowsum = torch.empty(self.m, dtype=torch.float32, device=device)
        # the K1 build step() runs: "default" = the plan; bench.select_k1 may pick
        # another hand-written build that is faster on this box
        self.variant = "default"

    @property
    def flops(self) -> float:
        return 2.0 * self.m * self.n * self.k

    def step(self) -> None:
        if self.variant == "default":
            self.ops.gemm_bf16(self.a, self.b, self.c)
        else:
            self.ops.gemm_bf16(self.a, self.b, self.c, variant=self.variant)

    def step_checked(self) -> None:
        """K1 with the fused ABFT row-checksum epilogue."""
        self.ops.gemm_bf16_rowsum(self.a, self.b, self.c, self.rowsum)

    def abft(self, corrupt: bool = False):
        """Check the last ``step_checked`` output in O(n^2)."""
        if corrupt:
            self.c.view(-1)[4321 % self.c.numel()] += 256.0
        return self.ops.abft_check(self.a, self.b, self.c, self.rowsum)

    def verify(self, corrupt: bool = False):
        if corrupt:
            self.c.view(-1)[12345 % self.c.numel()] += 1.0
        ref = self.ops.ref_gemm_f32(self.a, self.b)
        atol, rtol = self.ops.gemm_tolerance(self.k)
        rep = self.ops.verify_bf16(self.c, ref, atol, rtol)
        del ref
        return rep


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _time_loop(fn, iters: int, device: torch.device) -> float:
    """Seconds per call: events on the current stream (wall clock on CPU)."""
    if device.type != "cuda":
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) / iters
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize(device)
    return s.elapsed_time(e) / 1e3 / iters


def hbm_check(device: torch.device, nbytes: int, iters: int, backend=None) -> dict:
    from .. import ops as native

    o = backend or native
    if device.type == "cuda":
        free, total = torch.cuda.mem_get_info(device)
    else:  # rehearsal: host memory stands in, capacity not meaningful
        free, total = 4 * nbytes, 0
    nbytes = min(nbytes, int(free * 0.4)) // 16 * 16
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
    dst = torch.empty_like(src)
    src.uniform_()
    o.stream_copy(src, dst)
    _sync(device)
    copy_ok = bool(torch.equal(src, dst))
    sink = torch.zeros(2048, dtype=torch.float32, device=device)
    t_copy = _time_loop(lambda: o.stream_copy(src, dst), iters, device)
    t_read = _time_loop(lambda: o.stream_read(src, sink), iters, device)
    del src, dst
    return {
        "bytes": nbytes,
        "copy_GBps": 2 * nbytes / t_copy / 1e9,
        "read_GBps": nbytes / t_read / 1e9,
        "copy_ok": copy_ok,
        "capacity_total_gb": total / 1e9,
        "capacity_free_gb": free / 1e9,
    }


@dataclass
class ValidationReport:
    rank: int
    world_size: int
    device_name: str
    gemm: dict
    hbm: dict
    allreduce: list
    phases: dict
    failures: list

    @property
    def passed(self) -> bool:
        return not self.failures

    def as_dict(self) -> dict:
        d = asdict(self)
        d["passed"] = self.passed
        return d


def run_validation(env: DistEnv, cfg: ValidationConfig, clock: PhaseClock | None = None,
                   with_hbm: bool = True, with_allreduce: bool = True,
                   backend=None) -> ValidationReport:
    """Run the whole validation Job on this rank's GPU; collective across ranks.

    ``backend`` defaults to the native gfx950 ops; ``ops.reference`` (CPU)
    is for rehearsing the multi-rank logic in tests only."""
    clock = clock or PhaseClock()
    dev = env.device
    if dev.type == "cuda":
        torch.cuda.init()
    _ = torch.empty(1, device=dev)
    clock.mark("hip_init")
    failures: list[str] = []
    fi = cfg.fault_inject

    wl = GemmWorkload(cfg.size, dev, cfg.seed + env.rank, backend=backend)
    _sync(dev)
    clock.mark("buffers_ready")
    wl.step()
    _sync(dev)
    clock.mark("first_kernel")

    gemm: dict = {"m": wl.m, "n": wl.n, "k": wl.k}
    if cfg.check:
        corrupt = fi == "corrupt_gemm" and env.rank == env.world_size - 1
        rep = wl.verify(corrupt=corrupt)
        gemm["verify"] = rep.as_dict()
        if not rep.ok:
            failures.append(f"gemm verification: {rep.bad} elements out of tolerance")
    for _ in range(cfg.gemm_warmup):
        wl.step()
    barrier(env)
    sec = _time_loop(wl.step, cfg.gemm_iters, dev)
    gemm["ms"] = sec * 1e3
    gemm["tflops"] = wl.flops / sec / 1e12
    if cfg.tflops_floor and gemm["tflops"] < cfg.tflops_floor:
        failures.append(f"gemm {gemm['tflops']:.1f} TFLOP/s below floor {cfg.tflops_floor}")
    if cfg.abft_iters:
        sec_chk = _time_loop(wl.step_checked, cfg.abft_iters, dev)
        corrupt = fi == "corrupt_abft" and env.rank == env.world_size - 1
        rep = wl.abft(corrupt=corrupt)
        gemm["abft"] = rep.as_dict()
        gemm["abft_tflops"] = wl.flops / sec_chk / 1e12
        if not rep.ok:
            failures.append(f"gemm ABFT checksum: {rep.bad_acc} accumulator / "
                            f"{rep.bad_store} stored rows inconsistent")
    clock.mark("gemm_verified")
    del wl

    hbm: dict = {}
    if with_hbm:
        hbm = hbm_check(dev, cfg.hbm_bytes, cfg.hbm_iters, backend=backend)
        if not hbm["copy_ok"]:
            failures.append("hbm copy mismatch")
        if cfg.hbm_floor_GBps and hbm["copy_GBps"] < cfg.hbm_floor_GBps:
            failures.append(f"hbm {hbm['copy_GBps']:.0f} GB/s below floor {cfg.hbm_floor_GBps}")
        if cfg.min_hbm_capacity_gb and hbm["capacity_total_gb"] < cfg.min_hbm_capacity_gb:
            failures.append(f"hbm capacity {hbm['capacity_total_gb']:.0f} GB below "
                            f"{cfg.min_hbm_capacity_gb} GB")
    clock.mark("hbm_checked")

    ar: list = []
    if with_allreduce and env.world_size > 1:
        sizes = coll.sweep_sizes(cfg.allreduce_min_bytes, cfg.allreduce_max_bytes, factor=4)
        impl = None
        if fi == "corrupt_allreduce" and env.rank == 0:
            import torch.distributed as tdist

            def impl(t):  # noqa: E306 - fault injection: rank 0 adds garbage
                t.view(-1)[0] += 3
                tdist.all_reduce(t)
        res = coll.all_reduce_sweep(env, sizes, dtype="bf16", iters=cfg.allreduce_iters,
                                    warmup=2, impl=impl)
        ar = [r.as_dict() for r in res]
        errs = all_reduce_sum(env, float(sum(r.errors for r in res)))
        if errs:
            failures.append(f"all-reduce mismatch: {int(errs)} wrong elements (sum over ranks)")
    clock.mark("collectives_checked")

    # every rank must agree on pass/fail
    nfail = all_reduce_max(env, float(len(failures)))
    if nfail and not failures:
        failures.append("another rank failed validation")
    clock.mark("done")
    return ValidationReport(
        rank=env.rank, world_size=env.world_size,
        device_name=torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu",
        gemm=gemm, hbm=hbm, allreduce=ar,
        phases=clock.as_dict(), failures=failures)
