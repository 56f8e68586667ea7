"""C1: all-reduce bandwidth sweep (nccl-tests semantics) over RCCL / xGMI.

SURVEY.md §2.7 C1: ``AllReduce(sum, bf16 and fp32)``, sizes 8 B -> 8 GiB
doubling, ranks 2/4/8 on one node, one process + one GPU per rank, report
algbw and busbw = algbw * 2(n-1)/n.

MI355X sizing notes (not a translation of any NCCL pattern; the reference
has none): an 8x MI355X node is a fully connected xGMI mesh, 7 links x
~153 GB/s per GPU. A ring moves every chunk over one link per hop, so a single
ring is per-link bound; RCCL gets more by running channels over disjoint
links. The hand-written mesh path in :mod:`.xgmi` drives all 7 links at once.

Correctness: rank r contributes ``r + 1`` (plus a position-dependent integer
pattern small enough to stay exact in bf16), so the expected sum is known
exactly and every element is checked, not a sample.
"""
from __future__ import annotations

import math
import time
from dataclasses import asdict, dataclass

import torch
import torch.distributed as tdist

from .dist import DistEnv, all_reduce_max, barrier

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}


def bus_factor(op: str, n: int) -> float:
    """nccl-tests bus-bandwidth factor for ``op`` at ``n`` ranks."""
    if n <= 1:
        return 1.0 if op != "all_reduce" else 0.0
    if op == "all_reduce":
        return 2.0 * (n - 1) / n
    if op in ("all_gather", "reduce_scatter", "all_to_all"):
        return (n - 1) / n
    if op in ("broadcast", "reduce"):
        return 1.0
    raise ValueError(op)


def sweep_sizes(min_bytes: int, max_bytes: int, factor: int = 2) -> list[int]:
    if min_bytes <= 0 or max_bytes < min_bytes or factor < 2:
        raise ValueError("bad sweep bounds")
    out, s = [], min_bytes
    while s <= max_bytes:
        out.append(s)
        s *= factor
    return out


@dataclass
class CollResult:
    op: str
    dtype: str
    bytes: int
    count: int
    ranks: int
    time_us: float
    algbw_GBps: float
    busbw_GBps: float
    errors: int

    def as_dict(self) -> dict:
        return asdict(self)


def _periodic(count: int, scale: int, dtype: torch.dtype, device) -> torch.Tensor:
    # [1, 2, 4, 8] * scale repeated: no index temporaries, so multi-GiB sweeps
    # (up to 8 GiB) allocate only the message itself
    unit = torch.tensor([1, 2, 4, 8], dtype=torch.float32, device=device) * scale
    return unit.to(dtype).repeat((count + 3) // 4)[:count].contiguous()


def _pattern(count: int, rank: int, dtype: torch.dtype, device) -> torch.Tensor:
    # 2^(i%4) * (rank+1): every partial sum is 2^j * s with s <= n(n+1)/2 <= 36
    # for n <= 8, an integer < 256 -> exact in bf16 whatever the reduction order
    return _periodic(count, rank + 1, dtype, device)


def _expected(count: int, n: int, dtype: torch.dtype, device) -> torch.Tensor:
    return _periodic(count, n * (n + 1) // 2, dtype, device)


def max_message_bytes(env: DistEnv, want: int, buffers: int = 3) -> int:
    """Largest power-of-two message <= ``want`` such that ``buffers`` copies fit
    in 40 % of this rank's free HBM (the sweep holds buffer, expected, mask)."""
    if env.device.type != "cuda":
        return want
    free, _ = torch.cuda.mem_get_info(env.device)
    cap = int(0.4 * free) // buffers
    b = 8
    while b * 2 <= min(want, cap):
        b *= 2
    return b


def _sync(env: DistEnv) -> None:
    if env.device.type == "cuda":
        torch.cuda.synchronize(env.device)


def all_reduce_sweep(env: DistEnv, sizes: list[int], dtype: str = "bf16", iters: int = 20,
                     warmup: int = 5, check: bool = True,
                     impl=None) -> list[CollResult]:
    """Time ``all_reduce(sum)`` at every size; returns one result per size.

    ``impl(tensor)`` overrides the collective (e.g. the xGMI mesh path); the
    default is ``torch.distributed.all_reduce`` (RCCL on GPUs, gloo on CPU).
    An ``impl`` with a ``buffer(count)`` method (``XgmiAllReduce``) gets its
    operand there, so the sweep times its zero-copy in-place path - the same
    in-place semantics as RCCL's ``all_reduce(t)``.
    """
    tdt = _DTYPES[dtype]
    esz = torch.empty((), dtype=tdt).element_size()
    n = env.world_size
    run = impl or (lambda t: tdist.all_reduce(t) if n > 1 else None)
    results = []
    for nbytes in sizes:
        count = max(1, nbytes // esz)
        buf = _pattern(count, env.rank, tdt, env.device)
        if hasattr(impl, "buffer"):
            buf = impl.buffer(count).view(tdt).copy_(buf)
        errors = 0
        if check:
            run(buf)
            _sync(env)
            exp = _expected(count, n, tdt, env.device)
            errors = int((buf != exp).sum().item())
            del exp
        for _ in range(warmup):
            run(buf)
        _sync(env)
        barrier(env)
        t0 = time.perf_counter()
        for _ in range(iters):
            run(buf)
        _sync(env)
        dt = (time.perf_counter() - t0) / iters
        dt = all_reduce_max(env, dt)
        algbw = count * esz / dt / 1e9 if dt > 0 else math.inf
        results.append(CollResult(
            op="all_reduce", dtype=dtype, bytes=count * esz, count=count, ranks=n,
            time_us=dt * 1e6, algbw_GBps=algbw, busbw_GBps=algbw * bus_factor("all_reduce", n),
            errors=errors))
    return results


@dataclass
class P2pMatrix:
    """Point-to-point send bandwidth for every ordered rank pair (one at a time)."""
    ranks: int
    bytes: int
    gbps: list          # gbps[dst][src], None on the diagonal
    errors: int         # received elements that differ from the sender's pattern

    def min_gbps(self) -> float | None:
        vals = [v for row in self.gbps for v in row if v is not None]
        return min(vals) if vals else None

    def as_dict(self) -> dict:
        return {"ranks": self.ranks, "bytes": self.bytes,
                # 4 decimals: a loaded CPU/gloo rehearsal moves < 0.05 GB/s, which
                # one decimal rounded to 0 and read as a dead link
                "GBps": [[None if v is None else round(v, 4) for v in row] for row in self.gbps],
                "min_GBps": None if self.min_gbps() is None else round(self.min_gbps(), 4),
                "errors": self.errors}


def p2p_matrix(env: DistEnv, nbytes: int = 256 << 20, iters: int = 3) -> P2pMatrix:
    """Every ordered pair (src -> dst) in turn: src sends ``iters`` messages of
    ``nbytes`` to dst (RCCL send/recv over the one xGMI link between the two
    GPUs, gloo on CPU) while the other ranks wait at the barrier.

    This is the one-process-per-GPU counterpart of amdgpu-validate's C3 link
    matrix (validation/src/validate_main.cpp ``run_p2p``): on a fully connected
    8x MI355X mesh every pair is one link, so a degraded link is one cell.
    Timed on the receiver between the pair's barrier and its last completed
    receive; the first message of each pair is checked element for element.
    """
    n = env.world_size
    count = max(1, nbytes // 4)
    gbps = [[None] * n for _ in range(n)]
    local = torch.zeros(n * n, dtype=torch.float64)
    errors = 0
    if n > 1:
        mine = (torch.arange(count, device=env.device, dtype=torch.int32) % 1021
                + 1024 * env.rank).to(torch.float32)
        recv = torch.empty(count, device=env.device, dtype=torch.float32)
        for src in range(n):
            for dst in range(n):
                if src == dst:
                    continue
                barrier(env)
                if env.rank == src:
                    for _ in range(iters):
                        tdist.send(mine, dst)
                    _sync(env)
                elif env.rank == dst:
                    t0 = time.perf_counter()
                    for it in range(iters):
                        tdist.recv(recv, src)
                        if it == 0:
                            _sync(env)
                            want = (torch.arange(count, device=env.device, dtype=torch.int32)
                                    % 1021 + 1024 * src).to(torch.float32)
                            errors += int((recv != want).sum().item())
                            t0 = time.perf_counter()   # time the remaining messages
                    _sync(env)
                    dt = time.perf_counter() - t0
                    timed = iters - 1 if iters > 1 else 1
                    local[dst * n + src] = count * 4 * timed / dt / 1e9 if dt > 0 else 0.0
        barrier(env)
    # one collective to put the whole matrix (and the error count) on every rank
    flat = torch.cat([local, torch.tensor([float(errors)], dtype=torch.float64)])
    if n > 1:
        dev_flat = flat.to(env.device)
        tdist.all_reduce(dev_flat)
        flat = dev_flat.cpu()
    for d in range(n):
        for s_ in range(n):
            if d != s_:
                gbps[d][s_] = float(flat[d * n + s_])
    return P2pMatrix(ranks=n, bytes=count * 4, gbps=gbps, errors=int(flat[-1]))


def peak_busbw(results: list[CollResult]) -> float:
    return max((r.busbw_GBps for r in results), default=0.0)


def format_table(results: list[CollResult]) -> str:
    lines = [f"{'bytes':>12} {'count':>11} {'type':>5} {'time(us)':>10} {'algbw(GB/s)':>12} "
             f"{'busbw(GB/s)':>12} {'#wrong':>7}"]
    for r in results:
        lines.append(f"{r.bytes:>12d} {r.count:>11d} {r.dtype:>5} {r.time_us:>10.1f} "
                     f"{r.algbw_GBps:>12.2f} {r.busbw_GBps:>12.2f} {r.errors:>7d}")
    return "\n".join(lines)
