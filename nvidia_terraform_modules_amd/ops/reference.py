"""PyTorch reference implementations of the ``ops`` API (K1/K2/K3).

Used ONLY by ``bench.py --rehearsal`` and CPU tests to rehearse the
multi-process orchestration (torch.distributed.run launch, barriers, max over
ranks, the JSON contract) on machines without an MI355X. Never selected
implicitly: the real entry points in ``ops`` load the gfx950 library or raise
``NativeLibraryMissing`` - there is no silent fallback.

Semantics match the native kernels: ``gemm_bf16`` = bf16(fp32 a @ b.T),
``fill_uniform_`` is a deterministic U[-1, 1) fill (a different generator than
the device hash RNG: rehearsal numbers are not comparable to device ones).
"""
from __future__ import annotations

import torch

from .kernels import AbftReport, VerifyReport, gemm_shape_ok, gemm_tolerance  # noqa: F401


def fill_uniform_(t: torch.Tensor, seed: int, scale: float = 1.0) -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    v = torch.rand(t.shape, generator=g, dtype=torch.float32) * 2 - 1
    t.copy_((v * scale).to(t.dtype))
    return t


def gemm_bf16(a, b, out=None, variant="default"):
    r = (a.float() @ b.float().T).to(torch.bfloat16)
    if out is None:
        return r
    out.copy_(r)
    return out


def gemm_bf16_rowsum(a, b, out=None, rowsum=None):
    acc = a.float() @ b.float().T
    out = gemm_bf16(a, b, out)
    if rowsum is None:
        rowsum = torch.empty(a.shape[0], dtype=torch.float32, device=a.device)
    rowsum.copy_(acc.sum(1))
    return out, rowsum


def ref_gemm_f32(a, b):
    return a.float() @ b.float().T


def verify_bf16(c, ref, atol, rtol) -> VerifyReport:
    err = (c.float() - ref).abs()
    bad = int((~(err <= atol + rtol * ref.abs())).sum())
    rel = float((err.double().pow(2).sum() / ref.double().pow(2).sum()).sqrt())
    return VerifyReport(n=c.numel(), bad=bad, max_abs_err=float(err.max()), rel_rms_err=rel)


def abft_check(a, b, c, rowsum) -> AbftReport:
    r = a.double() @ b.double().sum(0)
    cd = c.double()
    norm = cd.norm(dim=1)
    e_acc = (rowsum.double() - r).abs()
    e_st = (cd.sum(1) - rowsum.double()).abs()
    return AbftReport(
        rows=a.shape[0],
        bad_acc=int((~(e_acc <= 1e-3 + 2**-14 * norm)).sum()),
        bad_store=int((~(e_st <= 1e-3 + 2**-6 * norm)).sum()),
        max_rel_acc=float((e_acc / norm.clamp_min(1e-30)).max()),
        max_rel_store=float((e_st / norm.clamp_min(1e-30)).max()))


def stream_copy(src, dst, config="tuned") -> None:
    dst.view(-1)[: src.numel()].copy_(src.view(-1))


def stream_read(src, sink, config="tuned") -> None:
    s = float(src.float().sum())
    if s != s:
        sink[0] = s
