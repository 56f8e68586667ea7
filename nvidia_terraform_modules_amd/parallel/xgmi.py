"""C2: the hand-written xGMI all-reduce from Python.

Two entry points over the same HIP kernels (validation/include/ntm/
xgmi_allreduce.hpp):

* :func:`simulate_allreduce` - the whole N-rank communicator on ONE device
  (rank r = blocks [r*nblk, (r+1)*nblk)). Exercises the complete two-shot
  algorithm and its release/acquire flag protocol across XCDs; it is how the
  kernel is tested on a single MI355X.
* :class:`XgmiAllReduce` - one process per GPU (torch.distributed env): each
  rank allocates in/out/signal buffers, exchanges HIP IPC handles with
  ``all_gather_object`` and opens its peers' buffers, then every call runs the
  two-shot kernel over the xGMI mesh. Multi-GPU numbers are pending hardware
  (this environment exposes one GPU); bench.py runs it only with ``--xgmi``.
"""
from __future__ import annotations

import ctypes

import torch

from ..ops._lib import check, lib, stream_handle

MAX_RANKS = 8


def _declare() -> ctypes.CDLL:
    L = lib()
    c_int, c_size, c_vp = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    pp = ctypes.POINTER(c_vp)
    L.ntm_xgmi_allreduce_bf16.argtypes = [pp, pp, pp, c_int, c_int, c_int, c_int, c_size,
                                          ctypes.c_uint, c_vp, c_int, c_vp]
    L.ntm_xgmi_allreduce_bf16.restype = c_int
    L.ntm_xgmi_signal_bytes.argtypes = [c_int]
    L.ntm_xgmi_signal_bytes.restype = c_size
    L.ntm_malloc.argtypes = [ctypes.POINTER(c_vp), c_size, c_int]
    L.ntm_malloc.restype = c_int
    L.ntm_free.argtypes = [c_vp]
    L.ntm_free.restype = c_int
    L.ntm_memset_async.argtypes = [c_vp, c_int, c_size, c_vp]
    L.ntm_memset_async.restype = c_int
    L.ntm_ipc_handle.argtypes = [c_vp, c_vp]
    L.ntm_ipc_handle.restype = c_int
    L.ntm_ipc_open.argtypes = [c_vp, ctypes.POINTER(c_vp)]
    L.ntm_ipc_open.restype = c_int
    L.ntm_ipc_close.argtypes = [c_vp]
    L.ntm_ipc_close.restype = c_int
    return L


def _ptrs(xs) -> "ctypes.Array":
    arr = (ctypes.c_void_p * len(xs))()
    for i, x in enumerate(xs):
        arr[i] = x
    return arr


def simulate_allreduce(inputs: list[torch.Tensor], nblk: int = 16, one_shot: bool = False,
                       epoch: int = 1) -> tuple[list[torch.Tensor], int]:
    """All-reduce (sum) N same-shaped bf16 tensors living on ONE device, as N
    simulated ranks. Returns (outputs, timeout_code) - 0 means no barrier
    timed out."""
    n = len(inputs)
    if not 1 <= n <= MAX_RANKS:
        raise ValueError("1..8 ranks")
    count = inputs[0].numel()
    if count % (8 * n):
        raise ValueError("count must be a multiple of 8 * nranks")
    for t in inputs:
        if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.numel() != count:
            raise ValueError("inputs must be contiguous bf16 of equal size")
    L = _declare()
    dev = inputs[0].device
    outs = [torch.empty_like(t) for t in inputs]
    sig_bytes = L.ntm_xgmi_signal_bytes(nblk)
    sigs = [torch.zeros(sig_bytes // 4, dtype=torch.int32, device=dev) for _ in range(n)]
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = L.ntm_xgmi_allreduce_bf16(
        _ptrs([t.data_ptr() for t in inputs]), _ptrs([t.data_ptr() for t in outs]),
        _ptrs([s.data_ptr() for s in sigs]), n, 0, n, nblk, count, epoch, err.data_ptr(),
        1 if one_shot else 0, stream_handle())
    check(rc, "ntm_xgmi_allreduce_bf16")
    torch.cuda.synchronize(dev)
    return outs, int(err.item())


class XgmiAllReduce:
    """Two-shot all-reduce across the ranks of a torch.distributed group, one
    process per GPU, buffers shared through HIP IPC (xGMI peer mappings)."""

    def __init__(self, env, max_bytes: int, nblk: int = 64):
        from .dist import all_gather_obj

        if env.world_size > MAX_RANKS:
            raise ValueError("at most 8 ranks (one MI355X node)")
        self.env, self.nblk, self.max_bytes = env, nblk, max_bytes
        self.L = L = _declare()
        self._own = []
        handles = {}
        for name, nbytes, uncached in (("in", max_bytes, 0), ("out", max_bytes, 0),
                                       ("sig", L.ntm_xgmi_signal_bytes(nblk), 1)):
            p = ctypes.c_void_p()
            check(L.ntm_malloc(ctypes.byref(p), nbytes, uncached), "ntm_malloc")
            self._own.append(p.value)
            h = ctypes.create_string_buffer(64)
            check(L.ntm_ipc_handle(p.value, h), "ntm_ipc_handle")
            handles[name] = (p.value, h.raw)
        check(L.ntm_memset_async(handles["sig"][0], 0, L.ntm_xgmi_signal_bytes(nblk), None),
              "memset")
        torch.cuda.synchronize()
        gathered = all_gather_obj(env, {k: v[1] for k, v in handles.items()})
        self._opened = []
        self.ptrs = {"in": [], "out": [], "sig": []}
        for r, hs in enumerate(gathered):
            for k in ("in", "out", "sig"):
                if r == env.rank:
                    self.ptrs[k].append(handles[k][0])
                else:
                    p = ctypes.c_void_p()
                    check(L.ntm_ipc_open(hs[k], ctypes.byref(p)), "ntm_ipc_open")
                    self._opened.append(p.value)
                    self.ptrs[k].append(p.value)
        self.epoch = 0
        self.err = torch.zeros(1, dtype=torch.int32, device=env.device)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks of bf16 tensor ``t`` (staged through the
        registered buffers)."""
        nbytes = t.numel() * t.element_size()
        if t.dtype != torch.bfloat16 or nbytes > self.max_bytes or not t.is_contiguous():
            raise ValueError("contiguous bf16 up to max_bytes")
        n = self.env.world_size
        count = t.numel()
        if count % (8 * n):
            raise ValueError("numel must be a multiple of 8 * world_size")
        self.epoch += 1
        # stage t into my registered "in" buffer; the host barrier after the
        # stream sync guarantees every peer's input is complete before any
        # rank's kernel reads it over xGMI
        _copy_d2d(self.ptrs["in"][self.env.rank], t.data_ptr(), nbytes)
        torch.cuda.current_stream().synchronize()
        from .dist import barrier
        barrier(self.env)
        rc = self.L.ntm_xgmi_allreduce_bf16(
            _ptrs(self.ptrs["in"]), _ptrs(self.ptrs["out"]), _ptrs(self.ptrs["sig"]), n,
            self.env.rank, 1, self.nblk, count, self.epoch, self.err.data_ptr(), 0,
            stream_handle())
        check(rc, "ntm_xgmi_allreduce_bf16")
        _copy_d2d(t.data_ptr(), self.ptrs["out"][self.env.rank], nbytes)
        return t

    def timed_out(self) -> bool:
        return bool(self.err.item())

    def close(self) -> None:
        torch.cuda.synchronize()
        for p in self._opened:
            self.L.ntm_ipc_close(p)
        for p in self._own:
            self.L.ntm_free(p)
        self._opened, self._own = [], []


def _copy_d2d(dst: int, src: int, nbytes: int) -> None:
    """Stream-ordered device->device copy through the native stream kernel."""
    if nbytes % 16 == 0:
        check(lib().ntm_stream_copy(src, dst, nbytes, stream_handle()), "ntm_stream_copy")
    else:
        raise ValueError("sizes must be 16-byte multiples")
