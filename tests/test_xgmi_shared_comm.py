"""bench.py's C2 block (xgmi.c2_sweep = tune + the main sweep)
runs on ONE XgmiAllReduce - 3 ntm_ipc_handle calls per rank in all - with
reconfigure() in between, over a host-memory stub of the native library.

The stub is functional, not a mock: ntm_malloc hands out POSIX shared memory,
the "IPC handle" is its name, ntm_ipc_open maps the peer's segment, and the
all-reduce "kernel" sums every rank's registered buffer (two gloo barriers
stand in for the device-side entry / exit barriers). So the real
all_reduce_sweep runs through the real XgmiAllReduce code - zero-copy
buffer(), in-place two-shot, one-shot + copy-out, element checks - on CPU,
world 2 and 4."""
import ctypes
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_parallel_cpu import _free_port


def _worker(rank, world, port, fn_name, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from nvidia_terraform_modules_amd.parallel import dist
    env = dist.init(backend="gloo", device_type="cpu")
    try:
        q.put((rank, globals()[fn_name](env)))
    finally:
        dist.shutdown(env)


def _run(world, fn_name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


class _ShmLib:
    """The ntm_* surface XgmiAllReduce uses, on host shared memory."""

    SIG_PER_BLOCK = 3 * 8 * 4        # [phases][ranks] u32 per block, as the kernel's

    def __init__(self, env, refuse_first: int = 0):
        from multiprocessing import shared_memory

        self._shm = shared_memory
        self.env = env
        self.own, self.opened = {}, {}
        self.calls = {"ntm_ipc_handle": 0, "ntm_ipc_open": 0, "ntm_malloc": 0,
                      "ntm_xgmi_allreduce_bf16_ex": 0, "ntm_memset_async": 0}
        self.refuse_left = refuse_first
        self.seq = 0

    def ntm_xgmi_signal_bytes(self, nblk):
        return self.SIG_PER_BLOCK * nblk

    def ntm_malloc(self, pp, nbytes, uncached):
        self.calls["ntm_malloc"] += 1
        self.seq += 1
        name = f"ntm_t{os.getpid()}_{self.seq}"
        seg = self._shm.SharedMemory(name=name, create=True, size=max(nbytes, 1))
        addr = ctypes.addressof(ctypes.c_char.from_buffer(seg.buf))
        self.own[addr] = seg
        ctypes.cast(pp, ctypes.POINTER(ctypes.c_void_p))[0] = addr
        return 0

    def ntm_free(self, p):
        seg = self.own.pop(p)
        import gc
        gc.collect()
        try:
            seg.close()
        except BufferError:          # a torch view still exports the buffer: leave it mapped
            pass
        seg.unlink()
        return 0

    def ntm_memset_async(self, p, v, nbytes, stream):
        self.calls["ntm_memset_async"] += 1
        ctypes.memset(p, v, nbytes)
        return 0

    def ntm_ipc_handle(self, p, out):
        self.calls["ntm_ipc_handle"] += 1
        if self.refuse_left:
            self.refuse_left -= 1
            return 1                  # hipErrorInvalidValue
        name = next(s.name for a, s in self.own.items() if a == p).encode()
        out.raw = name + bytes(64 - len(name))
        return 0

    def ntm_ipc_open(self, h, pp):
        self.calls["ntm_ipc_open"] += 1
        seg = self._shm.SharedMemory(name=bytes(h).rstrip(b"\0").decode())
        addr = ctypes.addressof(ctypes.c_char.from_buffer(seg.buf))
        self.opened[addr] = seg
        pp._obj.value = addr
        return 0

    def ntm_ipc_close(self, p):
        seg = self.opened.pop(p)
        import gc
        gc.collect()
        try:
            seg.close()
        except BufferError:
            pass
        return 0

    def ntm_stream_copy(self, src, dst, nbytes, stream):
        ctypes.memmove(dst, src, nbytes)
        return 0

    def ntm_xgmi_allreduce_bf16_ex(self, ins, outs, sigs, n, rank, nhere, nblk, count, epoch,
                                   err, one_shot, spin, entry_spin, stream):
        from nvidia_terraform_modules_amd.parallel.dist import barrier

        self.calls["ntm_xgmi_allreduce_bf16_ex"] += 1
        assert nblk * self.SIG_PER_BLOCK <= self.ntm_xgmi_signal_bytes(256)

        def view(ptr):
            raw = (ctypes.c_char * (count * 2)).from_address(ptr)
            return torch.frombuffer(raw, dtype=torch.bfloat16)

        barrier(self.env)                                  # entry: every input in place
        tot = sum(view(ins[q]).float() for q in range(n)).to(torch.bfloat16)
        barrier(self.env)                                  # every peer has read its inputs
        view(outs[rank]).copy_(tot)
        return 0


def _c2(env):
    """bench.py's C2 block on the stub: tune over every TUNE_NBLKS value, then
    the main sweep, one communicator."""
    from nvidia_terraform_modules_amd.parallel import xgmi as xg

    lib = _ShmLib(env)
    made = []

    def factory(nb, mb):
        ar = xg.XgmiAllReduce(env, max_bytes=mb, nblk=nb, lib=lib)
        made.append(ar)
        return ar

    n = env.world_size
    xs = [b for b in (512, 2048, 8192, 32768) if (b // 2) % (8 * n) == 0]
    out, xr = xg.c2_sweep(env, xs, 64 << 10, factory=factory, iters=1, warmup=0,
                          tune_kwargs={"sizes": (16 << 10, 64 << 10), "iters": 1, "warmup": 0})
    return {"calls": lib.calls, "communicators": len(made), "out": out,
            "leaked": len(lib.own) + len(lib.opened)}


def _refused(env):
    """One refused export on rank 0 (hipErrorInvalidValue): retried, counted,
    and the refused range freed once every export succeeded."""
    from nvidia_terraform_modules_amd.parallel import xgmi as xg

    lib = _ShmLib(env, refuse_first=1 if env.rank == 0 else 0)
    ar = xg.XgmiAllReduce(env, max_bytes=4096, nblk=16, lib=lib)
    st, rep = ar.stats(), ar.setup_report
    owned_after_setup = len(lib.own)
    ar.close()
    return {"stats": st, "report": rep, "owned": owned_after_setup, "calls": lib.calls}


@pytest.mark.parametrize("world", [2, 4])
def test_tune_and_main_sweep_share_one_communicator(world):
    from nvidia_terraform_modules_amd.parallel.xgmi import TUNE_NBLKS

    res = _run(world, "_c2")
    for rank, r in res.items():
        out = r["out"]
        assert out["ok"] is True, out
        assert r["communicators"] == 1
        assert r["calls"]["ntm_ipc_handle"] == 3, r["calls"]           # in, out, signals
        assert r["calls"]["ntm_ipc_open"] == 3 * (world - 1)
        assert r["calls"]["ntm_malloc"] == 3
        assert r["leaked"] == 0
        assert out["xgmi_exports_per_rank"] == [3] * world
        assert out["xgmi_export_retries"] == 0 and out["xgmi_export_refusals"] == []
        tune = out["xgmi_tune"]
        assert tune["shared_communicator"] is True and tune["errors"] == 0
        assert tune["nblks"] == list(TUNE_NBLKS)
        # one reconfigure per swept nblk, one for the hand-over to the main sweep
        assert out["xgmi_reconfigures"] == len(TUNE_NBLKS) + 1
        assert out["xgmi_blocks_per_rank"] == tune["best_nblk"]
        assert out["xgmi_config_source"] == "xgmi_tune"
        assert all(x["errors"] == 0 for x in out["xgmi_allreduce_bf16"])
        # every reset of the signal area is one memset: set-up + each reconfigure
        assert r["calls"]["ntm_memset_async"] == 1 + out["xgmi_reconfigures"]


def test_refused_export_is_counted_and_freed():
    res = _run(2, "_refused")
    r0, r1 = res[0], res[1]
    assert r0["stats"]["exports"] == 4 and r0["stats"]["export_retries"] == 1
    assert r1["stats"]["exports"] == 3 and r1["stats"]["export_retries"] == 0
    (ref,) = r0["stats"]["refusals"]
    assert ref["attempt"] == 1 and ref["code"] == 1
    assert ref["overlaps_prev_export"] is False       # a fresh process: nothing freed before
    assert r0["owned"] == 3                            # the refused range went back
    # every rank sees every rank's refusals
    assert [x["rank"] for x in r1["report"]["refusals"]] == [0]


def test_non_invalid_value_refusal_is_not_retried():
    """only hipErrorInvalidValue is retried; any other code raises at once."""
    from nvidia_terraform_modules_amd.parallel.xgmi import _alloc_exported

    class L:
        n = 0

        def ntm_malloc(self, pp, nbytes, uncached):
            ctypes.cast(pp, ctypes.POINTER(ctypes.c_void_p))[0] = 0x1000
            return 0

        def ntm_ipc_handle(self, p, out):
            L.n += 1
            return 2          # hipErrorOutOfMemory

    own = []
    with pytest.raises(RuntimeError, match="hipError 2"):
        _alloc_exported(L(), 64, 0, own)
    assert L.n == 1 and own == [0x1000]


def test_overlap_with_a_freed_export_is_reported():
    from nvidia_terraform_modules_amd.parallel import xgmi as xg

    xg._FREED_EXPORTS.append((0x10000, 0x1000, 0.0))
    try:
        assert xg._overlaps_freed_export(0x10800, 64)["overlaps_prev_export"] is True
        assert xg._overlaps_freed_export(0x11000, 64)["overlaps_prev_export"] is False
    finally:
        xg._FREED_EXPORTS.pop()


def _c2_bad_reconfigure(env):
    """A communicator whose reconfigure fails collectively: c2_sweep records the
    error on every rank and returns instead of raising mid-bench."""
    from nvidia_terraform_modules_amd.parallel import xgmi as xg

    class Bad(xg.ReferenceAllReduce):
        def reconfigure(self, nblk, one_shot_max_bytes=None):
            if self.reconfigures >= 2:
                raise RuntimeError("XgmiAllReduce.reconfigure failed: injected")
            super().reconfigure(nblk, one_shot_max_bytes)

    out, xr = xg.c2_sweep(env, [512, 2048], 64 << 10,
                          factory=lambda nb, mb: Bad(env, mb, nblk=nb), iters=1, warmup=0,
                          tune_kwargs={"sizes": (16 << 10,), "nblks": (16, 32, 64),
                                       "iters": 1, "warmup": 0})
    return {"ok": out["ok"], "err": out.get("xgmi_error", ""), "xr": len(xr),
            "tune_err": out["xgmi_tune"].get("error", "")}


def test_c2_sweep_survives_a_collective_reconfigure_failure():
    res = _run(2, "_c2_bad_reconfigure")
    for r in res.values():
        # the third reconfigure (inside tune) fails: tune records it, and the hand-over
        # reconfigure fails too - reported, no exception escapes, no main sweep
        assert r["ok"] is False and "injected" in r["tune_err"]
        assert "injected" in r["err"] and r["xr"] == 0
