"""C2 hand-written all-reduce: the full N-rank protocol simulated on one
MI355X (each rank's blocks co-resident), checked against a torch fp32 sum."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nranks", [1, 2, 4, 8])
@pytest.mark.parametrize("one_shot", [False, True])
@pytest.mark.parametrize("nblk", [16, 32, 64, 128, 256])   # xgmi.TUNE_NBLKS: every swept value
def test_simulated_allreduce_matches_fp32_sum(nranks, one_shot, nblk):
    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.parallel.xgmi import TUNE_NBLKS, simulate_allreduce

    assert nblk in TUNE_NBLKS
    if nranks * nblk > 1024:
        pytest.skip("all ranks' blocks must be co-resident on the one GPU")
    count = 8 * nranks * 4096 + 8 * nranks * 3   # uneven per-block slices
    ins = [ops.fill_uniform_(torch.empty(count, dtype=torch.bfloat16, device="cuda"), seed=r + 1)
           for r in range(nranks)]
    outs, err = simulate_allreduce(ins, nblk=nblk, one_shot=one_shot)
    assert err == 0
    ref = torch.stack([t.float() for t in ins]).sum(0)
    for o in outs:   # every rank holds the full, identical result
        assert torch.allclose(o.float(), ref, atol=2e-2, rtol=2 ** -7)
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("nranks", [2, 8])
def test_simulated_allreduce_in_place(nranks):
    """Two-shot with in == out (the zero-copy path of XgmiAllReduce.run)."""
    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.parallel.xgmi import simulate_allreduce

    count = 8 * nranks * 8192 + 8 * nranks * 7
    ins = [ops.fill_uniform_(torch.empty(count, dtype=torch.bfloat16, device="cuda"), seed=r + 11)
           for r in range(nranks)]
    ref = torch.stack([t.float() for t in ins]).sum(0)
    outs, err = simulate_allreduce(ins, nblk=32, inplace=True)
    assert err == 0
    for o, i in zip(outs, ins):
        assert o.data_ptr() == i.data_ptr()
        assert torch.allclose(o.float(), ref, atol=2e-2, rtol=2 ** -7)
        assert torch.equal(o, outs[0])


def test_simulated_allreduce_epochs_reuse_signals():
    """Back-to-back calls on the SAME signal buffers with increasing epochs
    (mixed one-shot / two-shot / in-place) must not see stale flags."""
    from nvidia_terraform_modules_amd.parallel.xgmi import _declare, simulate_allreduce

    n, nblk = 4, 8
    sb = _declare().ntm_xgmi_signal_bytes(nblk)
    sigs = [torch.zeros(sb // 4, dtype=torch.int32, device="cuda") for _ in range(n)]
    for epoch in range(1, 7):
        ins = [torch.full((8 * n * 1024,), float(r + epoch), dtype=torch.bfloat16, device="cuda")
               for r in range(n)]
        outs, err = simulate_allreduce(ins, nblk=nblk, epoch=epoch, sigs=sigs,
                                       one_shot=epoch % 3 == 0, inplace=epoch % 3 == 1)
        assert err == 0
        exp = sum(r + epoch for r in range(n))
        assert all(torch.all(o == exp) for o in outs)


def test_rejects_bad_counts():
    from nvidia_terraform_modules_amd.parallel.xgmi import simulate_allreduce

    ins = [torch.zeros(100, dtype=torch.bfloat16, device="cuda") for _ in range(2)]
    with pytest.raises(ValueError):
        simulate_allreduce(ins)
    ok = [torch.zeros(8 * 8 * 64, dtype=torch.bfloat16, device="cuda") for _ in range(8)]
    with pytest.raises(ValueError):      # 8 x 256 blocks cannot all be resident
        simulate_allreduce(ok, nblk=256)
    with pytest.raises(ValueError):
        simulate_allreduce(ok, one_shot=True, inplace=True)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_allreduce_processes(world):
    """XgmiAllReduce across ``world`` PROCESSES (IPC handles + cross-process
    flags), all on the one GPU of the box; every element checked exactly. At
    world 8 this is the bench's N = 8 set-up (7 peers' buffers opened per rank,
    8-way device-side barriers) minus only the xGMI links. Each worker keeps to
    one hardware queue, so the 8 ranks' kernels are co-resident rather than
    time-sliced (the barrier needs them all running)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from pathlib import Path

    worker = Path(__file__).with_name("xgmi_ipc_worker.py")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GPU_MAX_HW_QUEUES="1")
        procs.append(subprocess.Popen([sys.executable, str(worker)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            assert p.returncode == 0, e[-3000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rep in outs:
        for r in rep["results"]:
            assert not r["timeout"], rep
            assert r["wrong"] == 0, rep
        # bench.py's N > 1 C2 knob sweep (xgmi.tune), every co-resident nblk
        tune = rep["tune"]
        assert tune["errors"] == 0 and not tune["timed_out"], tune
        from nvidia_terraform_modules_amd.parallel.xgmi import TUNE_NBLKS

        assert {t["nblk"] for t in tune["table"]} == {nb for nb in TUNE_NBLKS if nb * world <= 1024}
        assert tune["best_nblk"] in {t["nblk"] for t in tune["table"]}
        # tune + main sweep on ONE communicator (3 exports per rank),
        # after a first communicator was closed; no export refused on any rank
        c2 = rep["c2"]
        assert tune["shared_communicator"] is True and c2["ok"] is True, c2
        assert c2["xgmi_exports_per_rank"] == [3] * world, c2
        assert c2["xgmi_export_retries"] == 0, c2["xgmi_export_refusals"]
        assert rep["first_comm"]["exports"] == 3 and rep["first_comm"]["export_retries"] == 0
        assert all(x["errors"] == 0 for x in c2["xgmi_allreduce_bf16"])


@pytest.mark.parametrize("one_shot", [False, True])
@pytest.mark.parametrize("nranks", [2, 8])
def test_missing_rank_times_out_with_nan(nranks, one_shot):
    """Failure contract: a rank that never launches. The others'
    entry barrier gives up after the (short, per-call) spin limit, reports
    phase 1 and fills every output element they own with NaN - never a
    silently partial sum. The limits are kernel arguments, so this takes
    milliseconds instead of the default minutes."""
    from nvidia_terraform_modules_amd.parallel.xgmi import simulate_allreduce

    count = 8 * nranks * 1024
    ins = [torch.ones(count, dtype=torch.bfloat16, device="cuda") for _ in range(nranks)]
    outs, err = simulate_allreduce(ins, nblk=8, one_shot=one_shot, nranks_here=nranks - 1,
                                   spin_limit=4096, entry_spin_limit=4096)
    assert err == 1                                   # the entry barrier
    for o in outs[:nranks - 1]:                       # the ranks that ran
        assert torch.isnan(o.float()).all()


def test_ipc_missing_rank_raises():
    """The same across two PROCESSES (IPC): rank 1 never calls; rank 0's
    ``ar(t, check=True)`` raises, names the entry phase, and its tensor is NaN."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from pathlib import Path

    worker = Path(__file__).with_name("xgmi_timeout_worker.py")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, str(worker)],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                                       GPU_MAX_HW_QUEUES="1"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(2)]
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=120)
            assert p.returncode == 0, e[-3000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    r0 = next(r for r in outs if r["rank"] == 0)
    for k in ("0", "1"):
        assert "entry phase" in r0["raised_" + k] and "NaN" in r0["raised_" + k], r0
        assert r0["all_nan_" + k], r0
    assert r0["timed_out"] is True


@pytest.mark.parametrize("nranks", [2, 8])
def test_simulated_allreduce_stress_back_to_back(nranks):
    """Race screen for the device-side barrier protocol: 120 calls back to back
    on ONE stream with no host sync between them, reusing the signal buffers
    with growing epochs, alternating one-shot / two-shot / in-place and
    changing the data every call. Exact integer patterns (every partial sum of
    <= 8 ranks is exact in bf16), every element of every call checked."""
    from nvidia_terraform_modules_amd.parallel.xgmi import _declare, _ptrs, MAX_RANKS  # noqa: F401
    from nvidia_terraform_modules_amd.ops._lib import check, stream_handle

    L = _declare()
    nblk = 1024 // nranks // 4
    count = 8 * nranks * 2048 + 8 * nranks * 5
    sb = L.ntm_xgmi_signal_bytes(nblk)
    sigs = [torch.zeros(sb // 4, dtype=torch.int32, device="cuda") for _ in range(nranks)]
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    base = (2.0 ** (torch.arange(count, device="cuda") % 4))
    outs_keep, exps = [], []
    for it in range(120):
        one_shot, inplace = it % 3 == 0, it % 3 == 2
        ins = [(base * ((r + it) % 5 + 1)).to(torch.bfloat16) for r in range(nranks)]
        outs = ins if inplace else [torch.empty_like(t) for t in ins]
        rc = L.ntm_xgmi_allreduce_bf16(
            _ptrs([t.data_ptr() for t in ins]), _ptrs([t.data_ptr() for t in outs]),
            _ptrs([s.data_ptr() for s in sigs]), nranks, 0, nranks, nblk, count, it + 1,
            err.data_ptr(), 1 if one_shot else 0, stream_handle())
        check(rc, "xgmi")
        outs_keep.append(outs)
        exps.append(base * sum((r + it) % 5 + 1 for r in range(nranks)))
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    for it, (outs, exp) in enumerate(zip(outs_keep, exps)):
        e = exp.to(torch.bfloat16)
        for o in outs:
            assert torch.equal(o, e), f"call {it}"
