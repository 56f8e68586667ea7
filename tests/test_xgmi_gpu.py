"""C2 hand-written all-reduce: the full N-rank protocol simulated on one
MI355X (each rank's blocks co-resident), checked against a torch fp32 sum."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nranks", [1, 2, 4, 8])
@pytest.mark.parametrize("one_shot", [False, True])
def test_simulated_allreduce_matches_fp32_sum(nranks, one_shot):
    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.parallel.xgmi import simulate_allreduce

    count = 8 * nranks * 4096 + 8 * nranks * 3   # uneven per-block slices
    ins = [ops.fill_uniform_(torch.empty(count, dtype=torch.bfloat16, device="cuda"), seed=r + 1)
           for r in range(nranks)]
    outs, err = simulate_allreduce(ins, nblk=16, one_shot=one_shot)
    assert err == 0
    ref = torch.stack([t.float() for t in ins]).sum(0)
    for o in outs:   # every rank holds the full, identical result
        assert torch.allclose(o.float(), ref, atol=2e-2, rtol=2 ** -7)
        assert torch.equal(o, outs[0])


def test_simulated_allreduce_epochs_reuse_signals():
    """Back-to-back calls with increasing epochs must not see stale flags."""
    from nvidia_terraform_modules_amd.parallel.xgmi import simulate_allreduce

    n = 4
    for epoch in (1, 2, 3):
        ins = [torch.full((8 * n * 1024,), float(r + epoch), dtype=torch.bfloat16, device="cuda")
               for r in range(n)]
        outs, err = simulate_allreduce(ins, nblk=8, epoch=epoch)
        assert err == 0
        exp = sum(r + epoch for r in range(n))
        assert all(torch.all(o == exp) for o in outs)


def test_rejects_bad_counts():
    from nvidia_terraform_modules_amd.parallel.xgmi import simulate_allreduce

    ins = [torch.zeros(100, dtype=torch.bfloat16, device="cuda") for _ in range(2)]
    with pytest.raises(ValueError):
        simulate_allreduce(ins)


def test_ipc_allreduce_two_processes():
    """XgmiAllReduce across two PROCESSES (IPC handles + cross-process flags),
    both on the one GPU of the box; every element checked exactly."""
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
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
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
