"""Distributed harness on CPU: gloo backend, world_size 2 (and 4), real
process groups via torch.multiprocessing (127.0.0.1 rendezvous)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from nvidia_terraform_modules_amd.parallel import collectives as coll


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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


def _sweep(env):
    res = coll.all_reduce_sweep(env, coll.sweep_sizes(8, 1 << 16, 4), dtype="bf16", iters=2, warmup=1)
    res32 = coll.all_reduce_sweep(env, [1024], dtype="fp32", iters=2, warmup=1)
    return [r.as_dict() for r in res + res32]


def _p2p(env):
    return coll.p2p_matrix(env, nbytes=1 << 16, iters=2).as_dict()


def _faulty_sweep(env):
    import torch.distributed as tdist

    def impl(t):
        if env.rank == 1:
            t.view(-1)[3] += 1
        tdist.all_reduce(t)
    res = coll.all_reduce_sweep(env, [4096], dtype="bf16", iters=1, warmup=0, impl=impl)
    return res[0].errors


def _consensus(env):
    from nvidia_terraform_modules_amd.parallel import dist
    mx = dist.all_reduce_max(env, float(env.rank * 10))
    sm = dist.all_reduce_sum(env, 1.0)
    objs = dist.all_gather_obj(env, {"rank": env.rank})
    return mx, sm, [o["rank"] for o in objs]


def test_bus_factor_and_sizes():
    assert coll.bus_factor("all_reduce", 8) == pytest.approx(1.75)
    assert coll.bus_factor("all_gather", 4) == pytest.approx(0.75)
    assert coll.bus_factor("all_reduce", 1) == 0.0
    assert coll.sweep_sizes(8, 64) == [8, 16, 32, 64]
    with pytest.raises(ValueError):
        coll.sweep_sizes(0, 64)


def test_pattern_exact_in_bf16():
    # expected sums stay exactly representable for up to 8 ranks
    for n in range(1, 9):
        exp = coll._expected(4096, n, torch.bfloat16, "cpu").float()
        acc = sum(coll._pattern(4096, r, torch.bfloat16, "cpu").float() for r in range(n))
        assert torch.equal(acc, exp)


def test_allreduce_sweep_gloo_world2():
    out = _run(2, "_sweep")
    for rank, res in out.items():
        assert all(r["errors"] == 0 for r in res), res
        assert all(r["ranks"] == 2 for r in res)
        assert all(r["busbw_GBps"] == pytest.approx(r["algbw_GBps"]) for r in res)  # 2(n-1)/n = 1


def test_allreduce_detects_corrupted_rank():
    out = _run(2, "_faulty_sweep")
    assert out[0] > 0 and out[1] > 0   # every rank sees the bad element


def test_consensus_helpers_world4():
    out = _run(4, "_consensus")
    for rank, (mx, sm, ranks) in out.items():
        assert mx == 30.0 and sm == 4.0 and ranks == [0, 1, 2, 3]


def test_single_rank_sweep_has_no_group():
    from nvidia_terraform_modules_amd.parallel import dist
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    env = dist.init(backend="gloo", device_type="cpu")
    assert env.world_size == 1 and env.is_main
    res = coll.all_reduce_sweep(env, [64], iters=1, warmup=0)
    assert res[0].errors == 0 and res[0].busbw_GBps == 0.0


def _validation_job(env):
    """The validation Job's multi-rank logic (reference ops on CPU): the last
    rank's GEMM is corrupted; EVERY rank must report failure (consensus)."""
    from nvidia_terraform_modules_amd.models.validation_job import ValidationConfig, run_validation
    from nvidia_terraform_modules_amd.ops import reference

    cfg = ValidationConfig(size=256, gemm_iters=2, gemm_warmup=1, abft_iters=1,
                           hbm_bytes=1 << 16, hbm_iters=1, allreduce_min_bytes=1 << 10,
                           allreduce_max_bytes=1 << 14, allreduce_iters=1,
                           fault_inject="corrupt_gemm")
    rep = run_validation(env, cfg, backend=reference)
    clean = ValidationConfig(size=256, gemm_iters=2, gemm_warmup=1, abft_iters=1,
                             hbm_bytes=1 << 16, hbm_iters=1, allreduce_min_bytes=1 << 10,
                             allreduce_max_bytes=1 << 14, allreduce_iters=1, fault_inject="")
    rep2 = run_validation(env, clean, backend=reference)
    return rep.passed, rep.failures, rep2.passed, len(rep2.allreduce)


def test_validation_job_consensus_world2():
    out = _run(2, "_validation_job")
    # rank 1 (last) is corrupted: it names the GEMM, rank 0 learns via consensus
    assert out[1][0] is False and any("gemm verification" in f for f in out[1][1])
    assert out[0][0] is False and any("another rank" in f for f in out[0][1])
    for rank in (0, 1):
        assert out[rank][2] is True and out[rank][3] > 0   # clean run passes, sweep ran


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_matrix_every_ordered_pair(world):
    out = _run(world, "_p2p")
    m = out[0]
    assert all(out[r] == m or out[r]["GBps"] == m["GBps"] for r in out)   # same matrix everywhere
    assert m["ranks"] == world and m["errors"] == 0 and m["bytes"] == 1 << 16
    for d in range(world):
        for s in range(world):
            v = m["GBps"][d][s]
            assert (v is None) == (d == s)
            assert d == s or v > 0
    assert m["min_GBps"] > 0
