"""bench.py's multi-process orchestration, rehearsed on CPU (gloo + reference
ops): the same launch path the driver uses for N = 2/4/8 on an MI355X node
(torch.distributed.run, RANK/WORLD_SIZE env, barrier + max over ranks, ONE
JSON line from rank 0). Numbers here are not measurements."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CONTRACT_KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(stdout):
    out = []
    for ln in stdout.splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            out.append(json.loads(ln))
    return out


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "1"
    return e


@pytest.mark.parametrize("nproc", [1, 2, 4, 8])
def test_torchrun_launch_one_json_line(nproc):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           str(ROOT / "bench.py"), "--gpus", str(nproc), "--steps", "3", "--warmup", "1",
           "--size", "256", "--allreduce-max-mib", "1", "--rehearsal", "--p2p", "--prewarm-s", "0.2"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]          # rank 0 only
    d = lines[0]
    assert CONTRACT_KEYS <= set(d)
    baseline = json.loads((ROOT / "BASELINE.json").read_text())
    assert d["metric"] == baseline["metric"]                # BASELINE.json's metric, verbatim
    assert d["n_gpus"] == nproc and d["steps"] == 3 and d["warmup"] == 1
    assert d["config"]["parallelism"] == f"dp{nproc}" and d["config"]["global_batch"] == nproc
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert d["value"] > 0 and d["verified"] is True and d["rehearsal"] is True
    assert "extras_timed_out" not in d                  # the deadline did not fire
    topo = d["node_topology"]                           # what the run ran on, per rank
    assert [r["rank"] for r in topo["ranks"]] == list(range(nproc))
    assert topo["torch"]
    assert "NOT a measurement" in d["data"]
    # clock-settle pre-warm (untimed, wall-time based) and event timing are reported
    assert d["prewarm_s"] >= 0.2 and d["prewarm_launches"] > 0
    assert d["timed_region_wall_s"] > 0 and "HIP events" in d["timing"]
    # the Job binary step runs (here: no GPU -> its environment-error verdict) and the
    # other ranks have left before it without breaking the one-line contract
    job = d["validation_job"]
    assert job["ran"] is False or job["passed"] is False
    assert d["time_to_gpu_ready_in_node_s"] is None
    # per-rank view of the weak-scaling run: every rank's own
    # TF/s, the clock its GEMM ran at and its MFMA-load clock (None on the CPU rehearsal)
    assert len(d["per_rank_tflops"]) == nproc and all(t > 0 for t in d["per_rank_tflops"])
    assert d["per_rank_clock_GHz"] == [None] * nproc
    assert len(d["per_rank_clock_probe"]) == nproc
    assert d["per_rank_gemm_clock_GHz"] == [None] * nproc
    assert d["per_rank_gemm_clock_p10_GHz"] == [None] * nproc
    assert len(d["per_rank_gemm_clock"]) == nproc
    # the timed loop's own clock and each rank's power / throttle
    # window are reported per rank (None without a GPU)
    assert d["per_rank_timed_loop_clock_GHz"] == [None] * nproc
    assert d["per_rank_power"] == [None] * nproc
    assert d["per_rank_power_steady"] == [None] * nproc
    assert d["per_rank_power_window"] == [None] * nproc
    assert d["per_rank_avg_power_W"] == [None] * nproc
    assert d["per_rank_ppt_throttle_pct"] == [None] * nproc
    assert d["per_rank_thermal_throttle_pct"] == [None] * nproc
    if nproc > 1:
        # C2 knob sweep: blocks per rank 16..256 x one/two-shot at the
        # tune sizes that fit the sweep cap (1 MiB here; 64 / 256 MiB on a real node),
        # best per size, the favoured cutoff and ONE best nblk (over torch.distributed
        # here: shape only) - and the main C2 sweep runs exactly that configuration
        from nvidia_terraform_modules_amd.parallel.xgmi import TUNE_NBLKS, TUNE_SIZES

        tune = d["xgmi_tune"]
        assert tune["errors"] == 0 and tune["timed_out"] is False
        assert tune["nblks"] == list(TUNE_NBLKS) and tune["nblks_skipped"] == []
        assert max(TUNE_SIZES) == 256 << 20 and max(TUNE_NBLKS) == 256
        assert tune["sizes"] == [s for s in TUNE_SIZES if s <= 1 << 20]
        assert {r["nblk"] for r in tune["table"]} == set(tune["nblks"])
        one = [r for r in tune["table"] if r["algo"] == "1shot"]
        assert one and all(r["bytes"] <= max(tune["cutoffs"]) for r in one)
        assert len(tune["best_per_size"]) == len(tune["sizes"])
        assert tune["best_one_shot_max_bytes"] in tune["cutoffs"]
        assert set(tune["cutoff_total_time_us"]) == {str(c) for c in tune["cutoffs"]}
        assert tune["best_nblk"] in tune["nblks"]
        assert d["xgmi_config_source"] == "xgmi_tune"
        assert d["xgmi_blocks_per_rank"] == tune["best_nblk"]
        # (the shared communicator is sized for the larger of the two sweeps)
        comm_bytes = max([r["bytes"] for r in d["xgmi_allreduce_bf16"]] + tune["sizes"])
        assert d["xgmi_one_shot_max_bytes"] == min(tune["best_one_shot_max_bytes"], comm_bytes)
        assert all(r["errors"] == 0 for r in d["xgmi_allreduce_bf16"])
        # tune and the main sweep share ONE communicator (one
        # reconfigure per swept nblk + the hand-over); set-up accounting per rank
        assert tune["shared_communicator"] is True
        assert d["xgmi_reconfigures"] == len(tune["nblks"]) + 1
        assert d["xgmi_exports_per_rank"] == [0] * nproc     # the reference path exports nothing
        assert d["xgmi_export_retries"] == 0 and d["xgmi_export_refusals"] == []
    if nproc > 1:
        assert all(r["errors"] == 0 for r in d["allreduce_bf16"] + d["allreduce_fp32"])
        assert d["allreduce_bf16"][0]["bytes"] == 8
        pm = d["p2p_send_GBps"]
        assert pm["ranks"] == nproc and pm["errors"] == 0 and pm["min_GBps"] > 0


@pytest.mark.parametrize("phase", ["xgmi", "rccl_sweep"])
def test_hung_collective_still_prints_the_line(phase):
    """A peer that hangs after the timed region (here rank 1, injected at the start
    of a collective phase) must not swallow the JSON line: at the extras deadline
    rank 0 prints the line it has, naming the phase, and every rank exits."""
    env = _env()
    env["NTM_BENCH_INJECT_HANG"] = f"{phase}:1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--size", "256",
           "--allreduce-max-mib", "1", "--rehearsal", "--prewarm-s", "0.1",
           "--extras-timeout-s", "25"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout[-2000:]
    d = lines[0]
    assert CONTRACT_KEYS <= set(d) and d["value"] > 0 and d["n_gpus"] == 2
    assert d["extras_timed_out"] == phase and d["extras_timeout_s"] == 25
    assert d["verified"] is True            # the GEMM check ran before the hang
    assert "validation_job" not in d
    if phase == "xgmi":                     # what ran before the hang is kept
        assert d["allreduce_bf16"] and "xgmi_allreduce_bf16" not in d
    else:
        assert "allreduce_bf16" not in d


def test_extras_watchdog_ownership():
    """Exactly one of the main thread and the deadline prints the line: a claim
    before the deadline cancels it; a deadline that fired first keeps it."""
    import threading
    import time

    sys.path.insert(0, str(ROOT))
    import bench

    fired, exited = threading.Event(), []

    def on_expire(phase):
        fired.set()
        return 7

    wd = bench.ExtrasWatchdog(0.2, 0, on_expire, exit_fn=exited.append)
    assert wd.claim() is True
    time.sleep(0.4)
    assert not fired.is_set() and exited == []
    wd = bench.ExtrasWatchdog(0.05, 0, on_expire, exit_fn=exited.append)
    wd.enter("xgmi")
    assert fired.wait(2.0)
    time.sleep(0.05)
    assert exited == [7] and wd.claim() is False
    assert bench.ExtrasWatchdog(0, 0, on_expire).claim() is True     # 0 = no deadline


def test_select_k1_keeps_the_default_unless_clearly_faster(monkeypatch):
    """select_k1 times the candidate K1 builds interleaved and switches away from
    the default plan only for a median K1_SELECT_MARGIN faster."""
    import types

    sys.path.insert(0, str(ROOT))
    import bench

    wl = types.SimpleNamespace(m=8192, n=8192, k=8192, a=None, b=None, c=None,
                               flops=2.0 * 8192 ** 3, variant="default", step=lambda: None)
    calls = []
    backend = types.SimpleNamespace(
        k1_candidates=lambda m, n, k: ["default", "dma4k_d3"],
        gemm_bf16=lambda a, b, c, variant="default": calls.append(variant))
    monkeypatch.setattr(bench, "prewarm_settle", lambda fn, sync, s: fn())
    for t_alt, want in ((0.990, "dma4k_d3"), (0.997, "default"), (1.02, "default")):
        monkeypatch.setattr(bench, "interleaved_compare", lambda fns, dev, rounds, launches, t=t_alt: {
            "default": {"median_s": 1.0}, "dma4k_d3": {"median_s": t}})
        wl.variant = "default"
        sel = bench.select_k1(wl, backend, None, lambda: None)
        assert sel["chosen"] == wl.variant == want
        assert set(sel["tflops_median"]) == {"default", "dma4k_d3"}
    assert {"default", "dma4k_d3"} <= set(calls)          # both builds really ran
    one = types.SimpleNamespace(k1_candidates=lambda m, n, k: ["default"])
    assert bench.select_k1(wl, one, None, lambda: None) is None


def test_k1_candidates_shape_rule():
    from nvidia_terraform_modules_amd.ops.kernels import k1_candidates

    assert k1_candidates(8192, 8192, 8192) == ["default", "dma4k_d3"]
    assert k1_candidates(8192, 8192, 4096) == ["default", "dma4k_d3"]
    assert k1_candidates(8192, 8000, 8192) == ["default"]        # N % 256
    assert k1_candidates(4096, 4096, 192) == ["default"]         # K % 128 and K >= 256
    assert k1_candidates(256, 256, 8192, lda=8196) == ["default"]  # 16-B rows


def test_self_relaunch_as_child_process():
    """`python bench.py --gpus 2` without WORLD_SIZE starts torch.distributed.run
    as a CHILD (never exec) and propagates its exit status."""
    env = _env()
    env["MASTER_PORT"] = str(_port())
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--size", "256", "--allreduce-max-mib", "1", "--rehearsal"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2


@pytest.mark.gpu
def test_bench_on_one_gpu_json_contract(tmp_path):
    """The real path on one MI355X (small config): one JSON line with the contract keys,
    verified GEMM, hipBLASLt comparison, HBM check and the Job binary's verdict time."""
    out = tmp_path / "b.json"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "5", "--warmup", "2",
                        "--size", "2048", "--out", str(out)],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert CONTRACT_KEYS <= set(d) and d["n_gpus"] == 1 and d["verified"] is True
    assert d["value"] > 50 and "rehearsal" not in d
    # the K1 build the timed loop ran: the faster hand-written one on this box
    sel = d["per_rank_k1_selection"][0]
    assert d["per_rank_k1_variant"][0] == sel["chosen"] in ("default", "dma4k_d3")
    assert all(v > 0 for v in sel["tflops_median"].values())
    topo = d["node_topology"]
    assert topo["ranks"][0]["cus"] == 256 and "gfx950" in (topo["ranks"][0]["gcn_arch"] or "")
    assert topo["visible_gpus"] >= 1 and topo["peer_access"][0][0] is True
    assert d["hipblaslt_tflops_per_gpu_rank0"] > 0 and d["hbm_copy_GBps_rank0"] > 1000
    cmp_ = d["interleaved_compare_rank0"]       # K1 vs hipBLASLt, ABAB rounds
    assert cmp_["rounds"] == len(cmp_["k1_tflops_rounds"]) == len(cmp_["hipblaslt_tflops_rounds"])
    assert cmp_["k1_over_hipblaslt"] > 0.5 and d["prewarm_s"] >= 0.5
    # the GEMM's own clock (stamped build) and the MFMA-only probe's, both plausible
    g = d["per_rank_gemm_clock"][0]
    assert 0.5 < d["per_rank_gemm_clock_GHz"][0] < 3.0, g
    assert g["p10_GHz"] <= g["median_GHz"] and g["workgroups"] > 0
    assert 0.5 < d["per_rank_clock_GHz"][0] < 3.0
    # at 2048^3 the timed loop runs a small tile, not the clock build's pingpong8o:
    # no timed-loop clock is derived from the clock build's cycles
    assert d["per_rank_timed_loop_clock_GHz"] == [None]
    pw = d["per_rank_power"][0]
    assert "error" not in pw, pw
    # (a 5-step 2048^3 window is shorter than the metrics refresh: stale, no 0 W)
    assert pw["avg_power_W"] is None or pw["avg_power_W"] > 0, pw
    assert pw["stale"] is (pw["avg_power_W"] is None), pw
    # the >= 0.5 s steady-state window beside it always has data, and the reported
    # power comes from whichever window advanced
    st = d["per_rank_power_steady"][0]
    assert "error" not in st and st["seconds"] >= 0.5 and st["stale"] is False, st
    assert 50 < st["avg_power_W"] < 2000 and 0 <= st["ppt_pct"] <= 100, st
    src = d["per_rank_power_window"][0]
    assert src == ("timed_loop" if pw["avg_power_W"] is not None and pw["seconds"] >= 0.1
                   else "steady_window")
    assert d["per_rank_avg_power_W"][0] == (pw if src == "timed_loop" else st)["avg_power_W"]
    # the stream-K split-mode shape through the default dispatch under
    # NTM_SK_CHECK=1, verified and with a clear placement word
    sk = d["sk_check_rank0"]
    assert sk["ok"] and sk["bad"] == 0 and sk["sk_xcc_error"] == 0, sk
    assert sk["variant"] in ("pp192x256s", "pp256x192s") and d["sk_xcc_error"] == 0
    # every SMI read is timed, the stamped clock batch count is
    # reported, and both kernels' energy per flop is measured
    assert len(d["per_rank_smi_sample_ms"][0]) >= 5
    assert 1 <= d["per_rank_clock_batches"][0] <= 3
    assert 0.1 < d["k1_joules_per_tflop"] < 10 and 0.1 < d["hipblaslt_joules_per_tflop"] < 10
    en = d["energy_rank0"]
    assert en["order"] == ["k1", "hipblaslt", "hipblaslt", "k1"]
    assert all(s >= 0.6 for s in en["k1"]["windows_s"] + en["hipblaslt"]["windows_s"]), en
    job = d["validation_job"]
    assert job["ran"] and job["passed"], job
    assert 0 < d["time_to_gpu_ready_in_node_s"] < 30
    assert json.loads(out.read_text()) == d


def test_pair_busbw_pairs_xgmi_with_rccl_sizes():
    """bench.py's C2-vs-RCCL table: one row per size both sweeps ran; the xGMI
    sweep's sizes are a subset of the RCCL bf16 sweep's (512 B .. 1 GiB)."""
    from types import SimpleNamespace as R

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from nvidia_terraform_modules_amd.parallel import collectives as coll

    rccl = [R(bytes=b, busbw_GBps=100.0 + i) for i, b in enumerate(coll.sweep_sizes(8, 1 << 33, 4))]
    n = 8
    xs = [b for b in coll.sweep_sizes(8, 1 << 33, 4) if 512 <= b <= 1 << 30 and (b // 2) % (8 * n) == 0]
    assert xs and set(xs) <= {r.bytes for r in rccl}
    xgmi = [R(bytes=b, busbw_GBps=200.0) for b in xs]
    rows = bench.pair_busbw(rccl, xgmi)
    assert [r["bytes"] for r in rows] == xs
    assert all(r["xgmi_over_rccl"] > 1.0 for r in rows)
    assert bench.pair_busbw([R(bytes=512, busbw_GBps=0.0)], [R(bytes=512, busbw_GBps=1.0)])[0][
        "xgmi_over_rccl"] is None


def test_power_window_samples_under_load():
    """bench.power_window: both telemetry samples are read while launches are
    queued (never on an idle GPU), and the window covers at least min_s."""
    sys.path.insert(0, str(ROOT))
    import bench

    queued, events = [0], []

    def fn():
        queued[0] += 1

    def sync():
        queued[0] = 0
        events.append("sync")

    def sample():
        events.append(("sample", queued[0]))
        return {"host_ns": len(events)}

    before, after, run = bench.power_window(fn, sync, sample, 0.05, chunk=4)
    samples = [e for e in events if e != "sync"]
    assert samples == [("sample", 4), ("sample", 4)]
    assert events[-1] == "sync" and events.index(samples[0]) == 0
    assert run["seconds"] >= 0.05 and run["launches"] >= 4
    assert before["host_ns"] < after["host_ns"]


def test_energy_compare_abba_joules_per_tflop():
    """bench.energy_compare: ABBA windows, each >= window_s of one
    kernel, J/TFLOP = mean window power / that kernel's TF/s."""
    sys.path.insert(0, str(ROOT))
    import bench

    t = [0.0]
    cur = {"k": None}
    power = {"a": 1400.0, "b": 1500.0}
    energy = [0.0]

    def mk(name):
        def fn():
            cur["k"] = name
            t[0] += 0.001
            energy[0] += power[name] * 0.001
        return fn

    def sample():
        return {"host_ns": int(t[0] * 1e9), "energy_uj": int(energy[0] * 1e6)}

    class Smi:
        @staticmethod
        def window(b, a):
            from nvidia_terraform_modules_amd.ops import smi
            return smi.window(b, a)

    out = bench.energy_compare({"a": (mk("a"), 1600.0), "b": (mk("b"), 1500.0)},
                               lambda: None, sample, Smi, window_s=0.01)
    assert out["order"] == ["a", "b", "b", "a"]
    assert out["a"]["avg_power_W"] == pytest.approx(1400.0, rel=1e-3)
    assert out["a"]["joules_per_tflop"] == pytest.approx(1400 / 1600, rel=1e-3)
    assert out["b"]["joules_per_tflop"] == pytest.approx(1.0, rel=1e-3)
    assert out["a_over_b_joules_per_tflop"] == pytest.approx(0.875, rel=1e-3)
    assert len(out["a"]["windows_W"]) == 2


def test_gemm_clock_stable_restamps_a_drifting_batch(monkeypatch):
    """kernels.gemm_clock_stable: a batch whose per-launch windows
    drift > 3 % is stamped again (up to 3), each behind the pre-queued launches."""
    from nvidia_terraform_modules_amd.ops import kernels

    batches = iter([[640.0, 861.0, 664.0], [660.0, 668.0, 664.0], [600.0, 700.0, 650.0]])
    calls = []

    def fake(a, b, out=None, steps=1, prequeue=None, prequeue_launches=0):
        calls.append(prequeue_launches)
        return {"per_launch_window_us_median": next(batches), "bound_GHz": 1.6}

    monkeypatch.setattr(kernels, "gemm_clock_ghz", fake)
    r = kernels.gemm_clock_stable(None, None, steps=3, prequeue=lambda: None,
                                  prequeue_launches=40)
    assert r["clock_batches"] == 2 and r["clock_stable"] is True
    assert r["per_launch_window_us_median"] == [660.0, 668.0, 664.0]
    assert r["clock_batch_drift_pct"][0] > 30 and r["clock_batch_drift_pct"][1] < 3
    assert calls == [40, 40]
    # never stable: the least drifted of the 3 batches, flagged
    batches = iter([[600.0, 700.0], [600.0, 640.0], [600.0, 900.0]])
    r = kernels.gemm_clock_stable(None, None, steps=2, prequeue=lambda: None)
    assert r["clock_batches"] == 3 and r["clock_stable"] is False
    assert r["per_launch_window_us_median"] == [600.0, 640.0]


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu_real_kernels(tmp_path):
    """The N > 1 path with the real kernels (VERDICT r5 #1's first-8-GPU-run risk,
    rehearsed on one GPU): 2 ranks on cuda:0 with a gloo group. C2 runs the real
    XgmiAllReduce over HIP IPC - tune and the main sweep on one communicator, 3
    exports per rank, no refusal - and every per-rank GPU probe (clock batches,
    energy, SMI timings) comes back from both ranks."""
    env = _env()
    env["GPU_MAX_HW_QUEUES"] = "1"      # both ranks' C2 blocks co-resident
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--size", "2048",
           "--allreduce-max-mib", "16", "--shared-gpu", "--no-job", "--compare-rounds", "3"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["shared_gpu_rehearsal"] is True and d["verified"] is True
    assert "NOT a measurement" in d["data"]
    assert d["xgmi_exports_per_rank"] == [3, 3] and d["xgmi_export_retries"] == 0, d.get(
        "xgmi_export_refusals")
    assert d["xgmi_tune"]["shared_communicator"] is True and d["xgmi_tune"]["errors"] == 0
    assert d["xgmi_timed_out"] is False
    assert all(r["errors"] == 0 for r in d["xgmi_allreduce_bf16"] + d["allreduce_bf16"])
    assert len(d["per_rank_clock_batches"]) == 2 and all(d["per_rank_clock_batches"])
    assert len(d["per_rank_smi_sample_ms"]) == 2
    assert d["k1_joules_per_tflop"] and d["sk_check_rank0"]["ok"]
