"""The standalone ``amdgpu-validate`` Job binary (validation/src/validate_main.cpp).

CPU tests cover argument handling and the no-GPU environment error (exit 2);
GPU tests run the real checks on one MI355X, including native fault injection
(the binary must exit 1 and name the failed check) and the Kubernetes
termination-message / Prometheus textfile outputs.
"""
import json
import os
import socket
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "validation" / "build" / "amdgpu-validate"


def _have_bin():
    if not BIN.exists():
        pytest.skip("amdgpu-validate not built (python -m nvidia_terraform_modules_amd.ops.build)")


def _run(*args, env=None, timeout=300):
    e = dict(os.environ)
    e.pop("NTM_FAULT_INJECT", None)
    e.pop("NODE_NAME", None)          # set per test: the outputs then carry it
    e.update(env or {})
    p = subprocess.run([str(BIN), *args], capture_output=True, text=True, timeout=timeout, env=e)
    return p.returncode, p.stdout, p.stderr


def test_rejects_unknown_argument():
    _have_bin()
    rc, _, err = _run("--definitely-not-an-option", timeout=60)
    assert rc == 2 and "usage" in err


def test_no_gpu_is_environment_error():
    _have_bin()
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    rc, out, _ = _run("--size", "256", timeout=60, env={"NODE_NAME": "gpu-node-3"})
    assert rc == 2
    rep = json.loads(out.strip().splitlines()[-1])
    assert rep["passed"] is False and rep["node"] == "gpu-node-3"   # the Job's pod names its node


def _last_json(out):
    return json.loads(out.strip().splitlines()[-1])


@pytest.mark.gpu
def test_binary_passes_and_writes_sidecar_outputs(tmp_path):
    _have_bin()
    term, prom, full = tmp_path / "term", tmp_path / "m.prom", tmp_path / "full.json"
    rc, out, err = _run("--gpus", "1", "--size", "2048", "--iters", "10", "--min-hbm-gb", "250",
                        "--termination-log", str(term), "--prom-out", str(prom),
                        "--out", str(full))
    assert rc == 0, out + err
    rep = _last_json(out)
    assert rep["passed"] and rep["gpus"][0]["gemm_wrong"] == 0
    assert rep["gpus"][0]["abft_bad_rows"] == 0
    assert rep["gpus"][0]["gemm_fp8_wrong"] == 0 and rep["gpus"][0]["gemm_fp8_tflops"] > 0
    assert rep["gpus"][0]["gemm_fp8_abft_bad_rows"] == 0
    assert rep["gpus"][0]["hbm_read_GBps"] > 1000
    # the stream-K split-mode self-check ran on a 192-wide tile,
    # matched the fp32 reference and left the placement error word zero
    g0 = rep["gpus"][0]
    assert g0["sk_split_variant"] in (54, 55) and g0["sk_split_wrong"] == 0, g0
    assert g0["sk_xcc_error"] == 0 and 0 < g0["sk_split_ms"] < 50, g0
    assert rep["start_epoch_s"] > 1.6e9 and rep["end_epoch_s"] >= rep["start_epoch_s"]
    t = json.loads(term.read_text())
    assert t["passed"] is True and len(term.read_bytes()) < 4096
    metrics = prom.read_text()
    assert "amdgpu_validate_passed 1" in metrics
    assert 'amdgpu_validate_gemm_tflops{gpu="0"}' in metrics
    assert 'amdgpu_validate_gemm_fp8_tflops{gpu="0"}' in metrics
    assert json.loads(full.read_text()) == rep


@pytest.mark.gpu
def test_binary_names_its_node_in_every_output(tmp_path):
    """One validation pod per GPU node: the Job sets NODE_NAME (downward API), and
    the verdict, the termination message and the metrics carry it."""
    _have_bin()
    term, prom = tmp_path / "term", tmp_path / "m.prom"
    rc, out, err = _run("--gpus", "1", "--size", "1024", "--iters", "5", "--no-fp8",
                        "--termination-log", str(term), "--prom-out", str(prom),
                        env={"NODE_NAME": "gpu-node-7"})
    assert rc == 0, out + err
    assert _last_json(out)["node"] == "gpu-node-7"
    assert json.loads(term.read_text())["node"] == "gpu-node-7"
    assert 'amdgpu_validate_passed{node="gpu-node-7"} 1' in prom.read_text()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,needle", [("corrupt_gemm", "GEMM verification failed"),
                                         ("corrupt_abft", "ABFT"),
                                         ("corrupt_fp8", "fp8 GEMM verification failed"),
                                         ("corrupt_fp8_abft", "fp8 GEMM ABFT checksum failed")])
def test_binary_fault_injection_fails_loudly(tmp_path, kind, needle):
    _have_bin()
    term = tmp_path / "term"
    rc, out, _ = _run("--size", "1024", "--iters", "5", "--termination-log", str(term),
                      env={"NTM_FAULT_INJECT": kind})
    assert rc == 1
    rep = _last_json(out)
    assert not rep["passed"] and any(needle in f for f in rep["failures"])
    assert json.loads(term.read_text())["passed"] is False


@pytest.mark.gpu
def test_binary_sk_placement_fault_fails_the_job(tmp_path):
    """NTM_FAULT_INJECT=sk_xcc makes the split-mode launch claim a
    wrong XCC; the kernel's placement check sets the error word and the Job fails
    (exit 1) naming it - with C still numerically right, so only the word can
    catch it. The Job's verdict stays under 1 s at 1 GPU without the fault."""
    _have_bin()
    rc, out, _ = _run("--size", "1024", "--iters", "5", "--no-fp8",
                      env={"NTM_FAULT_INJECT": "sk_xcc"})
    rep = _last_json(out)
    assert rc == 1 and not rep["passed"]
    g0 = rep["gpus"][0]
    assert g0["sk_xcc_error"] & 0x80000000, g0
    assert any("different XCDs" in f for f in rep["failures"]), rep["failures"]
    rc, out, _ = _run("--gpus", "1", "--size", "8192", "--iters", "10")
    rep = _last_json(out)
    assert rc == 0 and rep["gpus"][0]["sk_xcc_error"] == 0
    assert rep["phases_s"]["end"] < 1.0, rep["phases_s"]


@pytest.mark.gpu
def test_binary_p2p_matrix_loopback_and_fault():
    """C3 (per-link xGMI pull matrix) on one GPU: --p2p-loopback runs the pair
    path as 0 <- 0; the copy is verified and a corrupted byte fails the Job."""
    _have_bin()
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8")
    g = _last_json(out)
    assert rc == 0 and g["xgmi_p2p_GBps"] == [] and g["xgmi_p2p_min_GBps"] is None
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--p2p-loopback",
                      "--p2p-mib", "64")
    g = _last_json(out)
    assert rc == 0, g["failures"]
    assert len(g["xgmi_p2p_GBps"]) == 1 and g["xgmi_p2p_GBps"][0][0] > 100
    assert g["xgmi_p2p_bad_pairs"] == 0 and g["xgmi_p2p_min_GBps"] > 100
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--p2p-loopback",
                      "--p2p-mib", "64", env={"NTM_FAULT_INJECT": "corrupt_p2p"})
    g = _last_json(out)
    assert rc == 1 and g["xgmi_p2p_bad_pairs"] == 1
    assert any("xGMI P2P copy" in f for f in g["failures"])
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--p2p-loopback",
                      "--p2p-mib", "64", "--p2p-floor-gbps", "1e9")
    assert rc == 1 and any("below floor" in f for f in _last_json(out)["failures"])


@pytest.mark.gpu
def test_binary_rccl_one_rank_sweep_and_fault():
    """C1 runs at N = 1 (ncclCommInitAll on one device): the code path the
    8-GPU node uses, every element checked, busbw factor 0; corrupt_allreduce
    makes the Job exit 1."""
    _have_bin()
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8")
    assert rc == 0 and _last_json(out)["rccl_allreduce"] == []     # auto: n > 1 only
    rc, out, err = _run("--size", "512", "--iters", "2", "--no-fp8", "--rccl",
                        "--allreduce-max-mib", "64")
    g = _last_json(out)
    assert rc == 0, (g["failures"], err[-2000:])
    rows = g["rccl_allreduce"]
    assert {r["dtype"] for r in rows} == {"bf16", "fp32"}
    assert rows[0]["bytes"] == 8 and max(r["bytes"] for r in rows) == 32 << 20
    assert all(r["wrong"] == 0 and r["busbw_GBps"] == 0 and r["algbw_GBps"] is None
               for r in rows)
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--rccl", "--allreduce-max-mib", "1",
                      env={"NTM_FAULT_INJECT": "corrupt_allreduce"})
    g = _last_json(out)
    assert rc == 1 and any("RCCL all-reduce" in f for f in g["failures"])


@pytest.mark.gpu
@pytest.mark.parametrize("nsim", [2, 8])
def test_binary_xgmi_simulated_ranks(nsim):
    """C2 through the binary's own run_xgmi driver with N simulated ranks on
    one GPU (--xgmi-sim): one-shot and two-shot sizes, device-side barriers,
    back-to-back epochs with no host sync; every element checked."""
    _have_bin()
    rc, out, err = _run("--size", "512", "--iters", "2", "--no-fp8", "--no-rccl",
                        "--xgmi-sim", str(nsim), "--allreduce-max-mib", "64")
    g = _last_json(out)
    assert rc == 0, (g["failures"], err[-2000:])
    rows = g["xgmi_allreduce_bf16"]
    assert g["xgmi_simulated_ranks"] == nsim and g["rccl_allreduce"] == []
    assert {r["dtype"] for r in rows} == {"bf16", "bf16-1shot"}
    assert all(r["wrong"] == 0 and r["time_us"] > 0 for r in rows)
    assert max(r["bytes"] for r in rows) >= 16 << 20


@pytest.mark.gpu
def test_binary_xgmi_simulated_fault_fails():
    _have_bin()
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--no-rccl", "--xgmi-sim", "4",
                      "--allreduce-max-mib", "4", env={"NTM_FAULT_INJECT": "corrupt_allreduce"})
    g = _last_json(out)
    assert rc == 1 and any("xGMI all-reduce" in f for f in g["failures"])


@pytest.mark.gpu
def test_binary_busbw_floors_fire():
    """the readiness gate gates the interconnect. An impossible
    floor fails the Job on both collectives (N = 1: RCCL busbw is 0 on a
    one-rank communicator; C2 on 4 simulated ranks); no floor, no failure."""
    _have_bin()
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--rccl", "--no-xgmi",
                      "--allreduce-max-mib", "1", "--rccl-busbw-floor-gbps", "1")
    g = _last_json(out)
    assert rc == 1 and any("RCCL all-reduce peak bf16 busbw" in f for f in g["failures"]), g
    assert g["rccl_peak_busbw_bf16_GBps"] == 0
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--no-rccl", "--xgmi-sim", "4",
                      "--allreduce-max-mib", "4", "--xgmi-busbw-floor-gbps", "1e9")
    g = _last_json(out)
    assert rc == 1 and any("xGMI all-reduce peak bf16 busbw" in f for f in g["failures"]), g
    assert g["xgmi_peak_busbw_bf16_GBps"] > 0
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--no-rccl", "--xgmi-sim", "4",
                      "--allreduce-max-mib", "4", "--xgmi-busbw-floor-gbps", "0.001")
    assert rc == 0, _last_json(out)["failures"]


@pytest.mark.gpu
@pytest.mark.parametrize("nblk,one_shot_max", [(16, 0), (32, 1 << 20), (128, 64 << 10)])
def test_binary_xgmi_knobs(nblk, one_shot_max):
    """--xgmi-nblk / --xgmi-one-shot-max (what bench.py sweeps at N > 1): every
    combination stays exact; 0 sends every size to the two-shot kernel."""
    _have_bin()
    rc, out, err = _run("--size", "512", "--iters", "2", "--no-fp8", "--no-rccl", "--xgmi-sim", "4",
                        "--allreduce-max-mib", "16", "--xgmi-nblk", str(nblk),
                        "--xgmi-one-shot-max", str(one_shot_max))
    g = _last_json(out)
    assert rc == 0, (g["failures"], err[-2000:])
    assert g["xgmi_nblk"] == nblk and g["xgmi_one_shot_max_bytes"] == one_shot_max
    rows = g["xgmi_allreduce_bf16"]
    assert all(r["wrong"] == 0 for r in rows)
    one = [r["bytes"] for r in rows if r["dtype"] == "bf16-1shot"]
    assert all(b <= one_shot_max for b in one) and (one_shot_max > 0) == bool(one)


@pytest.mark.gpu
@pytest.mark.parametrize("nsim", [2, 4])
def test_binary_xgmi_tune(nsim):
    """--xgmi-tune (what the Job passes at N > 1): a mini-sweep
    of blocks per rank x one-shot cutoff picks the configuration the main C2
    sweep then runs; every swept point and every main-sweep element exact, and
    the whole tune a small fraction of the Job's time."""
    _have_bin()
    rc, out, err = _run("--size", "512", "--iters", "2", "--no-fp8", "--no-rccl", "--xgmi-sim",
                        str(nsim), "--allreduce-max-mib", "128", "--xgmi-tune")
    g = _last_json(out)
    assert rc == 0, (g["failures"], err[-2000:])
    t = g["xgmi_tune"]
    assert t["ran"] is True and t["seconds"] < 10
    swept = {r["nblk"] for r in t["table"]}
    assert swept == {nb for nb in (32, 64, 128, 256) if nb * nsim <= 1024}
    assert {r["bytes"] for r in t["table"]} == {256 << 10, 1 << 20, 64 << 20}
    assert g["xgmi_nblk"] in swept and g["xgmi_one_shot_max_bytes"] in (0, 256 << 10, 1 << 20)
    # the chosen point is the fastest total over the three sizes
    def total(nb, cut):
        tt = {(r["bytes"], r["algo"]): r["time_us"] for r in t["table"] if r["nblk"] == nb}
        return sum(tt[(b, "1shot" if b <= cut else "2shot")] for b in (256 << 10, 1 << 20, 64 << 20))
    best = min(total(nb, c) for nb in swept for c in (0, 256 << 10, 1 << 20))
    assert total(g["xgmi_nblk"], g["xgmi_one_shot_max_bytes"]) == pytest.approx(best)
    rows = g["xgmi_allreduce_bf16"]
    assert rows and all(r["wrong"] == 0 for r in rows)
    one = [r["bytes"] for r in rows if r["dtype"] == "bf16-1shot"]
    assert all(b <= g["xgmi_one_shot_max_bytes"] for b in one)


@pytest.mark.gpu
def test_binary_reports_and_enforces_host_prep():
    """The in-pod host-prep check (--require-host-prep): the report always
    carries what the pod sees; the flag fails the Job exactly when a setting is
    missing (the GPU boxes are not prepared nodes, so either outcome is legal -
    the test pins that the verdict follows the observation)."""
    _have_bin()
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8")
    hp = _last_json(out)["host_prep"]
    assert set(hp) == {"numa_balancing", "memlock_unlimited", "iommu_pt"} and rc == 0
    prepared = hp["numa_balancing"] == 0 and hp["memlock_unlimited"]
    rc, out, _ = _run("--size", "512", "--iters", "2", "--no-fp8", "--require-host-prep")
    fails = [f for f in _last_json(out)["failures"] if f.startswith("host prep")]
    assert (rc == 0 and not fails) if prepared else (rc == 1 and fails)


def test_xgmi_knob_arguments_are_checked():
    _have_bin()
    rc, _, err = _run("--xgmi-nblk", "0", timeout=60)
    assert rc == 2 and "--xgmi-nblk" in err


@pytest.mark.gpu
def test_binary_no_fp8_skips_the_fp8_check():
    _have_bin()
    rc, out, _ = _run("--size", "1024", "--iters", "3", "--no-fp8")
    assert rc == 0
    g = _last_json(out)["gpus"][0]
    assert g["gemm_fp8_wrong"] is None and g["gemm_fp8_tflops"] == 0
    assert g["gemm_fp8_abft_bad_rows"] is None


# ------------------------------------------------ validation image runtime
COLLECT = ROOT / "validation" / "image" / "collect-runtime.sh"


@pytest.fixture(scope="module")
def closure(tmp_path_factory):
    _have_bin()
    dest = tmp_path_factory.mktemp("rt")
    subprocess.run(["bash", str(COLLECT), str(BIN), str(dest)], check=True, timeout=600,
                   capture_output=True)
    return dest


def _loaded_from(out_err: str) -> set:
    return {ln.split()[-1] for ln in out_err.splitlines() if "calling init:" in ln}


def _run_closure(closure, *args, timeout=300):
    env = dict(os.environ, LD_LIBRARY_PATH=str(closure / "lib"), LD_DEBUG="libs")
    env.pop("NTM_FAULT_INJECT", None)
    p = subprocess.run([str(closure / "bin" / "amdgpu-validate"), *args], capture_output=True,
                       text=True, timeout=timeout, env=env)
    return p.returncode, p.stdout, p.stderr


def test_runtime_closure_is_self_contained(closure):
    """What the runtime image ships is enough: no library of the ROCm SDK
    install is loaded when only the closure is on the search path."""
    names = {p.name for p in (closure / "lib").iterdir()}
    assert {"libamdhip64.so.7", "librccl.so.1", "libhsa-runtime64.so.1"} <= names
    assert not any(n.startswith(("libhipblaslt", "librocblas", "libMIOpen")) for n in names)
    rc, out, err = _run_closure(closure, "--size", "256", "--iters", "1", timeout=120)
    loaded = _loaded_from(err)
    assert loaded, err[-2000:]
    assert not [p for p in loaded if p.startswith("/opt/rocm")], loaded
    assert rc in (0, 2)   # 2 = no GPU in this container


def test_runtime_closure_rccl_is_cut_to_gfx950(closure):
    """collect-runtime.sh runs strip-fatbin.py: the closure's librccl carries a
    host + gfx950 bundle only (profiles/r5_fatbin)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "strip_fatbin", ROOT / "validation" / "image" / "strip-fatbin.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    lib = closure / "lib" / "librccl.so.1"
    off, size = m.section(str(lib))
    with open(lib, "rb") as f:
        f.seek(off)
        head = f.read(64)
    assert head[:4] == b"CCOB" and m.bundle_bytes(head) < size // 4
    res = m.strip(str(lib), "gfx950", "/opt/rocm/lib/llvm/bin/clang-offload-bundler", dry_run=True)
    assert res["targets"] == 2 and res["changed"] is False, res


@pytest.mark.gpu
def test_runtime_closure_runs_validation_on_gpu(closure):
    """The image's closure on MI355X, RCCL included: its librccl is cut to
    gfx950, and the all-reduce sweep still runs and verifies."""
    rc, out, err = _run_closure(closure, "--size", "1024", "--iters", "5", "--rccl",
                                "--allreduce-max-mib", "4", "--no-p2p")
    assert rc == 0, out + err[-3000:]
    rep = _last_json(out)
    assert rep["passed"]
    ar = rep.get("rccl_allreduce") or []
    assert ar and all(not r.get("wrong") for r in ar), ar
    assert not [p for p in _loaded_from(err) if p.startswith("/opt/rocm")]


# ------------------------------------------- host AddressSanitizer / UBSan
ASAN_BIN = ROOT / "validation" / "build" / "amdgpu-validate-asan"


def _run_asan(*args, leaks=True, timeout=300):
    if not ASAN_BIN.exists():
        pytest.skip("asan binary not built (python -m nvidia_terraform_modules_amd.ops.build --asan)")
    env = dict(os.environ, ASAN_OPTIONS=f"detect_leaks={1 if leaks else 0}:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("NTM_FAULT_INJECT", None)
    p = subprocess.run([str(ASAN_BIN), *args], capture_output=True, text=True, timeout=timeout,
                       env=env)
    return p.returncode, p.stdout, p.stderr


def test_asan_host_paths_clean_without_gpu():
    rc, out, err = _run_asan("--size", "256", "--termination-log", "/dev/null")
    assert "AddressSanitizer" not in err and "runtime error" not in err, err[-3000:]
    assert rc in (0, 2)
    rc, _, err = _run_asan("--gpus", "x", "--size")          # malformed arguments
    assert rc == 2 and "AddressSanitizer" not in err


@pytest.mark.gpu
def test_asan_full_validation_on_gpu(tmp_path):
    # the HIP runtime keeps allocations alive until exit: leak checking off
    rc, out, err = _run_asan("--size", "1024", "--iters", "5",
                             "--termination-log", str(tmp_path / "t"),
                             "--prom-out", str(tmp_path / "m"), leaks=False)
    assert "AddressSanitizer" not in err and "runtime error" not in err, err[-3000:]
    assert rc == 0, out + err[-2000:]
    assert _last_json(out)["passed"]


# ------------------------------------------------------------- Pushgateway
@pytest.mark.gpu
def test_pushgateway_push(tmp_path):
    """--pushgateway POSTs the Prometheus text to
    <url>/metrics/job/amdgpu_validate/instance/<host>; the JSON reports it."""
    import http.server
    import threading

    got = {}

    class H(http.server.BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            n = int(self.headers["Content-Length"])
            got["path"] = self.path
            got["body"] = self.rfile.read(n).decode()
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = http.server.HTTPServer(("127.0.0.1", 0), H)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}/gw"
        _have_bin()
        rc, out, err = _run("--size", "1024", "--iters", "3", "--pushgateway", url)
    finally:
        srv.shutdown()
    assert rc == 0, out + err
    rep = _last_json(out)
    assert rep["pushgateway"] == "ok"
    assert got["path"].startswith("/gw/metrics/job/amdgpu_validate/instance/")
    assert "amdgpu_validate_passed 1" in got["body"]
    assert 'amdgpu_validate_gemm_tflops{gpu="0"}' in got["body"]


@pytest.mark.gpu
def test_pushgateway_unreachable_is_not_fatal():
    _have_bin()
    with socket.socket() as s:        # a port nobody listens on
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    rc, out, _ = _run("--size", "512", "--iters", "2", "--pushgateway", f"http://127.0.0.1:{port}")
    rep = _last_json(out)
    assert rc == 0 and rep["passed"] is True
    assert rep["pushgateway"].startswith("error")


def test_help_exits_zero_without_touching_the_gpu():
    """The pre-pull DaemonSet's init container (modules/amd-gpu-stack/validation.tf)
    runs `amdgpu-validate --help` on nodes whose driver may not be loaded yet:
    it must link, print usage and exit 0 without any HIP call."""
    _have_bin()
    rc, out, err = _run("--help", timeout=60)
    assert rc == 0 and "usage" in err


def test_cpp_and_python_collective_sweeps_agree():
    """the Job binary's C1/C2 sweeps (C++) and the torch
    sweeps bench.py runs (parallel/collectives.py) must not drift: same sizes,
    same nccl-tests busbw factor (host-only --describe-sweep, no GPU)."""
    _have_bin()
    import sys
    sys.path.insert(0, str(ROOT))
    from nvidia_terraform_modules_amd.parallel import collectives as coll

    for mib in (1, 64, 8192):
        rc, out, err = _run("--describe-sweep", "--allreduce-max-mib", str(mib), timeout=60)
        assert rc == 0, err
        d = json.loads(out)
        assert d["rccl_bytes"] == coll.sweep_sizes(8, mib << 20, 4)
        assert d["bus_factor"] == pytest.approx([coll.bus_factor("all_reduce", n)
                                                 for n in range(1, 9)])
        for n in range(1, 9):
            # bench.py's C2 list (paired with its RCCL rows): same rule, same cap
            py = [b for b in coll.sweep_sizes(8, mib << 20, 4)
                  if 512 <= b <= 1 << 30 and (b // 2) % (8 * n) == 0]
            assert d["xgmi_bytes"][str(n)] == py
