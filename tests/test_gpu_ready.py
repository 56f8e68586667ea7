"""Time-to-GPU-ready instrumentation: phase clock, apply-log timeline and the
plan-graph critical-path model (all CPU)."""
import json
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.gpu_ready.apply_timeline import (
    build_timeline, gpu_allocatable_time, parse_apply_json, parse_ts)
from nvidia_terraform_modules_amd.gpu_ready.critical_path import critical_path, phase_of
from nvidia_terraform_modules_amd.gpu_ready.phases import CLUSTER_PHASES, PhaseClock, process_start_time
from nvidia_terraform_modules_amd.tfcheck.graph import build_graph


def _ev(typ, addr, ts, action="create", elapsed=None):
    hook = {"resource": {"addr": addr}, "action": action}
    if elapsed is not None:
        hook["elapsed_seconds"] = elapsed
    return json.dumps({"@level": "info", "@timestamp": ts, "type": typ, "hook": hook})


SYNTH_APPLY = [
    '{"@level":"info","@message":"Terraform 1.9.5","type":"version"}',
    _ev("apply_start", "module.vpc.aws_vpc.this[0]", "2025-01-17T10:00:00.000000+00:00"),
    _ev("apply_complete", "module.vpc.aws_vpc.this[0]", "2025-01-17T10:02:30.123456+00:00", elapsed=150),
    _ev("apply_start", "module.eks.aws_eks_cluster.this[0]", "2025-01-17T10:02:31Z"),
    _ev("apply_complete", "module.eks.aws_eks_cluster.this[0]", "2025-01-17T10:15:31Z", elapsed=780),
    _ev("apply_start", "module.amd_gpu_stack.helm_release.amd_gpu_operator[0]", "2025-01-17T10:15:40Z"),
    _ev("apply_complete", "module.amd_gpu_stack.helm_release.amd_gpu_operator[0]", "2025-01-17T10:17:40Z", elapsed=120),
    _ev("apply_start", "module.amd_gpu_stack.helm_release.device_config[0]", "2025-01-17T10:17:41Z"),
    _ev("apply_complete", "module.amd_gpu_stack.helm_release.device_config[0]", "2025-01-17T10:17:50Z", elapsed=9),
    _ev("apply_start", "module.amd_gpu_stack.kubernetes_job_v1.gpu_validation[0]", "2025-01-17T10:17:51Z"),
    _ev("apply_complete", "module.amd_gpu_stack.kubernetes_job_v1.gpu_validation[0]", "2025-01-17T10:22:51Z", elapsed=300),
]


def test_parse_ts_variants():
    a = parse_ts("2025-01-17T10:00:00Z")
    b = parse_ts("2025-01-17T10:00:00.000000+00:00")
    c = parse_ts("2025-01-17T10:00:00.123456789+00:00")  # nanoseconds truncated
    assert a == b and 0.12 < c - a < 0.124


def test_parse_apply_json_pairs_start_and_complete():
    res = parse_apply_json(SYNTH_APPLY)
    by = {r["address"]: r for r in res}
    assert by["module.eks.aws_eks_cluster.this[0]"]["elapsed_s"] == 780
    assert all(r["start"] is not None and r["end"] is not None for r in res)
    assert not any(r["errored"] for r in res)


def test_timeline_phases_and_total():
    tl = build_timeline(SYNTH_APPLY)
    d = tl.phase_durations()
    assert list(d) == [p for p in CLUSTER_PHASES if p in d]
    assert tl.time_to_gpu_ready_s == pytest.approx(22 * 60 + 51, abs=1)
    assert d["validation_done"] == pytest.approx(301, abs=1)


def test_k8s_events_override_allocatable():
    events = {"items": [
        {"reason": "Scheduled", "lastTimestamp": "2025-01-17T10:18:00Z", "message": "no gpu here"},
        {"reason": "NodeAllocatable", "lastTimestamp": "2025-01-17T10:19:30Z",
         "message": "Updated Node Allocatable limit across pods", "note": "amd.com/gpu: 8"},
    ]}
    assert gpu_allocatable_time(events) == parse_ts("2025-01-17T10:19:30Z")
    tl = build_timeline(SYNTH_APPLY, k8s_events=events)
    assert tl.phases["gpu_allocatable"] == parse_ts("2025-01-17T10:19:30Z")


def test_errored_resource_is_flagged():
    lines = SYNTH_APPLY[:3] + [_ev("apply_start", "google_container_cluster.this", "2025-01-17T10:03:00Z"),
                               _ev("apply_errored", "google_container_cluster.this", "2025-01-17T10:04:00Z")]
    res = {r["address"]: r for r in parse_apply_json(lines)}
    assert res["google_container_cluster.this"]["errored"]


def test_phase_clock_monotone():
    c = PhaseClock(origin=100.0)
    c.mark("a", 101.0)
    c.mark("b", 100.5)   # clock step backwards -> clamped
    c.mark("c", 103.0)
    d = c.durations()
    assert d["a"] == 1.0 and d["b"] == 0.0 and d["c"] == 2.0
    assert c.as_dict()["total_s"] == 3.0
    assert process_start_time() <= __import__("time").time()


def test_phase_of_mapping():
    assert phase_of("module.vpc") == "network"
    assert phase_of("google_container_node_pool.gpu_nodes") == "gpu_nodes_ready"
    assert phase_of("module.amd_gpu_stack.kubernetes_job_v1.gpu_validation") == "validation_done"


@pytest.mark.parametrize("root,mode", [("eks", "operator"), ("gke", "daemonsets"), ("aks", "operator")])
def test_critical_path_ends_with_validation(repo, root, mode):
    cp = critical_path(build_graph(repo / root), stack_mode=mode)
    assert cp.path[-1][0].endswith("kubernetes_job_v1.gpu_validation")
    assert cp.total_s > 0 and abs(sum(s for _, s in cp.path) - cp.total_s) < 1e-6
    assert "validation_done" in cp.phases


def test_critical_path_uses_measured_durations(repo):
    g = build_graph(repo / "aks")
    base = critical_path(g).total_s
    faster = critical_path(g, {"azurerm_kubernetes_cluster_node_pool.mi355x": 60.0}).total_s
    assert faster < base


def test_validation_image_prepull_is_off_the_path_and_hides_the_pull(repo, monkeypatch):
    import nvidia_terraform_modules_amd.gpu_ready.critical_path as cpm

    g = build_graph(repo / "eks")
    pre = [n for n in g.topo_order() if cpm.PREPULL_MARK in n]
    assert pre, "modules/amd-gpu-stack should pre-pull the validation image"
    # it does not wait for the operator / driver stack, and nothing waits for it
    assert not any("helm_release" in d or "daemon_set" in d for d in g.deps(pre[0]))
    assert not any(pre[0] in g.deps(n) for n in g.topo_order())
    job = lambda cp: dict(cp.path)[cp.path[-1][0]]  # noqa: E731
    with_pull = critical_path(g)
    monkeypatch.setattr(cpm, "PREPULL_MARK", "no-such-resource")
    without = critical_path(g)
    assert job(without) - job(with_pull) == pytest.approx(cpm.IMAGE_PULL_S)
    assert with_pull.total_s < without.total_s


# --------------------------------------------------------------- CLI record
TF_STUB = r'''#!/usr/bin/env python3
import json, sys, time
from datetime import datetime, timezone
def ts(): return datetime.now(timezone.utc).isoformat()
def emit(typ, addr, action="create", **kw):
    hook = {"resource": {"addr": addr}, "action": action, **kw}
    print(json.dumps({"@timestamp": ts(), "type": typ, "hook": hook}), flush=True)
print(json.dumps({"@timestamp": ts(), "type": "version", "terraform": "1.9.0"}), flush=True)
for addr in ["module.vpc.aws_vpc.this[0]", "module.eks.aws_eks_cluster.this[0]",
             "module.amd_gpu_stack.helm_release.amd_gpu_operator[0]",
             "module.amd_gpu_stack.kubernetes_job_v1.gpu_validation[0]"]:
    emit("apply_start", addr)
    time.sleep(0.3)
    emit("apply_complete", addr, elapsed_seconds=0.3)
'''

KUBECTL_STUB = r'''#!/usr/bin/env python3
import json, sys, os
state = os.environ["STUB_STATE"]
n = int(open(state).read()) if os.path.exists(state) else 0
open(state, "w").write(str(n + 1))
args = sys.argv[1:]
if n < 2:
    sys.exit(1)                       # cluster not there yet
if "nodes" in args:
    # every GPU node (STUB_PODS of them) reports its GPUs
    print(json.dumps({"items": [{"metadata": {"name": f"gpu-node-{i}"},
                                 "status": {"allocatable": {"amd.com/gpu": "8"}}}
                                for i in range(int(os.environ.get("STUB_PODS", "1")))]}))
elif "pods" in args:
    # one validation pod per GPU node (STUB_PODS), finishing a second apart
    items = []
    for i in range(int(os.environ.get("STUB_PODS", "1"))):
        msg = json.dumps({"passed": True, "n_gpus": 8, "gemm_tflops_aggregate": 12345.0 + i})
        items.append({"metadata": {"name": f"amd-gpu-validation-{i}"},
                      "spec": {"nodeName": f"gpu-node-{i}"},
                      "status": {"containerStatuses": [{"state": {"terminated": {
                          "exitCode": 0, "message": msg,
                          "finishedAt": f"2030-01-01T00:00:0{i}Z"}}}]}})
    print(json.dumps({"items": items}))
else:
    sys.exit(1)
'''


def _stub(path, body):
    path.write_text(body)
    path.chmod(0o755)


def test_cli_record_with_stub_terraform_and_kubectl(tmp_path):
    import os
    import subprocess
    import sys

    bindir = tmp_path / "bin"
    bindir.mkdir()
    _stub(bindir / "terraform", TF_STUB)
    _stub(bindir / "kubectl", KUBECTL_STUB)
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}",
               STUB_STATE=str(tmp_path / "kstate"))
    out = tmp_path / "run"
    p = subprocess.run([sys.executable, "-m", "nvidia_terraform_modules_amd.gpu_ready", "record",
                        "--out", str(out), "--kubectl", "kubectl", "--poll", "0.2", "--",
                        "terraform", "apply", "-json", "-auto-approve"],
                       capture_output=True, text=True, env=env, timeout=120,
                       cwd=Path(__file__).resolve().parents[1])
    assert p.returncode == 0, p.stderr
    assert "time_to_gpu_ready_s" in p.stdout
    ev = json.loads((out / "k8s_events.json").read_text())["items"]
    assert ev and "amd.com/gpu allocatable 8" in ev[0]["message"]
    rep = json.loads((out / "validation.json").read_text())
    assert rep["passed"] and rep["end_epoch_s"] > 1.8e9          # finishedAt 2030
    tl = json.loads((out / "timeline.json").read_text())
    assert tl["phase_end"]["gpu_allocatable"] <= tl["phase_end"]["validation_done"]
    assert tl["time_to_gpu_ready_s"] > 0
    # the saved log replays through the `timeline` subcommand
    p2 = subprocess.run([sys.executable, "-m", "nvidia_terraform_modules_amd.gpu_ready", "timeline",
                         str(out / "apply.jsonl"), "--json"], capture_output=True, text=True,
                        timeout=60, cwd=Path(__file__).resolve().parents[1])
    assert p2.returncode == 0 and json.loads(p2.stdout)["resources"]


def test_cli_record_waits_for_every_node_pod(tmp_path):
    """With one validation pod per GPU node, validation_done is the LAST pod's
    finish and the report lists every node's verdict."""
    import os
    import subprocess
    import sys

    bindir = tmp_path / "bin"
    bindir.mkdir()
    _stub(bindir / "terraform", TF_STUB)
    _stub(bindir / "kubectl", KUBECTL_STUB)
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}",
               STUB_STATE=str(tmp_path / "kstate"), STUB_PODS="3")
    out = tmp_path / "run"
    p = subprocess.run([sys.executable, "-m", "nvidia_terraform_modules_amd.gpu_ready", "record",
                        "--out", str(out), "--kubectl", "kubectl", "--poll", "0.2",
                        "--validation-pods", "3", "--",
                        "terraform", "apply", "-json", "-auto-approve"],
                       capture_output=True, text=True, env=env, timeout=120,
                       cwd=Path(__file__).resolve().parents[1])
    assert p.returncode == 0, p.stderr
    ev = json.loads((out / "k8s_events.json").read_text())["items"]
    assert sorted(e["involvedObject"]["name"] for e in ev) == ["gpu-node-0", "gpu-node-1",
                                                             "gpu-node-2"]
    rep = json.loads((out / "validation.json").read_text())
    assert rep["nodes_validated"] == rep["nodes_expected"] == 3
    assert [n["node"] for n in rep["per_node"]] == ["gpu-node-0", "gpu-node-1", "gpu-node-2"]
    assert all(n["passed"] for n in rep["per_node"])
    assert rep["end_epoch_s"] == max(n["end_epoch_s"] for n in rep["per_node"])
    assert rep["gemm_tflops_aggregate"] == 12347.0          # the last pod's verdict
    assert not any(k.startswith("_") for k in rep)


def test_watcher_reports_partial_coverage_when_apply_returns_first():
    from nvidia_terraform_modules_amd.gpu_ready.__main__ import ClusterWatcher

    w = ClusterWatcher(["false"], "ns", 0.1, expected_pods=2)
    w.reports["p0"] = {"passed": True, "end_epoch_s": 5.0, "_node": "n0"}
    w.poll_once()                      # kubectl fails: nothing new, still waiting for p1
    assert w.report is None
    w.finish()
    assert w.report["nodes_validated"] == 1 and w.report["nodes_expected"] == 2


def test_cli_critical_path_json(tmp_path):
    import subprocess
    import sys

    root = Path(__file__).resolve().parents[1]
    p = subprocess.run([sys.executable, "-m", "nvidia_terraform_modules_amd.gpu_ready",
                        "critical-path", str(root / "gke"), "--json"], capture_output=True,
                       text=True, timeout=60, cwd=root)
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout)
    assert d["total_s"] > 0 and d["path"][-1][0].endswith("kubernetes_job_v1.gpu_validation")


def test_named_priors_beat_type_priors(repo):
    """A CR-only chart (the DeviceConfig) has nothing for helm's wait to wait on:
    its type.name prior (5 s) applies instead of the operator-chart prior."""
    # a fast GPU pool puts the stack branch on the critical path
    fast = {"module.gpu_node_pool": 10.0}
    cp = critical_path(build_graph(repo / "eks"), fast)
    path = dict(cp.path)
    assert path["module.amd_gpu_stack.helm_release.device_config"] == 5.0
    assert path["module.amd_gpu_stack.helm_release.amd_gpu_operator"] == 120.0
    over = critical_path(build_graph(repo / "eks"), {**fast, "helm_release.device_config": 50.0})
    assert dict(over.path)["module.amd_gpu_stack.helm_release.device_config"] == 50.0
