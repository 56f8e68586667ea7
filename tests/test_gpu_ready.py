"""Time-to-GPU-ready instrumentation: phase clock, apply-log timeline and the
plan-graph critical-path model (all CPU)."""
import json

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
    lines = SYNTH_APPLY[:3] + [_ev("apply_start", "google_container_cluster.holoscan", "2025-01-17T10:03:00Z"),
                               _ev("apply_errored", "google_container_cluster.holoscan", "2025-01-17T10:04:00Z")]
    res = {r["address"]: r for r in parse_apply_json(lines)}
    assert res["google_container_cluster.holoscan"]["errored"]


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
    faster = critical_path(g, {"azurerm_kubernetes_cluster_node_pool.holoscan": 60.0}).total_s
    assert faster < base
