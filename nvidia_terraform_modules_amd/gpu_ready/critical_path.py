"""Offline time-to-GPU-ready model: critical path through the plan graph.

Terraform applies independent nodes in parallel (default -parallelism=10),
so apply wall time ~= the longest dependency chain weighted by each node's
create time. This module weights the graph from
:mod:`nvidia_terraform_modules_amd.tfcheck.graph` with per-resource-type
durations and returns the critical path and its length, split into the six
BASELINE phases.

The durations are PRIORS (documented cloud-API behaviour, [ext]) and are
meant to be replaced by measured ones: :func:`durations_from_timeline`
derives them from a ``terraform apply -json`` log (see
:mod:`.apply_timeline`), and the in-node validation phase is measured on real
MI355X hardware by ``bench.py`` / the validation binary.

Reference anchor: the only number the reference publishes is the ~5 min from
"apply returned" to "GPU operator Running" (/root/reference/gke/README.md:50),
i.e. work that happens OFF its critical path after apply; here that work is
ON the path (apply waits for the validation Job), so the comparable figure is
operator_deployed -> validation_done.
"""
from __future__ import annotations

from dataclasses import dataclass

from ..tfcheck.graph import Graph

# seconds; priors by resource type / module source (EKS/GKE/AKS docs [ext])
DEFAULT_DURATIONS = {
    # network
    "module.vpc": 150.0,                     # VPC + subnets + NAT gateways
    "google_compute_network": 25.0,
    "google_compute_subnetwork": 20.0,
    "azurerm_resource_group": 5.0,
    # control plane
    "module.eks": 600.0,                     # cluster ACTIVE (~10 min), no node groups
    "module.cpu_node_pool": 180.0,           # system nodes boot + join
    # MI355X nodes boot + join + Ready, incl. the one-time iommu=pt reboot
    # before the join (eks gpu_node_iommu_passthrough = "reboot", ~90 s)
    "module.gpu_node_pool": 390.0,
    "aws_eks_addon": 60.0,
    "google_container_cluster": 420.0,
    "azurerm_kubernetes_cluster": 360.0,
    # node pools (GPU nodes boot + join + Ready)
    "google_container_node_pool": 300.0,
    "azurerm_kubernetes_cluster_node_pool": 420.0,
    # IAM / add-ons
    "module.ebs_csi_irsa_role": 15.0,
    "terraform_data": 0.0,
    # GPU software stack
    "kubernetes_namespace_v1": 2.0,
    "kubernetes_resource_quota_v1": 1.0,
    "helm_release": 120.0,                   # operator chart wait=true
    # CR-only / monitor-only charts: helm's wait has no workload to wait for
    "helm_release.device_config": 5.0,
    "helm_release.service_monitor": 5.0,
    "helm_release.crd_janitor": 3.0,         # hooks run at destroy only: nothing to wait for
    "kubernetes_daemon_set_v1": 30.0,
    "kubernetes_service_v1": 1.0,
    "kubernetes_service_account_v1": 1.0,
    "kubernetes_cluster_role_v1": 1.0,
    "kubernetes_cluster_role_binding_v1": 1.0,
}

# The validation image's pull, from its measured size: the runtime closure
# (validation/image/collect-runtime.sh, librccl cut to gfx950 by
# strip-fatbin.py) is 150.2 MB gzip'd (profiles/r5_fatbin; 648.7 MB with the
# vendor's 13-target RCCL), plus the ubuntu:24.04 base layer (~29 MB [ext]),
# at a per-node registry pull + extract rate (ECR / Artifact Registry / ACR,
# one image on a fresh node [ext]) after a fixed manifest / auth / layer set-up.
IMAGE_BYTES = 150.2e6 + 29e6
PULL_BYTES_PER_S = 40e6
IMAGE_PULL_S = 5.0 + IMAGE_BYTES / PULL_BYTES_PER_S
# the rest of the Job: pod scheduling, container start and the run itself. The
# process's own start -> verdict is measured on MI355X (0.44 s at 1 GPU,
# ~2.4 s with the RCCL sweep: BENCH_r04, profiles/r5_fatbin); the rest [ext].
JOB_RUN_S = 30.0
# validation Job: pod schedule + image pull + run. The pull is hidden behind the
# driver install when the pre-pull DaemonSet (modules/amd-gpu-stack/validation.tf)
# is in the graph, since it pulls on each GPU node as the node joins.
DEFAULT_DURATIONS["kubernetes_job_v1"] = JOB_RUN_S + IMAGE_PULL_S
PREPULL_MARK = "kubernetes_daemon_set_v1.validation_prepull"

# extra readiness that happens INSIDE nodes after their Terraform resource
# completed: driver install (DKMS build or operator KMM), device plugin
# registration. Attributed to the node that waits on it.
DRIVER_READY_S = {"operator": 240.0, "daemonsets": 300.0}
# gpu_driver_preinstalled (node image ships amdgpu; module driver_enabled =
# false): no KMM build / DKMS compile, only the device plugin registering
# amd.com/gpu with the kubelet and the labeller - the SURVEY §7.4 lever
PLUGIN_READY_S = 30.0
# the host-prep gate (node-prep DaemonSet with the startup taint): prep script,
# the queued containerd restart (done before kubelet can start the next
# container), the gate container's image pull, its first verify + untaint
# (a failed verify waits node_prep_gate_interval_s, 30 s, for the next check).
# It runs beside the driver install, so the Job waits for the LONGER of the
# two: off the path with a driver to install, on it with a preinstalled driver.
PREP_GATE_S = 45.0
PREP_GATE_MARK = "kubernetes_cluster_role_v1.node_prep"

PHASE_OF_KIND = [
    ("network", ("module.vpc", "google_compute_network", "google_compute_subnetwork",
                 "azurerm_resource_group")),
    ("control_plane", ("google_container_cluster", "azurerm_kubernetes_cluster.",
                       "module.ebs_csi_irsa_role", "module.eks", "module.cpu_node_pool",
                       "aws_eks_addon", "google_container_node_pool.system")),
    ("gpu_nodes_ready", ("module.gpu_node_pool", "google_container_node_pool",
                         "azurerm_kubernetes_cluster_node_pool")),
    ("operator_deployed", ("helm_release.amd_gpu_operator", "helm_release.device_config",
                           "kubernetes_namespace_v1", "kubernetes_resource_quota_v1")),
    ("gpu_allocatable", ("kubernetes_daemon_set_v1", "kubernetes_service", "kubernetes_cluster_role",
                         "helm_release.service_monitor")),
    ("validation_done", ("kubernetes_job_v1",)),
]


def node_type(addr: str) -> str:
    """Resource type (or module key) of a flattened graph address."""
    parts = addr.split(".")
    # strip leading module.X. prefixes of LOCAL modules
    while len(parts) > 2 and parts[0] == "module" and parts[2] in ("module",) + tuple(
            k for k in DEFAULT_DURATIONS if "." not in k):
        parts = parts[2:]
    while len(parts) > 3 and parts[0] == "module":
        parts = parts[2:]
    if parts[0] == "module":
        return ".".join(parts[:2])
    if parts[0] == "data":
        return "data." + parts[1]
    if parts[0] == "provider":
        return "provider"
    return parts[0]


def phase_of(addr: str) -> str:
    for phase, keys in PHASE_OF_KIND:
        for k in keys:
            if k in addr:
                return phase
    return "other"


@dataclass
class CriticalPath:
    total_s: float
    path: list           # [(address, duration_s)] in execution order
    phases: dict         # phase -> seconds on the critical path

    def as_dict(self) -> dict:
        return {"total_s": self.total_s, "path": self.path, "phases": self.phases}


def critical_path(g: Graph, durations: dict | None = None, stack_mode: str = "operator",
                  driver_preinstalled: bool = False) -> CriticalPath:
    """``driver_preinstalled``: the root's gpu_driver_preinstalled = true (the
    driver-install phase drops to device-plugin registration)."""
    dur = dict(DEFAULT_DURATIONS)
    dur.update(durations or {})

    prepull = any(PREPULL_MARK in n for n in g.topo_order())
    gated = any(PREP_GATE_MARK in n for n in g.topo_order())

    def d(addr: str) -> float:
        if addr in dur:
            return dur[addr]
        t = node_type(addr)
        named = f"{t}.{addr.split(t + '.', 1)[1].split('[')[0]}" if (t + ".") in addr else t
        base = dur.get(named, dur.get(t, 0.0))
        if t == "kubernetes_job_v1":
            # GPUs allocatable only after the driver (or just the plugin, preinstalled)
            driver = PLUGIN_READY_S if driver_preinstalled else DRIVER_READY_S.get(stack_mode, 0.0)
            pull = dur.get("image_pull", IMAGE_PULL_S)
            if prepull:  # pulled while the driver installed: only the excess remains
                base -= min(pull, driver)
            # the Job schedules once GPUs are allocatable AND the prep gate lifted
            base += max(driver, dur.get("prep_gate", PREP_GATE_S)) if gated else driver
        return base

    finish: dict = {}
    parent: dict = {}
    for n in g.topo_order():
        start, best = 0.0, None
        for dep in g.deps(n):
            f = finish.get(dep, 0.0)
            if f > start:
                start, best = f, dep
        finish[n] = start + d(n)
        parent[n] = best
    if not finish:
        return CriticalPath(0.0, [], {})
    end = max(finish, key=lambda k: finish[k])
    chain = []
    cur = end
    while cur is not None:
        chain.append((cur, d(cur)))
        cur = parent[cur]
    chain.reverse()
    phases: dict = {}
    for addr, s in chain:
        ph = phase_of(addr)
        phases[ph] = phases.get(ph, 0.0) + s
    return CriticalPath(finish[end], chain, phases)


def durations_from_timeline(events: list[dict]) -> dict:
    """{address: seconds} from apply_timeline.parse_apply_json() events."""
    out = {}
    for ev in events:
        if ev.get("elapsed_s") is not None:
            out[ev["address"]] = float(ev["elapsed_s"])
    return out
