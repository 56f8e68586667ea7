"""Round-3 module features, offline (tfcheck plan + evaluator):

* MI355X host prep on every cloud: the node-prep DaemonSet in
  modules/amd-gpu-stack, the validation Job's in-pod check of it, and the EKS
  user data's bounded iommu=pt reboot;
* the preinstalled-driver fast path (reference
  /root/reference/aks/main.tf:89-91 ``driver.enabled=false``);
* the interconnect floors of the validation Job.
"""
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.gpu_ready.critical_path import (DRIVER_READY_S, PLUGIN_READY_S,
                                                                  critical_path)
from nvidia_terraform_modules_amd.tfcheck.analysis import analyze
from nvidia_terraform_modules_amd.tfcheck.config import load_module
from nvidia_terraform_modules_amd.tfcheck.docs import render
from nvidia_terraform_modules_amd.tfcheck.graph import build_graph
from nvidia_terraform_modules_amd.tfcheck.plan import plan

ROOT = Path(__file__).resolve().parents[1]
STACK = "module.amd_gpu_stack."
BASE_VARS = {
    "eks": ["cluster_name=c", "gpu_instance_type=x.48xlarge"],
    "gke": ["project_id=p", "region=us-central1", "cluster_name=c", "gpu_instance_type=m"],
    "aks": ["location=westus3", "gpu_machine_type=Standard_ND_MI355X"],
}
IMAGE = ["gpu_validation_image=registry.example/amdgpu-validate:1"]


def _vars(root, *extra):
    v = BASE_VARS[root] + IMAGE + list(extra)
    return v


def _plan(root, tmp_path, *extra, daemonsets=False):
    vf = None
    lines = []
    if root == "gke":
        lines.append('node_zones = ["us-central1-a"]')
    if root == "aks":
        lines.append("admin_group_object_ids = []")
    if daemonsets:
        lines.append('gpu_stack_mode = "daemonsets"')
    if lines:
        vf = tmp_path / f"{root}.tfvars"
        vf.write_text("\n".join(lines) + "\n")
    return plan(ROOT / root, cli_vars=_vars(root, *extra), var_files=[vf] if vf else [])


def _stack_local(name, **overrides):
    """Evaluate local.<name> of modules/amd-gpu-stack with defaults + overrides."""
    from nvidia_terraform_modules_amd.tfcheck.evaluate import Evaluator, Scope, convert

    mod = load_module(ROOT / "modules" / "amd-gpu-stack")
    ev = Evaluator()
    variables = {}
    for vn, v in mod.variables.items():
        if vn in overrides:
            variables[vn] = overrides[vn]
        elif not v.required:
            variables[vn] = convert(ev.eval(v.block.body.attr("default"), Scope({}, {})),
                                    v.type_expr)
    scope = Scope(variables, {n: e for n, (e, _, _) in mod.locals.items()}, str(mod.path))
    return ev.eval(mod.locals[name][0], scope)


# ------------------------------------------------------------------ host prep
@pytest.mark.parametrize("root", ["eks", "gke", "aks"])
def test_every_cloud_gets_the_mi355x_host_prep(root, tmp_path):
    r = _plan(root, tmp_path)
    assert r.ok, r.errors
    assert STACK + "kubernetes_daemon_set_v1.node_prep[0]" in r.resources
    # the Job depends on the prep and re-checks it from inside its pod
    stack = load_module(ROOT / "modules" / "amd-gpu-stack")
    job = stack.resources["kubernetes_job_v1.gpu_validation"].block
    assert "kubernetes_daemon_set_v1.node_prep" in render(job.body.attr("depends_on"))
    assert "--require-host-prep" in _stack_local("validation_args")


def test_node_prep_script_covers_the_three_settings_and_reboots_at_most_once():
    m = load_module(ROOT / "modules" / "amd-gpu-stack")
    s = "".join(p for p in m.locals["node_prep_script"][0].parts if isinstance(p, str))
    assert "kernel.numa_balancing = 0" in s and "/proc/sys/kernel/numa_balancing" in s
    assert "containerd.service.d" in s and "LimitMEMLOCK=infinity" in s
    assert "systemctl --no-block restart containerd" in s
    assert "iommu=pt" in s and "/proc/cmdline" in s
    # bounded reboot: sentinel written before the reboot, a second miss proceeds
    assert s.index("touch \"$sentinel\"") < s.index("systemctl --no-block reboot")
    assert "absent-after-reboot" in s
    v = m.variables["node_prep_iommu_mode"]
    assert v.default == "check" and v.validations


def test_node_prep_daemonset_tolerates_the_gpu_taint():
    """tfcheck's gpu-toleration rule covers every GPU-node workload, this one too."""
    findings = analyze(load_module(ROOT / "modules" / "amd-gpu-stack"))
    assert not [f for f in findings if f.rule == "gpu-toleration"], findings


@pytest.mark.parametrize("root,mode,require_iommu", [
    ("gke", "reboot", True), ("gke", "check", False), ("aks", "off", False)])
def test_gke_aks_iommu_mode_reaches_the_stack(root, mode, require_iommu):
    m = load_module(ROOT / root)
    body = m.modules["amd_gpu_stack"].block.body
    assert "var.gpu_node_iommu_passthrough" in render(body.attr("node_prep_iommu_mode"))
    assert m.variables["gpu_node_iommu_passthrough"].default == "check"
    on = _stack_local("validation_args", validation_require_iommu_pt=require_iommu)
    assert ("--require-iommu-pt" in on) == require_iommu


def test_eks_iommu_reboot_is_bounded():
    """a node whose iommu=pt does not stick must not reboot forever,
    and a failing grub edit must not abort the bootstrap under set -e."""
    m = load_module(ROOT / "eks")
    prep = "".join(p for p in m.locals["mi355x_host_prep"][0].parts if isinstance(p, str))
    assert "/var/lib/mi355x-iommu-rebooted" in prep
    assert prep.index('touch "$sentinel"') < prep.index("systemctl reboot")
    assert "reboot-failed" in prep and "update-grub || " in prep
    assert "iommu=pt still absent after one reboot" in prep


def test_eks_has_no_cross_package_moves_and_documents_the_state_mv():
    """moves out of the registry module "eks" fail every plan.
    The rule runs on the real root; the upgrade path is `terraform state mv`."""
    from nvidia_terraform_modules_amd.tfcheck.analysis import moved_findings

    assert moved_findings(load_module(ROOT / "eks")) == []
    readme = (ROOT / "eks" / "README.md").read_text()
    for frm, to in (('module.eks.module.eks_managed_node_group["gpu_node_pool"]', "module.gpu_node_pool"),
                    ('module.eks.module.eks_managed_node_group["cpu_node_pool"]', "module.cpu_node_pool"),
                    ('module.eks.aws_eks_addon.this["aws-ebs-csi-driver"]', "aws_eks_addon.ebs_csi")):
        assert f"terraform state mv '{frm}' '{to}'" in readme


# ------------------------------------------------------- preinstalled driver
@pytest.mark.parametrize("root", ["eks", "gke", "aks"])
def test_preinstalled_driver_skips_the_install(root, tmp_path):
    extra = ["gpu_driver_preinstalled=true"] + (["gpu_ami_id=ami-0123"] if root == "eks" else [])
    ds = _plan(root, tmp_path, *extra, daemonsets=True)
    assert ds.ok, ds.errors
    assert STACK + "kubernetes_daemon_set_v1.rocm_device_plugin[0]" in ds.resources
    assert STACK + "kubernetes_daemon_set_v1.amdgpu_dkms[0]" not in ds.resources
    full = _plan(root, tmp_path, daemonsets=True)
    assert STACK + "kubernetes_daemon_set_v1.amdgpu_dkms[0]" in full.resources
    body = load_module(ROOT / root).modules["amd_gpu_stack"].block.body
    assert "!var.gpu_driver_preinstalled" in render(body.attr("driver_enabled"))
    # operator mode: no KMM, DeviceConfig driver disabled
    vals = _stack_local("operator_values", driver_enabled=False, cluster_name="c")
    assert vals["kmm"]["enabled"] is False
    dc = _stack_local("device_config_values", driver_enabled=False, cluster_name="c")
    assert dc["spec"]["driver"]["enable"] is False


def test_eks_preinstalled_driver_requires_a_pinned_ami(tmp_path):
    r = _plan("eks", tmp_path, "gpu_driver_preinstalled=true")
    assert any("driver_preinstalled_guard" in e for e in r.errors), r.errors


@pytest.mark.parametrize("root", ["eks", "gke", "aks"])
def test_preinstalled_driver_shortens_the_critical_path(root):
    g = build_graph(ROOT / root)
    for mode in ("operator", "daemonsets"):
        full = critical_path(g, stack_mode=mode)
        fast = critical_path(g, stack_mode=mode, driver_preinstalled=True)
        assert fast.total_s < full.total_s
        # the whole driver phase goes, bar the device plugin (and what the
        # pre-pull no longer hides behind it)
        assert full.total_s - fast.total_s <= DRIVER_READY_S[mode] - PLUGIN_READY_S + 1e-9


def test_readme_documents_baking_the_driver():
    text = (ROOT / "README.md").read_text()
    assert "## Preinstalled driver" in text
    sec = text.split("## Preinstalled driver", 1)[1].split("\n## ", 1)[0]
    assert "gpu_driver_preinstalled" in sec and "gpu_ami_id" in sec and "amdgpu-dkms" in sec


# ------------------------------------------------------- interconnect floors
def test_busbw_floors_only_apply_with_more_than_one_gpu():
    off = _stack_local("validation_args")
    assert "--rccl-busbw-floor-gbps" not in off and "--xgmi-busbw-floor-gbps" not in off
    one = _stack_local("validation_args", validation_rccl_busbw_floor_gbps=300,
                       validation_gpu_count=1)
    assert "--rccl-busbw-floor-gbps" not in one      # busbw is 0 at n = 1
    eight = _stack_local("validation_args", validation_rccl_busbw_floor_gbps=300,
                         validation_xgmi_busbw_floor_gbps=400, validation_gpu_count=8)
    assert eight[eight.index("--rccl-busbw-floor-gbps") + 1] == "300"
    assert eight[eight.index("--xgmi-busbw-floor-gbps") + 1] == "400"
    # the Job's C2 runs tuned at N > 1, never at N = 1
    assert "--xgmi-tune" in eight and "--xgmi-tune" not in one
    m = load_module(ROOT / "modules" / "amd-gpu-stack")
    for v in ("validation_rccl_busbw_floor_gbps", "validation_xgmi_busbw_floor_gbps"):
        assert m.variables[v].default == 0 and m.variables[v].validations


# ------------------------------------------------- startup-taint gate
def _eval(mdir, expr, **overrides):
    """Evaluate an expression of module ``mdir`` with variable defaults + overrides."""
    from nvidia_terraform_modules_amd.tfcheck.evaluate import Evaluator, Scope, convert

    mod = load_module(mdir)
    ev = Evaluator()
    variables = {}
    for vn, v in mod.variables.items():
        if vn in overrides:
            variables[vn] = overrides[vn]
        elif not v.required:
            variables[vn] = convert(ev.eval(v.block.body.attr("default"), Scope({}, {})),
                                    v.type_expr)
    return ev.eval(expr, Scope(variables, {n: e for n, (e, _, _) in mod.locals.items()},
                               str(mod.path)))


def _blocks(body, btype):
    return [b for b in body.blocks if b.type == btype]


def _pod_spec(res):
    spec = _blocks(res.block.body, "spec")[0]
    tmpl = _blocks(spec.body, "template")[0]
    return _blocks(tmpl.body, "spec")[0].body


PREP = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"


@pytest.mark.parametrize("root", ["eks", "gke", "aks"])
def test_gpu_pools_join_with_the_prep_startup_taint(root, tmp_path):
    m = load_module(ROOT / root)
    if root == "eks":
        expr = m.modules["gpu_node_pool"].block.body.attr("taints")
        on, off = _eval(ROOT / root, expr), _eval(ROOT / root, expr, gpu_node_prep_taint=False)
        assert on["mi355x_prep"] == {"key": PREP, "value": "pending", "effect": "NO_SCHEDULE"}
        assert set(off) == {"amd_gpu"} and on["amd_gpu"]["key"] == "amd.com/gpu"
    elif root == "gke":
        ncfg = _blocks(m.resources["google_container_node_pool.mi355x"].block.body, "node_config")[0]
        dyn = [b for b in _blocks(ncfg.body, "dynamic") if b.labels == ["taint"]][0]
        assert _eval(ROOT / root, dyn.body.attr("for_each")) == [PREP]
        assert _eval(ROOT / root, dyn.body.attr("for_each"), gpu_node_prep_taint=False) == []
        content = _blocks(dyn.body, "content")[0].body
        assert render(content.attr("value")) == '"pending"'
        assert render(content.attr("effect")) == '"NO_SCHEDULE"'
    else:
        expr = m.resources["azurerm_kubernetes_cluster_node_pool.mi355x"].block.body.attr("node_taints")
        assert _eval(ROOT / root, expr) == ["amd.com/gpu=present:NoSchedule",
                                             f"{PREP}=pending:NoSchedule"]
        assert _eval(ROOT / root, expr, gpu_node_prep_taint=False) == ["amd.com/gpu=present:NoSchedule"]
    # the stack gets the same key and the switch; its gate RBAC is planned
    body = m.modules["amd_gpu_stack"].block.body
    assert render(body.attr("node_prep_startup_taint")) == "var.gpu_node_prep_taint"
    assert _eval(ROOT / root, body.attr("node_prep_taint_key")) == PREP
    r = _plan(root, tmp_path)
    assert r.ok, r.errors
    for res in ("kubernetes_service_account_v1.node_prep[0]",
                "kubernetes_cluster_role_v1.node_prep[0]",
                "kubernetes_cluster_role_binding_v1.node_prep[0]"):
        assert STACK + res in r.resources
    off = _plan(root, tmp_path, "gpu_node_prep_taint=false")
    assert off.ok and STACK + "kubernetes_cluster_role_v1.node_prep[0]" not in off.resources


def test_only_the_gpu_stack_tolerates_the_startup_taint():
    """Every GPU-node DaemonSet of the stack (and every operator component)
    tolerates the prep taint; the validation Job does not, so it cannot land
    on a node whose prep is not verified."""
    stack = load_module(ROOT / "modules" / "amd-gpu-stack")
    ds = [r for r in stack.managed if r.type == "kubernetes_daemon_set_v1"]
    assert len(ds) >= 6
    for r in ds:
        dyn = [b for b in _blocks(_pod_spec(r), "dynamic") if b.labels == ["toleration"]]
        assert dyn and render(dyn[0].body.attr("for_each")) == "local.prep_tolerations", r.address
    job = _pod_spec(stack.resources["kubernetes_job_v1.gpu_validation"])
    assert not [b for b in _blocks(job, "dynamic") if b.labels == ["toleration"]]
    tols = [render(b.body.attr("key")) for b in _blocks(job, "toleration")]
    assert tols == ["var.gpu_node_taint_key"]
    on = _stack_local("gpu_tolerations", node_prep_startup_taint=True)
    assert {"key": PREP, "operator": "Exists", "effect": "NoSchedule"} in on
    assert len(_stack_local("gpu_tolerations")) == 1          # off by default in the module
    # operator mode: every component carries gpu_tolerations (gpu-toleration rule)
    assert not [f for f in analyze(stack) if f.rule == "gpu-toleration"]


def test_prep_gate_rbac_and_reboot_wait():
    """The gate itself (reconciler container, fake-/proc runs) is covered by
    tests/test_node_prep_gate.py; here: it is on with the startup taint, its
    verification reads what the Job checks, the reboot path never lets it start
    first, and its RBAC is get + patch on nodes only."""
    stack = load_module(ROOT / "modules" / "amd-gpu-stack")
    assert _stack_local("prep_gate", node_prep_startup_taint=True) is True
    assert _stack_local("prep_gate") is False
    v = "".join(p for p in stack.locals["node_prep_gate_script"][0].parts if isinstance(p, str))
    assert "/sys/kernel/numa_balancing" in v and "Max locked memory *unlimited" in v
    # the reboot path waits for the reboot instead of letting the gate start first
    s = "".join(p for p in stack.locals["node_prep_script"][0].parts if isinstance(p, str))
    assert s.index("systemctl --no-block reboot") < s.index("sleep 600") < s.index("exit 1")
    role = stack.resources["kubernetes_cluster_role_v1.node_prep"].block.body
    rules = _blocks(role, "rule")
    assert len(rules) == 1
    assert render(rules[0].body.attr("resources")) == '["nodes"]'
    assert render(rules[0].body.attr("verbs")) == '["get", "patch"]'


@pytest.mark.parametrize("root", ["eks", "gke", "aks"])
def test_prep_gate_in_the_critical_path(root):
    """The Job waits for the longer of the driver install and the prep gate:
    invisible with a driver to install, the in-node wait with a preinstalled
    driver (the gate's priors: critical_path.PREP_GATE_S)."""
    from nvidia_terraform_modules_amd.gpu_ready.critical_path import PREP_GATE_S

    g = build_graph(ROOT / root)
    assert any("kubernetes_cluster_role_v1.node_prep" in n for n in g.topo_order())
    full = critical_path(g)
    fast = critical_path(g, driver_preinstalled=True)
    slow_gate = critical_path(g, durations={"prep_gate": PREP_GATE_S + 100},
                              driver_preinstalled=True)
    assert abs((slow_gate.total_s - fast.total_s) - 100) < 1e-6
    assert critical_path(g, durations={"prep_gate": 1.0}).total_s == full.total_s
