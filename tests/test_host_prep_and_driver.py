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
    m = load_module(ROOT / "modules" / "amd-gpu-stack")
    for v in ("validation_rccl_busbw_floor_gbps", "validation_xgmi_busbw_floor_gbps"):
        assert m.variables[v].default == 0 and m.variables[v].validations
