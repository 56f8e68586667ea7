"""Static checks, call-surface contract and plan-graph ordering of the
Terraform modules (offline stand-in for terraform fmt/validate/plan)."""
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.gpu_ready.critical_path import critical_path
from nvidia_terraform_modules_amd.tfcheck.analysis import analyze, errors
from nvidia_terraform_modules_amd.tfcheck.config import find_modules, load_module
from nvidia_terraform_modules_amd.tfcheck.contract import compare, extract, load_expected
from nvidia_terraform_modules_amd.tfcheck.graph import build_graph
from nvidia_terraform_modules_amd.tfcheck.hcl import evaluate_static

REF = Path("/root/reference")
ROOTS = ["eks", "gke", "aks"]


def _modules(repo):
    return [d for d in find_modules(repo) if "charts" not in d.parts]


def test_every_module_is_clean(repo):
    for d in _modules(repo):
        fs = analyze(load_module(d))
        assert not fs, f"{d}: " + "; ".join(map(str, fs))


def test_contract_against_frozen_reference_surface(repo):
    exp = load_expected(repo / "tests/fixtures/reference_surface.json")
    for diff in compare(exp, repo):
        assert diff.ok, diff


@pytest.mark.skipif(not REF.exists(), reason="reference not mounted")
def test_fixture_matches_live_reference(repo):
    assert extract(REF) == load_expected(repo / "tests/fixtures/reference_surface.json")


@pytest.mark.skipif(not REF.exists(), reason="reference not mounted")
def test_checker_finds_the_reference_defects():
    """The survey's hand-found defects must be machine-found."""
    eks = {(f.rule, f.message) for f in analyze(load_module(REF / "eks"))}
    assert ("unused-local", "local 'ami_id' is never used") in eks
    for dead in ("aws_profile", "region", "enable_dns_support", "additional_user_data",
                 "cpu_node_pool_additional_user_data"):
        assert ("unused-variable", f"variable {dead!r} is never used") in eks
    assert any(r == "provider-missing" and "helm" in m for r, m in eks)
    assert any(r == "vendor-lint" for r, _ in eks)
    gke = analyze(load_module(REF / "gke"))
    assert any(f.rule == "unused-data" and "holoscan-cluster" in f.message for f in gke)
    aks = analyze(load_module(REF / "aks"))
    assert {f.message for f in aks if f.rule == "unused-variable"} == {
        "variable 'cpu_os_sku' is never used", "variable 'gpu_os_sku' is never used"}
    # deployment-practice rules (SURVEY §2.4-2.5 / §5 race hazards), each a shipped defect:
    # az aks get-credentials + kubelogin + helm via local-exec (aks/main.tf:52-91)
    assert sum(f.rule == "local-exec" for f in aks) == 4
    # the always-open helm gate count = length(data.aws_instances.nodes) > 0 (eks/main.tf:186)
    assert any(r == "count-object-length" and "aws_instances.nodes" in m for r, m in eks)
    # ssh_key in both node groups is not an input of the eks module (eks/main.tf:109, :118)
    ign = sorted(m for r, m in eks if r == "eks-ignored-input")
    assert len(ign) == 2 and all("ssh_key is ignored" in m for m in ign)
    eks_cn = analyze(load_module(REF / "eks/examples/cnpack"))
    dup = [f for f in eks_cn if f.rule == "duplicate-resource"]   # aws-fluentbit.tf:22-25
    assert len(dup) == 1 and "attach-cloudwatch-to-cpu-ng" in dup[0].message
    gke_cn = analyze(load_module(REF / "gke/examples/cnpack"))
    assert any(f.rule == "iam-authoritative" for f in gke_cn)     # gcp-prometheus.tf:33
    aks_cn = analyze(load_module(REF / "aks/examples/cnpack"))
    sec = [f for f in aks_cn if f.rule == "secret-in-command"]     # azure-fluentbit.tf:28
    assert len(sec) == 1 and "primary_shared_key" in sec[0].message


def test_no_vendor_strings_anywhere(repo):
    for d in _modules(repo):
        m = load_module(d)
        assert not [f for f in analyze(m) if f.rule == "vendor-lint"]


def test_unknown_reference_and_function_are_errors(tmp_path):
    (tmp_path / "main.tf").write_text(
        'terraform {\n  required_providers {\n    null = { source = "hashicorp/null" }\n  }\n}\n'
        'resource "null_resource" "a" {\n  triggers = { x = var.nope, y = frobnicate(1) }\n}\n'
        'output "o" {\n  value = each.key\n}\n')
    rules = sorted(f.rule for f in errors(analyze(load_module(tmp_path))))
    assert rules == ["ref-context", "ref-undefined", "unknown-function"]


def test_module_input_checks(tmp_path):
    child = tmp_path / "child"
    child.mkdir()
    (child / "v.tf").write_text('variable "need" {}\nvariable "opt" {\n  default = 1\n}\noutput "out" {\n  value = var.need\n}\n')
    (tmp_path / "main.tf").write_text(
        'module "c" {\n  source = "./child"\n  bogus  = 1\n}\noutput "x" {\n  value = module.c.missing\n}\n')
    rules = sorted(f.rule for f in errors(analyze(load_module(tmp_path))))
    assert rules == ["module-input", "module-output", "module-required"]


@pytest.mark.parametrize("root", ROOTS)
def test_validation_job_waits_for_gpu_nodes_and_stack(repo, root):
    g = build_graph(repo / root)
    assert not g.hard_cycles()
    (job,) = g.find("kubernetes_job_v1.gpu_validation")
    pools = {"eks": ["module.gpu_node_pool"], "gke": ["google_container_node_pool.mi355x"],
             "aks": ["azurerm_kubernetes_cluster_node_pool.mi355x"]}[root]
    for p in pools:
        assert g.depends_on(job, p), f"{job} must wait for {p}"
    stack = [n for n in g.nodes if "helm_release.device_config" in n or "rocm_device_plugin" in n]
    assert stack and all(g.depends_on(job, s) for s in stack)


GPU_POOL = {"eks": "module.gpu_node_pool", "gke": "google_container_node_pool.mi355x",
            "aks": "azurerm_kubernetes_cluster_node_pool.mi355x"}


@pytest.mark.parametrize("root", ROOTS)
def test_operator_install_overlaps_gpu_node_boot(repo, root):
    """Only the Job needs GPUs: the operator, its DeviceConfig and the CRD
    janitor must NOT wait for the GPU pool (on EKS the whole stack
    hung off module.eks, which contained the GPU node group)."""
    g = build_graph(repo / root)
    pool = GPU_POOL[root]
    for name in ("helm_release.amd_gpu_operator", "helm_release.device_config",
                 "helm_release.crd_janitor", "kubernetes_namespace_v1.gpu_stack"):
        (n,) = g.find(name)
        assert not g.depends_on(n, pool), f"{n} waits for {pool}"
    (job,) = g.find("kubernetes_job_v1.gpu_validation")
    assert g.depends_on(job, pool)


def test_eks_critical_path_runs_stack_beside_gpu_boot(repo):
    """With the node groups outside module "eks", the GPU pool boot and the
    operator install are parallel branches that meet at the validation Job."""
    from nvidia_terraform_modules_amd.gpu_ready.critical_path import DEFAULT_DURATIONS

    g = build_graph(repo / "eks")
    (op,) = g.find("helm_release.amd_gpu_operator")
    assert g.depends_on(op, "module.cpu_node_pool") and g.depends_on(op, "module.eks")
    cp = critical_path(g)
    serial = (DEFAULT_DURATIONS["module.vpc"] + DEFAULT_DURATIONS["module.eks"]
              + DEFAULT_DURATIONS["module.gpu_node_pool"] + 2 * DEFAULT_DURATIONS["helm_release"])
    assert cp.total_s < serial + 300        # not pool-then-operator any more
    on_path = [a for a, _ in cp.path]
    assert not ("module.gpu_node_pool" in on_path and any("amd_gpu_operator" in a for a in on_path))


def test_gpu_workloads_tolerate_the_gpu_taint(repo):
    """Every pod spec placed on the tainted MI355X nodes tolerates the taint -
    the operator's KMM driver pods included (DeviceConfig spec.driver)."""
    m = load_module(repo / "modules/amd-gpu-stack")
    assert not [f for f in analyze(m) if f.rule == "gpu-toleration"]
    dc = m.locals["device_config_values"][0]
    spec = dc.get("spec")
    from nvidia_terraform_modules_amd.tfcheck.analysis import _object_keys
    for comp in ("driver", "devicePlugin", "metricsExporter"):
        assert any(k.endswith("olerations") for k in _object_keys(spec.get(comp))), comp


def test_gpu_toleration_rule_fires(tmp_path):
    (tmp_path / "main.tf").write_text('''terraform {
  required_providers {
    kubernetes = { source = "hashicorp/kubernetes" }
  }
}
variable "gpu_node_selector" {
  default = {}
}
variable "gpu_node_taint_key" {
  default = "amd.com/gpu"
}
locals {
  gpu_tolerations = [{ key = var.gpu_node_taint_key, operator = "Exists" }]
  dc = {
    spec = {
      driver       = { enable = true }
      devicePlugin = { devicePluginTolerations = local.gpu_tolerations }
      selector     = var.gpu_node_selector
    }
  }
}
resource "kubernetes_daemon_set_v1" "x" {
  metadata {
    name = "x"
  }
  spec {
    template {
      spec {
        node_selector = var.gpu_node_selector
        container {
          name  = "c"
          image = "i"
        }
      }
    }
  }
}
output "o" {
  value = local.dc
}
''')
    fs = [f for f in analyze(load_module(tmp_path)) if f.rule == "gpu-toleration"]
    msgs = " ".join(f.message for f in fs)
    assert len(fs) == 2 and "kubernetes_daemon_set_v1.x" in msgs and "'driver'" in msgs


def test_eks_gpu_node_host_prep_takes_effect(repo):
    """iommu=pt must be in effect on the node's first serving
    boot and RLIMIT_MEMLOCK must reach pods (containerd's unit, not PAM)."""
    m = load_module(repo / "eks")
    prep = "".join(p for p in m.locals["mi355x_host_prep"][0].parts if isinstance(p, str))
    assert "containerd.service.d" in prep and "LimitMEMLOCK=infinity" in prep
    assert "systemctl restart containerd" in prep and "limits.d" not in prep
    assert "/proc/cmdline" in prep and "systemctl reboot" in prep and "update-grub" in prep
    assert "cloud-init single --name scripts_user --frequency always" in prep
    assert "set -u" not in prep and "#!/bin/bash" not in prep   # inlined before bootstrap.sh
    pool = m.modules["gpu_node_pool"].block.body
    assert "mi355x_host_prep" in str(pool.attr("pre_bootstrap_user_data"))
    assert m.variables["gpu_node_iommu_passthrough"].default == "reboot"
    assert m.variables["gpu_node_iommu_passthrough"].validations


def test_operator_release_lifecycle_and_destroy_order(repo):
    """reset_values like the reference (eks/main.tf:193-196); CRDs cleaned up on
    destroy (reference operator.cleanupCRD=true, aks/main.tf:89-91); destroy
    order DeviceConfig -> operator -> CRD janitor -> namespace."""
    m = load_module(repo / "modules/amd-gpu-stack")
    op = m.resources["helm_release.amd_gpu_operator"].block.body
    for flag in ("reset_values", "atomic", "cleanup_on_fail"):
        assert evaluate_static(op.attr(flag)) is True, flag
    assert m.variables["gpu_operator_crd_cleanup"].default is True
    crds = m.variables["gpu_operator_crds"].default
    assert "deviceconfigs.amd.com" in crds and any("kmm" in c for c in crds)
    chart = repo / "modules/amd-gpu-stack/charts/amd-gpu-crd-janitor/templates/cleanup.yaml"
    text = chart.read_text()
    assert "helm.sh/hook: pre-delete" in text and "kubectl" in text and "delete" in text
    g = build_graph(repo / "eks")
    (dc,) = g.find("helm_release.device_config")
    (opn,) = g.find("helm_release.amd_gpu_operator")
    (jan,) = g.find("helm_release.crd_janitor")
    (ns,) = g.find("kubernetes_namespace_v1.gpu_stack")
    # destroy runs in reverse dependency order
    assert g.depends_on(dc, opn) and g.depends_on(opn, jan) and g.depends_on(jan, ns)


def test_validation_image_has_no_unpublished_default(repo):
    m = load_module(repo / "modules/amd-gpu-stack")
    assert m.variables["validation_image"].default == ""
    job = m.resources["kubernetes_job_v1.gpu_validation"].block.body
    pre = [p for lc in job.blocks_of("lifecycle") for p in lc.body.blocks_of("precondition")]
    assert pre and "validation_image" in str(pre[0].body.attr("condition"))
    for root in ROOTS:
        assert load_module(repo / root).variables["gpu_validation_image"].default == ""


@pytest.mark.parametrize("root", ROOTS)
def test_root_forwards_tflops_floor(repo, root):
    call = load_module(repo / root).modules["amd_gpu_stack"].block.body
    assert "gpu_validation_tflops_floor" in str(call.attr("validation_tflops_floor"))


def test_kubernetes_and_helm_providers_are_bounded(repo):
    for d in _modules(repo):
        for name, req in load_module(d).required_providers.items():
            if name in ("kubernetes", "helm"):
                v = str(req)
                assert "<" in v, f"{d}: {name} {v}"


def test_stack_defaults_are_amd_mi355x(repo):
    m = load_module(repo / "modules/amd-gpu-stack")
    assert m.variables["gpu_operator_chart_repository"].default.startswith("https://rocm.github.io")
    assert m.variables["validation_gpu_count"].default == 8
    assert m.variables["validation_min_hbm_gb"].default >= 250   # 288 GB HBM3E
    major = int(m.variables["gpu_operator_driver_version"].default.split(".")[0])
    assert major >= 7   # ROCm 7 for gfx950
    job = m.resources["kubernetes_job_v1.gpu_validation"].block
    assert job.body.attr("wait_for_completion") is not None


def test_tfvars_only_set_declared_variables(repo):
    for d in _modules(repo):
        m = load_module(d)
        for fname, body in m.tfvars.items():
            for key in body.attributes:
                assert key in m.variables, f"{d}/{fname}: {key}"
            for key, attr in body.attributes.items():
                evaluate_static(attr.expr)  # tfvars must be static


def test_examples_use_root_module_outputs_that_exist(repo):
    # module-output rule is part of analyze(); re-assert explicitly for the examples
    for ex in ("eks/examples/cnpack", "gke/examples/cnpack", "aks/examples/cnpack"):
        fs = [f for f in analyze(load_module(repo / ex)) if f.rule.startswith("module-")]
        assert not fs, fs


def test_namespace_order_rule(tmp_path):
    """namespace-order: a namespaced resource in a module that creates its
    namespace must take the name from that resource (here through a local) or
    depend on it; Helm-created and built-in namespaces are exempt."""
    (tmp_path / "main.tf").write_text('''terraform {
  required_providers {
    kubernetes = { source = "hashicorp/kubernetes" }
    helm       = { source = "hashicorp/helm" }
  }
}
variable "ns" {
  default = "gpu"
}
resource "kubernetes_namespace_v1" "ns" {
  metadata {
    name = var.ns
  }
}
locals {
  namespace = kubernetes_namespace_v1.ns.metadata[0].name
}
resource "kubernetes_config_map_v1" "ok_local" {
  metadata {
    name      = "a"
    namespace = local.namespace
  }
}
resource "kubernetes_config_map_v1" "ok_depends" {
  metadata {
    name      = "b"
    namespace = var.ns
  }
  depends_on = [kubernetes_namespace_v1.ns]
}
resource "kubernetes_config_map_v1" "ok_system" {
  metadata {
    name      = "c"
    namespace = "kube-system"
  }
}
resource "kubernetes_config_map_v1" "racy" {
  metadata {
    name      = "d"
    namespace = var.ns
  }
}
resource "helm_release" "racy_chart" {
  name      = "x"
  chart     = "x"
  namespace = var.ns
}
resource "helm_release" "helm_creates" {
  name             = "y"
  chart            = "y"
  namespace        = var.ns
  create_namespace = true
}
resource "kubernetes_cluster_role_v1" "cluster_scoped" {
  metadata {
    name = "r"
  }
}
''')
    fs = [f for f in analyze(load_module(tmp_path)) if f.rule == "namespace-order"]
    assert sorted(f.message.split(":")[0] for f in fs) == [
        "helm_release.racy_chart", "kubernetes_config_map_v1.racy"]


@pytest.mark.parametrize("root", ["modules/amd-gpu-stack", "eks", "gke", "aks"])
def test_modules_order_namespaced_resources(repo, root):
    mod = load_module(repo / root)
    assert any(r.type == "kubernetes_namespace_v1" for r in mod.managed) or root != "modules/amd-gpu-stack"
    assert [f for f in analyze(mod) if f.rule == "namespace-order"] == []


def test_eks_ignored_input_rule(tmp_path):
    """eks-ignored-input on the node-group submodule: post_bootstrap_user_data
    needs a custom AMI + enable_bootstrap_user_data; pre_bootstrap is fine."""
    (tmp_path / "main.tf").write_text('''module "custom" {
  source                     = "terraform-aws-modules/eks/aws//modules/eks-managed-node-group"
  ami_id                     = "ami-1"
  enable_bootstrap_user_data = true
  post_bootstrap_user_data   = "echo ok"
}
module "optimized_pre" {
  source                  = "terraform-aws-modules/eks/aws//modules/eks-managed-node-group"
  pre_bootstrap_user_data = "echo ok"
}
module "optimized_post" {
  source                   = "terraform-aws-modules/eks/aws//modules/eks-managed-node-group"
  post_bootstrap_user_data = "echo dropped"
}
''')
    fs = [f for f in analyze(load_module(tmp_path)) if f.rule == "eks-ignored-input"]
    assert len(fs) == 1 and "module.optimized_post" in fs[0].message


def test_moved_rules(tmp_path):
    """moved-cross-package / moved-from-exists / moved-kind:
    the round-3 EKS moves out of the registry module "eks" fire; a move of a
    whole registry call, or into a local child module, does not."""
    from nvidia_terraform_modules_amd.tfcheck.analysis import moved_findings

    child = tmp_path / "child"
    child.mkdir()
    (child / "c.tf").write_text(
        'module "inner" {\n  source = "terraform-aws-modules/eks/aws"\n}\n'
        'resource "null_resource" "r" {}\n')
    (tmp_path / "main.tf").write_text(
        'module "eks" {\n  source  = "terraform-aws-modules/eks/aws"\n  version = "~> 20.31"\n}\n'
        'module "local" {\n  source = "./child"\n}\n'
        'module "ng" {\n  source = "terraform-aws-modules/eks/aws//modules/eks-managed-node-group"\n}\n'
        'resource "aws_eks_addon" "ebs" {}\n'
        # bad: inside a registry package
        'moved {\n  from = module.eks.module.eks_managed_node_group["gpu"]\n  to   = module.ng\n}\n'
        'moved {\n  from = module.eks.aws_eks_addon.this["ebs"]\n  to   = aws_eks_addon.ebs\n}\n'
        # bad: through a local child into its registry call
        'moved {\n  from = module.local.module.inner.aws_iam_role.x\n  to   = aws_eks_addon.ebs\n}\n'
        # good: whole call rename, and into a local child package
        'moved {\n  from = module.old_ng\n  to   = module.ng\n}\n'
        'moved {\n  from = null_resource.r\n  to   = module.local.null_resource.r\n}\n'
        # bad: from still declared; resource -> module
        'moved {\n  from = aws_eks_addon.ebs\n  to   = aws_eks_addon.ebs2\n}\n'
        'moved {\n  from = null_resource.gone\n  to   = module.ng\n}\n'
        'removed {\n  from = module.eks.aws_kms_key.this\n}\n')
    fs = moved_findings(load_module(tmp_path))
    text = (tmp_path / "main.tf").read_text().splitlines()

    def froms(rule):
        return sorted(text[int(f.where.split(":")[1])].strip() for f in fs if f.rule == rule)

    assert froms("moved-cross-package") == [
        "from = module.eks.aws_eks_addon.this[\"ebs\"]", "from = module.eks.aws_kms_key.this",
        "from = module.eks.module.eks_managed_node_group[\"gpu\"]",
        "from = module.local.module.inner.aws_iam_role.x"], fs
    assert froms("moved-from-exists") == ["from = aws_eks_addon.ebs"]
    assert froms("moved-kind") == ["from = null_resource.gone"]
    # ...and the real roots are clean (test_every_module_is_clean runs it too)
    for d in _modules(Path(__file__).resolve().parents[1]):
        assert moved_findings(load_module(d)) == [], d


def test_import_target_rule(tmp_path):
    """import-target: an import must land on a managed resource the
    configuration declares (through local child modules too), never on a module
    call or a data source, and only in a root module."""
    from nvidia_terraform_modules_amd.tfcheck.analysis import import_findings

    child = tmp_path / "child"
    child.mkdir()
    (child / "c.tf").write_text('resource "aws_iam_role" "r" {}\n')
    (tmp_path / "main.tf").write_text(
        'module "local" {\n  source = "./child"\n}\n'
        'module "eks" {\n  source = "terraform-aws-modules/eks/aws"\n}\n'
        'resource "aws_kms_key" "k" {}\n'
        'data "aws_caller_identity" "me" {}\n'
        # good: a declared resource, one in a local child, one inside a registry package
        'import {\n  to = aws_kms_key.k\n  id = "key-1"\n}\n'
        'import {\n  to = module.local.aws_iam_role.r\n  id = "role"\n}\n'
        'import {\n  to = module.eks.aws_iam_role.this[0]\n  id = "role"\n}\n'
        # bad: undeclared, undeclared in the child, a module call, a data source
        'import {\n  to = aws_kms_key.gone\n  id = "x"\n}\n'
        'import {\n  to = module.local.aws_iam_role.nope\n  id = "x"\n}\n'
        'import {\n  to = module.local\n  id = "x"\n}\n'
        'import {\n  to = data.aws_caller_identity.me\n  id = "x"\n}\n')
    fs = import_findings(load_module(tmp_path))
    text = (tmp_path / "main.tf").read_text().splitlines()
    bad = sorted(text[int(f.where.split(":")[1])].strip() for f in fs)
    assert bad == ["to = aws_kms_key.gone", "to = data.aws_caller_identity.me",
                   "to = module.local", "to = module.local.aws_iam_role.nope"], fs
    nonroot = tmp_path / "modules" / "m"
    nonroot.mkdir(parents=True)
    (nonroot / "m.tf").write_text('resource "aws_kms_key" "k" {}\n'
                                  'import {\n  to = aws_kms_key.k\n  id = "x"\n}\n')
    fs = import_findings(load_module(nonroot))
    assert [f.rule for f in fs] == ["import-target"] and "non-root" in fs[0].message
    for d in _modules(Path(__file__).resolve().parents[1]):
        assert import_findings(load_module(d)) == [], d
