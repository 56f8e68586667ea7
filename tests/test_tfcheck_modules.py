"""Static checks, call-surface contract and plan-graph ordering of the
Terraform modules (offline stand-in for terraform fmt/validate/plan)."""
from pathlib import Path

import pytest

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
    pools = {"eks": ["module.eks"], "gke": ["google_container_node_pool.mi355x"],
             "aks": ["azurerm_kubernetes_cluster_node_pool.mi355x"]}[root]
    for p in pools:
        assert g.depends_on(job, p), f"{job} must wait for {p}"
    stack = [n for n in g.nodes if "helm_release.device_config" in n or "rocm_device_plugin" in n]
    assert stack and all(g.depends_on(job, s) for s in stack)


@pytest.mark.parametrize("root", ["gke", "aks"])
def test_operator_install_overlaps_gpu_node_boot(repo, root):
    """Only the Job needs GPUs: the operator must NOT wait for the GPU pool."""
    g = build_graph(repo / root)
    (op,) = g.find("helm_release.amd_gpu_operator")
    pool = {"gke": "google_container_node_pool.mi355x",
            "aks": "azurerm_kubernetes_cluster_node_pool.mi355x"}[root]
    assert not g.depends_on(op, pool)


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
