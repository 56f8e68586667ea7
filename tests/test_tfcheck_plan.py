"""Offline plan (tfcheck/plan.py, BASELINE config #1) and the expression
evaluator behind it."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.tfcheck.evaluate import UNKNOWN, Evaluator, Scope, convert
from nvidia_terraform_modules_amd.tfcheck.hcl import parse_file
from nvidia_terraform_modules_amd.tfcheck.plan import plan

ROOT = Path(__file__).resolve().parents[1]


def _expr(tmp_path, src):
    f = tmp_path / "e.tf"
    f.write_text(f"locals {{\n  x = {src}\n}}\n")
    return parse_file(str(f)).blocks[0].body.attr("x")


@pytest.mark.parametrize("src,variables,expected", [
    ('"${var.a}-x"', {"a": "n"}, "n-x"),
    ('var.n * 2 + 1', {"n": 3}, 7),
    ('var.b ? "y" : "z"', {"b": False}, "z"),
    ('[for k, v in var.m : "${k}=${v}" if v != null]', {"m": {"a": 1, "b": None}}, ["a=1"]),
    ('{for s in var.l : s => upper(s)}', {"l": ["a", "b"]}, {"a": "A", "b": "B"}),
    ('merge(var.m, { c = 3 })["c"]', {"m": {"a": 1}}, 3),
    ('length(concat(var.l, ["z"]))', {"l": ["a"]}, 2),
    ('contains(["RAPID", "REGULAR"], var.s)', {"s": "REGULAR"}, True),
    ('can(regex("^amd-instinct-mi3[0-9]{2}x?$", var.s))', {"s": "amd-instinct-mi355x"}, True),
    ('can(regex("^amd-instinct-mi3[0-9]{2}x?$", var.s))', {"s": "nvidia-tesla-v100"}, False),
    ('try(var.m.missing, "dflt")', {"m": {}}, "dflt"),
    ('var.objs[*].name', {"objs": [{"name": "p"}, {"name": "q"}]}, ["p", "q"]),
    ('cidrsubnet("10.0.0.0/16", 3, 1)', {}, "10.0.32.0/19"),
    ('format("tf-%s-%d", var.a, 2)', {"a": "c"}, "tf-c-2"),
    ('one(var.l)', {"l": ["only"]}, "only"),
    ('data.aws_ami.x.id', {}, UNKNOWN),
    ('"${data.aws_region.current.name}-x"', {}, UNKNOWN),
    ('length(module.eks.ids) > 0 ? 1 : 0', {}, UNKNOWN),
    ('var.n > 0 && true', {"n": 1}, True),
])
def test_evaluator(tmp_path, src, variables, expected):
    assert Evaluator().eval(_expr(tmp_path, src), Scope(variables, {})) == expected


def test_locals_resolve_lazily_and_detect_cycles(tmp_path):
    f = tmp_path / "l.tf"
    f.write_text('locals {\n  a = "${local.b}!"\n  b = upper(var.x)\n  c = local.d\n  d = local.c\n}\n')
    body = parse_file(str(f)).blocks[0].body
    locs = {n: a.expr for n, a in body.attributes.items()}
    ev = Evaluator()
    from nvidia_terraform_modules_amd.tfcheck.hcl import Traversal
    assert ev.eval(Traversal("local", [("attr", "a")]), Scope({"x": "q"}, locs)) == "Q!"
    with pytest.raises(Exception):
        ev.eval(Traversal("local", [("attr", "c")]), Scope({}, locs))


def test_type_conversion(tmp_path):
    t = parse_file(str(_write(tmp_path, 'variable "v" {\n  type = number\n}\n'))).blocks[0].body.attr("type")
    assert convert("2", t) == 2
    t = parse_file(str(_write(tmp_path, 'variable "v" {\n  type = list(number)\n}\n'))).blocks[0].body.attr("type")
    assert convert(["1", "2.5"], t) == [1, 2.5]


def _write(tmp_path, text, name="v.tf"):
    p = tmp_path / name
    p.write_text(text)
    return p


# ------------------------------------------------------------ plans on the modules
def test_eks_plan_clean():
    r = plan(ROOT / "eks", cli_vars=["cluster_name=mi355x", "gpu_instance_type=x.48xlarge",
                                     "gpu_validation_image=registry.example/amdgpu-validate:1"])
    assert r.ok, r.errors
    assert "module.amd_gpu_stack.kubernetes_job_v1.gpu_validation[0]" in r.resources
    assert "module.amd_gpu_stack.helm_release.amd_gpu_operator[0]" in r.resources
    assert any(m.startswith("module.eks ") for m in r.registry_modules)
    assert "data.aws_ami.lookup" in r.data_sources


def test_plan_requires_a_validation_image_while_validating():
    """No unpublished default image: plan stops with a clear message instead of
    an apply that sits in ImagePullBackOff for validation_timeout."""
    r = plan(ROOT / "eks", cli_vars=["cluster_name=mi355x", "gpu_instance_type=x.48xlarge"])
    assert any("validation_enabled needs validation_image" in e for e in r.errors), r.errors
    r = plan(ROOT / "eks", cli_vars=["cluster_name=mi355x", "gpu_instance_type=x.48xlarge",
                                     "gpu_validation_enabled=false"])
    assert r.ok, r.errors


def test_eks_plan_requires_cluster_name_and_instance_type():
    r = plan(ROOT / "eks")
    assert any("No value for required variable var.cluster_name" in e for e in r.errors)
    assert any("Resource precondition failed: terraform_data.gpu_instance_type_guard" in e
               for e in r.errors)


def test_gke_plan_rejects_nvidia_gpu_type():
    base = ["project_id=p", "region=us-central1", "cluster_name=c", "gpu_instance_type=m"]
    r = plan(ROOT / "gke", cli_vars=base + ["node_zones=x"])
    # node_zones is list(string): a bare string is a type error, like terraform
    assert any("node_zones" in e for e in r.errors)
    vf = ROOT / "gke" / "terraform.tfvars"
    r = plan(ROOT / "gke", cli_vars=base + ["gpu_type=nvidia-tesla-v100"])
    assert any("Invalid value for variable var.gpu_type" in e for e in r.errors), r.errors


def test_gke_daemonsets_mode_expands_the_stack(tmp_path):
    vf = _write(tmp_path, 'project_id = "p"\nregion = "us-central1"\ncluster_name = "c"\n'
                'node_zones = ["us-central1-a"]\ngpu_instance_type = "m"\n'
                'gpu_validation_image = "registry.example/amdgpu-validate:1"\n', "t.tfvars")
    r = plan(ROOT / "gke", var_files=[vf])
    assert r.ok, r.errors
    for a in ("module.amd_gpu_stack.kubernetes_daemon_set_v1.amdgpu_dkms[0]",
              "module.amd_gpu_stack.kubernetes_daemon_set_v1.rocm_device_plugin[0]",
              "module.amd_gpu_stack.kubernetes_resource_quota_v1.critical_pods[0]"):
        assert a in r.resources
    assert not any("helm_release.amd_gpu_operator" in a for a in r.resources)


def test_module_validation_errors_surface(tmp_path):
    vf = _write(tmp_path, 'location = "westus3"\nadmin_group_object_ids = []\n'
                'gpu_machine_type = "Standard_X"\ngpus_per_node = 3\n', "t.tfvars")
    r = plan(ROOT / "aks", var_files=[vf])
    assert any("validation_gpu_count" in e or "gpus_per_node" in e for e in r.errors), r.errors


def test_unknown_count_is_a_plan_error(tmp_path):
    d = tmp_path / "m"
    d.mkdir()
    (d / "main.tf").write_text(
        'data "aws_instances" "n" {\n}\n'
        'resource "helm_release" "gated" {\n  count = length(data.aws_instances.n.ids) > 0 ? 1 : 0\n'
        '  name = "x"\n}\n'
        'resource "null_resource" "each" {\n  for_each = { a = 1, b = 2 }\n}\n')
    r = plan(d)
    assert any("helm_release.gated: Invalid count argument" in e for e in r.errors)
    assert 'null_resource.each["a"]' in r.resources and 'null_resource.each["b"]' in r.resources


def test_cli_plan_json():
    p = subprocess.run([sys.executable, "-m", "nvidia_terraform_modules_amd.tfcheck", "--plan",
                        "aks", "--var", "location=westus3", "--var", "gpu_machine_type=S",
                        "--var-file", "/dev/null", "--json"],
                       capture_output=True, text=True, timeout=60, cwd=ROOT)
    d = json.loads(p.stdout)
    assert p.returncode == 1                      # admin_group_object_ids is required
    assert any("admin_group_object_ids" in e for e in d["errors"])
    assert d["summary"].startswith("Plan: ")


def _stack_local(name, **overrides):
    """Evaluate local.<name> of modules/amd-gpu-stack with variable defaults + overrides."""
    from nvidia_terraform_modules_amd.tfcheck.config import load_module

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


def test_validation_job_args_carry_the_fp8_check():
    args = _stack_local("validation_args")
    i = args.index("--fp8-tflops-floor")
    assert float(args[i + 1]) == 2000 and "--no-fp8" not in args
    assert args[-2:] == ["--termination-log", "/dev/termination-log"]
    off = _stack_local("validation_args", validation_fp8=False)
    assert "--no-fp8" in off and "--fp8-tflops-floor" not in off
    assert "--p2p-floor-gbps" not in args
    p2p = _stack_local("validation_args", validation_p2p_floor_gbps=40)
    assert p2p[p2p.index("--p2p-floor-gbps") + 1] == "40"


def test_crd_janitor_deletes_only_crds_this_release_installs():
    """the destroy-time janitor must not delete KMM / NFD CRDs that
    belong to a separate cluster-wide install (a CRD delete cascades to every CR
    of that kind in the cluster)."""
    full = _stack_local("crd_cleanup_list")
    assert "deviceconfigs.amd.com" in full
    assert any(c.endswith(".kmm.sigs.x-k8s.io") for c in full)
    assert any(c.endswith(".nfd.k8s-sigs.io") for c in full)
    no_kmm = _stack_local("crd_cleanup_list", driver_enabled=False)
    assert not any(c.endswith(".kmm.sigs.x-k8s.io") for c in no_kmm)
    assert any(c.endswith(".nfd.k8s-sigs.io") for c in no_kmm)
    no_nfd = _stack_local("crd_cleanup_list", install_node_feature_discovery=False)
    assert not any(c.endswith(".nfd.k8s-sigs.io") for c in no_nfd)
    assert no_nfd[0] == "deviceconfigs.amd.com"


def _stack_eval(expr, **overrides):
    """Evaluate an expression of modules/amd-gpu-stack (variable defaults +
    overrides, the module's locals; cluster_name defaults to "c")."""
    from nvidia_terraform_modules_amd.tfcheck.config import load_module

    overrides.setdefault("cluster_name", "c")
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
    return ev.eval(expr, scope)


def _job_spec():
    from nvidia_terraform_modules_amd.tfcheck.config import load_module

    job = load_module(ROOT / "modules" / "amd-gpu-stack").resources[
        "kubernetes_job_v1.gpu_validation"].block.body
    return job.blocks_of("spec")[0].body


@pytest.mark.parametrize("nodes,backoff", [(1, 1), (3, 0)])
def test_validation_job_runs_one_pod_per_gpu_node(nodes, backoff):
    """Every GPU node the pools start with gets its own validation pod, all at
    once, and apply waits for all of them; with several nodes a failed pod is
    not retried (the retry could land on a node that already passed)."""
    spec = _job_spec()
    assert _stack_eval(spec.attr("completions"), validation_node_count=nodes) == nodes
    assert _stack_eval(spec.attr("parallelism"), validation_node_count=nodes) == nodes
    assert _stack_eval(spec.attr("backoff_limit"), validation_node_count=nodes) == backoff
    tmpl = spec.blocks_of("template")[0].body
    pod_labels = _stack_eval(tmpl.blocks_of("metadata")[0].body.attr("labels"))
    pod = tmpl.blocks_of("spec")[0].body
    anti = pod.blocks_of("affinity")[0].body.blocks_of("pod_anti_affinity")[0].body
    req = anti.blocks_of("required_during_scheduling_ignored_during_execution")[0].body
    assert _stack_eval(req.attr("topology_key")) == "kubernetes.io/hostname"
    sel = _stack_eval(req.blocks_of("label_selector")[0].body.attr("match_labels"))
    assert sel.items() <= pod_labels.items()       # the pods repel each other
    # each pod's verdict names its node (NODE_NAME from the downward API)
    ctr = pod.blocks_of("container")[0].body
    envs = [e.body for e in ctr.blocks_of("env")]
    node = [e for e in envs if e.attr("name") is not None and _stack_eval(e.attr("name")) == "NODE_NAME"]
    assert node, "no NODE_NAME env"
    ref = node[0].blocks_of("value_from")[0].body.blocks_of("field_ref")[0].body
    assert _stack_eval(ref.attr("field_path")) == "spec.nodeName"


def test_validation_node_count_must_be_a_whole_positive_number(tmp_path):
    from nvidia_terraform_modules_amd.tfcheck.config import load_module

    v = load_module(ROOT / "modules" / "amd-gpu-stack").variables["validation_node_count"]
    cond = v.block.body.blocks_of("validation")[0].body.attr("condition")
    ev = Evaluator()
    for n, ok in ((1, True), (4, True), (0, False), (1.5, False)):
        assert ev.eval(cond, Scope({"validation_node_count": n}, {})) is ok


@pytest.mark.parametrize("root,variables,expected", [
    ("eks", {"desired_count_gpu_nodes": 3}, 3),
    ("eks", {"desired_count_gpu_nodes": 0}, 1),
    ("gke", {"num_gpu_nodes": 2, "node_zones": ["z-a", "z-b"]}, 4),
    ("gke", {"num_gpu_nodes": 1, "node_zones": ["z-a"]}, 1),
    ("aks", {"gpu_node_pool_count": 2}, 2),
])
def test_roots_validate_every_gpu_node_they_create(root, variables, expected):
    """The roots size the Job from the GPU pools' node count at creation (GKE:
    node_count is per zone)."""
    from nvidia_terraform_modules_amd.tfcheck.config import load_module

    call = load_module(ROOT / root).modules["amd_gpu_stack"].block.body
    assert Evaluator().eval(call.attr("validation_node_count"), Scope(variables, {})) == expected
