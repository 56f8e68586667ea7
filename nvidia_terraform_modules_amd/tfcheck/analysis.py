"""Static checks over a parsed Terraform module (``terraform validate``-like,
minus provider schemas, which need the network).

Rules (each finding is ``Finding(rule, severity, where, message)``):

ref-undefined      var./local./module./data./resource references that resolve nowhere
ref-context        each.* outside for_each, count.* outside count, self outside provisioners
unused-variable    declared variable never referenced (reference had 5: SURVEY §2.6)
unused-local       local never referenced (reference: local.ami_id, eks/main.tf:179)
unused-data        data source never referenced (reference: gke/data.tf:4-8, aks/main.tf:61-65)
provider-missing   resource/provider type not declared in required_providers
count-and-foreach  both meta-arguments on one block
depends-on         depends_on entry that names no resource/module
module-source      local module source directory missing
module-input       argument not declared as a variable of a local callee
module-required    required variable of a local callee not passed
module-output      module.X.Y where Y is not an output of local callee X
unknown-function   call to a function Terraform does not have
vendor-lint        NVIDIA/CUDA-specific strings in literals (AMD-only build)
local-exec         a local-exec provisioner: runs on the operator's workstation, only on create,
                   outside Terraform state (reference: az/kubelogin/helm, aks/main.tf:52-91)
secret-in-command  a local-exec command interpolating a key/secret/password/token attribute:
                   the value lands in the process list and logs (reference:
                   aks/examples/cnpack/azure-fluentbit.tf:28)
iam-authoritative  an authoritative IAM binding/policy that strips every other member of the
                   role (reference: gke/examples/cnpack/gcp-prometheus.tf:33)
duplicate-resource two attachment/member/assignment resources with identical arguments - the
                   second is a copy-paste that left its intended target unattached (reference:
                   eks/examples/cnpack/aws-fluentbit.tf:22-25)
count-object-length count = length(data.X.Y) > 0 counts the data source's ATTRIBUTES, so the
                   gate is always open (reference: eks/main.tf:186)
provider-unbounded a provider version constraint with no upper bound (a major release can
                   change the schema under an unchanged configuration)
eks-ignored-input  an EKS managed-node-group input the upstream module silently ignores:
                   `ssh_key` (v18+ reads key_name / remote_access; reference eks/main.tf:109,
                   :118) or post_bootstrap_user_data on a group without a custom AMI and
                   enable_bootstrap_user_data = true (EKS-optimized AMIs run only the
                   pre-bootstrap hook)
namespace-order    a namespaced kubernetes_* / helm_release resource in a module that creates
                   its namespace neither takes the namespace name from that resource (directly
                   or through locals) nor depends_on it, so Terraform may create it first and
                   the API server rejects it ("namespaces ... not found")
gpu-toleration     a pod spec (or operator component) placed on the GPU nodes through
                   the GPU node selector does not tolerate the GPU node taint, so it
                   would never schedule and `apply` would wait out validation_timeout
moved-cross-package a moved/removed address that reaches INSIDE a module call whose source
                   is not a local path (a registry / git / remote package): Terraform only
                   moves objects within one module package and rejects the whole
                   configuration at plan time ("Cross-package move statement")
moved-from-exists  a moved `from` that is still declared in the configuration ("Moved
                   object still exists")
moved-kind         a moved block between a resource and a module call (both ends must be
                   the same kind)
import-target      an import block whose `to` is not a managed resource declared in the
                   configuration (a module call, a data source, or an address nothing
                   declares: "Configuration for import target does not exist"), or an import
                   block in a module that is not a root (Terraform accepts them only there)
fmt                terraform fmt layout: indentation, spacing, = / comment alignment
                   (errors); tabs / trailing whitespace (warnings)
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from pathlib import Path

from .config import Module, load_module
from .hcl import (Block, Body, Call, Literal, ObjectExpr, Template, Traversal, iter_calls,
                  iter_strings, key_name, walk_refs)

BUILTIN_ROOTS = {"path", "terraform"}

TF_FUNCTIONS = {
    # numeric
    "abs", "ceil", "floor", "log", "max", "min", "parseint", "pow", "signum",
    # string
    "chomp", "endswith", "format", "formatlist", "indent", "join", "lower", "regex", "regexall",
    "replace", "split", "startswith", "strcontains", "strrev", "substr", "templatestring", "title",
    "trim", "trimprefix", "trimspace", "trimsuffix", "upper",
    # collection
    "alltrue", "anytrue", "chunklist", "coalesce", "coalescelist", "compact", "concat", "contains",
    "distinct", "element", "flatten", "index", "keys", "length", "list", "lookup", "map", "matchkeys",
    "merge", "one", "range", "reverse", "setintersection", "setproduct", "setsubtract", "setunion",
    "slice", "sort", "sum", "transpose", "values", "zipmap",
    # encoding
    "base64decode", "base64encode", "base64gzip", "csvdecode", "jsondecode", "jsonencode",
    "textdecodebase64", "textencodebase64", "urlencode", "yamldecode", "yamlencode",
    # filesystem
    "abspath", "dirname", "pathexpand", "basename", "file", "fileexists", "fileset", "filebase64",
    "templatefile",
    # date/time
    "formatdate", "plantimestamp", "timeadd", "timecmp", "timestamp",
    # hash/crypto
    "base64sha256", "base64sha512", "bcrypt", "filebase64sha256", "filebase64sha512", "filemd5",
    "filesha1", "filesha256", "filesha512", "md5", "rsadecrypt", "sha1", "sha256", "sha512", "uuid",
    "uuidv5",
    # ip
    "cidrhost", "cidrnetmask", "cidrsubnet", "cidrsubnets",
    # type conversion
    "can", "issensitive", "nonsensitive", "sensitive", "tobool", "tolist", "tomap", "tonumber",
    "toset", "tostring", "try", "type",
}

# type-constraint keywords appear as calls / bare words inside `type = ...`
TYPE_WORDS = {"string", "number", "bool", "any", "list", "map", "set", "object", "tuple", "optional"}

VENDOR_PATTERNS = [
    re.compile(p, re.I) for p in (
        r"nvidia\.com/gpu", r"helm\.ngc\.nvidia\.com", r"\bcuda\b", r"nvidia-smi", r"\bdcgm",
        r"nvidia/gpu-operator", r"nvidia-tesla", r"\bnvidia-(?:driver|container|device)",
    )
]


@dataclass(frozen=True)
class Finding:
    rule: str
    severity: str   # "error" | "warning"
    where: str
    message: str

    def __str__(self) -> str:
        return f"{self.severity}: [{self.rule}] {self.where}: {self.message}"


class _Scope:
    def __init__(self, block_type: str, has_count: bool, has_for_each: bool, iterators: set,
                 in_provisioner: bool):
        self.block_type = block_type
        self.has_count = has_count
        self.has_for_each = has_for_each
        self.iterators = iterators
        self.in_provisioner = in_provisioner


def _iter_body_exprs(body: Body, scope: _Scope, skip_attrs: tuple = ()):
    """Yield (expr, scope, line) for every attribute expression, descending
    into nested blocks (dynamic blocks add their iterator name)."""
    for name, attr in body.attributes.items():
        if name in skip_attrs:
            continue
        yield attr.expr, scope, attr.line, name
    for b in body.blocks:
        if b.type == "dynamic":
            it = b.labels[0] if b.labels else "dynamic"
            it_expr = b.body.attr("iterator")
            if isinstance(it_expr, Traversal):
                it = it_expr.root
            fe = b.body.attr("for_each")
            if fe is not None:
                yield fe, scope, b.line, "for_each"
            inner = _Scope(scope.block_type, scope.has_count, scope.has_for_each,
                           scope.iterators | {it}, scope.in_provisioner)
            for c in b.body.blocks_of("content"):
                yield from _iter_body_exprs(c.body, inner)
            for an, attr in b.body.attributes.items():
                if an in ("for_each", "iterator", "labels"):
                    continue
                yield attr.expr, inner, attr.line, an
        elif b.type in ("provisioner", "connection"):
            inner = _Scope(scope.block_type, scope.has_count, scope.has_for_each, scope.iterators, True)
            yield from _iter_body_exprs(b.body, inner)
        elif b.type == "lifecycle":
            for an, attr in b.body.attributes.items():
                if an in ("ignore_changes", "replace_triggered_by"):
                    continue  # bare attribute names, not references
                yield attr.expr, scope, attr.line, an
            for c in b.body.blocks:
                yield from _iter_body_exprs(c.body, scope)
        else:
            yield from _iter_body_exprs(b.body, scope)


def _block_scope(b: Block) -> _Scope:
    return _Scope(b.type, "count" in b.body.attributes, "for_each" in b.body.attributes, set(), False)


def module_exprs(mod: Module):
    """Yield (expr, scope, where, attr_name, owner) over the whole module."""
    for fname, body in mod.files.items():
        for b in body.blocks:
            if b.type in ("resource", "data", "module"):
                owner = ".".join(([] if b.type == "resource" else [b.type]) + list(b.labels))
                skip = ("source", "version", "providers") if b.type == "module" else ("provider",)
                for e, sc, line, an in _iter_body_exprs(b.body, _block_scope(b), skip):
                    yield e, sc, f"{fname}:{line}", an, owner
            elif b.type in ("output", "locals", "provider", "check"):
                sc = _Scope(b.type, False, False, set(), False)
                for e, s2, line, an in _iter_body_exprs(b.body, sc):
                    yield e, s2, f"{fname}:{line}", an, b.type
            elif b.type == "variable":
                sc = _Scope("variable", False, False, set(), False)
                for e, s2, line, an in _iter_body_exprs(b.body, sc):
                    if an == "type":
                        continue
                    yield e, s2, f"{fname}:{line}", an, f"var.{b.labels[0]}"
            elif b.type == "terraform":
                continue


def analyze(mod: Module, *, strict_unused: bool = True, vendor_lint: bool = True,
            check_fmt: bool = True, callee_loader=load_module) -> list[Finding]:
    out: list[Finding] = [Finding("parse", "error", str(mod.path), e) for e in mod.errors]
    used_vars: set[str] = set()
    used_locals: set[str] = set()
    used_data: set[str] = set()
    used_resources: set[str] = set()
    used_modules: set[str] = set()
    resource_types = {r.type for r in mod.managed}
    data_types = {r.type for r in mod.data}
    callees: dict[str, Module] = {}
    for name, mc in mod.modules.items():
        if mc.is_local:
            p = (mod.path / mc.source).resolve()
            if not p.is_dir() or not list(p.glob("*.tf")):
                out.append(Finding("module-source", "error", f"{mc.file}:{mc.block.line}",
                                   f"module {name!r}: source {mc.source!r} not found"))
            else:
                callees[name] = callee_loader(p)

    for expr, scope, where, attr, owner in module_exprs(mod):
        if attr == "depends_on":
            for ref, _ in walk_refs(expr):
                tgt = ".".join([ref.root] + ref.path()[:2 if ref.root == "data" else 1])
                if ref.root == "module":
                    ok = bool(ref.path()) and ref.path()[0] in mod.modules
                    if ok:
                        used_modules.add(ref.path()[0])
                elif ref.root == "data":
                    ok = tgt in mod.resources
                    used_data.add(tgt)
                else:
                    ok = tgt in mod.resources
                    used_resources.add(tgt)
                if not ok:
                    out.append(Finding("depends-on", "error", where, f"depends_on entry {tgt!r} not found"))
            continue
        for call in iter_calls(expr):
            if call.name not in TF_FUNCTIONS and not (attr == "type" and call.name in TYPE_WORDS):
                out.append(Finding("unknown-function", "error", where, f"unknown function {call.name}()"))
        for ref, bound in walk_refs(expr):
            root = ref.root
            path = ref.path()
            if root in bound or root in scope.iterators:
                continue
            if root == "var":
                if not path or path[0] not in mod.variables:
                    out.append(Finding("ref-undefined", "error", where, f"undefined variable var.{path[0] if path else '?'}"))
                else:
                    used_vars.add(path[0])
            elif root == "local":
                if not path or path[0] not in mod.locals:
                    out.append(Finding("ref-undefined", "error", where, f"undefined local.{path[0] if path else '?'}"))
                else:
                    used_locals.add(path[0])
            elif root == "module":
                if not path or path[0] not in mod.modules:
                    out.append(Finding("ref-undefined", "error", where, f"undefined module.{path[0] if path else '?'}"))
                else:
                    used_modules.add(path[0])
                    callee = callees.get(path[0])
                    if callee is not None and len(path) > 1 and path[1] not in callee.outputs \
                            and not path[1].isdigit():
                        out.append(Finding("module-output", "error", where,
                                           f"module.{path[0]} has no output {path[1]!r}"))
            elif root == "data":
                if len(path) < 2 or f"data.{path[0]}.{path[1]}" not in mod.resources:
                    out.append(Finding("ref-undefined", "error", where, f"undefined data.{'.'.join(path[:2])}"))
                else:
                    used_data.add(f"data.{path[0]}.{path[1]}")
            elif root == "each":
                if not scope.has_for_each:
                    out.append(Finding("ref-context", "error", where, "each.* used without for_each"))
            elif root == "count":
                if not scope.has_count:
                    out.append(Finding("ref-context", "error", where, "count.* used without count"))
            elif root == "self":
                if not scope.in_provisioner:
                    out.append(Finding("ref-context", "error", where, "self used outside a provisioner"))
            elif root in BUILTIN_ROOTS:
                continue
            elif root in resource_types:
                addr = f"{root}.{path[0]}" if path else root
                if addr not in mod.resources:
                    out.append(Finding("ref-undefined", "error", where, f"undefined resource {addr}"))
                used_resources.add(addr)
            elif attr == "type" or root in TYPE_WORDS and owner.startswith("var."):
                continue
            else:
                out.append(Finding("ref-undefined", "error", where, f"unknown reference root {root!r}"))

    # module call arguments vs callee variables
    for name, mc in mod.modules.items():
        callee = callees.get(name)
        if callee is None:
            continue
        meta = {"source", "version", "count", "for_each", "providers", "depends_on"}
        passed = set(mc.block.body.attributes) - meta
        for arg in sorted(passed - set(callee.variables)):
            out.append(Finding("module-input", "error", f"{mc.file}:{mc.block.line}",
                               f"module {name!r}: callee has no variable {arg!r}"))
        for v in sorted(n for n, var in callee.variables.items() if var.required and n not in passed):
            out.append(Finding("module-required", "error", f"{mc.file}:{mc.block.line}",
                               f"module {name!r}: required variable {v!r} not set"))

    if strict_unused:
        for n, v in mod.variables.items():
            if n not in used_vars:
                out.append(Finding("unused-variable", "warning", f"{v.file}:{v.block.line}",
                                   f"variable {n!r} is never used"))
        for n, (_, f, line) in mod.locals.items():
            if n not in used_locals:
                out.append(Finding("unused-local", "warning", f"{f}:{line}", f"local {n!r} is never used"))
        for r in mod.data:
            if r.address not in used_data:
                out.append(Finding("unused-data", "warning", f"{r.file}:{r.block.line}",
                                   f"{r.address} is never referenced"))

    # providers
    declared = set(mod.required_providers) | {"terraform"}
    for r in mod.resources.values():
        p = r.provider_name
        if p not in declared:
            out.append(Finding("provider-missing", "error", f"{r.file}:{r.block.line}",
                               f"{r.address}: provider {p!r} not in required_providers"))
    for pb in mod.providers:
        if pb.labels and pb.labels[0] not in declared:
            out.append(Finding("provider-missing", "error", f"provider:{pb.line}",
                               f"provider block {pb.labels[0]!r} not in required_providers"))

    for r in list(mod.resources.values()) + list(mod.modules.values()):
        attrs = r.block.body.attributes
        if "count" in attrs and "for_each" in attrs:
            out.append(Finding("count-and-foreach", "error", f"{r.file}:{r.block.line}",
                               "count and for_each are mutually exclusive"))

    if vendor_lint:
        out.extend(vendor_findings(mod))
    out.extend(toleration_findings(mod))
    out.extend(practice_findings(mod))
    out.extend(namespace_findings(mod))
    out.extend(eks_node_group_findings(mod))
    out.extend(moved_findings(mod, callee_loader))
    out.extend(import_findings(mod, callee_loader))
    if check_fmt:
        out.extend(fmt_findings(mod.path))
    return out


def vendor_findings(mod: Module) -> list[Finding]:
    out = []
    for expr, _, where, _, _ in module_exprs(mod):
        for s in iter_strings(expr):
            for pat in VENDOR_PATTERNS:
                if pat.search(s):
                    out.append(Finding("vendor-lint", "error", where,
                                       f"NVIDIA/CUDA-specific string {s.strip()[:60]!r}"))
    for fname, body in mod.tfvars.items():
        for name, attr in body.attributes.items():
            for s in iter_strings(attr.expr):
                if any(p.search(s) for p in VENDOR_PATTERNS):
                    out.append(Finding("vendor-lint", "error", f"{fname}:{attr.line}",
                                       f"NVIDIA/CUDA-specific string in {name}"))
    return out


GPU_SELECTOR = "gpu_node_selector"
GPU_TAINT = "gpu_node_taint_key"
GPU_TOLERATIONS = "gpu_tolerations"   # local list built from the taint key


def _refers_to(expr, name: str) -> bool:
    return any(name in ref.path() or ref.root == name for ref, _ in walk_refs(expr))


def _pod_specs(body: Body, where: str):
    """Every block body (recursively) that sets node_selector."""
    if body.attr("node_selector") is not None:
        yield body, where
    for b in body.blocks:
        yield from _pod_specs(b.body, where)


def _tolerates(body: Body) -> bool:
    for b in body.blocks:
        if b.type == "toleration" and _refers_to(b.body.attr("key") or ObjectExpr([]), GPU_TAINT):
            return True
        if b.type == "dynamic" and b.labels and b.labels[0] == "toleration":
            fe = b.body.attr("for_each")
            if fe is not None and (_refers_to(fe, GPU_TOLERATIONS) or _refers_to(fe, GPU_TAINT)):
                return True
    return False


def _object_keys(expr) -> dict:
    """Static keys -> values of an object constructor, or of merge(...) of them."""
    if isinstance(expr, ObjectExpr):
        return {key_name(k): v for k, v in expr.items if key_name(k)}
    if isinstance(expr, Call) and expr.name == "merge":
        out: dict = {}
        for a in expr.args:
            out.update(_object_keys(a))
        return out
    return {}


def _selector_objects(expr):
    """Object constructors (anywhere inside expr) that carry a `selector` key."""
    stack = [expr]
    while stack:
        e = stack.pop()
        if isinstance(e, ObjectExpr):
            if e.get("selector") is not None:
                yield e
            stack.extend(v for _, v in e.items)
        elif isinstance(e, Call):
            stack.extend(e.args)


def toleration_findings(mod: Module) -> list[Finding]:
    """gpu-toleration: Kubernetes pod specs whose node_selector references the
    GPU node selector need a toleration keyed on the GPU taint; operator CRs
    (DeviceConfig) whose `selector` is the GPU node selector need a
    *olerations entry referencing the GPU tolerations in every component."""
    out = []
    for r in mod.managed:
        for body, _ in _pod_specs(r.block.body, r.address):
            if _refers_to(body.attr("node_selector"), GPU_SELECTOR) and not _tolerates(body):
                out.append(Finding("gpu-toleration", "error", f"{r.file}:{r.block.line}",
                                   f"{r.address}: pod spec selects the GPU nodes but does not "
                                   f"tolerate var.{GPU_TAINT}"))
    for name, (expr, f, line) in mod.locals.items():
        for obj in _selector_objects(expr):
            if not _refers_to(obj.get("selector"), GPU_SELECTOR):
                continue
            for comp, val in _object_keys(obj).items():
                keys = _object_keys(val)
                if not keys:
                    continue      # scalar settings next to the components
                tol = [v for k, v in keys.items() if k.lower().endswith("tolerations")]
                if not tol or not all(_refers_to(v, GPU_TOLERATIONS) for v in tol):
                    out.append(Finding("gpu-toleration", "error", f"{f}:{line}",
                                       f"local.{name}: component {comp!r} runs on the GPU "
                                       f"nodes without local.{GPU_TOLERATIONS}"))
    return out


SECRET_WORDS = re.compile(r"(key|secret|password|passwd|token|credential)", re.I)
AUTHORITATIVE_IAM = {"google_project_iam_binding", "google_project_iam_policy",
                     "google_folder_iam_binding", "google_folder_iam_policy",
                     "google_organization_iam_binding", "google_organization_iam_policy"}
DUP_TYPES = re.compile(r"(attachment|iam_member|role_assignment)$")
CLUSTER_CLIS = re.compile(r"\b(kubectl|helm|kubelogin|az\s+aks|aws\s+eks|gcloud\s+container)\b")


def _provisioners(body: Body):
    for b in body.blocks:
        if b.type == "provisioner":
            yield b
        else:
            yield from _provisioners(b.body)


def _bounded(constraint: str) -> bool:
    parts = [p.strip() for p in constraint.split(",") if p.strip()]
    return any(p.startswith(("<", "~>")) or p[0].isdigit() or p.startswith("=") and
               not p.startswith("=>") for p in parts)


def practice_findings(mod: Module) -> list[Finding]:
    """Deployment-practice rules (each one a defect the reference shipped)."""
    from .docs import render

    out = []
    seen_args: dict = {}
    for r in mod.managed:
        where = f"{r.file}:{r.block.line}"
        for pb in _provisioners(r.block.body):
            if not pb.labels or pb.labels[0] != "local-exec":
                continue
            cmd = pb.body.attr("command")
            text = " ".join(iter_strings(cmd)) if cmd is not None else ""
            what = ("runs cluster CLIs (kubeconfig side effects) " if CLUSTER_CLIS.search(text)
                    else "")
            out.append(Finding("local-exec", "warning", where,
                               f"{r.address}: local-exec provisioner {what}- create-time only, "
                               "outside state; use a provider resource"))
            if cmd is not None:
                for ref, _ in walk_refs(cmd):
                    last = (ref.path() or [ref.root])[-1]
                    if SECRET_WORDS.search(last):
                        out.append(Finding("secret-in-command", "error", where,
                                           f"{r.address}: command line carries {ref.root}."
                                           f"{'.'.join(ref.path())}"))
        if r.type in AUTHORITATIVE_IAM:
            out.append(Finding("iam-authoritative", "warning", where,
                               f"{r.address}: authoritative IAM {r.type} removes every other "
                               "member of the role; use the *_iam_member form"))
        if DUP_TYPES.search(r.type):
            attrs = {k: render(a.expr) for k, a in r.block.body.attributes.items()
                     if k not in ("count", "for_each", "depends_on", "provider")}
            key = (r.type, tuple(sorted(attrs.items())))
            if key in seen_args:
                out.append(Finding("duplicate-resource", "error", where,
                                   f"{r.address}: same arguments as {seen_args[key]}"))
            else:
                seen_args[key] = r.address
        cnt = r.block.body.attr("count")
        if cnt is not None:
            for call in iter_calls(cnt):
                if call.name == "length" and len(call.args) == 1 and \
                        isinstance(call.args[0], Traversal) and call.args[0].root == "data" and \
                        len(call.args[0].path()) == 2:
                    out.append(Finding("count-object-length", "warning", where,
                                       f"{r.address}: length() of data.{'.'.join(call.args[0].path())}"
                                       " counts its attributes - the gate is always open"))
    for name, spec in mod.required_providers.items():
        v = spec.get("version") if isinstance(spec, dict) else None
        if v and not _bounded(v):
            out.append(Finding("provider-unbounded", "warning", "terraform",
                               f"provider {name!r} constraint {v!r} has no upper bound"))
    return out


EKS_MODULE = "terraform-aws-modules/eks/aws"
EKS_NG_IGNORED = {"ssh_key": "the module reads key_name (or remote_access)"}


def _true(expr) -> bool:
    return isinstance(expr, Literal) and expr.value is True


def _node_group_inputs(mod: Module):
    """(where, label, get) for every EKS managed node group: entries of module
    "eks"'s eks_managed_node_groups map, and eks-managed-node-group submodule
    calls (their own arguments)."""
    for mc in mod.modules.values():
        src = mc.source
        where = f"{mc.file}:{mc.block.line}"
        if src == EKS_MODULE:
            groups = mc.block.body.attr("eks_managed_node_groups")
            if isinstance(groups, ObjectExpr):
                for k, v in groups.items:
                    if isinstance(v, ObjectExpr):
                        yield where, f"module.{mc.name} node group {key_name(k)!r}", v.get
        elif src.startswith(EKS_MODULE + "//modules/eks-managed-node-group"):
            yield where, f"module.{mc.name}", mc.block.body.attr


def eks_node_group_findings(mod: Module) -> list[Finding]:
    """eks-ignored-input: node-group inputs the upstream module never reads."""
    out = []
    for where, label, get in _node_group_inputs(mod):
        for key, why in EKS_NG_IGNORED.items():
            if get(key) is not None:
                out.append(Finding("eks-ignored-input", "error", where,
                                   f"{label}: {key} is ignored - {why}"))
        if get("post_bootstrap_user_data") is not None and not (
                _true(get("enable_bootstrap_user_data")) and get("ami_id") is not None):
            out.append(Finding("eks-ignored-input", "error", where,
                               f"{label}: post_bootstrap_user_data is ignored without a custom "
                               "ami_id and enable_bootstrap_user_data = true - use "
                               "pre_bootstrap_user_data"))
    return out


def _address_steps(t: Traversal) -> list:
    """A moved/removed address as (kind, value) steps, root included."""
    return [("attr", t.root)] + list(t.ops)


def _cross_package(t: Traversal, mod: Module, loader):
    """The first module call with a non-local source that `t` reaches inside
    of (a different module package), or None. The address of a whole call
    (`module.x`, `module.x["k"]`) stays in the caller's package."""
    steps = _address_steps(t)
    cur, i = mod, 0
    while i + 1 < len(steps) and steps[i] == ("attr", "module") and steps[i + 1][0] == "attr":
        mc = cur.modules.get(steps[i + 1][1]) if cur is not None else None
        i += 2
        if i < len(steps) and steps[i][0] == "index":
            i += 1
        if i >= len(steps) or mc is None:
            return None
        if not mc.is_local:
            return mc
        p = (cur.path / mc.source).resolve()
        cur = loader(p) if p.is_dir() else None
    return None


def _declared(t: Traversal, mod: Module) -> bool:
    """A local (this-module) resource or module-call address is declared."""
    steps = [v for k, v in _address_steps(t) if k == "attr"]
    if steps[:1] == ["module"]:
        return len(steps) == 2 and steps[1] in mod.modules
    if steps[:1] == ["data"]:
        return len(steps) == 3 and f"data.{steps[1]}.{steps[2]}" in mod.resources
    return len(steps) == 2 and f"{steps[0]}.{steps[1]}" in mod.resources


def _is_module_addr(t: Traversal) -> bool:
    """The address names a module call (its last named step is module.X)."""
    names = [v for k, v in _address_steps(t) if k == "attr"]
    return len(names) >= 2 and names[-2] == "module"


def moved_findings(mod: Module, loader=load_module) -> list[Finding]:
    """moved-cross-package / moved-from-exists / moved-kind (Terraform's own
    plan-time checks on refactoring blocks, which an offline parser would
    otherwise pass: round 3 shipped moves out of the registry module "eks")."""
    from .docs import render

    out = []
    blocks = [(b, f, "moved", ("from", "to")) for b, f in mod.moved] + \
             [(b, f, "removed", ("from",)) for b, f in mod.removed]
    for b, f, kind, keys in blocks:
        where = f"{f}:{b.line}"
        ends = {k: b.body.attr(k) for k in keys}
        for key, t in ends.items():
            if not isinstance(t, Traversal):
                continue
            mc = _cross_package(t, mod, loader)
            if mc is not None:
                out.append(Finding("moved-cross-package", "error", where,
                                   f"{kind} {key} = {render(t)} reaches inside module.{mc.name} "
                                   f"(source {mc.source!r}), another module package: Terraform "
                                   "rejects cross-package moves - use `terraform state mv`"))
        frm, to = ends.get("from"), ends.get("to")
        if kind == "moved" and isinstance(frm, Traversal) and isinstance(to, Traversal):
            if _declared(frm, mod):
                out.append(Finding("moved-from-exists", "error", where,
                                   f"moved from {render(frm)} is still declared"))
            if _is_module_addr(frm) != _is_module_addr(to):
                out.append(Finding("moved-kind", "error", where,
                                   f"moved {render(frm)} -> {render(to)}: one end is a module "
                                   "call, the other a resource"))
    return out


def _resolve_target(t: Traversal, mod: Module, loader):
    """(module holding the resource, "type.name", is_data) for a resource address
    through local module calls; module None when the path enters another package
    (unverifiable offline), or when the address names no resource."""
    steps = _address_steps(t)
    cur, i = mod, 0
    while i + 1 < len(steps) and steps[i] == ("attr", "module") and steps[i + 1][0] == "attr":
        mc = cur.modules.get(steps[i + 1][1])
        if mc is None:
            return cur, f"module.{steps[i + 1][1]}", False  # an undeclared call: not found below
        i += 2
        if i < len(steps) and steps[i][0] == "index":
            i += 1
        if not mc.is_local:
            return None, "", False
        p = (cur.path / mc.source).resolve()
        if not p.is_dir():
            return None, "", False
        cur = loader(p)
    names = [v for k, v in steps[i:] if k == "attr"]
    if names[:1] == ["data"]:
        return cur, ".".join(names[1:3]), True
    return cur, ".".join(names[:2]), False


def import_findings(mod: Module, loader=load_module) -> list[Finding]:
    """import-target: Terraform's plan-time checks on import blocks."""
    from .docs import render

    out = []
    non_root = "modules" in mod.path.parts
    for b, f in mod.imports:
        where = f"{f}:{b.line}"
        if non_root:
            out.append(Finding("import-target", "error", where,
                               "import block in a non-root module (Terraform allows them only "
                               "in the root module)"))
        to = b.body.attr("to")
        if not isinstance(to, Traversal):
            out.append(Finding("import-target", "error", where, "import without a `to` address"))
            continue
        if _is_module_addr(to):
            out.append(Finding("import-target", "error", where,
                               f"import to = {render(to)}: a module call, not a resource"))
            continue
        holder, addr, is_data = _resolve_target(to, mod, loader)
        if holder is None:
            continue  # inside another package: not checkable offline
        if is_data:
            out.append(Finding("import-target", "error", where,
                               f"import to = {render(to)}: a data source cannot be imported"))
        elif addr not in holder.resources:
            out.append(Finding("import-target", "error", where,
                               f"import to = {render(to)}: no resource {addr} is declared "
                               "there (\"Configuration for import target does not exist\")"))
    return out


NAMESPACE_TYPES = {"kubernetes_namespace", "kubernetes_namespace_v1"}
# cluster-scoped kinds: no namespace to wait for
CLUSTER_SCOPED = re.compile(r"^kubernetes_(namespace|cluster_role|cluster_role_binding|"
                            r"storage_class|priority_class|persistent_volume|"
                            r"(validating|mutating)_webhook_configuration|"
                            r"custom_resource_definition|csi_driver|runtime_class)(_v1)?$")


def _namespace_expr(r):
    """The namespace expression of a namespaced resource, or None."""
    if r.type == "helm_release":
        return r.block.body.attr("namespace")
    if r.type.startswith("kubernetes_") and not CLUSTER_SCOPED.match(r.type):
        for b in r.block.body.blocks:
            if b.type == "metadata":
                return b.body.attr("namespace")
    return None


def _reaches_namespace(expr, mod: Module, seen: set) -> bool:
    """expr references a namespace resource, directly or through locals."""
    for ref, _ in walk_refs(expr):
        if ref.root in NAMESPACE_TYPES:
            return True
        if ref.root == "local" and ref.path():
            name = ref.path()[0]
            if name in seen or name not in mod.locals:
                continue
            seen.add(name)
            if _reaches_namespace(mod.locals[name][0], mod, seen):
                return True
    return False


def namespace_findings(mod: Module) -> list[Finding]:
    """namespace-order: every namespaced resource must be ordered after the
    namespace resource the module creates (implicit reference or depends_on)."""
    if not any(r.type in NAMESPACE_TYPES for r in mod.managed):
        return []
    out = []
    for r in mod.managed:
        ns = _namespace_expr(r)
        if ns is None:
            continue
        cn = r.block.body.attr("create_namespace") if r.type == "helm_release" else None
        if isinstance(cn, Literal) and cn.value is True:
            continue  # Helm creates it
        if isinstance(ns, Template) and ns.literal() in ("default", "kube-system"):
            continue
        if isinstance(ns, Literal) and ns.value in ("default", "kube-system"):
            continue
        if _reaches_namespace(ns, mod, set()):
            continue
        dep = r.block.body.attr("depends_on")
        if dep is not None and any(ref.root in NAMESPACE_TYPES for ref, _ in walk_refs(dep)):
            continue
        out.append(Finding("namespace-order", "error", f"{r.file}:{r.block.line}",
                           f"{r.address}: namespace is not taken from (nor depends_on) the "
                           "namespace resource this module creates"))
    return out


def fmt_findings(path: Path) -> list[Finding]:
    """``terraform fmt -check`` offline: tabs and trailing whitespace (warnings)
    plus every line whose indentation, spacing or ``=`` / comment alignment is
    not the canonical layout (errors; tfcheck/fmt.py, ``--fmt-write`` fixes them)."""
    from .fmt import FmtLexError, fmt_diff

    out = []
    for f in sorted(Path(path).glob("*.tf")) + sorted(Path(path).glob("*.tfvars")):
        text = f.read_text()
        for i, line in enumerate(text.splitlines(), 1):
            if "\t" in line:
                out.append(Finding("fmt", "warning", f"{f.name}:{i}", "tab character"))
            if line != line.rstrip():
                out.append(Finding("fmt", "warning", f"{f.name}:{i}", "trailing whitespace"))
        try:
            diff = fmt_diff(text)
        except FmtLexError as e:
            out.append(Finding("fmt", "error", f.name, f"cannot lay out: {e}"))
            continue
        for i, have, want in diff:
            out.append(Finding("fmt", "error", f"{f.name}:{i}",
                               f"terraform fmt would rewrite {have.strip()!r} as {want!r}"))
    return out


def errors(findings: list[Finding]) -> list[Finding]:
    return [f for f in findings if f.severity == "error"]
