"""Offline ``terraform plan`` stand-in (BASELINE config #1: "terraform validate
+ plan on eks/ with null provider / local backend").

No terraform binary and no provider schemas are available offline, so this is
not a provider-accurate plan. It does perform the plan-time checks that do
not need providers, in Terraform's order:

1. input variables: tfvars (``terraform.tfvars``, ``*.auto.tfvars``, then
   ``--var-file`` and ``--var``) + defaults, "No value for required variable",
   type conversion, every ``validation {}`` block;
2. ``count`` / ``for_each`` of every resource, data source and module call,
   expanded into instance addresses; an argument that is only known after
   apply is the same error Terraform reports ("Invalid count argument");
3. resource ``lifecycle { precondition }`` and output ``precondition``
   blocks that are decidable;
4. recursion into LOCAL child modules with their evaluated inputs (registry
   modules are listed, not expanded: their source is not vendored).

The result is the list of resource instances a create-from-scratch apply
would add, plus errors. Unknown values propagate like Terraform's.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

from .config import Module, load_module
from .evaluate import UNKNOWN, EvalError, Evaluator, Scope, convert, is_unknown
from .hcl import Template, parse_file

META_ARGS = {"source", "version", "count", "for_each", "providers", "depends_on"}


@dataclass
class PlanResult:
    resources: list = field(default_factory=list)    # instance addresses to create
    data_sources: list = field(default_factory=list)
    registry_modules: list = field(default_factory=list)
    errors: list = field(default_factory=list)
    warnings: list = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return not self.errors

    def summary(self) -> str:
        s = f"Plan: {len(self.resources)} to add, 0 to change, 0 to destroy."
        if self.registry_modules:
            s += f" (+ {len(self.registry_modules)} registry module(s) not expanded offline)"
        return s

    def as_dict(self) -> dict:
        return {"resources": self.resources, "data_sources": self.data_sources,
                "registry_modules": self.registry_modules, "errors": self.errors,
                "warnings": self.warnings, "summary": self.summary()}


def _msg(block, attr="error_message") -> str:
    e = block.body.attr(attr)
    if isinstance(e, Template):
        return e.literal() or "(dynamic message)"
    return ""


def _parse_cli_var(s: str):
    if "=" not in s:
        raise ValueError(f"--var expects NAME=VALUE, got {s!r}")
    k, v = s.split("=", 1)
    return k, v


def load_inputs(root: Path, var_files=(), cli_vars=(), ev: Evaluator | None = None) -> dict:
    ev = ev or Evaluator()
    empty = Scope({}, {})
    files = []
    if (root / "terraform.tfvars").exists():
        files.append(root / "terraform.tfvars")
    files += sorted(root.glob("*.auto.tfvars"))
    files += [Path(f) for f in var_files]
    values = {}
    for f in files:
        body = parse_file(f)
        for name, attr in body.attributes.items():
            values[name] = ev.eval(attr.expr, empty)
    for s in cli_vars:
        k, v = _parse_cli_var(s)
        values[k] = v          # strings; converted by the declared type later
    return values


def _instances(block, scope: Scope, ev: Evaluator, addr: str, res: PlanResult):
    """[(instance address, scope)] after count / for_each expansion."""
    count = block.body.attr("count")
    fe = block.body.attr("for_each")
    if count is not None:
        try:
            n = ev.eval(count, scope)
        except EvalError as x:
            res.errors.append(f"{addr}: invalid count argument: {x}")
            return []
        if n is UNKNOWN:
            res.errors.append(f"{addr}: Invalid count argument: the value depends on resource "
                              "attributes that cannot be determined until apply")
            return []
        try:
            n = int(n if not isinstance(n, bool) else int(n))
        except (TypeError, ValueError):
            res.errors.append(f"{addr}: count must be a whole number, got {n!r}")
            return []
        return [(f"{addr}[{i}]", scope.child(count={"index": i})) for i in range(n)]
    if fe is not None:
        try:
            v = ev.eval(fe, scope)
        except EvalError as x:
            res.errors.append(f"{addr}: invalid for_each argument: {x}")
            return []
        if is_unknown(v) if not isinstance(v, dict) else any(k is UNKNOWN for k in v):
            res.errors.append(f"{addr}: Invalid for_each argument: the keys depend on values "
                              "known only after apply")
            return []
        if isinstance(v, dict):
            items = list(v.items())
        elif isinstance(v, list):
            if not all(isinstance(x, str) for x in v):
                res.errors.append(f"{addr}: for_each over a list needs a set of strings (toset())")
                return []
            items = [(x, x) for x in v]
        else:
            res.errors.append(f"{addr}: for_each needs a map or set, got {type(v).__name__}")
            return []
        return [(f'{addr}["{k}"]', scope.child(each={"key": k, "value": val})) for k, val in items]
    return [(addr, scope)]


def _plan_module(mod: Module, inputs: dict, prefix: str, res: PlanResult, ev: Evaluator,
                 is_root: bool, depth: int = 0) -> None:
    if depth > 16:
        res.errors.append(f"{prefix}: module nesting too deep")
        return
    variables = {}
    empty = Scope({}, {})
    for name, v in mod.variables.items():
        where = f"{prefix}var.{name}"
        if name in inputs:
            val = inputs[name]
        elif not v.required:
            try:
                val = ev.eval(v.block.body.attr("default"), empty)
            except EvalError as x:
                res.errors.append(f"{where}: default cannot be evaluated: {x}")
                val = UNKNOWN
        else:
            what = "No value for required variable" if is_root else "Missing required argument"
            res.errors.append(f"{what} {where}")
            val = UNKNOWN
        try:
            val = convert(val, v.type_expr)
        except EvalError as x:
            res.errors.append(f"Invalid value for variable {where}: {x}")
        variables[name] = val
    for name in inputs:
        if name not in mod.variables and not is_root:
            res.errors.append(f"{prefix}: unsupported argument {name!r} (no such variable)")
        elif name not in mod.variables:
            res.warnings.append(f"value for undeclared variable {name!r} (ignored)")
    locals_exprs = {n: e for n, (e, _, _) in mod.locals.items()}
    scope = Scope(variables, locals_exprs, module_path=str(mod.path))

    # 1. variable validation blocks
    for name, v in mod.variables.items():
        for vb in v.validations:
            try:
                c = ev.eval(vb.body.attr("condition"), Scope(variables, {}, str(mod.path)))
            except EvalError as x:
                res.errors.append(f"{prefix}var.{name}: validation condition failed to evaluate: {x}")
                continue
            if c is False:
                res.errors.append(f"Invalid value for variable {prefix}var.{name}: {_msg(vb)}")

    # 2. resources and data sources
    for r in mod.resources.values():
        addr = prefix + r.address
        for inst, s in _instances(r.block, scope, ev, addr, res):
            (res.resources if r.mode == "managed" else res.data_sources).append(inst)
            for lc in r.block.body.blocks_of("lifecycle"):
                for pc in lc.body.blocks_of("precondition"):
                    try:
                        c = ev.eval(pc.body.attr("condition"), s)
                    except EvalError as x:
                        res.errors.append(f"{inst}: precondition failed to evaluate: {x}")
                        continue
                    if c is False:
                        res.errors.append(f"Resource precondition failed: {inst}: {_msg(pc)}")

    # 2b. output preconditions (Terraform checks them at plan time too)
    for name, o in mod.outputs.items():
        for pc in o.block.body.blocks_of("precondition"):
            try:
                c = ev.eval(pc.body.attr("condition"), scope)
            except EvalError as x:
                res.errors.append(f"{prefix}output.{name}: precondition failed to evaluate: {x}")
                continue
            if c is False:
                res.errors.append(f"Module output precondition failed: {prefix}output.{name}: "
                                  f"{_msg(pc)}")

    # 3. module calls
    for name, mc in mod.modules.items():
        addr = f"{prefix}module.{name}"
        for inst, s in _instances(mc.block, scope, ev, addr, res):
            if not mc.is_local:
                res.registry_modules.append(f"{inst} ({mc.source}{' ' + mc.version if mc.version else ''})")
                continue
            child = load_module((Path(mod.path) / mc.source).resolve())
            child_inputs = {}
            for an, attr in mc.block.body.attributes.items():
                if an in META_ARGS:
                    continue
                try:
                    child_inputs[an] = ev.eval(attr.expr, s)
                except EvalError as x:
                    res.errors.append(f"{inst}: argument {an!r}: {x}")
                    child_inputs[an] = UNKNOWN
            _plan_module(child, child_inputs, inst + ".", res, ev, is_root=False, depth=depth + 1)


def plan(root, var_files=(), cli_vars=()) -> PlanResult:
    root = Path(root)
    ev = Evaluator()
    res = PlanResult()
    try:
        inputs = load_inputs(root, var_files, cli_vars, ev)
    except (EvalError, ValueError) as x:
        res.errors.append(f"tfvars: {x}")
        return res
    _plan_module(load_module(root), inputs, "", res, ev, is_root=True)
    return res
