"""terraform-docs-style README sections, generated from the parsed modules.

The reference keeps its Requirements / Providers / Modules / Resources /
Inputs / Outputs tables as ``terraform-docs markdown .`` output pasted into
each README (reference CONTRIBUTING.md:14, eks/README.md:77-166), regenerated
by hand - and they drifted (eks/examples/cnpack/Readme.md:229 vs
variables.tf:56-60). Here the same tables are generated offline from the
tfcheck AST and a test (tests/test_docs.py) fails when a README is stale, so
the docs cannot drift.

    python -m nvidia_terraform_modules_amd.tfcheck --docs .         # rewrite
    python -m nvidia_terraform_modules_amd.tfcheck --docs-check .   # CI gate

The generated block lives between ``<!-- BEGIN_TF_DOCS -->`` and
``<!-- END_TF_DOCS -->`` (terraform-docs' own markers); text outside them is
hand-written and left alone.
"""
from __future__ import annotations

import json
from pathlib import Path

from .config import Module
from .hcl import (Call, Conditional, Directive, ForExpr, Literal, ObjectExpr, Postfix, Template,
                  Traversal, TupleExpr, BinOp, UnOp, key_name)

BEGIN = "<!-- BEGIN_TF_DOCS -->"
END = "<!-- END_TF_DOCS -->"


# ------------------------------------------------------------ expression text
def _ops(ops) -> str:
    out = ""
    for kind, v in ops:
        if kind == "attr":
            out += f".{v}"
        elif kind == "index":
            out += f"[{render(v)}]"
        elif kind == "splat":
            out += "[*]"
        else:
            out += ".*"
    return out


def _lit(v) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (int, float)):
        return str(v)
    return json.dumps(str(v))


def render(e) -> str:
    """HCL-ish source text of an expression (single line)."""
    if e is None:
        return ""
    if isinstance(e, Literal):
        return _lit(e.value)
    if isinstance(e, Template):
        s = ""
        for p in e.parts:
            if isinstance(p, str):
                s += p.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")
            elif isinstance(p, Directive):
                s += "%{" + p.kind + (" " + render(p.expr) if p.expr is not None else "") + "}"
            else:
                s += "${" + render(p) + "}"
        return f'"{s}"'
    if isinstance(e, Traversal):
        return e.root + _ops(e.ops)
    if isinstance(e, Postfix):
        return render(e.base) + _ops(e.ops)
    if isinstance(e, Call):
        args = ", ".join(render(a) for a in e.args)
        return f"{e.name}({args}{'...' if e.expand else ''})"
    if isinstance(e, TupleExpr):
        return "[" + ", ".join(render(i) for i in e.items) + "]"
    if isinstance(e, ObjectExpr):
        if not e.items:
            return "{}"
        parts = []
        for k, v in e.items:
            kn = key_name(k)
            parts.append(f"{kn if kn is not None else '(' + render(k) + ')'} = {render(v)}")
        return "{ " + ", ".join(parts) + " }"
    if isinstance(e, ForExpr):
        names = f"{e.key_var}, {e.val_var}" if e.key_var else e.val_var
        body = (f"{render(e.key_expr)} => {render(e.val_expr)}" if e.is_object
                else render(e.val_expr))
        cond = f" if {render(e.cond)}" if e.cond is not None else ""
        o, c = ("{", "}") if e.is_object else ("[", "]")
        return f"{o}for {names} in {render(e.coll)} : {body}{'...' if e.grouping else ''}{cond}{c}"
    if isinstance(e, Conditional):
        return f"{render(e.cond)} ? {render(e.true)} : {render(e.false)}"
    if isinstance(e, BinOp):
        return f"{render(e.left)} {e.op} {render(e.right)}"
    if isinstance(e, UnOp):
        return f"{e.op}{render(e.operand)}"
    return "<expr>"


# ---------------------------------------------------------------- the tables
def _cell(s: str) -> str:
    return s.replace("|", "\\|").replace("\n", " ").strip()


def _code(s: str) -> str:
    return f"`{_cell(s)}`" if s else "n/a"


def _desc(block) -> str:
    e = block.body.attr("description")
    if isinstance(e, Template):
        return e.literal() or render(e)
    return ""


def generate(mod: Module) -> str:
    """The markdown block (without markers) for one module."""
    out = []
    # Requirements
    out += ["## Requirements", "", "| Name | Version |", "|------|---------|"]
    if mod.required_version:
        out.append(f"| terraform | {_cell(mod.required_version)} |")
    for name in sorted(mod.required_providers):
        ver = (mod.required_providers[name] or {}).get("version") or "n/a"
        out.append(f"| {name} | {_cell(ver)} |")
    # Providers actually used by this module's resources / data sources
    used = sorted({r.provider_name for r in mod.resources.values()} - {"terraform"})
    out += ["", "## Providers", "", "| Name | Version |", "|------|---------|"]
    for name in used:
        ver = (mod.required_providers.get(name) or {}).get("version") or "n/a"
        out.append(f"| {name} | {_cell(ver)} |")
    # Modules
    out += ["", "## Modules", "", "| Name | Source | Version |", "|------|--------|---------|"]
    for name in sorted(mod.modules):
        m = mod.modules[name]
        out.append(f"| {name} | {_cell(m.source)} | {_cell(m.version or 'n/a')} |")
    # Resources
    out += ["", "## Resources", "", "| Name | Type |", "|------|------|"]
    for r in sorted(mod.resources.values(), key=lambda r: (r.mode != "managed", r.address)):
        kind = "resource" if r.mode == "managed" else "data source"
        out.append(f"| {r.address} | {kind} |")
    # Inputs
    out += ["", "## Inputs", "", "| Name | Description | Type | Default | Required |",
            "|------|-------------|------|---------|:--------:|"]
    for name in sorted(mod.variables):
        v = mod.variables[name]
        typ = render(v.type_expr) if v.type_expr is not None else "any"
        dflt = "n/a" if v.required else _code(render(v.block.body.attr("default")))
        out.append(f"| {name} | {_cell(v.description)} | {_code(typ)} | {dflt} | "
                   f"{'yes' if v.required else 'no'} |")
    # Outputs
    out += ["", "## Outputs", "", "| Name | Description |", "|------|-------------|"]
    for name in sorted(mod.outputs):
        o = mod.outputs[name]
        d = _desc(o.block)
        if o.sensitive:
            d = (d + " (sensitive)").strip()
        out.append(f"| {name} | {_cell(d)} |")
    return "\n".join(out) + "\n"


def readme_path(mod_dir: Path) -> Path:
    for n in ("README.md", "Readme.md", "readme.md"):
        if (mod_dir / n).exists():
            return mod_dir / n
    return mod_dir / "README.md"


def splice(text: str, block: str) -> str:
    """Replace (or append) the generated block in a README's text."""
    gen = f"{BEGIN}\n{block}{END}"
    if BEGIN in text and END in text:
        a = text.index(BEGIN)
        b = text.index(END) + len(END)
        return text[:a] + gen + text[b:]
    sep = "" if text.endswith("\n\n") or not text else ("\n" if text.endswith("\n") else "\n\n")
    return text + sep + gen + "\n"


def update(mod: Module, check: bool = False) -> bool:
    """Write (or, with check=True, only compare) the module's README block.
    Returns True when the README is (was) up to date."""
    p = readme_path(Path(mod.path))
    old = p.read_text() if p.exists() else ""
    new = splice(old, generate(mod))
    if new == old:
        return True
    if not check:
        p.write_text(new)
    return False
