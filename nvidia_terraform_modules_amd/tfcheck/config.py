"""Terraform module model built from parsed .tf files (one directory = one module)."""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

from .hcl import Block, Body, Expr, Literal, Template, Traversal, evaluate_static, parse_file


@dataclass
class Variable:
    name: str
    block: Block
    file: str

    @property
    def required(self) -> bool:
        return "default" not in self.block.body.attributes

    @property
    def default(self):
        e = self.block.body.attr("default")
        if e is None:
            return None
        try:
            return evaluate_static(e)
        except ValueError:
            return e

    @property
    def type_expr(self) -> Expr | None:
        return self.block.body.attr("type")

    @property
    def description(self) -> str:
        e = self.block.body.attr("description")
        if isinstance(e, Template):
            return e.literal() or ""
        return ""

    @property
    def sensitive(self) -> bool:
        e = self.block.body.attr("sensitive")
        return isinstance(e, Literal) and e.value is True

    @property
    def validations(self) -> list[Block]:
        return self.block.body.blocks_of("validation")


@dataclass
class Output:
    name: str
    block: Block
    file: str

    @property
    def sensitive(self) -> bool:
        e = self.block.body.attr("sensitive")
        return isinstance(e, Literal) and e.value is True

    @property
    def value(self) -> Expr | None:
        return self.block.body.attr("value")


@dataclass
class Resource:
    mode: str          # "managed" | "data"
    type: str
    name: str
    block: Block
    file: str

    @property
    def address(self) -> str:
        return f"{self.type}.{self.name}" if self.mode == "managed" else f"data.{self.type}.{self.name}"

    @property
    def provider_name(self) -> str:
        e = self.block.body.attr("provider")
        if isinstance(e, Traversal):
            return e.root
        return provider_of_type(self.type)


@dataclass
class ModuleCall:
    name: str
    block: Block
    file: str

    @property
    def source(self) -> str:
        e = self.block.body.attr("source")
        return e.literal() if isinstance(e, Template) else ""

    @property
    def version(self) -> str | None:
        e = self.block.body.attr("version")
        return e.literal() if isinstance(e, Template) else None

    @property
    def is_local(self) -> bool:
        return self.source.startswith("./") or self.source.startswith("../")


@dataclass
class Module:
    path: Path
    files: dict = field(default_factory=dict)            # filename -> Body
    variables: dict = field(default_factory=dict)
    outputs: dict = field(default_factory=dict)
    locals: dict = field(default_factory=dict)           # name -> (Expr, file, line)
    resources: dict = field(default_factory=dict)        # address -> Resource
    modules: dict = field(default_factory=dict)
    providers: list = field(default_factory=list)        # Block
    required_providers: dict = field(default_factory=dict)  # local name -> {source, version}
    required_version: str | None = None
    checks: list = field(default_factory=list)
    moved: list = field(default_factory=list)            # (Block, file) of moved blocks
    removed: list = field(default_factory=list)          # (Block, file) of removed blocks
    imports: list = field(default_factory=list)          # (Block, file) of import blocks
    tfvars: dict = field(default_factory=dict)           # filename -> Body
    errors: list = field(default_factory=list)

    @property
    def managed(self) -> list[Resource]:
        return [r for r in self.resources.values() if r.mode == "managed"]

    @property
    def data(self) -> list[Resource]:
        return [r for r in self.resources.values() if r.mode == "data"]


def provider_of_type(rtype: str) -> str:
    if rtype == "terraform_data":
        return "terraform"
    return rtype.split("_", 1)[0]


def load_module(path: str | Path) -> Module:
    """Parse every ``*.tf`` (and ``*.tfvars``) in a directory (not recursive)."""
    path = Path(path)
    mod = Module(path=path)
    for f in sorted(path.glob("*.tf")):
        body = parse_file(f)
        mod.files[f.name] = body
        _index(mod, body, f.name)
    for f in sorted(path.glob("*.tfvars")):
        mod.tfvars[f.name] = parse_file(f)
    return mod


def _dup(mod: Module, kind: str, name: str, file: str, line: int) -> None:
    mod.errors.append(f"{file}:{line}: duplicate {kind} {name!r}")


def _index(mod: Module, body: Body, fname: str) -> None:
    for b in body.blocks:
        if b.type == "variable":
            n = b.labels[0]
            if n in mod.variables:
                _dup(mod, "variable", n, fname, b.line)
            mod.variables[n] = Variable(n, b, fname)
        elif b.type == "output":
            n = b.labels[0]
            if n in mod.outputs:
                _dup(mod, "output", n, fname, b.line)
            mod.outputs[n] = Output(n, b, fname)
        elif b.type == "locals":
            for name, attr in b.body.attributes.items():
                if name in mod.locals:
                    _dup(mod, "local", name, fname, attr.line)
                mod.locals[name] = (attr.expr, fname, attr.line)
        elif b.type in ("resource", "data"):
            mode = "managed" if b.type == "resource" else "data"
            r = Resource(mode, b.labels[0], b.labels[1], b, fname)
            if r.address in mod.resources:
                _dup(mod, b.type, r.address, fname, b.line)
            mod.resources[r.address] = r
        elif b.type == "module":
            n = b.labels[0]
            if n in mod.modules:
                _dup(mod, "module", n, fname, b.line)
            mod.modules[n] = ModuleCall(n, b, fname)
        elif b.type == "provider":
            mod.providers.append(b)
        elif b.type == "terraform":
            rv = b.body.attr("required_version")
            if isinstance(rv, Template):
                mod.required_version = rv.literal()
            for rp in b.body.blocks_of("required_providers"):
                for pname, attr in rp.body.attributes.items():
                    try:
                        spec = evaluate_static(attr.expr)
                    except ValueError:
                        spec = {}
                    if isinstance(spec, str):
                        spec = {"version": spec}
                    mod.required_providers[pname] = spec
        elif b.type == "check":
            mod.checks.append(b)
        elif b.type == "moved":
            mod.moved.append((b, fname))
        elif b.type == "removed":
            mod.removed.append((b, fname))
        elif b.type == "import":
            mod.imports.append((b, fname))
        else:
            mod.errors.append(f"{fname}:{b.line}: unknown top-level block {b.type!r}")


def find_modules(root: str | Path) -> list[Path]:
    """Every directory under ``root`` holding at least one ``*.tf`` file."""
    root = Path(root)
    dirs = sorted({p.parent for p in root.rglob("*.tf") if ".terraform" not in p.parts})
    return dirs
