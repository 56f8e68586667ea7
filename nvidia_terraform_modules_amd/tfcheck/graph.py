"""Dependency graph of a root module, with local child modules flattened.

Nodes are resource/data addresses (``module.amd_gpu_stack.kubernetes_job_v1.
gpu_validation``), module-call nodes (``module.eks``) for REMOTE modules
(their internals are unknown offline), and ``provider.<name>`` nodes.
Variables, locals and outputs are resolved through, so an edge A -> B means
"A needs B to exist first" exactly as Terraform's graph would order them
(implicit references + depends_on + provider configuration).

Used for: ordering guarantees (validation Job after the GPU node pool; the
operator after the pool; no cycles) and the critical-path model in
:mod:`nvidia_terraform_modules_amd.gpu_ready.critical_path`.
"""
from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass, field
from pathlib import Path

from .analysis import module_exprs
from .config import Module, load_module
from .hcl import Traversal, walk_refs


@dataclass
class Graph:
    nodes: dict = field(default_factory=dict)                 # address -> kind
    edges: dict = field(default_factory=lambda: defaultdict(set))  # a -> {deps}

    def add(self, addr: str, kind: str) -> None:
        self.nodes.setdefault(addr, kind)

    def dep(self, a: str, b: str) -> None:
        if a != b:
            self.edges[a].add(b)

    def deps(self, a: str) -> set:
        return self.edges.get(a, set())

    def ancestors(self, a: str) -> set:
        """Everything ``a`` (transitively) depends on."""
        seen, stack = set(), [a]
        while stack:
            for d in self.deps(stack.pop()):
                if d not in seen:
                    seen.add(d)
                    stack.append(d)
        return seen

    def depends_on(self, a: str, b: str) -> bool:
        return b in self.ancestors(a)

    def find(self, suffix: str) -> list[str]:
        return sorted(n for n in self.nodes if n == suffix or n.endswith("." + suffix) or n.endswith(suffix))

    def cycles(self) -> list[list[str]]:
        color: dict = {}
        out = []

        def visit(n, path):
            color[n] = 1
            for d in sorted(self.deps(n)):
                if color.get(d) == 1:
                    out.append(path[path.index(d):] + [d] if d in path else [n, d])
                elif color.get(d) is None:
                    visit(d, path + [d])
            color[n] = 2

        for n in sorted(self.nodes):
            if color.get(n) is None:
                visit(n, [n])
        return out

    def hard_cycles(self) -> list[list[str]]:
        """Cycles that Terraform would reject. Cycles made only of REMOTE
        module-call nodes are not: Terraform orders module internals per
        value (e.g. eks <-> its IRSA role module, reference eks/main.tf:135,151)."""
        return [c for c in self.cycles() if any(self.nodes.get(n) != "module" for n in c)]

    def topo_order(self) -> list[str]:
        order, seen = [], set()

        def visit(n):
            if n in seen:
                return
            seen.add(n)
            for d in sorted(self.deps(n)):
                visit(d)
            order.append(n)

        for n in sorted(self.nodes):
            visit(n)
        return order


class _Builder:
    def __init__(self):
        self.g = Graph()

    def build(self, mod: Module, prefix: str = "", inputs: dict | None = None) -> dict:
        """Add ``mod``'s objects under ``prefix``; returns {output_name: set(deps)}.

        ``inputs`` maps variable name -> set of graph nodes its value depends on.
        """
        inputs = inputs or {}
        p = prefix
        local_deps: dict = {}
        child_outputs: dict = {}
        providers_by_name = {}

        for pb in mod.providers:
            name = pb.labels[0]
            alias = pb.body.attr("alias")
            key = f"{p}provider.{name}"
            if isinstance(alias, Traversal):
                pass
            providers_by_name[name] = key
            self.g.add(key, "provider")

        # resources / data first (nodes), so references can resolve
        for r in mod.resources.values():
            self.g.add(p + r.address, r.mode)
        for name, mc in mod.modules.items():
            if not mc.is_local:
                self.g.add(f"{p}module.{name}", "module")

        # resolve a reference traversal to graph nodes
        def resolve(ref: Traversal, stack=()) -> set:
            root, path = ref.root, ref.path()
            if root == "var" and path:
                return set(inputs.get(path[0], set()))
            if root == "local" and path:
                if path[0] in stack:
                    return set()
                if path[0] not in local_deps:
                    expr = mod.locals.get(path[0], (None,))[0]
                    local_deps[path[0]] = expr_deps(expr, stack + (path[0],))
                return set(local_deps[path[0]])
            if root == "data" and len(path) >= 2:
                a = f"{p}data.{path[0]}.{path[1]}"
                return {a} if a in self.g.nodes else set()
            if root == "module" and path:
                name = path[0]
                if name in child_outputs:
                    outs = child_outputs[name]
                    if len(path) > 1 and path[1] in outs:
                        return set(outs[path[1]])
                    return set().union(*outs.values()) if outs else set()
                a = f"{p}module.{name}"
                return {a} if a in self.g.nodes else set()
            if path:
                a = f"{p}{root}.{path[0]}"
                if a in self.g.nodes:
                    return {a}
            return set()

        def expr_deps(expr, stack=()) -> set:
            out = set()
            for ref, bound in walk_refs(expr):
                if ref.root in bound:
                    continue
                out |= resolve(ref, stack)
            return out

        # child modules (local) are built recursively with their input deps
        for name, mc in mod.modules.items():
            meta = {"source", "version", "count", "for_each", "providers", "depends_on"}
            explicit = set()
            dep_expr = mc.block.body.attr("depends_on")
            if dep_expr is not None:
                explicit = expr_deps(dep_expr)
            if mc.is_local:
                child = load_module((mod.path / mc.source).resolve())
                child_inputs = {}
                for an, attr in mc.block.body.attributes.items():
                    if an in meta:
                        continue
                    child_inputs[an] = expr_deps(attr.expr) | explicit
                # variables not passed still inherit the module-level depends_on
                for vn in child.variables:
                    child_inputs.setdefault(vn, set(explicit))
                before = set(self.g.nodes)
                child_outputs[name] = self.build(child, f"{p}module.{name}.", child_inputs)
                # every object of the child honours the call's depends_on and
                # the parent's provider configurations
                for n in set(self.g.nodes) - before:
                    for d in explicit:
                        self.g.dep(n, d)
            else:
                a = f"{p}module.{name}"
                for an, attr in mc.block.body.attributes.items():
                    if an in ("source", "version"):
                        continue
                    for d in expr_deps(attr.expr):
                        self.g.dep(a, d)

        # provider configuration edges
        for pb in mod.providers:
            key = f"{p}provider.{pb.labels[0]}"
            for an, attr in pb.body.attributes.items():
                for d in expr_deps(attr.expr):
                    self.g.dep(key, d)
            for b in pb.body.blocks:
                stack = [b]
                while stack:
                    blk = stack.pop()
                    for an, attr in blk.body.attributes.items():
                        for d in expr_deps(attr.expr):
                            self.g.dep(key, d)
                    stack.extend(blk.body.blocks)

        # resource / data edges
        for expr, scope, where, attr, owner in module_exprs(mod):
            if owner in ("output", "locals", "provider", "check") or owner.startswith("var."):
                continue
            node = p + owner if not owner.startswith("module.") else None
            if owner.startswith("module."):
                continue  # handled above
            if node not in self.g.nodes:
                continue
            for d in expr_deps(expr):
                self.g.dep(node, d)
        for r in mod.resources.values():
            node = p + r.address
            prov = r.provider_name
            pnode = providers_by_name.get(prov)
            if pnode is None:
                # provider configured by an ancestor module
                for anc in self._provider_scopes(p):
                    cand = f"{anc}provider.{prov}"
                    if cand in self.g.nodes:
                        pnode = cand
                        break
            if pnode:
                self.g.dep(node, pnode)
            for d in set().union(*inputs.values()) if False else set():
                self.g.dep(node, d)

        outputs = {}
        for oname, o in mod.outputs.items():
            outputs[oname] = expr_deps(o.value)
        return outputs

    @staticmethod
    def _provider_scopes(prefix: str) -> list[str]:
        parts = prefix.split("module.")
        scopes = []
        acc = ""
        for i, part in enumerate(parts):
            acc = acc + ("module." if i else "") + part
            scopes.append(acc)
        return list(reversed(scopes[:-1])) + [""]


def build_graph(path: str | Path) -> Graph:
    b = _Builder()
    b.build(load_module(path))
    return b.g
