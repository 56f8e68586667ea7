"""Call-surface contract: variable names (+ required-ness) and output names of
each module must be a superset of the reference module's surface, so a user of
``nvidia-terraform-modules`` can switch ``source =`` and keep every argument.

The expected surface is extracted from the reference by this same parser and
frozen in ``tests/fixtures/reference_surface.json`` (see :func:`extract`), so
the contract test runs without /root/reference.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path

from .config import load_module

# reference module dir -> this repo's module dir
MODULE_MAP = {
    "eks": "eks",
    "gke": "gke",
    "aks": "aks",
    "eks/examples/cnpack": "eks/examples/cnpack",
    "gke/examples/cnpack": "gke/examples/cnpack",
    "aks/examples/cnpack": "aks/examples/cnpack",
}


@dataclass
class Surface:
    variables: dict      # name -> {"required": bool}
    outputs: list
    tfvars_keys: list    # keys set (uncommented) in terraform.tfvars

    def as_dict(self) -> dict:
        return {"variables": self.variables, "outputs": self.outputs, "tfvars_keys": self.tfvars_keys}


def surface_of(path: str | Path) -> Surface:
    m = load_module(path)
    tfv = m.tfvars.get("terraform.tfvars")
    return Surface(
        variables={n: {"required": v.required} for n, v in sorted(m.variables.items())},
        outputs=sorted(m.outputs),
        tfvars_keys=sorted(tfv.attributes) if tfv else [],
    )


def extract(reference_root: str | Path) -> dict:
    root = Path(reference_root)
    return {rel: surface_of(root / rel).as_dict() for rel in MODULE_MAP}


@dataclass
class ContractDiff:
    module: str
    missing_variables: list
    required_mismatch: list   # (name, ref_required, ours_required)
    missing_outputs: list
    tfvars_unknown: list      # keys in the reference tfvars that our module has no variable for

    @property
    def ok(self) -> bool:
        return not (self.missing_variables or self.required_mismatch or self.missing_outputs
                    or self.tfvars_unknown)


def compare(expected: dict, repo_root: str | Path) -> list[ContractDiff]:
    out = []
    for rel, ours_rel in MODULE_MAP.items():
        exp = expected[rel]
        ours = surface_of(Path(repo_root) / ours_rel)
        missing_v = sorted(set(exp["variables"]) - set(ours.variables))
        mism = []
        for n, spec in exp["variables"].items():
            if n in ours.variables and spec["required"] != ours.variables[n]["required"]:
                # making a reference-required variable optional never breaks a caller;
                # only optional -> required does.
                if not spec["required"] and ours.variables[n]["required"]:
                    mism.append((n, spec["required"], ours.variables[n]["required"]))
        missing_o = sorted(set(exp["outputs"]) - set(ours.outputs))
        tfv = sorted(k for k in exp["tfvars_keys"] if k not in ours.variables)
        out.append(ContractDiff(rel, missing_v, mism, missing_o, tfv))
    return out


def load_expected(path: str | Path) -> dict:
    return json.loads(Path(path).read_text())
