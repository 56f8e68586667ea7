"""HCL2 parser: reference modules + syntax edge cases."""
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.tfcheck.config import find_modules, load_module
from nvidia_terraform_modules_amd.tfcheck.hcl import (
    Call, Conditional, ForExpr, Literal, ObjectExpr, Template, Traversal, TupleExpr,
    evaluate_static, parse, parse_expression, walk_refs,
)
from nvidia_terraform_modules_amd.tfcheck.lexer import HCLSyntaxError

REF = Path("/root/reference")


@pytest.mark.skipif(not REF.exists(), reason="reference not mounted")
def test_reference_modules_parse_with_survey_counts():
    counts = {}
    for d in find_modules(REF):
        m = load_module(d)
        assert not m.errors
        counts[str(d.relative_to(REF))] = (len(m.variables), len(m.outputs))
    # EKS 36 vars, GKE 25, AKS 18; outputs 11 / 10 / 5
    assert counts["eks"] == (36, 11)
    assert counts["gke"] == (25, 10)
    assert counts["aks"] == (18, 5)


def test_repo_modules_parse(repo):
    mods = [d for d in find_modules(repo) if "charts" not in d.parts]
    names = {str(d.relative_to(repo)) for d in mods}
    assert {"eks", "gke", "aks", "modules/amd-gpu-stack", "eks/examples/cnpack",
            "gke/examples/cnpack", "aks/examples/cnpack"} <= names
    for d in mods:
        assert not load_module(d).errors


def test_blocks_labels_attributes():
    b = parse('resource "aws_x" "y" {\n  a = 1\n  nested {\n    b = "s"\n  }\n}\n')
    (blk,) = b.blocks
    assert blk.type == "resource" and blk.labels == ["aws_x", "y"]
    assert isinstance(blk.body.attr("a"), Literal)
    assert blk.body.blocks[0].body.attr("b").literal() == "s"


def test_single_line_block_and_comments():
    b = parse('# c1\n// c2\n/* multi\nline */\nlocals { x = 1 }\nvariable "v" {}\n')
    assert [x.type for x in b.blocks] == ["locals", "variable"]


def test_template_interpolation_and_escape():
    e = parse_expression('"a-${var.x}-$${literal}-%%{lit}"')
    assert isinstance(e, Template)
    refs = [r.root + "." + ".".join(r.path()) for r, _ in walk_refs(e)]
    assert refs == ["var.x"]
    assert "${literal}" in "".join(p for p in e.parts if isinstance(p, str))


def test_heredoc_indent_and_directives():
    src = 'x = <<-EOT\n    hello ${local.a}\n    %{ for n in var.list ~}\n    ${n}\n    %{ endfor ~}\n  EOT\n'
    b = parse(src)
    e = b.attr("x")
    roots = sorted(r.root for r, bound in walk_refs(e) if r.root not in bound)
    assert roots == ["local", "var"]


def test_operators_precedence_and_conditional():
    e = parse_expression("a.b + 2 * 3 == 7 && !c ? [1, 2] : {k = v}")
    assert isinstance(e, Conditional)
    assert isinstance(e.true, TupleExpr) and isinstance(e.false, ObjectExpr)


def test_for_expressions_bind_names():
    e = parse_expression("{for k, v in var.m : k => upper(v) if v != local.skip}")
    assert isinstance(e, ForExpr) and e.is_object
    free = sorted(r.root for r, bound in walk_refs(e) if r.root not in bound)
    assert free == ["local", "var"]


def test_splats_and_index():
    e = parse_expression("module.vpc[*].private_subnets[0]")
    assert isinstance(e, Traversal)
    assert e.root == "module" and e.path() == ["vpc"]
    e2 = parse_expression("google_container_cluster.c.master_auth.0.ca")
    assert e2.path() == ["c", "master_auth", "0", "ca"]


def test_function_call_expansion():
    e = parse_expression("merge(local.a, var.list...)")
    assert isinstance(e, Call) and e.expand and len(e.args) == 2


def test_multiline_collections():
    b = parse('x = [\n  "a",\n  "b",\n]\ny = {\n  k1 = 1\n  k2 = 2\n}\n')
    assert evaluate_static(b.attr("x")) == ["a", "b"]
    assert evaluate_static(b.attr("y")) == {"k1": 1, "k2": 2}


def test_paren_object_keys_are_references():
    e = parse_expression("{ (local.k) = 1, plain = 2 }")
    roots = [r.root for r, _ in walk_refs(e)]
    assert roots == ["local"]


def test_syntax_errors_report_line():
    with pytest.raises(HCLSyntaxError) as ei:
        parse('a = 1\nb = [1, 2\nc = 3\n', "f.tf")
    assert "f.tf" in str(ei.value)
    with pytest.raises(HCLSyntaxError):
        parse('x = "unterminated\n')
    with pytest.raises(HCLSyntaxError):
        parse("a = 1 b = 2\n")
