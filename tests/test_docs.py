"""README tables are generated from the code and must not drift (the
reference's did: SURVEY.md §4)."""
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.tfcheck.config import find_modules, load_module
from nvidia_terraform_modules_amd.tfcheck.docs import BEGIN, END, generate, render, splice, update
from nvidia_terraform_modules_amd.tfcheck.hcl import parse_file

ROOT = Path(__file__).resolve().parents[1]
MODULE_DIRS = [m for m in find_modules(ROOT)
               if not any(p in ("charts", "fixtures") for p in m.parts)]


@pytest.mark.parametrize("mdir", MODULE_DIRS, ids=lambda p: str(p.relative_to(ROOT)))
def test_readme_tables_are_current(mdir):
    assert update(load_module(mdir), check=True), \
        f"stale README in {mdir}: run python -m nvidia_terraform_modules_amd.tfcheck --docs ."


def test_every_variable_and_output_documented():
    for mdir in MODULE_DIRS:
        mod = load_module(mdir)
        text = generate(mod)
        for v in mod.variables:
            assert f"| {v} |" in text
        for o in mod.outputs:
            assert f"| {o} |" in text


def test_splice_keeps_hand_written_text():
    old = f"# Title\n\nintro\n\n{BEGIN}\nold table\n{END}\n\nfooter\n"
    new = splice(old, "new table\n")
    assert new.startswith("# Title\n\nintro\n\n") and new.endswith("\n\nfooter\n")
    assert "new table" in new and "old table" not in new
    assert splice("# T\n", "x\n").endswith(f"{BEGIN}\nx\n{END}\n")


def test_render_round_trips_common_expressions(tmp_path):
    src = '''variable "v" {
  type = object({ a = string, b = list(number) })
  default = { a = "x", b = [1, 2] }
}
locals {
  c = var.x ? [for k, v in var.m : "${k}=${v}" if v != null] : null
  d = merge(local.a, { "k" = 1 })[0].name
}
'''
    f = tmp_path / "main.tf"
    f.write_text(src)
    body = parse_file(str(f))
    v = body.blocks[0].body
    assert render(v.attr("type")) == "object({ a = string, b = list(number) })"
    assert render(v.attr("default")) == '{ a = "x", b = [1, 2] }'
    loc = body.blocks[1].body
    assert render(loc.attr("c")) == 'var.x ? [for k, v in var.m : "${k}=${v}" if v != null] : null'
    assert render(loc.attr("d")) == 'merge(local.a, { k = 1 })[0].name'


def test_standing_summary_reproduces_the_committed_round5_standing():
    """tools/standing_summary.py over profiles/r5_standing (box<X>_*.log) gives
    exactly the committed summary.jsonl."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    out = subprocess.run([sys.executable, str(root / "tools" / "standing_summary.py"),
                          str(root / "profiles" / "r5_standing")],
                         capture_output=True, text=True, check=True).stdout
    want = (root / "profiles" / "r5_standing" / "summary.jsonl").read_text()
    assert sorted(out.splitlines()) == sorted(want.splitlines())
