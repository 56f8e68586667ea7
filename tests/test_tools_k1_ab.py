"""tools/k1_ab.py (the one K1 plan A/B harness): its CLI and the
host-side pieces, on CPU. The timed paths need a GPU and are developer tools."""
import importlib.util
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _mod():
    spec = importlib.util.spec_from_file_location("k1_ab", ROOT / "tools" / "k1_ab.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_subcommands_parse():
    m = _mod()
    p = m.build_parser()
    a = p.parse_args(["ragged", "--n", "3", "--seed", "23", "--candidates"])
    assert a.cmd == "ragged" and a.n == 3 and a.candidates
    a = p.parse_args(["plan", "--cases", "3072x3072x3072=3072:pingpong8c:tile128"])
    assert list(m._cases(a.cases)) == [((3072, 3072, 3072), (3072, "pingpong8c", "tile128", 1),
                                       "3072:pingpong8c:tile128")]
    a = p.parse_args(["margin", "--dtype", "fp8", "--ragged"])
    assert a.n == 3000 and a.old_margin == 1.1 and a.ragged
    assert p.parse_args(["pp-tiles", "--split-only"]).seed == 11
    with pytest.raises(SystemExit):
        p.parse_args([])


def test_ragged_shapes_are_seeded_one_round_and_ragged():
    m = _mod()
    s = m.ragged_shapes(40, 5)
    assert s == m.ragged_shapes(40, 5) and s != m.ragged_shapes(40, 6)
    for mm, nn, k in s:
        tiles = ((mm + 255) // 256) * ((nn + 255) // 256)
        assert 0.3 * 256 < tiles <= 256 and not (mm % 256 == 0 and nn % 256 == 0)
        assert mm % 8 == nn % 8 == k % 8 == 0 and 1024 <= k <= 16384
    assert all(x % 16 == 0 for sh in m.uniform_shapes(20, 1, 16) for x in sh)
    assert m.parse_shapes("8x16x32,64x64x64") == [(8, 16, 32), (64, 64, 64)]


def test_every_tool_script_compiles_and_indexes():
    """Every script under tools/ at least byte-compiles (no silent rot in the
    developer tools), and every experiment is indexed in tools/README.md."""
    import py_compile

    scripts = sorted((ROOT / "tools").rglob("*.py"))
    assert len(scripts) > 20
    for f in scripts:
        py_compile.compile(str(f), doraise=True, cfile=None)
    index = (ROOT / "tools" / "README.md").read_text()
    missing = [f.name for f in (ROOT / "tools" / "experiments").glob("*.py")
               if f"`{f.name}`" not in index]
    assert not missing, f"not in tools/README.md: {missing}"
