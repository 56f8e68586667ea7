"""validation/image/strip-fatbin.py (the validation image keeps only gfx950
device code in vendor libraries, librccl.so above all): on CPU, a two-target
HIP shared library built here is cut to gfx950 in place - ELF layout and file
size unchanged, the section's bundle lists host + gfx950 only, a second run is
a no-op. The runtime side (RCCL from the cut library, all-reduce verified) was
measured on MI355X: profiles/r5_fatbin."""
import importlib.util
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"


def _mod():
    spec = importlib.util.spec_from_file_location("strip_fatbin",
                                                  ROOT / "validation/image/strip-fatbin.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(BUNDLER)), reason="no ROCm toolchain")
def test_two_target_library_is_cut_to_gfx950(tmp_path):
    src = tmp_path / "k.hip"
    src.write_text('#include <hip/hip_runtime.h>\n'
                   '__global__ void k(float* x) { x[threadIdx.x] *= 2.0f; }\n'
                   'extern "C" int launch(float* x) { hipLaunchKernelGGL(k, 1, 64, 0, 0, x); return 0; }\n')
    lib = tmp_path / "libk.so"
    subprocess.run([HIPCC, "-shared", "-fPIC", "-O2", "--offload-arch=gfx942", "--offload-arch=gfx950",
                    str(src), "-o", str(lib)], check=True, capture_output=True)
    m = _mod()
    size0 = lib.stat().st_size
    off, sec = m.section(str(lib))
    res = m.strip(str(lib), "gfx950", BUNDLER)
    assert res["changed"] is True and res["dropped_targets"] == 1, res
    assert res["kept"][-1].endswith("--gfx950") and res["bundle_bytes"] <= sec
    assert lib.stat().st_size == size0 and m.section(str(lib)) == (off, sec)
    data = lib.read_bytes()[off:off + sec]
    n = m.bundle_bytes(data)
    assert data[:4] == b"CCOB" and n == res["bundle_bytes"] and not any(data[n:])
    cut = tmp_path / "cut.bin"
    cut.write_bytes(data[:n])
    tg = m.targets(BUNDLER, str(cut))
    assert len(tg) == 2 and any(t.endswith("--gfx950") for t in tg) and any(t.startswith("host-") for t in tg)
    # idempotent: the zero tail is not part of the bundle
    again = m.strip(str(lib), "gfx950", BUNDLER)
    assert again["changed"] is False and "no other target" in again["reason"]
    # a host-only library has no section and is left alone
    host = tmp_path / "libh.so"
    shutil.copy("/usr/lib/x86_64-linux-gnu/libz.so.1" if os.path.exists(
        "/usr/lib/x86_64-linux-gnu/libz.so.1") else lib, host)
    if host.read_bytes() != lib.read_bytes():
        assert m.strip(str(host), "gfx950", BUNDLER)["changed"] is False


def test_bundle_length_from_the_compressed_header():
    m = _mod()
    import struct

    v3 = b"CCOB" + struct.pack("<HH", 3, 1) + struct.pack("<Q", 40) + bytes(100)
    v2 = b"CCOB" + struct.pack("<HH", 2, 1) + struct.pack("<I", 24) + bytes(100)
    assert m.bundle_bytes(v3) == 40 and m.bundle_bytes(v2) == 24
    assert m.bundle_bytes(b"__CLANG_OFFLOAD_BUNDLE__" + bytes(8)) == 32


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(BUNDLER)), reason="no ROCm toolchain")
def test_two_source_files_two_bundles_both_cut(tmp_path):
    """a library compiled WITHOUT -fgpu-rdc has one bundle per source
    file in .hip_fatbin. Each must be cut at its own offset - cutting only the
    first and zero-filling the rest would drop the second file's device code."""
    srcs = []
    for name, body in (("a", "x[threadIdx.x] *= 2.0f;"), ("b", "x[threadIdx.x] += 3.0f;")):
        p = tmp_path / f"{name}.hip"
        p.write_text('#include <hip/hip_runtime.h>\n'
                     f'__global__ void k{name}(float* x) {{ {body} }}\n'
                     f'extern "C" int l{name}(float* x) {{ hipLaunchKernelGGL(k{name}, 1, 64, 0, 0, x); '
                     'return 0; }\n')
        srcs.append(str(p))
    lib = tmp_path / "lib2.so"
    subprocess.run([HIPCC, "-shared", "-fPIC", "-O2", "--offload-arch=gfx942", "--offload-arch=gfx950",
                    *srcs, "-o", str(lib)], check=True, capture_output=True)
    m = _mod()
    off, sec = m.section(str(lib))
    before = m.bundles(lib.read_bytes()[off:off + sec])
    assert len(before) == 2 and before[0][0] == 0 and before[1][0] > before[0][1]
    res = m.strip(str(lib), "gfx950", BUNDLER)
    assert res["changed"] and res["bundles"] == 2 and res["rewritten_bundles"] == 2, res
    data = lib.read_bytes()[off:off + sec]
    after = m.bundles(data)
    assert [b0 for b0, _ in after] == [b0 for b0, _ in before]      # each at its own offset
    for i, (b0, n) in enumerate(after):
        assert data[b0:b0 + 4] == b"CCOB"
        cut = tmp_path / f"cut{i}.bin"
        cut.write_bytes(data[b0:b0 + n])
        tg = m.targets(BUNDLER, str(cut))
        assert len(tg) == 2 and any(t.endswith("--gfx950") for t in tg), tg
        # that file's own kernel is still in its gfx950 code object
        obj = tmp_path / f"obj{i}.o"
        gfx = next(t for t in tg if t.endswith("--gfx950"))
        subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={cut}", f"--targets={gfx}",
                        f"--output={obj}"], check=True)
        assert (b"ka" if i == 0 else b"kb") in obj.read_bytes()
    assert m.strip(str(lib), "gfx950", BUNDLER)["changed"] is False      # idempotent


def test_bundles_rejects_unknown_bytes_between_bundles():
    m = _mod()
    import struct

    one = b"CCOB" + struct.pack("<HH", 3, 1) + struct.pack("<Q", 24) + bytes(8)
    assert m.bundles(one + bytes(40) + one) == [(0, 24), (64, 24)]
    with pytest.raises(ValueError, match="between bundles"):
        m.bundles(one + b"\x01" + bytes(39) + one)
    unc = m.MAGIC + struct.pack("<Q", 1) + struct.pack("<QQQ", 64, 16, 4) + b"host" + bytes(64)
    assert m.bundle_bytes(unc) == 80
