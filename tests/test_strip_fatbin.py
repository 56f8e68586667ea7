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
