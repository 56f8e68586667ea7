"""Build the MI355X-native validation code (gfx950 only).

Outputs (all in-tree, so they travel to the GPU box with the repo snapshot):

* ``nvidia_terraform_modules_amd/ops/libntm_validation.so`` - K1/K2/K3 kernels
  behind a C ABI, loaded by :mod:`nvidia_terraform_modules_amd.ops._lib`.
* ``nvidia_terraform_modules_amd/ops/libntm_experimental.so`` - non-default
  K1 builds, schedule knobs and diagnostics (tests and tools only; never
  linked into the shipping library or the Job binary).
* ``validation/build/amdgpu-validate`` - the standalone validation-Job binary
  (HIP + RCCL, no Python/PyTorch in the container image).
* ``nvidia_terraform_modules_amd/ops/libntm_smi.so`` - host-only power /
  thermal / throttle sampler on libamd_smi (bench.py's per-rank telemetry).

The reference has no native code at all; this replaces the
CUDA ``vectorAdd`` validator that the NVIDIA GPU Operator chart ran
(``/root/reference/eks/main.tf:185-203``).
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from pathlib import Path

ARCH = "gfx950"
REPO = Path(__file__).resolve().parents[2]
VALIDATION = REPO / "validation"
INCLUDE = VALIDATION / "include"
SRC = VALIDATION / "src"
BUILD = VALIDATION / "build"
PKG_OPS = Path(__file__).resolve().parent
LIB_NAME = "libntm_validation.so"
EXP_LIB_NAME = "libntm_experimental.so"
# the shipping sources: the Job binary and libntm_validation.so link exactly these
SHIPPING_SRCS = ("ntm_validation.hip", "xgmi_allreduce.hip")
BIN_NAME = "amdgpu-validate"

COMMON_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"-I{INCLUDE}",
    "-Wall",
    "-Wno-unused-function",
]


def hipcc() -> str:
    exe = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(exe):
        raise RuntimeError("hipcc not found: the ROCm toolchain is required to build")
    return exe


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _deps() -> list[Path]:
    return sorted(INCLUDE.rglob("*.hpp")) + sorted(SRC.glob("*.hip")) + sorted(SRC.glob("*.cpp"))


def _build_so(name: str, srcs: list[Path], force: bool, verbose: bool) -> Path:
    out = PKG_OPS / name
    if force or _stale(out, _deps()):
        BUILD.mkdir(parents=True, exist_ok=True)
        tmp = BUILD / (name + ".tmp")
        _run([hipcc(), *COMMON_FLAGS, "-shared", *map(str, srcs), "-o", str(tmp)], verbose)
        os.replace(tmp, out)
    return out


def build_library(force: bool = False, verbose: bool = True) -> Path:
    return _build_so(LIB_NAME, [SRC / s for s in SHIPPING_SRCS], force, verbose)


def build_experimental(force: bool = False, verbose: bool = True) -> Path:
    return _build_so(EXP_LIB_NAME, [SRC / "ntm_experimental.hip"], force, verbose)


# Host-only AddressSanitizer / UBSan variant of the Job binary: instruments the
# host code (argument parsing, per-GPU threads, RCCL driver, JSON/report
# writers) and leaves the gfx950 device code untouched - GPU ASan / xnack+ code
# objects are not used. Each -fsanitize= sits directly after -Xarch_host.
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
              "-Xarch_host", "-fno-omit-frame-pointer", "-g"]


def build_binary(force: bool = False, verbose: bool = True, asan: bool = False) -> Path:
    out = BUILD / (BIN_NAME + ("-asan" if asan else ""))
    main = SRC / "validate_main.cpp"
    if not main.exists():
        return out
    if force or _stale(out, _deps()):
        BUILD.mkdir(parents=True, exist_ok=True)
        srcs = [str(SRC / s) for s in SHIPPING_SRCS]
        cmd = [
            hipcc(), *COMMON_FLAGS, *(ASAN_FLAGS if asan else []), "-x", "hip", str(main), *srcs,
            "-I/opt/rocm/include", "-L/opt/rocm/lib", "-lrccl", "-lpthread",
            "-Wl,-rpath,/opt/rocm/lib", "-o", str(out) + ".tmp",
        ]
        _run(cmd, verbose)
        os.replace(str(out) + ".tmp", out)
    return out


def build_exporter(force: bool = False, verbose: bool = True) -> Path:
    """amdgpu-exporter: host-only C++ on libamd_smi (no device code)."""
    out = BUILD / "amdgpu-exporter"
    src = SRC / "amdgpu_exporter.cpp"
    if not src.exists():
        return out
    if force or _stale(out, [src]):
        BUILD.mkdir(parents=True, exist_ok=True)
        cxx = shutil.which("g++") or "/opt/rocm/llvm/bin/clang++"
        cmd = [cxx, "-std=c++17", "-O2", "-Wall", "-I/opt/rocm/include", str(src),
               "-L/opt/rocm/lib", "-lamd_smi", "-Wl,-rpath,/opt/rocm/lib", "-o", str(out) + ".tmp"]
        _run(cmd, verbose)
        os.replace(str(out) + ".tmp", out)
    return out


SMI_LIB_NAME = "libntm_smi.so"


def build_smi(force: bool = False, verbose: bool = True) -> Path:
    """libntm_smi.so: host-only C++ on libamd_smi (power, temperature, clocks,
    throttle residencies of one GPU by PCI address; ops/smi.py)."""
    out = PKG_OPS / SMI_LIB_NAME
    src = SRC / "ntm_smi.cpp"
    if force or _stale(out, [src]):
        BUILD.mkdir(parents=True, exist_ok=True)
        tmp = BUILD / (SMI_LIB_NAME + ".tmp")
        cxx = shutil.which("g++") or "/opt/rocm/llvm/bin/clang++"
        _run([cxx, "-std=c++17", "-O2", "-Wall", "-fPIC", "-shared", "-I/opt/rocm/include",
              str(src), "-L/opt/rocm/lib", "-lamd_smi", "-Wl,-rpath,/opt/rocm/lib", "-o", str(tmp)],
             verbose)
        os.replace(tmp, out)
    return out


def build_all(force: bool = False, verbose: bool = True, asan: bool = False) -> dict[str, str]:
    lib = build_library(force=force, verbose=verbose)
    binary = build_binary(force=force, verbose=verbose)
    res = {"library": str(lib), "binary": str(binary),
           "experimental": str(build_experimental(force=force, verbose=verbose)),
           "exporter": str(build_exporter(force=force, verbose=verbose)),
           "smi": str(build_smi(force=force, verbose=verbose))}
    if asan:
        res["binary_asan"] = str(build_binary(force=force, verbose=verbose, asan=True))
    return res


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-q", "--quiet", action="store_true")
    ap.add_argument("--asan", action="store_true",
                    help="also build the host-ASan/UBSan amdgpu-validate-asan")
    args = ap.parse_args(argv)
    res = build_all(force=args.force, verbose=not args.quiet, asan=args.asan)
    for k, v in res.items():
        print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
