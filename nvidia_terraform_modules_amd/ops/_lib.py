"""ctypes binding to ``libntm_validation.so`` (the gfx950 HIP kernels) and,
on demand, ``libntm_experimental.so`` (non-default K1 builds and diagnostics,
for tests and tools only).

The library is loaded AFTER ``torch`` so that its ``libamdhip64.so.7``
dependency binds to the HIP runtime PyTorch already mapped (same soname): one
runtime, one set of streams. Loading fails loudly - there is deliberately no
eager/PyTorch fallback for the validation kernels.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must be imported before the HIP library)

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "libntm_validation.so"
EXP_LIB_PATH = _HERE / "libntm_experimental.so"

_lib: ctypes.CDLL | None = None
_exp: ctypes.CDLL | None = None


class NativeLibraryMissing(RuntimeError):
    pass


def _declare(lib: ctypes.CDLL) -> None:
    c_int, c_size, c_float, c_vp = ctypes.c_int, ctypes.c_size_t, ctypes.c_float, ctypes.c_void_p
    sig = {
        "ntm_version": ([], ctypes.c_char_p),
        "ntm_gemm_shape_ok": ([c_int, c_int, c_int], c_int),
        "ntm_gemm_bf16": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_gemm_bf16_variant": (
            [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_gemm_fp8": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_gemm_fp8_shape_ok": ([c_int, c_int, c_int], c_int),
        "ntm_gemm_fp8_variant": ([c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_vp], c_int),
        "ntm_k1_fp8_plan": ([c_int, c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "ntm_k1_fp8_plan_splitk": ([c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
        "ntm_fp8_splitk_ws_bytes": ([c_int, c_int, c_int, c_int], c_size),
        "ntm_gemm_fp8_splitk": ([c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_vp, c_size, c_vp], c_int),
        "ntm_gemm_fp8_ex": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                             c_size, c_vp], c_int),
        "ntm_gemm_bf16_rowsum": (
            [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_abft_check": ([c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                            c_vp, c_vp, c_vp], c_int),
        "ntm_abft_result_bytes": ([], c_int),
        "ntm_gemm_fp8_rowsum": (
            [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_abft_check_fp8": ([c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                c_vp, c_vp, c_vp], c_int),
        "ntm_fill_uniform_bf16": ([c_vp, c_size, ctypes.c_ulonglong, c_float, c_vp], c_int),
        "ntm_k1_plan": ([c_int, c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "ntm_k1_plan_splitk": ([c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
        "ntm_gemm_bf16_ex": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                              c_size, c_vp], c_int),
        "ntm_splitk_ws_bytes": ([c_int, c_int, c_int, c_int], c_size),
        "ntm_sk_ws_bytes": ([c_int, c_int, c_int], c_size),
        "ntm_skh_ws_bytes": ([c_int, c_int, c_int, c_int], c_size),
        "ntm_gemm_bf16_skh": ([c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_vp, c_size, c_vp], c_int),
        "ntm_k1_plan_times": ([c_int, c_int, c_int, c_vp, c_vp], c_int),
        "ntm_gemm_bf16_sk": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                              c_size, c_vp], c_int),
        "ntm_gemm_bf16_splitk": ([c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                  c_int, c_int, c_vp, c_size, c_vp], c_int),
        "ntm_fill_uniform_e4m3": ([c_vp, c_size, ctypes.c_ulonglong, c_float, c_vp], c_int),
        "ntm_ref_gemm_f32_e4m3": (
            [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_ref_gemm_f32": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_verify_bf16": ([c_vp, c_vp, c_size, c_float, c_float, c_vp, c_vp], c_int),
        "ntm_verify_result_bytes": ([], c_int),
        "ntm_clock_probe": ([c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "ntm_gemm_bf16_clock_grid": ([c_int, c_int], c_int),
        "ntm_gemm_bf16_clock_words": ([], c_int),
        "ntm_sk_error_word_index": ([], c_int),
        "ntm_set_sk_fault_inject": ([c_int], None),
        "ntm_gemm_bf16_skh_ex": ([c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_vp, c_size, c_int, c_vp], c_int),
        "ntm_plan_cus": ([], c_int),
        "ntm_set_cus_override": ([c_int], None),
        "ntm_set_plan_pp_tiles": ([c_int], None),
        "ntm_set_plan_splitk": ([ctypes.c_double, c_int, c_int], None),
        "ntm_set_plan_splitk_ragged": ([c_int], None),
        "ntm_pp3h_vmcnt": ([c_int, c_int, c_int], c_int),
        "ntm_gemm_bf16_clock": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
                                 c_vp], c_int),
        "ntm_stream_copy": ([c_vp, c_vp, c_size, c_vp], c_int),
        "ntm_stream_read": ([c_vp, c_size, c_vp, c_vp], c_int),
        "ntm_stream_copy_ex": ([c_vp, c_vp, c_size, c_int, c_int, c_int, c_vp], c_int),
        "ntm_stream_read_ex": ([c_vp, c_size, c_vp, c_int, c_int, c_int, c_vp], c_int),
    }
    for name, (argt, rest) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rest


def lib() -> ctypes.CDLL:
    """Return the loaded library, raising if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeLibraryMissing(
            f"{LIB_PATH} not found. Build it with "
            "`python -m nvidia_terraform_modules_amd.ops.build` (needs hipcc, gfx950)."
        )
    mode = os.RTLD_NOW | getattr(os, "RTLD_GLOBAL", 0)
    _lib = ctypes.CDLL(str(LIB_PATH), mode=mode)
    _declare(_lib)
    return _lib


def _declare_experimental(lib: ctypes.CDLL) -> None:
    c_int, c_vp, c_size = ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    gemm = [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]
    sig = {
        "ntm_experimental_version": ([], ctypes.c_char_p),
        "ntm_gemm_bf16_experimental": (gemm, c_int),
        "ntm_gemm_bf16_knob": (gemm, c_int),
        "ntm_gemm_bf16_ws_knob": ([c_int] + gemm, c_int),
        "ntm_gemm_bf16_stamp": (
            [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp], c_int),
        "ntm_mfma_f8_probe": ([c_vp, c_vp, c_vp, c_vp], c_int),
        "ntm_mfma_rate": ([c_int, c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "ntm_mfma_toggle": ([c_int, c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "ntm_dma_probe": ([c_int, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
        "ntm_gemm_fp8_knob": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_vp], c_int),
        "ntm_gemm_bf16_sk_rev": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_vp, c_size, c_vp], c_int),
        "ntm_gemm_bf16_sk_nopair": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_vp, c_size, c_vp], c_int),
        "ntm_gemm_bf16_sk_stamp": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_vp, c_size, c_vp, c_vp], c_int),
        "ntm_gemm_bf16_pp6_stamp": ([c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                     c_int, c_int, c_vp, c_vp], c_int),
    }
    for name, (argt, rest) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rest


def lib_experimental() -> ctypes.CDLL:
    """The experimental/diagnostic library (non-default K1 builds, schedule
    knobs, probes). Loaded on first use; the shipping paths never touch it."""
    global _exp
    if _exp is not None:
        return _exp
    lib()  # HIP runtime binding order: the shipping library (and torch) first
    if not EXP_LIB_PATH.exists():
        raise NativeLibraryMissing(
            f"{EXP_LIB_PATH} not found. Build it with "
            "`python -m nvidia_terraform_modules_amd.ops.build`.")
    _exp = ctypes.CDLL(str(EXP_LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_GLOBAL", 0))
    _declare_experimental(_exp)
    return _exp


def available() -> bool:
    try:
        lib()
        return True
    except (NativeLibraryMissing, OSError):
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def stream_handle(stream: "torch.cuda.Stream | None" = None) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def version() -> str:
    return lib().ntm_version().decode()
