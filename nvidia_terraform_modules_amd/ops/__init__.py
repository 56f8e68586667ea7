"""MI355X (gfx950) HIP kernels used by the post-provision validation Job.

K1 ``gemm_bf16``      - 256x256x64 LDS-DMA + MFMA bf16 GEMM (the headline).
K2 ``stream_copy``    - float4 HBM stream.
K3 ``fill_uniform_``, ``ref_gemm_f32``, ``verify_bf16`` - synthetic data and checks.

Import is cheap; the native library is loaded on first kernel call and raises
``NativeLibraryMissing`` if it was not built (no silent fallback).
"""
from ._lib import NativeLibraryMissing, available, version  # noqa: F401
from .kernels import (  # noqa: F401
    VerifyReport,
    fill_uniform_,
    gemm_bf16,
    gemm_shape_ok,
    gemm_tolerance,
    ref_gemm_f32,
    stream_copy,
    stream_read,
    verify_bf16,
)
