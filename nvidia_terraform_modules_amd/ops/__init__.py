"""MI355X (gfx950) HIP kernels used by the post-provision validation Job.

K1 ``gemm_bf16``      - 256x256x64 LDS-DMA + MFMA bf16 GEMM (the headline; small,
                        mid-size and ragged C also on 128x128 / 256x128 / 160x160 /
                        160x128 / 128x160 tiles, skinny long-K C split-K; see
                        ``k1_plan`` / ``k1_splitk_plan``);
   ``gemm_bf16_rowsum`` - same kernel with the fused ABFT row-checksum epilogue;
   ``gemm_fp8``         - the same kernels on OCP e4m3 operands (f8f6f4 MFMA; 256x256
                          and the wave-specialised tiles, ``k1_fp8_plan``).
K2 ``stream_copy``, ``stream_read`` - tuned float4 HBM streams.
K3 ``fill_uniform_``, ``ref_gemm_f32``, ``verify_bf16``, ``abft_check`` - synthetic
   data, full fp32 reference check and the O(n^2) checksum check;
   ``clock_probe_ghz`` - the shader clock held under a dense MFMA load;
   ``gemm_clock_ghz`` - the clock K1's own 8192^3-class launches run at
   (``gemm_clock_stable``: the same, re-stamped until a batch is transient-free).

Import is cheap; the native library is loaded on first kernel call and raises
``NativeLibraryMissing`` if it was not built (no silent fallback).
"""
from ._lib import NativeLibraryMissing, available, version  # noqa: F401
from .kernels import (  # noqa: F401
    AbftReport,
    VerifyReport,
    abft_check,
    clock_probe_ghz,
    fill_uniform_,
    gemm_bf16,
    gemm_bf16_rowsum,
    clock_summary,
    gemm_clock_ghz,
    gemm_clock_stable,
    gemm_fp8,
    gemm_fp8_rowsum,
    gemm_fp8_shape_ok,
    gemm_shape_ok,
    gemm_tolerance,
    FP8_VARIANTS,
    k1_fp8_plan,
    k1_fp8_splitk_plan,
    k1_candidates,
    k1_plan,
    k1_splitk_plan,
    ref_gemm_f32,
    set_plan_pp_tiles,
    set_plan_splitk,
    set_plan_splitk_ragged,
    set_cus_override,
    sk_ws_bytes,
    sk_xcc_error,
    SkPlacementError,
    set_sk_fault_inject,
    sk_check_enabled,
    stream_copy,
    stream_read,
    verify_bf16,
)
