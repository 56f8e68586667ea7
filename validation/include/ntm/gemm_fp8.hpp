// K1-fp8: OCP e4m3 GEMM on the f8f6f4 matrix path of CDNA4
// (v_mfma_f32_16x16x128_f8f6f4; its MX-scaled form with unit E8M0 scales
// gives bit-identical results): twice the bf16 MFMA rate per CU clock
// (cdna_hip_programming.md "MFMA rate per dtype").
//
// The validation Job uses it to exercise the fp8 matrix cores that MI355X
// inference workloads run on; the reference's GPU Operator validator has no
// counterpart (SURVEY.md §2.7 lists only the bf16 K1).
//
// Diagnostics (operand-map probe, MFMA rate probe) and the experimental
// schedule knobs live in gemm_fp8_diag.hpp, built only into
// libntm_experimental.so - never into the shipping library or Job binary.
#pragma once

#include "ntm/common.hpp"
#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace fp8 {

using ::ntm::gemm::i32x8;

// fmt codes of the f8f6f4 instruction (cbsz / blgp): 0 = fp8 e4m3, 1 = bf8 e5m2
constexpr int kFmtE4M3 = 0;
constexpr int kScaleOne = 127;  // E8M0 exponent bias: 2^(127-127) = 1

__device__ __forceinline__ f32x4 mfma_f8(const i32x8& a, const i32x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, kFmtE4M3, kFmtE4M3, 0,
                                                          kScaleOne, 0, kScaleOne);
}

// C[M x N] (bf16) = A[M x K] (e4m3) * B[N x K]^T (e4m3), fp32 accumulation,
// on the pingpong8c schedule (gemm_bf16_pp3.hpp, F8 = true) with its default
// LDS-staged epilogue. lda / ldb / ldc in elements (fp8 for A/B, bf16 for C).
// Shape rule: 16-byte aligned rows; M, N, K % 256 run the exact build; any M
// with N % 8 and K % 16 the masked one (edge tiles clamp their DMA source rows
// and skip stores past C; a partial last K-tile loads zeros past K;
// gemm_bf16_pp3.hpp).
__host__ __device__ inline bool shape_exact(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 256 && (M % 256) == 0 && (N % 256) == 0 && (K % 256) == 0;
}
__host__ __device__ inline bool shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && (N % 8) == 0 && (K % 16) == 0;  // K % 256: exact K loop
}

inline hipError_t launch_gemm_fp8(const void* A, const void* B, __bf16* C, int M, int N, int K,
                                  int lda, int ldb, int ldc, hipStream_t stream) {
  using namespace ::ntm::gemm;
  if (!shape_ok(M, N, K) || lda < K || ldb < K || ldc < N || (lda % 16) || (ldb % 16) ||
      (ldc % 8))
    return hipErrorInvalidValue;
  GemmArgs a;
  a.A = (const __bf16*)A;  // byte image: two fp8 per bf16 slot
  a.B = (const __bf16*)B;
  a.C = C;
  a.M = M;
  a.N = N;
  a.K = K / 2;
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  const dim3 g((unsigned)(((M + BM - 1) / BM) * ((N + BN - 1) / BN))), b(kThreads);
  // F8 = 3: the plain v_mfma_f32_16x16x128_f8f6f4 (no v_mfma_ld_scale_b32
  // prefix; the hardware's default scales are 2^0, bit-identical results):
  // +1 % at 8192^3, +2.5 % at 4096^3, +3.6 % at 6144^3 over the scaled form
  // with unit VGPR scales in 15 interleaved rounds (profiles/r1_fp8b/knobs_plain.log).
  using ::ntm::gemm3::kEpiDefault;
  if (shape_exact(M, N, K))
    hipLaunchKernelGGL((::ntm::gemm3::gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault, 0, 3>),
                       g, b, 0, stream, a);
  else if (K % 256)  // partial last K-tile: 16-value chunks past K load zeros
    hipLaunchKernelGGL((::ntm::gemm3::gemm_bf16_pp3_kernel<false, kGroupM, false,
                                                           kEpiDefault | kEpiMask | kEpiKTail, 0, 3>),
                       g, b, 0, stream, a);
  else
    hipLaunchKernelGGL((::ntm::gemm3::gemm_bf16_pp3_kernel<false, kGroupM, false,
                                                           kEpiDefault | kEpiMask, 0, 3>),
                       g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace fp8
}  // namespace ntm
