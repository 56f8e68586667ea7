// K1-fp8 diagnostics and experiments - built ONLY into libntm_experimental.so
// (tests and tools), never into libntm_validation.so or the Job binary.
//
// mfma_f8_probe: one wave, one MFMA on operands pre-arranged per lane by the
// host (64 lanes x 32 bytes each for A and B) -> the 16x16 fp32 result in the
// dtype-independent C/D layout (col = lane & 15, row = 4 * (lane >> 4) + j).
// Used by tests/test_kernels_gpu.py to pin the operand lane map with exact
// data before the GEMM relies on it (playbook: "Other dtypes: check the map
// with exact integer data").
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"
#include "ntm/gemm_fp8.hpp"
#include "ntm/gemm_bf16_pp6.hpp"
#include "ntm/gemm_w4k.hpp"

namespace ntm {
namespace fp8 {

__global__ void __launch_bounds__(64) mfma_f8_probe_kernel(const i32x8* a, const i32x8* b,
                                                           f32x4* d) {
  const int l = threadIdx.x;
  d[l] = mfma_f8(a[l], b[l], f32x4{0.f, 0.f, 0.f, 0.f});
}

// Experimental knobs (tools/gemm_fp8_check.py --knobs): 0 = the default above;
// 1 = B-fragment-outer MFMA order (scaled form); 2 = GROUP_M 4; 3 = static s_setprio(1) on
// wave row 1; 4 = register (widened + nontemporal) epilogue instead of the
// LDS-staged one; 5 = the scaled MFMA form with unit VGPR scales (the previous default;
// knobs 1-4 use it too). Knob 12 (the 4-wave dma4k kernel) was deleted in round 4.
// Knobs 6-9 (persistent, early / register epilogues, GROUP_M 4 on
// the plain form) measured 1-2 % slower or tied (profiles/r2_fp8ws/knobs_6_9.log) and were
// deleted (git history).
inline hipError_t launch_gemm_fp8_knob(const void* A, const void* B, __bf16* C, int M, int N,
                                       int K, int lda, int ldb, int ldc, int knob,
                                       hipStream_t s) {
  using namespace ::ntm::gemm;
  using ::ntm::gemm3::gemm_bf16_pp3_kernel;
  using ::ntm::gemm3::kEpiDefault;
  if (!shape_ok(M, N, K) || lda < K || ldb < K || ldc < N || (lda % 16) || (ldb % 16) ||
      (ldc % 8))
    return hipErrorInvalidValue;
  GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = C;
  a.M = M;
  a.N = N;
  a.K = K / 2;
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  const dim3 g((unsigned)((M / BM) * (N / BN))), b(kThreads);
  switch (knob) {
    case 0: return launch_gemm_fp8(A, B, C, M, N, K, lda, ldb, ldc, s);
    // 30: the persistent overlap kernel (pingpong8o) with f8f6f4 MFMAs on VGPR
    // accumulators (gemm_bf16_pp6.hpp F8)
    case 30: return ::ntm::gemm6::launch_gemm_fp8_pp6(A, B, C, M, N, K, lda, ldb, ldc, s);
    // 31: the same with the boundary stores spread over 7 phases (SPREAD, as the
    // shipping bf16 build)
    case 31: return ::ntm::gemm6::launch_gemm_fp8_pp6<true>(A, B, C, M, N, K, lda, ldb, ldc, s);
    // 12 (restored in round 6 for the energy study, profiles/r6_fp8): the 4-wave
    // one-barrier-per-K-tile kernel, 128x128 per wave, DMA every 2 MFMAs (gemm_w4k.hpp)
    case 12: return ::ntm::w4k::launch_gemm_fp8_w4k<2>(A, B, C, M, N, K, lda, ldb, ldc, s);
    // 32 (round 6): knob 31 + the next tile's K-tiles 0 / 1 touched into L2 over
    // K-tiles T-4 / T-3 (PF; fp8 K >= 768)
    case 32: return ::ntm::gemm6::launch_gemm_fp8_pp6<true, true>(A, B, C, M, N, K, lda, ldb, ldc, s);
    case 1: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault, 0, 2>), g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 4, false, kEpiDefault, 0, 1>), g, b, 0, s, a); break;
    case 3: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault, 2, 1>), g, b, 0, s, a); break;
    case 4: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiWide | kEpiNT, 0, 1>), g, b, 0, s, a); break;
    case 5: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault, 0, 1>), g, b, 0, s, a); break;
    // 23: ablation - the default fp8 build with C not stored (timing only, wrong C)
    case 23: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault | kEpiSkip, 0, 3>), g, b, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Matrix-core rate probe: every wave issues iters x 8 independent MFMAs
// (operands in registers, random bits from the seed) between two s_memtime
// stamps; one 256-thread workgroup (one wave per SIMD) per CU. F8 selects
// v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3, unit scales), else
// v_mfma_f32_16x16x32_bf16. out[wave] = {cycles, realtime ticks}; the sums
// keep the accumulators live.
template <bool F8, bool W32 = false>
__global__ void __launch_bounds__(256) mfma_rate_kernel(int iters, unsigned seed,
                                                        unsigned long long* out, float* sink) {
  const int lane = threadIdx.x & 63;
  i32x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    // e4m3 / bf16 bit patterns with the exponent kept small (no inf / nan)
    const unsigned h = (unsigned)mix64(((unsigned long long)seed << 32) ^ (lane * 8 + i));
    a[i] = (int)(h & 0x3B3B3B3Bu);
    b[i] = (int)((h >> 3) & 0x3B3B3B3Bu);
  }
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x16 acc32[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc32[j] = f32x16{};
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 al = {a[0], a[1], a[2], a[3]}, bl = {b[0], b[1], b[2], b[3]};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    // in-place AGPR accumulators (asm): the builtin form let hipcc rotate the
    // 8 accumulators through v_accvgpr_mov chains every iteration
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (F8 && W32)  // f8f6f4 32x32x64: 2x the MACs per instruction
        asm("v_mfma_f32_32x32x64_f8f6f4 %0, %1, %2, %0" : "+a"(acc32[j & 3]) : "v"(a), "v"(b));
      else if constexpr (F8)
        ::ntm::gemm::mfma_f8_agpr(acc[j], a, b);
      else if constexpr (W32)  // 32x32x16: 2x the MACs per instruction, 4 accumulators of 16
        asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
            : "+a"(acc32[j & 3])
            : "v"(al), "v"(bl));
      else
        asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(al), "v"(bl));
    }
  }
  ::ntm::gemm::mfma_drain();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if constexpr (W32) {
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc32[j][0] + acc32[j][15];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (s == 12345.678f) sink[0] = s;
  if (lane == 0) {
    const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = r1 - r0;
  }
}

// Operand-toggle energy probe (round 6): mfma_rate_kernel issues the same two
// operand registers on every MFMA, so its power is that of an idle operand
// path. This probe issues 16 v_mfma_f32_16x16x32_bf16 per iteration into 8
// AGPR accumulators with the operands of a pp6 quadrant (a[4][2], b[2][2],
// random bf16 bits) in one of these orders:
//   PAT 0  fixed: a[0][0] x b[0][0] every MFMA (mfma_rate_kernel's load)
//   PAT 1  zero operands
//   PAT 2  one operand changes per MFMA (b alternates, a fixed)
//   PAT 3  both operands change on every MFMA
//   PAT 4  mma_q's order: ks, mt, nt (both change at every mt step)
//   PAT 5  snake: ks, mt, nt reversed on odd mt (one operand changes per MFMA
//          inside a ks; the 8-MFMA distance between dependent MFMAs is kept)
//   PAT 6  PAT 4 with the accumulators in arch VGPRs (K1 bf16's form) instead
//          of AGPRs (hipBLASLt's form)
// asm volatile pins the issue order.
template <int PAT>
__global__ void __launch_bounds__(256) mfma_toggle_kernel(int iters, unsigned seed,
                                                          unsigned long long* out, float* sink) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  i32x4 a[4][2], b[2][2];
#pragma unroll
  for (int s = 0; s < 12; ++s) {
    i32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned h =
          (unsigned)mix64(((unsigned long long)seed << 32) ^ (unsigned)((lane * 12 + s) * 4 + i));
      v[i] = PAT == 1 ? 0 : (int)(h & 0xBFBFBFBFu);  // |x| < 2, random sign / mantissa
    }
    if (s < 8) a[s >> 1][s & 1] = v;
    else b[(s - 8) >> 1][s & 1] = v;
  }
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int nt = PAT == 5 && (mt & 1) ? 1 - i : i;
          const int j = mt * 2 + nt;
          const int q = (ks * 4 + mt) * 2 + i;  // issue slot 0..15
          const i32x4& sa = PAT <= 1   ? a[0][0]
                            : PAT == 2 ? a[0][0]
                            : PAT == 3 ? a[q & 1][0]
                                       : a[mt][ks];
          const i32x4& sb = PAT <= 1 ? b[0][0] : PAT <= 3 ? b[q & 1][0] : b[nt][ks];
          if constexpr (PAT == 6)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(sb), "v"(sa));
          else
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(sb), "v"(sa));
        }
  }
  ::ntm::gemm::mfma_drain();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (s == 12345.678f) sink[0] = s;
  if (lane == 0) {
    const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = r1 - r0;
  }
}

}  // namespace fp8
}  // namespace ntm
