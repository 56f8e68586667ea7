// DIAGNOSTIC build of K1 "pingpong8c" (gemm_bf16_pp3.hpp, default epilogue)
// for ablation timing (cdna_hip_programming.md §5.4 rule 17, §7 "In-kernel
// stamps"; MI355X_MICROARCH.md "DVFS give-back" item 6). Never used for
// results: outputs of modes 1-3 are garbage by construction, and the stamps
// only go to their own buffer.
//
// MODE 0: the real kernel (+ one s_memtime / s_memrealtime pair per wave at
//         start and end -> in-kernel clock and WG span);
// MODE 1: no LDS traffic: fragment reads and LDS-DMA removed, MFMAs + both
//         barriers kept (the matrix + barrier floor);
// MODE 2: no MFMAs: reads + DMA + barriers kept, fragments kept live with an
//         empty asm (the load floor);
// MODE 3: MFMAs only, no barriers, no loads (the per-SIMD matrix peak at the
//         clock this body sustains);
// MODE 4: fragment reads kept, LDS-DMA removed (reads hit stale LDS);
// MODE 5: LDS-DMA kept, fragment reads removed (registers of K-tile 0).
// Modes 4 / 5 split MODE 1's saving into LDS-read and global->LDS energy.
// (A first version stamped every barrier: 16 s_memtime per K-tile made the
// kernel 10x slower, since each stamp's return forces lgkmcnt(0) on the LDS
// reads in flight.)
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gemm3s {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::issue_half3;
using ::ntm::gemm3::kEpiDefault;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::shape_ok3;

// u64 slots per wave in the stamp buffer
enum : int { kStart = 0, kEnd, kRtStart, kRtEnd, kHwId, kXccId, kRtLoop0, kRtLoop1, kSlots = 8 };

__device__ __forceinline__ void keep(const bf16x8 (&x)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(x[i][j]));
}
__device__ __forceinline__ void keep(const bf16x8 (&x)[4][2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(x[i][j]));
}

template <int P, bool ODD, int MODE>
__device__ __forceinline__ void phase_a(const Ctx& c, Frags3& f,
                                        f32x4 (&acc)[2][2][4][2], int t, int T) {
  bf16x8(&bcur)[2][2] = ODD ? f.b1 : f.b0;
  bf16x8(&both)[2][2] = ODD ? f.b0 : f.b1;
  const int cur = t & 1;
  constexpr bool kReads = MODE == 0 || MODE == 2 || MODE == 4;
  constexpr bool kDma = MODE == 0 || MODE == 2 || MODE == 5;
  if constexpr (kReads) {
    if constexpr (P == 0) read_a<kALo>(c, f.a, cur);
    if constexpr (P == 1) read_b<kBHi>(c, both, cur);
    if constexpr (P == 2) read_a<kAHi>(c, f.a, cur);
    if constexpr (P == 3) read_b<kBLo>(c, both, cur ^ 1);
  }
  if constexpr (kDma) {
    if constexpr (P == 0) issue_half3<kAHi>(c, t + 1, cur ^ 1, T);
    if constexpr (P == 1) issue_half3<kBLo>(c, t + 2, cur, T);
    if constexpr (P == 2) issue_half3<kALo>(c, t + 2, cur, T);
    if constexpr (P == 3) issue_half3<kBHi>(c, t + 2, cur, T);
    wait_vmcnt<10>();
  }
  if constexpr (MODE != 3) raw_barrier();
  if constexpr (MODE == 2) {
    if constexpr (P == 0 || P == 2) keep(f.a);
    if constexpr (P == 1 || P == 3) keep(both);
  } else {
    if constexpr (P == 0) mma_quadrant<false>(acc[0][0], f.a, bcur);
    if constexpr (P == 1) mma_quadrant<false>(acc[0][1], f.a, both);
    if constexpr (P == 2) mma_quadrant<false>(acc[1][1], f.a, both);
    if constexpr (P == 3) mma_quadrant<false>(acc[1][0], f.a, bcur);
  }
  if constexpr (MODE != 3) raw_barrier();
}

template <bool ODD, int MODE>
__device__ __forceinline__ void tile_a(const Ctx& c, Frags3& f,
                                       f32x4 (&acc)[2][2][4][2], int t, int T) {
  phase_a<0, ODD, MODE>(c, f, acc, t, T);
  phase_a<1, ODD, MODE>(c, f, acc, t, T);
  phase_a<2, ODD, MODE>(c, f, acc, t, T);
  phase_a<3, ODD, MODE>(c, f, acc, t, T);
}

template <int MODE>
__global__ void __launch_bounds__(kThreads, 2)
    gemm_bf16_pp3_stamp_kernel(GemmArgs p, unsigned long long* stamps) {
  static_assert(MODE >= 0 && MODE <= 5, "ablation mode");
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long ts0 = __builtin_amdgcn_s_memtime();

  int tm, tn;
  tile_coords<kGroupM>(p.M, p.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  Ctx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    const __bf16* a0 = p.A + (size_t)(m0 + c.w * 16 + r) * p.lda + cl * 8;
    const __bf16* b0 = p.B + (size_t)(n0 + c.w * 16 + r) * p.ldb + cl * 8;
    c.src[kALo] = a0;
    c.src[kAHi] = a0 + (size_t)128 * p.lda;
    c.src[kBLo] = b0;
    c.src[kBHi] = b0 + (size_t)128 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][j][m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  Frags3 f;
  const int T = p.K / BK;
  issue_half<kBLo>(c, 0, 0);
  issue_half<kALo>(c, 0, 0);
  issue_half<kBHi>(c, 0, 0);
  issue_half<kAHi>(c, 0, 0);
  issue_half<kBLo>(c, 1, 1);
  issue_half<kALo>(c, 1, 1);
  issue_half<kBHi>(c, 1, 1);
  wait_vmcnt<10>();
  raw_barrier();
  read_b<kBLo>(c, f.b0, 0);
  if constexpr (MODE == 1 || MODE == 3 || MODE == 5) {
    // fragments of K-tile 0 stand in for every K-tile (no LDS traffic)
    read_a<kALo>(c, f.a, 0);
    read_b<kBHi>(c, f.b1, 0);
  }
  if (c.wr == 1) raw_barrier();
  // prologue / K loop / epilogue split (realtime stamps, 100 MHz): two SMEM
  // returns per workgroup, outside the loop
  const unsigned long long rl0 = __builtin_amdgcn_s_memrealtime();

  for (int t = 0; t < T; t += 2) {
    tile_a<false, MODE>(c, f, acc, t, T);
    tile_a<true, MODE>(c, f, acc, t + 1, T);
  }
  if (c.wr == 0) raw_barrier();
  const unsigned long long rl1 = __builtin_amdgcn_s_memrealtime();
  wait_vmcnt<0>();
  store_tile_epi<false, kEpiDefault>(p, c, acc, m0, n0, lane);
  const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();

  if (lane == 0) {
    unsigned long long* o = stamps + ((size_t)blockIdx.x * 8 + c.w) * kSlots;
    o[kStart] = ts0;
    o[kEnd] = ts1;
    o[kRtStart] = rt0;
    o[kRtEnd] = rt1;
    o[kRtLoop0] = rl0;
    o[kRtLoop1] = rl1;
    // HW_REG_HW_ID (4) and HW_REG_XCC_ID (20), full 32 bits: which CU ran it
    o[kHwId] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    o[kXccId] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
}

// stamps: (M/256)*(N/256) * 8 waves * kSlots u64, written by lane 0 of each wave.
inline hipError_t launch_gemm_bf16_pp3_stamp(const GemmArgs& a, int mode,
                                             unsigned long long* stamps, hipStream_t stream) {
  if (!shape_ok3(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) || !stamps)
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  switch (mode) {
    case 0: hipLaunchKernelGGL(gemm_bf16_pp3_stamp_kernel<0>, g, b, 0, stream, a, stamps); break;
    case 1: hipLaunchKernelGGL(gemm_bf16_pp3_stamp_kernel<1>, g, b, 0, stream, a, stamps); break;
    case 2: hipLaunchKernelGGL(gemm_bf16_pp3_stamp_kernel<2>, g, b, 0, stream, a, stamps); break;
    case 3: hipLaunchKernelGGL(gemm_bf16_pp3_stamp_kernel<3>, g, b, 0, stream, a, stamps); break;
    case 4: hipLaunchKernelGGL(gemm_bf16_pp3_stamp_kernel<4>, g, b, 0, stream, a, stamps); break;
    case 5: hipLaunchKernelGGL(gemm_bf16_pp3_stamp_kernel<5>, g, b, 0, stream, a, stamps); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace gemm3s
}  // namespace ntm
