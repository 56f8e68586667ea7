// K1 v6 ("pingpong8w"): pingpong8c with WIDE segments. Each wave alternates a
// load segment (fragment reads + LDS-DMA issue) and a 32-MFMA compute segment
// (one 64-row half of its 128x64 output over K = 64) instead of 16-MFMA
// quadrant segments, so a K-tile costs 4 barrier intervals instead of 8.
//
// Why: in the 4-phase schedule every SIMD hands its matrix pipe from one wave
// to its partner at every barrier (8 hand-offs per K-tile, 256 MFMA cycles
// each); the hand-off (barrier release + first MFMA issue) is not covered by
// matrix work. The K-fit (profiles/r1_pp3_knobs/kfit.log) put pingpong8c's
// steady-state loop at 1693 TF-equivalent vs hipBLASLt's 1760 at 8192^2; its
// hipBLASLt counterpart (4 waves, 128x128 per wave) does not hand off at all.
// Halving the hand-offs keeps the 8-wave ping-pong (one wave's LDS reads and
// DMA issue hidden under its partner's MFMAs) at half the switching cost.
//
// Per wave and K-tile t (buffer cur = t & 1), group 1 (wr = 1) one barrier
// behind group 0:
//   LS0(t): read A-lo(t), B-lo(t), B-hi(t)   [16 ds_read_b128]
//           issue A-hi(t+1) -> buffer cur^1   [2 LDS-DMA pieces]
//           vmcnt(8); lgkmcnt(0); barrier
//   C0(t):  32 MFMA: rows 0-63 of the wave tile (A-lo x B-lo, A-lo x B-hi); barrier
//   LS1(t): read A-hi(t)                      [8 ds_read_b128]
//           issue A-lo, B-lo, B-hi(t+2) -> cur [6 pieces]
//           vmcnt(8); lgkmcnt(0); barrier
//   C1(t):  32 MFMA: rows 64-127 (A-hi x B-lo, A-hi x B-hi); barrier
// Registers: 128 fp32 accumulators + 8 A + 8 B fragments (bf16x8) per lane.
//
// Ordering proof (load segments numbered s = 2t / 2t+1 per wave; a group-1
// segment s runs one barrier after group 0's):
//  RAW: every load segment issues exactly the pieces of one LS0 (2) plus one
//       LS1 (6) in any two consecutive segments, so vmcnt(8) at the end of
//       segment s retires every piece issued in segments <= s-2, and the
//       barrier that ends s publishes them to both groups for segment s+1.
//       A-hi(t+1) is issued in 2t and read in 2t+3; A-lo/B-lo/B-hi(t+2)
//       issued in 2t+1 and read in 2t+4: distance 3 >= 3 everywhere.
//  WAR: a load segment ends with lgkmcnt(0) before its barrier, so its reads
//       have returned before any later segment of either group starts. The
//       pieces issued in segment s overwrite only regions last read in s-1:
//       A-hi(t+1) -> A-hi region of buffer cur^1, last read in LS1(t-1);
//       lo/B(t+2) -> A-lo/B-lo/B-hi of buffer cur, last read in LS0(t).
//  Tiles >= T issue dummy pieces into a 16 KiB scratch region nobody reads
//  (as pingpong8c), so the count is uniform and the loop has no tail; all
//  pieces are drained (vmcnt(0)) before the epilogue.
// Shape rule: T = K / 64 even (K % 128 == 0), T >= 2; M, N % 256.
#pragma once

#include "ntm/gemm_bf16.hpp"
#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gemm5 {

using namespace ::ntm::gemm;
using ::ntm::gemm3::issue_half3;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::shape_ok3;

__device__ __forceinline__ void wait_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

struct Frags5 {
  bf16x8 a[4][2];   // current A half (64 rows of this wave) x 2 k-steps
  bf16x8 bl[2][2];  // B-lo: 32 cols x 2 k-steps
  bf16x8 bh[2][2];  // B-hi
};

// ISSUE_FIRST: issue the segment's DMA pieces before its fragment reads
// (longer DMA flight) instead of after (reads first, as pingpong8c).
template <int CUR, bool ISSUE_FIRST>
__device__ __forceinline__ void k_tile5(const Ctx& c, Frags5& f,
                                        f32x4 (&acc)[2][2][4][2], int t, int T) {
  // ---- LS0(t)
  if constexpr (ISSUE_FIRST) issue_half3<kAHi>(c, t + 1, CUR ^ 1, T);
  read_b<kBLo>(c, f.bl, CUR);
  read_b<kBHi>(c, f.bh, CUR);
  read_a<kALo>(c, f.a, CUR);
  if constexpr (!ISSUE_FIRST) issue_half3<kAHi>(c, t + 1, CUR ^ 1, T);
  wait_vmcnt<8>();
  wait_lgkm0();
  raw_barrier();
  // ---- C0(t)
  mma_quadrant<false>(acc[0][0], f.a, f.bl);
  mma_quadrant<false>(acc[0][1], f.a, f.bh);
  raw_barrier();
  // ---- LS1(t)
  if constexpr (ISSUE_FIRST) {
    issue_half3<kALo>(c, t + 2, CUR, T);
    issue_half3<kBLo>(c, t + 2, CUR, T);
    issue_half3<kBHi>(c, t + 2, CUR, T);
  }
  read_a<kAHi>(c, f.a, CUR);
  if constexpr (!ISSUE_FIRST) {
    issue_half3<kALo>(c, t + 2, CUR, T);
    issue_half3<kBLo>(c, t + 2, CUR, T);
    issue_half3<kBHi>(c, t + 2, CUR, T);
  }
  wait_vmcnt<8>();
  wait_lgkm0();
  raw_barrier();
  // ---- C1(t)
  mma_quadrant<false>(acc[1][0], f.a, f.bl);
  mma_quadrant<false>(acc[1][1], f.a, f.bh);
  raw_barrier();
}

// WIDE: widened dwordx4 epilogue (store_tile_wide) instead of dwordx2.
template <bool kRowSum, bool ISSUE_FIRST = false, bool WIDE = false>
__global__ void __launch_bounds__(kThreads, 2)
    gemm_bf16_pp5_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];

  int tm, tn;
  tile_coords(p.M, p.N, tm, tn);
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

  Frags5 f;
  const int T = p.K / BK;

  // Prologue = virtual segments LS1(-2), LS0(-1), LS1(-1):
  //   lo/B(0) [6 pieces], A-hi(0) [2], lo/B(1) [6]; vmcnt(8) retires lo/B(0).
  issue_half<kALo>(c, 0, 0);
  issue_half<kBLo>(c, 0, 0);
  issue_half<kBHi>(c, 0, 0);
  issue_half<kAHi>(c, 0, 0);
  issue_half3<kALo>(c, 1, 1, T);
  issue_half3<kBLo>(c, 1, 1, T);
  issue_half3<kBHi>(c, 1, 1, T);
  wait_vmcnt<8>();
  raw_barrier();
  if (c.wr == 1) raw_barrier();  // ping-pong stagger

  for (int t = 0; t < T; t += 2) {
    k_tile5<0, ISSUE_FIRST>(c, f, acc, t, T);
    k_tile5<1, ISSUE_FIRST>(c, f, acc, t + 1, T);
  }
  if (c.wr == 0) raw_barrier();
  wait_vmcnt<0>();  // dummy pieces: nothing may land after the WG exits

  if constexpr (WIDE)
    store_tile_wide<kRowSum>(p, c, acc, m0, n0, lane);
  else
    store_tile<kRowSum>(p, c, acc, m0, n0, lane);
}

// mode bit 0: ISSUE_FIRST, bit 1: WIDE epilogue.
template <bool kRowSum>
inline void launch5(const GemmArgs& a, int mode, dim3 g, dim3 b, hipStream_t s) {
  switch (mode & 3) {
    case 0: hipLaunchKernelGGL((gemm_bf16_pp5_kernel<kRowSum, false, false>), g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL((gemm_bf16_pp5_kernel<kRowSum, true, false>), g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemm_bf16_pp5_kernel<kRowSum, false, true>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((gemm_bf16_pp5_kernel<kRowSum, true, true>), g, b, 0, s, a); break;
  }
}

// The wide epilogue stores 16 B per lane: ldc % 8 keeps every row 16-B aligned.
inline hipError_t launch_gemm_bf16_pp5(const GemmArgs& a, int mode, hipStream_t stream) {
  if (!shape_ok3(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  if (a.rowsum)
    launch5<true>(a, mode, g, b, stream);
  else
    launch5<false>(a, mode, g, b, stream);
  return hipGetLastError();
}

}  // namespace gemm5
}  // namespace ntm
