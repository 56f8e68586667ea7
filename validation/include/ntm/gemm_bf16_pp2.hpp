// K1 v3 ("pingpong8b"): the 8-wave ping-pong kernel of gemm_bf16.hpp with a
// re-derived LDS schedule. Same tile, waves, LDS layout, swizzle, fragment
// registers and epilogue; what changes is WHEN fragments are read and WHEN
// half-tiles are staged.
//
// Why (profiles/r1_pmc_v1_vs_hipblaslt): v1 reads 12 / 4 / 8 / 0 fragments
// (ds_read_b128) in phases 0..3. Eight waves x 12 reads = 384 LDS cycles in
// phase 0 against the partner group's 256-cycle MFMA window, so the SIMDs
// idle there (SQ_WAIT_INST_LDS 3.4x hipBLASLt's) while phase 3's LDS is unused.
//
// Here B has two fragment buffers: the next tile's B-lo is read in phase 3
// into the buffer B-hi just vacated (b1) and moved to b0 at the end of the
// tile (16 v_mov, overlapped with MFMAs - letting the buffers alternate by
// tile parity instead makes the register allocator spill ~250 VGPRs), so
// reads are 8 / 4 / 8 / 4 with no extra VGPRs (A 32 + 2 x B 16 as in v1).
//
//   phase  reads (into)          MFMA quadrant      LDS-DMA issue
//   4t+0   A-lo(t)   (A)         (A-lo, Bcur=B-lo)  A-hi(t+1)
//   4t+1   B-hi(t)   (Both)      (A-lo, Both)       B-lo(t+2)
//   4t+2   A-hi(t)   (A)         (A-hi, Both)       A-lo(t+2)
//   4t+3   B-lo(t+1) (Both)      (A-hi, Bcur)       B-hi(t+2)
//   then Bcur := Both.    Buffer of tile t = t & 1.
//
// Ordering proof (group 1 lags group 0 by one barrier; reads of phase R are
// complete before the reader's end-of-R barrier):
//  RAW: every piece is read exactly 6 phases after its issue; vmcnt(10) in
//       phase X (5 pieces = 10 glds in flight) retires everything issued at
//       <= X-5 before the mid barrier that precedes both groups' reads of X+1.
//  WAR: each half is re-staged exactly 2 phases after its last read (A-hi:
//       read 4t-2, restaged 4t; B-lo: 4t-1 / 4t+1; A-lo: 4t / 4t+2; B-hi:
//       4t+1 / 4t+3) - the minimum that is safe under the one-barrier lag.
//  Prologue: B-lo0 A-lo0 B-hi0 A-hi0 B-lo1 A-lo1 B-hi1 (virtual phases -7..-1),
//       vmcnt(10) + barrier, read B-lo0 into Bcur.
//  Tail: tile T-2 issues only A-hi(T-1) (phase L = 4(T-2)); waits after L
//       allow L - X + 5 pieces: 8, 6, 4, 2, 0, none, none.
#pragma once

#include "ntm/gemm_bf16.hpp"

namespace ntm {
namespace gemm2 {

using namespace ::ntm::gemm;

struct Frags2 {
  bf16x8 a[4][2];
  bf16x8 b0[2][2];
  bf16x8 b1[2][2];
};

// One phase. P: phase in tile; ISSUE: whether this phase stages a half;
// VMC: counted vmcnt (-1 = none); READ_NEXT (phase 3): whether tile t+1
// exists. Bcur = f.b0, Both = f.b1.
template <int P, bool ISSUE, int VMC, bool READ_NEXT = true>
__device__ __forceinline__ void phase2(const Ctx& c, Frags2& f,
                                       f32x4 (&acc)[2][2][4][2], int t) {
  const int cur = t & 1;
  if constexpr (P == 0) read_a<kALo>(c, f.a, cur);
  if constexpr (P == 1) read_b<kBHi>(c, f.b1, cur);
  if constexpr (P == 2) read_a<kAHi>(c, f.a, cur);
  if constexpr (P == 3 && READ_NEXT) read_b<kBLo>(c, f.b1, cur ^ 1);
  if constexpr (ISSUE) {
    if constexpr (P == 0) issue_half<kAHi>(c, t + 1, cur ^ 1);
    if constexpr (P == 1) issue_half<kBLo>(c, t + 2, cur);
    if constexpr (P == 2) issue_half<kALo>(c, t + 2, cur);
    if constexpr (P == 3) issue_half<kBHi>(c, t + 2, cur);
  }
  wait_vmcnt<VMC>();
  raw_barrier();
  if constexpr (P == 0) mma_quadrant(acc[0][0], f.a, f.b0);
  if constexpr (P == 1) mma_quadrant(acc[0][1], f.a, f.b1);
  if constexpr (P == 2) mma_quadrant(acc[1][1], f.a, f.b1);
  if constexpr (P == 3) mma_quadrant(acc[1][0], f.a, f.b0);
  if constexpr (P == 3 && READ_NEXT) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) f.b0[i][j] = f.b1[i][j];
  }
  raw_barrier();
}

__device__ __forceinline__ void steady_tile(const Ctx& c, Frags2& f,
                                            f32x4 (&acc)[2][2][4][2], int t) {
  phase2<0, true, 10>(c, f, acc, t);
  phase2<1, true, 10>(c, f, acc, t);
  phase2<2, true, 10>(c, f, acc, t);
  phase2<3, true, 10>(c, f, acc, t);
}

// tiles T-2 and T-1
__device__ __forceinline__ void tail_tiles(const Ctx& c, Frags2& f,
                                           f32x4 (&acc)[2][2][4][2], int t) {
  phase2<0, true, 10>(c, f, acc, t);
  phase2<1, false, 8>(c, f, acc, t);
  phase2<2, false, 6>(c, f, acc, t);
  phase2<3, false, 4>(c, f, acc, t);
  phase2<0, false, 2>(c, f, acc, t + 1);
  phase2<1, false, 0>(c, f, acc, t + 1);
  phase2<2, false, -1>(c, f, acc, t + 1);
  phase2<3, false, -1, false>(c, f, acc, t + 1);
}

__device__ __forceinline__ void issue_prologue(const Ctx& c) {
  issue_half<kBLo>(c, 0, 0);
  issue_half<kALo>(c, 0, 0);
  issue_half<kBHi>(c, 0, 0);
  issue_half<kAHi>(c, 0, 0);
  issue_half<kBLo>(c, 1, 1);
  issue_half<kALo>(c, 1, 1);
  issue_half<kBHi>(c, 1, 1);
}

template <bool kRowSum, int EPI = 0>
__global__ void __launch_bounds__(kThreads, 2)
    gemm_bf16_pp2_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];

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

  Frags2 f;
  const int T = p.K / BK;

  issue_prologue(c);
  wait_vmcnt<10>();
  raw_barrier();
  read_b<kBLo>(c, f.b0, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger

  int t = 0;
  for (; t < T - 2; ++t) steady_tile(c, f, acc, t);
  tail_tiles(c, f, acc, t);
  if (c.wr == 0) raw_barrier();

  store_tile_epi<kRowSum, EPI>(p, c, acc, m0, n0, lane);
}

// Same epilogue choice as pingpong8c: widened + nontemporal when ldc % 8 == 0.
inline hipError_t launch_gemm_bf16_pp2(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.M / BM) * (a.N / BN));
  constexpr int E = kEpiWide | kEpiNT;
  const bool wide = (a.ldc % 8) == 0;
  if (a.rowsum && wide)
    hipLaunchKernelGGL((gemm_bf16_pp2_kernel<true, E>), dim3(grid), dim3(kThreads), 0, stream, a);
  else if (a.rowsum)
    hipLaunchKernelGGL(gemm_bf16_pp2_kernel<true>, dim3(grid), dim3(kThreads), 0, stream, a);
  else if (wide)
    hipLaunchKernelGGL((gemm_bf16_pp2_kernel<false, E>), dim3(grid), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(gemm_bf16_pp2_kernel<false>, dim3(grid), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemm2
}  // namespace ntm
