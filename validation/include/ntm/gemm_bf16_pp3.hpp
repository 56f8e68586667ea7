// K1 v4 ("pingpong8c"): pingpong8b's balanced 8/4/8/4 read schedule with
// (a) B fragment buffers that alternate by K-tile parity (no b1 -> b0 copy)
// and (b) a UNIFORM K loop: every K-tile, including the last two, issues its
// four LDS-DMA pieces. Pieces that would stage a tile >= T instead re-read an
// L2-hot, in-bounds slice into a 16 KiB scratch region of LDS that nobody
// reads, so the counted vmcnt(10) is right in every phase and there is no
// tail code at all.
//
// Why: in pingpong8b the compiler sinks the b1 -> b0 copy into phase 0 of the
// next tile and has to put s_waitcnt lgkmcnt(0) BEFORE phase 0's mid
// barrier, exposing the LDS latency of 8 A reads on the critical path (see
// gemm_bf16_pp2.hpp); letting the buffers alternate under the old
// pair-loop + two-parity tail made the register allocator spill ~250 VGPRs.
// One straight 2-tile loop body keeps the register roles fixed at the back
// edge, so neither happens.
//
// Schedule and ordering proof: identical to gemm_bf16_pp2.hpp (reads at
// 4t+0..3 = A-lo(t), B-hi(t), A-hi(t), B-lo(t+1); issues A-hi(t+1),
// B-lo(t+2), A-lo(t+2), B-hi(t+2); RAW distance 6 with vmcnt(10); WAR
// distance 2). Dummy pieces only write the scratch region (WAW among
// themselves is harmless) and are drained by vmcnt(0) before the epilogue,
// so no LDS-DMA is in flight when the workgroup exits.
// Shape rule: T = K / 64 even (K % 128 == 0), T >= 2; M, N % 256.
#pragma once

#include "ntm/gemm_bf16.hpp"

namespace ntm {
namespace gemm3 {

using namespace ::ntm::gemm;

constexpr int kScratch = kLdsBytes;                 // 128 KiB: dummy DMA target
constexpr int kLdsBytes3 = kLdsBytes + kHalfBytes;  // 144 KiB (1 WG / CU anyway)

__host__ __device__ inline bool shape_ok3(int M, int N, int K) {
  return shape_ok(M, N, K) && (K % (2 * BK)) == 0;
}

struct Frags3 {
  bf16x8 a[4][2];
  bf16x8 b0[2][2];
  bf16x8 b1[2][2];
};

// Stage half H of K-tile kt into buffer buf, or a dummy piece if kt >= T.
// TAIL (partial-K build): a lane chunk starting at k >= K loads 16 zero bytes.
template <int H, bool TAIL = false>
__device__ __forceinline__ void issue_half3(const Ctx& c, int kt, int buf, int T) {
  const bool real = kt < T;
  const int k_eff = real ? kt : T - 1;
  const __bf16* s = c.src[H] + (size_t)k_eff * BK;
  const int off = real ? buf * kTileBytes + H * kHalfBytes : kScratch;
  char* d = c.lds + off + (2 * c.w) * 1024;
  if constexpr (TAIL) {
    const int col = k_eff * BK + c.lane_col;
    glds16(col < c.K ? s : (const __bf16*)kZeroChunk16, d);
    glds16(col + 32 < c.K ? s + 32 : (const __bf16*)kZeroChunk16, d + 1024);
  } else {
    glds16(s, d);
    glds16(s + 32, d + 1024);
  }
}

template <int P, bool ODD, bool PRIO, int F8 = 0, bool TAIL = false>
__device__ __forceinline__ void phase3(const Ctx& c, Frags3& f,
                                       f32x4 (&acc)[2][2][4][2], int t, int T) {
  bf16x8(&bcur)[2][2] = ODD ? f.b1 : f.b0;
  bf16x8(&both)[2][2] = ODD ? f.b0 : f.b1;
  const int cur = t & 1;
  if constexpr (P == 0) read_a<kALo>(c, f.a, cur);
  if constexpr (P == 1) read_b<kBHi>(c, both, cur);
  if constexpr (P == 2) read_a<kAHi>(c, f.a, cur);
  if constexpr (P == 3) read_b<kBLo>(c, both, cur ^ 1);  // tile t+1 (junk at t = T-1)
  if constexpr (P == 0) issue_half3<kAHi, TAIL>(c, t + 1, cur ^ 1, T);
  if constexpr (P == 1) issue_half3<kBLo, TAIL>(c, t + 2, cur, T);
  if constexpr (P == 2) issue_half3<kALo, TAIL>(c, t + 2, cur, T);
  if constexpr (P == 3) issue_half3<kBHi, TAIL>(c, t + 2, cur, T);
  wait_vmcnt<10>();
  raw_barrier();
  if constexpr (F8) {
    if constexpr (P == 0) mma_quadrant_f8<F8>(acc[0][0], f.a, bcur);
    if constexpr (P == 1) mma_quadrant_f8<F8>(acc[0][1], f.a, both);
    if constexpr (P == 2) mma_quadrant_f8<F8>(acc[1][1], f.a, both);
    if constexpr (P == 3) mma_quadrant_f8<F8>(acc[1][0], f.a, bcur);
  } else {
    if constexpr (P == 0) mma_quadrant<PRIO>(acc[0][0], f.a, bcur);
    if constexpr (P == 1) mma_quadrant<PRIO>(acc[0][1], f.a, both);
    if constexpr (P == 2) mma_quadrant<PRIO>(acc[1][1], f.a, both);
    if constexpr (P == 3) mma_quadrant<PRIO>(acc[1][0], f.a, bcur);
  }
  raw_barrier();
}

template <bool ODD, bool PRIO, int F8 = 0, bool TAIL = false>
__device__ __forceinline__ void tile3(const Ctx& c, Frags3& f,
                                      f32x4 (&acc)[2][2][4][2], int t, int T) {
  phase3<0, ODD, PRIO, F8, TAIL>(c, f, acc, t, T);
  phase3<1, ODD, PRIO, F8, TAIL>(c, f, acc, t, T);
  phase3<2, ODD, PRIO, F8, TAIL>(c, f, acc, t, T);
  phase3<3, ODD, PRIO, F8, TAIL>(c, f, acc, t, T);
}

// GROUP_M / PRIO are tuning knobs (tools/gemm_check.py --variants knobN). The
// defaults are the measured best (profiles/r1_pp3_knobs, 15 interleaved
// rounds): s_setprio(1) around the MFMA block COSTS 1.3-1.7 % here - the
// partner group's LDS reads and DMA issue are what the ping-pong must not
// starve - and GROUP_M 4 vs 8 is a tie (16 / 32 thrash the XCD's L2: -6/-18 %).
// EPI: epilogue options, bit mask of kEpiWide (store_tile_wide), kEpiNT
// (nontemporal C stores) and kEpiEarly (wave row 0 stores its tile while row 1
// runs its last MFMA segment, before the stagger-balancing barrier).
// SPRIO: static s_setprio(1) for the whole K loop on wave row SPRIO - 1
// (0 = off); MI355X_MICROARCH.md "Two waves per SIMD" item 4.
// F8 (nonzero): the operands are OCP e4m3 (K1-fp8, gemm_fp8.hpp); p's K / lda /
// ldb are then counted in bf16-sized pairs of fp8 values (the LDS image is the
// same); the value is mma_quadrant_f8's MFMA order (1 = default).
template <bool kRowSum, int GROUP_M = kGroupM, bool PRIO = false, int EPI = 0, int SPRIO = 0,
          int F8 = 0>
__global__ void __launch_bounds__(kThreads, 2)
    gemm_bf16_pp3_kernel(GemmArgs p) {
  static_assert(!((EPI & kEpiLds) && (EPI & kEpiEarly)), "LDS staging needs all waves");
  static_assert(!(EPI & kEpiMask) || ((EPI & kEpiLds) && !kRowSum), "masked: LDS epilogue, no ABFT");
  static_assert(!(EPI & kEpiKTail) || (EPI & kEpiMask), "partial K rides on the masked build");
  constexpr bool TAIL = (EPI & kEpiKTail) != 0;
  static_assert(kLdsBytes3 >= BM * kStagePitch, "LDS staging buffer");
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];

  int tm, tn;
  tile_coords<GROUP_M>(p.M, p.N, tm, tn);
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
    int ra = m0 + c.w * 16 + r, rb = n0 + c.w * 16 + r;
    if constexpr ((EPI & kEpiMask) != 0) {
      // Ragged C: each lane's four source rows are fixed for the whole K loop,
      // so clamping them once keeps every load in bounds at no loop cost; the
      // clamped rows only feed C rows / columns the epilogue does not store.
      c.src[kALo] = p.A + (size_t)min(ra, p.M - 1) * p.lda + cl * 8;
      c.src[kAHi] = p.A + (size_t)min(ra + 128, p.M - 1) * p.lda + cl * 8;
      c.src[kBLo] = p.B + (size_t)min(rb, p.N - 1) * p.ldb + cl * 8;
      c.src[kBHi] = p.B + (size_t)min(rb + 128, p.N - 1) * p.ldb + cl * 8;
    } else {
      const __bf16* a0 = p.A + (size_t)ra * p.lda + cl * 8;
      const __bf16* b0 = p.B + (size_t)rb * p.ldb + cl * 8;
      c.src[kALo] = a0;
      c.src[kAHi] = a0 + (size_t)128 * p.lda;
      c.src[kBLo] = b0;
      c.src[kBHi] = b0 + (size_t)128 * p.ldb;
    }
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
  // partial-K build: ceil(K / 64) K-tiles rounded up to an even count (the
  // loop body is two K-tiles); chunks past K load zeros
  const int T = TAIL ? ((p.K + 2 * BK - 1) / (2 * BK)) * 2 : p.K / BK;
  if constexpr (TAIL) {
    c.K = p.K;
    const int r = lane >> 2;
    c.lane_col = ((lane & 3) ^ (((r >> 3) & 1) << 1)) * 8;  // as in the source setup above
  }

  // prologue: B-lo0 A-lo0 B-hi0 A-hi0 B-lo1 A-lo1 B-hi1 (virtual phases -7..-1)
  if constexpr (TAIL) {
    issue_half3<kBLo, true>(c, 0, 0, T);
    issue_half3<kALo, true>(c, 0, 0, T);
    issue_half3<kBHi, true>(c, 0, 0, T);
    issue_half3<kAHi, true>(c, 0, 0, T);
    issue_half3<kBLo, true>(c, 1, 1, T);
    issue_half3<kALo, true>(c, 1, 1, T);
    issue_half3<kBHi, true>(c, 1, 1, T);
  } else {
    issue_half<kBLo>(c, 0, 0);
    issue_half<kALo>(c, 0, 0);
    issue_half<kBHi>(c, 0, 0);
    issue_half<kAHi>(c, 0, 0);
    issue_half<kBLo>(c, 1, 1);
    issue_half<kALo>(c, 1, 1);
    issue_half<kBHi>(c, 1, 1);
  }
  wait_vmcnt<10>();
  raw_barrier();
  read_b<kBLo>(c, f.b0, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger
  if constexpr (SPRIO != 0) {
    if (c.wr == SPRIO - 1) __builtin_amdgcn_s_setprio(1);
  }

  if constexpr (TAIL) {
    // Iteration t issues K-tiles up to t+3; until that reaches the partial
    // one (ceil(K/64) - 1) the plain issue path runs, so the per-lane zero
    // selects cost nothing in the bulk of the loop.
    const int t_real = (p.K + BK - 1) / BK;
    int t = 0;
    for (; t + 4 < t_real; t += 2) {
      tile3<false, PRIO, F8, false>(c, f, acc, t, T);
      tile3<true, PRIO, F8, false>(c, f, acc, t + 1, T);
    }
    for (; t < T; t += 2) {
      tile3<false, PRIO, F8, true>(c, f, acc, t, T);
      tile3<true, PRIO, F8, true>(c, f, acc, t + 1, T);
    }
  } else {
    for (int t = 0; t < T; t += 2) {
      tile3<false, PRIO, F8>(c, f, acc, t, T);
      tile3<true, PRIO, F8>(c, f, acc, t + 1, T);
    }
  }
  if constexpr (SPRIO != 0) __builtin_amdgcn_s_setprio(0);
  if constexpr (F8) mfma_drain();  // asm MFMAs: results must land before VALU reads
  if constexpr ((EPI & kEpiEarly) != 0) {
    // Row 0 finished its last MFMA one barrier before row 1: drain its (dummy)
    // DMA pieces, store, then meet row 1's last barrier. No LDS is touched.
    wait_vmcnt<0>();
    store_tile_epi<kRowSum, EPI>(p, c, acc, m0, n0, lane);
    if (c.wr == 0) raw_barrier();
  } else {
    if (c.wr == 0) raw_barrier();
    wait_vmcnt<0>();  // dummy pieces: nothing may land after the WG exits
    store_tile_epi<kRowSum, EPI>(p, c, acc, m0, n0, lane);
  }
}

// Default epilogue whenever rows are 16-B aligned (ldc % 8 == 0): the tile is
// staged through LDS and leaves as full 512-B rows with nontemporal stores.
// Measured over the dwordx2 epilogue: the widened dwordx4 stores +2-4 %,
// nontemporal +2 % more (C is written once; it no longer evicts the A/B panels
// the XCD's other tiles still read from L2), then the LDS staging +0.5 % at
// 8192^3 / +1.5 % at 4096^3 (15 interleaved rounds) and WRITE_SIZE down from
// 159 MB to the exact 128 MB of C (profiles/r1_epilogue, r1_pmc_r6).
constexpr int kEpiDefault = kEpiLds | kEpiNT;

inline hipError_t launch_gemm_bf16_pp3(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok3(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  const bool wide = (a.ldc % 8) == 0;
  if (a.rowsum && wide)
    hipLaunchKernelGGL((gemm_bf16_pp3_kernel<true, kGroupM, false, kEpiDefault>), g, b, 0, stream, a);
  else if (a.rowsum)
    hipLaunchKernelGGL(gemm_bf16_pp3_kernel<true>, g, b, 0, stream, a);
  else if (wide)
    hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault>), g, b, 0, stream, a);
  else
    hipLaunchKernelGGL(gemm_bf16_pp3_kernel<false>, g, b, 0, stream, a);
  return hipGetLastError();
}

// Ragged C on the 256x256 kernel ("pingpong8cm"): any M, N % 8 (16-B row
// chunks of the LDS-staged epilogue), K % 8 (K % 128 != 0: the partial-K
// build); edge tiles clamp their loads and mask their stores. No ABFT row sum.
inline bool shape_ok3m(int M, int N, int K) {
  return M > 0 && N > 0 && (N % 8) == 0 && K > 0 && (K % 8) == 0;
}

inline hipError_t launch_gemm_bf16_pp3_masked(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok3m(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)(((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN))), b(kThreads);
  if (a.K % (2 * BK))
    hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault | kEpiMask | kEpiKTail>),
                       g, b, 0, stream, a);
  else
    hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault | kEpiMask>), g, b, 0,
                       stream, a);
  return hipGetLastError();
}

// Experimental knob sweep: knob = GROUP_M code (0:4, 1:8, 2:16, 3:32) + 4 * !PRIO;
// 8..11: GROUP_M 1, 2, 3, 6 without setprio (all with the dwordx2 epilogue, so
// knob 5 is the pre-r1_epilogue default); 12..15: epilogue options.
inline hipError_t launch_gemm_bf16_pp3_knob(const GemmArgs& a, int knob, hipStream_t s) {
  if (!shape_ok3(a.M, a.N, a.K) || a.rowsum) return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  switch (knob) {
    case 0: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 4, true>), g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 8, true>), g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 16, true>), g, b, 0, s, a); break;
    case 3: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 32, true>), g, b, 0, s, a); break;
    case 4: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 4, false>), g, b, 0, s, a); break;
    case 5: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 8, false>), g, b, 0, s, a); break;
    case 6: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 16, false>), g, b, 0, s, a); break;
    case 7: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 32, false>), g, b, 0, s, a); break;
    case 8: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 1, false>), g, b, 0, s, a); break;
    case 9: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 2, false>), g, b, 0, s, a); break;
    case 10: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 3, false>), g, b, 0, s, a); break;
    case 11: hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 6, false>), g, b, 0, s, a); break;
    // 12..15: default schedule + epilogue options (widened stores need ldc % 8)
    case 12: case 13: case 14: case 15: {
      if (a.ldc % 8) return hipErrorInvalidValue;
      constexpr int W = kEpiWide, N = kEpiNT, E = kEpiEarly;
      if (knob == 12) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, W>), g, b, 0, s, a);
      if (knob == 13) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, W | E>), g, b, 0, s, a);
      if (knob == 14) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, W | N>), g, b, 0, s, a);
      if (knob == 15) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, W | N | E>), g, b, 0, s, a);
      break;
    }
    // 16..18: GROUP_M 4 / 16 / 2 with the default (wide + nontemporal) epilogue
    case 16: case 17: case 18: {
      if (a.ldc % 8) return hipErrorInvalidValue;
      if (knob == 16) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 4, false, kEpiDefault>), g, b, 0, s, a);
      if (knob == 17) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 16, false, kEpiDefault>), g, b, 0, s, a);
      if (knob == 18) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 2, false, kEpiDefault>), g, b, 0, s, a);
      break;
    }
    // 21 / 22: LDS-staged full-row epilogue, nontemporal / default policy
    case 21: case 22: {
      if (a.ldc % 8) return hipErrorInvalidValue;
      if (knob == 21) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiLds | kEpiNT>), g, b, 0, s, a);
      if (knob == 22) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiLds>), g, b, 0, s, a);
      break;
    }
    case 24:  // ablation: the default build with C not stored (timing only, wrong C)
      if (a.ldc % 8) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault | kEpiSkip>), g, b, 0, s, a);
      break;
    case 23:  // LDS-staged nontemporal epilogue + GROUP_M 4
      if (a.ldc % 8) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, 4, false, kEpiLds | kEpiNT>), g, b, 0, s, a);
      break;
    // 19 / 20: default epilogue + static priority for wave row 1 (the lagging,
    // younger half) / wave row 0
    case 19: case 20: {
      if (a.ldc % 8) return hipErrorInvalidValue;
      if (knob == 19) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault, 2>), g, b, 0, s, a);
      if (knob == 20) hipLaunchKernelGGL((gemm_bf16_pp3_kernel<false, kGroupM, false, kEpiDefault, 1>), g, b, 0, s, a);
      break;
    }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace gemm3
}  // namespace ntm
