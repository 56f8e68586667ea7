// EXPERIMENTAL (libntm_experimental.so): "pingpong8or" - pingpong8o
// (gemm_bf16_pp6.hpp) with the LDS-DMA and the C stores split between the two
// wave rows, so that no wave that waits on LDS-DMA ever issues a store.
//
// Why (profiles/r3_stores): storing C costs 2.2 % of the 8192^3 time (6.5 % at
// 8192x8192x4096). Loads, stores and LDS-DMA retire vmcnt in issue order, so in
// pingpong8o a counted wait for a piece issued after a tile's C stores also
// waits for those stores, and the K loop stalls until they drain. Here:
//  * wave row 0 issues ALL the LDS-DMA: its own 16 rows of each half and those
//    of the row-1 wave below it (4 glds16 per load segment instead of 2; the
//    counted wait is vmcnt(20) = 5 phases x 4), and never stores C;
//  * wave row 1 issues no DMA, never waits on vmcnt, and stores all of C. At
//    each boundary quadrant row 0 packs its quadrant to bf16, writes it into
//    the 16 KiB scratch region (the dummy-piece target, free while a next tile
//    exists: dummies only run on a CU's last tile, which stores nothing at a
//    boundary) and waits lgkmcnt(0); the phase's mid barrier publishes it. Row 1,
//    whose load segment runs half a phase later (ping-pong stagger), reads it
//    back in the same lane layout and stores it beside its own quadrant. Row 0
//    rewrites the scratch only in its next load segment, after the barrier that
//    row 1 reaches once it has consumed the reads.
// Results are bitwise equal to pingpong8o / pingpong8c (same MFMAs, same order).
#pragma once

#include "ntm/gemm_bf16_pp6.hpp"

namespace ntm {
namespace gemm7 {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::kScratch;
using ::ntm::gemm6::Edge;
using ::ntm::gemm6::mma_q;
using ::ntm::gemm6::shape_ok6;
using ::ntm::gemm6::tile_origin;
using ::ntm::gemm6::wait_vm;
using ::ntm::gemm6::zero_quadrant;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Ctx7 {
  long rows64[4];  // 64 rows of each half's operand, in elements (row 0's second piece pair)
};

// Row 0 only: the pieces of half H of K-tile kt for this wave's 16 rows and for
// the 16 rows of the row-1 wave w + 4 (64 rows below, LDS 8 KiB further).
template <int H, bool NX>
__device__ __forceinline__ void issue7(const Ctx& c, const Ctx7& c7, int kt, int buf, int T,
                                       bool has_next, long dA, long dB) {
  const __bf16* s;
  int off = buf * kTileBytes + H * kHalfBytes;
  if constexpr (!NX) {
    s = c.src[H] + (size_t)kt * BK;
  } else {
    const long d = (H == kALo || H == kAHi) ? dA : dB;
    s = c.src[H] + (has_next ? d + (long)(kt - T) * BK : (long)(T - 1) * BK);
    off = has_next ? off : kScratch;
  }
  char* d = c.lds + off + (2 * c.w) * 1024;
  glds16(s, d);
  glds16(s + 32, d + 1024);
  glds16(s + c7.rows64[H], d + 8 * 1024);
  glds16(s + c7.rows64[H] + 32, d + 9 * 1024);
}

// Row 0: its quadrant, packed as store_quadrant packs it, into scratch block wc.
__device__ __forceinline__ void park_quadrant(const Ctx& c, const f32x4 (&q)[4][2], int lane) {
  const int g = lane >> 4;
  const int coff = (g & 1) * 16 + (g >> 1) * 8;
  char* blk = c.lds + kScratch + c.wc * 4096 + (lane & 15) * 64 + coff * 2;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const f32x4 v0 = q[mt][0], v1 = q[mt][1];
    unsigned w0[2], w1[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const auto r = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v0[2 * h], v0[2 * h + 1]),
                                                      pack_bf16x2(v1[2 * h], v1[2 * h + 1]),
                                                      false, false);
      w0[h] = r[0];
      w1[h] = r[1];
    }
    *(u32x4*)(blk + mt * 16 * 64) = u32x4{w0[0], w0[1], w1[0], w1[1]};
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // parked before the mid barrier
}

// Row 1: the row-0 quadrant above it (scratch block wc) to C, then its own.
template <int MH, int NH, int POL>
__device__ __forceinline__ void store_pair(const GemmArgs& p, const Ctx& c, const f32x4 (&q)[4][2],
                                          int m0, int n0, int c_lane, int lane) {
  const int g = lane >> 4;
  const int coff = (g & 1) * 16 + (g >> 1) * 8;
  const char* blk = c.lds + kScratch + c.wc * 4096 + (lane & 15) * 64 + coff * 2;
  __bf16* tile = p.C + (size_t)(m0 + MH * 128) * p.ldc + (n0 + NH * 128);
  const int c_up = c_lane - 64 * p.ldc;  // the row-0 wave's rows
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
    store_c16<POL>(tile + (size_t)mt * 16 * p.ldc + c_up, *(const u32x4*)(blk + mt * 16 * 64));
  ::ntm::gemm6::store_quadrant<MH, NH, POL>(p, q, m0, n0, c_lane);
}

// One phase (phase6 of gemm_bf16_pp6.hpp with the row roles above). CONV: the
// quadrant that leaves in this phase when ON (-1 none; 3 = the previous tile's).
template <int P, bool ODD, int CONV, bool NX, int POL>
__device__ __forceinline__ void phase7(const GemmArgs& p, const Ctx& c, const Ctx7& c7, Frags3& f,
                                       f32x4 (&acc)[2][2][4][2], int t, int T, const Edge& e,
                                       bool on, int c_lane, int lane) {
  bf16x8(&bcur)[2][2] = ODD ? f.b1 : f.b0;
  bf16x8(&both)[2][2] = ODD ? f.b0 : f.b1;
  const int cur = t & 1;
  if constexpr (P == 0) read_a<kALo>(c, f.a, cur);
  if constexpr (P == 1) read_b<kBHi>(c, both, cur);
  if constexpr (P == 2) read_a<kAHi>(c, f.a, cur);
  if constexpr (P == 3) read_b<kBLo>(c, both, cur ^ 1);
  if (c.wr == 0) {
    if constexpr (P == 0) issue7<kAHi, NX>(c, c7, t + 1, cur ^ 1, T, e.has_next, e.dA, e.dB);
    if constexpr (P == 1) issue7<kBLo, NX>(c, c7, t + 2, cur, T, e.has_next, e.dA, e.dB);
    if constexpr (P == 2) issue7<kALo, NX>(c, c7, t + 2, cur, T, e.has_next, e.dA, e.dB);
    if constexpr (P == 3) issue7<kBHi, NX>(c, c7, t + 2, cur, T, e.has_next, e.dA, e.dB);
    wait_vm<20>();
  }
  if constexpr (CONV >= 0) {
    if (on) {
      constexpr int MH = (CONV == 2 || CONV == 3) ? 1 : 0;
      constexpr int NH = (CONV == 1 || CONV == 2) ? 1 : 0;
      if (c.wr == 0)
        park_quadrant(c, acc[MH][NH], lane);
      else
        store_pair<MH, NH, POL>(p, c, acc[MH][NH], CONV == 3 ? e.pm0 : e.m0,
                                CONV == 3 ? e.pn0 : e.n0, c_lane, lane);
      zero_quadrant(acc[MH][NH]);
    }
  }
  raw_barrier();
  if constexpr (P == 0) mma_q(acc[0][0], f.a, bcur);
  if constexpr (P == 1) mma_q(acc[0][1], f.a, both);
  if constexpr (P == 2) mma_q(acc[1][1], f.a, both);
  if constexpr (P == 3) mma_q(acc[1][0], f.a, bcur);
  raw_barrier();
}

#define NTM_PH7(P, ODD, CV, NX, ON) \
  phase7<P, ODD, CV, NX, POL>(p, c, c7, f, acc, t, T, e, ON, c_lane, lane)

template <int POL>
__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_pp7_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];
  const int ntiles = (p.M / BM) * (p.N / BN);
  const int G = (int)gridDim.x;
  int tile = (int)blockIdx.x;

  Ctx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  Ctx7 c7;
  c7.rows64[kALo] = c7.rows64[kAHi] = 64l * p.lda;
  c7.rows64[kBLo] = c7.rows64[kBHi] = 64l * p.ldb;
  Edge e;
  tile_origin(p, tile, ntiles, e.m0, e.n0);
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    const __bf16* a0 = p.A + (size_t)(e.m0 + c.w * 16 + r) * p.lda + cl * 8;
    const __bf16* b0 = p.B + (size_t)(e.n0 + c.w * 16 + r) * p.ldb + cl * 8;
    c.src[kALo] = a0;
    c.src[kAHi] = a0 + (size_t)128 * p.lda;
    c.src[kBLo] = b0;
    c.src[kBHi] = b0 + (size_t)128 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
  const int c_lane = (c.wr * 64 + (lane & 15)) * p.ldc + c.wc * 32 +
                     ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) zero_quadrant(acc[i][j]);
  Frags3 f;
  const int T = p.K / BK;
  e.prev = false;
  e.pm0 = e.pn0 = 0;
  int nm0 = 0, nn0 = 0;
  e.has_next = tile + G < ntiles;
  e.dA = e.dB = 0;
  if (e.has_next) {
    tile_origin(p, tile + G, ntiles, nm0, nn0);
    e.dA = (long)(nm0 - e.m0) * p.lda;
    e.dB = (long)(nn0 - e.n0) * p.ldb;
  }

  // prologue of the first tile: B-lo0 A-lo0 B-hi0 A-hi0 B-lo1 A-lo1 B-hi1, all by row 0
  if (c.wr == 0) {
    issue7<kBLo, false>(c, c7, 0, 0, T, false, 0, 0);
    issue7<kALo, false>(c, c7, 0, 0, T, false, 0, 0);
    issue7<kBHi, false>(c, c7, 0, 0, T, false, 0, 0);
    issue7<kAHi, false>(c, c7, 0, 0, T, false, 0, 0);
    issue7<kBLo, false>(c, c7, 1, 1, T, false, 0, 0);
    issue7<kALo, false>(c, c7, 1, 1, T, false, 0, 0);
    issue7<kBHi, false>(c, c7, 1, 1, T, false, 0, 0);
    wait_vm<20>();
  }
  raw_barrier();
  read_b<kBLo>(c, f.b0, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger

  for (;;) {
    int t = 0;
    NTM_PH7(0, false, 3, false, e.prev);
    NTM_PH7(1, false, -1, false, e.prev);
    NTM_PH7(2, false, -1, false, e.prev);
    NTM_PH7(3, false, -1, false, e.prev);
    t = 1;
    NTM_PH7(0, true, -1, false, e.prev);
    NTM_PH7(1, true, -1, false, e.prev);
    NTM_PH7(2, true, -1, false, e.prev);
    NTM_PH7(3, true, -1, false, e.prev);
#pragma nounroll
    for (t = 2; t < T - 2; t += 2) {
      NTM_PH7(0, false, -1, false, false);
      NTM_PH7(1, false, -1, false, false);
      NTM_PH7(2, false, -1, false, false);
      NTM_PH7(3, false, -1, false, false);
      ++t;
      NTM_PH7(0, true, -1, false, false);
      NTM_PH7(1, true, -1, false, false);
      NTM_PH7(2, true, -1, false, false);
      NTM_PH7(3, true, -1, false, false);
      --t;
    }
    t = T - 2;
    NTM_PH7(0, false, -1, false, false);
    NTM_PH7(1, false, -1, true, false);
    NTM_PH7(2, false, -1, true, false);
    NTM_PH7(3, false, -1, true, false);
    t = T - 1;
    NTM_PH7(0, true, -1, true, false);
    NTM_PH7(1, true, 0, true, e.has_next);
    NTM_PH7(2, true, 1, true, e.has_next);
    NTM_PH7(3, true, 2, true, e.has_next);
    if (!e.has_next) break;
#pragma unroll
    for (int h = 0; h < 4; ++h) c.src[h] += (h == kALo || h == kAHi) ? e.dA : e.dB;
    e.pm0 = e.m0;
    e.pn0 = e.n0;
    e.m0 = nm0;
    e.n0 = nn0;
    e.prev = true;
    tile += G;
    e.has_next = tile + G < ntiles;
    if (e.has_next) {
      tile_origin(p, tile + G, ntiles, nm0, nn0);
      e.dA = (long)(nm0 - e.m0) * p.lda;
      e.dB = (long)(nn0 - e.n0) * p.ldb;
    }
  }
  if (c.wr == 0) raw_barrier();  // balance the stagger
  wait_vm<0>();                  // row 0: dummy pieces; row 1: its C stores
  store_tile_lds<false, POL == 1, false, POL>(p, c, acc, e.m0, e.n0, lane);
}
#undef NTM_PH7

template <int POL>
inline hipError_t launch_gemm_bf16_pp7(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok6(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8))
    return hipErrorInvalidValue;
  const int ntiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((gemm_bf16_pp7_kernel<POL>), dim3((unsigned)::ntm::gemm6::pp6_grid(ntiles)),
                     dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemm7
}  // namespace ntm
