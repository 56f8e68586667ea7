// Stream-K split mode on the 192-wide ping-pong tiles ("pp192x256s" /
// "pp256x192s"): gemm_bf16_sk.hpp's split mode (each tile cut into S equal K
// slices, all slices of a tile on one XCD in one round, wait-free fix-up) with
// gemm_bf16_pp3h.hpp's 192x256 / 256x192 tile as the segment body.
//
// Why: split mode serves C of at most half a round of 256x256 tiles with a long
// K. Where the XCD's tile count does not divide its 32 CUs, a third of them
// idle: 4152x1096x16056 is 85 tiles = 11 per XCD, so S = 2 and 22 of 32 CUs are
// busy. On 192-wide tiles the same C is 110 tiles = 14 per XCD:
// S = 2 still, but 28 of 32 CUs busy, each with 0.75 of the work.
//
// Everything but the tile geometry is gemm_bf16_sks_kernel's: slice q of tile
// v runs K-tile pairs [q Tp / S, (q + 1) Tp / S); S = 2 uses the head / tail
// protocol (one partial write and one read per tile), S >= 3 the S-slice
// counter (count + XCC id + its square), both checking that every part ran on
// the combiner's XCD (kErrWord). The partial layout is the 256x256 one with the
// unused accumulators of the 64-row half skipped, so a slot keeps the same size
// and the workspace (sk_ws_bytes) is the 256x256 kernel's.
#pragma once

#include "ntm/gemm_bf16_pp3h.hpp"
#include "ntm/gemm_bf16_sk.hpp"

namespace ntm {
namespace gemmskh {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::kLdsBytes3;
using namespace ::ntm::gemmsk;
using ::ntm::gemm3h::Geo;

// Split mode only: every XCD's TM x TN tiles fit its CUs at least twice.
template <int TM, int TN>
__host__ __device__ inline bool sk_decompose_h(int M, int N, int K, int cus, SkArgs& s) {
  if (M <= 0 || N <= 0 || K <= 0 || cus < 8 || (cus % 8) != 0 || cus + 8 > kErrWord) return false;
  s.ntiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  s.G = cus;
  s.Tp = (K + 2 * BK - 1) / (2 * BK);
  s.D = 0;
  s.S = 0;
  if (s.ntiles > s.G) return false;
  const int per_xcd = (s.ntiles + 7) / 8, W = s.G / 8;
  int S = W / per_xcd;
  if (S > kMaxSlices) S = kMaxSlices;
  if (S > s.Tp) S = s.Tp;
  if (S < 2) return false;
  s.S = S;
  return true;
}

// The accumulators the tile uses: the A-hi (mh = 1) half has kMtHi m-tiles per
// wave, the B-hi (nh = 1) half kNtHi n-tiles.
template <int AH, int BH>
__device__ __forceinline__ constexpr bool used(int i, int j, int m, int n) {
  return (i == 0 || m < Geo<AH, BH>::kMtHi) && (j == 0 || n < Geo<AH, BH>::kNtHi);
}

template <int AH, int BH>
__device__ __forceinline__ void write_partial_h(float* dst, const f32x4 (&acc)[2][2][4][2]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)kPartialBytes, 0x00020000);
  const int off = (int)threadIdx.x * 16;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          if (used<AH, BH>(i, j, m, n))
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j][m][n]), rsrc,
                                                   off + (((i * 2 + j) * 4 + m) * 2 + n) * kThreads * 16,
                                                   0, 16);
}

template <int AH, int BH>
__device__ __forceinline__ void add_partial_h(const float* src, f32x4 (&acc)[2][2][4][2]) {
  const f32x4* s = (const f32x4*)src + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          if (used<AH, BH>(i, j, m, n)) acc[i][j][m][n] += s[(((i * 2 + j) * 4 + m) * 2 + n) * kThreads];
      __builtin_amdgcn_sched_barrier(0);
    }
}

template <int AH, int BH, bool TAIL, bool PAIR>
__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_sksh_kernel(GemmArgs p, SkArgs s) {
  using G = Geo<AH, BH>;
  static_assert(kLdsBytes3 >= G::TM * kStagePitch, "LDS staging buffer");
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3 + 16];  // ONE __shared__ array
  int* bcast = (int*)(smem + kLdsBytes3);
  const int b = (int)blockIdx.x;
  const int x = b & 7, j = b >> 3;
  const int nx = (s.ntiles - x + 7) >> 3;
  if (nx <= 0 || j >= nx * s.S) return;  // uniform: the whole workgroup leaves
  const int slice = j / nx, k = j - slice * nx;
  const int tile = x + 8 * k;
  Ctx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
  if constexpr (TAIL) {
    c.K = p.K;
    const int r = lane >> 2;
    c.lane_col = ((lane & 3) ^ (((r >> 3) & 1) << 1)) * 8;
  }
  int tm, tn;
  gemm3h::tile_coords_of_h<G::TM, G::TN>(tile, s.ntiles, p.M, p.N, tm, tn);
  const int m0 = __builtin_amdgcn_readfirstlane(tm * G::TM);
  const int n0 = __builtin_amdgcn_readfirstlane(tn * G::TN);
  gemm3h::set_sources_h<AH, BH>(p, c, m0, n0, lane_now());
  Frags3 f;
  f32x4 acc[2][2][4][2];
  zero_acc(acc);
  const int pa = slice * s.Tp / s.S, pb = (slice + 1) * s.Tp / s.S;
  gemm3h::k_range_h<AH, BH, TAIL>(p, c, f, acc, 2 * pa, 2 * pb);
  float* part = s.ws + (kCounterBytes + (size_t)tile * s.S * kPartialBytes) / 4;
  unsigned* cnt = s.cnt + tile;
  if constexpr (PAIR) {
    // S = 2: the head / tail protocol (slice 0 = head, the writer)
    const bool tail = slice == 1;
    const unsigned arrive = tail ? 4u : 1u, written = arrive << 1;
    const unsigned other_written = tail ? 2u : 8u;
    const unsigned xc = xcc_id() ^ (tail ? 0u : s.fault);
    const unsigned tag = (xc + 1u) << (tail ? kTailTagShift : kHeadTagShift);
    float* mine = part + (tail ? kPartialBytes / 4 : 0);
    const float* other = part + (tail ? 0 : kPartialBytes / 4);
    unsigned o = tail ? counter_add<false>(cnt, arrive + tag, bcast) : 0u;
    if (!(o & other_written)) {
      write_partial_h<AH, BH>(mine, acc);
      o = counter_add<true>(cnt, written + (tail ? 0u : tag), bcast);
    }
    if (!(o & other_written)) return;  // uniform: the other slice combines
    const unsigned other_xcc = ((o >> (tail ? kHeadTagShift : kTailTagShift)) & 0xFFu) - 1u;
    if (other_xcc != xc)
      report_xcc_error(s.cnt, 1u << 28 | (unsigned)(tile & 0xFFFF) << 8 | (xc & 0xF) << 4 |
                                  (other_xcc & 0xF));
    acquire_all();
    add_partial_h<AH, BH>(other, acc);
    reset_counter(cnt);
    gemm3h::store_tile_h<AH, BH>(p, c, acc, m0, n0, lane_now());
    return;
  }
  write_partial_h<AH, BH>(part + (size_t)slice * (kPartialBytes / 4), acc);
  const unsigned xc = xcc_id() ^ (slice == 0 ? s.fault : 0u);
  const unsigned tag = 1u + (xc << 8) + ((xc * xc) << 16);
  const unsigned o = counter_add<true>(cnt, tag, bcast);
  if ((o & 0xFFu) != (unsigned)(s.S - 1)) return;  // uniform
  const unsigned all = o + tag, S = (unsigned)s.S;
  if (((all >> 8) & 0xFFu) != S * xc || (all >> 16) != S * xc * xc)
    report_xcc_error(s.cnt, 1u << 28 | (unsigned)(tile & 0xFFFF) << 8 | (xc & 0xF) << 4);
  acquire_all();
  zero_acc(acc);
  for (int q = 0; q < s.S; ++q) add_partial_h<AH, BH>(part + (size_t)q * (kPartialBytes / 4), acc);
  reset_counter(cnt);
  gemm3h::store_tile_h<AH, BH>(p, c, acc, m0, n0, lane_now());
}

// Launch on `cus` workgroups with a stream-K workspace (sk_ws_bytes(cus); its
// counter block zero on entry, left zero). hipErrorInvalidValue where split
// mode on this tile does not serve (M, N, K).
template <int AH, int BH>
inline hipError_t launch_gemm_bf16_skh(const GemmArgs& a, int cus, void* ws, size_t ws_bytes,
                                       hipStream_t stream, int fault = -1) {
  using G = Geo<AH, BH>;
  SkArgs s;
  if (!shape_ok_sk(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) ||
      !sk_decompose_h<G::TM, G::TN>(a.M, a.N, a.K, cus, s) || ws == nullptr ||
      ws_bytes < sk_ws_bytes(s.G) || (reinterpret_cast<size_t>(ws) % 16))
    return hipErrorInvalidValue;
  s.ws = (float*)ws;
  s.cnt = (unsigned*)ws;
  s.fault = fault < 0 ? sk_fault_inject() : (unsigned)fault;  // -1: the process-wide value
  const dim3 g((unsigned)s.G), blk(kThreads);
  const bool pair = s.S == 2;
  if (a.K % (2 * BK)) {
    if (pair)
      hipLaunchKernelGGL((gemm_bf16_sksh_kernel<AH, BH, true, true>), g, blk, 0, stream, a, s);
    else
      hipLaunchKernelGGL((gemm_bf16_sksh_kernel<AH, BH, true, false>), g, blk, 0, stream, a, s);
  } else {
    if (pair)
      hipLaunchKernelGGL((gemm_bf16_sksh_kernel<AH, BH, false, true>), g, blk, 0, stream, a, s);
    else
      hipLaunchKernelGGL((gemm_bf16_sksh_kernel<AH, BH, false, false>), g, blk, 0, stream, a, s);
  }
  return hipGetLastError();
}

}  // namespace gemmskh
}  // namespace ntm
