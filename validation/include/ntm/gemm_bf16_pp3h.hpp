// K1 on ragged one-round C with 192-wide tiles: 192x256 ("pp192x256") and
// 256x192 ("pp256x192") on pingpong8c's 8-wave ping-pong schedule, and
// 224x256 ("pp224x256") for C of 0.86-1.0 rounds of 256x256 tiles.
//
// Why: a C of 150-200 256x256 tiles leaves 60-100 of 256 CUs idle for the
// whole launch. hipBLASLt fills that round with 192-wide macro tiles
// (MT256x192 / MT192x256 in its column-major naming, rocprofv3 trace of
// 3904x2584x12760, 7288x1344x5768, 3512x3456x16040: profiles/r5_h192/), e.g.
// 3904x2584 = 21 x 11 tiles of 192x256 (231 CUs busy, 0.75 of the work per CU)
// instead of 16 x 11 of 256x256 (176 CUs).
//
// Design: pingpong8c (gemm_bf16_pp3.hpp) with one half of A (or B) cut from
// 128 to 64 rows. The tile is still four half-tiles in LDS and four phases
// per K-tile with the same read / issue order; the 64-row half is staged by
// ONE 16-B LDS-DMA piece per lane (wave w: rows 16 (w >> 1) .., k-half w & 1)
// instead of two, is read with half the fragments, and its quadrants run half
// the MFMAs. Because the pieces per phase are no longer uniform, the counted
// vmcnt of phase P is (pieces of all four halves) + (pieces of the half issued
// in P): the loads of the 5 most recent issues stay in flight, so the RAW
// distance (6 phases) and WAR distance (2) of pingpong8c's proof hold
// unchanged. Dummy pieces (K-tiles >= T) go to the scratch region as there.
// A 96-row A-hi half (224x256) is staged like a 128-row one whose waves 6 and
// 7 load dummy pieces into the scratch region, so its counts stay pingpong8c's;
// each wave row then owns 3 of its 16-row m-tiles.
// Accumulators: 96 (192-wide tiles) / 112 (224x256) fp32 x4 per lane, 128 in
// pingpong8c. Epilogue: LDS-staged masked stores of full rows (192- or
// 256-wide), as pingpong8cm.
// Shapes: any M, N % 8, K % 8 (K % 128 != 0: the partial-K build);
// lda / ldb / ldc % 8.
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gemm3h {

using namespace ::ntm::gemm;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::kScratch;

// AH / BH: rows of the A-hi half (128, 96 or 64) / B-hi half (128 or 64); the tile is
// (128 + AH) x (128 + BH).
template <int AH, int BH>
struct Geo {
  static_assert((AH == 128 || AH == 96 || AH == 64) && (BH == 128 || BH == 64), "half rows");
  static constexpr int TM = 128 + AH, TN = 128 + BH;
  static constexpr int kMtHi = AH / 32;  // A-hi m-tiles per wave (16 rows each): 4, 3 or 2
  static constexpr int kNtHi = BH / 64;  // B-hi n-tiles per wave: 2 or 1
  static constexpr int pieces(int h) { return (h == kAHi ? AH : h == kBHi ? BH : 128) == 64 ? 1 : 2; }
  static constexpr int kAll = pieces(kALo) + pieces(kAHi) + pieces(kBLo) + pieces(kBHi);
  // phase P issues A-hi / B-lo / A-lo / B-hi (P = 0 / 1 / 2 / 3)
  static constexpr int vmc(int P) {
    return kAll + pieces(P == 0 ? kAHi : P == 1 ? kBLo : P == 2 ? kALo : kBHi);
  }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 12, "vmcnt range");
  if constexpr (N % 2 == 0) {
    wait_vmcnt<N>();
  } else {
    if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    if constexpr (N == 11) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
  }
}

// Stage half H (ROWS rows) of K-tile kt into buffer buf, or a dummy piece into
// the scratch region if kt >= T. TAIL: chunks starting at k >= K load zeros.
template <int H, int ROWS, bool TAIL>
__device__ __forceinline__ void issue_h(const Ctx& c, int kt, int buf, int T) {
  const bool real = kt < T;
  const int k_eff = real ? kt : T - 1;
  const __bf16* s = c.src[H] + (size_t)k_eff * BK;
  // 96 rows: staged as a 128-row half whose waves 6 and 7 load dummy pieces
  const bool live = ROWS != 96 || c.w < 6;
  const int off = real && live ? buf * kTileBytes + H * kHalfBytes : kScratch;
  if constexpr (ROWS != 64) {
    char* d = c.lds + off + (2 * c.w) * 1024;
    if constexpr (TAIL) {
      const int col = k_eff * BK + c.lane_col;
      glds16(col < c.K ? s : (const __bf16*)kZeroChunk16, d);
      glds16(col + 32 < c.K ? s + 32 : (const __bf16*)kZeroChunk16, d + 1024);
    } else {
      glds16(s, d);
      glds16(s + 32, d + 1024);
    }
  } else {
    // subtile w = (16-row block w >> 1, k-half w & 1); the k-half is already in src
    char* d = c.lds + off + c.w * 1024;
    if constexpr (TAIL) {
      const int col = k_eff * BK + c.lane_col + (c.w & 1) * 32;
      glds16(col < c.K ? s : (const __bf16*)kZeroChunk16, d);
    } else {
      glds16(s, d);
    }
  }
}

template <int H, int MT>
__device__ __forceinline__ void read_a_h(const Ctx& c, bf16x8 (&a)[4][2], int buf) {
  const char* base = c.lds + buf * kTileBytes + H * kHalfBytes + c.frag_off;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      a[mt][ks] = *(const bf16x8*)(base + ((c.wr * MT + mt) * 2 + ks) * 1024);
}

template <int H, int NT>
__device__ __forceinline__ void read_b_h(const Ctx& c, bf16x8 (&b)[2][2], int buf) {
  const char* base = c.lds + buf * kTileBytes + H * kHalfBytes + c.frag_off;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      b[nt][ks] = *(const bf16x8*)(base + ((c.wc * NT + nt) * 2 + ks) * 1024);
}

template <int MT, int NT>
__device__ __forceinline__ void mma_q(f32x4 (&acc)[4][2], const bf16x8 (&a)[4][2],
                                      const bf16x8 (&b)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt][ks], a[mt][ks], acc[mt][nt], 0,
                                                               0, 0);
}

template <int AH, int BH, int P, bool ODD, bool TAIL>
__device__ __forceinline__ void phase_h(const Ctx& c, gemm3::Frags3& f,
                                        f32x4 (&acc)[2][2][4][2], int t, int T) {
  using G = Geo<AH, BH>;
  bf16x8(&bcur)[2][2] = ODD ? f.b1 : f.b0;
  bf16x8(&both)[2][2] = ODD ? f.b0 : f.b1;
  const int cur = t & 1;
  if constexpr (P == 0) read_a_h<kALo, 4>(c, f.a, cur);
  if constexpr (P == 1) read_b_h<kBHi, G::kNtHi>(c, both, cur);
  if constexpr (P == 2) read_a_h<kAHi, G::kMtHi>(c, f.a, cur);
  if constexpr (P == 3) read_b_h<kBLo, 2>(c, both, cur ^ 1);  // tile t+1 (junk at t = T-1)
  if constexpr (P == 0) issue_h<kAHi, AH, TAIL>(c, t + 1, cur ^ 1, T);
  if constexpr (P == 1) issue_h<kBLo, 128, TAIL>(c, t + 2, cur, T);
  if constexpr (P == 2) issue_h<kALo, 128, TAIL>(c, t + 2, cur, T);
  if constexpr (P == 3) issue_h<kBHi, BH, TAIL>(c, t + 2, cur, T);
  wait_vm<G::vmc(P)>();
  raw_barrier();
  if constexpr (P == 0) mma_q<4, 2>(acc[0][0], f.a, bcur);
  if constexpr (P == 1) mma_q<4, G::kNtHi>(acc[0][1], f.a, both);
  if constexpr (P == 2) mma_q<G::kMtHi, G::kNtHi>(acc[1][1], f.a, both);
  if constexpr (P == 3) mma_q<G::kMtHi, 2>(acc[1][0], f.a, bcur);
  raw_barrier();
}

template <int AH, int BH, bool ODD, bool TAIL>
__device__ __forceinline__ void tile_h(const Ctx& c, gemm3::Frags3& f,
                                       f32x4 (&acc)[2][2][4][2], int t, int T) {
  phase_h<AH, BH, 0, ODD, TAIL>(c, f, acc, t, T);
  phase_h<AH, BH, 1, ODD, TAIL>(c, f, acc, t, T);
  phase_h<AH, BH, 2, ODD, TAIL>(c, f, acc, t, T);
  phase_h<AH, BH, 3, ODD, TAIL>(c, f, acc, t, T);
}

// Block -> output tile: tile_coords_of's bijective XCD remap + GROUP_M raster
// on TM x TN tiles; `bid` of `nwg` (blockIdx.x of gridDim.x, or a split-mode
// workgroup's tile index of the tile count).
template <int TM, int TN, int GROUP_M = kGroupM>
__device__ __forceinline__ void tile_coords_of_h(int bid, int nwg, int M, int N, int& tm,
                                                 int& tn) {
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_m = (M + TM - 1) / TM, tiles_n = (N + TN - 1) / TN;
  const int group = GROUP_M * tiles_n;
  const int gid = wgid / group;
  const int first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - gid * group;
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

template <int TM, int TN, int GROUP_M = kGroupM>
__device__ __forceinline__ void tile_coords_h(int M, int N, int& tm, int& tn) {
  tile_coords_of_h<TM, TN, GROUP_M>((int)blockIdx.x, (int)gridDim.x, M, N, tm, tn);
}

// Each lane's source rows are fixed for the whole K loop; clamping them once
// keeps every load in bounds (the clamped rows only feed C rows / columns the
// epilogue does not store). A 64-row half: wave w stages 16-row block w >> 1,
// k-half w & 1 (folded into the source).
template <int AH, int BH>
__device__ __forceinline__ void set_sources_h(const GemmArgs& p, Ctx& c, int m0, int n0,
                                              int lane) {
  const int r = lane >> 2;
  const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
  const int ra = m0 + c.w * 16 + r, rb = n0 + c.w * 16 + r;
  const int ra_hi = AH != 64 ? ra + 128 : m0 + 128 + (c.w >> 1) * 16 + r;
  const int rb_hi = BH == 128 ? rb + 128 : n0 + 128 + (c.w >> 1) * 16 + r;
  const int ka_hi = AH != 64 ? 0 : (c.w & 1) * 32, kb_hi = BH == 128 ? 0 : (c.w & 1) * 32;
  c.src[kALo] = p.A + (size_t)min(ra, p.M - 1) * p.lda + cl * 8;
  c.src[kAHi] = p.A + (size_t)min(ra_hi, p.M - 1) * p.lda + cl * 8 + ka_hi;
  c.src[kBLo] = p.B + (size_t)min(rb, p.N - 1) * p.ldb + cl * 8;
  c.src[kBHi] = p.B + (size_t)min(rb_hi, p.N - 1) * p.ldb + cl * 8 + kb_hi;
}

// K-tiles [t0, t1) (t0 even, t1 > t0 even; pieces at K-tiles >= t1 are dummies)
// accumulated onto acc; drained (vmcnt(0)) on return, stagger balanced.
// prologue: B-lo A-lo B-hi A-hi of t0, B-lo A-lo B-hi of t0 + 1 (virtual phases
// -7..-1; the wait is phase -1's, a B-hi issue: vmc(3))
template <int AH, int BH, bool TAIL>
__device__ __forceinline__ void k_range_h(const GemmArgs& p, const Ctx& c, gemm3::Frags3& f,
                                          f32x4 (&acc)[2][2][4][2], int t0, int t1) {
  using G = Geo<AH, BH>;
  issue_h<kBLo, 128, TAIL>(c, t0, 0, t1);
  issue_h<kALo, 128, TAIL>(c, t0, 0, t1);
  issue_h<kBHi, BH, TAIL>(c, t0, 0, t1);
  issue_h<kAHi, AH, TAIL>(c, t0, 0, t1);
  issue_h<kBLo, 128, TAIL>(c, t0 + 1, 1, t1);
  issue_h<kALo, 128, TAIL>(c, t0 + 1, 1, t1);
  issue_h<kBHi, BH, TAIL>(c, t0 + 1, 1, t1);
  wait_vm<G::vmc(3)>();
  raw_barrier();
  read_b_h<kBLo, 2>(c, f.b0, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger
  int t = t0;
  if constexpr (TAIL) {
    // the zero-filling issue path only where a piece can reach past K
    const int t_real = (p.K + BK - 1) / BK;
    for (; t < t1 && t + 4 < t_real; t += 2) {
      tile_h<AH, BH, false, false>(c, f, acc, t, t1);
      tile_h<AH, BH, true, false>(c, f, acc, t + 1, t1);
    }
    for (; t < t1; t += 2) {
      tile_h<AH, BH, false, true>(c, f, acc, t, t1);
      tile_h<AH, BH, true, true>(c, f, acc, t + 1, t1);
    }
  } else {
    for (; t < t1; t += 2) {
      tile_h<AH, BH, false, false>(c, f, acc, t, t1);
      tile_h<AH, BH, true, false>(c, f, acc, t + 1, t1);
    }
  }
  if (c.wr == 0) raw_barrier();  // balance the stagger
  wait_vmcnt<0>();                // dummy pieces: nothing lands after this
}

// LDS-staged masked epilogue (store_tile_lds's layout, pitch kStagePitch):
// quadrants with two n-tiles per wave leave as 16-B permlane16-swapped rows,
// the one-n-tile B-hi quadrants as 8-B rows; then full TN-wide rows go out
// with nontemporal 16-B stores, rows >= M and 8-column chunks >= N skipped.
template <int AH, int BH>
__device__ __forceinline__ void store_tile_h(const GemmArgs& p, const Ctx& c,
                                             const f32x4 (&acc)[2][2][4][2], int m0, int n0,
                                             int lane) {
  using G = Geo<AH, BH>;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  raw_barrier();
  const int g = lane >> 4;
  const int coff = (g & 1) * 16 + (g >> 1) * 8;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    constexpr int kMt0 = 4;
    const int mts = mh ? G::kMtHi : kMt0;
#pragma unroll
    for (int nh = 0; nh < 2; ++nh) {
      const int nts = nh ? G::kNtHi : 2;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if (mt >= mts) continue;
        const int row = mh * 128 + c.wr * mts * 16 + mt * 16 + (lane & 15);
        if (nts == 2) {
          const int col = nh * 128 + c.wc * 32 + coff;
          const f32x4 v0 = acc[mh][nh][mt][0], v1 = acc[mh][nh][mt][1];
          unsigned w0[2], w1[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const auto r = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v0[2 * h], v0[2 * h + 1]),
                                                            pack_bf16x2(v1[2 * h], v1[2 * h + 1]),
                                                            false, false);
            w0[h] = r[0];
            w1[h] = r[1];
          }
          *(u32x4*)(c.lds + row * kStagePitch + col * 2) = u32x4{w0[0], w0[1], w1[0], w1[1]};
        } else {
          const int col = nh * 128 + c.wc * 16 + (lane >> 4) * 4;
          const f32x4 v = acc[mh][nh][mt][0];
          *(u32x2*)(c.lds + row * kStagePitch + col * 2) =
              u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
        }
      }
    }
  }
  raw_barrier();
  // wave w stores rows (TM / 8) w .. ; two rows per instruction, TN / 8 chunks a row
  constexpr int kRowsPerWave = G::TM / 8;
  constexpr int kChunks = G::TN / 8;
#pragma unroll
  for (int i = 0; i < kRowsPerWave / 2; ++i) {
    const int row = c.w * kRowsPerWave + i * 2 + (lane >> 5);
    const int chunk = lane & 31;
    if (chunk >= kChunks || m0 + row >= p.M || n0 + chunk * 8 >= p.N) continue;
    const u32x4 val = *(const u32x4*)(c.lds + row * kStagePitch + chunk * 16);
    store_c16<1>(p.C + (size_t)(m0 + row) * p.ldc + n0 + chunk * 8, val);
  }
}

template <int AH, int BH, bool TAIL>
__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_pp3h_kernel(GemmArgs p) {
  using G = Geo<AH, BH>;
  static_assert(kLdsBytes3 >= G::TM * kStagePitch, "LDS staging buffer");
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];

  int tm, tn;
  tile_coords_h<G::TM, G::TN>(p.M, p.N, tm, tn);
  const int m0 = tm * G::TM, n0 = tn * G::TN;

  Ctx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  set_sources_h<AH, BH>(p, c, m0, n0, lane);
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

  gemm3::Frags3 f;
  // partial-K build: ceil(K / 64) K-tiles rounded up to an even count
  const int T = TAIL ? ((p.K + 2 * BK - 1) / (2 * BK)) * 2 : p.K / BK;
  if constexpr (TAIL) {
    c.K = p.K;
    const int r = lane >> 2;
    c.lane_col = ((lane & 3) ^ (((r >> 3) & 1) << 1)) * 8;
  }
  k_range_h<AH, BH, TAIL>(p, c, f, acc, 0, T);
  store_tile_h<AH, BH>(p, c, acc, m0, n0, lane);
}

inline bool shape_ok_h(int M, int N, int K) {
  return M > 0 && N > 0 && (N % 8) == 0 && K > 0 && (K % 8) == 0;
}

template <int AH, int BH>
inline hipError_t launch_gemm_bf16_pp3h(const GemmArgs& a, hipStream_t stream) {
  using G = Geo<AH, BH>;
  if (!shape_ok_h(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)(((a.M + G::TM - 1) / G::TM) * ((a.N + G::TN - 1) / G::TN))), b(kThreads);
  if (a.K % (2 * BK))
    hipLaunchKernelGGL((gemm_bf16_pp3h_kernel<AH, BH, true>), g, b, 0, stream, a);
  else
    hipLaunchKernelGGL((gemm_bf16_pp3h_kernel<AH, BH, false>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemm3h
}  // namespace ntm
