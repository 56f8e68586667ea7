// K1 v5 ("pingpong8p"): persistent pingpong8c. One workgroup per CU walks
// tiles blockIdx.x, blockIdx.x + G, ... (G = grid = #CUs) and keeps the
// LDS-DMA pipeline running ACROSS tile boundaries: the uniform K loop of
// gemm_bf16_pp3.hpp already issues pieces for K-tiles t+1 / t+2, and past the
// end of a tile those are simply the next tile's K-tiles 0 / 1 (its
// "prologue" is absorbed), so the only per-tile cost left is the epilogue.
//
// Why (profiles/r1_pp3_knobs/kfit.log, t = fixed + K * slope at M = N):
//   8192^2: fixed 40 us (ours) vs 28 us (hipBLASLt) for 4 tiles per CU,
// i.e. ~10 us per tile boundary: relaunch ramp + first-data latency + every
// CU storing its 128 KiB C tile at the same moment. Here the stores of tile
// i drain while tile i+1's MFMAs run.
//
// vmcnt with stores in the stream: VMEM loads complete in order, stores may
// complete before older loads. Counted waits stay exact if every wait targets
// loads NEWER than all outstanding stores (pending loads are then a suffix of
// the load stream). So at a boundary: s_waitcnt vmcnt(0) (the in-flight
// pieces are the next tile's first K-tiles, mostly L2 hits and ~1 phase
// old), THEN the epilogue stores; every later wait is for pieces issued after
// them. Pieces past the last tile are dummies into the scratch LDS region,
// exactly as in pingpong8c; the final drain is vmcnt(0) before exit.
//
// Schedule / ordering proof of a tile: identical to gemm_bf16_pp2.hpp
// (RAW distance 6 with vmcnt(10), WAR distance 2); T = K / 64 must be even so
// a tile's K-tile parity equals the global parity and buffers line up across
// tiles. Shape rule: shape_ok3 (K % 128 == 0).
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gemmp {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::kScratch;
using ::ntm::gemm3::shape_ok3;

// Per-lane source pointers (tile-independent part) + the uniform per-tile
// element offsets.
struct PCtx {
  char* lds;
  const __bf16* a_lane;  // A + (w*16 + r) * lda + chunk
  const __bf16* b_lane;  // B + (w*16 + r) * ldb + chunk
  size_t a_hi, b_hi;     // 128 rows further, in elements
  int frag_off;
  int w, wr, wc;
};

struct TileRef {
  size_t a_off, b_off;  // m0 * lda, n0 * ldb (elements)
  int m0, n0;
};

__device__ __forceinline__ TileRef tile_ref(const GemmArgs& p, int tile, int ntiles) {
  int tm, tn;
  tile_coords_of<kGroupM>(tile, ntiles, p.M, p.N, tm, tn);
  return TileRef{(size_t)tm * BM * p.lda, (size_t)tn * BN * p.ldb, tm * BM, tn * BN};
}

// Stage half H of K-tile `kt` (counted from the CURRENT tile's start; kt >= T
// means the next tile) into buffer `buf`, or a dummy piece past the end.
template <int H>
__device__ __forceinline__ void issue_p(const PCtx& c, const TileRef& cur, const TileRef& nxt,
                                        bool has_next, int kt, int T, int buf) {
  const bool in_cur = kt < T;
  const bool real = in_cur || has_next;
  const TileRef& tr = in_cur ? cur : nxt;
  const int k_eff = !real ? T - 1 : (in_cur ? kt : kt - T);
  const bool is_a = (H == kALo || H == kAHi);
  const bool hi = (H == kAHi || H == kBHi);
  const __bf16* base = is_a ? c.a_lane : c.b_lane;
  const size_t off = (is_a ? tr.a_off : tr.b_off) + (hi ? (is_a ? c.a_hi : c.b_hi) : 0) +
                     (size_t)k_eff * BK;
  const __bf16* s = base + off;
  const int loff = real ? buf * kTileBytes + H * kHalfBytes : kScratch;
  char* d = c.lds + loff + (2 * c.w) * 1024;
  glds16(s, d);
  glds16(s + 32, d + 1024);
}

__device__ __forceinline__ void read_a_p(const PCtx& c, bf16x8 (&a)[4][2], int half, int buf) {
  const char* base = c.lds + buf * kTileBytes + half * kHalfBytes + c.frag_off;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      a[mt][ks] = *(const bf16x8*)(base + ((c.wr * 4 + mt) * 2 + ks) * 1024);
}

__device__ __forceinline__ void read_b_p(const PCtx& c, bf16x8 (&b)[2][2], int half, int buf) {
  const char* base = c.lds + buf * kTileBytes + half * kHalfBytes + c.frag_off;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      b[nt][ks] = *(const bf16x8*)(base + ((c.wc * 2 + nt) * 2 + ks) * 1024);
}

template <int P, bool ODD, int F8 = 0>
__device__ __forceinline__ void phase_p(const PCtx& c, Frags3& f, f32x4 (&acc)[2][2][4][2],
                                        const TileRef& cur, const TileRef& nxt,
                                        bool has_next, int t, int T) {
  bf16x8(&bcur)[2][2] = ODD ? f.b1 : f.b0;
  bf16x8(&both)[2][2] = ODD ? f.b0 : f.b1;
  const int b = t & 1;
  if constexpr (P == 0) read_a_p(c, f.a, kALo, b);
  if constexpr (P == 1) read_b_p(c, both, kBHi, b);
  if constexpr (P == 2) read_a_p(c, f.a, kAHi, b);
  if constexpr (P == 3) read_b_p(c, both, kBLo, b ^ 1);  // next K-tile (maybe next tile)
  if constexpr (P == 0) issue_p<kAHi>(c, cur, nxt, has_next, t + 1, T, b ^ 1);
  if constexpr (P == 1) issue_p<kBLo>(c, cur, nxt, has_next, t + 2, T, b);
  if constexpr (P == 2) issue_p<kALo>(c, cur, nxt, has_next, t + 2, T, b);
  if constexpr (P == 3) issue_p<kBHi>(c, cur, nxt, has_next, t + 2, T, b);
  wait_vmcnt<10>();
  raw_barrier();
  if constexpr (F8) {  // K1-fp8 (experimental persistent build, gemm_fp8_diag.hpp knob 6)
    if constexpr (P == 0) mma_quadrant_f8<F8>(acc[0][0], f.a, bcur);
    if constexpr (P == 1) mma_quadrant_f8<F8>(acc[0][1], f.a, both);
    if constexpr (P == 2) mma_quadrant_f8<F8>(acc[1][1], f.a, both);
    if constexpr (P == 3) mma_quadrant_f8<F8>(acc[1][0], f.a, bcur);
  } else {
    if constexpr (P == 0) mma_quadrant<false>(acc[0][0], f.a, bcur);
    if constexpr (P == 1) mma_quadrant<false>(acc[0][1], f.a, both);
    if constexpr (P == 2) mma_quadrant<false>(acc[1][1], f.a, both);
    if constexpr (P == 3) mma_quadrant<false>(acc[1][0], f.a, bcur);
  }
  raw_barrier();
}

template <bool ODD, int F8 = 0>
__device__ __forceinline__ void ktile_p(const PCtx& c, Frags3& f, f32x4 (&acc)[2][2][4][2],
                                        const TileRef& cur, const TileRef& nxt, bool has_next,
                                        int t, int T) {
  phase_p<0, ODD, F8>(c, f, acc, cur, nxt, has_next, t, T);
  phase_p<1, ODD, F8>(c, f, acc, cur, nxt, has_next, t, T);
  phase_p<2, ODD, F8>(c, f, acc, cur, nxt, has_next, t, T);
  phase_p<3, ODD, F8>(c, f, acc, cur, nxt, has_next, t, T);
}

template <bool kRowSum, int EPI = 0, int F8 = 0>
__global__ void __launch_bounds__(kThreads, 2)
    gemm_bf16_pp4_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];
  const int ntiles = (p.M / BM) * (p.N / BN);
  const int G = (int)gridDim.x;
  int tile = (int)blockIdx.x;  // launcher guarantees G <= ntiles

  PCtx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.a_lane = p.A + (size_t)(c.w * 16 + r) * p.lda + cl * 8;
    c.b_lane = p.B + (size_t)(c.w * 16 + r) * p.ldb + cl * 8;
    c.a_hi = (size_t)128 * p.lda;
    c.b_hi = (size_t)128 * p.ldb;
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
  TileRef cur = tile_ref(p, tile, ntiles);
  int nt = tile + G;
  bool has_next = nt < ntiles;
  TileRef nxt = has_next ? tile_ref(p, nt, ntiles) : cur;

  // prologue of the FIRST tile only: B-lo0 A-lo0 B-hi0 A-hi0 B-lo1 A-lo1 B-hi1
  issue_p<kBLo>(c, cur, nxt, has_next, 0, T, 0);
  issue_p<kALo>(c, cur, nxt, has_next, 0, T, 0);
  issue_p<kBHi>(c, cur, nxt, has_next, 0, T, 0);
  issue_p<kAHi>(c, cur, nxt, has_next, 0, T, 0);
  issue_p<kBLo>(c, cur, nxt, has_next, 1, T, 1);
  issue_p<kALo>(c, cur, nxt, has_next, 1, T, 1);
  issue_p<kBHi>(c, cur, nxt, has_next, 1, T, 1);
  wait_vmcnt<10>();
  raw_barrier();
  read_b_p(c, f.b0, kBLo, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger

  while (true) {
    for (int t = 0; t < T; t += 2) {
      ktile_p<false, F8>(c, f, acc, cur, nxt, has_next, t, T);
      ktile_p<true, F8>(c, f, acc, cur, nxt, has_next, t + 1, T);
    }
    if constexpr (F8) mfma_drain();  // asm MFMAs: results land before the VALU reads
    // boundary: retire every load in flight BEFORE any store (see header)
    wait_vmcnt<0>();
    store_tile_epi<kRowSum, EPI>(p, Ctx{c.lds, {}, c.frag_off, c.w, c.wr, c.wc}, acc, cur.m0, cur.n0,
                        lane);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[i][j][m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (!has_next) break;
    tile = nt;
    cur = nxt;
    nt = tile + G;
    has_next = nt < ntiles;
    if (has_next) nxt = tile_ref(p, nt, ntiles);
  }
  if (c.wr == 0) raw_barrier();
  wait_vmcnt<0>();  // dummy pieces: nothing may land after the WG exits
}

inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

// wide = widened nontemporal dwordx4 epilogue (store_tile_wide, needs ldc % 8).
inline hipError_t launch_gemm_bf16_pp4(const GemmArgs& a, hipStream_t stream, bool wide = false) {
  if (!shape_ok3(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % (wide ? 8 : 4)))
    return hipErrorInvalidValue;
  const int ntiles = (a.M / BM) * (a.N / BN);
  int g = cu_count();
  g = g - g % 8;  // keep tile % 8 == blockIdx % 8 (same XCD as the remap assumes)
  if (g <= 0) g = 8;
  if (g > ntiles) g = ntiles;
  if (wide && a.rowsum)
    hipLaunchKernelGGL((gemm_bf16_pp4_kernel<true, kEpiWide | kEpiNT>), dim3(g), dim3(kThreads), 0, stream, a);
  else if (wide)
    hipLaunchKernelGGL((gemm_bf16_pp4_kernel<false, kEpiWide | kEpiNT>), dim3(g), dim3(kThreads), 0, stream, a);
  else if (a.rowsum)
    hipLaunchKernelGGL(gemm_bf16_pp4_kernel<true>, dim3(g), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(gemm_bf16_pp4_kernel<false>, dim3(g), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemmp
}  // namespace ntm
