// EXPERIMENTAL (libntm_experimental.so only): pingpong8c / K1-fp8 with the
// XCDs' tile boundaries desynchronised by split first tiles - a timing study
// of profiles/r3_stores (C stores cost 2-17 % because every CU stores its
// tile at the same moment and in-order vmcnt holds the next loads behind them).
//
// Work items, per XCD group x = blockIdx & 7 (blocks are dealt round-robin to
// the 8 XCDs), item j = blockIdx >> 3 of that group's sequence:
//   j <  S          head of split tile j: K-tiles [0, kh_x)
//   S <= j < q      full tile j
//   q <= j < q + S  tail of split tile j - q: K-tiles [kh_x, T)
// with q = tiles / 8 the XCD's tiles (the bijective XCD remap's chunk, same
// tile -> XCD map and group-M raster as the data-parallel kernel), S = 32 (one
// split tile per CU of the XCD) and kh_x = x T / 8 rounded down to even: XCD
// x starts x/8 of a tile out of phase with XCD 0 and stays so, and every CU
// still does exactly q / 32 tiles of work (a head and a tail make one tile).
// MODE 0 (timing only, wrong C): heads store nothing and tails store their
// part of the sum - the partial-sum hand-off is not built; this bounds what
// desynchronised boundaries can recover before paying for it.
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gdsync {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::kEpiDefault;
using ::ntm::gemm3::kLdsBytes3;

constexpr int kSplitPerXcd = 32;

template <int F8>
__global__ void __launch_bounds__(kThreads, 2) gemm_desync_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];
  const int ntiles = (p.M / BM) * (p.N / BN);
  const int q = ntiles >> 3;
  const int x = (int)(blockIdx.x & 7u), j = (int)(blockIdx.x >> 3);
  const int Tfull = p.K / BK;
  int kh = ((x * Tfull / 8) / 2) * 2;
  if (kh < 2 || Tfull - kh < 2) kh = 0;
  int tl, k0, T;
  bool store;
  if (j < kSplitPerXcd) {
    if (kh == 0) return;  // XCD 0 (or a K too short to split): its split tiles run whole as tails
    tl = j, k0 = 0, T = kh, store = false;
  } else if (j < q) {
    tl = j, k0 = 0, T = Tfull, store = true;
  } else {
    tl = j - q, k0 = kh, T = Tfull - kh, store = true;
  }
  int tm, tn;
  tile_coords_of<kGroupM>((tl << 3) | x, ntiles, p.M, p.N, tm, tn);
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
    const __bf16* a0 = p.A + (size_t)(m0 + c.w * 16 + r) * p.lda + cl * 8 + (size_t)k0 * BK;
    const __bf16* b0 = p.B + (size_t)(n0 + c.w * 16 + r) * p.ldb + cl * 8 + (size_t)k0 * BK;
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
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][jj][m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  Frags3 f;
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
  if (c.wr == 1) raw_barrier();  // ping-pong stagger
  for (int t = 0; t < T; t += 2) {
    ::ntm::gemm3::tile3<false, false, F8>(c, f, acc, t, T);
    ::ntm::gemm3::tile3<true, false, F8>(c, f, acc, t + 1, T);
  }
  if constexpr (F8) mfma_drain();
  if (c.wr == 0) raw_barrier();
  wait_vmcnt<0>();
  if (store || p.ldc < 0)  // heads: no store (the impossible ldc keeps the MFMAs live)
    store_tile_epi<false, kEpiDefault>(p, c, acc, m0, n0, lane);
}

inline bool desync_shape_ok(const GemmArgs& a) {
  const int ntiles = (a.M / BM) * (a.N / BN);
  return a.M > 0 && a.N > 0 && a.M % BM == 0 && a.N % BN == 0 && a.K % (2 * BK) == 0 &&
         a.K >= 8 * BK && ntiles % 8 == 0 && ntiles / 8 >= kSplitPerXcd && a.ldc % 8 == 0 &&
         !a.rowsum;
}

// bf16 (F8 = 0) or e4m3 bytes in bf16-sized pairs (F8 = 3: K, lda, ldb halved by the caller).
template <int F8>
inline hipError_t launch_gemm_desync(const GemmArgs& a, hipStream_t s) {
  if (!desync_shape_ok(a)) return hipErrorInvalidValue;
  const int q = (a.M / BM) * (a.N / BN) / 8;
  hipLaunchKernelGGL((gemm_desync_kernel<F8>), dim3((unsigned)(8 * (q + kSplitPerXcd))),
                     dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace gdsync
}  // namespace ntm
