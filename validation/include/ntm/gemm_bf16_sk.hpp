// K1 stream-K tiles: the wave-specialised tile kernel (gemm_bf16_tile_ws_kernel,
// gemm_bf16_t128.hpp) run persistently over an even split of ALL K-tile
// iterations of the GEMM, for shapes whose tile count is a poor multiple of
// the 256 CUs.
//
// Why: at 3200^3 the 160x160 tile gives 400 tiles = 1.56 rounds, so the
// second round runs 144 workgroups on 256 CUs and K1 trailed hipBLASLt by 6 %
// (profiles/r2_ws/policy_default.log); hipBLASLt's kernels there are stream-K
// builds ("SK3" in their names, profiles/r2_ws/tiles_kernel_stats.csv).
//
// Work split, XCD-local: the tiles (in the tile kernel's group-M order) are
// dealt to the 8 XCDs as 8 contiguous ranges of whole tiles; the Gx = G / 8
// workgroups of XCD x (blockIdx % 8 == x, index j = blockIdx / 8) split that
// range's units (tile, K-tile) evenly: workgroup j takes
// [j Ux / Gx, (j+1) Ux / Gx) of its XCD's Ux = tiles_x T units. The host
// requires Ux / Gx >= T, so a tile meets at most two ranges: a HEAD segment
// [0, a) at the end of range j and a TAIL segment [a, T) at the start of range
// j+1 - both on the same XCD, so the partial moves through that XCD's L2.
// A range is walked in unit order, so every tail is computed first in its
// workgroup and every head last:
//   full segment [0, T): store C (bf16) as the tile kernel does;
//   tail [a, T): store each consumer wave's fp32 partial to slot blockIdx,
//     s_waitcnt vmcnt(0) (the stores reached the XCD's L2), then
//     flag[blockIdx][wave] = epoch (device-scope store);
//   head [0, a): poll flag[blockIdx + 8][wave] >= epoch, read that slot
//     (never read before in this launch, so no stale L1 line; the L2 is
//     shared by the XCD), add, store C.
// No agent-scope fences: on gfx950 they compile to buffer_wbl2 / buffer_inv
// of the whole XCD L2, costing every workgroup on the XCD its cached A/B
// panels; and partials crossing XCDs would need device-scope dword traffic
// (both measured: 400-580 TF/s at 3200^3 instead of ~1000).
// The head waits for a tail that its partner computed at the START of its
// range, so the wait is short; every spin is bounded. The same consumer wave
// index owns the same output block in both workgroups, so partials pair up
// wave by wave with no workgroup-level sync. Epochs only grow (one per launch,
// host counter), so flags never need resetting.
//
// Per segment both roles run the tile kernel's pipeline on [kb, ke): the
// producer prologue issues tiles kb .. kb+S-2 (dummies past ke re-read tile
// ke-1 into scratch), one barrier per K-tile, and one extra barrier at the
// segment end so no consumer still reads the ring (the stale "tile ke" reads
// of its last iteration) when the producers start the next segment's prologue.
// That prologue then overlaps the consumers' epilogue.
// A split tile's sum is (head partial) + (tail partial) instead of one
// sequential chain: results are within the fp32-accumulation tolerance, not
// bitwise equal to the tile kernel.
#pragma once

#include "ntm/gemm_bf16_t128.hpp"

namespace ntm {
namespace gemmsk {

using ::ntm::gemm::GemmArgs;
using namespace ::ntm::gemmt;

constexpr unsigned kSkSpinLimit = 1u << 22;  // ~0.3 s of s_sleep polling

struct SkArgs {
  GemmArgs g;
  f32x4* part;      // [G][4 waves][MT NT][64 lanes] fp32 partials
  unsigned* flags;  // [G][4 waves]
  unsigned epoch;
  int T;            // K-tiles per tile
  long long units;  // tiles x T
  int diag;         // diagnostics only (0 in every real call): bit 0 skip the head's
                    // wait, bit 1 skip the tail's partial store + flag
};

template <int MT, int NT>
__device__ __forceinline__ void tile_mn(int tile, int M, int N, int& tm, int& tn) {
  const int tiles_m = M / Cfg<MT, NT>::TM, tiles_n = N / Cfg<MT, NT>::TN;
  const int group = kGroupMT * tiles_n;
  const int gid = tile / group;
  const int first_m = gid * kGroupMT;
  const int gsz = min(tiles_m - first_m, kGroupMT);
  const int in_group = tile - gid * group;
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

// LDS-DMA piece `piece` of logical K-step i (ring slot i % S) of a segment of
// n K-steps whose step i reads K-tile (k0 + i) mod T; i >= n: a dummy piece
// (re-reads the segment's last K-tile into this wave's scratch).
template <int MT, int NT>
__device__ __forceinline__ void issue_piece_rot(const CtxT& c, int i, int n, int k0, int T,
                                                int piece) {
  using C = Cfg<MT, NT>;
  const bool real = i < n;
  int kt = k0 + (real ? i : n - 1);
  if (kt >= T) kt -= T;
  const bool is_a = piece < MT;
  const int g = is_a ? c.w * MT + piece : c.w * NT + (piece - MT);
  const int rb = g >> 1, kh = g & 1;
  const size_t koff = (size_t)kt * TK + kh * 32;
  char* slot = c.lds + (i % C::S) * C::kSlot;
  const __bf16* src = (is_a ? c.a_src + rb * c.a_rb16 : c.b_src + rb * c.b_rb16) + koff;
  char* dst = real ? slot + (is_a ? 0 : C::kA) + (rb * 2 + kh) * 1024
                   : c.lds + C::kScratch + c.w * 1024;
  glds16(src, dst);
}

// C store of one consumer wave's block, optionally adding a tail partial
// (the accumulators are only read: a VALU write would move them to VGPRs).
template <int MT, int NT, bool ADD>
__device__ __forceinline__ void store_c(const GemmArgs& p, const CtxT& c, const f32x4 (&acc)[MT][NT],
                                        const f32x4* part, int m0, int n0, int lane) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int row = m0 + c.wr * (16 * MT) + mt * 16 + (lane & 15);
      const int col = n0 + c.wc * (16 * NT) + nt * 16 + (lane >> 4) * 4;
      f32x4 v = acc[mt][nt];
      if constexpr (ADD) v += part[(mt * NT + nt) * 64 + lane];
      bf16x4 o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      *(bf16x4*)(p.C + (size_t)row * p.ldc + col) = o;
      __builtin_amdgcn_sched_barrier(0);  // one element in flight: no 128-VGPR hoist
    }
}

template <int MT, int NT>
__global__ void __launch_bounds__(2 * kThreadsT, 1) gemm_bf16_tile_sk_kernel(SkArgs s) {
  using C = Cfg<MT, NT>;
  (void)sizeof(CfgWS<MT, NT>);
  __shared__ __attribute__((aligned(16))) char smem[C::kLds];
  const GemmArgs& p = s.g;
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, j = bid >> 3, Gx = G >> 3;  // G % 8 == 0 (host)
  const long long tiles = s.units / s.T;
  const long long t0 = xcd * tiles / 8, ux = ((xcd + 1) * tiles / 8 - t0) * s.T;
  const long long u0 = t0 * s.T + j * ux / Gx, u1 = t0 * s.T + (j + 1) * ux / Gx;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int T = s.T;

  CtxT c;
  c.lds = smem;
  c.w = wave & 3;
  c.wr = c.w >> 1;
  c.wc = c.w & 1;
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
  c.a_rb16 = (size_t)16 * p.lda;
  c.b_rb16 = (size_t)16 * p.ldb;
  const int r = lane >> 2;
  const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);

  long long u = u0;
  int tau = 0;  // K-steps this workgroup has run so far (its clock)
  while (u < u1) {
    const int tile = (int)(u / T);
    const int pos = (int)(u - (long long)tile * T);
    const int n = (int)min((long long)(T - pos), u1 - u);
    // first segment (range starts mid-tile): K-tiles [0, n), partial published;
    // last segment (range ends mid-tile): K-tiles [T-n, T), partial of the next
    // workgroup added; full tile: all T K-tiles rotated to start at tau mod T,
    // so every workgroup reads K-tile (clock mod T) at the same time.
    const bool publish = pos > 0;
    const bool fixup = !publish && n < T;
    const int k0 = publish ? 0 : fixup ? T - n : tau % T;
    u += n;
    tau += n;
    int tm, tn;
    tile_mn<MT, NT>(tile, p.M, p.N, tm, tn);
    const int m0 = tm * C::TM, n0 = tn * C::TN;
    c.a_src = p.A + (size_t)(m0 + r) * p.lda + cl * 8;
    c.b_src = p.B + (size_t)(n0 + r) * p.ldb + cl * 8;

    if (wave >= 4) {  // producer: the tile kernel's pipeline over the n K-steps
#pragma unroll
      for (int st = 0; st < C::S - 1; ++st)
#pragma unroll
        for (int i = 0; i < C::P; ++i) issue_piece_rot<MT, NT>(c, st, n, k0, T, i);
      wait_vmcnt_n<C::VMC>();
      raw_barrier();
      for (int t = 0; t < n; ++t) {
#pragma unroll
        for (int i = 0; i < C::P; ++i) issue_piece_rot<MT, NT>(c, t + C::S - 1, n, k0, T, i);
        wait_vmcnt_n<C::VMC>();
        raw_barrier();
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      raw_barrier();  // segment end
      continue;
    }

    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jj = 0; jj < NT; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    FragsT<MT, NT> f;
    raw_barrier();  // step 0 visible
#pragma unroll
    for (int i = 0; i < MT + NT; ++i) read_half<MT, NT, 0>(c, f, 0, 0, i);
    constexpr int NM = MT * NT, NR = MT + NT;
    for (int t = 0; t < n; ++t) {
#pragma unroll
      for (int jj = 0; jj < NM; ++jj) {
        mfma_acc(acc[jj / NT][jj % NT], f.b[jj % NT][0], f.a[jj / NT][0]);
        if ((jj * NR) / NM != ((jj + 1) * NR) / NM)
          read_half<MT, NT, 0>(c, f, t, 1, (jj * NR) / NM);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
#pragma unroll
      for (int jj = 0; jj < NM; ++jj) {
        mfma_acc(acc[jj / NT][jj % NT], f.b[jj % NT][1], f.a[jj / NT][1]);
        if ((jj * NR) / NM != ((jj + 1) * NR) / NM)
          read_half<MT, NT, 0>(c, f, t + 1, 0, (jj * NR) / NM);  // t + 1 == n: stale, unused
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();  // segment end: the ring is free for the next prologue
    ::ntm::gemm::mfma_drain();
    // Opaque lane index: keeps the epilogue's per-lane addressing inside the
    // segment loop (hoisted out of it, ~100 address VGPRs stayed live across
    // the K loop and spilled).
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    const int ln = lane + vz;

    if (publish && (s.diag & 2)) continue;
    if (publish) {  // first segment: publish this wave's partial in slot blockIdx
      f32x4* dst = s.part + (size_t)(bid * 4 + c.w) * NM * 64;  // uniform base
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          dst[(mt * NT + nt) * 64 + ln] = acc[mt][nt];
          __builtin_amdgcn_sched_barrier(0);
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every partial store reached L2
      if (lane == 0)
        __hip_atomic_store(&s.flags[bid * 4 + c.w], s.epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (fixup) {  // last segment: add the partial of workgroup j+1 on this XCD (same wave)
      const unsigned* fl = &s.flags[(bid + 8) * 4 + c.w];
      unsigned spins = (s.diag & 1) ? kSkSpinLimit : 0;
      while ((int)(__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - s.epoch) <
                 0 &&
             ++spins < kSkSpinLimit)
        __builtin_amdgcn_s_sleep(2);
      asm volatile("" ::: "memory");
      store_c<MT, NT, true>(p, c, acc, s.part + (size_t)((bid + 8) * 4 + c.w) * NM * 64, m0, n0, ln);
    } else {
      store_c<MT, NT, false>(p, c, acc, nullptr, m0, n0, ln);
    }
  }
}

// Workspace for a grid of G workgroups: fp32 partials and flags (slot = blockIdx).
template <int MT, int NT>
inline size_t sk_part_bytes(int G) {
  return (size_t)G * 4 * MT * NT * 64 * sizeof(f32x4);
}
inline size_t sk_flag_bytes(int G) { return (size_t)G * 4 * sizeof(unsigned); }

// True iff the stream-K split applies: the tile kernel's shape rule, G % 8 == 0,
// and at least T units per workgroup on every XCD (a tile meets at most two
// ranges, both on one XCD).
template <int MT, int NT>
__host__ inline bool sk_ok(int M, int N, int K, int G) {
  if (!shape_ok_t<MT, NT>(M, N, K) || G < 8 || G % 8) return false;
  const long long T = K / TK;
  const long long tiles = (long long)(M / Cfg<MT, NT>::TM) * (N / Cfg<MT, NT>::TN);
  return (tiles / 8) * T / (G / 8) >= T;  // the smallest XCD share
}

template <int MT, int NT>
inline hipError_t launch_gemm_bf16_tile_sk(const GemmArgs& a, void* part, void* flags,
                                           unsigned epoch, int G, hipStream_t stream,
                                           int diag = 0) {
  if (!sk_ok<MT, NT>(a.M, a.N, a.K, G) || !part || !flags || a.lda < a.K || a.ldb < a.K ||
      a.ldc < a.N || (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  SkArgs s;
  s.g = a;
  s.part = (f32x4*)part;
  s.flags = (unsigned*)flags;
  s.epoch = epoch;
  s.diag = diag;
  s.T = a.K / TK;
  s.units = (long long)(a.M / Cfg<MT, NT>::TM) * (a.N / Cfg<MT, NT>::TN) * s.T;
  hipLaunchKernelGGL((gemm_bf16_tile_sk_kernel<MT, NT>), dim3(G), dim3(2 * kThreadsT), 0, stream,
                     s);
  return hipGetLastError();
}

}  // namespace gemmsk
}  // namespace ntm
