// K1 "pingpong8s": stream-K over the last two rounds of 256x256 tiles, and
// (split mode, gemm_bf16_sks_kernel below) over at most half a round of them.
//
// Why: a 256x256 part whose tile count is not a multiple of the 256 CUs leaves
// CUs idle in its last round. At 4472 x 5688 x 5832 (18 x 23 = 414 tiles) the
// data-parallel kernels run 2 rounds for 1.62 rounds of work, 0.95x hipBLASLt
// (profiles/r3_tiles), whose stream-K kernel spreads the K-work instead. The
// row-split plan (top rows on 256x256, the rest on a small tile) cannot fill a
// round either when M x N is ragged in both directions.
//
// Decomposition ("data-parallel + one-tile stream-K", Osama et al. 2023): with
// G = 256 workgroups (one per CU: the kernel takes 144 KiB of LDS) and
// ntiles = R G + L tiles (R >= 1, 0 < L < G):
//   * tiles [0, D), D = (R - 1) G, run whole: workgroup b takes b, b + G, ...
//   * the last G + L tiles are cut into K-tile PAIRS (128 of K; Tp per tile)
//     and dealt out per XCD: the tiles v = D + x + 8k belong to XCD x (as in
//     the data-parallel raster, so an XCD keeps reading the A / B panels its own
//     L2 holds), and that XCD's G / 8 workgroups j = b >> 3 take equal
//     contiguous ranges [j U / W, (j + 1) U / W) of its U = n_x Tp pairs.
// Each range is >= Tp pairs (n_x >= W), so a tile is cut at most once: into a
// HEAD [0, p) that is the last segment of workgroup j and a TAIL [p, Tp) that
// is the first segment of workgroup j + 1. A workgroup's middle segments are
// whole tiles. Split tile of the boundary below workgroup b: slot b.
//
// Fix-up without waiting on anyone: one atomic counter per split tile with an
// ARRIVE and a WRITTEN bit per part (head 1 / 2, tail 4 / 8). A part
//   o = cnt += ARRIVE; the other part's WRITTEN set -> add its partial, store C
//   else: write my partial, drain, o2 = cnt += WRITTEN;
//         the other's WRITTEN set in o2 -> add its partial, store C
//         else done (the other part combines, at its arrival or its WRITTEN add)
// Exactly one part combines: the one whose add comes after the other's
// WRITTEN. Its add is then the counter's last, so it resets the counter to 0
// for the next launch. The first part to arrive writes its partial; the second
// usually finds it written and only reads it, so a split tile costs one
// partial write and one read. No workgroup ever spins, so no launch order or
// co-residency is assumed. fp32 addition is commutative, so C is the same
// whichever part combines (REV, a test build with the segment order below
// reversed, takes the other branches and must be bitwise equal).
// The part the segment order runs first skips its ARRIVE (it writes without
// looking; if the other part had written too, the later WRITTEN add combines),
// which saves it one counter round trip.
//
// Segment body: pingpong8c's uniform K loop (gemm_bf16_pp3.hpp) started at an
// even absolute K-tile t0 and ended at t1 (dummy pieces past t1), on clamped
// sources and the masked LDS-staged epilogue (pingpong8cm), so any M, N % 8,
// K % 8 (TAIL: K % 128 != 0, chunks past K load zeros).
// Memory order (agent scope; cdna_hip_programming.md §6 Guideline 16 R1): the
// partial is stored write-through (sc1), every storing wave waits vmcnt(0),
// barrier, thread 0 adds to the counter; the combiner's thread 0 acquires
// (this CU's L1) before any wave reads the partial with plain loads.
//
// That acquire is enough only because every part of a split tile runs on the
// SAME XCD (so its plain loads hit the L2 the partial was written through to,
// never a stale line another XCD's L2 kept from an earlier launch): both modes
// deal tiles per XCD by the dispatcher's round robin, blockIdx & 7. The kernels
// CHECK that invariant instead of assuming it: each part's first counter add
// also carries the XCC_ID register of the XCD it runs on (tag fields above the
// protocol bits; split mode adds the id and its square, so the S parts agree
// iff sum = S x and sum of squares = S x^2), and the combiner compares them with
// its own. A mismatch sets the workspace's error word (kErrWord, sticky until
// the host clears it; ops.sk_xcc_error): C is then not trusted.
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gemmsk {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::issue_half3;
using ::ntm::gemm3::kEpiDefault;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::tile3;

constexpr size_t kPartialBytes = (size_t)BM * BN * 4;  // one fp32 256x256 partial
constexpr size_t kCounterBytes = 4096;                 // counter block at the workspace start
// error word (last of the counter block): 0, or the first XCD-placement
// violation a combiner saw: 0x80000000 | mode << 28 | tile << 8 | mine << 4 | other
constexpr int kErrWord = (int)(kCounterBytes / 4) - 1;
// two-round mode: the head's / tail's XCC tag (id + 1) above the protocol bits
constexpr int kHeadTagShift = 8, kTailTagShift = 16;

struct SkArgs {
  float* ws;      // kCounterBytes of counters (zero on entry, left zero), then G slots x 2 partials
  unsigned* cnt;  // = ws
  int G;          // workgroups (a multiple of 8)
  int D;          // tiles run whole
  int Tp;         // K-tile pairs per tile
  int ntiles;
  int S = 0;      // split mode (at most half a round of tiles): K slices per tile, else 0
  unsigned long long* stamps = nullptr;  // STAMP builds: 16 per workgroup
  // fault injection (tests, the Job's self-check): the head / slice 0 of every
  // split tile claims XCC_ID ^ fault, so every placement check fails; 0 = off
  unsigned fault = 0;
};

// Process-wide fault-injection value the launchers copy into SkArgs::fault
// (ntm_set_sk_fault_inject; host only).
inline unsigned& sk_fault_inject() {
  static unsigned v = 0;
  return v;
}

// Tiles, pairs and the whole-tile prefix for (M, N, K) on `cus` CUs.
// Two-round mode (S = 0): more tiles than CUs, not a multiple of them.
// Split mode (S >= 2, gemm_bf16_sks_kernel): every XCD's tiles fit its CUs at
// least twice over, so each tile is cut into S equal K slices and every slice
// runs at once on its own CU (one round, slices at the same K offsets in
// lockstep); S = the most slices that fit, at most kMaxSlices and one pair each.
constexpr int kMaxSlices = 8;

__host__ __device__ inline bool sk_decompose(int M, int N, int K, int cus, SkArgs& s) {
  // one 4-byte counter per workgroup slot (or per tile) in the kCounterBytes block
  if (M <= 0 || N <= 0 || K <= 0 || cus < 8 || (cus % 8) != 0 || cus + 8 > kErrWord)
    return false;
  s.ntiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  s.G = cus;
  s.Tp = (K + 2 * BK - 1) / (2 * BK);
  s.S = 0;
  if (s.ntiles <= s.G) {
    const int per_xcd = (s.ntiles + 7) / 8, W = s.G / 8;
    int S = W / per_xcd;
    if (S > kMaxSlices) S = kMaxSlices;
    if (S > s.Tp) S = s.Tp;
    if (S < 2) return false;
    s.S = S;
    s.D = 0;
    return true;
  }
  if ((s.ntiles % s.G) == 0) return false;
  s.D = (s.ntiles / s.G - 1) * s.G;
  return true;
}

inline size_t sk_ws_bytes(int G) { return kCounterBytes + (size_t)G * 2 * kPartialBytes; }

__host__ __device__ inline bool shape_ok_sk(int M, int N, int K) {
  return M > 0 && N > 0 && (N % 8) == 0 && K >= 2 * BK && (K % 8) == 0;
}

// Clamped per-lane sources of tile (m0, n0) at K-tile 0 (pingpong8cm's setup).
__device__ __forceinline__ void set_sources(const GemmArgs& p, Ctx& c, int m0, int n0, int lane) {
  const int r = lane >> 2;
  const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
  const int ra = m0 + c.w * 16 + r, rb = n0 + c.w * 16 + r;
  c.src[kALo] = p.A + (size_t)min(ra, p.M - 1) * p.lda + cl * 8;
  c.src[kAHi] = p.A + (size_t)min(ra + 128, p.M - 1) * p.lda + cl * 8;
  c.src[kBLo] = p.B + (size_t)min(rb, p.N - 1) * p.ldb + cl * 8;
  c.src[kBHi] = p.B + (size_t)min(rb + 128, p.N - 1) * p.ldb + cl * 8;
}

// Lane id that the compiler cannot hoist: with the plain lane id, LICM lifts
// the epilogue's 16 row / mask values out of the segment loop and they spill
// across the K loop (gemm_bf16_pp6.hpp opaque_lane, same reason).
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ void zero_acc(f32x4 (&acc)[2][2][4][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][j][m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// K-tiles [t0, t1) of the tile whose sources are in c (t0 even, t1 > t0 even),
// accumulated onto acc; drained (vmcnt(0)) on return, stagger balanced.
template <bool TAIL>
__device__ __forceinline__ void k_range(const GemmArgs& p, const Ctx& c, Frags3& f,
                                        f32x4 (&acc)[2][2][4][2], int t0, int t1) {
  // prologue: B-lo A-lo B-hi A-hi of t0, B-lo A-lo B-hi of t0 + 1 (buffers 0 / 1)
  issue_half3<kBLo, TAIL>(c, t0, 0, t1);
  issue_half3<kALo, TAIL>(c, t0, 0, t1);
  issue_half3<kBHi, TAIL>(c, t0, 0, t1);
  issue_half3<kAHi, TAIL>(c, t0, 0, t1);
  issue_half3<kBLo, TAIL>(c, t0 + 1, 1, t1);
  issue_half3<kALo, TAIL>(c, t0 + 1, 1, t1);
  issue_half3<kBHi, TAIL>(c, t0 + 1, 1, t1);
  wait_vmcnt<10>();
  raw_barrier();
  read_b<kBLo>(c, f.b0, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger
  int t = t0;
  if constexpr (TAIL) {
    // the zero-filling issue path only where a piece can reach past K
    const int t_real = (p.K + BK - 1) / BK;
    for (; t < t1 && t + 4 < t_real; t += 2) {
      tile3<false, false, 0, false>(c, f, acc, t, t1);
      tile3<true, false, 0, false>(c, f, acc, t + 1, t1);
    }
    for (; t < t1; t += 2) {
      tile3<false, false, 0, true>(c, f, acc, t, t1);
      tile3<true, false, 0, true>(c, f, acc, t + 1, t1);
    }
  } else {
    for (; t < t1; t += 2) {
      tile3<false, false, 0, false>(c, f, acc, t, t1);
      tile3<true, false, 0, false>(c, f, acc, t + 1, t1);
    }
  }
  if (c.wr == 0) raw_barrier();  // balance the stagger
  wait_vmcnt<0>();                // dummy pieces: nothing lands after this
}

// This lane's fp32 partial in a slot half: accumulator i of thread tid at
// float4 index i * 512 + tid (each store / load instruction covers 8 KiB).
// Stored write-through (sc1: buffer store, aux 16), so publishing it needs no
// release fence - no write-back of the XCD's whole L2, whose dirty lines are
// every other workgroup's partials and C (cdna_hip_programming.md §6 Guideline
// 16 R1): every storing wave drains vmcnt, then the counter add.
__device__ __forceinline__ void write_partial(float* dst, const f32x4 (&acc)[2][2][4][2]) {
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
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j][m][n]), rsrc,
                                                 off + (((i * 2 + j) * 4 + m) * 2 + n) * kThreads * 16,
                                                 0, 16);
}

// One quadrant (8 loads, 32 VGPRs) at a time: issued all at once the 32 loads
// need 128 VGPRs on top of the accumulators and the kernel spills.
__device__ __forceinline__ void add_partial(const float* src, f32x4 (&acc)[2][2][4][2]) {
  const f32x4* s = (const f32x4*)src + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][j][m][n] += s[(((i * 2 + j) * 4 + m) * 2 + n) * kThreads];
      __builtin_amdgcn_sched_barrier(0);
    }
}

// Thread 0 adds `v` to the counter and every thread gets the old value. DRAIN:
// every wave's (write-through) partial stores complete first.
template <bool DRAIN>
__device__ __forceinline__ unsigned counter_add(unsigned* cnt, unsigned v, int* bcast) {
  if constexpr (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    *bcast = (int)__hip_atomic_fetch_add(cnt, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return (unsigned)__builtin_amdgcn_readfirstlane(*bcast);
}

// Thread 0 acquires (agent scope) before any thread reads a peer's partial.
__device__ __forceinline__ void acquire_all() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's L1 (L2 is kept)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__device__ __forceinline__ void reset_counter(unsigned* cnt) {
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// First placement violation wins (the word is read and cleared by the host).
__device__ __forceinline__ void report_xcc_error(unsigned* cnt_base, unsigned code) {
  if (threadIdx.x == 0) {
    unsigned expect = 0u;
    __hip_atomic_compare_exchange_strong(cnt_base + kErrWord, &expect, 0x80000000u | code,
                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

constexpr int kEpiSk = kEpiDefault | kEpiMask;

// REV (test build): each workgroup runs its stream-K segments in range order
// (tail, whole tiles, head), so tails tend to arrive first (the protocol's
// other branches).
// STAMP (diagnostic build, experimental library): thread 0 records
// s_memrealtime (100 MHz) at kernel start [0] and, per stream-K segment q < 3,
// at its K loop's start / end, after the fix-up and after the C store
// [1 + 4q .. 4 + 4q]; [13 + q] = segment q's kind (0 whole, 1 head, 2 tail).
template <bool TAIL, bool REV = false, bool STAMP = false>
__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_sk_kernel(GemmArgs p, SkArgs s) {
  // ONE __shared__ array: a second __shared__ object (even a 4-byte flag) makes
  // hipcc wait vmcnt(0) before the K loop's ds_reads, draining the LDS-DMA
  // pipeline (cdna_hip_programming.md, projection-GEMM trap 4a; measured here:
  // 0.55x). The fix-up's broadcast word sits past the staging / scratch bytes.
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3 + 16];
  int* bcast = (int*)(smem + kLdsBytes3);
  auto stamp = [&](int i) {
    if constexpr (STAMP) {
      unsigned long long rt;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      if (threadIdx.x == 0 && i < 16) s.stamps[16 * (size_t)blockIdx.x + i] = rt;
    }
  };
  stamp(0);
  const int b = (int)blockIdx.x;
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
  const int T = 2 * s.Tp;
  Frags3 f;
  f32x4 acc[2][2][4][2];

  // whole tiles [0, D)
  for (int tile = b; tile < s.D; tile += s.G) {
    int tm, tn;
    tile_coords_of<kGroupM>(tile, s.ntiles, p.M, p.N, tm, tn);
    set_sources(p, c, tm * BM, tn * BN, lane_now());
    zero_acc(acc);
    k_range<TAIL>(p, c, f, acc, 0, T);
    store_tile_epi<false, kEpiSk>(p, c, acc, tm * BM, tn * BN, lane_now());
    raw_barrier();  // staging reads done before the next prologue's DMA
  }

  // stream-K over the last G + L tiles, per XCD: pairs [u0, u1) of this XCD's
  // tile list, i.e. tiles k0 .. k1 from pair pa0 of k0 to pair pb1 of k1.
  // All of it is uniform; readfirstlane keeps it out of VGPRs, which the K
  // loop needs every one of.
  const int x = b & 7, j = b >> 3, W = s.G >> 3;
  const unsigned my_xcc = xcc_id();
  const int nx = (s.ntiles - s.D - x + 7) >> 3;  // this XCD's stream-K tiles
  const int U = nx * s.Tp;
  const int u0 = __builtin_amdgcn_readfirstlane((int)((long)j * U / W));
  const int u1 = __builtin_amdgcn_readfirstlane((int)((long)(j + 1) * U / W));
  const int k0 = __builtin_amdgcn_readfirstlane(u0 / s.Tp);
  const int k1 = __builtin_amdgcn_readfirstlane((u1 - 1) / s.Tp);
  const int pa0 = u0 - k0 * s.Tp, pb1 = u1 - k1 * s.Tp;
  // Segment order keeps an XCD's workgroups in K-lockstep, as the data-parallel
  // kernel is, so the A / B panels they share are read from L2 once: whole
  // tiles first (every workgroup at K = t), then the head (K = t, or t - Tp
  // after a whole tile), then the tail, which every workgroup reaches at the
  // same K = t + Tp - U / W. In range order (tail first, REV) each workgroup's
  // K offset is different, and the same launch fetched 4.7x the bytes from
  // HBM at 0.56x the speed (profiles/r4_sk).
  const int has_tail = pa0 > 0, has_head = pb1 < s.Tp;
  const int kw0 = k0 + has_tail, nw = k1 + 1 - has_head - kw0;
  for (int q = 0; q <= k1 - k0; ++q) {
    const int k = REV ? k0 + q : q < nw ? kw0 + q : (q == nw && has_head) ? k1 : k0;
    const int pa = k == k0 ? pa0 : 0;
    const int pb = k == k1 ? pb1 : s.Tp;
    int tm, tn;
    tile_coords_of<kGroupM>(s.D + x + 8 * k, s.ntiles, p.M, p.N, tm, tn);
    const int m0 = __builtin_amdgcn_readfirstlane(tm * BM);
    const int n0 = __builtin_amdgcn_readfirstlane(tn * BN);
    set_sources(p, c, m0, n0, lane_now());
    zero_acc(acc);
    stamp(1 + 4 * q);
    k_range<TAIL>(p, c, f, acc, 2 * pa, 2 * pb);
    stamp(2 + 4 * q);
    const bool tail = pa > 0;                // begun by workgroup b - 8 (slot b)
    const bool head = !tail && pb < s.Tp;    // continued by workgroup b + 8 (slot b + 8)
    bool store = !head && !tail;
    if (head || tail) {
      const int slot = tail ? b : b + 8;
      float* part = s.ws + (kCounterBytes + (size_t)slot * 2 * kPartialBytes) / 4;
      float* mine = part + (tail ? kPartialBytes / 4 : 0);
      const float* other = part + (tail ? 0 : kPartialBytes / 4);
      unsigned* cnt = s.cnt + slot;
      const unsigned arrive = tail ? 4u : 1u, written = arrive << 1;
      const unsigned other_written = tail ? 2u : 8u;
      // this part's XCC tag rides on its first counter add
      const unsigned me = tail ? my_xcc : my_xcc ^ s.fault;
      const unsigned tag = (me + 1u) << (tail ? kTailTagShift : kHeadTagShift);
      // the part this segment order runs first (the head; REV: the tail) writes
      // without looking: the other part has almost never written yet
      const bool writer = REV ? tail : head;
      unsigned o = writer ? 0u : counter_add<false>(cnt, arrive + tag, bcast);
      if (!(o & other_written)) {
        write_partial(mine, acc);
        o = counter_add<true>(cnt, written + (writer ? tag : 0u), bcast);
      }
      if (o & other_written) {
        // the other part's first add (which carried its tag) precedes its WRITTEN
        const unsigned other_xcc = ((o >> (tail ? kHeadTagShift : kTailTagShift)) & 0xFFu) - 1u;
        if (other_xcc != me)
          report_xcc_error(s.cnt, (unsigned)(slot & 0xFFFF) << 8 | (me & 0xF) << 4 |
                                      (other_xcc & 0xF));
        acquire_all();
        add_partial(other, acc);
        reset_counter(cnt);
        store = true;
      }
    }
    stamp(3 + 4 * q);
    if constexpr (STAMP) {
      if (threadIdx.x == 0 && q < 3) s.stamps[16 * (size_t)blockIdx.x + 13 + q] = head ? 1 : tail ? 2 : 0;
    }
    if (store) store_tile_epi<false, kEpiSk>(p, c, acc, m0, n0, lane_now());
    raw_barrier();  // staging reads done before the next prologue's DMA
    stamp(4 + 4 * q);
  }
}

// Split mode ("pingpong8s" on at most half a round of tiles): XCD x's tiles
// v = x + 8k (k < n_x), each in S K slices [s Tp / S, (s + 1) Tp / S) pairs;
// workgroup j of the XCD runs slice j / n_x of tile k = j % n_x (the rest of
// the XCD's workgroups exit at once). S >= 3: every slice writes its fp32
// partial (write-through) and adds 1 to the tile's counter; the one that draws
// S - 1 sums the other S - 1 partials into its registers, stores C and resets
// the counter. Nobody waits. C is the same whoever combines: it sums all S
// partials from memory in slice order. S = 2: the head / tail protocol of the
// two-round mode (round 5: one partial write + one read per tile).
// PAIR (S = 2 only, chosen at launch): the head / tail protocol below; a
// separate instantiation, so the S >= 3 build keeps round 4's register
// allocation (sharing one body cost it 18-24 % at S = 4 with K % 128 != 0).
template <bool TAIL, bool PAIR = false>
__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_sks_kernel(GemmArgs p, SkArgs s) {
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
  tile_coords_of<kGroupM>(tile, s.ntiles, p.M, p.N, tm, tn);
  const int m0 = __builtin_amdgcn_readfirstlane(tm * BM);
  const int n0 = __builtin_amdgcn_readfirstlane(tn * BN);
  set_sources(p, c, m0, n0, lane_now());
  Frags3 f;
  f32x4 acc[2][2][4][2];
  zero_acc(acc);
  const int pa = slice * s.Tp / s.S, pb = (slice + 1) * s.Tp / s.S;
  k_range<TAIL>(p, c, f, acc, 2 * pa, 2 * pb);
  float* part = s.ws + (kCounterBytes + (size_t)tile * s.S * kPartialBytes) / 4;
  unsigned* cnt = s.cnt + tile;
  if constexpr (PAIR) {
    // two slices: the two-round mode's head / tail protocol (slice 0 = head, the
    // writer). The first to finish writes its partial; the other usually finds it
    // written and adds it to its own registers - one partial write and one read
    // per tile instead of two and two. own + other is commutative in fp32, so C
    // is the same whichever slice combines.
    const bool tail = slice == 1;
    const unsigned arrive = tail ? 4u : 1u, written = arrive << 1;
    const unsigned other_written = tail ? 2u : 8u;
    const unsigned xc = xcc_id() ^ (tail ? 0u : s.fault);
    const unsigned tag = (xc + 1u) << (tail ? kTailTagShift : kHeadTagShift);
    float* mine = part + (tail ? kPartialBytes / 4 : 0);
    const float* other = part + (tail ? 0 : kPartialBytes / 4);
    unsigned o = tail ? counter_add<false>(cnt, arrive + tag, bcast) : 0u;
    if (!(o & other_written)) {
      write_partial(mine, acc);
      o = counter_add<true>(cnt, written + (tail ? 0u : tag), bcast);
    }
    if (!(o & other_written)) return;  // uniform: the other slice combines
    const unsigned other_xcc = ((o >> (tail ? kHeadTagShift : kTailTagShift)) & 0xFFu) - 1u;
    if (other_xcc != xc)
      report_xcc_error(s.cnt, 1u << 28 | (unsigned)(tile & 0xFFFF) << 8 | (xc & 0xF) << 4 |
                                  (other_xcc & 0xF));
    acquire_all();
    add_partial(other, acc);
    reset_counter(cnt);
    store_tile_epi<false, kEpiSk>(p, c, acc, m0, n0, lane_now());
    return;
  }
  write_partial(part + (size_t)slice * (kPartialBytes / 4), acc);
  // count (bits 0-7) + XCC id (8-15) + its square (16-31): S <= 8 parts, id < 16
  const unsigned xc = xcc_id() ^ (slice == 0 ? s.fault : 0u);
  const unsigned tag = 1u + (xc << 8) + ((xc * xc) << 16);
  const unsigned o = counter_add<true>(cnt, tag, bcast);
  if ((o & 0xFFu) != (unsigned)(s.S - 1)) return;  // uniform
  const unsigned all = o + tag, S = (unsigned)s.S;
  if (((all >> 8) & 0xFFu) != S * xc || (all >> 16) != S * xc * xc)
    report_xcc_error(s.cnt, 1u << 28 | (unsigned)(tile & 0xFFFF) << 8 | (xc & 0xF) << 4);
  acquire_all();
  // every slice's partial (its own too, already written) summed in slice order,
  // so C does not depend on which slice combines (no second accumulator set)
  zero_acc(acc);
  for (int q = 0; q < s.S; ++q) add_partial(part + (size_t)q * (kPartialBytes / 4), acc);
  reset_counter(cnt);
  store_tile_epi<false, kEpiSk>(p, c, acc, m0, n0, lane_now());
}

// Launch on `cus` workgroups with the caller's workspace (sk_ws_bytes(cus)).
// Its first kCounterBytes (the counters) must be zero on entry, and a completed
// launch leaves them zero, so a caller zeroes a workspace once and then reuses
// it for every stream-K launch on one stream (no per-call memset dispatch). Returns hipErrorInvalidValue
// for shapes stream-K does not serve (sk_decompose: tiles a multiple of the
// CUs, or one round of them with fewer than 2 K slices per tile).
// HT = false (experimental A/B build): split mode's S-partial protocol also for S = 2.
template <bool REV = false, bool STAMP = false, bool HT = true>
inline hipError_t launch_gemm_bf16_sk(const GemmArgs& a, int cus, void* ws, size_t ws_bytes,
                                      hipStream_t stream, unsigned long long* stamps = nullptr) {
  SkArgs s;
  if (!shape_ok_sk(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) || !sk_decompose(a.M, a.N, a.K, cus, s) ||
      ws == nullptr || ws_bytes < sk_ws_bytes(s.G) || (reinterpret_cast<size_t>(ws) % 16))
    return hipErrorInvalidValue;
  s.ws = (float*)ws;
  s.cnt = (unsigned*)ws;
  s.stamps = stamps;
  s.fault = sk_fault_inject();
  if (STAMP && stamps == nullptr) return hipErrorInvalidValue;
  const dim3 g((unsigned)s.G), blk(kThreads);
  if (s.S >= 2) {  // split mode (REV / STAMP do not apply)
    if (REV || STAMP) return hipErrorInvalidValue;
    const bool pair = HT && s.S == 2;
    if (a.K % (2 * BK)) {
      if (pair)
        hipLaunchKernelGGL((gemm_bf16_sks_kernel<true, true>), g, blk, 0, stream, a, s);
      else
        hipLaunchKernelGGL((gemm_bf16_sks_kernel<true, false>), g, blk, 0, stream, a, s);
    } else {
      if (pair)
        hipLaunchKernelGGL((gemm_bf16_sks_kernel<false, true>), g, blk, 0, stream, a, s);
      else
        hipLaunchKernelGGL((gemm_bf16_sks_kernel<false, false>), g, blk, 0, stream, a, s);
    }
    return hipGetLastError();
  }
  if (a.K % (2 * BK))
    hipLaunchKernelGGL((gemm_bf16_sk_kernel<true, REV, STAMP>), g, blk, 0, stream, a, s);
  else
    hipLaunchKernelGGL((gemm_bf16_sk_kernel<false, REV, STAMP>), g, blk, 0, stream, a, s);
  return hipGetLastError();
}

}  // namespace gemmsk
}  // namespace ntm
