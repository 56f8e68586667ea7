// K1 "pingpong8o" (variant 25): persistent pingpong8c whose C stores OVERLAP
// the next tile's K loop. The default plan runs it in place of pingpong8c when
// the 256x256 part has more tiles than CUs (ntm_validation.hip plan_k1).
//
// Why: at 8192^3 every CU runs 4 tiles back to back, and each tile boundary
// costs ~5 us of wall in the data-parallel kernel (profiles/r2_k1/
// stamp8192_phase_split.log: prologue 1.5 us, epilogue 2.2-2.5 us, 1.4 us
// between workgroups), ~3 % of the launch; kfit puts our fixed cost 10 us above
// hipBLASLt's. The earlier persistent build (pingpong8p, round 1, deleted) kept
// the LDS-DMA pipeline running across tiles but drained it with vmcnt(0) and
// then stored the whole tile at the boundary, so every CU still stalled there
// at the same moment: no gain (profiles/r1_pp4).
//
// Here nothing drains at a boundary. The four 64x32 accumulator quadrants of a
// wave finish one phase apart in the last K-tile (P0: acc[0][0], P1: acc[0][1],
// P2: acc[1][1], P3: acc[1][0]), and each is first rewritten one phase later in
// the next tile's first K-tile. So quadrant q is converted to bf16 and stored
// from registers (4 dwordx4 stores per lane, widened layout of store_tile_wide)
// in the LOAD segment of the phase after its last MFMA - where the partner wave
// row runs its MFMAs (ping-pong) - and the next tile's first MFMA on it starts
// from a zero C operand instead of a zeroing pass:
//   P1(T-1): q0   P2(T-1): q1   P3(T-1): q2   P0(0 of the next tile): q3
// The LDS-DMA stream is the uniform one of pingpong8c; pieces that pingpong8c
// pointed past the tile (dummy pieces) stage the next tile's K-tiles 0 / 1, so
// the next tile's prologue is absorbed too. Only the CU's last tile drains and
// stores through the LDS-staged epilogue.
//
// vmcnt with stores in the stream: loads, stores and LDS-DMA decrement vmcnt in
// issue order (MI355X_MICROARCH.md, last paragraph of the cycle constants), so
// a counted wait stays exact if it counts the stores younger than its target.
// Each phase issues 2 pieces, then waits, then (conversion phases) 4 stores;
// the wait of phase j retires the pieces of phase j-5 (RAW distance 6, as in
// pingpong8c), so it is vmcnt(10 + stores issued in phases j-5 .. j-1):
//   P1(T-1) 10, P2(T-1) 14, P3(T-1) 18, P0(0) 22, P1(0) 26, P2(0) 26, P3(0) 22,
//   P0(1) 18, P1(1) 14, P2(1) 10.
// WAR and the reads are pingpong8c's (gemm_bf16_pp2.hpp proof); the stores
// touch no LDS. Every wave runs the same barrier count per tile.
//
// Measured (tools/gemm_check.py, one process, medians of 13 rounds,
// profiles/r3_k1o/): 8192^3 1634 vs pingpong8c 1622 TF/s (hipBLASLt 1642),
// 5120^3 1394 vs 1374, 8192x8192x6144 1611 vs 1590; race screen clean.
// Rejected variants (deleted): sc1 write-through C stores -3.5 %, plain
// (L2-allocating) stores -2 %, static priority on wave row 1 a tie.
//
// Shape rule: M, N % 256, K % 128, K >= 256 (T = K / 64 even and >= 4), no ABFT
// row sum. Grid = min(tiles, CUs): workgroup b walks tiles b, b + G, ... in the
// non-persistent kernel's block order, so with G % 8 == 0 each XCD keeps its
// 32 lock-step tiles and their shared L2 panels.
#pragma once

#include "ntm/gemm_bf16_pp3.hpp"

namespace ntm {
namespace gemm6 {

using namespace ::ntm::gemm;
using ::ntm::gemm3::Frags3;
using ::ntm::gemm3::kLdsBytes3;
using ::ntm::gemm3::kScratch;

__host__ __device__ inline bool shape_ok6(int M, int N, int K) {
  return M > 0 && N > 0 && (M % BM) == 0 && (N % BN) == 0 && (K % (2 * BK)) == 0 && K >= 4 * BK;
}

// Masked build ("pingpong8om"): ragged C (any M, N % 8) on whole K-tile pairs
// (K % 128, K >= 256); edge tiles clamp their source rows and mask their stores.
// With TAIL (K % 128 != 0): K % 8 and K > 128 (ceil(K / 128) * 2 >= 4 K-tiles);
// 16-B chunks past K load zeros, so the partial K-tile pair adds nothing.
__host__ __device__ inline bool shape_ok6m(int M, int N, int K) {
  return M > 0 && N > 0 && (N % 8) == 0 && K > 2 * BK && (K % 8) == 0 &&
         ((K % (2 * BK)) != 0 || K >= 4 * BK);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Where the pieces of K-tile kt (counted from the current tile's start) come
// from: the current tile (NX false), or (NX true, kt >= T) the next tile when
// there is one (dA / dB = its element offset from this tile) and otherwise an
// L2-hot in-bounds dummy slice into the scratch region nobody reads.
// Lane id recomputed where it is used (2 VALU). The masked builds need lane-
// derived values (clamped source rows, store masks, the K-tail column) only
// at tile boundaries; kept live through the K loop they push the kernel past
// 256 VGPRs, and hipcc then reloads spills with vmcnt(0) inside the loop,
// draining the LDS-DMA pipeline. The asm is volatile, so it is neither hoisted
// nor shared across uses.
__device__ __forceinline__ int opaque_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Source of half H of a tile at (m0, n0) for this lane, rows clamped to the
// matrix (masked build): the clamped rows only feed C rows / columns that the
// masked stores skip. (Whole-tile builds step c.src by per-tile deltas instead.)
template <int H>
__device__ __forceinline__ const __bf16* src_clamped(const GemmArgs& p, int m0, int n0, int w,
                                                     int lane) {
  const int r = lane >> 2;
  const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
  const int hi = (H == kAHi || H == kBHi) ? 128 : 0;
  if constexpr (H == kALo || H == kAHi)
    return p.A + (size_t)min(m0 + hi + w * 16 + r, p.M - 1) * p.lda + cl * 8;
  else
    return p.B + (size_t)min(n0 + hi + w * 16 + r, p.N - 1) * p.ldb + cl * 8;
}

// TL (partial-K builds, only where a piece can reach past K): a 16-B chunk
// starting at k >= K loads zeros (as pingpong8cm's TAIL build).
template <int H, bool NX, bool MASK = false, bool TL = false>
__device__ __forceinline__ void issue6(const GemmArgs& p, const Ctx& c, int kt, int buf, int T,
                                       bool has_next, long dA, long dB, int nm0, int nn0,
                                       int lane) {
  const __bf16* s;
  int off = buf * kTileBytes + H * kHalfBytes;
  if constexpr (!NX) {
    s = c.src[H] + (size_t)kt * BK;
  } else if constexpr (MASK) {
    s = has_next ? src_clamped<H>(p, nm0, nn0, c.w, opaque_lane()) + (long)(kt - T) * BK
                 : c.src[H] + (long)(T - 1) * BK;
    off = has_next ? off : kScratch;
  } else {
    const long d = (H == kALo || H == kAHi) ? dA : dB;
    s = c.src[H] + (has_next ? d + (long)(kt - T) * BK : (long)(T - 1) * BK);
    off = has_next ? off : kScratch;
  }
  char* d = c.lds + off + (2 * c.w) * 1024;
  if constexpr (TL && !NX) {
    const int l = opaque_lane();
    const int col = kt * BK + ((l & 3) ^ (((l >> 5) & 1) << 1)) * 8;
    glds16(col < c.K ? s : (const __bf16*)kZeroChunk16, d);
    glds16(col + 32 < c.K ? s + 32 : (const __bf16*)kZeroChunk16, d + 1024);
  } else {
    glds16(s, d);
    glds16(s + 32, d + 1024);
  }
}

// PF builds (round 5): touch half H of the NEXT tile's K-tile
// T + KO (KO = 0 / 1) into L2 a few phases before the real pieces stage it,
// as an LDS-DMA into the scratch slice nobody reads (the same form as the
// dummy pieces, so it needs no VGPR; it counts in vmcnt like them). Without a
// next tile it re-reads this tile's last K-tile (L2-hot), keeping the counted
// waits uniform. At a tile boundary every CU of an XCD turns to new A / B
// panels at once, and pingpong8o's boundary phases waited ~2.7 k cycles for
// them to come from HBM (profiles/r4_stamps).
template <int H, int KO>
__device__ __forceinline__ void prefetch6(const Ctx& c, int T, bool has_next, long dA, long dB) {
  const long d = (H == kALo || H == kAHi) ? dA : dB;
  // an opaque copy of the source pointer, so the eight touch addresses are
  // formed here and not hoisted out of the K loop (16 more live VGPRs spill)
  const __bf16* base;
  asm volatile("" : "=v"(base) : "0"(c.src[H]));
  const __bf16* s = base + (has_next ? d + (long)KO * BK : (long)(T - 1) * BK);
  // one 16-B chunk per lane: a lane quad spans 64 B of a row, and the piece's
  // second chunk (s + 32) lies in the same 128-B L2 lines
  glds16(s, c.lds + kScratch + (2 * c.w) * 1024);
}

// fp8 (F8 builds): v_mfma_f32_16x16x128_f8f6f4 (e4m3 x e4m3, default unit
// scales) updating a VGPR accumulator in place. K1-fp8's pingpong8c keeps its
// accumulators in AGPRs (gemm_bf16.hpp mfma_f8_agpr), which caps its VGPRs at
// 128 at two waves per SIMD and left no room for the boundary conversion; in
// VGPRs the fp8 kernel has the bf16 kernel's register shape. hipcc pads nothing
// inside the asm: the accumulators are written by VALU only at tile boundaries
// (zero_quadrant, >= 1 barrier before their next MFMA) and read by VALU only
// after mfma_wait_states.
__device__ __forceinline__ void mfma_f8_vgpr(f32x4& acc, const i32x8& a, const i32x8& b) {
  asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

// MFMA result -> VALU read of it (the 16-pass f8f6f4 needs passes + 3 = 19).
__device__ __forceinline__ void mfma_wait_states() {
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
}

// 16 MFMAs of one quadrant (mma_quadrant without the setprio); F8: 8 f8f6f4
// MFMAs over the same LDS image (K1-fp8's order: mt outer, nt inner).
template <bool F8 = false>
__device__ __forceinline__ void mma_q(f32x4 (&acc)[4][2], const bf16x8 (&a)[4][2],
                                      const bf16x8 (&b)[2][2]) {
  if constexpr (F8) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        mfma_f8_vgpr(acc[mt][nt], cat_f8(b[nt][0], b[nt][1]), cat_f8(a[mt][0], a[mt][1]));
  } else {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt][ks], a[mt][ks], acc[mt][nt], 0, 0, 0);
  }
}

// Masked 16-B C store that is always issued: a lane outside C gets an offset
// past the buffer's range, which the buffer store's range check drops. A
// branch around the store (hipcc's s_cbranch_execz when a whole wave is
// outside C, at ragged edges) would issue fewer stores than the counted vmcnt
// waits assume, and they would then release before their LDS-DMA pieces land.
// blk = the 16-row block's origin (wave-uniform), off = the lane's element offset.
template <int POL>
__device__ __forceinline__ void store_c16_masked(const __bf16* blk, int off, bool ok,
                                                 const unsigned __attribute__((ext_vector_type(4))) & v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(blk), 0, 0x7FFFFFFF,
                                                      0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, ok ? off * 2 : (int)0x80000000, 0, POL == 1 ? 2 : 0);
}

// One quadrant of the previous tile (origin m0, n0) to C, in store_tile_wide's
// layout: after a permlane16 swap per dword pair every lane holds 8 consecutive
// columns. c_lane = the lane's element offset inside the tile (one VGPR).
// MASK: store only rows < M and 8-column chunks < N (lrow / lcol = the lane's
// row / column inside the quadrant's 16-row block origin, tile-relative).
template <int MH, int NH, int POL, bool MASK = false>
__device__ __forceinline__ void store_quadrant(const GemmArgs& p, const f32x4 (&q)[4][2],
                                               int m0, int n0, int c_lane, int lrow = 0,
                                               int lcol = 0) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
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
    __bf16* tile = p.C + (size_t)(m0 + MH * 128 + mt * 16) * p.ldc + (n0 + NH * 128);
    if constexpr (MASK) {
      const int l = opaque_lane();
      const int lr = lrow + (l & 15);                              // lrow = 64 wr
      const int lc = lcol + ((l >> 4) & 1) * 16 + (l >> 5) * 8;    // lcol = 32 wc
      const bool ok = m0 + MH * 128 + mt * 16 + lr < p.M && n0 + NH * 128 + lc < p.N;
      store_c16_masked<POL>(tile, c_lane, ok, u32x4{w0[0], w0[1], w1[0], w1[1]});
      continue;
    }
    store_c16<POL>(tile + c_lane, u32x4{w0[0], w0[1], w1[0], w1[1]});
  }
}

// One 16-row block (mt) of a quadrant: the SPREAD build's unit of store
// (MASK: rows < M and 8-column chunks < N only, as store_quadrant).
template <int MH, int NH, int MT, int POL, bool MASK = false>
__device__ __forceinline__ void store_block(const GemmArgs& p, const f32x4 (&q)[4][2], int m0,
                                            int n0, int c_lane, int lrow = 0, int lcol = 0) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const f32x4 v0 = q[MT][0], v1 = q[MT][1];
  unsigned w0[2], w1[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto r = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v0[2 * h], v0[2 * h + 1]),
                                                    pack_bf16x2(v1[2 * h], v1[2 * h + 1]),
                                                    false, false);
    w0[h] = r[0];
    w1[h] = r[1];
  }
  __bf16* tile = p.C + (size_t)(m0 + MH * 128 + MT * 16) * p.ldc + (n0 + NH * 128);
  if constexpr (MASK) {
    const int l = opaque_lane();
    const int lr = lrow + (l & 15);
    const int lc = lcol + ((l >> 4) & 1) * 16 + (l >> 5) * 8;
    const bool ok = m0 + MH * 128 + MT * 16 + lr < p.M && n0 + NH * 128 + lc < p.N;
    store_c16_masked<POL>(tile, c_lane, ok, u32x4{w0[0], w0[1], w1[0], w1[1]});
  } else {
    store_c16<POL>(tile + c_lane, u32x4{w0[0], w0[1], w1[0], w1[1]});
  }
}

__device__ __forceinline__ void zero_quadrant(f32x4 (&q)[4][2]);

// SPREAD: the store unit of boundary phase O (0 = P1 of K-tile T-1 .. 6 = P3
// of the next tile's K-tile 0) for quadrant Q (finishing order q0..q3): block
// mt = O - Q, zeroing the quadrant after its last block. q0..q2's blocks in
// O <= 2 belong to this tile, everything from O = 3 on to the previous one.
template <int O, int Q, int POL, bool MASK = false>
__device__ __forceinline__ void spread_unit(const GemmArgs& p, f32x4 (&acc)[2][2][4][2],
                                            int m0, int n0, int pm0, int pn0, int c_lane,
                                            int lrow = 0, int lcol = 0) {
  constexpr int MT = O - Q;
  if constexpr (MT >= 0 && MT <= 3) {
    constexpr int MH = (Q == 2 || Q == 3) ? 1 : 0;
    constexpr int NH = (Q == 1 || Q == 2) ? 1 : 0;
    store_block<MH, NH, MT, POL, MASK>(p, acc[MH][NH], O >= 3 ? pm0 : m0, O >= 3 ? pn0 : n0,
                                       c_lane, lrow, lcol);
    if constexpr (MT == 3) zero_quadrant(acc[MH][NH]);
  }
}

// Zero a stored quadrant in place (32 v_mov): an MFMA with an inline-zero C
// operand instead lets hipcc give the result fresh registers, and the copies
// back at the loop's back edge spilled.
__device__ __forceinline__ void zero_quadrant(f32x4 (&q)[4][2]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) q[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
}

struct Edge {
  int pm0, pn0;   // previous tile's origin (its quadrants leave in K-tile 0)
  bool prev;      // there is a previous tile (not the CU's first)
  bool has_next;  // there is a next tile (this tile's quadrants leave in K-tile T-1)
  long dA, dB;    // next tile's element offsets from this one
  int nm0, nn0;   // next tile's origin (masked build: its sources are clamped per tile)
  int m0, n0;     // this tile's origin
};

// One phase. CONV: quadrant stored in this phase's load segment when ON (-1
// none; 0..3 = q0..q3 in finishing order; q3 belongs to the previous tile, so
// its origin is e.pm0 / e.pn0; 10 + O = boundary phase O of the SPREAD build);
// ON: e.prev (K-tiles 0 / 1) or e.has_next (K-tile T-1); VMC: the counted wait
// when ON (10 otherwise); NX: this phase's piece is past the tile (issue6). A
// stored quadrant is zeroed for the next tile.
template <int P, bool ODD, int CONV, int VMC, bool NX, int POL, bool MASK = false, bool TL = false,
          bool F8 = false, int PF = -1, int XV = 0>
__device__ __forceinline__ void phase6(const GemmArgs& p, const Ctx& c, Frags3& f,
                                       f32x4 (&acc)[2][2][4][2], int t, int T, const Edge& e,
                                       bool on, int c_lane, int lane = 0, int lrow = 0,
                                       int lcol = 0) {
  bf16x8(&bcur)[2][2] = ODD ? f.b1 : f.b0;
  bf16x8(&both)[2][2] = ODD ? f.b0 : f.b1;
  const int cur = t & 1;
  if constexpr (P == 0) read_a<kALo>(c, f.a, cur);
  if constexpr (P == 1) read_b<kBHi>(c, both, cur);
  if constexpr (P == 2) read_a<kAHi>(c, f.a, cur);
  if constexpr (P == 3) read_b<kBLo>(c, both, cur ^ 1);  // K-tile t+1 (next tile's 0 at t = T-1)
  if constexpr (P == 0) issue6<kAHi, NX, MASK, TL>(p, c, t + 1, cur ^ 1, T, e.has_next, e.dA, e.dB, e.nm0, e.nn0, lane);
  if constexpr (P == 1) issue6<kBLo, NX, MASK, TL>(p, c, t + 2, cur, T, e.has_next, e.dA, e.dB, e.nm0, e.nn0, lane);
  if constexpr (P == 2) issue6<kALo, NX, MASK, TL>(p, c, t + 2, cur, T, e.has_next, e.dA, e.dB, e.nm0, e.nn0, lane);
  if constexpr (P == 3) issue6<kBHi, NX, MASK, TL>(p, c, t + 2, cur, T, e.has_next, e.dA, e.dB, e.nm0, e.nn0, lane);
  // PF: one L2 touch of the next tile's K-tile 0 / 1 (halves in B-lo A-lo B-hi A-hi
  // order, the real pieces' order) after this phase's piece
  if constexpr (PF >= 0) {
    constexpr int H = (PF & 3) == 0 ? kBLo : (PF & 3) == 1 ? kALo : (PF & 3) == 2 ? kBHi : kAHi;
    prefetch6<H, PF / 4>(c, T, e.has_next, e.dA, e.dB);
  }
  // POL 2 (C not stored): no stores in the stream, so the pieces-only count
  // (round 3's ablation kept the store-counting waits, which then under-waited);
  // XV: the prefetch ops younger than the awaited piece (PF builds)
  if constexpr (VMC == 10 || POL == 2) {
    wait_vm<10 + XV>();
  } else {
    if (on)
      wait_vm<VMC + XV>();
    else
      wait_vm<10 + XV>();
  }
  if constexpr (F8 && CONV >= 0) {
    if (on) mfma_wait_states();
  }
  if constexpr (CONV >= 10) {  // SPREAD build: boundary phase O = CONV - 10
    if (on) {
      constexpr int O = CONV - 10;
      spread_unit<O, 0, POL, MASK>(p, acc, e.m0, e.n0, e.pm0, e.pn0, c_lane, lrow, lcol);
      spread_unit<O, 1, POL, MASK>(p, acc, e.m0, e.n0, e.pm0, e.pn0, c_lane, lrow, lcol);
      spread_unit<O, 2, POL, MASK>(p, acc, e.m0, e.n0, e.pm0, e.pn0, c_lane, lrow, lcol);
      spread_unit<O, 3, POL, MASK>(p, acc, e.m0, e.n0, e.pm0, e.pn0, c_lane, lrow, lcol);
    }
  } else if constexpr (CONV >= 0) {
    if (on) {
      constexpr int MH = (CONV == 2 || CONV == 3) ? 1 : 0;
      constexpr int NH = (CONV == 1 || CONV == 2) ? 1 : 0;
      if constexpr (POL == 2) {  // ablation (experimental library): C not stored
        if (p.ldc < 0)
          store_quadrant<MH, NH, 1>(p, acc[MH][NH], CONV == 3 ? e.pm0 : e.m0,
                                    CONV == 3 ? e.pn0 : e.n0, c_lane);
      } else {
        store_quadrant<MH, NH, POL, MASK>(p, acc[MH][NH], CONV == 3 ? e.pm0 : e.m0,
                                          CONV == 3 ? e.pn0 : e.n0, c_lane, lrow, lcol);
      }
      zero_quadrant(acc[MH][NH]);
    }
  }
  raw_barrier();
  // F8 + SPREAD: a quadrant zeroed in this phase's load segment (its last store
  // block, boundary phase O >= 3) is srcC of this segment's asm MFMAs, which
  // hipcc does not pad; hipcc may sink the zeroing to the barrier, so the pad
  // goes after it (unconditionally: 16 cycles in 4 phases per tile)
  if constexpr (F8 && CONV >= 13) asm volatile("s_nop 15" ::: "memory");
  if constexpr (P == 0) mma_q<F8>(acc[0][0], f.a, bcur);
  if constexpr (P == 1) mma_q<F8>(acc[0][1], f.a, both);
  if constexpr (P == 2) mma_q<F8>(acc[1][1], f.a, both);
  if constexpr (P == 3) mma_q<F8>(acc[1][0], f.a, bcur);
  raw_barrier();
}

#define NTM_PHT(P, ODD, CV, VMC, NX, ON, TL) \
  phase6<P, ODD, CV, VMC, NX, POL, MASK, TL, F8>(p, c, f, acc, t, T, e, ON, c_lane, lane, lrow, lcol)
#define NTM_PH(P, ODD, CV, VMC, NX, ON) NTM_PHT(P, ODD, CV, VMC, NX, ON, false)
// PF builds: steady-state phase with prefetch PF and XV extra ops in its wait
#define NTM_PHP(P, ODD, CV, VMC, NX, ON, PFI, XVI) \
  phase6<P, ODD, CV, VMC, NX, POL, MASK, false, F8, PFI, XVI>(p, c, f, acc, t, T, e, ON, c_lane, lane, lrow, lcol)
// STAMP 2: shader-clock stamp I of wave 0 at a phase start of the workgroup's
// first tile boundary (K-tiles T-2 / T-1 of its first tile: I = 0..7, K-tiles
// 0 / 1 of its second: I = 8..15, 16 = after K-tile 1), into p.stamps[17 b + I]
#define NTM_ST(I, FIRST)                                                          \
  if constexpr (STAMP == 2) {                                                     \
    if (tile == (int)blockIdx.x + ((FIRST) ? 0 : G)) {                            \
      unsigned long long st_t, st_rt;                                             \
      clock_stamp(st_t, st_rt);                                                   \
      if (threadIdx.x == 0) p.stamps[17 * (size_t)blockIdx.x + (I)] = st_t;       \
    }                                                                             \
  }

__device__ __forceinline__ void tile_origin(const GemmArgs& p, int tile, int ntiles, int& m0,
                                            int& n0) {
  int tm, tn;
  tile_coords_of<kGroupM>(tile, ntiles, p.M, p.N, tm, tn);
  m0 = tm * BM;
  n0 = tn * BN;
}

// Words per workgroup of the STAMP 1 clock build's record.
constexpr int kClockStampWords = 6;

// Clock stamp (STAMP builds): shader-clock and 100 MHz real-time counters read
// together, the wait inside the statement (cdna_hip_programming.md §7).
__device__ __forceinline__ void clock_stamp(unsigned long long& t, unsigned long long& rt) {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(t), "=s"(rt)::"memory");
  __builtin_amdgcn_sched_barrier(0);
}

// POL: C store policy of store_c16 (1 = nontemporal, the shipping build).
// STAMP 1 (the clock build, never in the default dispatch): lane 0 of wave 0
// records s_memtime / s_memrealtime at kernel start and after the last store,
// then the raw XCC_ID and HW_ID registers, into p.stamps[kClockStampWords *
// blockIdx.x ..]: the GEMM's own clock = d(memtime) / d(realtime) x 100 MHz,
// grouped by the XCD that really ran the workgroup.
// MASK ("pingpong8om"): ragged C - ceil(M/256) x
// ceil(N/256) tiles, sources clamped per tile (src_clamped), stores masked.
// TAIL (with MASK): K % 128 != 0 - T = ceil(K / 128) * 2 K-tiles; the pieces
// that can reach past K (K-tiles T-2 / T-1, issued from K-tiles T-4 .. T-2, or
// from K-tiles 0 / 1 when T = 4) zero-fill their chunks past K.
// SPREAD (the shipping build, "pingpong8od"): each boundary quadrant's 4 store
// blocks go out one per phase over the 4 phases it has before its reuse
// (stores per phase 1,2,3,4,3,2,1 from P1 of K-tile T-1 to P3 of the next
// tile's K-tile 0, instead of 4,4,4,4); counted waits 10 + stores in phases
// j-5 .. j-1: P1(T-1) 10, P2 11, P3 13, P0(0) 16, P1 20, P2 23, P3 24,
// P0(1) 23, P1 20, P2 16, P3 13 (P0(2) needs 11; the loop's 10 over-waits by
// one store issued 5 phases earlier).
// F8: OCP e4m3 operands (K / lda / ldb in bf16-sized pairs, as K1-fp8's
// pingpong8c), f8f6f4 MFMAs on VGPR accumulators (mfma_f8_vgpr; pingpong8c's
// fp8 build keeps them in AGPRs, and with 128 + 128 registers there its
// boundary conversion spilled).
// (Round 4 also measured a whole-128-B-line C layout, with and without LDS
// staging of the boundary stores: exactly 128 MB written instead of 157 MB,
// no faster. Removed after measurement, profiles/r4_stg/; git history has it.)
template <int POL, int STAMP = 0, bool MASK = false, bool TAIL = false, bool SPREAD = false,
          bool F8 = false, bool PF = false>
__global__ void __launch_bounds__(kThreads, 2) gemm_bf16_pp6_kernel(GemmArgs p) {
  static_assert(!TAIL || MASK, "partial K rides on the masked build");
  static_assert(!PF || (!MASK && !TAIL), "the L2 prefetch is on the whole-tile build");
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes3];
  unsigned long long t0 = 0, rt0 = 0;
  if constexpr (STAMP == 1) clock_stamp(t0, rt0);
  const int ntiles = MASK ? ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN) : (p.M / BM) * (p.N / BN);
  const int G = (int)gridDim.x;
  int tile = (int)blockIdx.x;

  Ctx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  Edge e;
  tile_origin(p, tile, ntiles, e.m0, e.n0);
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    const int rb = c.w * 16 + r;
    const __bf16* a0 = p.A + (size_t)(e.m0 + c.w * 16 + r) * p.lda + cl * 8;
    const __bf16* b0 = p.B + (size_t)(e.n0 + rb) * p.ldb + cl * 8;
    c.src[kALo] = a0;
    c.src[kAHi] = a0 + (size_t)128 * p.lda;
    c.src[kBLo] = b0;
    c.src[kBHi] = b0 + (size_t)128 * p.ldb;
    if constexpr (MASK) {
      c.src[kALo] = src_clamped<kALo>(p, e.m0, e.n0, c.w, lane);
      c.src[kAHi] = src_clamped<kAHi>(p, e.m0, e.n0, c.w, lane);
      c.src[kBLo] = src_clamped<kBLo>(p, e.m0, e.n0, c.w, lane);
      c.src[kBHi] = src_clamped<kBHi>(p, e.m0, e.n0, c.w, lane);
    }
  }
  // masked stores: the wave's row / column offset inside a quadrant (uniform;
  // the lane part is recomputed at the store, opaque_lane)
  const int lrow = c.wr * 64;
  const int lcol = c.wc * 32;
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
  const int c_lane = (c.wr * 64 + (lane & 15)) * p.ldc + c.wc * 32 +
                     ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) zero_quadrant(acc[i][j]);
  Frags3 f;
  const int T = TAIL ? ((p.K + 2 * BK - 1) / (2 * BK)) * 2 : p.K / BK;
  if constexpr (TAIL) c.K = p.K;
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
  e.nm0 = nm0;
  e.nn0 = nn0;

  // prologue of the first tile: B-lo0 A-lo0 B-hi0 A-hi0 B-lo1 A-lo1 B-hi1
  issue_half<kBLo>(c, 0, 0);
  issue_half<kALo>(c, 0, 0);
  issue_half<kBHi>(c, 0, 0);
  issue_half<kAHi>(c, 0, 0);
  issue_half<kBLo>(c, 1, 1);
  issue_half<kALo>(c, 1, 1);
  issue_half<kBHi>(c, 1, 1);
  wait_vm<10>();
  raw_barrier();
  read_b<kBLo>(c, f.b0, 0);
  if (c.wr == 1) raw_barrier();  // ping-pong stagger

  // One iteration per tile; the only data-dependent control flow is uniform
  // branches around the boundary stores / waits, so the accumulators keep
  // their registers around the back edge.
  for (;;) {
    int t = 0;
    // STAMP 3 (ablation, experimental library only; C is wrong): a workgroup on an
    // odd XCD cuts its LAST tile's K loop by 2 p.splitk_kc K-tiles - the timing of
    // a launch whose odd XCDs (the slower ones, profiles/r6_xcd) carry less work
    const int Tl = STAMP == 3 && !e.has_next && (blockIdx.x & 1) ? T - 2 * p.splitk_kc : T;
    // K-tile 0: q3 of the previous tile leaves in P0 (SPREAD: blocks of q0..q3 in P0..P3)
    NTM_ST(8, false);
    NTM_PHT(0, false, SPREAD ? 13 : 3, SPREAD ? 16 : 22, false, e.prev, TAIL);
    NTM_ST(9, false);
    NTM_PHT(1, false, SPREAD ? 14 : -1, SPREAD ? 20 : 26, false, e.prev, TAIL);
    NTM_ST(10, false);
    NTM_PHT(2, false, SPREAD ? 15 : -1, SPREAD ? 23 : 26, false, e.prev, TAIL);
    NTM_ST(11, false);
    NTM_PHT(3, false, SPREAD ? 16 : -1, SPREAD ? 24 : 22, false, e.prev, TAIL);
    t = 1;
    NTM_ST(12, false);
    NTM_PHT(0, true, -1, SPREAD ? 23 : 18, false, e.prev, TAIL);
    NTM_ST(13, false);
    NTM_PHT(1, true, -1, SPREAD ? 20 : 14, false, e.prev, TAIL);
    NTM_ST(14, false);
    NTM_PHT(2, true, -1, SPREAD ? 16 : 10, false, e.prev, TAIL);
    NTM_ST(15, false);
    NTM_PHT(3, true, -1, SPREAD ? 13 : 10, false, e.prev, TAIL);
    NTM_ST(16, false);
    // PF: the last steady pair (T-4 / T-3; T >= 6) is peeled to carry the L2
    // touches. Phase j's wait retires phase j-5's piece; every touch issued
    // after it - phases j-5 .. j, each after its own piece - may stay in flight
    // (one op each): vmcnt 11 12 13 14 15 16 16 16 (T-4, T-3), 15 14 13 12 (T-2),
    // 11 (T-1 P0)
#pragma nounroll
    for (t = 2; t < Tl - (TAIL ? 4 : 2) - (PF ? 2 : 0); t += 2) {
      NTM_PH(0, false, -1, 10, false, false);
      NTM_PH(1, false, -1, 10, false, false);
      NTM_PH(2, false, -1, 10, false, false);
      NTM_PH(3, false, -1, 10, false, false);
      ++t;
      NTM_PH(0, true, -1, 10, false, false);
      NTM_PH(1, true, -1, 10, false, false);
      NTM_PH(2, true, -1, 10, false, false);
      NTM_PH(3, true, -1, 10, false, false);
      --t;
    }
    if constexpr (TAIL) {
      // the K-tile pair T-4 / T-3 issues K-tiles T-3 .. T-1: zero-fill past K
      if (T >= 6) {
        t = T - 4;
        NTM_PHT(0, false, -1, 10, false, false, true);
        NTM_PHT(1, false, -1, 10, false, false, true);
        NTM_PHT(2, false, -1, 10, false, false, true);
        NTM_PHT(3, false, -1, 10, false, false, true);
        ++t;
        NTM_PHT(0, true, -1, 10, false, false, true);
        NTM_PHT(1, true, -1, 10, false, false, true);
        NTM_PHT(2, true, -1, 10, false, false, true);
        NTM_PHT(3, true, -1, 10, false, false, true);
      }
    }
    if constexpr (PF) {  // T >= 6 (the launcher's rule for PF builds)
      t = T - 4;
      NTM_PHP(0, false, -1, 10, false, false, 0, 1);
      NTM_PHP(1, false, -1, 10, false, false, 1, 2);
      NTM_PHP(2, false, -1, 10, false, false, 2, 3);
      NTM_PHP(3, false, -1, 10, false, false, 3, 4);
      ++t;
      NTM_PHP(0, true, -1, 10, false, false, 4, 5);
      NTM_PHP(1, true, -1, 10, false, false, 5, 6);
      NTM_PHP(2, true, -1, 10, false, false, 6, 6);
      NTM_PHP(3, true, -1, 10, false, false, 7, 6);
    }
    // K-tile T-2 stages the next tile's K-tile 0, K-tile T-1 its K-tile 1 (or
    // dummies); with a next tile, q0..q2 leave in P1..P3 of K-tile T-1 (LINE:
    // row half 0 in P2)
    t = Tl - 2;
    if constexpr (PF) {
      NTM_ST(0, true);
      NTM_PHP(0, false, -1, 10, false, false, -1, 5);
      NTM_ST(1, true);
      NTM_PHP(1, false, -1, 10, true, false, -1, 4);
      NTM_ST(2, true);
      NTM_PHP(2, false, -1, 10, true, false, -1, 3);
      NTM_ST(3, true);
      NTM_PHP(3, false, -1, 10, true, false, -1, 2);
    } else {
      NTM_ST(0, true);
      NTM_PHT(0, false, -1, 10, false, false, TAIL);
      NTM_ST(1, true);
      NTM_PH(1, false, -1, 10, true, false);
      NTM_ST(2, true);
      NTM_PH(2, false, -1, 10, true, false);
      NTM_ST(3, true);
      NTM_PH(3, false, -1, 10, true, false);
    }
    t = Tl - 1;
    NTM_ST(4, true);
    if constexpr (PF)
      NTM_PHP(0, true, -1, 10, true, false, -1, 1);
    else
      NTM_PH(0, true, -1, 10, true, false);
    NTM_ST(5, true);
    NTM_PH(1, true, SPREAD ? 10 : 0, 10, true, e.has_next);
    NTM_ST(6, true);
    NTM_PH(2, true, SPREAD ? 11 : 1, SPREAD ? 11 : 14, true, e.has_next);
    NTM_ST(7, true);
    NTM_PH(3, true, SPREAD ? 12 : 2, SPREAD ? 13 : 18, true, e.has_next);
    if (!e.has_next) break;
    // advance to the next tile
    if constexpr (MASK) {
      const int l = opaque_lane();
      c.src[kALo] = src_clamped<kALo>(p, nm0, nn0, c.w, l);
      c.src[kAHi] = src_clamped<kAHi>(p, nm0, nn0, c.w, l);
      c.src[kBLo] = src_clamped<kBLo>(p, nm0, nn0, c.w, l);
      c.src[kBHi] = src_clamped<kBHi>(p, nm0, nn0, c.w, l);
    } else {
#pragma unroll
      for (int h = 0; h < 4; ++h) c.src[h] += (h == kALo || h == kAHi) ? e.dA : e.dB;
    }
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
    e.nm0 = nm0;
    e.nn0 = nn0;
  }
  if (c.wr == 0) raw_barrier();  // balance the stagger
  wait_vm<0>();                  // dummy pieces: nothing may land after the WG exits
  if constexpr (F8) mfma_wait_states();  // asm MFMAs: results land before VALU reads
  if (POL != 2 || p.ldc < 0)
    store_tile_lds<false, POL != 0, MASK, POL == 0 ? 0 : 1>(p, c, acc, e.m0, e.n0, lane);
  if constexpr (STAMP == 1) {
    unsigned long long t1, rt1;
    clock_stamp(t1, rt1);
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const unsigned xcc = xcc_id_raw();
    if (threadIdx.x == 0) {
      unsigned long long* o = p.stamps + kClockStampWords * (size_t)blockIdx.x;
      o[0] = t0;
      o[1] = rt0;
      o[2] = t1;
      o[3] = rt1;
      o[4] = xcc;
      o[5] = hw;
    }
  }
}
#undef NTM_PH
#undef NTM_PHT
#undef NTM_ST

// The CUs the persistent / stream-K grids are sized for (one workgroup per CU)
// and the default plan prices its rounds over: the device's count (its compute
// partition's in DPX / CPX modes), 256 without a device. cu_override() > 0
// replaces it (tests of the plan on other partition sizes, ntm_set_cus_override).
inline int& cu_override() {
  static int v = 0;
  return v;
}

inline int device_cus() {
  if (cu_override() > 0) return cu_override();
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
      cus = 256;
    else
      cus = prop.multiProcessorCount;
  }
  return cus;
}

// Grid: one workgroup per CU (LDS allows no more), fewer if there are fewer tiles.
inline int pp6_grid(int ntiles) {
  const int cus = device_cus();
  return ntiles < cus ? ntiles : cus;
}

// Experimental: an explicit grid (a multiple of 8, at most the tile count) and
// POL 2 (C not stored) - the store-bandwidth study of profiles/r3_stores.
template <int POL, int STAMP = 0, bool SPREAD = false, bool PF = false>
inline hipError_t launch_gemm_bf16_pp6_grid(const GemmArgs& a, int grid, hipStream_t stream) {
  if (!shape_ok6(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) || grid <= 0 || grid % 8 ||
      grid > (a.M / BM) * (a.N / BN) || (PF && a.K < 6 * BK))
    return hipErrorInvalidValue;
  if (STAMP != 0 && a.stamps == nullptr) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_bf16_pp6_kernel<POL, STAMP, false, false, SPREAD, false, PF>),
                     dim3((unsigned)grid), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

template <int POL, int STAMP = 0, bool SPREAD = false, bool PF = false>
inline hipError_t launch_gemm_bf16_pp6(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok6(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) ||
      (STAMP != 0 && STAMP != 3 && a.stamps == nullptr) || (PF && a.K < 6 * BK) ||
      (STAMP == 3 && (a.splitk_kc < 0 || a.K / BK - 2 * a.splitk_kc < 4)))
    return hipErrorInvalidValue;
  const int ntiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((gemm_bf16_pp6_kernel<POL, STAMP, false, false, SPREAD, false, PF>),
                     dim3((unsigned)pp6_grid(ntiles)),
                     dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

// K1-fp8 on the persistent overlap kernel (experimental): whole 256x256 tiles,
// fp8 K % 256 (bf16-pair K % 128); A / B are e4m3 byte images, K / lda / ldb in
// fp8 elements here.
inline bool fp8_pp6_ok(int M, int N, int K, int lda, int ldb, int ldc) {
  return (K % 2) == 0 && (lda % 16) == 0 && (ldb % 16) == 0 && shape_ok6(M, N, K / 2) &&
         lda >= K && ldb >= K && ldc >= N && (ldc % 8) == 0;
}

// PF: the next tile's K-tiles 0 / 1 touched into L2 over K-tiles T-4 / T-3
// (round 6: K1-fp8 is not power-bound, so the boundary cycles the touches save
// can reach the launch time; bf16 lost 0.5-1 % to their energy, profiles/r5_pf).
template <bool SPREAD = false, bool PF = false>
inline hipError_t launch_gemm_fp8_pp6(const void* A, const void* B, __bf16* C, int M, int N,
                                      int K, int lda, int ldb, int ldc, hipStream_t stream) {
  GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = C;
  a.M = M;
  a.N = N;
  a.K = K / 2;
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  if ((K % 2) || (lda % 16) || (ldb % 16) || !shape_ok6(a.M, a.N, a.K) || a.lda < a.K ||
      a.ldb < a.K || a.ldc < a.N || (a.ldc % 8) || (PF && a.K < 6 * BK))
    return hipErrorInvalidValue;
  const int ntiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((gemm_bf16_pp6_kernel<1, 0, false, false, SPREAD, true, PF>),
                     dim3((unsigned)pp6_grid(ntiles)), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

// pingpong8om: ragged C (any M, N % 8), K % 8 and K > 128 (K % 128 != 0 on
// the partial-K build).
template <int POL, bool SPREAD = false>
inline hipError_t launch_gemm_bf16_pp6_masked(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok6m(a.M, a.N, a.K) || a.rowsum || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8))
    return hipErrorInvalidValue;
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const dim3 g((unsigned)pp6_grid(ntiles)), b(kThreads);
  if (a.K % (2 * BK))
    hipLaunchKernelGGL((gemm_bf16_pp6_kernel<POL, 0, true, true, SPREAD>), g, b, 0, stream, a);
  else
    hipLaunchKernelGGL((gemm_bf16_pp6_kernel<POL, 0, true, false, SPREAD>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemm6
}  // namespace ntm
