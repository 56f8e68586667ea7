// K1 4-wave persistent overlap build ("dma4ko"): dma4k (gemm_w4k.hpp: 4 waves,
// one per SIMD, 128x128 outputs per wave, one barrier per K-tile, two K-tile
// LDS-DMA buffers) made persistent, with every tile's C stores OVERLAPPING the
// next tile's K loop. bf16 (v_mfma_f32_16x16x32_bf16) and e4m3
// (v_mfma_f32_16x16x128_f8f6f4) operands, bf16 C.
//
// Why: the per-tile fixed cost, not the loop, is what separates K1 from
// hipBLASLt at 8192^3 (profiles/r3_k1/README.md): a dma4k tile pays a 2.9 K
// cycle prologue, a 10.3 K cycle epilogue (every CU stores its 128 KiB tile
// at the same moment) and the gap to the next workgroup; kfit puts K1-fp8's
// fixed cost at 44 us against hipBLASLt's 27-32 us at equal loop rates, and
// for e4m3 the loop is half as long, so that cost weighs twice as much. The
// 8-wave overlap kernel (pingpong8o, gemm_bf16_pp6.hpp) recovered part of it
// for bf16 but cannot be built for e4m3: two waves per SIMD leave 256
// registers per wave and the e4m3 consumer already holds 128 + 128. Here one
// wave per SIMD has 512: 256 AGPR accumulators, 128 VGPRs of fragments, and
// room for the boundary conversion.
//
// Boundary schedule (T K-tiles per output tile; step t = dma4k's step: row 0 of
// the 8x8 MFMA slots, wait + barrier, rows 1..7 with tile t+2's DMA pieces and
// tile t+1's fragment reads):
//  * accumulator row r (acc[r][0..7], 16 output rows x 128 columns per wave) is
//    final after slot row r of step T-1 and is first rewritten in slot row r of
//    the next tile's step 0. It is converted to bf16 four slot rows later, in
//    the middle of that window: rows 0..3 during slot rows 4..7 of step T-1,
//    rows 4..7 during slot rows 0..3 of the next tile's step 0. Per pair of
//    accumulators (2q, 2q+1): the even one is packed at slot 2q, the odd one
//    at slot 2q+1, which also does the permlane16 swap and one 16-byte
//    nontemporal buffer store (store_tile's lane layout: 8 consecutive columns
//    per lane). Every VALU read of an accumulator is >= 4 slot rows after the
//    asm MFMA that wrote it. Nothing zeroes an accumulator: step 0's MFMAs take
//    C = 0 as an inline constant (mma_z), so no VALU writes an AGPR that an
//    asm MFMA then reads (hipcc pads that hazard only for MFMAs it sees).
//  * The DMA stream is uniform: steps T-2 and T-1 stage the NEXT tile's K-tiles
//    0 and 1 (dma4k staged dummies there), so the next tile's prologue is
//    absorbed; the CU's last tile stages dummies (in-bounds re-reads of its last
//    K-tile into the buffer nobody reads again).
//  * Waits. Loads, stores and LDS-DMA retire vmcnt in issue order, so a
//    barrier's wait counts the stores younger than the last piece it needs:
//    step 0 of a non-first tile waits vmcnt(kStoresAfterLast + 4) (the stores
//    of step T-1 issued at or after its last piece, plus the 4 of its own slot
//    row 0); every other barrier waits vmcnt(0) as in dma4k (step 1's covers the
//    12 stores of step 0's slot rows 1..3, issued >= 20 slots earlier).
//  * The CU's last tile converts rows 4..7 after its loop (behind an MFMA
//    drain: those rows were written just before), then vmcnt(0).
// Operand / C addressing: buffer descriptors; the tile origin rides in the
// scalar soffset (per-lane offsets are tile-independent), so moving to the next
// tile and every C store cost no address VALU.
// Results are bitwise equal to dma4k and the 8-wave default (same K order per
// accumulator). Shape rule: M, N % 256; bf16 K % 128, K >= 256; e4m3 K % 256,
// K >= 512; 16-byte aligned rows; A, B and C < 2 GiB (32-bit buffer offsets).
// Grid = min(tiles, CUs): workgroup b walks tiles b, b + G, ... (G % 8 == 0 keeps
// each XCD's tiles on that XCD).
#pragma once

#include "ntm/gemm_bf16_pp6.hpp"
#include "ntm/gemm_w4k.hpp"

namespace ntm {
namespace w4o {

using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::pack_bf16x2;
using ::ntm::gemm::raw_barrier;
using ::ntm::w4k::BM;
using ::ntm::w4k::BN;
using ::ntm::w4k::Frags8;
using ::ntm::w4k::kBuf;
using ::ntm::w4k::kOp;
using ::ntm::w4k::kThreads;
using ::ntm::w4k::u32x4;

constexpr int kLds = 2 * kBuf;  // 128 KiB: two K-tile buffers (no LDS-staged epilogue)
constexpr int kGroupM = 8;
constexpr int kNtStore = 2;     // buffer-instruction aux: nt (gfx940+ cache policy)

// Stores issued in step T-1 at or after its last DMA piece (pieces at slot
// j % DI == 0, j / DI < 16, j = (slot row - 1) * 8 + nt; stores at odd nt of
// slot rows 4..7; within a slot the piece is issued before the store).
constexpr int stores_after_last_piece(int DI) {
  const int last = 15 * DI;
  int n = 0;
  for (int row = 4; row < 8; ++row)
    for (int nt = 1; nt < 8; nt += 2)
      if ((row - 1) * 8 + nt >= last) ++n;
  return n;
}

struct Ctx {
  char* lds;
  __amdgpu_buffer_rsrc_t rsa, rsb, rsc;
  int voff_a, voff_b;      // lane's source chunk in the wave's first row block (bytes, tile-independent)
  int rowblk_a, rowblk_b;  // 16 rows in bytes
  int rd_a, rd_b;          // lane's fragment offset + wave's first A / B subtile
  int voff_c;              // lane's 16-byte C chunk in a tile, accumulator row 0, pair 0 (bytes)
  int rows16_c;            // 16 rows of C in bytes
};

// Per-tile scalar state: byte offsets of the tile origin in A / B / C.
struct Tile {
  int sa, sb, sc;     // this tile
  int nsa, nsb;       // next tile (== this tile when there is none)
  int psc;            // previous tile's C origin
  __amdgpu_buffer_rsrc_t rsp;  // C descriptor of the previous tile's stores: num_records 0
                               // (every store dropped) on the CU's first tile
  bool has_next;
};

// Piece i (0..15) of K-tile kt of this tile (dma4k's piece map). NX: kt >= T,
// i.e. the next tile's K-tile kt - T, or an in-bounds dummy re-read of this
// tile's last K-tile when there is no next tile.
template <bool NX>
__device__ __forceinline__ void issue_piece(const Ctx& c, const Tile& s, int kt, int T, int buf,
                                            int w, int i) {
  const bool is_b = i >= 8;
  const int rbi = (i >> 1) & 3, ks = i & 1;
  int base, kb;
  if constexpr (NX) {
    base = s.has_next ? (is_b ? s.nsb : s.nsa) : (is_b ? s.sb : s.sa);
    kb = (s.has_next ? kt - T : T - 1) * 128;
  } else {
    base = is_b ? s.sb : s.sa;
    kb = kt * 128;
  }
  char* dst = c.lds + buf * kBuf + (is_b ? kOp : 0) + ((w * 4 + rbi) * 2 + ks) * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(is_b ? c.rsb : c.rsa, (NTM_AS3 void*)dst, 16,
                                           is_b ? c.voff_b : c.voff_a,
                                           base + kb + ks * 64 + rbi * (is_b ? c.rowblk_b : c.rowblk_a),
                                           0, 0);
}

__device__ __forceinline__ void read_a(const Ctx& c, Frags8& f, int buf, int mt) {
  const char* p = c.lds + buf * kBuf + c.rd_a + mt * 2048;
  f.a[mt][0] = *(const bf16x8*)p;
  f.a[mt][1] = *(const bf16x8*)(p + 1024);
}

__device__ __forceinline__ void read_b(const Ctx& c, Frags8& f, int buf, int nt) {
  const char* p = c.lds + buf * kBuf + c.rd_b + nt * 2048;
  f.b[nt][0] = *(const bf16x8*)p;
  f.b[nt][1] = *(const bf16x8*)(p + 1024);
}

// First MFMA slot of a tile on accumulator acc: C = 0 as an inline constant,
// so nothing writes the accumulator registers before it. (Zeroing them in C++
// made hipcc park a zero f32x4 in VGPRs and copy it into the AGPRs right
// before each asm MFMA, inside the VALU-write -> MFMA-srcC hazard window that
// it does not pad for inline asm: element 0 of the first accumulators read
// stale data. profiles/r3_w4o/README.md.)
template <bool F8>
__device__ __forceinline__ void mma_z(f32x4& acc, const Frags8& f, int mt, int nt) {
  if constexpr (F8) {
    asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, 0"
        : "=a"(acc)
        : "v"(::ntm::gemm::cat_f8(f.b[nt][0], f.b[nt][1])), "v"(::ntm::gemm::cat_f8(f.a[mt][0], f.a[mt][1])));
  } else {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(f.b[nt][0]), "v"(f.a[mt][0]));
    ::ntm::w4k::mfma_bf16(acc, f.b[nt][1], f.a[mt][1]);
  }
}

// Conversion of accumulator acc[.][2q + ODD] at its slot: pack to bf16 (the
// next tile's first MFMA on it ignores its old value: mma_z); the odd slot also swaps the pair into 8 consecutive columns per lane and
// stores 16 bytes (C row block r of the tile at byte offset sc).
template <bool ODD>
__device__ __forceinline__ void conv(const Ctx& c, __amdgpu_buffer_rsrc_t rs, f32x4& acc,
                                     unsigned (&pk)[2][2], int q, int r, int sc) {
  pk[ODD][0] = pack_bf16x2(acc[0], acc[1]);
  pk[ODD][1] = pack_bf16x2(acc[2], acc[3]);

  if constexpr (ODD) {
    unsigned w0[2], w1[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const auto x = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
      w0[h] = x[0];
      w1[h] = x[1];
    }
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{w0[0], w0[1], w1[0], w1[1]}, rs,
                                           c.voff_c + q * 64, sc + r * c.rows16_c, kNtStore);
  }
}

// One K-tile step on buffer BUF (fragments of tile t in f on entry, of t+1 on
// exit); dma4k's step plus the boundary work. CV 0: none; 1 (step T-1):
// convert rows 0..3 of this tile in slot rows 4..7; 2 (step 0): convert rows
// 4..7 of the previous tile in slot rows 0..3. On the CU's first tile step 0
// runs the same code on the (zero) accumulators with a C descriptor of no
// records, so its stores are dropped: a branch around the conversions made the
// accumulators merge at every slot and spilled.
template <int BUF, int DI, bool F8, bool NX, int CV>
__device__ __forceinline__ void step(const Ctx& c, const Tile& s, f32x4 (&acc)[8][8], Frags8& f,
                                     int t, int T, int w, bool prev) {
  static_assert(DI >= 1 && 15 * DI <= 55, "16 pieces within rows 1..7");
  constexpr int kAfter = stores_after_last_piece(DI);
  unsigned pk[2][2];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    if constexpr (CV == 2)
      mma_z<F8>(acc[0][nt], f, 0, nt);
    else
      ::ntm::w4k::mma<F8>(acc[0][nt], f, 0, nt);
    if constexpr (CV == 2) {
      if (nt & 1)
        conv<true>(c, s.rsp, acc[4][nt], pk, nt >> 1, 4, s.psc);
      else
        conv<false>(c, s.rsp, acc[4][nt], pk, nt >> 1, 4, s.psc);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (CV == 2) {
    // (the first tile waits for everything: its dropped row-0 stores retire
    // at once, and whether they count at all is not something to rely on)
    if (prev)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kAfter + 4) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 landed (this wave's pieces)
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();  // tile t+1 visible; every read of tile t retired
#pragma unroll
  for (int mt = 1; mt < 8; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      if constexpr (CV == 2)
        mma_z<F8>(acc[mt][nt], f, mt, nt);
      else
        ::ntm::w4k::mma<F8>(acc[mt][nt], f, mt, nt);
      const int j = (mt - 1) * 8 + nt;  // 0..55
      if ((j % DI) == 0 && j / DI < 16) issue_piece<NX>(c, s, t + 2, T, BUF, w, j / DI);
      if (nt == 1) read_a(c, f, BUF ^ 1, mt - 1);
      if (mt == 7) read_b(c, f, BUF ^ 1, nt);
      if constexpr (CV == 1) {
        if (mt >= 4) {
          if (nt & 1)
            conv<true>(c, c.rsc, acc[mt - 4][nt], pk, nt >> 1, mt - 4, s.sc);
          else
            conv<false>(c, c.rsc, acc[mt - 4][nt], pk, nt >> 1, mt - 4, s.sc);
        }
      }
      if constexpr (CV == 2) {
        if (mt <= 3) {
          if (nt & 1)
            conv<true>(c, s.rsp, acc[mt + 4][nt], pk, nt >> 1, mt + 4, s.psc);
          else
            conv<false>(c, s.rsp, acc[mt + 4][nt], pk, nt >> 1, mt + 4, s.psc);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  read_a(c, f, BUF ^ 1, 7);
  __builtin_amdgcn_sched_barrier(0);
}

// Rows 4..7 of the CU's last tile, converted after its K loop.
__device__ __forceinline__ void conv_rows_4_7(const Ctx& c, f32x4 (&acc)[8][8], int sc) {
  unsigned pk[2][2];
#pragma unroll
  for (int r = 4; r < 8; ++r)
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      if (nt & 1)
        conv<true>(c, c.rsc, acc[r][nt], pk, nt >> 1, r, sc);
      else
        conv<false>(c, c.rsc, acc[r][nt], pk, nt >> 1, r, sc);
    }
}

__device__ __forceinline__ void tile_origin(const GemmArgs& p, int tile, int ntiles, int& m0,
                                            int& n0) {
  int tm, tn;
  ::ntm::gemm::tile_coords_of<kGroupM>(tile, ntiles, p.M, p.N, tm, tn);
  m0 = tm * BM;
  n0 = tn * BN;
}

__device__ __forceinline__ void set_origin(const GemmArgs& p, int m0, int n0, int& sa, int& sb,
                                           int& sc) {
  sa = m0 * p.lda * 2;
  sb = n0 * p.ldb * 2;
  sc = (m0 * p.ldc + n0) * 2;
}

// GemmArgs carries e4m3 operands as bf16-sized pairs (K, lda, ldb in pairs),
// so the byte geometry is the same for both dtypes.
template <int DI, bool F8>
__global__ void __launch_bounds__(kThreads, 1) gemm_w4o_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int ntiles = (p.M / BM) * (p.N / BN);
  const int G = (int)gridDim.x;
  int tile = (int)blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  Ctx c;
  c.lds = smem;
  c.rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 2, 0x00020000);
  c.rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.N * p.ldb * 2, 0x00020000);
  c.rsc = __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, p.M * p.ldc * 2, 0x00020000);
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.voff_a = ((w * 64 + r) * p.lda + cl * 8) * 2;
    c.voff_b = ((w * 64 + r) * p.ldb + cl * 8) * 2;
    c.rowblk_a = 16 * p.lda * 2;
    c.rowblk_b = 16 * p.ldb * 2;
    const int fo = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
    c.rd_a = fo + wr * 8 * 2048;
    c.rd_b = kOp + fo + wc * 8 * 2048;
    const int g = lane >> 4;
    const int coff = (g & 1) * 16 + (g >> 1) * 8;
    c.voff_c = ((wr * 128 + (lane & 15)) * p.ldc + wc * 128 + coff) * 2;
    c.rows16_c = 16 * p.ldc * 2;
  }

  Tile s;
  {
    int m0, n0;
    tile_origin(p, tile, ntiles, m0, n0);
    set_origin(p, m0, n0, s.sa, s.sb, s.sc);
  }
  s.psc = s.sc;
  s.rsp = __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, 0, 0x00020000);
  s.has_next = tile + G < ntiles;
  s.nsa = s.sa;
  s.nsb = s.sb;
  int nsc = s.sc;
  if (s.has_next) {
    int m0, n0;
    tile_origin(p, tile + G, ntiles, m0, n0);
    set_origin(p, m0, n0, s.nsa, s.nsb, nsc);
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / 64;  // K-tiles of 128 bytes per row; even, >= 4
  Frags8 f;
  // prologue of the first tile: K-tiles 0 and 1 in flight, 0 landed and read
#pragma unroll
  for (int i = 0; i < 16; ++i) issue_piece<false>(c, s, 0, T, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) issue_piece<false>(c, s, 1, T, 1, w, i);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    read_a(c, f, 0, i);
    read_b(c, f, 0, i);
  }

  bool prev = false;
  for (;;) {
    step<0, DI, F8, false, 2>(c, s, acc, f, 0, T, w, prev);
    step<1, DI, F8, false, 0>(c, s, acc, f, 1, T, w, prev);
    for (int t = 2; t < T - 2; t += 2) {
      step<0, DI, F8, false, 0>(c, s, acc, f, t, T, w, prev);
      step<1, DI, F8, false, 0>(c, s, acc, f, t + 1, T, w, prev);
    }
    step<0, DI, F8, true, 0>(c, s, acc, f, T - 2, T, w, prev);
    step<1, DI, F8, true, 1>(c, s, acc, f, T - 1, T, w, prev);
    if (!s.has_next) break;
    // advance: the next tile's K-tiles 0 / 1 are in flight, 0's fragments in f
    s.psc = s.sc;
    s.rsp = c.rsc;
    s.sa = s.nsa;
    s.sb = s.nsb;
    s.sc = nsc;
    prev = true;
    tile += G;
    s.has_next = tile + G < ntiles;
    if (s.has_next) {
      int m0, n0;
      tile_origin(p, tile + G, ntiles, m0, n0);
      set_origin(p, m0, n0, s.nsa, s.nsb, nsc);
    }
  }
  ::ntm::gemm::mfma_drain();  // the last asm MFMAs wrote rows 4..7 just now
  conv_rows_4_7(c, acc, s.sc);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy pieces and stores retired
}

inline bool sizes_ok(const GemmArgs& a) {
  return (long long)a.M * a.lda * 2 < (1ll << 31) && (long long)a.N * a.ldb * 2 < (1ll << 31) &&
         (long long)a.M * a.ldc * 2 < (1ll << 31);
}

// Grid: one workgroup per CU (the accumulators allow no more), fewer if there
// are fewer tiles.
inline int grid_for(int ntiles) { return ::ntm::gemm6::pp6_grid(ntiles); }

// bf16: M, N % 256, K % 128, K >= 256.
template <int DI = 3>
inline hipError_t launch_gemm_bf16_w4o(const GemmArgs& a, hipStream_t stream) {
  if (a.M <= 0 || a.N <= 0 || a.K < 256 || (a.M % BM) || (a.N % BN) || (a.K % 128) ||
      a.lda < a.K || a.ldb < a.K || a.ldc < a.N || (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) ||
      a.rowsum || !sizes_ok(a))
    return hipErrorInvalidValue;
  const int ntiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((gemm_w4o_kernel<DI, false>), dim3((unsigned)grid_for(ntiles)), dim3(kThreads),
                     0, stream, a);
  return hipGetLastError();
}

// e4m3: K, lda, ldb in fp8 elements; M, N % 256, K % 256, K >= 512.
template <int DI = 2>
inline hipError_t launch_gemm_fp8_w4o(const void* A, const void* B, __bf16* C, int M, int N, int K,
                                      int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K < 512 || (M % BM) || (N % BN) || (K % 256) || lda < K || ldb < K ||
      ldc < N || (lda % 16) || (ldb % 16) || (ldc % 8))
    return hipErrorInvalidValue;
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
  if (!sizes_ok(a)) return hipErrorInvalidValue;
  const int ntiles = (M / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_w4o_kernel<DI, true>), dim3((unsigned)grid_for(ntiles)), dim3(kThreads),
                     0, stream, a);
  return hipGetLastError();
}

}  // namespace w4o
}  // namespace ntm
