// K1 v7 ("ring4"): bf16 / e4m3 GEMM with 4 waves, one per SIMD, each owning a
// 128x128 block of a 256x256 output tile; ONE barrier per K-tile and an
// LDS-DMA ring of five half-K-tile slots, so every DMA piece gets one to two
// K-tiles of lead.
//
//   C[M x N] (bf16) = A[M x K] * B[N x K]^T, fp32 accumulate; bf16 operands on
//   v_mfma_f32_16x16x32_bf16 (two per MFMA slot), e4m3 on
//   v_mfma_f32_16x16x128_f8f6f4 (one per slot).
//
// Lineage (profiles/r3_k1): the 4-wave 128x128-per-wave core reads 0.25
// ds_read_b128 per bf16 MFMA and runs at 1.38x the 8-wave default with its
// staging removed. The half-step ring of gemm_bf16_r4d.hpp paid a barrier
// every 64 MFMAs: 1450-1480 TF/s at 8192^3. The one-barrier-per-K-tile step of
// gemm_fp8_r4d.hpp ("dma4k") reached the default's rate (1645-1653 vs 1636,
// hipBLASLt 1649) but its two K-tile buffers give a DMA piece at most one
// K-tile of lead, so it must cram the 16 pieces into the first 46 slots.
//
// Ring: slot h % 5 holds half-step h = (K-tile h / 2, k-half h % 2): A[256 x 32
// bf16] then B[256 x 32], 16x32-bf16 subtiles (1 KiB = one fragment), the
// XOR-swizzled lane-linear image of every K1 kernel (swizzle on the source).
// Step t (K-tile t, 64 MFMA slots as 8 rows x 8 columns; fragments of tile t
// in registers on entry):
//   row 0; s_waitcnt vmcnt(8) + lgkmcnt(0); s_barrier (= barrier t);
//   rows 1..7: 16 DMA pieces, one every DI slots - half-step 2t+5 (tile t+2,
//   high half) into slot 2t % 5, then half-step 2t+6 (tile t+3, low half) into
//   slot (2t+1) % 5 - and the fragment reads of tile t+1 (slots (2t+2) % 5 and
//   (2t+3) % 5): A[mt-1] once row mt-1 has issued, B[nt] after slot (7, nt),
//   A[7] at the end.
// RAW: at barrier t the wave's pieces of half-steps 2t+2 (issued in step
//      t-2) and 2t+3 (step t-1) have landed: only half-step 2t+4's 8 pieces
//      (the second batch of step t-1) are younger -> vmcnt(8).
// WAR: slots 2t % 5 and (2t+1) % 5 held tile t, read during step t-1 after
//      barrier t-1 and retired (lgkmcnt(0)) before barrier t; the DMA of step
//      t follows barrier t.
// Registers: one fragment set (128 VGPRs; an MFMA reads its sources at
//      issue) + 256 AGPR accumulators.
// Past the end the pieces re-read the last half-step into their (free) slot,
// so the counted waits are exact with no tail code; vmcnt(0) before the
// epilogue reuses LDS for the C tile.
// Shape rule: M, N % 256; K % 128 (bf16) / K % 256 (e4m3), K-tiles >= 2;
// 16-byte aligned rows; operands < 2 GiB.
#pragma once

#include "ntm/gemm_bf16_r4.hpp"
#include "ntm/gemm_fp8.hpp"

namespace ntm {
namespace ring {

using ::ntm::gemm::cat_f8;
using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::raw_barrier;

constexpr int BM = 256, BN = 256;
constexpr int kThreads = 256;
constexpr int kHalfOp = 256 * 64;    // 16 KiB: one operand of a half-step (32 bf16 / 64 e4m3)
constexpr int kSlot = 2 * kHalfOp;   // 32 KiB
constexpr int kSlots = 5;
constexpr int kLds = kSlots * kSlot; // 160 KiB (>= the 132 KiB C staging)
static_assert(kLds >= ::ntm::gemmr::kLds, "C staging fits the ring");
constexpr int kGroupM = 8;

struct Ctx {
  char* lds;
  __amdgpu_buffer_rsrc_t rsa, rsb;
  int voff_a, voff_b;      // lane's source chunk in row block 4w, half-step 0 (bytes)
  int rowblk_a, rowblk_b;  // 16 rows in bytes
  int rd_a, rd_b;          // lane's fragment offset + wave's first A / B subtile
};

struct Frags {
  bf16x8 a[8][2];  // [m-tile][k-half]
  bf16x8 b[8][2];
};

// Slot geometry. K-split (AB = false): half-step h = (K-tile h / 2, k-half
// h % 2), A[256 x 64 B] then B[256 x 64 B], subtile (row block rb) at rb KiB.
// Operand-split (AB = true): half-step h = (K-tile h / 2, operand h % 2: A
// then B), [256 x 128 B], subtile (rb, k-half ks) at (2 rb + ks) KiB - a DMA
// piece pair fetches both 64-byte halves of a 128-byte line back to back (the
// K-split ring fetches them a K-tile apart).
// Piece i (0..7) of half-step hs into slot s; past the end, the last K-tile.
template <bool AB>
__device__ __forceinline__ void issue_piece(const Ctx& c, int hs, int H, int s, int w, int i) {
  char* dst;
  int soff;
  bool is_b;
  if constexpr (AB) {
    const int kt = (hs >> 1) < (H >> 1) ? (hs >> 1) : (H >> 1) - 1;
    is_b = hs & 1;
    const int rbi = i >> 1, ks = i & 1;
    dst = c.lds + s * kSlot + ((w * 4 + rbi) * 2 + ks) * 1024;
    soff = kt * 128 + ks * 64 + rbi * (is_b ? c.rowblk_b : c.rowblk_a);
  } else {
    const int kb = (hs < H ? hs : H - 1) * 64;  // 64 bytes per half-step row
    is_b = i >= 4;
    const int rbi = i & 3;
    dst = c.lds + s * kSlot + (is_b ? kHalfOp : 0) + (w * 4 + rbi) * 1024;
    soff = kb + rbi * (is_b ? c.rowblk_b : c.rowblk_a);
  }
  __builtin_amdgcn_raw_ptr_buffer_load_lds(is_b ? c.rsb : c.rsa, (NTM_AS3 void*)dst, 16,
                                           is_b ? c.voff_b : c.voff_a, soff, 0, 0);
}

// Fragments of one K-tile: K-split -> k-half 0 from slot s_lo, 1 from s_hi;
// operand-split -> A from s_lo, B from s_hi.
template <bool AB>
__device__ __forceinline__ void read_a(const Ctx& c, Frags& f, int s_lo, int s_hi, int mt) {
  if constexpr (AB) {
    const char* p = c.lds + s_lo * kSlot + c.rd_a + mt * 2048;
    f.a[mt][0] = *(const bf16x8*)p;
    f.a[mt][1] = *(const bf16x8*)(p + 1024);
  } else {
    f.a[mt][0] = *(const bf16x8*)(c.lds + s_lo * kSlot + c.rd_a + mt * 1024);
    f.a[mt][1] = *(const bf16x8*)(c.lds + s_hi * kSlot + c.rd_a + mt * 1024);
  }
}

template <bool AB>
__device__ __forceinline__ void read_b(const Ctx& c, Frags& f, int s_lo, int s_hi, int nt) {
  if constexpr (AB) {
    const char* p = c.lds + s_hi * kSlot + c.rd_b + nt * 2048;
    f.b[nt][0] = *(const bf16x8*)p;
    f.b[nt][1] = *(const bf16x8*)(p + 1024);
  } else {
    f.b[nt][0] = *(const bf16x8*)(c.lds + s_lo * kSlot + c.rd_b + nt * 1024);
    f.b[nt][1] = *(const bf16x8*)(c.lds + s_hi * kSlot + c.rd_b + nt * 1024);
  }
}

template <bool F8>
__device__ __forceinline__ void mma(f32x4& acc, const Frags& f, int mt, int nt) {
  if constexpr (F8) {
    ::ntm::gemm::mfma_f8_agpr_plain(acc, cat_f8(f.b[nt][0], f.b[nt][1]),
                                    cat_f8(f.a[mt][0], f.a[mt][1]));
  } else {
    ::ntm::gemmr::mfma(acc, f.b[nt][0], f.a[mt][0]);
    ::ntm::gemmr::mfma(acc, f.b[nt][1], f.a[mt][1]);
  }
}

__device__ __forceinline__ int wrap5(int x) { return x >= kSlots ? x - kSlots : x; }

// K-tile step t; h0 = (2t) % 5, the slot of tile t's first half-step (a
// rotating scalar: a runtime "% 5" let hipcc fold the division into every
// fragment address, 37 VALU per step). DI: slots between DMA pieces (16
// pieces from the barrier on).
template <bool F8, int DI, bool AB>
__device__ __forceinline__ void step(const Ctx& c, f32x4 (&acc)[8][8], Frags& f, int t, int h0,
                                     int H, int w) {
  static_assert(DI >= 1 && 15 * DI <= 55, "16 pieces within rows 1..7");
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    mma<F8>(acc[0][nt], f, 0, nt);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile t+1 (half-steps 2t+2, 2t+3) landed
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();  // tile t+1 visible; every read of tile t retired
  const int d0 = h0, d1 = wrap5(h0 + 1);                      // tile t's slots: free now
  const int s_lo = wrap5(h0 + 2), s_hi = wrap5(h0 + 3);       // tile t+1
#pragma unroll
  for (int mt = 1; mt < 8; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      mma<F8>(acc[mt][nt], f, mt, nt);
      const int j = (mt - 1) * 8 + nt;  // 0..55
      if ((j % DI) == 0 && j / DI < 16) {
        const int p = j / DI;
        if (p < 8)
          issue_piece<AB>(c, 2 * t + 5, H, d0, w, p);      // tile t+2, high half
        else
          issue_piece<AB>(c, 2 * t + 6, H, d1, w, p - 8);  // tile t+3, low half
      }
      if (nt == 1) read_a<AB>(c, f, s_lo, s_hi, mt - 1);
      if (mt == 7) read_b<AB>(c, f, s_lo, s_hi, nt);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  read_a<AB>(c, f, s_lo, s_hi, 7);
  __builtin_amdgcn_sched_barrier(0);
}

template <bool F8, int DI = 3, bool AB = false, int GROUP_M = kGroupM>
__global__ void __launch_bounds__(kThreads, 1) gemm_ring4_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  int tm, tn;
  ::ntm::gemm::tile_coords<GROUP_M>(p.M, p.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  Ctx c;
  c.lds = smem;
  // e4m3 operands ride as bf16-sized pairs: K, lda, ldb in pairs (launchers)
  c.rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 2, 0x00020000);
  c.rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.N * p.ldb * 2, 0x00020000);
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.voff_a = ((m0 + w * 64 + r) * p.lda + cl * 8) * 2;
    c.voff_b = ((n0 + w * 64 + r) * p.ldb + cl * 8) * 2;
    c.rowblk_a = 16 * p.lda * 2;
    c.rowblk_b = 16 * p.ldb * 2;
  }
  {
    const int fo = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
    c.rd_a = fo + wr * 8 * (AB ? 2048 : 1024);
    c.rd_b = (AB ? 0 : kHalfOp) + fo + wc * 8 * (AB ? 2048 : 1024);
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / 64;  // K-tiles (128 bytes per row each)
  const int H = 2 * T;     // half-steps
  Frags f;
  // prologue: half-steps 0..4 (tiles 0, 1 and the low half of 2) in flight;
  // tile 0 landed (24 younger pieces) and read
#pragma unroll
  for (int hs = 0; hs < 5; ++hs)
#pragma unroll
    for (int i = 0; i < 8; ++i) issue_piece<AB>(c, hs, H, hs, w, i);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    read_a<AB>(c, f, 0, 1, i);
    read_b<AB>(c, f, 0, 1, i);
  }

  // one step per iteration; the last step is peeled (a loop exit straight
  // into the epilogue made hipcc keep scratch copies of accumulators, r4d)
  int t = 0, h0 = 0;
  do {
    step<F8, DI, AB>(c, acc, f, t, h0, H, w);
    ++t;
    h0 = wrap5(h0 + 2);
  } while (t < T - 1);
  step<F8, DI, AB>(c, acc, f, t, h0, H, w);

  ::ntm::gemm::mfma_drain();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy pieces landed before LDS reuse
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  ::ntm::gemmr::Ctx e;
  e.lds = smem;
  ::ntm::gemmr::store_tile<true>(p, e, acc, m0, n0, w, wr, wc, lane);
}

inline bool shape_ok_bf16(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 128 && (M % BM) == 0 && (N % BN) == 0 && (K % 64) == 0;
}

template <int DI = 3, bool AB = false>
inline hipError_t launch_gemm_bf16_ring4(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok_bf16(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) || a.rowsum ||
      (long long)a.M * a.lda * 2 >= (1ll << 31) || (long long)a.N * a.ldb * 2 >= (1ll << 31))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_ring4_kernel<false, DI, AB>), g, b, 0, stream, a);
  return hipGetLastError();
}

// e4m3: K, lda, ldb in fp8 elements (K % 128, K >= 256).
template <int DI = 3, bool AB = false>
inline hipError_t launch_gemm_fp8_ring4(const void* A, const void* B, __bf16* C, int M, int N,
                                        int K, int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K < 256 || (M % BM) || (N % BN) || (K % 128) || lda < K || ldb < K ||
      ldc < N || (lda % 16) || (ldb % 16) || (ldc % 8) || (long long)M * lda >= (1ll << 31) ||
      (long long)N * ldb >= (1ll << 31))
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
  const dim3 g((unsigned)((M / BM) * (N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_ring4_kernel<true, DI, AB>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace ring
}  // namespace ntm
