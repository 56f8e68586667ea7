// K1 v6 ("dma4"): bf16 GEMM with 4 waves, one per SIMD, each owning a
// 128x128 block of a 256x256 output tile (0.25 ds_read_b128 per MFMA, as
// gemm_bf16_r4.hpp), operands staged HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4) through a ring of half-K-tile slots.
//
//   C[M x N] (bf16) = A[M x K] (bf16) * B[N x K]^T (bf16), fp32 accumulate.
//
// Why not the register-staged kernel: its timing ablations
// (profiles/r3_k1/r4_ablation.log) put its MFMA + fragment-read core at 1.38x
// the 8-wave default's throughput, but the 16 ds_write_b128 per K-tile and
// wave alone cost 25 % (a store moves its data VGPRs through the CU's LDS
// write path) and the register staging 33 % in all. LDS-DMA writes LDS from
// the memory pipeline with no VGPR transfer and no LDS instruction - it is
// what hipBLASLt's 4-wave MT256x256x64 kernel does (16 VMEM and 32 LDS
// instructions per K-tile and wave: profiles/r2_k1/pmc_bf16_8192_vs_hipblaslt.json).
//
// Ring: S = D + 1 slots of one half-step (k = 32): A[256 x 32] then B[256 x 32]
// as 16x32 bf16 subtiles (1 KiB = one MFMA fragment), the XOR-swizzled
// lane-linear image of every K1 kernel (swizzle on the DMA source).
// Half-step h (64 MFMAs on fragment set F[h & 1]):
//   * the wave's 8 DMA pieces of half-step h+D into slot (h+D) % S, spread
//     over the MFMAs (past the end: the last half-step re-read into the same,
//     free slot, so every counted wait is exact and there is no tail code);
//   * after MFMA JB: s_waitcnt vmcnt(pieces younger than half-step h+1's) +
//     lgkmcnt(0), s_barrier (= barrier h);
//   * then the 16 fragment reads of half-step h+1 into F[(h+1) & 1].
// RAW: half-step h+1 landed for this wave before barrier h (counted vmcnt),
//      for every wave after it; it is read only after it.
// WAR: slot (h+D) % S last held half-step h+D-S = h-1, read in half-step h-2
//      after barrier h-2 and retired (lgkmcnt(0)) before barrier h-1, which
//      precedes every DMA of half-step h.
// Registers: F[(h+1) & 1] last fed MFMAs in half-step h-1.
// Drain: vmcnt(0) before the epilogue reuses LDS for the C tile.
// Shape rule: M, N % 256, K % 128, K >= 256, 16-byte aligned rows, operands
// < 2 GiB (32-bit buffer offsets).
#pragma once

#include "ntm/gemm_bf16_r4.hpp"

namespace ntm {
namespace gemmrd {

using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::raw_barrier;
using ::ntm::gemmr::Frags;
using ::ntm::gemmr::kStagePitch;
using ::ntm::gemmr::mfma;

constexpr int BM = 256, BN = 256;
constexpr int BKH = 32;                   // k per half-step
constexpr int kThreads = 256;
constexpr int kHalfOp = 256 * BKH * 2;    // 16 KiB: one operand of a half-step
constexpr int kSlot = 2 * kHalfOp;        // 32 KiB
constexpr int kGroupM = 8;

template <int D>
struct Cfg {
  static_assert(D == 3 || D == 4, "prefetch distance (half-steps)");
  static constexpr int S = D + 1;
  static constexpr int kLds = (S * kSlot > 256 * kStagePitch) ? S * kSlot : 256 * kStagePitch;
  static_assert(kLds <= 163840, "160 KiB of LDS");
};

struct Ctx {
  char* lds;
  __amdgpu_buffer_rsrc_t rsa, rsb;  // whole-operand descriptors (wave-uniform)
  int voff_a, voff_b;               // lane's source chunk in row block 4w, k = 0 (bytes)
  int rowblk_a, rowblk_b;           // 16 rows in bytes (SGPR soffset steps)
  int rd_a, rd_b;                   // lane's fragment offset + wave's first A / B subtile
};

// Piece i (0..7) of half-step hs into `slot`: i < 4 -> A row block 4w + i, else
// B row block 4w + i - 4. hs is clamped to the last half-step (dummy pieces).
// buffer_load_dwordx4 ... lds: one VGPR offset per operand, the row block and
// the k step in the SGPR soffset, the LDS destination in M0 - no per-piece
// VALU address math and no 64-bit address VGPRs (the global_load_lds form
// needed 16 of them per half-step pair and spilled).
// M0SHARE: the 4 pieces of an operand share one M0 (the LDS base of the
// wave's 4 subtiles) and step the LDS destination with the instruction offset
// field (it moves the global address too, so soffset takes it back out):
// one M0 write per 4 pieces instead of one per piece.
template <bool M0SHARE = false>
__device__ __forceinline__ void issue_piece(const Ctx& c, int hs, int H, int slot_off, int w,
                                            int i) {
  const int kb = (hs < H ? hs : H - 1) * (BKH * 2);
  const bool is_b = i >= 4;
  const int rbi = i & 3;
  const int row_soff = kb + rbi * (is_b ? c.rowblk_b : c.rowblk_a);
  if constexpr (M0SHARE) {
    char* dst = c.lds + slot_off + (is_b ? kHalfOp : 0) + (w * 4) * 1024;
    // rowblk >= 16 rows x 256 x 2 B > rbi * 1024: soffset stays positive
    const auto rs = is_b ? c.rsb : c.rsa;
    const int vo = is_b ? c.voff_b : c.voff_a, so = row_soff - rbi * 1024;
    NTM_AS3 void* d = (NTM_AS3 void*)dst;
    switch (rbi) {  // the offset operand must be a literal
      case 0: __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, d, 16, vo, so, 0, 0); break;
      case 1: __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, d, 16, vo, so, 1024, 0); break;
      case 2: __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, d, 16, vo, so, 2048, 0); break;
      default: __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, d, 16, vo, so, 3072, 0); break;
    }
  } else {
    char* dst = c.lds + slot_off + (is_b ? kHalfOp : 0) + (w * 4 + rbi) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(is_b ? c.rsb : c.rsa, (NTM_AS3 void*)dst, 16,
                                             is_b ? c.voff_b : c.voff_a, row_soff, 0, 0);
  }
}

// Fragment read r (0..15): a[0], b[0..7], a[1..7].
__device__ __forceinline__ void read_frag(const Ctx& c, Frags& f, int slot_off, int r) {
  const char* base = c.lds + slot_off;
  if (r == 0)
    f.a[0] = *(const bf16x8*)(base + c.rd_a);
  else if (r <= 8)
    f.b[r - 1] = *(const bf16x8*)(base + c.rd_b + (r - 1) * 1024);
  else
    f.a[r - 8] = *(const bf16x8*)(base + c.rd_a + (r - 8) * 1024);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// One half-step. fc: fragments consumed; fn: fragments read for hs+1.
// PB: DMA pieces issued before the barrier (the rest after it).
template <int D, int JB, int PB, bool M0S = false>
__device__ __forceinline__ void half_step(const Ctx& c, f32x4 (&acc)[8][8], const Frags& fc,
                                          Frags& fn, int hs, int H, int slot_next, int slot_dma,
                                          int w) {
  static_assert(PB >= 0 && PB <= 8 && JB >= PB && JB <= 56, "schedule");
  constexpr int NR = 64 - JB;
  constexpr int PA = 8 - PB;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    mfma(acc[j >> 3][j & 7], fc.b[j & 7], fc.a[j >> 3]);
    if (j < JB) {
      if (PB > 0 && (j * PB) / JB != ((j + 1) * PB) / JB)
        issue_piece<M0S>(c, hs + D, H, slot_dma, w, (j * PB) / JB);
    } else {
      const int x = j - JB;
      if (PA > 0 && (x * PA) / NR != ((x + 1) * PA) / NR)
        issue_piece<M0S>(c, hs + D, H, slot_dma, w, PB + (x * PA) / NR);
      if ((x * 16) / NR != ((x + 1) * 16) / NR) read_frag(c, fn, slot_next, (x * 16) / NR);
    }
    if (j == JB - 1) {
      // half-step hs+1 landed: younger = half-steps hs+2 .. hs+D-1 + PB pieces
      wait_vm<8 * (D - 2) + PB>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int D = 4, int JB = 8, int PB = 0, int GROUP_M = kGroupM, bool M0S = false>
__global__ void __launch_bounds__(kThreads, 1) gemm_bf16_r4d_kernel(GemmArgs p) {
  using C = Cfg<D>;
  __shared__ __attribute__((aligned(16))) char smem[C::kLds];
  int tm, tn;
  ::ntm::gemm::tile_coords<GROUP_M>(p.M, p.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  Ctx c;
  c.lds = smem;
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
    c.rd_a = fo + wr * 8 * 1024;
    c.rd_b = kHalfOp + fo + wc * 8 * 1024;
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int H = p.K / BKH;  // half-steps (even, >= 8)
  Frags f0, f1;
  // prologue: half-steps 0 .. D-1 in flight, 0 landed, its fragments read
#pragma unroll
  for (int s = 0; s < D; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) issue_piece(c, s, H, s * kSlot, w, i);
  wait_vm<8 * (D - 1)>();
  raw_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) read_frag(c, f0, 0, r);

  // two half-steps per iteration keep the fragment roles fixed; slots rotate
  // mod S at run time (wave-uniform: SGPR arithmetic + one VGPR add per read base)
  int sn = 1, sd = D;  // slot of half-step h+1, slot of h+D
  // (the last pair is peeled: with the loop exit feeding the epilogue directly,
  // hipcc's register allocator kept a scratch copy of 16 accumulators per
  // iteration)
  int hs = 0;
  do {
    half_step<D, JB, PB, M0S>(c, acc, f0, f1, hs, H, sn * kSlot, sd * kSlot, w);
    sn = sn + 1 == C::S ? 0 : sn + 1;
    sd = sd + 1 == C::S ? 0 : sd + 1;
    half_step<D, JB, PB, M0S>(c, acc, f1, f0, hs + 1, H, sn * kSlot, sd * kSlot, w);
    sn = sn + 1 == C::S ? 0 : sn + 1;
    sd = sd + 1 == C::S ? 0 : sd + 1;
    hs += 2;
  } while (hs < H - 2);
  half_step<D, JB, PB, M0S>(c, acc, f0, f1, hs, H, sn * kSlot, sd * kSlot, w);
  sn = sn + 1 == C::S ? 0 : sn + 1;
  sd = sd + 1 == C::S ? 0 : sd + 1;
  half_step<D, JB, PB, M0S>(c, acc, f1, f0, hs + 1, H, sn * kSlot, sd * kSlot, w);

  ::ntm::gemm::mfma_drain();
  wait_vm<0>();  // dummy pieces landed before LDS is reused
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  ::ntm::gemmr::Ctx e;
  e.lds = smem;
  ::ntm::gemmr::store_tile<true>(p, e, acc, m0, n0, w, wr, wc, lane);
}

inline bool args_ok(const GemmArgs& a) {
  return a.M > 0 && a.N > 0 && a.K >= 256 && (a.M % BM) == 0 && (a.N % BN) == 0 &&
         (a.K % 128) == 0 && a.lda >= a.K && a.ldb >= a.K && a.ldc >= a.N && (a.lda % 8) == 0 &&
         (a.ldb % 8) == 0 && (a.ldc % 8) == 0 && !a.rowsum &&
         (long long)a.M * a.lda * 2 < (1ll << 31) && (long long)a.N * a.ldb * 2 < (1ll << 31);
}

template <int D = 4, int JB = 8, int PB = 0, bool M0S = false>
inline hipError_t launch_gemm_bf16_r4d(const GemmArgs& a, hipStream_t stream) {
  if (!args_ok(a) || (M0S && (16 * a.lda * 2 < 4096 || 16 * a.ldb * 2 < 4096)))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_bf16_r4d_kernel<D, JB, PB, kGroupM, M0S>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemmrd
}  // namespace ntm
