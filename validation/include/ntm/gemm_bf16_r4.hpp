// K1 v5 ("regstage4"): bf16 GEMM with 4 waves, one per SIMD, each owning a
// 128x128 block of a 256x256 output tile; operands staged HBM -> VGPR -> LDS.
//
//   C[M x N] (bf16) = A[M x K] (bf16) * B[N x K]^T (bf16), fp32 accumulate.
//
// Why (profiles/r2_k1/pmc_bf16_8192_vs_hipblaslt.json): the 8-wave
// ping-pong kernel (gemm_bf16_pp3.hpp) matches hipBLASLt's MFMA-busy cycles at
// 8192^3 but issues 1.52x the LDS instructions (0.375 ds_read_b128 per MFMA:
// each wave owns 128x64 outputs) and 1.42x the SALU, and the power-capped
// clock (1.668 vs 1.702 GHz) is the whole gap. A 128x128 block per wave needs
// 16 A + 16 B fragment reads per 128 MFMAs = 0.25 per MFMA, the ratio of
// hipBLASLt's MT256x256x64 (WG32_8_1 = 4 waves), and 256 fp32 accumulators per
// lane, so one wave per SIMD (512 registers: 256 AGPR accumulators + VGPRs).
//
// With one wave per SIMD nothing hides an LDS-DMA piece's issue cost (~60
// cycles among bare MFMAs, MI355X_MICROARCH.md constants table; it is why the
// 4-wave tile kernels lost to the wave-specialised ones, gemm_bf16_t128.hpp),
// so the operands are staged through registers instead: buffer_load_dwordx4
// (SGPR descriptor + one VGPR offset per operand: no per-load VALU address
// math, the K step is an SGPR soffset) and ds_write_b128 into the SAME
// lane-linear, XOR-swizzled LDS image the LDS-DMA kernels use (16x32 subtiles
// of 1 KiB, chunk ^= row bit 3), so fragment reads are conflict-free
// ds_read_b128 with immediate offsets.
//
// Per K-tile t (BK = 64; LDS = two 64 KiB buffers, tile t in buf t & 1;
// registers: F0 / F1 = the k-half 0 / 1 fragments, S = one staged K-tile):
//   phase 0: 64 MFMAs (k-half 0 of t, F0) with the 16 F1 reads of t, the
//            first 8 ds_writes of tile t+1 (S -> buf (t+1) & 1), each followed
//            by the buffer_load of the same piece of tile t+2 into its S slot
//   phase 1: 64 MFMAs (k-half 1 of t, F1) with the last 8 write/load pairs;
//            after MFMA JB: s_waitcnt lgkmcnt(0), s_barrier (= barrier t),
//            then the 16 F0 reads of tile t+1 among the remaining MFMAs
//   RAW: every wave's writes of tile t+1 retire (lgkmcnt(0)) before barrier t;
//        tile t+1 is read only after it.
//   WAR: tile t+1 overwrites tile t-1, whose last reads (F1, phase 0 of t-1)
//        each wave retired before barrier t-1; the writes start after it.
//   Registers: an F register is re-read >= 8 MFMAs after its last MFMA
//        (sources are read at issue); an S slot is reloaded right after the
//        ds_write that consumed it (hipcc orders the VGPR WAR and counts vmcnt:
//        there is no LDS-DMA in flight to confuse its waits).
// Shape rule: M, N % 256, K % 128 (even K-tile count), 16-byte aligned rows,
// every operand < 2 GiB (32-bit buffer offsets).
#pragma once

#include "ntm/gemm_bf16.hpp"

namespace ntm {
namespace gemmr {

using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::raw_barrier;

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int kThreads = 256;
constexpr int kOpBytes = 256 * BK * 2;     // 32 KiB: one operand of a K-tile
constexpr int kBufBytes = 2 * kOpBytes;    // A then B: 64 KiB
constexpr int kStagePitch = 528;           // epilogue staging row pitch (bytes)
constexpr int kLds = 256 * kStagePitch;    // 132 KiB: 2 buffers, then the C tile
static_assert(kLds >= 2 * kBufBytes, "LDS holds two K-tile buffers");
constexpr int kGroupM = 8;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// K >= 256: the two-tile loop body runs at least once, so the tail is reached
// by ONE path (a second path - the loop skipped - made the register allocator
// permute accumulators with v_accvgpr_mov at the join, right before asm
// MFMAs that read them as srcC: an unpadded hazard, wrong results).
__host__ __device__ inline bool shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 4 * BK && (M % BM) == 0 && (N % BN) == 0 &&
         (K % (2 * BK)) == 0;
}

// Diagnostic builds (timing ablations, results wrong): DIAG 1 = no
// buffer_loads in the loop (the ds_writes store stale S), 2 = neither loads
// nor ds_writes, 3 = no fragment reads (MFMAs on stale fragments).
enum : int { kDiagNone = 0, kDiagNoLoad = 1, kDiagNoStage = 2, kDiagNoRead = 3 };

struct Ctx {
  __amdgpu_buffer_rsrc_t rsa, rsb;  // whole-operand descriptors (wave-uniform)
  int voff_a, voff_b;               // lane's chunk in row block 4w, K-tile 0 (bytes)
  int rowblk_a, rowblk_b;           // 16 rows of A / B in bytes
  char* lds;
  int wbase;                        // lane * 16 + wave's first subtile (bytes)
  int rd_a, rd_b;                   // lane's fragment offset + wave's A / B rows
};

struct Frags {
  bf16x8 a[8];  // [m-tile] of one k-half
  bf16x8 b[8];  // [n-tile]
};

// Piece i (0..15) of this wave for K-tile kt: i < 8 -> A, else B; row block
// 4w + ((i >> 1) & 3), k-half i & 1 (the two halves of a row's 128-B line are
// fetched by adjacent instructions).
__device__ __forceinline__ u32x4 load_piece(const Ctx& c, int kt, int i) {
  const bool is_b = i >= 8;
  const int rbi = (i >> 1) & 3, ks = i & 1;
  const int soff = kt * (BK * 2) + rbi * (is_b ? c.rowblk_b : c.rowblk_a);
  return __builtin_amdgcn_raw_buffer_load_b128(is_b ? c.rsb : c.rsa,
                                               (is_b ? c.voff_b : c.voff_a) + ks * 64, soff, 0);
}

template <int BUF>
__device__ __forceinline__ void write_piece(const Ctx& c, const u32x4& v, int i) {
  const bool is_b = i >= 8;
  const int rbi = (i >> 1) & 3, ks = i & 1;
  *(u32x4*)(c.lds + BUF * kBufBytes + (is_b ? kOpBytes : 0) + c.wbase + (rbi * 2 + ks) * 1024) = v;
}

// Fragment read r (0..15) of k-half KS: a[0], b[0..7], a[1..7] - the order the
// next phase's first MFMA row consumes them.
template <int BUF, int KS>
__device__ __forceinline__ void read_frag(const Ctx& c, Frags& f, int r) {
  const char* base = c.lds + BUF * kBufBytes + KS * 1024;
  if (r == 0)
    f.a[0] = *(const bf16x8*)(base + c.rd_a);
  else if (r <= 8)
    f.b[r - 1] = *(const bf16x8*)(base + c.rd_b + (r - 1) * 2048);
  else
    f.a[r - 8] = *(const bf16x8*)(base + c.rd_a + (r - 8) * 2048);
}

__device__ __forceinline__ void mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// One K-tile t held in buffer BUF. WRITES: stage tile t+1 (in S) into the other
// buffer; LOADS: refill S with tile t+2; NEXT: barrier t + F0 reads of tile t+1.
// JB: the phase-1 MFMA after which the barrier sits.
template <int BUF, bool WRITES_, bool LOADS_, bool NEXT, int JB, int DIAG = 0>
__device__ __forceinline__ void ktile(const Ctx& c, f32x4 (&acc)[8][8], Frags& f0, Frags& f1,
                                      u32x4 (&s)[16], int t) {
  static_assert(JB >= 32 && JB <= 56, "barrier after the write/load pairs, reads after it");
  constexpr bool WRITES = WRITES_ && DIAG != kDiagNoStage;
  constexpr bool LOADS = LOADS_ && DIAG != kDiagNoStage && DIAG != kDiagNoLoad;
  constexpr bool READS = DIAG != kDiagNoRead;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    mfma(acc[j >> 3][j & 7], f0.b[j & 7], f0.a[j >> 3]);
    if (READS && (j & 3) == 0) read_frag<BUF, 1>(c, f1, j >> 2);
    if constexpr (WRITES) {
      if ((j & 7) == 2) write_piece<BUF ^ 1>(c, s[j >> 3], j >> 3);
    }
    if constexpr (LOADS) {
      if ((j & 7) == 6) s[j >> 3] = load_piece(c, t + 2, j >> 3);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  constexpr int NR = 64 - JB;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    mfma(acc[j >> 3][j & 7], f1.b[j & 7], f1.a[j >> 3]);
    if (j < 32) {
      if constexpr (WRITES) {
        if ((j & 3) == 1) write_piece<BUF ^ 1>(c, s[8 + (j >> 2)], 8 + (j >> 2));
      }
      if constexpr (LOADS) {
        if ((j & 3) == 3) s[8 + (j >> 2)] = load_piece(c, t + 2, 8 + (j >> 2));
      }
    }
    if constexpr (NEXT) {
      if (j == JB - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
      }
      if (READS && j >= JB && ((j - JB) * 16) / NR != ((j - JB + 1) * 16) / NR)
        read_frag<BUF ^ 1, 0>(c, f0, ((j - JB) * 16) / NR);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// LDS-staged epilogue: the 256x256 bf16 tile goes through LDS (pitch 528 B:
// conflict-free ds_write_b128) and leaves as full 512-B rows, nontemporal.
template <bool NT>
__device__ __forceinline__ void store_tile(const GemmArgs& p, const Ctx& c, const f32x4 (&acc)[8][8],
                                          int m0, int n0, int w, int wr, int wc, int lane) {
  using ::ntm::gemm::pack_bf16x2;
  const int g = lane >> 4;
  const int coff = (g & 1) * 16 + (g >> 1) * 8;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = wr * 128 + mt * 16 + (lane & 15);
      const int col = wc * 128 + q * 32 + coff;
      const f32x4 v0 = acc[mt][2 * q], v1 = acc[mt][2 * q + 1];
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
    }
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int row = w * 64 + i * 2 + (lane >> 5);
    const int chunk = lane & 31;
    const u32x4 val = *(const u32x4*)(c.lds + row * kStagePitch + chunk * 16);
    u32x4* dst = (u32x4*)(p.C + (size_t)(m0 + row) * p.ldc + n0 + chunk * 8);
    if constexpr (NT)
      __builtin_nontemporal_store(val, dst);
    else
      *dst = val;
  }
}

template <int JB = 40, int GROUP_M = kGroupM, int DIAG = 0>
__global__ void __launch_bounds__(kThreads, 1) gemm_bf16_r4_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
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
    const int r = lane >> 2;                          // row in the 16-row block
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);  // swizzled source chunk
    c.voff_a = ((m0 + w * 64 + r) * p.lda + cl * 8) * 2;
    c.voff_b = ((n0 + w * 64 + r) * p.ldb + cl * 8) * 2;
    c.rowblk_a = 16 * p.lda * 2;
    c.rowblk_b = 16 * p.ldb * 2;
  }
  c.wbase = lane * 16 + w * 8 * 1024;
  {
    const int fo = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
    c.rd_a = fo + wr * 8 * 2048;
    c.rd_b = kOpBytes + fo + wc * 8 * 2048;
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / BK;
  Frags f0, f1;
  u32x4 s[16];
  // prologue: tile 0 -> buf 0, tile 1 -> S, F0 of tile 0
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = load_piece(c, 0, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) write_piece<0>(c, s[i], i);
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = load_piece(c, 1, i);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) read_frag<0, 0>(c, f0, r);

  // T even, >= 4: one straight two-tile body keeps buffer and register roles
  // fixed; do-while so that the tail has a single predecessor (shape_ok)
  int t = 0;
  do {
    ktile<0, true, true, true, JB, DIAG>(c, acc, f0, f1, s, t);
    ktile<1, true, true, true, JB, DIAG>(c, acc, f0, f1, s, t + 1);
    t += 2;
  } while (t < T - 2);
  ktile<0, true, false, true, JB, DIAG>(c, acc, f0, f1, s, t);
  ktile<1, false, false, false, JB, DIAG>(c, acc, f0, f1, s, t + 1);

  ::ntm::gemm::mfma_drain();  // asm MFMAs: results land before the epilogue reads them
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();  // every wave's last fragment reads done before the C staging overwrites LDS
  store_tile<true>(p, c, acc, m0, n0, w, wr, wc, lane);
}

inline bool args_ok(const GemmArgs& a) {
  return shape_ok(a.M, a.N, a.K) && a.lda >= a.K && a.ldb >= a.K && a.ldc >= a.N &&
         (a.lda % 8) == 0 && (a.ldb % 8) == 0 && (a.ldc % 8) == 0 &&
         (long long)a.M * a.lda * 2 < (1ll << 31) && (long long)a.N * a.ldb * 2 < (1ll << 31) &&
         !a.rowsum;
}

template <int JB = 40, int DIAG = 0>
inline hipError_t launch_gemm_bf16_r4(const GemmArgs& a, hipStream_t stream) {
  if (!args_ok(a)) return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_bf16_r4_kernel<JB, kGroupM, DIAG>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemmr
}  // namespace ntm
