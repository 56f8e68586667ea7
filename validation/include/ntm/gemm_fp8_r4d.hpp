// K1-fp8 v2 ("dma4"): OCP e4m3 GEMM with 4 waves, one per SIMD, each owning a
// 128x128 block of a 256x256 output tile; operands staged HBM -> LDS by
// LDS-DMA (buffer_load_dwordx4 ... lds) into two K-tile buffers.
//
//   C[M x N] (bf16) = A[M x K] (e4m3) * B[N x K]^T (e4m3), fp32 accumulate,
//   v_mfma_f32_16x16x128_f8f6f4 (plain form: hardware-default unit scales).
//
// Why: the 8-wave fp8 build (gemm_bf16_pp3.hpp, F8) runs at 0.94-0.96 of
// hipBLASLt fp8 at 4096^3 / 8192^3. A 128x128 block per wave
// reads 0.5 ds_read_b128 per f8f6f4 MFMA instead of 0.75, and every f8f6f4
// MFMA is 32 cycles long, so one wave per SIMD has ~3x the bf16 16x16x32
// kernel's issue slack between MFMAs for the DMA pieces and reads (the bf16
// 4-wave kernels lose 33-35 % to their staging, gemm_bf16_r4*.hpp).
//
// K-tile = 128 e4m3 (the 128-byte LDS row of every K1 kernel: 16x32-bf16
// subtiles, XOR swizzle on the DMA source; an f8f6f4 operand is the
// concatenation of a lane's two 16-byte fragment reads, ks = 0 and 1, the
// layout gemm_bf16.hpp mma_quadrant_f8 pins).
// Step t (64 MFMAs, rows mt = 0..7 of 8 (mt, nt) MFMAs each, buffer t & 1):
//   row 0; s_waitcnt vmcnt(0) + lgkmcnt(0); s_barrier (= barrier t);
//   rows 1..7 with the 16 DMA pieces of tile t+2 (into buffer t & 1: past the
//   end the last tile again, so the wait stays exact) and the fragment reads
//   of tile t+1 (buffer (t+1) & 1): A[mt-1] once row mt-1 has issued, B[nt]
//   after MFMA (7, nt), A[7] at the end (one fragment set: an MFMA reads its
//   sources at issue, 128 VGPRs + 256 AGPR accumulators).
// RAW: tile t+1's pieces (issued after barrier t-1) land (vmcnt(0)) before
//      barrier t; read after it.
// WAR: buffer t & 1 held tile t, read during step t-1 after barrier t-1 and
//      retired (lgkmcnt(0)) before barrier t; tile t+2's DMA follows barrier t.
// Shape rule: M, N % 256, K % 256 (fp8 elements), K >= 512, 16-byte aligned
// rows, operands < 2 GiB.
#pragma once

#include "ntm/gemm_bf16_r4.hpp"
#include "ntm/gemm_fp8.hpp"

namespace ntm {
namespace fp8r {

using ::ntm::gemm::cat_f8;
using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::i32x8;
using ::ntm::gemm::raw_barrier;

constexpr int BM = 256, BN = 256;
constexpr int kThreads = 256;
constexpr int kOp = 256 * 128;            // 32 KiB: one operand of a K-tile
constexpr int kBuf = 2 * kOp;             // 64 KiB
constexpr int kLds = ::ntm::gemmr::kLds;  // 2 buffers, then the 132 KiB C staging
static_assert(kLds >= 2 * kBuf, "two K-tile buffers");
constexpr int kGroupM = 8;

struct Ctx {
  char* lds;
  __amdgpu_buffer_rsrc_t rsa, rsb;
  int voff_a, voff_b;      // lane's source chunk, row block 4w, K-tile 0 (bytes)
  int rowblk_a, rowblk_b;  // 16 rows in bytes
  int rd_a, rd_b;          // lane's fragment offset + wave's first A / B subtile
};

struct Frags8 {
  bf16x8 a[8][2];  // [m-tile][ks]: 16-byte halves of the 32-byte f8f6f4 operand
  bf16x8 b[8][2];
};

// Piece i (0..15) of K-tile kt: i < 8 -> A, else B; row block 4w + ((i >> 1) & 3),
// half i & 1 (adjacent instructions fetch the two halves of a 128-byte line).
// (A split-wait build - low k-halves first, two barriers per K-tile - ran
// 9-14 % slower at 8192^3: profiles/r3_k1/fp8_r4k.log; git history.)
__device__ __forceinline__ void issue_piece(const Ctx& c, int kt, int T, int buf, int w, int i) {
  const int kb = (kt < T ? kt : T - 1) * 128;
  const bool is_b = i >= 8;
  const int rbi = (i >> 1) & 3, ks = i & 1;
  char* dst = c.lds + buf * kBuf + (is_b ? kOp : 0) + ((w * 4 + rbi) * 2 + ks) * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(is_b ? c.rsb : c.rsa, (NTM_AS3 void*)dst, 16,
                                           (is_b ? c.voff_b : c.voff_a) + ks * 64,
                                           kb + rbi * (is_b ? c.rowblk_b : c.rowblk_a), 0, 0);
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

// One "MFMA slot" of the step: e4m3 -> one 32-cycle f8f6f4 MFMA over the
// K-tile's 128 values; bf16 (F8 = false, the same image holds 64 bf16 per row)
// -> two 16-cycle 16x16x32 MFMAs, k-half 0 then 1 (per accumulator the order
// of the 8-wave default, so results are bitwise equal to it).
template <bool F8 = true>
__device__ __forceinline__ void mma(f32x4& acc, const Frags8& f, int mt, int nt) {
  if constexpr (F8) {
    ::ntm::gemm::mfma_f8_agpr_plain(acc, cat_f8(f.b[nt][0], f.b[nt][1]),
                                    cat_f8(f.a[mt][0], f.a[mt][1]));
  } else {
    ::ntm::gemmr::mfma(acc, f.b[nt][0], f.a[mt][0]);
    ::ntm::gemmr::mfma(acc, f.b[nt][1], f.a[mt][1]);
  }
}

// One K-tile step on buffer BUF (fragments of tile t in f on entry, of t+1 on exit).
// DI: one DMA piece every DI MFMAs from the barrier on (the last piece's lead
// to the next barrier is (56 - 16 DI) + 8 MFMAs).
template <int BUF, int DI = 3, bool F8 = true>
__device__ __forceinline__ void step(const Ctx& c, f32x4 (&acc)[8][8], Frags8& f, int t, int T,
                                     int w) {
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    mma<F8>(acc[0][nt], f, 0, nt);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 landed (this wave's pieces)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();  // tile t+1 visible; every read of tile t retired
#pragma unroll
  for (int mt = 1; mt < 8; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      mma<F8>(acc[mt][nt], f, mt, nt);
      const int j = (mt - 1) * 8 + nt;  // 0..55
      // 16 DMA pieces of tile t+2, one every DI MFMA slots from the barrier
      if ((j % DI) == 0 && j / DI < 16) issue_piece(c, t + 2, T, BUF, w, j / DI);
      if (nt == 1) read_a(c, f, BUF ^ 1, mt - 1);  // A[mt-1]: its last MFMA was row mt-1
      if (mt == 7) read_b(c, f, BUF ^ 1, nt);      // B[nt] after MFMA (7, nt)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  read_a(c, f, BUF ^ 1, 7);
  __builtin_amdgcn_sched_barrier(0);
}

template <int GROUP_M = kGroupM, int DI = 3, bool F8 = true>
__global__ void __launch_bounds__(kThreads, 1) gemm_fp8_r4d_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  int tm, tn;
  ::ntm::gemm::tile_coords<GROUP_M>(p.M, p.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  Ctx c;
  c.lds = smem;
  // GemmArgs carries fp8 operands as bf16-sized pairs: K, lda, ldb in pairs
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
    c.rd_a = fo + wr * 8 * 2048;
    c.rd_b = kOp + fo + wc * 8 * 2048;
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / 64;  // K-tiles of 128 e4m3 (64 pairs); even, >= 4
  Frags8 f;
  // prologue: tiles 0 and 1 in flight, 0 landed and read
#pragma unroll
  for (int i = 0; i < 16; ++i) issue_piece(c, 0, T, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) issue_piece(c, 1, T, 1, w, i);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    read_a(c, f, 0, i);
    read_b(c, f, 0, i);
  }

  // two steps per iteration keep the buffer roles compile-time; the last pair
  // is peeled (a loop exit straight into the epilogue made hipcc spill, r4d)
  int t = 0;
  do {
    step<0, DI, F8>(c, acc, f, t, T, w);
    step<1, DI, F8>(c, acc, f, t + 1, T, w);
    t += 2;
  } while (t < T - 2);
  step<0, DI, F8>(c, acc, f, t, T, w);
  step<1, DI, F8>(c, acc, f, t + 1, T, w);

  ::ntm::gemm::mfma_drain();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy pieces landed before LDS reuse
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  ::ntm::gemmr::Ctx e;
  e.lds = smem;
  ::ntm::gemmr::store_tile<true>(p, e, acc, m0, n0, w, wr, wc, lane);
}

// K, lda, ldb in fp8 elements (the launcher halves them, like launch_gemm_fp8).
template <int DI = 3>
inline hipError_t launch_gemm_fp8_r4d(const void* A, const void* B, __bf16* C, int M, int N, int K,
                                      int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K < 512 || (M % BM) || (N % BN) || (K % 256) || lda < K || ldb < K ||
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
  hipLaunchKernelGGL((gemm_fp8_r4d_kernel<kGroupM, DI>), g, b, 0, stream, a);
  return hipGetLastError();
}

// The same K-tile step on bf16 operands ("dma4k": one barrier per 128 MFMAs,
// the DMA ring of gemm_bf16_r4d.hpp had one per 64). Shape rule: M, N % 256,
// K % 128, K >= 256.
template <int DI = 2>
inline hipError_t launch_gemm_bf16_r4k(const GemmArgs& a, hipStream_t stream) {
  if (a.M <= 0 || a.N <= 0 || a.K < 256 || (a.M % BM) || (a.N % BN) || (a.K % 128) ||
      a.lda < a.K || a.ldb < a.K || a.ldc < a.N || (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) ||
      a.rowsum || (long long)a.M * a.lda * 2 >= (1ll << 31) || (long long)a.N * a.ldb * 2 >= (1ll << 31))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_fp8_r4d_kernel<kGroupM, DI, false>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace fp8r
}  // namespace ntm
