// K1 4-wave build ("dma4k"): bf16 / e4m3 GEMM with 4 waves, one per SIMD,
// each owning a 128x128 block of a 256x256 output tile; ONE barrier per K-tile
// and two K-tile LDS-DMA buffers (buffer_load_dwordx4 ... lds, SGPR
// descriptors: no per-piece address VALU).
//
//   C[M x N] (bf16) = A[M x K] * B[N x K]^T, fp32 accumulate; bf16 operands on
//   v_mfma_f32_16x16x32_bf16 (two per MFMA slot, k-half 0 then 1), e4m3 on
//   v_mfma_f32_16x16x128_f8f6f4 (one per slot, plain form: unit scales).
//
// Why: a 128x128 block per wave reads 0.25 ds_read_b128
// per bf16 MFMA (0.5 per f8f6f4 MFMA), hipBLASLt's MT256x256 ratio, against the
// 8-wave default's 0.375. Round 3 measured the family (profiles/r3_k1): a
// half-K-tile ring with a barrier every 64 MFMAs ran 1450-1480 TF/s at 8192^3,
// register staging 1497; this K-tile step reaches the 8-wave default's rate
// (bf16 1645-1672 vs 1636-1666, hipBLASLt 1649-1683; e4m3 3114-3201 vs
// 3048-3211, hipBLASLt 3105-3376). Its stamp build (gemm_r4k_stamp.hpp) is
// where the per-tile cycle budget in profiles/r3_k1/README.md comes from. The
// builds that lost were deleted (git history: gemm_bf16_r4.hpp,
// gemm_bf16_r4d.hpp, gemm_r4ring.hpp).
//
// K-tile = 128 bytes per row (64 bf16 / 128 e4m3): the LDS image of every K1
// kernel (16x32-bf16 subtiles of 1 KiB, chunk XOR row bit 3 on the DMA
// source); an f8f6f4 operand is the concatenation of a lane's two 16-byte
// fragment reads (ks = 0, 1), the layout gemm_bf16.hpp mma_quadrant_f8 pins.
// Step t (64 MFMA slots, rows mt = 0..7 of 8 (mt, nt) slots, buffer t & 1):
//   row 0; s_waitcnt vmcnt(0) + lgkmcnt(0); s_barrier (= barrier t);
//   rows 1..7 with the 16 DMA pieces of tile t+2 (into buffer t & 1; past the
//   end the last tile again, so the wait stays exact), one every DI slots, and
//   the fragment reads of tile t+1 (buffer (t+1) & 1): A[mt-1] once row mt-1
//   has issued, B[nt] after slot (7, nt), A[7] at the end (one fragment set:
//   an MFMA reads its sources at issue; 128 VGPRs + 256 AGPR accumulators).
// RAW: tile t+1's pieces (issued after barrier t-1) land (vmcnt(0)) before
//      barrier t; read after it.
// WAR: buffer t & 1 held tile t, read during step t-1 after barrier t-1 and
//      retired (lgkmcnt(0)) before barrier t; tile t+2's DMA follows barrier t.
// Epilogue: vmcnt(0) (the dummy pieces) + barrier, then the 256x256 bf16 tile
// is staged through LDS (pitch 528 B) and leaves as full 512-B rows,
// nontemporal.
// Shape rule: M, N % 256; an even K-tile count >= 4 (bf16 K % 128, K >= 256;
// e4m3 K % 256, K >= 512); 16-byte aligned rows; operands < 2 GiB (32-bit
// buffer offsets); no ABFT row sums.
#pragma once

#include "ntm/gemm_bf16.hpp"
#include "ntm/gemm_fp8.hpp"

namespace ntm {
namespace w4k {

using ::ntm::gemm::cat_f8;
using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::raw_barrier;

constexpr int BM = 256, BN = 256;
constexpr int kThreads = 256;
constexpr int kOp = 256 * 128;              // 32 KiB: one operand of a K-tile
constexpr int kBuf = 2 * kOp;               // 64 KiB
constexpr int kStagePitch = 528;            // epilogue staging row pitch (bytes)
constexpr int kLds = 256 * kStagePitch;     // 132 KiB: 2 buffers, then the C tile
static_assert(kLds >= 2 * kBuf, "two K-tile buffers");
constexpr int kGroupM = 8;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Ctx {
  char* lds;
  __amdgpu_buffer_rsrc_t rsa, rsb;
  int voff_a, voff_b;      // lane's source chunk, row block 4w, K-tile 0 (bytes)
  int rowblk_a, rowblk_b;  // 16 rows in bytes
  int rd_a, rd_b;          // lane's fragment offset + wave's first A / B subtile
};

struct Frags8 {
  bf16x8 a[8][2];  // [m-tile][ks]: 16-byte halves of the K-tile row segment
  bf16x8 b[8][2];
};

// Piece i (0..15) of K-tile kt: i < 8 -> A, else B; row block 4w + ((i >> 1) & 3),
// half i & 1 (adjacent instructions fetch the two halves of a 128-byte line:
// fetching them a K-tile apart cost 5-6 %, profiles/r3_k1/ring4*.log).
__device__ __forceinline__ void issue_piece(const Ctx& c, int kt, int T, int buf, int w, int i) {
  const int kb = (kt < T ? kt : T - 1) * 128;
  const bool is_b = i >= 8;
  const int rbi = (i >> 1) & 3, ks = i & 1;
  char* dst = c.lds + buf * kBuf + (is_b ? kOp : 0) + ((w * 4 + rbi) * 2 + ks) * 1024;
  // (the instruction offset field would move the LDS destination too: the
  // k-half step rides in soffset)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(is_b ? c.rsb : c.rsa, (NTM_AS3 void*)dst, 16,
                                           is_b ? c.voff_b : c.voff_a,
                                           kb + ks * 64 + rbi * (is_b ? c.rowblk_b : c.rowblk_a),
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

__device__ __forceinline__ void mfma_bf16(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// One MFMA slot: e4m3 -> one 32-cycle f8f6f4 MFMA over the K-tile's 128 values;
// bf16 -> two 16-cycle 16x16x32 MFMAs, k-half 0 then 1 (per accumulator the
// K order of the 8-wave default, so results are bitwise equal to it).
template <bool F8>
__device__ __forceinline__ void mma(f32x4& acc, const Frags8& f, int mt, int nt) {
  if constexpr (F8) {
    ::ntm::gemm::mfma_f8_agpr_plain(acc, cat_f8(f.b[nt][0], f.b[nt][1]),
                                    cat_f8(f.a[mt][0], f.a[mt][1]));
  } else {
    mfma_bf16(acc, f.b[nt][0], f.a[mt][0]);
    mfma_bf16(acc, f.b[nt][1], f.a[mt][1]);
  }
}

// One K-tile step on buffer BUF (fragments of tile t in f on entry, of t+1 on
// exit). DI: one DMA piece every DI slots from the barrier on.
template <int BUF, int DI, bool F8>
__device__ __forceinline__ void step(const Ctx& c, f32x4 (&acc)[8][8], Frags8& f, int t, int T,
                                     int w) {
  static_assert(DI >= 1 && 15 * DI <= 55, "16 pieces within rows 1..7");
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
      if ((j % DI) == 0 && j / DI < 16) issue_piece(c, t + 2, T, BUF, w, j / DI);
      if (nt == 1) read_a(c, f, BUF ^ 1, mt - 1);  // A[mt-1]: its last MFMA was row mt-1
      if (mt == 7) read_b(c, f, BUF ^ 1, nt);      // B[nt] after slot (7, nt)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  read_a(c, f, BUF ^ 1, 7);
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-staged epilogue (the caller drained its DMA and passed a barrier).
template <bool NT>
__device__ __forceinline__ void store_tile(const GemmArgs& p, char* lds, const f32x4 (&acc)[8][8],
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
      *(u32x4*)(lds + row * kStagePitch + col * 2) = u32x4{w0[0], w0[1], w1[0], w1[1]};
    }
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int row = w * 64 + i * 2 + (lane >> 5);
    const int chunk = lane & 31;
    const u32x4 val = *(const u32x4*)(lds + row * kStagePitch + chunk * 16);
    u32x4* dst = (u32x4*)(p.C + (size_t)(m0 + row) * p.ldc + n0 + chunk * 8);
    if constexpr (NT)
      __builtin_nontemporal_store(val, dst);
    else
      *dst = val;
  }
}

// Kernel prologue shared with the stamp build: tile coordinates, descriptors,
// lane offsets. GemmArgs carries e4m3 operands as bf16-sized pairs (K, lda,
// ldb in pairs), so the byte geometry is the same for both dtypes.
__device__ __forceinline__ void setup(const GemmArgs& p, char* smem, Ctx& c, int& m0, int& n0,
                                      int& lane, int& w, int& wr, int& wc) {
  int tm, tn;
  ::ntm::gemm::tile_coords<kGroupM>(p.M, p.N, tm, tn);
  m0 = tm * BM;
  n0 = tn * BN;
  lane = threadIdx.x & 63;
  w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  wr = w >> 1;
  wc = w & 1;
  c.lds = smem;
  c.rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 2, 0x00020000);
  c.rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.N * p.ldb * 2, 0x00020000);
  const int r = lane >> 2;
  const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
  c.voff_a = ((m0 + w * 64 + r) * p.lda + cl * 8) * 2;
  c.voff_b = ((n0 + w * 64 + r) * p.ldb + cl * 8) * 2;
  c.rowblk_a = 16 * p.lda * 2;
  c.rowblk_b = 16 * p.ldb * 2;
  const int fo = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;
  c.rd_a = fo + wr * 8 * 2048;
  c.rd_b = kOp + fo + wc * 8 * 2048;
}

// Tiles 0 and 1 in flight, tile 0 landed and read into f.
__device__ __forceinline__ void prologue(const Ctx& c, Frags8& f, int T, int w) {
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
}

template <int DI, bool F8>
__global__ void __launch_bounds__(kThreads, 1) gemm_w4k_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  Ctx c;
  int m0, n0, lane, w, wr, wc;
  setup(p, smem, c, m0, n0, lane, w, wr, wc);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / 64;  // K-tiles of 128 bytes per row; even, >= 4
  Frags8 f;
  prologue(c, f, T, w);
  // two steps per iteration keep the buffer roles compile-time; do-while and a
  // peeled last pair: a second path into the tail made the register allocator
  // permute accumulators right before asm MFMAs (an unpadded hazard), and a
  // loop exit straight into the epilogue made it keep scratch copies
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
  store_tile<true>(p, smem, acc, m0, n0, w, wr, wc, lane);
}

inline bool operands_ok(const GemmArgs& a) {
  return (long long)a.M * a.lda * 2 < (1ll << 31) && (long long)a.N * a.ldb * 2 < (1ll << 31);
}

// bf16: M, N % 256, K % 128, K >= 256.
template <int DI = 3>
inline hipError_t launch_gemm_bf16_w4k(const GemmArgs& a, hipStream_t stream) {
  if (a.M <= 0 || a.N <= 0 || a.K < 256 || (a.M % BM) || (a.N % BN) || (a.K % 128) ||
      a.lda < a.K || a.ldb < a.K || a.ldc < a.N || (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) ||
      a.rowsum || !operands_ok(a))
    return hipErrorInvalidValue;
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_w4k_kernel<DI, false>), g, b, 0, stream, a);
  return hipGetLastError();
}

// e4m3: K, lda, ldb in fp8 elements (the launcher halves them, like
// launch_gemm_fp8); M, N % 256, K % 256, K >= 512.
template <int DI = 2>
inline hipError_t launch_gemm_fp8_w4k(const void* A, const void* B, __bf16* C, int M, int N, int K,
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
  if (!operands_ok(a)) return hipErrorInvalidValue;
  const dim3 g((unsigned)((M / BM) * (N / BN))), b(kThreads);
  hipLaunchKernelGGL((gemm_w4k_kernel<DI, true>), g, b, 0, stream, a);
  return hipGetLastError();
}

}  // namespace w4k
}  // namespace ntm
