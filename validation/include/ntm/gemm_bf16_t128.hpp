// K1 "tile128": bf16 GEMM with a 128x128 macro tile for the sizes where the
// 256x256 kernels cannot fill the chip.
//
//   C[M x N] (bf16) = A[M x K] (bf16) * B[N x K]^T (bf16), fp32 accumulate.
//
// Why: at 2048^3 a 256x256 tile gives 64 workgroups for 256 CUs, and K1 ran at
// 464 TF/s against hipBLASLt's 759 (profiles/r1_round9/small_sizes_check.log).
// 128x128 tiles give 256 workgroups there (one per CU).
//
// Structure (one workgroup per CU, one wave per SIMD):
//  * 4 waves as 2 (M) x 2 (N), each owning 64x64 outputs = 4 x 4 MFMA tiles of
//    16x16 (64 fp32 accumulators per lane), v_mfma_f32_16x16x32_bf16.
//  * LDS ring of S = 4 K-tile slots (BK = 64): a slot is A[128 x 64] then
//    B[128 x 64] as 16x32 subtiles (1 KiB = one MFMA fragment), the same
//    XOR-swizzled image as the 256x256 kernels (gemm_bf16.hpp), filled by
//    LDS-DMA (global_load_lds_dwordx4, swizzle applied to the source).
//  * K loop, iteration t (fragments of tile t already in registers):
//      issue tile t+3 (8 pieces per wave; past the end: dummy pieces that
//        re-read the last tile into a scratch region nobody reads, so the
//        counted wait below is exact in every iteration and there is no tail)
//      16 MFMAs (k-half 0 of tile t)
//      s_waitcnt vmcnt(16) + lgkmcnt(0), s_barrier   -> tile t+1 visible
//      16 MFMAs (k-half 1 of tile t) with the 16 fragment reads of tile t+1
//  RAW: the wait leaves only tiles t+2 and t+3 (16 pieces) in flight, so tile
//       t+1 has landed for this wave; the barrier makes it so for all waves
//       before anyone reads it.
//  WAR: tile t+3 goes into the slot of tile t-1, whose fragments every wave
//       read in iteration t-2 and retired (lgkmcnt(0)) before barrier t-1,
//       which the issuing wave has passed.
//  Drain: vmcnt(0) before the epilogue, so no DMA lands after the WG exits.
// Shape rule: M, N % 128, K % 128 (an even K-tile count); 16-byte aligned rows.
#pragma once

#include "ntm/gemm_bf16.hpp"

namespace ntm {
namespace gemmt {

using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::glds16;
using ::ntm::gemm::raw_barrier;

constexpr int TM = 128;
constexpr int TN = 128;
constexpr int TK = 64;
constexpr int kThreadsT = 256;
constexpr int kStages = 4;
constexpr int kOperandBytes = TM * TK * 2;         // 16 KiB: 8 row blocks x 2 k-halves
constexpr int kSlotBytesT = 2 * kOperandBytes;     // A + B
constexpr int kScratchT = kStages * kSlotBytesT;   // dummy-piece target (4 KiB)
constexpr int kLdsBytesT = kScratchT + 4 * 1024;   // 132 KiB
constexpr int kGroupMT = 8;

__host__ __device__ inline bool shape_ok_t(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 2 * TK && (M % TM) == 0 && (N % TN) == 0 &&
         (K % (2 * TK)) == 0;
}

__device__ __forceinline__ void wait_vmcnt16() {
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

struct CtxT {
  char* lds;
  const __bf16* a_src;  // this lane's source for A row block 2w, k-tile 0
  const __bf16* b_src;
  size_t a_rb16;        // 16 rows of A, in elements
  size_t b_rb16;
  int frag_off;
  int w, wr, wc;
};

struct FragsT {
  bf16x8 a[4][2];  // [m-tile][k-half]
  bf16x8 b[4][2];  // [n-tile][k-half]
};

// This wave's 8 LDS-DMA pieces of K-tile kt: A row blocks 2w, 2w+1 and B row
// blocks 2w, 2w+1, both k-halves each. kt >= T: dummy pieces (source = the
// last K-tile, in bounds; destination = this wave's 1 KiB of scratch).
__device__ __forceinline__ void issue_tile(const CtxT& c, int kt, int T) {
  const bool real = kt < T;
  const size_t koff = (size_t)(real ? kt : T - 1) * TK;
  char* slot = c.lds + (kt % kStages) * kSlotBytesT;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rb = 2 * c.w + i;
    const __bf16* sa = c.a_src + i * c.a_rb16 + koff;
    const __bf16* sb = c.b_src + i * c.b_rb16 + koff;
    char* da = real ? slot + (rb * 2) * 1024 : c.lds + kScratchT + c.w * 1024;
    char* db = real ? slot + kOperandBytes + (rb * 2) * 1024 : c.lds + kScratchT + c.w * 1024;
    glds16(sa, da);
    glds16(sa + 32, real ? da + 1024 : da);
    glds16(sb, db);
    glds16(sb + 32, real ? db + 1024 : db);
  }
}

__device__ __forceinline__ void read_frags(const CtxT& c, FragsT& f, int kt) {
  const char* slot = c.lds + (kt % kStages) * kSlotBytesT + c.frag_off;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f.a[t][ks] = *(const bf16x8*)(slot + ((c.wr * 4 + t) * 2 + ks) * 1024);
      f.b[t][ks] = *(const bf16x8*)(slot + kOperandBytes + ((c.wc * 4 + t) * 2 + ks) * 1024);
    }
}

// MFMA with the accumulator pinned to AGPRs (asm): with the builtin, hipcc
// shuttled the 64 accumulators through ~95 v_accvgpr_mov + ~96 read/write
// pairs per K-tile pair. No VALU touches them in the loop; mfma_drain()
// fences the epilogue's reads (asm MFMAs get no hazard padding from hipcc).
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// 16 MFMAs over one k-half; B fragment first so a lane holds 4 consecutive
// output columns of one row (the epilogue's 8-byte stores).
__device__ __forceinline__ void mma_half(f32x4 (&acc)[4][4], const FragsT& f, int ks) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) mfma_acc(acc[mt][nt], f.b[nt][ks], f.a[mt][ks]);
}

__device__ __forceinline__ void ktile(const CtxT& c, f32x4 (&acc)[4][4], const FragsT& cur,
                                      FragsT& nxt, int t, int T) {
  issue_tile(c, t + 3, T);
  mma_half(acc, cur, 0);
  __builtin_amdgcn_sched_barrier(0);
  wait_vmcnt16();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  read_frags(c, nxt, t + 1);  // t + 1 == T: a slot of stale data, never used
  mma_half(acc, cur, 1);
  __builtin_amdgcn_sched_barrier(0);
}

template <int GROUP_M = kGroupMT>
__device__ __forceinline__ void tile_coords_t(int M, int N, int& tm, int& tn) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_m = M / TM, tiles_n = N / TN;
  const int group = GROUP_M * tiles_n;
  const int gid = wgid / group;
  const int first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - gid * group;
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

__global__ void __launch_bounds__(kThreadsT, 1) gemm_bf16_t128_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytesT];
  int tm, tn;
  tile_coords_t(p.M, p.N, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int lane = threadIdx.x & 63;

  CtxT c;
  c.lds = smem;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 1;
  c.wc = c.w & 1;
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.a_src = p.A + (size_t)(m0 + 2 * c.w * 16 + r) * p.lda + cl * 8;
    c.b_src = p.B + (size_t)(n0 + 2 * c.w * 16 + r) * p.ldb + cl * 8;
    c.a_rb16 = (size_t)16 * p.lda;
    c.b_rb16 = (size_t)16 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / TK;
  FragsT f0, f1;
  issue_tile(c, 0, T);
  issue_tile(c, 1, T);
  issue_tile(c, 2, T);
  wait_vmcnt16();  // tile 0 landed (tiles 1, 2 may be in flight)
  raw_barrier();
  read_frags(c, f0, 0);

  // T is even (shape rule): one straight loop body keeps the register roles
  // fixed at the back edge (an odd-T tail path made the allocator permute the
  // accumulators with ~63 v_accvgpr_mov at the join).
  for (int t = 0; t < T; t += 2) {
    ktile(c, acc, f0, f1, t, T);
    ktile(c, acc, f1, f0, t + 1, T);
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy pieces drained
  ::ntm::gemm::mfma_drain();                           // MFMA results land before the reads
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int row = m0 + c.wr * 64 + mt * 16 + (lane & 15);
      const int col = n0 + c.wc * 64 + nt * 16 + (lane >> 4) * 4;
      const f32x4 v = acc[mt][nt];
      bf16x4 o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      *(bf16x4*)(p.C + (size_t)row * p.ldc + col) = o;
    }
}

inline hipError_t launch_gemm_bf16_t128(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok_t(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.M / TM) * (a.N / TN));
  hipLaunchKernelGGL(gemm_bf16_t128_kernel, dim3(grid), dim3(kThreadsT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemmt
}  // namespace ntm
