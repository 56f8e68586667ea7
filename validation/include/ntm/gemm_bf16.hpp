// K1: bf16 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x32_bf16).
//
//   C[M x N] (bf16) = A[M x K] (bf16, row-major) * B[N x K]^T (bf16, row-major)
//   fp32 accumulation, round-to-nearest-even on the way out.
//
// This is the validation-Job workload that replaces the NVIDIA GPU Operator's
// CUDA validator (reference: helm_release.gpu_operator, /root/reference/eks/
// main.tf:185-203, gke/main.tf:195-213, aks/main.tf:89-91). Spec: SURVEY.md
// §2.7 K1. Design follows the CDNA4 playbook
// (/opt/skills/guides/cdna_hip_programming.md §5 "256^2 8-phase template"),
// re-derived here for a [N][K] B operand:
//
//  * 256x256 macro tile, BK = 64, 512 threads = 8 waves (2 M x 4 N). Each
//    wave owns 4 quadrants of 64x32 outputs; 128 fp32 accumulators / lane.
//  * Operands are staged HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA,
//    no VGPR round trip) into a 128 KiB double buffer cut into four 16 KiB
//    half-tiles (A-lo, A-hi, B-lo, B-hi). Every half-tile is an array of
//    16x32 bf16 subtiles (1 KiB = one MFMA fragment); inside a subtile the
//    16-byte chunk index is XOR-swizzled with row bit 3, which makes the
//    ds_read_b128 fragment read bank-conflict free. glds writes LDS lane-
//    linearly, so the swizzle is applied to the per-lane SOURCE address and
//    the same involution on the read (playbook §5.4 rule 21).
//  * One K-tile = 4 phases; each phase = {ds_read fragments, issue one
//    half-tile of LDS-DMA prefetch, counted vmcnt, s_barrier, 16 MFMAs,
//    s_barrier}. Loads run 4-6 phases ahead of their reader, the counted
//    s_waitcnt vmcnt(8) never drains the pipe inside the main loop, and the
//    two wave groups (wr = 0 / 1) are staggered by one barrier so that on
//    every SIMD one wave is in its MFMA segment while its partner reads LDS
//    and issues DMA (ping-pong).
//  * Bijective XCD-aware block remap + GROUP_M tile raster so that the 32
//    co-resident tiles of one XCD share A/B panels in that XCD's L2.
//
// LDS-ordering proof (barrier indices; group 1 lags group 0 by one barrier):
//  issue schedule  : phase 4t+0 B-hi(t+1), 4t+1 A-hi(t+1), 4t+2 A-lo(t+2),
//                    4t+3 B-lo(t+2)    (prologue: A-lo0 B-lo0 B-hi0 A-hi0
//                    A-lo1 B-lo1)
//  read schedule   : phase 4t+0 A-lo(t),B-lo(t); 4t+1 B-hi(t); 4t+2 A-hi(t)
//  RAW: a load issued in phase i is retired by vmcnt(8) in phase i+4 and may
//       be read in phase >= i+5 by either group; min issue->read distance is 5.
//  WAR: a half may be re-staged >= 2 phases after its last ds_read (reads are
//       retired by the MFMAs that consume them before the phase's 2nd
//       barrier); min distance in the schedule is 2 (A-lo).
#pragma once

#include "ntm/common.hpp"

namespace ntm {
namespace gemm {

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int kThreads = 512;
constexpr int kHalfBytes = 128 * BK * 2;    // 16 KiB: 128 rows x 64 k bf16
constexpr int kTileBytes = 4 * kHalfBytes;  // A-lo, A-hi, B-lo, B-hi
constexpr int kLdsBytes = 2 * kTileBytes;   // double buffer: 128 KiB
constexpr int kGroupM = 8;                  // tile-raster group height

enum : int { kALo = 0, kAHi = 1, kBLo = 2, kBHi = 3 };

struct GemmArgs {
  const __bf16* A;
  const __bf16* B;
  __bf16* C;
  int M, N, K;
  int lda, ldb, ldc;
  // optional ABFT checksum: rowsum[m] += sum_n of the fp32 accumulators of
  // row m (caller zeroes it). nullptr selects the plain kernel.
  float* rowsum = nullptr;
  // split-K (wave-specialised tiles only): workgroup (tile, blockIdx.y = s)
  // runs K range [s kc, (s+1) kc) and stores its fp32 partial to
  // splitk_ws[s][M][N]; splitk_reduce_kernel sums the slices into C.
  float* splitk_ws = nullptr;
  int splitk_kc = 0;
  // clock-stamp builds only (gemm_bf16_pp6.hpp STAMP): 4 u64 per workgroup
  unsigned long long* stamps = nullptr;
};

// Shapes the fast kernel accepts; the host launcher rejects anything else.
__host__ __device__ inline bool shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 2 * BK && (M % BM) == 0 && (N % BN) == 0 &&
         (K % BK) == 0;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= -1 && N <= 12, "vmcnt range");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

// Raw workgroup barrier. NOT __syncthreads(): that one carries a fence that
// makes hipcc emit s_waitcnt vmcnt(0), which would drain the LDS-DMA
// prefetch in flight (playbook §5 "Pipelining across barriers").
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void glds16(const __bf16* gsrc, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const void NTM_AS1*)gsrc,
                                   (void NTM_AS3*)lds_dst, 16, 0, 0);
}

struct Frags {
  bf16x8 a[4][2];   // [m-tile][k-step]   (64 rows of the current A half)
  bf16x8 bl[2][2];  // [n-tile][k-step]   (32 cols of B-lo)
  bf16x8 bh[2][2];  // [n-tile][k-step]   (32 cols of B-hi)
};

struct Ctx {
  char* lds;             // LDS base (one __shared__ array only)
  const __bf16* src[4];  // per-lane glds source for each half, K-tile 0
  int frag_off;          // per-lane byte offset of an MFMA fragment read
  int w, wr, wc;         // wave id, wave row (0..1), wave col (0..3)
  int K;                 // partial-K builds only (kEpiKTail): K, in elements
  int lane_col;          //   and this lane's 8-element source chunk offset
};

// Issue the two glds of this wave for half-tile H of K-tile kt into buffer.
template <int H>
__device__ __forceinline__ void issue_half(const Ctx& c, int kt, int buf) {
  const __bf16* s = c.src[H] + (size_t)kt * BK;
  char* d = c.lds + buf * kTileBytes + H * kHalfBytes + (2 * c.w) * 1024;
  glds16(s, d);
  glds16(s + 32, d + 1024);
}

template <int H>
__device__ __forceinline__ void read_a(const Ctx& c, bf16x8 (&a)[4][2], int buf) {
  const char* base = c.lds + buf * kTileBytes + H * kHalfBytes + c.frag_off;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      a[mt][ks] = *(const bf16x8*)(base + ((c.wr * 4 + mt) * 2 + ks) * 1024);
}

template <int H>
__device__ __forceinline__ void read_b(const Ctx& c, bf16x8 (&b)[2][2],
                                       int buf) {
  const char* base = c.lds + buf * kTileBytes + H * kHalfBytes + c.frag_off;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      b[nt][ks] = *(const bf16x8*)(base + ((c.wc * 2 + nt) * 2 + ks) * 1024);
}

// 16 MFMAs: one 64x32 quadrant over K = 64. Operand order is swapped (B
// fragment first) so each lane ends up holding 4 consecutive output columns
// of one row -> 8-byte stores in the epilogue.
template <bool PRIO = true>
__device__ __forceinline__ void mma_quadrant(f32x4 (&acc)[4][2],
                                             const bf16x8 (&a)[4][2],
                                             const bf16x8 (&b)[2][2]) {
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            b[nt][ks], a[mt][ks], acc[mt][nt], 0, 0, 0);
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
}

// fp8 (OCP e4m3) form of mma_quadrant for the same LDS image: the K-tile's
// 128 bytes per row are 128 fp8 values, and a lane's two bf16x8 fragment reads
// (ks = 0, 1: bytes 16c..16c+15 and 64+16c..64+16c+15 of its row, c = the
// lane's 16-B chunk) concatenate into one 32-byte operand of
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales). A dot product only
// needs A and B to use the same k order, which they do (same image, same
// reads; pinned by tools/experiments/fp8_layout_probe.py). 8 MFMAs of 32 cycles do twice
// the bf16 quadrant's work in the same 256 cycles.
typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ i32x8 cat_f8(const bf16x8& lo, const bf16x8& hi) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 x = __builtin_bit_cast(i32x4, lo), y = __builtin_bit_cast(i32x4, hi);
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

// The accumulators are pinned to AGPRs and updated in place by inline asm: with
// the builtin, hipcc (ROCm 7.2) writes each result to fresh VGPRs and the
// 8-register-aligned operand tuples push the kernel to 256 VGPRs + 13 spilled;
// the scratch reloads' vmcnt(0) then drained the LDS-DMA pipeline 4x per
// K-tile pair (2.06 PF vs hipBLASLt's 3.2 PF). hipcc pads nothing inside asm:
// operands come from ds_read (hipcc waits lgkmcnt on "v" inputs), the AGPR
// accumulators are never written by VALU inside the loop, and the kernel
// drains the MFMA pipe (mfma_drain) before any VALU reads them.
__device__ __forceinline__ void mfma_f8_agpr(f32x4& acc, const i32x8& a, const i32x8& b) {
  asm("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
      : "+a"(acc)
      : "v"(a), "v"(b), "v"(127));  // fmt e4m3 x e4m3 (cbsz = blgp = 0), E8M0 scale 2^0
}

// Experimental form (K1-fp8 knob 5): the plain f8f6f4 opcode without the
// v_mfma_ld_scale_b32 prefix (8 instead of 16 bytes; hardware default scales).
// (An SGPR scale operand does not assemble: the scales must be VGPRs.)
__device__ __forceinline__ void mfma_f8_agpr_plain(f32x4& acc, const i32x8& a, const i32x8& b) {
  asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int ORD>
__device__ __forceinline__ void mfma_f8_ord(f32x4& acc, const i32x8& a, const i32x8& b) {
  if constexpr (ORD == 3)
    mfma_f8_agpr_plain(acc, a, b);
  else
    mfma_f8_agpr(acc, a, b);
}

__device__ __forceinline__ void mfma_drain() {
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
}

// ORD 1: A-fragment outer (srcB held for 2 MFMAs); experimental: ORD 2 (knob 1)
// B-fragment outer (srcA held for 4 MFMAs); ORD 3 (knob 5) the plain MFMA form
// of mfma_f8_ord.
template <int ORD = 1>
__device__ __forceinline__ void mma_quadrant_f8(f32x4 (&acc)[4][2],
                                                const bf16x8 (&a)[4][2],
                                                const bf16x8 (&b)[2][2]) {
  if constexpr (ORD == 2) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        mfma_f8_agpr(acc[mt][nt], cat_f8(b[nt][0], b[nt][1]), cat_f8(a[mt][0], a[mt][1]));
  } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        mfma_f8_ord<ORD>(acc[mt][nt], cat_f8(b[nt][0], b[nt][1]), cat_f8(a[mt][0], a[mt][1]));
  }
}

// One phase of the K loop. P: phase within the K-tile (0..3); ISSUE: whether
// the prefetch item of this phase exists; VMC: counted vmcnt (-1 = none).
template <int P, bool ISSUE, int VMC>
__device__ __forceinline__ void phase(const Ctx& c, Frags& f,
                                      f32x4 (&acc)[2][2][4][2], int t) {
  const int cur = t & 1, nxt = cur ^ 1;
  // 1. fragment reads for this phase
  if constexpr (P == 0) {
    read_b<kBLo>(c, f.bl, cur);
    read_a<kALo>(c, f.a, cur);
  } else if constexpr (P == 1) {
    read_b<kBHi>(c, f.bh, cur);
  } else if constexpr (P == 2) {
    read_a<kAHi>(c, f.a, cur);
  }
  // 2. LDS-DMA prefetch of one half-tile
  if constexpr (ISSUE) {
    if constexpr (P == 0) issue_half<kBHi>(c, t + 1, nxt);
    if constexpr (P == 1) issue_half<kAHi>(c, t + 1, nxt);
    if constexpr (P == 2) issue_half<kALo>(c, t + 2, cur);
    if constexpr (P == 3) issue_half<kBLo>(c, t + 2, cur);
  }
  // 3. retire the loads the NEXT phase reads (never vmcnt(0) in steady state)
  wait_vmcnt<VMC>();
  raw_barrier();
  // 4. matrix work for one quadrant
  if constexpr (P == 0) mma_quadrant(acc[0][0], f.a, f.bl);
  if constexpr (P == 1) mma_quadrant(acc[0][1], f.a, f.bh);
  if constexpr (P == 2) mma_quadrant(acc[1][1], f.a, f.bh);
  if constexpr (P == 3) mma_quadrant(acc[1][0], f.a, f.bl);
  raw_barrier();
}

// Block -> output tile. Bijective XCD remap (nwg % 8 != 0 safe), then a
// GROUP_M raster inside each XCD's contiguous chunk. `bid` is the virtual
// block id (blockIdx.x, or a persistent kernel's tile index) out of `nwg`.
template <int GROUP_M = kGroupM>
__device__ __forceinline__ void tile_coords_of(int bid, int nwg, int M, int N,
                                               int& tm, int& tn) {
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wgid =
      (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;  // ceil: masked edge tiles
  const int group = GROUP_M * tiles_n;
  const int gid = wgid / group;
  const int first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - gid * group;
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

template <int GROUP_M = kGroupM>
__device__ __forceinline__ void tile_coords(int M, int N, int& tm, int& tn) {
  tile_coords_of<GROUP_M>((int)blockIdx.x, (int)gridDim.x, M, N, tm, tn);
}

// Fused ABFT row checksum: the 4 lanes {l, l+16, l+32, l+48} share row
// (l & 15); reduce their 16 accumulators each with two xor-shuffles, one
// fp32 atomic per (row, wave). 4 column-waves x N/256 tiles add per row.
__device__ __forceinline__ void abft_rowsum(const GemmArgs& p, const Ctx& c,
                                            const f32x4 (&acc)[2][2][4][2],
                                            int m0, int lane) {
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      float s = 0.f;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const f32x4 v = acc[mh][nh][mt][nt];
          s += (v[0] + v[1]) + (v[2] + v[3]);
        }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if (lane < 16)
        unsafeAtomicAdd(p.rowsum + m0 + mh * 128 + c.wr * 64 + mt * 16 + lane, s);
    }
}

// Epilogue shared by the K1 kernels: bf16 RNE stores (8 B per lane per
// 16x16 tile) and, with kRowSum, the fused ABFT row checksum.
template <bool kRowSum>
__device__ __forceinline__ void store_tile(const GemmArgs& p, const Ctx& c,
                                           const f32x4 (&acc)[2][2][4][2],
                                           int m0, int n0, int lane) {
  // Epilogue: lane holds C[row][col .. col+3] per 16x16 tile.
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int row = m0 + mh * 128 + c.wr * 64 + mt * 16 + (lane & 15);
          const int col = n0 + nh * 128 + c.wc * 32 + nt * 16 + (lane >> 4) * 4;
          const f32x4 v = acc[mh][nh][mt][nt];
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 o;
          o[0] = (__bf16)v[0];
          o[1] = (__bf16)v[1];
          o[2] = (__bf16)v[2];
          o[3] = (__bf16)v[3];
          *(bf16x4*)(p.C + (size_t)row * p.ldc + col) = o;
        }
  if constexpr (kRowSum) abft_rowsum(p, c, acc, m0, lane);
}

// Widened epilogue (playbook T21, adapted to the 16x16 layout): a lane holds
// 4 columns of tile nt = 0 and the same 4 columns + 16 of tile nt = 1. One
// v_permlane16_swap per dword pair exchanges lanes 16-31 (48-63) of the nt = 0
// register with lanes 0-15 (32-47) of the nt = 1 register, after which every
// lane holds 8 consecutive columns: lane group g = lane >> 4 stores 16 B at
// column offset (g & 1) * 16 + (g >> 1) * 8 of the 32-column pair. 16
// dwordx4 stores per wave instead of 32 dwordx2, same bytes.
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 q = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, q);
}

template <bool kRowSum, bool NT = false>
__device__ __forceinline__ void store_tile_wide(const GemmArgs& p, const Ctx& c,
                                                const f32x4 (&acc)[2][2][4][2],
                                                int m0, int n0, int lane) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int g = lane >> 4;
  const int coff = (g & 1) * 16 + (g >> 1) * 8;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int row = m0 + mh * 128 + c.wr * 64 + mt * 16 + (lane & 15);
        const int col = n0 + nh * 128 + c.wc * 32 + coff;
        const f32x4 v0 = acc[mh][nh][mt][0], v1 = acc[mh][nh][mt][1];
        unsigned w0[2], w1[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto r = __builtin_amdgcn_permlane16_swap(
              pack_bf16x2(v0[2 * h], v0[2 * h + 1]),
              pack_bf16x2(v1[2 * h], v1[2 * h + 1]), false, false);
          w0[h] = r[0];
          w1[h] = r[1];
        }
        u32x4* dst = (u32x4*)(p.C + (size_t)row * p.ldc + col);
        const u32x4 val = u32x4{w0[0], w0[1], w1[0], w1[1]};
        if constexpr (NT)
          __builtin_nontemporal_store(val, dst);
        else
          *dst = val;
      }
  if constexpr (kRowSum) abft_rowsum(p, c, acc, m0, lane);
}

// LDS-staged epilogue: the whole 256x256 bf16 tile goes through LDS (row
// pitch 528 B, so the 8-lane groups of a ds_write_b128 hit distinct banks)
// and leaves as full 512-B rows, 2 rows per wave instruction. Needs 135 KiB of
// LDS and a caller that has drained its LDS-DMA (vmcnt(0)); the barrier here
// orders every wave's last fragment read and DMA before the overwrite.
constexpr int kStagePitch = 528;

// 16-byte C store: POL 0 plain, 1 nontemporal. (Write-through sc1 / nt sc1 /
// sc0 sc1 forms in asm were measured in round 3 and lost 0-3.5 % at 8192^3:
// profiles/r3_k1o/sc1_epilogue.log.)
template <int POL>
__device__ __forceinline__ void store_c16(void* dst, const unsigned __attribute__((ext_vector_type(4))) & v) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  static_assert(POL == 0 || POL == 1, "store policy");
  if constexpr (POL == 0) *(u32x4*)dst = v;
  if constexpr (POL == 1) __builtin_nontemporal_store(v, (u32x4*)dst);
}

template <bool kRowSum, bool NT, bool MASK = false, int POL = NT ? 1 : 0>
__device__ __forceinline__ void store_tile_lds(const GemmArgs& p, const Ctx& c,
                                               const f32x4 (&acc)[2][2][4][2],
                                               int m0, int n0, int lane) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  raw_barrier();
  const int g = lane >> 4;
  const int coff = (g & 1) * 16 + (g >> 1) * 8;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int row = mh * 128 + c.wr * 64 + mt * 16 + (lane & 15);
        const int col = nh * 128 + c.wc * 32 + coff;
        const f32x4 v0 = acc[mh][nh][mt][0], v1 = acc[mh][nh][mt][1];
        unsigned w0[2], w1[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto r = __builtin_amdgcn_permlane16_swap(
              pack_bf16x2(v0[2 * h], v0[2 * h + 1]),
              pack_bf16x2(v1[2 * h], v1[2 * h + 1]), false, false);
          w0[h] = r[0];
          w1[h] = r[1];
        }
        *(u32x4*)(c.lds + row * kStagePitch + col * 2) = u32x4{w0[0], w0[1], w1[0], w1[1]};
      }
  raw_barrier();
  // wave w stores rows 32w .. 32w+31; lane -> (row pair half, 16-B chunk)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = c.w * 32 + i * 2 + (lane >> 5);
    const int chunk = lane & 31;
    const u32x4 val = *(const u32x4*)(c.lds + row * kStagePitch + chunk * 16);
    u32x4* dst = (u32x4*)(p.C + (size_t)(m0 + row) * p.ldc + n0 + chunk * 8);
    if constexpr (MASK) {  // edge tile: rows >= M / 8-column chunks >= N stay unwritten
      if (m0 + row >= p.M || n0 + chunk * 8 >= p.N) continue;
    }
    store_c16<POL>(dst, val);
  }
  if constexpr (kRowSum) abft_rowsum(p, c, acc, m0, lane);
}

// Epilogue selector for the kernels' EPI template bit mask.
// kEpiMask: ragged C (M, N not multiples of 256; N % 8): the LDS-staged stores
// skip rows / column chunks past C (the kernel clamps its loads).
// kEpiKTail (with kEpiMask): K % 128 != 0 - chunks past K load zeros (a build
// flag that rides on the EPI mask, like kEpiMask it changes the loads too).
enum : int { kEpiWide = 1, kEpiNT = 2, kEpiEarly = 4, kEpiLds = 8, kEpiMask = 16, kEpiKTail = 32,
             kEpiSkip = 64 };  // kEpiSkip: ablation (experimental library only), C not stored

__device__ __attribute__((aligned(16))) const unsigned kZeroChunk16[4] = {0u, 0u, 0u, 0u};

template <bool kRowSum, int EPI>
__device__ __forceinline__ void store_tile_epi(const GemmArgs& p, const Ctx& c,
                                               const f32x4 (&acc)[2][2][4][2],
                                               int m0, int n0, int lane) {
  if constexpr ((EPI & kEpiSkip) != 0) {
    // timing ablation: the store happens only for an impossible ldc, so the
    // accumulators (and every MFMA) stay live but no byte of C leaves
    if (p.ldc < 0)
      store_tile_lds<kRowSum, (EPI & kEpiNT) != 0, false>(p, c, acc, m0, n0, lane);
  } else if constexpr ((EPI & kEpiLds) != 0)
    store_tile_lds<kRowSum, (EPI & kEpiNT) != 0, (EPI & kEpiMask) != 0>(p, c, acc, m0, n0, lane);
  else if constexpr ((EPI & kEpiWide) != 0)
    store_tile_wide<kRowSum, (EPI & kEpiNT) != 0>(p, c, acc, m0, n0, lane);
  else
    store_tile<kRowSum>(p, c, acc, m0, n0, lane);
}

template <bool kRowSum>
__global__ void __launch_bounds__(kThreads, 2)
    gemm_bf16_256x256_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];

  int tm, tn;
  tile_coords(p.M, p.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  Ctx c;
  c.lds = smem;
  const int lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  // glds: lane -> (stored row, stored chunk) of the wave's subtile; source is
  // the logical chunk (inverse swizzle == swizzle, an involution).
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    const __bf16* a0 = p.A + (size_t)(m0 + c.w * 16 + r) * p.lda + cl * 8;
    const __bf16* b0 = p.B + (size_t)(n0 + c.w * 16 + r) * p.ldb + cl * 8;
    c.src[kALo] = a0;
    c.src[kAHi] = a0 + (size_t)128 * p.lda;
    c.src[kBLo] = b0;
    c.src[kBHi] = b0 + (size_t)128 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][j][m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  Frags f;
  const int T = p.K / BK;

  // Prologue: K-tile 0 complete + A-lo/B-lo of K-tile 1 (6 half-tiles).
  issue_half<kALo>(c, 0, 0);
  issue_half<kBLo>(c, 0, 0);
  issue_half<kBHi>(c, 0, 0);
  issue_half<kAHi>(c, 0, 0);
  issue_half<kALo>(c, 1, 1);
  issue_half<kBLo>(c, 1, 1);
  wait_vmcnt<8>();
  raw_barrier();
  // Ping-pong stagger: wave row 1 runs one barrier behind wave row 0.
  if (c.wr == 1) raw_barrier();

  int t = 0;
  for (; t < T - 2; ++t) {
    phase<0, true, 8>(c, f, acc, t);
    phase<1, true, 8>(c, f, acc, t);
    phase<2, true, 8>(c, f, acc, t);
    phase<3, true, 8>(c, f, acc, t);
  }
  // K-tile T-2: only K-tile T-1's hi halves remain to be loaded.
  phase<0, true, 8>(c, f, acc, t);
  phase<1, true, 8>(c, f, acc, t);
  phase<2, false, 6>(c, f, acc, t);
  phase<3, false, 4>(c, f, acc, t);
  ++t;
  // K-tile T-1: drain.
  phase<0, false, 2>(c, f, acc, t);
  phase<1, false, 0>(c, f, acc, t);
  phase<2, false, -1>(c, f, acc, t);
  phase<3, false, -1>(c, f, acc, t);
  // balance the stagger so both groups execute the same barrier count
  if (c.wr == 0) raw_barrier();

  store_tile<kRowSum>(p, c, acc, m0, n0, lane);
}

// Host launcher. Returns hipErrorInvalidValue for shapes the kernel does not
// tile (callers fall back to nothing: validation shapes are fixed).
inline hipError_t launch_gemm_bf16(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.M / BM) * (a.N / BN));
  if (a.rowsum)
    hipLaunchKernelGGL(gemm_bf16_256x256_kernel<true>, dim3(grid),
                       dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(gemm_bf16_256x256_kernel<false>, dim3(grid),
                       dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace ntm
