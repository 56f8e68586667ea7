// K1 (v2): bf16 GEMM, one wave per SIMD, 128x128 outputs per wave.
//
//   C[M x N] (bf16) = A[M x K] (bf16) * B[N x K]^T (bf16), fp32 accumulate.
//
// Why a second structure: a rocprofv3 PMC comparison of the 8-wave ping-pong
// kernel (gemm_bf16.hpp) against hipBLASLt's MT256x256x64 kernel on the same
// operands (profiles/r1_pmc_v1_vs_hipblaslt/summary.json) showed identical
// MFMA counts but 12x more wave-cycles parked on s_waitcnt/s_barrier
// (SQ_WAIT_ANY) and 77% vs 88% MFMA-busy: with two waves per SIMD each wave
// spends half its life waiting for its partner. Here each SIMD runs ONE wave
// that owns a 128x128 output block (256 fp32 accumulators, pinned to AGPRs),
// so operand reuse per LDS byte doubles and there is one barrier per 64 MFMAs.
//
// Pipeline (k-step = 32 deep; LDS ring of D+1 slots x 32 KiB; D = 3 or 4):
//   * slot holds A[256 x 32] + B[256 x 32] as 16x32 bf16 subtiles (1 KiB = one
//     MFMA fragment); chunk index XOR row bit 3 -> conflict-free ds_read_b128
//     (swizzle on the glds SOURCE address, playbook rule 21).
//   * k-step j: 64 MFMAs on fragment set j (registers); after the first 16
//     MFMAs a counted s_waitcnt vmcnt + s_barrier publishes k-step j+1, whose
//     16 fragments are then read (rows 2-5) into the other register set.
//   * LDS-DMA in PAIRS: even k-steps issue k-steps j+D and j+D+1 back to back
//     (rows 2-7), odd k-steps issue nothing. A 128-B line of a row holds 64 B
//     of each of two consecutive k-steps; fetching both halves by adjacent
//     instructions lets the CU's L1 merge them into one L2 request. Fetched a
//     k-step apart (first version), every line crossed L2->L1 twice
//     (TCP_TCC_READ_REQ 2x hipBLASLt's: profiles/r1_pmc2_w4/summary.json).
//   RAW: k-step x lands (own vmcnt) and is published (barrier) inside k-step
//        x-1, before any wave reads it there.
//   WAR: k-step j+D overwrites the slot of k-step j-1 (read in k-step j-2);
//        j+D+1 overwrites the slot of k-step j (read in k-step j-1, after its
//        barrier) - so the pair is issued only after k-step j's barrier.
//   vmcnt: see younger_pieces() - the pieces issued after the last piece of
//        k-step j+1, which may stay in flight.
#pragma once

#include "ntm/common.hpp"

namespace ntm {
namespace gemm4 {

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BKS = 32;                    // k-step depth
constexpr int kThreads = 256;              // 4 waves, 2 (M) x 2 (N)
constexpr int kHalf = 256 * BKS * 2;       // 16 KiB: one operand of one k-step
constexpr int kSlotBytes = 2 * kHalf;      // A + B
constexpr int kGroupM = 8;
constexpr int kWaitRow = 1;                // wait + barrier after MFMA row 1

struct Args {
  const __bf16* A;
  const __bf16* B;
  __bf16* C;
  int M, N, K;
  int lda, ldb, ldc;
};

// Minimum K: prologue + at least one steady-state pair + the fixed tail.
template <int D>
__host__ __device__ constexpr int min_ksteps() {
  return D + 5;  // k-steps 0,1 peeled + >= 1 loop pair + 4-step tail
}

// Pieces (8 per k-step and wave) issued after the last piece of k-step j+1,
// at the wait point of k-step j, with R = KS - j k-steps remaining (KS even).
// Even k-step e issues k-steps e+D, e+D+1 after its wait; k-steps 0..D-1 are
// issued by the prologue. Evaluated with a proxy KS (only R and parity matter).
__host__ __device__ constexpr int younger_pieces(int D, int R) {
  const int KS = 1 << 20, j = KS - R;
  int cnt = 0;
  for (int y = j + 2; y <= KS - 1; ++y) {
    const int e = ((y - D) % 2 == 0) ? y - D : y - D - 1;  // even issuer
    if (y < D || e < j) cnt += 8;
  }
  return cnt;
}

template <int D>
__host__ __device__ inline bool shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && (M % BM) == 0 && (N % BN) == 0 &&
         (K % (2 * BKS)) == 0 && K / BKS >= min_ksteps<D>();
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void glds16(const __bf16* gsrc, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const void NTM_AS1*)gsrc,
                                   (void NTM_AS3*)lds_dst, 16, 0, 0);
}

struct Ctx {
  char* lds;
  const __bf16* a_src;  // this lane's glds source, row block 4w, k-step 0
  const __bf16* b_src;
  int a_rb_stride;      // 16 rows of A, in elements
  int b_rb_stride;
  int frag_off;
  int w, wr, wc;
};

typedef bf16x8 Frag8[8];

// MFMA with the accumulator pinned to AGPRs. With 256 live fp32 accumulators
// + 128 fragment VGPRs, hipcc's register allocator (ROCm 7.2) otherwise
// shuttles accumulators between the AGPR and VGPR files every iteration and
// spills (measured: 420 VGPR spills, 1656 v_accvgpr moves in the K loop).
// Hazards (hipcc pads nothing inside asm, playbook §5.7): sources come from
// ds_read (waited by hipcc's lgkmcnt on the "v" operands); accumulators are
// never written by VALU (k-step 0 uses srcC = 0), and the epilogue's
// v_accvgpr_read is fenced by agpr_drain().
__device__ __forceinline__ void mfma_agpr(f32x4& acc, const bf16x8& a,
                                          const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma_agpr_init(f32x4& acc, const bf16x8& a,
                                               const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

// MFMA D -> VALU/v_accvgpr_read needs up to 18 wait states on gfx950.
__device__ __forceinline__ void agpr_drain() {
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
}

template <int D>
__device__ __forceinline__ int slot_of(int j) {
  if constexpr (((D + 1) & D) == 0)
    return j & D;  // power-of-two ring
  else
    return j % (D + 1);
}

// LDS-DMA piece i (0..7) of k-step j: this wave's 4 A subtiles, then 4 B.
template <int D>
__device__ __forceinline__ void issue_glds(const Ctx& c, int j, int i) {
  char* slot = c.lds + slot_of<D>(j) * kSlotBytes;
  if (i < 4)
    glds16(c.a_src + (size_t)i * c.a_rb_stride + (size_t)j * BKS,
           slot + (c.w * 4 + i) * 1024);
  else
    glds16(c.b_src + (size_t)(i - 4) * c.b_rb_stride + (size_t)j * BKS,
           slot + kHalf + (c.w * 4 + (i - 4)) * 1024);
}

template <int D>
__device__ __forceinline__ void read_a(const Ctx& c, int j, int mt, bf16x8& a) {
  const char* p = c.lds + slot_of<D>(j) * kSlotBytes + c.frag_off;
  a = *(const bf16x8*)(p + (c.wr * 8 + mt) * 1024);
}

template <int D>
__device__ __forceinline__ void read_b(const Ctx& c, int j, int nt, bf16x8& b) {
  const char* p = c.lds + slot_of<D>(j) * kSlotBytes + kHalf + c.frag_off;
  b = *(const bf16x8*)(p + (c.wc * 8 + nt) * 1024);
}

// One k-step. ISSUE_A / ISSUE_B: DMA of k-steps j+D / j+D+1 (even k-steps
// only, after the barrier); WAITN: vmcnt before the mid-step barrier (-1:
// neither); READ: fragments of k-step j+1; INIT: srcC = 0. Program order is
// pinned with sched_barrier(0): left alone, hipcc hoists all reads + DMAs
// above the (asm, latency-opaque) MFMAs, and since lgkmcnt saturates at 15
// the first MFMA then waits for every new read.
template <int D, bool ISSUE_A, bool ISSUE_B, int WAITN, bool READ, bool INIT>
__device__ __forceinline__ void kstep(const Ctx& c, f32x4 (&acc)[8][8],
                                      const Frag8& ca, const Frag8& cb,
                                      Frag8& na, Frag8& nb, int j) {
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      // outer index = the B fragment = MFMA srcA, held for 8 MFMAs (srcA
      // reuse, as hipBLASLt's MT256x256x64 loop does); inner = A fragment
      if constexpr (INIT)
        mfma_agpr_init(acc[nt][mt], cb[mt], ca[nt]);
      else
        mfma_agpr(acc[nt][mt], cb[mt], ca[nt]);
      if (nt == 3 || nt == 7) {
        __builtin_amdgcn_sched_barrier(0);
        if (mt == kWaitRow && nt == 7) {
          if constexpr (WAITN >= 0) {
            // lgkmcnt(0): this wave's reads of k-step j's slot (issued in
            // k-step j-1; fragments for rows 2-7 not consumed yet) retire
            // before the barrier after which k-step j+D+1 overwrites it.
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            wait_vmcnt<WAITN>();
            raw_barrier();
          }
        }
        if constexpr (READ) {
          if (mt >= 2 && mt < 6) {  // 2 reads per half-row in rows 2..5
            const int r = (mt - 2) * 2 + (nt >> 2);  // 0..7
            read_a<D>(c, j + 1, r, na[r]);
            read_b<D>(c, j + 1, r, nb[r]);
          }
        }
        // 16 pieces over the 12 half-rows of rows 2..7: all 8 pieces of
        // k-step j+D, then all 8 of j+D+1 (their 64-B halves of the same
        // lines follow 8 instructions later, still merged in L1). The order is
        // what younger_pieces() counts: interleaving x/x+1 piece by piece
        // would leave only ONE piece younger than x's last - a RAW race.
        if (mt >= 2) {
          const int h = (mt - 2) * 2 + (nt >> 2);  // 0..11
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int piece = h * 2 + q;  // 0..23, use 0..15
            if (piece < 8) {
              if constexpr (ISSUE_A) issue_glds<D>(c, j + D, piece);
            } else if (piece < 16) {
              if constexpr (ISSUE_B) issue_glds<D>(c, j + D + 1, piece - 8);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// Tail k-step with R k-steps remaining (this one included), j = KS - R.
template <int D, int R>
__device__ __forceinline__ void tail_step(const Ctx& c, f32x4 (&acc)[8][8],
                                          const Frag8& ca, const Frag8& cb,
                                          Frag8& na, Frag8& nb, int j) {
  constexpr bool kEven = (R % 2) == 0;
  constexpr bool kIssueA = kEven && R > D;
  constexpr bool kIssueB = kEven && R > D + 1;
  constexpr int kWait = R >= 2 ? younger_pieces(D, R) : -1;
  kstep<D, kIssueA, kIssueB, kWait, (R >= 2), false>(c, acc, ca, cb, na, nb, j);
}

__device__ __forceinline__ void tile_coords(int M, int N, int& tm, int& tn) {
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wgid =
      (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int group = kGroupM * tiles_n;
  const int gid = wgid / group;
  const int first_m = gid * kGroupM;
  const int gsz = min(tiles_m - first_m, kGroupM);
  const int in_group = wgid - gid * group;
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

template <int D>
__global__ void __launch_bounds__(kThreads, 1) gemm_bf16_w4_kernel(Args p) {
  static_assert(D == 3 || D == 4, "prefetch distance");
  __shared__ __attribute__((aligned(16))) char smem[(D + 1) * kSlotBytes];

  int tm, tn;
  tile_coords(p.M, p.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;

  Ctx c;
  c.lds = smem;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 1;
  c.wc = c.w & 1;
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.a_src = p.A + (size_t)(m0 + c.w * 64 + r) * p.lda + cl * 8;
    c.b_src = p.B + (size_t)(n0 + c.w * 64 + r) * p.ldb + cl * 8;
    c.a_rb_stride = 16 * p.lda;
    c.b_rb_stride = 16 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;

  f32x4 acc[8][8];
  const int KS = p.K / BKS;
  Frag8 a0, b0, a1, b1;

  // prologue: k-steps 0 .. D-1 in flight; k-step 0 landed; its fragments read
#pragma unroll
  for (int s = 0; s < D; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) issue_glds<D>(c, s, i);
  wait_vmcnt<8 * (D - 1)>();
  raw_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    read_a<D>(c, 0, i, a0[i]);
    read_b<D>(c, 0, i, b0[i]);
  }

  // steady-state waits by parity (R large): even / odd k-step
  constexpr int kWaitEven = younger_pieces(D, 1 << 10);
  constexpr int kWaitOdd = younger_pieces(D, (1 << 10) - 1);
  // k-steps 0 (initialises the accumulators, srcC = 0) and 1
  kstep<D, true, true, kWaitEven, true, true>(c, acc, a0, b0, a1, b1, 0);
  kstep<D, false, false, kWaitOdd, true, false>(c, acc, a1, b1, a0, b0, 1);
  int j = 2;
  // steady state: the even k-step of each pair issues j+D and j+D+1 < KS
  do {
    kstep<D, true, true, kWaitEven, true, false>(c, acc, a0, b0, a1, b1, j);
    kstep<D, false, false, kWaitOdd, true, false>(c, acc, a1, b1, a0, b0, j + 1);
    j += 2;
  } while (j + D + 1 < KS);
  // Exactly 4 k-steps remain (KS even, loop exit at R <= D+1 even, D <= 4),
  // reached by ONE straight-line path. (Two control paths into the tail made
  // the register allocator permute accumulators with v_accvgpr_mov right
  // before the asm MFMAs: an unpadded AGPR-write -> srcC hazard.)
  tail_step<D, 4>(c, acc, a0, b0, a1, b1, j);
  tail_step<D, 3>(c, acc, a1, b1, a0, b0, j + 1);
  tail_step<D, 2>(c, acc, a0, b0, a1, b1, j + 2);
  tail_step<D, 1>(c, acc, a1, b1, a0, b0, j + 3);

  agpr_drain();
  // epilogue: lane holds C[row][col..col+3] of each 16x16 tile
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const int row_base = m0 + c.wr * 128 + (lane & 15);
  const int col_base = n0 + c.wc * 128 + (lane >> 4) * 4;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt)
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const f32x4 v = acc[mt][nt];
      bf16x4 o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      *(bf16x4*)(p.C + (size_t)(row_base + mt * 16) * p.ldc + col_base + nt * 16) = o;
    }
}

template <int D>
inline hipError_t launch(const Args& a, hipStream_t stream) {
  if (!shape_ok<D>(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.M / BM) * (a.N / BN));
  hipLaunchKernelGGL(gemm_bf16_w4_kernel<D>, dim3(grid), dim3(kThreads), 0,
                     stream, a);
  return hipGetLastError();
}

}  // namespace gemm4
}  // namespace ntm
