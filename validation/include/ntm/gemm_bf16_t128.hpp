// K1 tile kernels: bf16 GEMM with (32 MT) x (32 NT) macro tiles for the sizes
// where the 256x256 kernels cannot fill the chip: "tile128" (MT = NT = 4,
// 128x128), "tile256x128" (8, 4), "tile160" (5, 5, 160x160) and
// "tile256x160" (8, 5); the wave-specialised kernel below also serves
// K1-fp8's small and mid tiles (F8 = true: its own consumer, same producers).
//
//   C[M x N] (bf16) = A[M x K] (bf16) * B[N x K]^T (bf16), fp32 accumulate.
//
// Why: at 2048^3 a 256x256 tile gives 64 workgroups for 256 CUs, and K1 ran at
// 464 TF/s against hipBLASLt's 759 (profiles/r1_round9/small_sizes_check.log).
// 128x128 tiles give 256 workgroups there (one per CU); 256x128 tiles fill the
// chip in one round from 2048 x 4096 up to 4096 x 4096 outputs.
//
// Structure (one workgroup per CU, one wave per SIMD):
//  * 4 waves as 2 (M) x 2 (N), each owning (16 MT) x (16 NT) outputs = MT x NT
//    MFMA tiles of 16x16 (4 MT NT fp32 accumulators per lane, AGPR-pinned),
//    v_mfma_f32_16x16x32_bf16.
//  * LDS ring of S K-tile slots (BK = 64; S = the most slots that fit the LDS
//    budget, at least 3): a slot is A[32 MT x 64] then B[32 NT x 64] as 16x32
//    subtiles (1 KiB = one MFMA fragment), the same XOR-swizzled image as the
//    256x256 kernels (gemm_bf16.hpp), filled by LDS-DMA
//    (global_load_lds_dwordx4, swizzle applied to the source). P = MT + NT
//    pieces per wave per K-tile (4 (MT + NT) per tile, split by global piece index).
//  * K loop, iteration t (fragments of tile t already in registers):
//      MT NT MFMAs (k-half 0 of tile t) with tile t+S-1's DMA pieces among
//        them (past the end: dummy pieces that re-read the last tile into a
//        scratch region nobody reads, so the counted wait below is exact in
//        every iteration and there is no tail)
//      s_waitcnt vmcnt((S-2) P) + lgkmcnt(0), s_barrier  -> tile t+1 visible
//      MT NT MFMAs (k-half 1 of tile t) with the fragment reads of tile t+1
//  RAW: the wait leaves only tiles t+2 .. t+S-1 ((S-2) P pieces) in flight, so
//       tile t+1 has landed for this wave; the barrier makes it so for all
//       waves before anyone reads it.
//  WAR: tile t+S-1 goes into the slot of tile t-1, whose fragments every wave
//       read in iteration t-2 and retired (lgkmcnt(0)) before barrier t-1,
//       which the issuing wave has passed.
//  Drain: vmcnt(0) before the epilogue, so no DMA lands after the WG exits.
// Shape rule: M % (32 MT), N % (32 NT), K % 128 (an even K-tile count);
// 16-byte aligned rows.
#pragma once

#include "ntm/gemm_bf16.hpp"

namespace ntm {
namespace gemmt {

using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::glds16;
using ::ntm::gemm::raw_barrier;

constexpr int TK = 64;
constexpr int kThreadsT = 256;
constexpr int kGroupMT = 8;

template <int MT, int NT = 4>
struct Cfg {
  static_assert(MT >= 4 && MT <= 8 && NT >= 4 && (NT <= 5 || (MT == 4 && NT == 8)),
                "tile shapes 128..256 x 128..160, and 128x256");
  static constexpr int TM = 32 * MT;
  static constexpr int TN = 32 * NT;
  static constexpr int kA = TM * TK * 2;             // A bytes of a slot
  static constexpr int kSlot = kA + TN * TK * 2;     // + B
  static constexpr int S = 4 * kSlot + 4096 <= 163840 ? 4 : 3;  // LDS ring depth (K-tiles)
  static constexpr int P = MT + NT;                  // pieces per wave per K-tile
  static constexpr int VMC = (S - 2) * P;            // counted wait
  static constexpr int kScratch = S * kSlot;         // dummy-piece target (4 KiB)
  static constexpr int kLds = kScratch + 4 * 1024;   // 132 / 148 / 124 / 160 KiB
  static_assert(kLds <= 163840, "160 KiB of LDS per CU");
  static_assert(VMC <= 63, "vmcnt is 6 bits");
};

template <int MT, int NT = 4>
__host__ __device__ inline bool shape_ok_t(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 2 * TK && (M % Cfg<MT, NT>::TM) == 0 &&
         (N % Cfg<MT, NT>::TN) == 0 && (K % (2 * TK)) == 0;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt_n() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct CtxT {
  char* lds;
  const __bf16* a_src;  // this lane's source in A row block 0 of the tile, k-tile 0
  const __bf16* b_src;
  size_t a_rb16;        // 16 rows of A, in elements
  size_t b_rb16;
  int frag_off;
  int w, wr, wc;
};

template <int MT, int NT = 4>
struct FragsT {
  bf16x8 a[MT][2];  // [m-tile][k-half]
  bf16x8 b[NT][2];  // [n-tile][k-half]
};

// LDS-DMA piece i (0 .. P-1) of this wave for K-tile kt. The tile's A has
// 4 MT pieces (2 MT row blocks of 16 rows x 2 k-halves), B has 4 NT; wave w
// stages A pieces g = w MT + i (i < MT) and B pieces g = w NT + (i - MT):
// row block g / 2, k-half g % 2 (for even MT / NT: row blocks w MT/2 .. and
// 2w, 2w+1 with both halves). kt >= T: a dummy piece (source = the last
// K-tile, in bounds; destination = this wave's 1 KiB of scratch).
template <int MT, int NT>
__device__ __forceinline__ void issue_piece(const CtxT& c, int kt, int T, int i) {
  using C = Cfg<MT, NT>;
  const bool real = kt < T;
  const bool is_a = i < MT;
  const int g = is_a ? c.w * MT + i : c.w * NT + (i - MT);
  const int rb = g >> 1, kh = g & 1;
  const size_t koff = (size_t)(real ? kt : T - 1) * TK + kh * 32;
  char* slot = c.lds + (kt % C::S) * C::kSlot;
  const __bf16* src = (is_a ? c.a_src + rb * c.a_rb16 : c.b_src + rb * c.b_rb16) + koff;
  char* dst = real ? slot + (is_a ? 0 : C::kA) + (rb * 2 + kh) * 1024
                   : c.lds + C::kScratch + c.w * 1024;
  glds16(src, dst);
}

// Fragment read r (0 .. 2 (MT + NT) - 1) of K-tile kt, k-half 0 first (that
// is what the next iteration's first MFMAs consume): per k-half MT A then NT B.
template <int MT, int NT>
__device__ __forceinline__ void read_frag(const CtxT& c, FragsT<MT, NT>& f, int kt, int r) {
  using C = Cfg<MT, NT>;
  const char* slot = c.lds + (kt % C::S) * C::kSlot + c.frag_off;
  const int ks = r / (MT + NT), i = r % (MT + NT);
  if (i < MT)
    f.a[i][ks] = *(const bf16x8*)(slot + ((c.wr * MT + i) * 2 + ks) * 1024);
  else
    f.b[i - MT][ks] = *(const bf16x8*)(slot + C::kA + ((c.wc * NT + (i - MT)) * 2 + ks) * 1024);
}

template <int MT, int NT>
__device__ __forceinline__ void read_frags(const CtxT& c, FragsT<MT, NT>& f, int kt) {
#pragma unroll
  for (int r = 0; r < 2 * (MT + NT); ++r) read_frag<MT, NT>(c, f, kt, r);
}

// MFMA with the accumulator pinned to AGPRs (asm): with the builtin, hipcc
// shuttled the accumulators through ~95 v_accvgpr_mov + ~96 read/write pairs
// per K-tile pair. No VALU touches them in the loop; mfma_drain() fences the
// epilogue's reads (asm MFMAs get no hazard padding from hipcc).
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// One K-tile. With one wave per SIMD nothing else hides an instruction that
// is not an MFMA, so the P DMA pieces are spread evenly over the first half's
// MT NT MFMAs and the 2 (MT + NT) fragment reads over the second half's (order
// pinned with sched_barrier; B fragment first in every MFMA so a lane holds 4
// consecutive output columns of one row for the epilogue's 8-byte stores).
template <int MT, int NT>
__device__ __forceinline__ void ktile(const CtxT& c, f32x4 (&acc)[MT][NT],
                                      const FragsT<MT, NT>& cur, FragsT<MT, NT>& nxt, int t,
                                      int T) {
  using C = Cfg<MT, NT>;
  constexpr int NM = NT * MT, P = C::P, NR = 2 * (MT + NT);
#pragma unroll
  for (int j = 0; j < NM; ++j) {
    mfma_acc(acc[j / NT][j % NT], cur.b[j % NT][0], cur.a[j / NT][0]);
    if ((j * P) / NM != ((j + 1) * P) / NM)
      issue_piece<MT, NT>(c, t + C::S - 1, T, (j * P) / NM);
    __builtin_amdgcn_sched_barrier(0);
  }
  wait_vmcnt_n<C::VMC>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int j = 0; j < NM; ++j) {
    mfma_acc(acc[j / NT][j % NT], cur.b[j % NT][1], cur.a[j / NT][1]);
    if ((j * NR) / NM != ((j + 1) * NR) / NM)
      read_frag<MT, NT>(c, nxt, t + 1, (j * NR) / NM);  // t + 1 == T: stale slot, unused
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int MT, int NT>
__device__ __forceinline__ void tile_coords_t(int M, int N, int& tm, int& tn) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // ceil: the wave-specialised kernel masks a partial last tile row / column
  const int tiles_m = (M + Cfg<MT, NT>::TM - 1) / Cfg<MT, NT>::TM;
  const int tiles_n = (N + Cfg<MT, NT>::TN - 1) / Cfg<MT, NT>::TN;
  const int group = kGroupMT * tiles_n;
  const int gid = wgid / group;
  const int first_m = gid * kGroupMT;
  const int gsz = min(tiles_m - first_m, kGroupMT);
  const int in_group = wgid - gid * group;
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

template <int MT, int NT = 4>
__global__ void __launch_bounds__(kThreadsT, 1) gemm_bf16_tile_kernel(GemmArgs p) {
  using C = Cfg<MT, NT>;
  __shared__ __attribute__((aligned(16))) char smem[C::kLds];
  int tm, tn;
  tile_coords_t<MT, NT>(p.M, p.N, tm, tn);
  const int m0 = tm * C::TM, n0 = tn * C::TN;
  const int lane = threadIdx.x & 63;

  CtxT c;
  c.lds = smem;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wr = c.w >> 1;
  c.wc = c.w & 1;
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.a_src = p.A + (size_t)(m0 + r) * p.lda + cl * 8;
    c.b_src = p.B + (size_t)(n0 + r) * p.ldb + cl * 8;
    c.a_rb16 = (size_t)16 * p.lda;
    c.b_rb16 = (size_t)16 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = p.K / TK;
  FragsT<MT, NT> f0, f1;
#pragma unroll
  for (int s = 0; s < C::S - 1; ++s)
#pragma unroll
    for (int i = 0; i < C::P; ++i) issue_piece<MT, NT>(c, s, T, i);
  wait_vmcnt_n<C::VMC>();  // tile 0 landed (tiles 1 .. S-2 may be in flight)
  raw_barrier();
  read_frags<MT, NT>(c, f0, 0);

  // T is even (shape rule): one straight loop body keeps the register roles
  // fixed at the back edge (an odd-T tail path made the allocator permute the
  // accumulators with ~63 v_accvgpr_mov at the join).
  for (int t = 0; t < T; t += 2) {
    ktile<MT, NT>(c, acc, f0, f1, t, T);
    ktile<MT, NT>(c, acc, f1, f0, t + 1, T);
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy pieces drained
  ::ntm::gemm::mfma_drain();                           // MFMA results land before the reads
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int row = m0 + c.wr * (16 * MT) + mt * 16 + (lane & 15);
      const int col = n0 + c.wc * (16 * NT) + nt * 16 + (lane >> 4) * 4;
      const f32x4 v = acc[mt][nt];
      bf16x4 o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      *(bf16x4*)(p.C + (size_t)row * p.ldc + col) = o;
    }
}

template <int MT, int NT = 4>
inline hipError_t launch_gemm_bf16_tile(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok_t<MT, NT>(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.M / Cfg<MT, NT>::TM) * (a.N / Cfg<MT, NT>::TN));
  hipLaunchKernelGGL((gemm_bf16_tile_kernel<MT, NT>), dim3(grid), dim3(kThreadsT), 0, stream, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Wave-specialised tile kernels ("tile128ws" / "tile256x128ws" / "tile160ws").
//
// Why: with one wave per SIMD the kernel above exposes the issue cost of every
// LDS-DMA piece (~60 cycles among bare MFMAs, MI355X_MICROARCH.md constants
// table) - at 256x128 that is 12 pieces against 64 16-cycle MFMAs per K-tile,
// about the 25-40 % gap to the 256x256 ping-pong kernel. Here a workgroup is
// 8 waves, two per SIMD: waves 0-3 ("consumers") own the same output blocks
// and issue ONLY ds_read_b128 + MFMA; waves 4-7 ("producers") issue ONLY the
// LDS-DMA pieces (the same pieces, the same LDS image), so a piece's issue
// cost lands on a wave that has nothing else to do while its SIMD partner
// keeps the matrix core busy.
//
// Registers: two waves per SIMD leave 256 per lane, so the consumers keep ONE
// fragment set (MT + NT) x 2 k-halves and refill each half as soon as its
// MFMAs are issued:
//   K-tile t, first half : MT NT MFMAs on k-half 0 of tile t; reads of
//                          k-half 1 of tile t (visible since barrier t).
//   lgkmcnt(0), barrier t+1
//   second half          : MT NT MFMAs on k-half 1 of tile t; reads of
//                          k-half 0 of tile t+1 (visible since barrier t+1).
// A k-half-0 register is refilled only after the barrier that follows its last
// MFMA; a k-half-1 register at least 5 MFMAs (>= 80 cycles) after its last
// MFMA (the previous iteration's second half), long after the MFMA read its
// sources at issue. Producers, per K-tile: issue tile t+S-1's P pieces
// (dummies into scratch past the end, as above), s_waitcnt vmcnt((S-2) P),
// barrier t+1. Both roles pass T+1 barriers.
//   RAW: a producer arrives at barrier t+1 only once its pieces of tile t+1
//        landed; consumers read tile t+1 only after that barrier.
//   WAR: tile t+S-1 overwrites the slot of tile t-1, whose last reads (k-half 1,
//        first half of iteration t-1) every consumer retired (lgkmcnt(0))
//        before barrier t, which the producer has passed.
//   Drain: producers vmcnt(0) before exit; MFMA order per accumulator is the
//        kernel above's, so results are bitwise equal to it.
// Same shape rule as the kernel above.
// Shape rule of the wave-specialised kernel: any M, N with N % 4 == 0 (8-byte
// C stores), any K with K % 8 == 0 (16-byte source chunks; a partial last
// K-tile reads zeros past K, see issue_piece_ws).
__host__ __device__ inline bool shape_ok_ws(int M, int N, int K) {
  return M > 0 && N > 0 && (N % 4) == 0 && K > 0 && (K % 8) == 0;
}

template <int MT, int NT>
struct CfgWS {
  static_assert(4 * MT * NT + 8 * (MT + NT) <= 232, "256 registers per lane at 2 waves / SIMD");
};

// Schedule knobs of the wave-specialised kernel (bitmask; 0 = as described):
//   kWsBFirst   read each k-half's B fragments before its A fragments: the
//               first MT NT / MT MFMAs need all NT B fragments but only A[0]
//   kWsEarly    issue the first half's reads within its first MT NT - 8 MFMAs,
//               so the lgkmcnt(0) before the barrier finds them landed
//   kWsPrio     consumers run at s_setprio 1 (MFMA issue wins over DMA issue)
//   kWsShallow  diagnostic: producers look one K-tile less ahead (S-2 tiles in
//               flight instead of S-1) - measures what prefetch depth is worth
constexpr int kWsBFirst = 1, kWsEarly = 2, kWsPrio = 4, kWsShallow = 8;

template <int MT, int NT, int KNOB>
__device__ __forceinline__ void read_half(const CtxT& c, FragsT<MT, NT>& f, int kt, int ks, int i) {
  const int r = (KNOB & kWsBFirst) ? (i < NT ? MT + i : i - NT) : i;
  read_frag<MT, NT>(c, f, kt, ks * (MT + NT) + r);
}

// Edge tiles (M or N not a multiple of the tile): a piece's source row is
// clamped to the last row of A / B, so every load stays in bounds; the rows
// and columns of C it feeds beyond M / N are computed but never stored.
// Partial last K-tile (K % 64 != 0): a lane whose 8-element chunk starts at
// k >= K takes its 16 bytes from a zero block instead, so the LDS image holds
// zeros past K in both operands - same instruction count, so every counted
// vmcnt stays exact, and no load leaves the row.
struct Clamp {
  const __bf16* A;
  const __bf16* B;
  int a_row, b_row;  // this lane's first row (tile origin + lane / 4)
  int a_last, b_last;
  int lda, ldb, col;  // col: this lane's swizzled 8-element column chunk
  int K;
};

__device__ __attribute__((aligned(16))) const unsigned kZeroChunk[4] = {0u, 0u, 0u, 0u};

template <int MT, int NT, bool CLAMP, bool TAIL>
__device__ __forceinline__ void issue_piece_ws(const CtxT& c, const Clamp& q, int kt, int T,
                                               int i) {
  using C = Cfg<MT, NT>;
  const bool real = kt < T;
  const bool is_a = i < MT;
  const int g = is_a ? c.w * MT + i : c.w * NT + (i - MT);
  const int rb = g >> 1, kh = g & 1;
  const int kcol = (real ? kt : T - 1) * TK + kh * 32;
  char* slot = c.lds + (kt % C::S) * C::kSlot;
  const __bf16* src;
  if constexpr (CLAMP)
    src = (is_a ? q.A + (size_t)min(q.a_row + rb * 16, q.a_last) * q.lda
                : q.B + (size_t)min(q.b_row + rb * 16, q.b_last) * q.ldb) + q.col + kcol;
  else
    src = (is_a ? c.a_src + rb * c.a_rb16 : c.b_src + rb * c.b_rb16) + kcol;
  if constexpr (TAIL) {
    if (kcol + q.col >= q.K) src = (const __bf16*)kZeroChunk;
  }
  char* dst = real ? slot + (is_a ? 0 : C::kA) + (rb * 2 + kh) * 1024
                   : c.lds + C::kScratch + c.w * 1024;
  glds16(src, dst);
}

// Producer loop of the wave-specialised kernel (see below).
template <int MT, int NT, int KNOB, bool CLAMP, bool TAIL>
__device__ __forceinline__ void ws_produce(const CtxT& c, const Clamp& q, int T) {
  using C = Cfg<MT, NT>;
  constexpr int LA = (KNOB & kWsShallow) ? C::S - 2 : C::S - 1;  // tiles issued ahead
  constexpr int VM = (LA - 1) * C::P;
  auto issue = [&](int kt, int i) { issue_piece_ws<MT, NT, CLAMP, TAIL>(c, q, kt, T, i); };
#pragma unroll
  for (int s = 0; s < LA; ++s)
#pragma unroll
    for (int i = 0; i < C::P; ++i) issue(s, i);
  wait_vmcnt_n<VM>();  // tile 0 landed
  raw_barrier();
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int i = 0; i < C::P; ++i) issue(t + LA, i);
    wait_vmcnt_n<VM>();  // tile t+1 landed
    raw_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy pieces drained
}

// fp8 consumer (K1-fp8 on the wave-specialised tiles, F8 = true). One
// v_mfma_f32_16x16x128_f8f6f4 per (mt, nt) and K-tile consumes BOTH k-halves of
// its A and B fragments (the LDS image is the bf16 one: a 128-byte K-tile row is
// 64 bf16 or 128 e4m3 values, gemm_fp8.hpp), so the bf16 consumer's half-tile
// ping-pong does not apply; instead each fragment of tile t+1 is read as soon
// as its last MFMA of tile t has issued (MFMAs read their A/B sources at issue):
//   row 0 of tile t (NT MFMAs); lgkmcnt(0); barrier t+1 (tile t+1 visible,
//   every read of tile t retired); rows 1 .. MT-1, with A[r] of tile t+1 read
//   after the first two MFMAs of row r+1, and in the last row B[nt] after MFMA
//   (MT-1, nt), A[MT-1] after the last one.
// Barriers and the RAW / WAR argument are the bf16 consumer's (T + 1 barriers,
// every read of tile t issued after barrier t and retired before barrier t+1),
// so the producer loop is unchanged. Next tile's row 0 needs B[nt] about NT
// 32-cycle MFMAs after its read was issued.
// Fragment i (A row block i < MT, else B column block i - MT) of K-tile kt,
// both k-halves: the 32-byte operand of one f8f6f4 MFMA.
template <int MT, int NT>
__device__ __forceinline__ void read_both_halves(const CtxT& c, FragsT<MT, NT>& f, int kt, int i) {
  read_frag<MT, NT>(c, f, kt, i);
  read_frag<MT, NT>(c, f, kt, MT + NT + i);
}

template <int MT, int NT>
__device__ __forceinline__ void ws_consume_f8(const CtxT& c, FragsT<MT, NT>& f,
                                              f32x4 (&acc)[MT][NT], int T) {
  using ::ntm::gemm::cat_f8;
  using ::ntm::gemm::mfma_f8_agpr_plain;
  auto mma = [&](int mt, int nt) {
    mfma_f8_agpr_plain(acc[mt][nt], cat_f8(f.b[nt][0], f.b[nt][1]), cat_f8(f.a[mt][0], f.a[mt][1]));
  };
  raw_barrier();  // tile 0 visible
#pragma unroll
  for (int i = 0; i < MT + NT; ++i) read_both_halves<MT, NT>(c, f, 0, i);
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      mma(0, nt);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();  // tile t+1 visible; every read of tile t retired
#pragma unroll
    for (int mt = 1; mt < MT; ++mt) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        mma(mt, nt);
        // A[mt-1] of tile t+1 (t + 1 == T: stale slot, unused): its last MFMA was row mt-1
        if (nt == 0) read_frag<MT, NT>(c, f, t + 1, mt - 1);
        if (nt == 1) read_frag<MT, NT>(c, f, t + 1, MT + NT + mt - 1);
        if (mt == MT - 1) read_both_halves<MT, NT>(c, f, t + 1, MT + nt);  // B[nt]
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    read_both_halves<MT, NT>(c, f, t + 1, MT - 1);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int MT, int NT = 4, int KNOB = 0, bool SPLIT = false, bool F8 = false>
__global__ void __launch_bounds__(2 * kThreadsT, 1) gemm_bf16_tile_ws_kernel(GemmArgs p) {
  using C = Cfg<MT, NT>;
  (void)sizeof(CfgWS<MT, NT>);
  __shared__ __attribute__((aligned(16))) char smem[C::kLds];
  int tm, tn;
  tile_coords_t<MT, NT>(p.M, p.N, tm, tn);
  const int m0 = tm * C::TM, n0 = tn * C::TN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // split-K: this workgroup's K slice [kb, kb + klen); else the whole K
  const int kb = SPLIT ? (int)blockIdx.y * p.splitk_kc : 0;
  const int klen = SPLIT ? min(p.splitk_kc, p.K - kb) : p.K;
  const int T = (klen + TK - 1) / TK;  // a partial last K-tile reads zeros past K

  CtxT c;
  c.lds = smem;
  c.w = wave & 3;  // producer: whose pieces; consumer: whose output block
  c.wr = c.w >> 1;
  c.wc = c.w & 1;
  {
    const int r = lane >> 2;
    const int cl = (lane & 3) ^ (((r >> 3) & 1) << 1);
    c.a_src = p.A + (size_t)(m0 + r) * p.lda + cl * 8 + kb;
    c.b_src = p.B + (size_t)(n0 + r) * p.ldb + cl * 8 + kb;
    c.a_rb16 = (size_t)16 * p.lda;
    c.b_rb16 = (size_t)16 * p.ldb;
  }
  c.frag_off = (lane & 15) * 64 + ((lane >> 4) ^ ((lane >> 2) & 2)) * 16;

  if (wave >= 4) {  // producer
    const int r = lane >> 2;
    const Clamp q{p.A + kb, p.B + kb, m0 + r, n0 + r, p.M - 1, p.N - 1, p.lda, p.ldb,
                  ((lane & 3) ^ (((r >> 3) & 1) << 1)) * 8, klen};
    const bool edge = m0 + C::TM > p.M || n0 + C::TN > p.N;  // uniform branches
    if (klen % TK) {
      if (edge)
        ws_produce<MT, NT, KNOB, true, true>(c, q, T);
      else
        ws_produce<MT, NT, KNOB, false, true>(c, q, T);
    } else if (edge) {
      ws_produce<MT, NT, KNOB, true, false>(c, q, T);
    } else {
      ws_produce<MT, NT, KNOB, false, false>(c, q, T);
    }
    return;
  }

  // consumer
  if constexpr (KNOB & kWsPrio) __builtin_amdgcn_s_setprio(1);
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  FragsT<MT, NT> f;
  if constexpr (F8) {
    static_assert(KNOB == 0, "fp8: default schedule only");
    ws_consume_f8<MT, NT>(c, f, acc, T);
  } else {
  raw_barrier();  // tile 0 visible
#pragma unroll
  for (int i = 0; i < MT + NT; ++i) read_half<MT, NT, KNOB>(c, f, 0, 0, i);

  constexpr int NM = MT * NT, NR = MT + NT;
  constexpr int NE = (KNOB & kWsEarly) && NM - 8 >= NR ? NM - 8 : NM;  // first-half read span
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int j = 0; j < NM; ++j) {
      mfma_acc(acc[j / NT][j % NT], f.b[j % NT][0], f.a[j / NT][0]);
      if (j < NE && (j * NR) / NE != ((j + 1) * NR) / NE)
        read_half<MT, NT, KNOB>(c, f, t, 1, (j * NR) / NE);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();  // tile t+1 visible; every read of tile t retired
#pragma unroll
    for (int j = 0; j < NM; ++j) {
      mfma_acc(acc[j / NT][j % NT], f.b[j % NT][1], f.a[j / NT][1]);
      if ((j * NR) / NM != ((j + 1) * NR) / NM)
        read_half<MT, NT, KNOB>(c, f, t + 1, 0, (j * NR) / NM);  // t + 1 == T: stale, unused
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  }  // bf16 consumer

  ::ntm::gemm::mfma_drain();
  if constexpr (SPLIT) {  // split-K: the fp32 partial of slice blockIdx.y
    float* w = p.splitk_ws + (size_t)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int row = m0 + c.wr * (16 * MT) + mt * 16 + (lane & 15);
        const int col = n0 + c.wc * (16 * NT) + nt * 16 + (lane >> 4) * 4;
        if (row < p.M && col < p.N) *(f32x4*)(w + (size_t)row * p.N + col) = acc[mt][nt];
      }
    return;
  }
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int row = m0 + c.wr * (16 * MT) + mt * 16 + (lane & 15);
      const int col = n0 + c.wc * (16 * NT) + nt * 16 + (lane >> 4) * 4;
      const f32x4 v = acc[mt][nt];
      bf16x4 o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      if (row < p.M && col < p.N)  // edge tiles: rows / columns past C are not stored
        *(bf16x4*)(p.C + (size_t)row * p.ldc + col) = o;
    }
}

// Split-K reduction: C = bf16(sum over S slices of ws[s][M][N]) (N % 4).
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* ws, __bf16* C, int M,
                                                            int N, int ldc, int S) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const size_t n4 = (size_t)M * N / 4, slice = (size_t)M * N;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 v = *(const f32x4*)(ws + i * 4);
    for (int s = 1; s < S; ++s) v += *(const f32x4*)(ws + s * slice + i * 4);
    const size_t e = i * 4;
    const int row = (int)(e / N), col = (int)(e % N);
    bf16x4 o;
    o[0] = (__bf16)v[0];
    o[1] = (__bf16)v[1];
    o[2] = (__bf16)v[2];
    o[3] = (__bf16)v[3];
    *(bf16x4*)(C + (size_t)row * ldc + col) = o;
  }
}

template <int MT, int NT = 4, int KNOB = 0>
inline hipError_t launch_gemm_bf16_tile_ws(const GemmArgs& a, hipStream_t stream) {
  if (!shape_ok_ws(a.M, a.N, a.K) || a.lda < a.K || a.ldb < a.K || a.ldc < a.N ||
      (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)(((a.M + Cfg<MT, NT>::TM - 1) / Cfg<MT, NT>::TM) *
                                   ((a.N + Cfg<MT, NT>::TN - 1) / Cfg<MT, NT>::TN));
  hipLaunchKernelGGL((gemm_bf16_tile_ws_kernel<MT, NT, KNOB>), dim3(grid), dim3(2 * kThreadsT), 0,
                     stream, a);
  return hipGetLastError();
}

// K1-fp8 on a wave-specialised tile: C (bf16) = A (e4m3) * B (e4m3)^T, M x N x
// K in fp8 elements (N % 8, K % 16, 16-byte aligned rows); the kernel sees the
// operands as bf16-sized pairs (K / 2, lda / 2, ldb / 2), exactly like the
// 256x256 fp8 build (gemm_fp8.hpp).
template <int MT, int NT>
inline hipError_t launch_gemm_fp8_tile_ws(const void* A, const void* B, __bf16* C, int M, int N,
                                          int K, int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (N % 8) || (K % 16) || lda < K || ldb < K || ldc < N ||
      (lda % 16) || (ldb % 16) || (ldc % 4))
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
  const unsigned grid = (unsigned)(((M + Cfg<MT, NT>::TM - 1) / Cfg<MT, NT>::TM) *
                                   ((N + Cfg<MT, NT>::TN - 1) / Cfg<MT, NT>::TN));
  hipLaunchKernelGGL((gemm_bf16_tile_ws_kernel<MT, NT, 0, false, true>), dim3(grid),
                     dim3(2 * kThreadsT), 0, stream, a);
  return hipGetLastError();
}

// Split-K over S slices of kc = ceil(K / S) rounded up to 64 (the last slice
// may be shorter; its partial K-tile reads zeros): the wave-specialised tile
// kernel on a (tiles, S) grid writes fp32 partials to ws (S M N floats), then
// splitk_reduce_kernel sums them into C. For C too small to fill the chip
// with a long K (hipBLASLt's GSU kernels serve these shapes the same way).
inline int splitk_kc(int K, int S) { return ((K + S - 1) / S + TK - 1) / TK * TK; }
inline int splitk_slices(int K, int S) { const int kc = splitk_kc(K, S); return (K + kc - 1) / kc; }

template <int MT, int NT>
inline hipError_t launch_gemm_bf16_tile_ws_splitk(const GemmArgs& a, int S, float* ws,
                                                  hipStream_t stream) {
  if (!shape_ok_ws(a.M, a.N, a.K) || S < 1 || !ws || a.lda < a.K || a.ldb < a.K ||
      a.ldc < a.N || (a.lda % 8) || (a.ldb % 8) || (a.ldc % 4))
    return hipErrorInvalidValue;
  GemmArgs b = a;
  b.splitk_ws = ws;
  b.splitk_kc = splitk_kc(a.K, S);
  const int slices = splitk_slices(a.K, S);
  const unsigned tiles = (unsigned)(((a.M + Cfg<MT, NT>::TM - 1) / Cfg<MT, NT>::TM) *
                                    ((a.N + Cfg<MT, NT>::TN - 1) / Cfg<MT, NT>::TN));
  hipLaunchKernelGGL((gemm_bf16_tile_ws_kernel<MT, NT, 0, true>), dim3(tiles, (unsigned)slices),
                     dim3(2 * kThreadsT), 0, stream, b);
  const size_t n4 = (size_t)a.M * a.N / 4;
  const unsigned rg = (unsigned)std::min<size_t>(4096, (n4 + 255) / 256);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(rg), dim3(256), 0, stream, ws, a.C, a.M, a.N,
                     a.ldc, slices);
  return hipGetLastError();
}

// Split-K for K1-fp8: the launch above on the fp8 consumer. K, lda, ldb in fp8
// elements (N % 8, K % 16, 16-byte aligned rows); slices of the K-tile range
// counted in bf16-sized pairs (128 e4m3 values per K-tile), ws holds
// splitk_slices(K / 2, S) M N floats.
template <int MT, int NT>
inline hipError_t launch_gemm_fp8_tile_ws_splitk(const void* A, const void* B, __bf16* C, int M,
                                                 int N, int K, int lda, int ldb, int ldc, int S,
                                                 float* ws, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (N % 8) || (K % 16) || lda < K || ldb < K || ldc < N ||
      (lda % 16) || (ldb % 16) || (ldc % 4) || S < 1 || !ws)
    return hipErrorInvalidValue;
  GemmArgs b;
  b.A = (const __bf16*)A;
  b.B = (const __bf16*)B;
  b.C = C;
  b.M = M;
  b.N = N;
  b.K = K / 2;
  b.lda = lda / 2;
  b.ldb = ldb / 2;
  b.ldc = ldc;
  b.splitk_ws = ws;
  b.splitk_kc = splitk_kc(b.K, S);
  const int slices = splitk_slices(b.K, S);
  const unsigned tiles = (unsigned)(((M + Cfg<MT, NT>::TM - 1) / Cfg<MT, NT>::TM) *
                                    ((N + Cfg<MT, NT>::TN - 1) / Cfg<MT, NT>::TN));
  hipLaunchKernelGGL((gemm_bf16_tile_ws_kernel<MT, NT, 0, true, true>), dim3(tiles, (unsigned)slices),
                     dim3(2 * kThreadsT), 0, stream, b);
  const size_t n4 = (size_t)M * N / 4;
  const unsigned rg = (unsigned)std::min<size_t>(4096, (n4 + 255) / 256);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(rg), dim3(256), 0, stream, ws, C, M, N, ldc,
                     slices);
  return hipGetLastError();
}

}  // namespace gemmt
}  // namespace ntm
