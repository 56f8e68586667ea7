// EXPERIMENTAL / DIAGNOSTIC K1 builds -> nvidia_terraform_modules_amd/ops/
// libntm_experimental.so. Loaded only by tests and tools/ (schedule studies,
// ablations, rate probes); never linked into libntm_validation.so or the
// validation-Job binary, which carry only the default-dispatch kernels.
//
// K1 variants (bf16, C = A B^T, the numbering of ops.kernels.GEMM_VARIANTS):
//   1      pingpong8: the first 8-wave 12/4/8/0 LDS-read schedule (gemm_bf16.hpp)
//   10..13 pingpong8c epilogue knobs: widened / + early row-0 stores /
//          nontemporal stores / both (gemm_bf16_pp3.hpp launch_gemm_bf16_pp3_knob)
//   41..46 pingpong8o studies: 128 workgroups, C not stored, whole-line C
//          layout (44), LDS-staged whole-line boundary stores (46)
//   19..21 tile128w4 / tile256x128w4 / tile160w4: the 4-wave (one wave per
//          SIMD) tile kernels that the wave-specialised ones replaced as
//          variants 15..17 (gemm_bf16_t128.hpp; profiles/r2_ws)
// Rejected builds are deleted once measured (git history keeps them: the 4-wave
// wave128 / wave128d4, the persistent pingpong8p / 8pw, the 32-MFMA-segment
// pingpong8w / wi / ww, fp8 knobs 6-9 - profiles/r1_pmc2_w4, r1_pp4, r2_fp8ws;
// round 3's register-staged, half-K-tile-ring, 5-slot-ring and SGPR-DMA
// builds - profiles/r3_k1; the overlap kernel's sc1 / plain-store / static-
// priority builds and pingpong8c's write-through epilogues - profiles/r3_k1o;
// round 4: the 4-wave persistent overlap dma4ko / fp8 knob 22 (gemm_w4o.hpp,
// profiles/r3_w4o), the dma4k stamp build (gemm_r4k_stamp.hpp) and dma4k itself
// (variant 39 / fp8 knob 12, gemm_w4k.hpp: 4 waves x 128x128 per wave, one
// barrier per K-tile; it tied the 8-wave default, profiles/r3_k1));
// what stays is used by a test or a tool under tools/.
#include "ntm/dma_probe.hpp"
#include "ntm/gemm_bf16.hpp"
#include "ntm/gemm_bf16_pp3.hpp"
#include "ntm/gemm_bf16_pp3h.hpp"
#include "ntm/gemm_bf16_pp3_stamp.hpp"
#include "ntm/gemm_bf16_pp6.hpp"
#include "ntm/gemm_bf16_sk.hpp"
#include "ntm/gemm_w4k.hpp"
#include "ntm/gemm_bf16_t128.hpp"
#include "ntm/gemm_fp8_diag.hpp"
#include "ntm/stream_policy_exp.hpp"

#define NTM_API extern "C" __attribute__((visibility("default")))

namespace {
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

ntm::gemm::GemmArgs args(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                         int ldb, int ldc) {
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  return a;
}
}  // namespace

NTM_API const char* ntm_experimental_version() { return "ntm-experimental 0.2.0 gfx950"; }

NTM_API int ntm_gemm_bf16_experimental(int variant, const void* A, const void* B, void* C, int M,
                                       int N, int K, int lda, int ldb, int ldc, void* stream) {
  const ntm::gemm::GemmArgs a = args(A, B, C, M, N, K, lda, ldb, ldc);
  switch (variant) {
    case 1: return (int)ntm::gemm::launch_gemm_bf16(a, S(stream));
    case 10:
    case 11:
    case 12:
    case 13: return (int)ntm::gemm3::launch_gemm_bf16_pp3_knob(a, variant + 2, S(stream));
    // 4 waves x 128x128, one barrier per K-tile, two K-tile LDS-DMA buffers, a DMA
    // piece every 3 MFMA pairs (gemm_w4k.hpp; restored in round 6 for the energy
    // study, profiles/r6_fp8)
    case 39: return (int)ntm::w4k::launch_gemm_bf16_w4k<3>(a, S(stream));
    // 56-58 (round 6, "dma4kh": the same 4-wave tile in two k-half passes per
    // K-tile) were removed after measurement: 4-9 % slower (profiles/r6_w4kh/).
    // 56 (round 6, "dma4kr": dma4k_d3 with each row's k-half 0 MFMAs before its
    // k-half 1 ones) was removed after measurement: 2 % slower (profiles/r6_w4kh/).
    // 59-61 (round 6, "dma4kx": hipBLASLt's wait structure - three barriers per
    // K-tile, per-operand LDS recycling, a counted vmcnt) were removed after
    // measurement: 4-6 % behind dma4k_d3 (profiles/r6_w4kh/).
    case 19: return (int)ntm::gemmt::launch_gemm_bf16_tile<4>(a, S(stream));
    case 20: return (int)ntm::gemmt::launch_gemm_bf16_tile<8>(a, S(stream));
    case 21: return (int)ntm::gemmt::launch_gemm_bf16_tile<5, 5>(a, S(stream));
    // store-bandwidth study (profiles/r3_stores): pingpong8o on 128 workgroups,
    // and with C not stored on 128 / 256 workgroups
    case 41: return (int)ntm::gemm6::launch_gemm_bf16_pp6_grid<1>(a, 128, S(stream));
    case 42: return (int)ntm::gemm6::launch_gemm_bf16_pp6_grid<2>(a, 128, S(stream));
    case 43: return (int)ntm::gemm6::launch_gemm_bf16_pp6_grid<2>(a, 256, S(stream));
    // 44-46 (round 4: whole-line C layouts, with and without LDS-staged boundary
    // stores) were removed after measurement (profiles/r4_stg/).
    // 48: boundary stores spread one block per phase (SPREAD) = the shipping 25
    case 48: return (int)ntm::gemm6::launch_gemm_bf16_pp6<1, 0, true>(a, S(stream));
    // 53 (round 5, pingpong8op: the next tile's K-tiles 0 / 1 touched into L2 over
    // K-tiles T-4 / T-3) was removed after measurement (profiles/r5_pf/).
    // 47: pingpong8om, the persistent overlap kernel on ragged C (masked edge
    // tiles, partial K; pingpong8cm where it does not serve). Off the plan since
    // round 4 (profiles/r4_om/), moved out of the shipping library in round 5.
    case 47:
      if (!ntm::gemm6::shape_ok6m(M, N, K) || (lda % 8) || (ldb % 8) || (ldc % 8))
        return (int)ntm::gemm3::launch_gemm_bf16_pp3_masked(a, S(stream));
      return (int)ntm::gemm6::launch_gemm_bf16_pp6_masked<1>(a, S(stream));
    // 29: 224x256 ping-pong tiles (gemm_bf16_pp3h.hpp, a 96-row A-hi half): on 11
    // shapes of 0.78-0.91 rounds of 256x256 tiles it won 2-6 % on five and lost
    // 1-7 % on four against pingpong8cm (profiles/r5_h192/pp224_sweep.log), so
    // the plan does not use it
    case 29: return (int)ntm::gemm3h::launch_gemm_bf16_pp3h<96, 128>(a, S(stream));
    // 51: pingpong8om (ragged C) with the spread boundary stores
    case 51: return (int)ntm::gemm6::launch_gemm_bf16_pp6_masked<1, true>(a, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

// Stream-K test build (gemm_bf16_sk.hpp REV): each workgroup runs its segments
// in range order, so tails usually reach the fix-up before heads; C must be
// bitwise equal to ntm_gemm_bf16_sk's.
NTM_API int ntm_gemm_bf16_sk_rev(const void* A, const void* B, void* C, int M, int N, int K,
                                 int lda, int ldb, int ldc, void* ws, size_t ws_bytes,
                                 void* stream) {
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  return (int)ntm::gemmsk::launch_gemm_bf16_sk<true>(a, ntm::gemm6::pp6_grid(1 << 30), ws,
                                                     ws_bytes, S(stream));
}

// Stream-K stamp build (gemm_bf16_sk.hpp STAMP): 16 u64 per workgroup.
NTM_API int ntm_gemm_bf16_sk_stamp(const void* A, const void* B, void* C, int M, int N, int K,
                                   int lda, int ldb, int ldc, void* ws, size_t ws_bytes,
                                   void* stamps, void* stream) {
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  return (int)ntm::gemmsk::launch_gemm_bf16_sk<false, true>(
      a, ntm::gemm6::pp6_grid(1 << 30), ws, ws_bytes, S(stream), (unsigned long long*)stamps);
}

// Stream-K split mode with the S-partial protocol also at S = 2 (the round-4
// build; the shipping one uses the head / tail protocol there): A/B only.
NTM_API int ntm_gemm_bf16_sk_nopair(const void* A, const void* B, void* C, int M, int N, int K,
                                    int lda, int ldb, int ldc, void* ws, size_t ws_bytes,
                                    void* stream) {
  const ntm::gemm::GemmArgs a = args(A, B, C, M, N, K, lda, ldb, ldc);
  return (int)ntm::gemmsk::launch_gemm_bf16_sk<false, false, false>(
      a, ntm::gemm6::pp6_grid(1 << 30), ws, ws_bytes, S(stream));
}

// Ablation (round 6, profiles/r6_xcd): the shipping pingpong8o with each odd-XCD
// workgroup's last tile cut by 2 * cut_pairs K-tiles (C is WRONG; timing only).
NTM_API int ntm_gemm_bf16_pp6_oddcut(int cut_pairs, const void* A, const void* B, void* C, int M,
                                     int N, int K, int lda, int ldb, int ldc, void* stream) {
  ntm::gemm::GemmArgs a = args(A, B, C, M, N, K, lda, ldb, ldc);
  a.splitk_kc = cut_pairs;
  return (int)ntm::gemm6::launch_gemm_bf16_pp6<1, 3, true>(a, S(stream));
}

// pingpong8o boundary-phase stamps (gemm_bf16_pp6.hpp STAMP 2): grid 128 or 256
// workgroups (a multiple of 8, <= tiles, each workgroup >= 2 tiles), store 1 =
// C stored (nontemporal) / 0 = not stored / 2 = stored, spread over the boundary
// phases (the shipping build); stamps: 17 u64 per workgroup.
NTM_API int ntm_gemm_bf16_pp6_stamp(int grid, int store, const void* A, const void* B, void* C,
                                    int M, int N, int K, int lda, int ldb, int ldc, void* stamps,
                                    void* stream) {
  ntm::gemm::GemmArgs a = args(A, B, C, M, N, K, lda, ldb, ldc);
  a.stamps = (unsigned long long*)stamps;
  if (grid * 2 > (M / 256) * (N / 256)) return (int)hipErrorInvalidValue;
  using namespace ntm::gemm6;
  switch (store) {
    case 0: return (int)launch_gemm_bf16_pp6_grid<2, 2>(a, grid, S(stream));
    case 1: return (int)launch_gemm_bf16_pp6_grid<1, 2>(a, grid, S(stream));
    case 2: return (int)launch_gemm_bf16_pp6_grid<1, 2, true>(a, grid, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

// pingpong8c tuning knobs (see launch_gemm_bf16_pp3_knob).
NTM_API int ntm_gemm_bf16_knob(int knob, const void* A, const void* B, void* C, int M, int N,
                               int K, int lda, int ldb, int ldc, void* stream) {
  return (int)ntm::gemm3::launch_gemm_bf16_pp3_knob(args(A, B, C, M, N, K, lda, ldb, ldc), knob,
                                                    S(stream));
}

// pingpong8c ablation builds with s_memtime stamps (gemm_bf16_pp3_stamp.hpp;
// mode 0 real, 1 no LDS traffic, 2 no MFMA, 3 MFMA only).
// stamps: (M/256)*(N/256)*8*4 u64.
NTM_API int ntm_gemm_bf16_stamp(int mode, const void* A, const void* B, void* C, int M, int N,
                                int K, int lda, int ldb, int ldc, void* stamps, void* stream) {
  return (int)ntm::gemm3s::launch_gemm_bf16_pp3_stamp(args(A, B, C, M, N, K, lda, ldb, ldc), mode,
                                                      (unsigned long long*)stamps, S(stream));
}

// Matrix-core issue rate (gemm_fp8_diag.hpp mfma_rate_kernel): f8 0 = bf16
// 16x16x32, 1 = e4m3 16x16x128, 2 = bf16 32x32x16; out: 2 u64 per wave (grid x
// 4 waves), sink: 1 float.
NTM_API int ntm_mfma_rate(int f8, int grid, int iters, void* out, float* sink, void* stream) {
  if (grid <= 0 || iters <= 0) return (int)hipErrorInvalidValue;
  if (f8 == 3)   // e4m3 v_mfma_f32_32x32x64_f8f6f4 (2x the MACs of 16x16x128)
    hipLaunchKernelGGL((ntm::fp8::mfma_rate_kernel<true, true>), dim3(grid), dim3(256), 0,
                       S(stream), iters, 7u, (unsigned long long*)out, sink);
  else if (f8 == 2)   // bf16 v_mfma_f32_32x32x16 (2x the MACs per instruction)
    hipLaunchKernelGGL((ntm::fp8::mfma_rate_kernel<false, true>), dim3(grid), dim3(256), 0,
                       S(stream), iters, 7u, (unsigned long long*)out, sink);
  else if (f8)
    hipLaunchKernelGGL(ntm::fp8::mfma_rate_kernel<true>, dim3(grid), dim3(256), 0, S(stream),
                       iters, 7u, (unsigned long long*)out, sink);
  else
    hipLaunchKernelGGL(ntm::fp8::mfma_rate_kernel<false>, dim3(grid), dim3(256), 0, S(stream),
                       iters, 7u, (unsigned long long*)out, sink);
  return (int)hipGetLastError();
}

// Operand-toggle energy probe (gemm_fp8_diag.hpp mfma_toggle_kernel): 16
// bf16 16x16x32 MFMAs per iteration in operand order pat 0..6.
NTM_API int ntm_mfma_toggle(int pat, int grid, int iters, void* out, float* sink, void* stream) {
  if (grid <= 0 || iters <= 0) return (int)hipErrorInvalidValue;
  auto* o = (unsigned long long*)out;
  switch (pat) {
#define NTM_TOGGLE(P)                                                                         \
  case P:                                                                                     \
    hipLaunchKernelGGL(ntm::fp8::mfma_toggle_kernel<P>, dim3(grid), dim3(256), 0, S(stream), \
                       iters, 7u, o, sink);                                                   \
    break;
    NTM_TOGGLE(0) NTM_TOGGLE(1) NTM_TOGGLE(2) NTM_TOGGLE(3) NTM_TOGGLE(4) NTM_TOGGLE(5)
    NTM_TOGGLE(6)
#undef NTM_TOGGLE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Wave-specialised tile kernel schedule knobs (gemm_bf16_t128.hpp kWs*):
// shape 0 = 128x128, 1 = 256x128, 2 = 160x160; knob 0..8.
template <int MT, int NT>
static hipError_t ws_knob(const ntm::gemm::GemmArgs& a, int knob, hipStream_t s) {
  using namespace ntm::gemmt;
  switch (knob) {
    case 0: return launch_gemm_bf16_tile_ws<MT, NT, 0>(a, s);
    case 1: return launch_gemm_bf16_tile_ws<MT, NT, 1>(a, s);
    case 2: return launch_gemm_bf16_tile_ws<MT, NT, 2>(a, s);
    case 3: return launch_gemm_bf16_tile_ws<MT, NT, 3>(a, s);
    case 4: return launch_gemm_bf16_tile_ws<MT, NT, 4>(a, s);
    case 5: return launch_gemm_bf16_tile_ws<MT, NT, 5>(a, s);
    case 6: return launch_gemm_bf16_tile_ws<MT, NT, 6>(a, s);
    case 7: return launch_gemm_bf16_tile_ws<MT, NT, 7>(a, s);
    case 8: return launch_gemm_bf16_tile_ws<MT, NT, 8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

NTM_API int ntm_gemm_bf16_ws_knob(int shape, int knob, const void* A, const void* B, void* C,
                                  int M, int N, int K, int lda, int ldb, int ldc, void* stream) {
  const ntm::gemm::GemmArgs a = args(A, B, C, M, N, K, lda, ldb, ldc);
  switch (shape) {
    case 0: return (int)ws_knob<4, 4>(a, knob, S(stream));
    case 1: return (int)ws_knob<8, 4>(a, knob, S(stream));
    case 2: return (int)ws_knob<5, 5>(a, knob, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

// K1-fp8 schedule knobs (gemm_fp8_diag.hpp launch_gemm_fp8_knob).
NTM_API int ntm_gemm_fp8_knob(const void* A, const void* B, void* C, int M, int N, int K,
                              int lda, int ldb, int ldc, int knob, void* stream) {
  return (int)ntm::fp8::launch_gemm_fp8_knob(A, B, (__bf16*)C, M, N, K, lda, ldb, ldc, knob,
                                             S(stream));
}

// One v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, unit scales) on
// per-lane operands: a_stage / b_stage 64 x 32 B, d 64 x 4 fp32.
NTM_API int ntm_mfma_f8_probe(const void* a_stage, const void* b_stage, float* d, void* stream) {
  hipLaunchKernelGGL(ntm::fp8::mfma_f8_probe_kernel, dim3(1), dim3(64), 0, S(stream),
                     (const ntm::fp8::i32x8*)a_stage, (const ntm::fp8::i32x8*)b_stage,
                     (ntm::f32x4*)d);
  return (int)hipGetLastError();
}

// K2 store-policy sweep (stream_policy_exp.hpp): unroll in {4, 8}, spol 0..5
// (none / nt / sc1 / sc0 sc1 / nt sc1 / nt sc0 sc1), grid > 0.
NTM_API int ntm_stream_copy_spol(const void* src, void* dst, size_t bytes, int unroll, int spol,
                                 int grid, void* stream) {
  if (bytes % 16 || grid <= 0 || spol < 0 || spol > 5 || (unroll != 4 && unroll != 8))
    return (int)hipErrorInvalidValue;
  const auto* a = (const ntm::f32x4*)src;
  auto* b = (ntm::f32x4*)dst;
  const size_t n4 = bytes / 16;
#define NTM_SPOL(U, P) \
  if (unroll == U && spol == P) \
    hipLaunchKernelGGL((ntm::k2x::copy_pipe_spol_kernel<U, P>), dim3(grid), dim3(256), 0, S(stream), a, b, n4);
  NTM_SPOL(4, 0) NTM_SPOL(4, 1) NTM_SPOL(4, 2) NTM_SPOL(4, 3) NTM_SPOL(4, 4) NTM_SPOL(4, 5)
  NTM_SPOL(8, 0) NTM_SPOL(8, 1) NTM_SPOL(8, 2) NTM_SPOL(8, 3) NTM_SPOL(8, 4) NTM_SPOL(8, 5)
#undef NTM_SPOL
  return (int)hipGetLastError();
}

// LDS-DMA access-pattern probe (dma_probe.hpp; tools/experiments/dma_probe.py): the 256x256
// ping-pong's loads with no MFMAs, mode 0 / 1 / 2, `grid` workgroups of 512.
NTM_API int ntm_dma_probe(int mode, const void* base, int pitch, int T, int reps, int grid,
                          void* stream) {
  return (int)ntm::dprobe::launch_dma_probe(mode, (const __bf16*)base, pitch, T, reps, grid,
                                            S(stream));
}
