// DIAGNOSTIC build of the 4-wave one-barrier-per-K-tile kernel ("dma4k",
// gemm_w4k.hpp, DI = 3) with per-step s_memtime stamps, for
// a cycle budget of the step: [row 0 MFMAs] t_a [s_waitcnt lgkmcnt(0) +
// vmcnt(0)] t_b [s_barrier] t_c [rows 1..7]. Each stamp's value is consumed
// one step later, after the next barrier's lgkmcnt(0) retired it, so the
// stamps add no wait of their own. Never used for results: modes 2-4 compute
// garbage by construction, and the stamps go to their own buffer.
//
// MODE 0: the real schedule + stamps;
// MODE 1: no LDS-DMA (fragment reads hit stale LDS; the vmcnt wait is empty);
// MODE 2: no fragment reads (registers of K-tile 0);
// MODE 3: no s_barrier (waits kept; reads race the DMA);
// MODE 4: MFMAs only (no DMA, reads or barrier).
// Per wave (lane 0): [start, end, wait, barrier, realtime start, realtime end,
// HW_ID, XCC_ID, loop start, loop end] (u64); wait / barrier: cycles summed
// over the K loop.
#pragma once

#include "ntm/gemm_w4k.hpp"

namespace ntm {
namespace r4ks {

using namespace ::ntm::w4k;
using ::ntm::gemm::GemmArgs;
using ::ntm::gemm::raw_barrier;

constexpr int kSlots = 10;

struct Stamps {
  unsigned long long wait = 0, bar = 0;
  unsigned long long ta = 0, tb = 0, tc = 0;
};

template <int BUF, int MODE, bool F8>
__device__ __forceinline__ void step_s(const Ctx& c, f32x4 (&acc)[8][8], Frags8& f, int t, int T,
                                       int w, Stamps& s) {
  constexpr int DI = 3;
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    mma<F8>(acc[0][nt], f, 0, nt);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the previous step's stamps have retired (lgkmcnt(0) at its barrier)
  if (t > 0) {
    s.wait += s.tb - s.ta;
    s.bar += s.tc - s.tb;
  }
  s.ta = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (MODE != 1 && MODE != 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  s.tb = __builtin_amdgcn_s_memtime();
  if constexpr (MODE != 3 && MODE != 4) raw_barrier();
  s.tc = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int mt = 1; mt < 8; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      mma<F8>(acc[mt][nt], f, mt, nt);
      const int j = (mt - 1) * 8 + nt;
      if constexpr (MODE != 1 && MODE != 4) {
        if ((j % DI) == 0 && j / DI < 16) issue_piece(c, t + 2, T, BUF, w, j / DI);
      }
      if constexpr (MODE != 2 && MODE != 4) {
        if (nt == 1) read_a(c, f, BUF ^ 1, mt - 1);
        if (mt == 7) read_b(c, f, BUF ^ 1, nt);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (MODE != 2 && MODE != 4) read_a(c, f, BUF ^ 1, 7);
  __builtin_amdgcn_sched_barrier(0);
}

template <int MODE, bool F8, bool NT>
__global__ void __launch_bounds__(kThreads, 1) gemm_r4k_stamp_kernel(GemmArgs p,
                                                                     unsigned long long* stamps) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  Ctx c;
  int m0, n0, lane, w, wr, wc;
  setup(p, smem, c, m0, n0, lane, w, wr, wc);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int T = p.K / 64;
  Frags8 f;
  prologue(c, f, T, w);
  Stamps s;
  const unsigned long long tl0 = __builtin_amdgcn_s_memtime();
  int t = 0;
  do {
    step_s<0, MODE, F8>(c, acc, f, t, T, w, s);
    step_s<1, MODE, F8>(c, acc, f, t + 1, T, w, s);
    t += 2;
  } while (t < T - 2);
  step_s<0, MODE, F8>(c, acc, f, t, T, w, s);
  step_s<1, MODE, F8>(c, acc, f, t + 1, T, w, s);
  ::ntm::gemm::mfma_drain();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  s.wait += s.tb - s.ta;
  s.bar += s.tc - s.tb;
  const unsigned long long tl1 = __builtin_amdgcn_s_memtime();
  raw_barrier();
  store_tile<NT>(p, smem, acc, m0, n0, w, wr, wc, lane);
  const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    unsigned long long* o = stamps + ((size_t)blockIdx.x * 4 + w) * kSlots;
    o[0] = ts0;
    o[1] = ts1;
    o[2] = s.wait;
    o[3] = s.bar;
    o[4] = rt0;
    o[5] = rt1;
    o[6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    o[7] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    o[8] = tl0;
    o[9] = tl1;
  }
}

// stamps: (M/256)*(N/256) * 4 waves * kSlots (10) u64. mode + 8: temporal C
// stores (default nontemporal); mode + 16: e4m3 operands (K, lda, ldb in fp8
// elements, as launch_gemm_fp8_w4k).
template <bool F8, bool NT>
inline hipError_t launch_stamp(const GemmArgs& a, int mode, unsigned long long* stamps,
                               hipStream_t stream) {
  const dim3 g((unsigned)((a.M / BM) * (a.N / BN))), b(kThreads);
  switch (mode) {
    case 0: hipLaunchKernelGGL((gemm_r4k_stamp_kernel<0, F8, NT>), g, b, 0, stream, a, stamps); break;
    case 1: hipLaunchKernelGGL((gemm_r4k_stamp_kernel<1, F8, NT>), g, b, 0, stream, a, stamps); break;
    case 2: hipLaunchKernelGGL((gemm_r4k_stamp_kernel<2, F8, NT>), g, b, 0, stream, a, stamps); break;
    case 3: hipLaunchKernelGGL((gemm_r4k_stamp_kernel<3, F8, NT>), g, b, 0, stream, a, stamps); break;
    case 4: hipLaunchKernelGGL((gemm_r4k_stamp_kernel<4, F8, NT>), g, b, 0, stream, a, stamps); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

inline hipError_t launch_gemm_r4k_stamp(GemmArgs a, int mode, unsigned long long* stamps,
                                        hipStream_t stream) {
  const bool f8 = (mode & 16) != 0, nt = (mode & 8) == 0;
  mode &= 7;
  if (f8) {
    if ((a.K % 256) || (a.lda % 16) || (a.ldb % 16)) return hipErrorInvalidValue;
    a.K /= 2;
    a.lda /= 2;
    a.ldb /= 2;
  }
  if (a.M <= 0 || a.N <= 0 || a.K < 256 || (a.M % BM) || (a.N % BN) || (a.K % 128) ||
      a.lda < a.K || a.ldb < a.K || a.ldc < a.N || (a.lda % 8) || (a.ldb % 8) || (a.ldc % 8) ||
      (long long)a.M * a.lda * 2 >= (1ll << 31) || (long long)a.N * a.ldb * 2 >= (1ll << 31) ||
      !stamps)
    return hipErrorInvalidValue;
  if (f8) return nt ? launch_stamp<true, true>(a, mode, stamps, stream)
                    : launch_stamp<true, false>(a, mode, stamps, stream);
  return nt ? launch_stamp<false, true>(a, mode, stamps, stream)
            : launch_stamp<false, false>(a, mode, stamps, stream);
}

}  // namespace r4ks
}  // namespace ntm
