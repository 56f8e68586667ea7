// LDS-DMA access-pattern probe (experimental library only): which per-CU
// resource makes K1 slow when the rows of A / B are only 16-byte aligned
// (K % 16 == 8, profiles/r5_h192/)? The loads of the 256x256 ping-pong are
// replayed with no MFMAs: per K-tile, four 128-row halves, each wave staging
// 16 rows x 64 k as two 16-B-per-lane glds pieces (k chunks 0-3, then 4-7),
// counted vmcnt(10) as in the kernel. Every workgroup streams the same 512
// rows, so the XCD's L2 serves them (as the GEMM's shared A / B panels).
//
// MODE 0: the kernel's pattern at the given row pitch (aligned or not).
// MODE 1: at a misaligned pitch, each row's K-tile t re-based to whole 64-B
//         quads that never straddle a line: piece 1 = the second half of the
//         row's aligned line t, piece 2 = the first half of line t + 1 - two
//         L1 accesses per row per K-tile as when aligned, but each line still
//         fetched by two different K-tiles (the accesses of a half-line ring
//         in LDS; the data is the wrong k window - timing only).
// MODE 2: at a misaligned pitch, each row re-based down to its aligned line -
//         the aligned pattern on the same rows (what a 3-line ring would load).
// MODE 3: MODE 0's bytes, but each instruction covers 8 rows x 128 B (8 lanes
//         per row: whole lines) instead of 16 rows x 64 B (each line split over
//         two instructions): the energy question of profiles/r6_edec.
#pragma once

#include "ntm/gemm_bf16.hpp"

namespace ntm {
namespace dprobe {

using namespace ::ntm::gemm;

template <int N>
__device__ __forceinline__ void wait_vm_deep() {
  if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
}

template <int AUX>
__device__ __forceinline__ void glds16_pol(const void* gsrc, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const void NTM_AS1*)gsrc, (void NTM_AS3*)lds_dst, 16, 0, AUX);
}

// VM: the counted wait after each half (10 = the kernel's: 5 halves in flight;
// deeper values only exist here, where nothing reads the LDS). AUX: the load's
// cache-policy bits (gfx950: 1 sc0, 2 nt, 16 sc1).
template <int MODE, int VM = 10, int AUX = 0>
__global__ void __launch_bounds__(512) dma_probe_kernel(const __bf16* base, int pitch, int T,
                                                        int reps) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kTileBytes];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = MODE == 3 ? lane >> 3 : lane >> 2, cl = MODE == 3 ? lane & 7 : lane & 3;
  const char* rows[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const char* p = (const char*)(base + (size_t)(h * 128 + w * 16 + r) * pitch);
    if constexpr (MODE == 1 || MODE == 2) p = (const char*)((size_t)p & ~(size_t)127);
    rows[h] = p;
  }
  for (int rep = 0; rep < reps; ++rep) {
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const char* s1;
        const char* s2;
        if constexpr (MODE == 1) {
          s1 = rows[h] + (size_t)t * 128 + 64 + cl * 16;
          s2 = rows[h] + (size_t)(t + 1) * 128 + cl * 16;
        } else if constexpr (MODE == 3) {   // rows r and r + 8, whole 128-B lines
          s1 = rows[h] + (size_t)t * 128 + cl * 16;
          s2 = s1 + (size_t)8 * pitch * 2;
        } else {
          s1 = rows[h] + (size_t)t * 128 + cl * 16;
          s2 = s1 + 64;
        }
        char* d = smem + (t & 1) * kTileBytes + h * kHalfBytes + (2 * w) * 1024;
        glds16_pol<AUX>(s1, d);
        glds16_pol<AUX>(s2, d + 1024);
        wait_vm_deep<VM>();
      }
    }
  }
  wait_vmcnt<0>();
}

// rows of the probe: 512 (4 halves x 128); the buffer must hold 512 rows of
// `pitch` elements plus (T + 1) * 64 + 64 elements past the last row start
inline hipError_t launch_dma_probe(int mode, const __bf16* base, int pitch, int T, int reps,
                                   int grid, hipStream_t s) {
  if (T < 1 || reps < 1 || grid < 1 || pitch < (T + 1) * 64 + 64) return hipErrorInvalidValue;
  // mode + 10 * d + 100 * a: d = 0..3 -> counted wait 10 / 16 / 24 / 32 (5 / 8 / 12 / 16
  // halves in flight); a = 1..5 -> cache policy sc0 / nt / sc0 nt / sc1 / sc1 nt (depth 10)
  if (mode >= 100) {
    const int a = mode / 100, m = mode % 100;
    if (m > 2) return hipErrorInvalidValue;
#define NTM_DPROBE_POL(A, AUXV)                                                                    \
  if (a == A) {                                                                                    \
    if (m == 0) hipLaunchKernelGGL((dma_probe_kernel<0, 10, AUXV>), dim3(grid), dim3(512), 0, s, base, pitch, T, reps); \
    if (m == 1) hipLaunchKernelGGL((dma_probe_kernel<1, 10, AUXV>), dim3(grid), dim3(512), 0, s, base, pitch, T, reps); \
    if (m == 2) hipLaunchKernelGGL((dma_probe_kernel<2, 10, AUXV>), dim3(grid), dim3(512), 0, s, base, pitch, T, reps); \
  }
    NTM_DPROBE_POL(1, 1) NTM_DPROBE_POL(2, 2) NTM_DPROBE_POL(3, 3) NTM_DPROBE_POL(4, 16)
    NTM_DPROBE_POL(5, 18)
#undef NTM_DPROBE_POL
    if (a > 5) return hipErrorInvalidValue;
    return hipGetLastError();
  }
  const int d = mode / 10;
  mode %= 10;
  if (mode == 3 && d == 0) {
    hipLaunchKernelGGL((dma_probe_kernel<3, 10>), dim3(grid), dim3(512), 0, s, base, pitch, T, reps);
    return hipGetLastError();
  }
  if (mode > 2 || d > 3) return hipErrorInvalidValue;
#define NTM_DPROBE(M, V) \
  if (mode == M && (V) == (d == 0 ? 10 : d == 1 ? 16 : d == 2 ? 24 : 32)) \
    hipLaunchKernelGGL((dma_probe_kernel<M, V>), dim3(grid), dim3(512), 0, s, base, pitch, T, reps);
  NTM_DPROBE(0, 10) NTM_DPROBE(1, 10) NTM_DPROBE(2, 10)
  NTM_DPROBE(0, 16) NTM_DPROBE(1, 16) NTM_DPROBE(2, 16)
  NTM_DPROBE(0, 24) NTM_DPROBE(1, 24) NTM_DPROBE(2, 24)
  NTM_DPROBE(0, 32) NTM_DPROBE(1, 32) NTM_DPROBE(2, 32)
#undef NTM_DPROBE
  return hipGetLastError();
}

}  // namespace dprobe
}  // namespace ntm
