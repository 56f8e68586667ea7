// EXPERIMENTAL (libntm_experimental.so only): K2 copy with the store cache
// policy spelled out in the instruction (inline asm global_store_dwordx4), to
// sweep modifiers the HIP builtins do not expose (sc0 / sc1 / nt
// combinations). Loads stay compiler-managed (__builtin_nontemporal_load), so
// the compiler's vmcnt tracking covers every use of loaded data; a store needs
// no wait (the wave's s_endpgm drains it), but its data VGPRs are read after
// issue: each asm store ends with s_nop 1 (cdna_hip_programming.md §5.7) or the
// next instruction may overwrite them first. Vector stores only.
#pragma once

#include "ntm/aux_kernels.hpp"

namespace ntm {
namespace k2x {

template <int SPOL>
__device__ __forceinline__ void store16(f32x4* p, const f32x4& v) {
  if constexpr (SPOL == 0) asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  if constexpr (SPOL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  if constexpr (SPOL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  if constexpr (SPOL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  if constexpr (SPOL == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  if constexpr (SPOL == 5) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// One-tile-ahead pipelined block-tiled copy (= aux stream_copy_pipe_kernel with
// nontemporal loads) with store policy SPOL.
template <int U, int SPOL>
__global__ void __launch_bounds__(256)
    copy_pipe_spol_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n4) {
  constexpr size_t kTile = 256 * U;
  const size_t ntiles = n4 / kTile;
  size_t t = blockIdx.x;
  f32x4 v[U];
  if (t < ntiles) {
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = __builtin_nontemporal_load(src + t * kTile + threadIdx.x + j * 256);
  }
  for (; t < ntiles; t += gridDim.x) {
    const size_t tn = t + gridDim.x;
    f32x4 w[U];
    if (tn < ntiles) {
#pragma unroll
      for (int j = 0; j < U; ++j) w[j] = __builtin_nontemporal_load(src + tn * kTile + threadIdx.x + j * 256);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) store16<SPOL>(dst + t * kTile + threadIdx.x + j * 256, v[j]);
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = w[j];
  }
  for (size_t i = ntiles * kTile + (size_t)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

}  // namespace k2x
}  // namespace ntm
