// Shared device/host helpers for the MI355X (gfx950, CDNA4) validation kernels.
//
// Reference parity: the reference repository ships no kernels at all; its GPU
// check is delegated to the NVIDIA GPU Operator validator pulled by
// helm_release.gpu_operator (/root/reference/eks/main.tf:185-203). These
// headers are the MI355X-native replacement.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

namespace ntm {

// 64-lane wavefronts on CDNA: never 32.
constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

#define NTM_AS1 __attribute__((address_space(1)))
#define NTM_AS3 __attribute__((address_space(3)))

// Round-to-nearest-even f32 -> bf16 bits. NaN is kept a NaN (quiet) so a
// corrupted accumulator can never masquerade as a finite value in the
// validation check (MI355X_MICROARCH.md §Correctness boundaries).
__host__ __device__ inline uint16_t f32_to_bf16_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__host__ __device__ inline float bf16_bits_to_f32(uint16_t h) {
  uint32_t u = ((uint32_t)h) << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

// OCP e4m3 ("fn": no infinities, S.1111.111 is NaN, max 448) <-> f32.
// Round-to-nearest-even with saturation to +-448, matching torch's
// float8_e4m3fn conversion (tests/test_kernels_gpu.py pins the equality).
__host__ __device__ inline uint8_t f32_to_e4m3_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 24) & 0x80u;
  u &= 0x7fffffffu;
  if (u > 0x7f800000u) return (uint8_t)(sign | 0x7f);  // NaN
  float a;
  __builtin_memcpy(&a, &u, 4);
  uint32_t code;
  const int E = (int)(u >> 23) - 127;
  if (E < -6) {  // subnormal range: units of 2^-9, RNE (code 8 == smallest normal)
    const float q = a * 512.0f;
    uint32_t m = (uint32_t)q;
    const float rem = q - (float)m;
    if (rem > 0.5f || (rem == 0.5f && (m & 1u))) ++m;
    code = m;
  } else {
    uint32_t r = (u & 0x7fffffu) >> 20;
    const uint32_t rem = u & 0xfffffu, half = 0x80000u;
    if (rem > half || (rem == half && (r & 1u))) ++r;
    int e = E + 7;
    if (r == 8) {
      r = 0;
      ++e;
    }
    if (e > 15 || (e == 15 && r == 7)) {  // saturate to 448 = S.1111.110
      e = 15;
      r = 6;
    }
    code = ((uint32_t)e << 3) | r;
  }
  return (uint8_t)(sign | code);
}

__host__ __device__ inline float e4m3_bits_to_f32(uint8_t v) {
  const int e = (v >> 3) & 0xf, m = v & 7;
  float f;
  if (e == 0xf && m == 7) {
    uint32_t q = 0x7fc00000u;
    __builtin_memcpy(&f, &q, 4);
    return f;
  }
  if (e == 0)
    f = (float)m * (1.0f / 512.0f);
  else
    f = (1.0f + (float)m * 0.125f) * __builtin_ldexpf(1.0f, e - 7);
  return (v & 0x80) ? -f : f;
}

// The XCD (XCC) this wave runs on, read from the hardware register (not
// inferred from blockIdx: the dispatcher's round robin is a convention, which
// compute partition modes change). Raw register; the id is its low 4 bits.
__device__ __forceinline__ unsigned xcc_id_raw() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v;
}

__device__ __forceinline__ unsigned xcc_id() { return xcc_id_raw() & 0xFu; }

// Stateless counter-based hash (splitmix64 finaliser). Used for the
// synthetic uniform [-1, 1) operands so every rank / run is reproducible
// from (seed, index) without any host->device copy.
__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__host__ __device__ inline float uniform_pm1(uint64_t seed, uint64_t idx) {
  uint64_t h = mix64(seed * 0x100000001B3ull ^ mix64(idx));
  // 24 random mantissa bits -> [0,1) -> [-1,1)
  float u = (float)(h >> 40) * (1.0f / 16777216.0f);
  return 2.0f * u - 1.0f;
}

}  // namespace ntm

#define NTM_HIP_CHECK(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      std::fprintf(stderr, "HIP error %s at %s:%d: %s\n", #expr, __FILE__,    \
                   __LINE__, hipGetErrorString(_e));                          \
      return (int)_e;                                                         \
    }                                                                         \
  } while (0)
