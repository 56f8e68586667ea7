// K2 (HBM stream) and K3 (fill / reference / verify) kernels for the
// validation Job. SURVEY.md §2.7: "K2: HBM stream/copy (float4, >= 6 TB/s
// target) to check memory. K3: fill/verify kernels: random uniform [-1,1)
// init and tolerance check vs an fp32 reference".
//
// No reference counterpart exists (the reference installs the NVIDIA
// operator, /root/reference/eks/main.tf:185-203, whose validator image is
// outside the repo); these are MI355X-first designs.
#pragma once

#include "ntm/common.hpp"

namespace ntm {
namespace aux {

// ---------------------------------------------------------------- K3: fill
// 8 bf16 per lane per iteration (16-byte stores, playbook Guideline 13).
__global__ void __launch_bounds__(256)
    fill_uniform_bf16_kernel(__bf16* __restrict__ out, size_t n, uint64_t seed,
                             float scale) {
  const size_t nvec = n / 8;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec;
       v += stride) {
    typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = f32_to_bf16_bits(scale * uniform_pm1(seed, v * 8 + j));
    *(u16x8*)(out + v * 8) = o;
  }
  // tail
  const size_t t0 = nvec * 8;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t0 + gid < n) {
    uint16_t h = f32_to_bf16_bits(scale * uniform_pm1(seed, t0 + gid));
    ((uint16_t*)out)[t0 + gid] = h;
  }
}

// ------------------------------------------------- K3: fp32 reference GEMM
// Straightforward LDS-tiled fp32 FMA GEMM, C_ref = A * B^T. Independent of
// the MFMA path on purpose (different unit, different summation order) so a
// systematic error in K1 cannot cancel against its own reference.
constexpr int kRefTile = 32;
__global__ void __launch_bounds__(256)
    ref_gemm_f32_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                        float* __restrict__ C, int M, int N, int K, int lda,
                        int ldb, int ldc) {
  __shared__ float As[kRefTile][kRefTile + 1];
  __shared__ float Bs[kRefTile][kRefTile + 1];
  const int tx = threadIdx.x & 31;       // column in tile
  const int ty = threadIdx.x >> 5;       // 0..7, 4 rows each
  const int row0 = blockIdx.y * kRefTile;
  const int col0 = blockIdx.x * kRefTile;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += kRefTile) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = ty * 4 + i;
      const int ga = row0 + r, gb = col0 + r, gk = k0 + tx;
      As[r][tx] = (ga < M && gk < K)
                      ? bf16_bits_to_f32(((const uint16_t*)A)[(size_t)ga * lda + gk])
                      : 0.f;
      Bs[r][tx] = (gb < N && gk < K)
                      ? bf16_bits_to_f32(((const uint16_t*)B)[(size_t)gb * ldb + gk])
                      : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < kRefTile; ++kk) {
      const float b = Bs[tx][kk];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = fmaf(As[ty * 4 + i][kk], b, acc[i]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = row0 + ty * 4 + i, cidx = col0 + tx;
    if (r < M && cidx < N) C[(size_t)r * ldc + cidx] = acc[i];
  }
}

// ------------------------------------------------------- K3: verification
// Per element: |c - ref| <= atol + rtol * |ref|. Accumulates the count of
// violations, the max abs error (as ordered uint bits) and the sum of
// squared errors. 2 atomics per block.
struct VerifyResult {
  unsigned long long bad;
  unsigned int max_err_bits;  // float bits, non-negative -> orderable
  unsigned int pad;
  double sum_sq_err;
  double sum_sq_ref;
};

__global__ void __launch_bounds__(256)
    verify_bf16_kernel(const __bf16* __restrict__ C, const float* __restrict__ R,
                       size_t n, float atol, float rtol,
                       VerifyResult* __restrict__ out) {
  __shared__ unsigned long long s_bad[4];
  __shared__ float s_max[4];
  __shared__ double s_e[4], s_r[4];
  unsigned long long bad = 0;
  float mx = 0.f;
  double se = 0.0, sr = 0.0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const float c = bf16_bits_to_f32(((const uint16_t*)C)[i]);
    const float r = R[i];
    const float e = fabsf(c - r);
    // NaN-safe: !(e <= tol) counts NaN as bad
    if (!(e <= atol + rtol * fabsf(r))) ++bad;
    mx = (e > mx || e != e) ? e : mx;
    se += (double)e * e;
    sr += (double)r * r;
  }
  // wave reduce (64 lanes)
  for (int o = 32; o > 0; o >>= 1) {
    bad += __shfl_xor(bad, o);
    const float om = __shfl_xor(mx, o);
    mx = (om > mx || om != om) ? om : mx;
    se += __shfl_xor(se, o);
    sr += __shfl_xor(sr, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_bad[w] = bad;
    s_max[w] = mx;
    s_e[w] = se;
    s_r[w] = sr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      bad += s_bad[i];
      mx = (s_max[i] > mx || s_max[i] != s_max[i]) ? s_max[i] : mx;
      se += s_e[i];
      sr += s_r[i];
    }
    atomicAdd(&out->bad, bad);
    unsigned int bits;
    __builtin_memcpy(&bits, &mx, 4);
    if (mx != mx) bits = 0x7fc00000u;
    atomicMax(&out->max_err_bits, bits);
    atomicAdd(&out->sum_sq_err, se);
    atomicAdd(&out->sum_sq_ref, sr);
  }
}

// ------------------------------------------------------------ K2: stream
// float4 copy, grid-stride, 16 B / lane (1 KiB per wave-instruction). Sized
// by the host to 256 CUs x 8 blocks (playbook Guideline 11).
__global__ void __launch_bounds__(256)
    stream_copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                       size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  // 4 independent loads in flight per lane
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const f32x4 a = __builtin_nontemporal_load(src + i);
    const f32x4 b = __builtin_nontemporal_load(src + i + stride);
    const f32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    const f32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n4; i += stride) dst[i] = src[i];
}

// Read-only stream with a reduction so nothing is dead-code eliminated.
__global__ void __launch_bounds__(256)
    stream_read_kernel(const f32x4* __restrict__ src, size_t n4,
                       float* __restrict__ sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const f32x4 a = __builtin_nontemporal_load(src + i);
    const f32x4 b = __builtin_nontemporal_load(src + i + stride);
    const f32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    const f32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    acc.x += a.x + b.x + c.x + d.x;
    acc.y += a.y + b.y + c.y + d.y;
    acc.z += a.z + b.z + c.z + d.z;
    acc.w += a.w + b.w + c.w + d.w;
  }
  for (; i < n4; i += stride) {
    const f32x4 a = src[i];
    acc.x += a.x;
    acc.y += a.y;
    acc.z += a.z;
    acc.w += a.w;
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  // only a NaN/inf can make this store happen; keeps the loads live
  if (s != s || s == __builtin_huge_valf()) sink[blockIdx.x] = s;
}

}  // namespace aux
}  // namespace ntm
