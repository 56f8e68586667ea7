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

// e4m3 operands for K1-fp8: the same uniform [-1, 1) stream, rounded to e4m3,
// 16 values (one 16-byte store) per lane per iteration.
__global__ void __launch_bounds__(256)
    fill_uniform_e4m3_kernel(uint8_t* __restrict__ out, size_t n, uint64_t seed, float scale) {
  const size_t nvec = n / 16;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t v = gid; v < nvec; v += stride) {
    typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));
    u8x16 o;
#pragma unroll
    for (int j = 0; j < 16; ++j) o[j] = f32_to_e4m3_bits(scale * uniform_pm1(seed, v * 16 + j));
    *(u8x16*)(out + v * 16) = o;
  }
  const size_t t0 = nvec * 16;
  if (t0 + gid < n) out[t0 + gid] = f32_to_e4m3_bits(scale * uniform_pm1(seed, t0 + gid));
}

// ------------------------------------------------- K3: fp32 reference GEMM
// Straightforward LDS-tiled fp32 FMA GEMM, C_ref = A * B^T. Independent of
// the MFMA path on purpose (different unit, different summation order) so a
// systematic error in K1 cannot cancel against its own reference.
constexpr int kRefTile = 32;

template <typename T>
__device__ __forceinline__ float ref_load(const T* p, size_t i);
template <>
__device__ __forceinline__ float ref_load<__bf16>(const __bf16* p, size_t i) {
  return bf16_bits_to_f32(((const uint16_t*)p)[i]);
}
template <>
__device__ __forceinline__ float ref_load<uint8_t>(const uint8_t* p, size_t i) {
  return e4m3_bits_to_f32(p[i]);  // e4m3 operands of K1-fp8
}

template <typename T>
__global__ void __launch_bounds__(256)
    ref_gemm_f32_kernel(const T* __restrict__ A, const T* __restrict__ B,
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
      As[r][tx] = (ga < M && gk < K) ? ref_load(A, (size_t)ga * lda + gk) : 0.f;
      Bs[r][tx] = (gb < N && gk < K) ? ref_load(B, (size_t)gb * ldb + gk) : 0.f;
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

// ------------------------------------------------- K3: ABFT row checksum
// Online check of a K1 GEMM in O(MK + NK + MN) instead of the O(MNK) fp32
// reference (Huang-Abraham checksums): since C = A B^T,
//   sum_n C[m,n] = sum_k A[m,k] * bsum[k],   bsum[k] = sum_n B[n,k].
// K1's epilogue accumulates rowsum[m] from its fp32 accumulators
// (gemm_bf16.hpp, kRowSum). Two comparisons per row, both scaled by the
// row's L2 norm ||C_m|| (the natural size of fp32 summation error):
//   acc   : |rowsum[m] - A_m . bsum|      <= 1e-3 + 2^-14 ||C_m||   (MFMA math)
//   store : |sum_n bf16(C[m,n]) - rowsum| <= 1e-3 + 2^-6  ||C_m||   (bf16 out)
// The store bound is ~8 sigma of independent round-to-nearest errors; it
// assumes rounding errors are uncorrelated (true for random operands).
struct AbftResult {
  unsigned long long bad_acc;
  unsigned long long bad_store;
  unsigned int max_rel_acc_bits;    // float bits of max err / ||C_m||
  unsigned int max_rel_store_bits;
};

// T: the operand type (__bf16 for K1, uint8_t = OCP e4m3 for K1-fp8).
template <typename T>
__global__ void __launch_bounds__(256)
    abft_colsum_kernel(const T* __restrict__ B, int N, int K, int ldb,
                       int rows_per_chunk, double* __restrict__ bsum) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const int n0 = blockIdx.y * rows_per_chunk;
  const int n1 = min(N, n0 + rows_per_chunk);
  double s = 0.0;
  for (int n = n0; n < n1; ++n) s += ref_load(B, (size_t)n * ldb + k);
  unsafeAtomicAdd(bsum + k, s);
}

__device__ __forceinline__ double block_sum_256(double v, double* s_tmp) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  return s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
}

__device__ __forceinline__ void atomic_max_nonneg(unsigned int* p, float v) {
  unsigned int bits;
  __builtin_memcpy(&bits, &v, 4);
  if (v != v) bits = 0x7fc00000u;
  atomicMax(p, bits);
}

template <typename T>
__global__ void __launch_bounds__(256)
    abft_row_check_kernel(const T* __restrict__ A, int lda,
                          const __bf16* __restrict__ C, int ldc,
                          const float* __restrict__ rowsum,
                          const double* __restrict__ bsum, int N, int K,
                          AbftResult* __restrict__ out) {
  __shared__ double s_tmp[4];
  const int m = blockIdx.x;
  const T* a = A + (size_t)m * lda;
  const uint16_t* c = (const uint16_t*)C + (size_t)m * ldc;
  double r = 0.0, sc = 0.0, ss = 0.0;
  for (int k = threadIdx.x; k < K; k += 256) r += ref_load(a, k) * bsum[k];
  for (int n = threadIdx.x; n < N; n += 256) {
    const double v = bf16_bits_to_f32(c[n]);
    sc += v;
    ss += v * v;
  }
  r = block_sum_256(r, s_tmp);
  sc = block_sum_256(sc, s_tmp);
  ss = block_sum_256(ss, s_tmp);
  if (threadIdx.x == 0) {
    const double norm = sqrt(ss);
    const double rs = (double)rowsum[m];
    const double e_acc = fabs(rs - r), e_st = fabs(sc - rs);
    // NaN-safe: !(e <= tol) flags NaN
    if (!(e_acc <= 1e-3 + 0x1p-14 * norm)) atomicAdd(&out->bad_acc, 1ull);
    if (!(e_st <= 1e-3 + 0x1p-6 * norm)) atomicAdd(&out->bad_store, 1ull);
    const double den = norm > 1e-30 ? norm : 1e-30;
    atomic_max_nonneg(&out->max_rel_acc_bits, (float)(e_acc / den));
    atomic_max_nonneg(&out->max_rel_store_bits, (float)(e_st / den));
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

// ---- K2 tuned: block-tiled stream, U independent 16-byte vectors in flight
// per lane, load/store cache policy chosen at compile time (0 = default,
// 1 = nontemporal). A block owns whole 256*U-vector tiles (one 4*U KiB
// contiguous span) and strides over tiles; the sub-tile tail is spread over
// the grid. Swept by tools/hbm_sweep.py; the C ABI default is the winner.
template <int P>
__device__ __forceinline__ f32x4 ld(const f32x4* p) {
  if constexpr (P == 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int P>
__device__ __forceinline__ void st(f32x4* p, f32x4 v) {
  if constexpr (P == 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int U, int LP, int SP>
__global__ void __launch_bounds__(256)
    stream_copy_tiled_kernel(const f32x4* __restrict__ src,
                             f32x4* __restrict__ dst, size_t n4) {
  constexpr size_t kTile = 256 * U;
  const size_t ntiles = n4 / kTile;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t base = t * kTile + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<LP>(src + base + j * 256);
#pragma unroll
    for (int j = 0; j < U; ++j) st<SP>(dst + base + j * 256, v[j]);
  }
  for (size_t i = ntiles * kTile + (size_t)blockIdx.x * 256 + threadIdx.x;
       i < n4; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

// Software-pipelined copy: tile t+grid's loads are in flight while tile t is
// stored, so the store stream never waits on a fresh load round trip.
template <int U, int LP, int SP>
__global__ void __launch_bounds__(256)
    stream_copy_pipe_kernel(const f32x4* __restrict__ src,
                            f32x4* __restrict__ dst, size_t n4) {
  constexpr size_t kTile = 256 * U;
  const size_t ntiles = n4 / kTile;
  size_t t = blockIdx.x;
  f32x4 v[U];
  if (t < ntiles) {
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<LP>(src + t * kTile + threadIdx.x + j * 256);
  }
  for (; t < ntiles; t += gridDim.x) {
    const size_t tn = t + gridDim.x;
    f32x4 w[U];
    if (tn < ntiles) {
#pragma unroll
      for (int j = 0; j < U; ++j) w[j] = ld<LP>(src + tn * kTile + threadIdx.x + j * 256);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) st<SP>(dst + t * kTile + threadIdx.x + j * 256, v[j]);
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = w[j];
  }
  for (size_t i = ntiles * kTile + (size_t)blockIdx.x * 256 + threadIdx.x;
       i < n4; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

// Chunked copy: block b owns one contiguous span of ceil(tiles / grid) tiles
// and walks it with the same one-tile-ahead software pipeline, so each CU
// streams through its own DRAM pages instead of all CUs marching through the
// same region (the tiled kernels above).
template <int U, int LP, int SP>
__global__ void __launch_bounds__(256)
    stream_copy_chunk_kernel(const f32x4* __restrict__ src,
                             f32x4* __restrict__ dst, size_t n4) {
  constexpr size_t kTile = 256 * U;
  const size_t ntiles = n4 / kTile;
  const size_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  size_t t = (size_t)blockIdx.x * per;
  const size_t end = t + per < ntiles ? t + per : ntiles;
  f32x4 v[U];
  if (t < end) {
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<LP>(src + t * kTile + threadIdx.x + j * 256);
  }
  for (; t < end; ++t) {
    f32x4 w[U];
    if (t + 1 < end) {
#pragma unroll
      for (int j = 0; j < U; ++j) w[j] = ld<LP>(src + (t + 1) * kTile + threadIdx.x + j * 256);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) st<SP>(dst + t * kTile + threadIdx.x + j * 256, v[j]);
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = w[j];
  }
  for (size_t i = ntiles * kTile + (size_t)blockIdx.x * 256 + threadIdx.x;
       i < n4; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

template <int U, int LP>
__global__ void __launch_bounds__(256)
    stream_read_tiled_kernel(const f32x4* __restrict__ src, size_t n4,
                             float* __restrict__ sink) {
  constexpr size_t kTile = 256 * U;
  const size_t ntiles = n4 / kTile;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t base = t * kTile + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<LP>(src + base + j * 256);
#pragma unroll
    for (int j = 0; j < U; ++j) acc += v[j];
  }
  for (size_t i = ntiles * kTile + (size_t)blockIdx.x * 256 + threadIdx.x;
       i < n4; i += (size_t)gridDim.x * 256)
    acc += src[i];
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s != s || s == __builtin_huge_valf()) sink[blockIdx.x] = s;
}

// Clock probe: the shader clock a GPU holds under a dense MFMA load, for
// telling a power- or thermally-limited GPU apart from a slow one in a
// multi-GPU run (bench.py per_rank_clock_GHz). Each wave runs `iters` x 8
// back-to-back v_mfma_f32_16x16x32_bf16 on random operands (the clock depends
// on the data: MI355X_MICROARCH.md "DVFS give-back" items 1, 6) and records
// Delta s_memtime (shader cycles) and Delta s_memrealtime (100 MHz ticks):
// clock = cycles / ticks * 0.1 GHz. One block of 4 waves per CU loads every
// SIMD. out: 2 u64 per wave; sink: one float nobody reads (keeps the MFMAs).
__global__ void __launch_bounds__(256) clock_probe_kernel(int iters, unsigned seed,
                                                          unsigned long long* out, float* sink) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  i32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // bf16 pairs with small exponents: random mantissas, no inf / nan
    const unsigned h = (unsigned)mix64(((unsigned long long)seed << 32) ^ (lane * 8 + i));
    a[i] = (int)(h & 0x3F7F3F7Fu);
    b[i] = (int)((h >> 5) & 0x3F7F3F7Fu);
  }
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
  }
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // MFMA results land before VALU reads
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (s == 12345.678f) sink[0] = s;
  if (lane == 0) {
    const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = r1 - r0;
  }
}

}  // namespace aux
}  // namespace ntm
