// C2: hand-written peer-to-peer all-reduce (sum, bf16) over the xGMI mesh.
//
// "peer-access one-shot all-reduce for <= 1 MiB and
// two-shot (reduce-scatter + all-gather over all 7 xGMI links) for large
// messages, compared against RCCL". The reference has no collective code
// (grep -> 0 hits); this is an MI355X-first design.
//
// Why: an 8x MI355X node is a FULL mesh (7 links x ~153 GB/s per GPU). A ring
// moves every chunk over one link per hop; a direct two-shot lets every GPU
// use all 7 links at once: reduce-scatter (rank r sums chunk r reading it
// from all peers) then all-gather (rank r copies chunk q from peer q), each
// link carrying 2S/N bytes -> theoretical busbw ~ 7 x 153 GB/s.
//
// Ranks are addressed through peer pointers (single process + hipDevice-
// EnablePeerAccess, or IPC-opened handles). The same kernel also runs all
// N "ranks" on ONE device (rank = blockIdx.x / blocks_per_rank) - that is how
// the protocol is tested on a single GPU.
//
// Synchronisation (cdna_hip_programming.md §6 Guideline 16, system scope):
//   block (r, b) stores its slice -> every storing wave s_waitcnt vmcnt(0) ->
//   __syncthreads -> lane 0: release fence (system) -> asm vmcnt(0) -> flag
//   store (system scope) into EVERY peer's signal slot [phase][r][b];
//   then block (r, b) polls its own slots [phase][q][b] for all q (relaxed,
//   bounded spin + s_sleep), ONE acquire fence (system), __syncthreads, reads.
// A block only ever waits for the block with the SAME index on the other
// ranks, so no intra-device grid barrier is needed; every spin is bounded and
// reports a timeout code instead of hanging.
//
// Three barriers per call, on per-phase epoch slots:
//   phase 0 (entry): "my input for this epoch is in place" - the kernel is
//     stream-ordered after this rank's producer, so passing the entry barrier
//     means every peer's input is complete. No host sync / host barrier.
//   phase 1: reduce-scatter done (slice b of my chunk is final).
//   phase 2 (exit): all-gather done - nobody's buffer is read any more, so the
//     caller may overwrite its input right after the kernel.
// Epochs only grow and a rank can reach phase p of epoch e+1 only after every
// peer signalled phase 2 of epoch e, so a waiter never misses a value; the
// wait is `slot >= epoch` (robust to a peer that already moved on).
// With the three barriers the two-shot runs IN PLACE (in == out): phase-1
// writes only touch slices no peer reads before the next barrier.
#pragma once

#include "ntm/common.hpp"

namespace ntm {
namespace xgmi {

constexpr int kMaxRanks = 8;
constexpr int kThreads = 256;
constexpr int kPhases = 3;                 // entry, reduce-scatter done, exit
// Default spin limits (s_sleep 2 + one uncached load per spin). The ENTRY
// barrier absorbs host-side skew between ranks (a checkpoint, a GC pause,
// uneven work before the call): it waits 16x longer (~minutes) than the
// in-kernel phases, which only wait for peers already running the same kernel
// (~seconds). Both are kernel arguments (0 = these defaults), so a test can
// time a missing rank out in milliseconds.
constexpr unsigned kSpinLimit = 1u << 24;
constexpr unsigned kEntrySpinLimit = 1u << 28;

struct Limits {
  unsigned spin;   // reduce-scatter / exit barriers
  unsigned entry;  // entry barrier
};
// A block whose barrier times out never leaves a stale sum behind: it fills
// the part of the output it owns with bf16 NaN (0x7FC0), so a caller that does
// not read the error word still cannot consume partial sums silently.
constexpr unsigned short kPoison = 0x7FC0;

struct Peers {
  const __bf16* in[kMaxRanks];
  __bf16* out[kMaxRanks];
  unsigned* sig[kMaxRanks];  // per rank: [kPhases][kMaxRanks][blocks] u32
};

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void add8(float (&acc)[8], const u16x8 v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] += bf16_bits_to_f32(v[i]);
}

__device__ __forceinline__ u16x8 pack8(const float (&acc)[8]) {
  u16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32_to_bf16_bits(acc[i]);
  return o;
}

// publish "block b of rank r finished phase ph" to every rank, then wait for
// the same block index of every rank. Returns false on timeout.
__device__ __forceinline__ bool cross_rank_barrier(const Peers& p, int nranks,
                                                   int rank, int b, int nblk,
                                                   int ph, unsigned epoch,
                                                   unsigned* err,
                                                   unsigned limit = kSpinLimit) {
  __shared__ int s_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int q = 0; q < nranks; ++q) {
      unsigned* slot = p.sig[q] + ((size_t)ph * kMaxRanks + rank) * nblk + b;
      __hip_atomic_store(slot, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (int q = 0; q < nranks && ok; ++q) {
      unsigned* mine = p.sig[rank] + ((size_t)ph * kMaxRanks + q) * nblk + b;
      unsigned spins = 0;
      while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > limit) {
          ok = false;
          atomicMax(err, 1u + (unsigned)ph);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return s_ok != 0;
}

// Two-shot all-reduce of `count` bf16 elements (count % (8 * nranks) == 0).
// grid = nranks_here * nblk blocks; rank = rank_base + blockIdx.x / nblk.
__global__ void __launch_bounds__(kThreads)
    allreduce_2shot_kernel(Peers p, int nranks, int rank_base, int nblk,
                           size_t count, unsigned epoch, unsigned* err, Limits lim) {
  const int rank = rank_base + (int)(blockIdx.x / nblk);
  const int b = (int)(blockIdx.x % nblk);
  const size_t chunk = count / nranks;        // elements per rank chunk
  const size_t nvec = chunk / 8;              // 16-byte vectors per chunk
  const size_t per_blk = (nvec + nblk - 1) / nblk;
  const size_t v0 = (size_t)b * per_blk;
  const size_t v1 = v0 + per_blk < nvec ? v0 + per_blk : nvec;
  const size_t base = (size_t)rank * chunk / 8;  // vector index of chunk `rank`

  // slice b of every chunk of my output: what this block writes (phase 1
  // writes chunk `rank`, phase 2 the others) - poisoned on a timeout
  auto poison = [&]() {
    u16x8 nan8;
#pragma unroll
    for (int i = 0; i < 8; ++i) nan8[i] = kPoison;
    for (int q = 0; q < nranks; ++q)
      for (size_t v = v0 + threadIdx.x; v < v1; v += kThreads)
        ((u16x8*)p.out[rank])[(size_t)q * chunk / 8 + v] = nan8;
  };
  // phase 0 (entry): every peer's input for this epoch is complete
  if (!cross_rank_barrier(p, nranks, rank, b, nblk, 0, epoch, err, lim.entry)) {
    poison();
    return;
  }

  // reduce-scatter - chunk `rank`, slice b, summed over all ranks. Start the
  // sum at a different peer per rank so the 7 links carry load at once.
  for (size_t v = v0 + threadIdx.x; v < v1; v += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int qq = 0; qq < nranks; ++qq) {
      const int q = (rank + qq) % nranks;
      add8(acc, ((const u16x8*)p.in[q])[base + v]);
    }
    ((u16x8*)p.out[rank])[base + v] = pack8(acc);
  }
  if (!cross_rank_barrier(p, nranks, rank, b, nblk, 1, epoch, err, lim.spin)) {
    poison();
    return;
  }

  // all-gather - copy chunk q, slice b, from rank q's output
  for (int qq = 1; qq < nranks; ++qq) {
    const int q = (rank + qq) % nranks;  // stagger peers -> all links busy
    const size_t qb = (size_t)q * chunk / 8;
    for (size_t v = v0 + threadIdx.x; v < v1; v += kThreads)
      ((u16x8*)p.out[rank])[qb + v] = ((const u16x8*)p.out[q])[qb + v];
  }
  // phase 2 (exit): nobody may overwrite its buffers before all peers copied.
  // A timeout here leaves a COMPLETE output (error code 3): only the buffers
  // may still be read by a late peer, so nothing is poisoned.
  cross_rank_barrier(p, nranks, rank, b, nblk, 2, epoch, err, lim.spin);
}

// One-shot all-reduce (small messages): every rank reads ALL of every peer's
// input and writes its full output (in != out). Entry barrier: peers' inputs
// are complete; exit barrier: no peer still reads my input when I return.
__global__ void __launch_bounds__(kThreads)
    allreduce_1shot_kernel(Peers p, int nranks, int rank_base, int nblk,
                           size_t count, unsigned epoch, unsigned* err, Limits lim) {
  const int rank = rank_base + (int)(blockIdx.x / nblk);
  const int b = (int)(blockIdx.x % nblk);
  const size_t nvec = count / 8;
  if (!cross_rank_barrier(p, nranks, rank, b, nblk, 0, epoch, err, lim.entry)) {
    u16x8 nan8;
#pragma unroll
    for (int i = 0; i < 8; ++i) nan8[i] = kPoison;
    for (size_t v = (size_t)b * kThreads + threadIdx.x; v < nvec; v += (size_t)nblk * kThreads)
      ((u16x8*)p.out[rank])[v] = nan8;
    return;
  }
  for (size_t v = (size_t)b * kThreads + threadIdx.x; v < nvec;
       v += (size_t)nblk * kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int q = 0; q < nranks; ++q) add8(acc, ((const u16x8*)p.in[q])[v]);
    ((u16x8*)p.out[rank])[v] = pack8(acc);
  }
  cross_rank_barrier(p, nranks, rank, b, nblk, 2, epoch, err, lim.spin);
}

// bytes of one rank's signal area for `nblk` blocks per rank
inline size_t signal_bytes(int nblk) {
  return (size_t)kPhases * kMaxRanks * nblk * sizeof(unsigned);
}

}  // namespace xgmi
}  // namespace ntm
