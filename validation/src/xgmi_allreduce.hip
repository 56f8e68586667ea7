// C ABI for C2, the hand-written xGMI all-reduce (see ntm/xgmi_allreduce.hpp).
#include "ntm/xgmi_allreduce.hpp"

#define NTM_API extern "C" __attribute__((visibility("default")))

// in_ptrs/out_ptrs/sig_ptrs: host arrays of `nranks` device pointers (peer-
// accessible from the launching device). Launches ranks rank_base ..
// rank_base + nranks_here - 1 on `stream` (nranks_here = nranks simulates the
// whole communicator on one device). `err` (device u32, zeroed by the caller)
// receives 1/2/3 if the entry / reduce-scatter / exit barrier timed out.
// count % (8*nranks) == 0. The barriers need every block of the launch
// resident at once: nranks_here * nblk <= 1024 (256 CUs x 4 blocks of 256
// threads, far below the CU limit). Two-shot may run in place (in_ptrs == out_ptrs);
// one-shot needs in != out. Every call on a communicator uses a fresh, larger
// epoch and the same nblk on all ranks. The kernel synchronises the ranks on
// the device (entry barrier), so callers need no host sync or host barrier.
// ntm_xgmi_allreduce_bf16_ex: the same with the barrier spin limits as
// arguments (0 = the defaults of xgmi_allreduce.hpp): a missing rank then
// times out in milliseconds (tests), and error code 1 / 2 poisons the owned
// output with NaN while 3 (exit barrier) leaves a complete result.
NTM_API int ntm_xgmi_allreduce_bf16_ex(const void* const* in_ptrs, void* const* out_ptrs,
                                       unsigned* const* sig_ptrs, int nranks, int rank_base,
                                       int nranks_here, int nblk, size_t count, unsigned epoch,
                                       unsigned* err, int one_shot, unsigned spin_limit,
                                       unsigned entry_spin_limit, void* stream) {
  using namespace ntm::xgmi;
  if (nranks < 1 || nranks > kMaxRanks || nranks_here < 1 || rank_base < 0 ||
      rank_base + nranks_here > nranks || nblk < 1 || nranks_here * nblk > 1024 || epoch == 0 ||
      count % (8 * (size_t)nranks) != 0 || !sig_ptrs || !err)
    return (int)hipErrorInvalidValue;
  if (one_shot)
    for (int r = 0; r < nranks; ++r)
      if (in_ptrs[r] == out_ptrs[r]) return (int)hipErrorInvalidValue;
  Peers p{};
  for (int r = 0; r < nranks; ++r) {
    p.in[r] = (const __bf16*)in_ptrs[r];
    p.out[r] = (__bf16*)out_ptrs[r];
    p.sig[r] = sig_ptrs[r];
  }
  const dim3 grid((unsigned)(nranks_here * nblk));
  const Limits lim{spin_limit ? spin_limit : kSpinLimit,
                   entry_spin_limit ? entry_spin_limit : kEntrySpinLimit};
  if (one_shot) {
    hipLaunchKernelGGL(allreduce_1shot_kernel, grid, dim3(kThreads), 0,
                       (hipStream_t)stream, p, nranks, rank_base, nblk, count, epoch, err, lim);
  } else {
    hipLaunchKernelGGL(allreduce_2shot_kernel, grid, dim3(kThreads), 0,
                       (hipStream_t)stream, p, nranks, rank_base, nblk, count,
                       epoch, err, lim);
  }
  return (int)hipGetLastError();
}

NTM_API int ntm_xgmi_allreduce_bf16(const void* const* in_ptrs, void* const* out_ptrs,
                                    unsigned* const* sig_ptrs, int nranks, int rank_base,
                                    int nranks_here, int nblk, size_t count, unsigned epoch,
                                    unsigned* err, int one_shot, void* stream) {
  return ntm_xgmi_allreduce_bf16_ex(in_ptrs, out_ptrs, sig_ptrs, nranks, rank_base, nranks_here,
                                    nblk, count, epoch, err, one_shot, 0u, 0u, stream);
}

NTM_API size_t ntm_xgmi_signal_bytes(int nblk) {
  return ntm::xgmi::signal_bytes(nblk);
}

// ---- buffers + IPC for the one-process-per-GPU path (torch.distributed):
// every rank allocates its in/out/signal buffers here, exchanges the 64-byte
// IPC handles (all_gather_object) and opens the peers' ones.
NTM_API int ntm_malloc(void** p, size_t bytes, int uncached) {
  return uncached ? (int)hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached)
                  : (int)hipMalloc(p, bytes);
}
NTM_API int ntm_free(void* p) { return (int)hipFree(p); }
NTM_API int ntm_memset_async(void* p, int v, size_t bytes, void* stream) {
  return (int)hipMemsetAsync(p, v, bytes, (hipStream_t)stream);
}
NTM_API int ntm_ipc_handle(void* p, void* out64) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e == hipSuccess) __builtin_memcpy(out64, &h, sizeof(h) < 64 ? sizeof(h) : 64);
  return (int)e;
}
NTM_API int ntm_ipc_open(const void* in64, void** p) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, in64, sizeof(h) < 64 ? sizeof(h) : 64);
  return (int)hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}
NTM_API int ntm_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }
NTM_API int ntm_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }
