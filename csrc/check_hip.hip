// mxstream — keyed-state invariant checker on gfx950 (rules in mxs_check.h). One 256-thread
// workgroup per sub-table; per-workgroup counts reduced with wave ballots, one atomic per counter
// per workgroup. Used by tests and by MXS_DEBUG runs after every step.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "mxs_check.h"

namespace mxs {
namespace {

__global__ __launch_bounds__(256) void check_table_kernel(const uint64_t* __restrict__ keys_g,
                                                          int nsub_log2, int cap_log2,
                                                          unsigned long long* __restrict__ stats) {
  __shared__ unsigned long long red[kChkN];
  const uint32_t sub = blockIdx.x;
  const uint32_t cap = 1u << cap_log2, mask = cap - 1;
  const uint64_t* keys = keys_g + ((size_t)sub << cap_log2);
  if (threadIdx.x < kChkN) red[threadIdx.x] = 0;
  __syncthreads();
  uint32_t live = 0, mis = 0, chain = 0, dup = 0;
  for (uint32_t s = threadIdx.x; s < cap; s += blockDim.x) {
    const uint64_t k = keys[s];
    if (k == kEmptyKey || k == kTombKey) continue;
    ++live;
    const uint32_t bad = check_slot(keys, s, mask, nsub_log2, sub);
    mis += bad & 1u;
    chain += (bad >> 1) & 1u;
    dup += (bad >> 2) & 1u;
  }
  atomicAdd(&red[kChkLive], (unsigned long long)live);
  if (mis) atomicAdd(&red[kChkMisplaced], (unsigned long long)mis);
  if (chain) atomicAdd(&red[kChkBrokenChain], (unsigned long long)chain);
  if (dup) atomicAdd(&red[kChkDuplicate], (unsigned long long)dup);
  __syncthreads();
  if (threadIdx.x < kChkN && red[threadIdx.x]) atomicAdd(&stats[threadIdx.x], red[threadIdx.x]);
}

}  // namespace

namespace gpu {
void check_table(const uint64_t* keys_g, int nsub, int nsub_log2, int cap_log2, uint64_t* stats,
                 intptr_t stream) {
  if (nsub <= 0) return;
  if (cap_log2 < 1 || cap_log2 > 20) throw std::invalid_argument("check_table: bad cap_log2");
  hipLaunchKernelGGL(check_table_kernel, dim3(nsub), dim3(256), 0, (hipStream_t)stream, keys_g,
                     nsub_log2, cap_log2, (unsigned long long*)stats);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e));
}
}  // namespace gpu
}  // namespace mxs
