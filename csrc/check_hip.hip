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

__global__ __launch_bounds__(256) void min_i64_kernel(const int64_t* __restrict__ x, int64_t n,
                                                      long long* __restrict__ out) {
  __shared__ long long red[4];
  long long m = INT64_MAX;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    m = x[i] < m ? x[i] : m;
  for (int o = 32; o > 0; o >>= 1) {
    const long long w = __shfl_xor(m, o);
    m = w < m ? w : m;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) m = red[w] < m ? red[w] : m;
    if (m != INT64_MAX) atomicMin(out, m);
  }
}

}  // namespace

namespace gpu {
void min_i64(const int64_t* x, int64_t n, int64_t* out, intptr_t stream) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(min_i64_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x,
                     n, (long long*)out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e));
}

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
