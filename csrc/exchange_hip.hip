// mxstream — the row exchange of keyed operators whose rows are not the partition kernels'
// (key, ts, value) records (parallel/exchange.py exchange_rows: the median pane arena's
// (key id, ts, f64) rows at G > 1, ComputeCpuMiddle.java:34-48 keyed by host).
//
// Rows of several columns travel as ONE packed row (the columns' words back to back) in ONE
// equal-split all-to-all of fixed-capacity per-destination slices:
//  1. xrows_hist:    per-workgroup (1024 rows) per-destination counts in LDS;
//  2. xrows_scan:    one wave per destination scans the workgroup counts -> each workgroup's
//                    base in every destination slice, and the destination totals;
//  3. xrows_scatter: the stable position of a row inside its destination slice = workgroup base
//                    + rows of earlier waves (LDS) + lower lanes of its wave with the same
//                    destination (ballot); the row's words are copied into the slice;
//  4. (the all-to-all, torch.distributed / RCCL)
//  5. xrows_unpack:  received slices -> compacted columns in (source rank, source row) order.
// A row's order inside its destination is its order in the input, so every key's rows keep
// their arrival order (keep-first templates, order-sensitive folds).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "mxs_kernels.h"

namespace mxs {
namespace gpu {
namespace {

constexpr int kXBlock = 1024;     // rows per workgroup: 16 wave64
constexpr int kXWaves = kXBlock / 64;
constexpr int kXMaxWorld = 64;

#define XR_CHECK(x)                                                                   \
  do {                                                                                \
    const hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess)                                                             \
      throw std::runtime_error(std::string("exchange_rows: ") + hipGetErrorString(e_)); \
  } while (0)

__device__ __forceinline__ int xlane() { return (int)(threadIdx.x & 63u); }

__global__ __launch_bounds__(kXBlock) void xrows_hist_kernel(const int64_t* __restrict__ dest,
                                                             int64_t n, int world,
                                                             uint32_t* __restrict__ blk_cnt,
                                                             uint32_t* __restrict__ bad) {
  __shared__ uint32_t h[kXMaxWorld];
  if (threadIdx.x < (unsigned)world) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kXBlock + threadIdx.x;
  if (i < n) {
    const int64_t d = dest[i];
    if (d >= 0 && d < world) atomicAdd(&h[d], 1u);
    else atomicOr(bad, 1u);
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)world) blk_cnt[(size_t)blockIdx.x * world + threadIdx.x] = h[threadIdx.x];
}

// One wave per destination: exclusive scan of the workgroup counts (in place) + the total.
__global__ __launch_bounds__(1024) void xrows_scan_kernel(uint32_t* __restrict__ blk_cnt,
                                                          int64_t nblk, int world,
                                                          uint32_t* __restrict__ counts) {
  const int lane = xlane(), w = (int)(threadIdx.x >> 6), nw = (int)(blockDim.x >> 6);
  for (int d = w; d < world; d += nw) {
    uint32_t run = 0;
    for (int64_t b0 = 0; b0 < nblk; b0 += 64) {
      const int64_t b = b0 + lane;
      const uint32_t c = b < nblk ? blk_cnt[(size_t)b * world + d] : 0u;
      uint32_t incl = c;
      for (int s = 1; s < 64; s <<= 1) {
        const uint32_t y = __shfl_up(incl, s);
        if (lane >= s) incl += y;
      }
      if (b < nblk) blk_cnt[(size_t)b * world + d] = run + incl - c;
      run += __shfl(incl, 63);
    }
    if (lane == 0) counts[d] = run;
  }
}

__global__ __launch_bounds__(kXBlock) void xrows_scatter_kernel(
    const int64_t* __restrict__ dest, int64_t n, int world, const uint32_t* __restrict__ blk_off,
    uint32_t cap, XRowCols c, uint32_t* __restrict__ send, uint32_t* __restrict__ ovf) {
  __shared__ uint32_t wcnt[kXWaves][kXMaxWorld];
  const int lane = xlane(), w = (int)(threadIdx.x >> 6);
  const int64_t i = (int64_t)blockIdx.x * kXBlock + threadIdx.x;
  const int64_t dl = i < n ? dest[i] : -1;
  const int d = (dl >= 0 && dl < world) ? (int)dl : -1;
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint32_t rank = 0;
  for (int dd = 0; dd < world; ++dd) {
    const unsigned long long m = __ballot(d == dd);
    if (d == dd) rank = (uint32_t)__popcll(m & lt);
    if (lane == 0) wcnt[w][dd] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (d < 0) return;
  uint32_t pos = blk_off[(size_t)blockIdx.x * world + d] + rank;
  for (int v = 0; v < w; ++v) pos += wcnt[v][d];
  if (pos >= cap) {
    atomicOr(ovf, 1u);
    return;
  }
  uint32_t* row = send + ((size_t)d * cap + pos) * (size_t)c.rw;
  int o = 0;
  for (int k = 0; k < c.ncol; ++k) {
    const uint32_t* src = c.src[k] + (size_t)i * c.words[k];
    for (int j = 0; j < c.words[k]; ++j) row[o + j] = src[j];
    o += c.words[k];
  }
}

// Slot (s, idx) of the received buffer -> output row prefix(rc, s) + idx when idx < rc[s].
__global__ __launch_bounds__(256) void xrows_unpack_kernel(const uint32_t* __restrict__ recv,
                                                           const uint32_t* __restrict__ rc,
                                                           int world, uint32_t cap, XRowCols c) {
  __shared__ uint32_t pre[kXMaxWorld + 1];
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int s = 0; s < world; ++s) {
      pre[s] = t;
      t += rc[s] < cap ? rc[s] : cap;
    }
    pre[world] = t;
  }
  __syncthreads();
  const uint64_t total = (uint64_t)world * cap;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const int s = (int)(q / cap);
    const uint32_t idx = (uint32_t)(q - (uint64_t)s * cap);
    if (idx >= rc[s]) continue;
    const size_t orow = (size_t)pre[s] + idx;
    const uint32_t* row = recv + q * (uint64_t)c.rw;
    int o = 0;
    for (int k = 0; k < c.ncol; ++k) {
      uint32_t* dst = c.dst[k] + orow * c.words[k];
      for (int j = 0; j < c.words[k]; ++j) dst[j] = row[o + j];
      o += c.words[k];
    }
  }
}

}  // namespace

int64_t xrows_blocks(int64_t n) { return (n + kXBlock - 1) / kXBlock; }

void xrows_count(const int64_t* dest, int64_t n, int world, uint32_t* blk_cnt, uint32_t* counts,
                 uint32_t* bad, intptr_t stream) {
  if (world < 1 || world > kXMaxWorld) throw std::invalid_argument("exchange_rows: 1..64 ranks");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nblk = xrows_blocks(n);
  if (nblk == 0) {
    XR_CHECK(hipMemsetAsync(counts, 0, sizeof(uint32_t) * world, st));
    return;
  }
  hipLaunchKernelGGL(xrows_hist_kernel, dim3((unsigned)nblk), dim3(kXBlock), 0, st, dest, n, world,
                     blk_cnt, bad);
  const int threads = 64 * (world < 16 ? world : 16);
  hipLaunchKernelGGL(xrows_scan_kernel, dim3(1), dim3(threads), 0, st, blk_cnt, nblk, world,
                     counts);
  XR_CHECK(hipGetLastError());
}

void xrows_scatter(const int64_t* dest, int64_t n, int world, const uint32_t* blk_off,
                   uint32_t cap, const XRowCols& c, uint32_t* send, uint32_t* ovf,
                   intptr_t stream) {
  const int64_t nblk = xrows_blocks(n);
  if (nblk == 0) return;
  hipLaunchKernelGGL(xrows_scatter_kernel, dim3((unsigned)nblk), dim3(kXBlock), 0,
                     (hipStream_t)stream, dest, n, world, blk_off, cap, c, send, ovf);
  XR_CHECK(hipGetLastError());
}

void xrows_unpack(const uint32_t* recv, const uint32_t* rc, int world, uint32_t cap,
                  const XRowCols& c, intptr_t stream) {
  const uint64_t total = (uint64_t)world * cap;
  if (total == 0) return;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipLaunchKernelGGL(xrows_unpack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, recv,
                     rc, world, cap, c);
  XR_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
