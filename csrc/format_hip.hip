// mxstream — gfx950 row formatter for print() sinks (csrc/row_format.h has the text rules).
//
// Two kernels around a device scan:
//  * fmt_len_kernel: one lane per row computes the row's byte length and flags rows the device
//    cannot format (the caller then formats that batch on the host);
//  * fmt_write_kernel: a 256-row workgroup writes its rows -- one contiguous byte range of the
//    output, [end[i0 - 1], end[i1 - 1]) -- into LDS, then stores the range with aligned 16-byte
//    vector stores (byte-wise row writes from 64 lanes ~30 bytes apart would touch every cache
//    line of the range once per byte). Ranges beyond the LDS budget write straight to HBM.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "mxs_kernels.h"
#include "row_format.h"

namespace mxs {
namespace {

constexpr int kFmtBlock = 256;
constexpr int kFmtLds = 32 * 1024;  // ~128 bytes a row; typical rows are 20-60 bytes

#define FMT_CHECK(x)                                                                   \
  do {                                                                                 \
    const hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess)                                                              \
      throw std::runtime_error(std::string("format: ") + hipGetErrorString(e_));      \
  } while (0)

__global__ __launch_bounds__(kFmtBlock) void fmt_len_kernel(FmtArgs a, int64_t n,
                                                            int64_t* __restrict__ len,
                                                            uint32_t* __restrict__ bad) {
  bool all_ok = true;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    bool ok = true;
    len[i] = fmt_row(a, i, nullptr, ok);
    all_ok = all_ok && ok;
  }
  if (__any(!all_ok) && __lane_id() == 0) atomicOr(bad, 1u);
}

__global__ __launch_bounds__(kFmtBlock) void fmt_write_kernel(FmtArgs a, int64_t n,
                                                              const int64_t* __restrict__ end,
                                                              char* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char buf[kFmtLds + 16];
  const int64_t i0 = (int64_t)blockIdx.x * kFmtBlock;
  if (i0 >= n) return;
  const int64_t i1 = i0 + kFmtBlock < n ? i0 + kFmtBlock : n;
  const int64_t lo = i0 ? end[i0 - 1] : 0, hi = end[i1 - 1];
  const int64_t i = i0 + threadIdx.x;
  const int pad = (int)((uintptr_t)(out + lo) & 15);
  bool ok = true;
  if (hi - lo + pad > kFmtLds) {  // long rows: straight to HBM
    if (i < i1) fmt_row(a, i, out + (i ? end[i - 1] : 0), ok);
    return;
  }
  if (i < i1) fmt_row(a, i, buf + pad + ((i ? end[i - 1] : 0) - lo), ok);
  __syncthreads();
  // [lo, hi) from buf + pad: unaligned head and tail bytes singly, the body as uint4
  const int64_t nb = hi - lo;
  int head = (16 - pad) & 15;
  if (head > nb) head = (int)nb;
  const int64_t nbody = (nb - head) >> 4;
  const int64_t tail0 = head + (nbody << 4);
  if (threadIdx.x < head) out[lo + threadIdx.x] = buf[pad + threadIdx.x];
  const uint4* s4 = reinterpret_cast<const uint4*>(buf + pad + head);  // buf + 16: aligned
  uint4* d4 = reinterpret_cast<uint4*>(out + lo + head);
  for (int64_t k = threadIdx.x; k < nbody; k += kFmtBlock) d4[k] = s4[k];
  if (threadIdx.x < nb - tail0) out[lo + tail0 + threadIdx.x] = buf[pad + tail0 + threadIdx.x];
}

}  // namespace

namespace gpu {

void format_rows_len(const FmtArgs& a, int64_t n, int64_t* len, uint32_t* bad, intptr_t stream) {
  if (n <= 0) return;
  if (a.ncols < 1 || a.ncols > kFmtMaxCols) throw std::invalid_argument("format: column count");
  int64_t g = (n + kFmtBlock - 1) / kFmtBlock;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(fmt_len_kernel, dim3((unsigned)g), dim3(kFmtBlock), 0, (hipStream_t)stream,
                     a, n, len, bad);
  FMT_CHECK(hipGetLastError());
}

void format_rows_write(const FmtArgs& a, int64_t n, const int64_t* end, char* out,
                       intptr_t stream) {
  if (n <= 0) return;
  if (a.ncols < 1 || a.ncols > kFmtMaxCols) throw std::invalid_argument("format: column count");
  const int64_t g = (n + kFmtBlock - 1) / kFmtBlock;  // one workgroup per 256-row tile
  if (g > 0x7FFFFFFF) throw std::invalid_argument("format: too many rows");
  hipLaunchKernelGGL(fmt_write_kernel, dim3((unsigned)g), dim3(kFmtBlock), 0,
                     (hipStream_t)stream, a, n, end, out);
  FMT_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
