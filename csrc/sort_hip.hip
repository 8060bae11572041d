// mxstream — device radix sort of (64-bit key, 64-bit value) pairs over a bit range.
//
// The keyed-state passes (rolling, sessions) order a step's records by (slot, arrival or event
// time). torch.sort sorts all 64 key bits and returns a permutation that the scan kernels then
// gather through (a random 8-byte read per record); sorting the value column along with the key
// and only over the bits that are in use (slot bits + time bits: ~35 instead of 64) removes both
// costs. rocPRIM's onesweep radix sort is the library primitive here.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdexcept>
#include <string>

#include "mxs_kernels.h"

namespace mxs {
namespace gpu {

size_t sort_pairs_temp_bytes(int64_t n, int begin_bit, int end_bit) {
  size_t bytes = 0;
  const hipError_t e = rocprim::radix_sort_pairs(
      nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint64_t*)nullptr,
      (uint64_t*)nullptr, (size_t)n, (unsigned)begin_bit, (unsigned)end_bit);
  if (e != hipSuccess) throw std::runtime_error(std::string("radix sort size: ") + hipGetErrorString(e));
  return bytes;
}

void sort_pairs(void* temp, size_t temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                const uint64_t* vals_in, uint64_t* vals_out, int64_t n, int begin_bit, int end_bit,
                intptr_t stream) {
  if (n <= 0) return;
  size_t need = sort_pairs_temp_bytes(n, begin_bit, end_bit);
  if (need > temp_bytes) throw std::runtime_error("sort_pairs: temporary buffer too small");
  const hipError_t e = rocprim::radix_sort_pairs(temp, need, keys_in, keys_out, vals_in, vals_out,
                                                 (size_t)n, (unsigned)begin_bit, (unsigned)end_bit,
                                                 (hipStream_t)stream);
  if (e != hipSuccess) throw std::runtime_error(std::string("radix sort: ") + hipGetErrorString(e));
}

}  // namespace gpu
}  // namespace mxs
