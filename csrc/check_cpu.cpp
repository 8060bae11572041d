// mxstream — bindings of the keyed-state invariant checker (rules and C++ twin in mxs_check.h,
// GPU kernel in check_hip.hip).
#include <pybind11/pybind11.h>

#include <cstring>
#include <stdexcept>

#include "mxs_check.h"
#include "mxs_runtime.h"

void bind_check(pybind11::module_& m) {
  using namespace mxs;
  m.def("gpu_check_table", [](intptr_t keys, int nsub, int nsub_log2, int cap_log2, intptr_t stats,
                              intptr_t stream) {
    gpu::check_table(reinterpret_cast<const uint64_t*>(keys), nsub, nsub_log2, cap_log2,
                     reinterpret_cast<uint64_t*>(stats), stream);
  });
  m.def("cpu_check_table", [](intptr_t keys, int nsub, int nsub_log2, int cap_log2, intptr_t stats) {
    if (cap_log2 < 1 || cap_log2 > 20) throw std::invalid_argument("check_table: bad cap_log2");
    cpu::check_table(reinterpret_cast<const uint64_t*>(keys), nsub, nsub_log2, cap_log2,
                     reinterpret_cast<uint64_t*>(stats));
  });
}
