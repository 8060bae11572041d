// mxstream — pybind11 bindings of the vector-metric window kernels (vector_hip.hip) and their
// CPU twins (vector_cpu.cpp). Plans are validated here before any launch.
#include <pybind11/pybind11.h>

#include <cstring>
#include <stdexcept>

#include "mxs_runtime.h"
#include "mxs_vector.h"

namespace py = pybind11;
using namespace mxs;

namespace {

template <class T>
T* VP(intptr_t p) {
  return reinterpret_cast<T*>(p);
}

void check_dim(int32_t dim) {
  if (dim <= 0 || dim % 32 || dim > 256)
    throw std::invalid_argument("dim must be a multiple of 32 in [32, 256]");
}

VecAggPlan make_vagg(py::dict d) {
  VecAggPlan p;
  std::memset(&p, 0, sizeof(p));
  p.cap_log2 = d["cap_log2"].cast<int32_t>();
  p.nsub = d["nsub"].cast<int32_t>();
  p.ring = d["ring"].cast<int32_t>();
  p.dim = d["dim"].cast<int32_t>();
  p.nsrc = d["nsrc"].cast<int32_t>();
  p.bucket_cap = d["bucket_cap"].cast<uint32_t>();
  p.np_step = d["np_step"].cast<int32_t>();
  p.positional = d["positional"].cast<int32_t>();
  p.rec_words = d["rec_words"].cast<int32_t>();
  p.mode = d["mode"].cast<int32_t>();
  p.pane_base = d["pane_base"].cast<int64_t>();
  p.p_lo = d["p_lo"].cast<int64_t>();
  p.fired_hi = d["fired_hi"].cast<int64_t>();
  if (p.ring <= 0 || (p.ring & (p.ring - 1))) throw std::invalid_argument("ring must be 2^k");
  if (p.cap_log2 < 6 || p.cap_log2 > 12) throw std::invalid_argument("cap_log2 must be 6..12");
  check_dim(p.dim);
  if (p.rec_words != 2 && p.rec_words != 3) throw std::invalid_argument("rec_words must be 2 or 3");
  if (p.mode != 0 && p.mode != 1) throw std::invalid_argument("mode must be 0 or 1");
  if (p.np_step > p.ring) throw std::invalid_argument("step touches more panes than the ring");
  return p;
}

VecFirePlan make_vfire(py::dict d) {
  VecFirePlan p;
  std::memset(&p, 0, sizeof(p));
  p.dim = d["dim"].cast<int32_t>();
  p.npanes = d["npanes"].cast<int32_t>();
  p.ring = d["ring"].cast<int32_t>();
  p.only_dirty = d["only_dirty"].cast<int32_t>();
  p.avg = d["avg"].cast<int32_t>();
  p.use_thr = d["use_thr"].cast<int32_t>();
  p.thr = d["thr"].cast<float>();
  p.nslots = d["nslots"].cast<int64_t>();
  p.p0 = d["p0"].cast<int64_t>();
  p.out_cap = d["out_cap"].cast<uint32_t>();
  check_dim(p.dim);
  if (p.npanes <= 0 || p.npanes > p.ring) throw std::invalid_argument("window panes exceed ring");
  return p;
}

}  // namespace

void bind_vector(py::module_& m) {
  m.def("vec_window_agg_lds", &gpu::vec_window_agg_lds);
  m.def("gpu_vec_window_agg", [](intptr_t recs, intptr_t counts, py::dict plan, intptr_t vec,
                                 intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g,
                                 intptr_t occ, intptr_t flags, intptr_t stream) {
    gpu::vec_window_agg(VP<void>(recs), VP<uint32_t>(counts), make_vagg(plan), VP<float>(vec),
                        VP<uint64_t>(keys_g), VP<float>(acc_g), VP<uint32_t>(cnt_g),
                        VP<uint8_t>(dirty_g), VP<uint32_t>(occ), VP<uint32_t>(flags), stream);
  });
  m.def("cpu_vec_window_agg", [](intptr_t recs, intptr_t counts, py::dict plan, intptr_t vec,
                                 intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g,
                                 intptr_t occ, intptr_t flags) {
    VecAggPlan p = make_vagg(plan);
    py::gil_scoped_release nogil;
    cpu::vec_window_agg(VP<void>(recs), VP<uint32_t>(counts), p, VP<float>(vec),
                        VP<uint64_t>(keys_g), VP<float>(acc_g), VP<uint32_t>(cnt_g),
                        VP<uint8_t>(dirty_g), VP<uint32_t>(occ), VP<uint32_t>(flags));
  });
  m.def("gpu_vec_window_fire", [](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g,
                                  intptr_t dirty_g, py::dict plan, intptr_t ok, intptr_t ov,
                                  intptr_t oc, intptr_t on, intptr_t stream) {
    gpu::vec_window_fire(VP<uint64_t>(keys_g), VP<float>(acc_g), VP<uint32_t>(cnt_g),
                         VP<uint8_t>(dirty_g), make_vfire(plan), VP<uint64_t>(ok), VP<float>(ov),
                         VP<uint32_t>(oc), VP<uint32_t>(on), stream);
  });
  m.def("cpu_vec_window_fire", [](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g,
                                  intptr_t dirty_g, py::dict plan, intptr_t ok, intptr_t ov,
                                  intptr_t oc, intptr_t on) {
    VecFirePlan p = make_vfire(plan);
    py::gil_scoped_release nogil;
    cpu::vec_window_fire(VP<uint64_t>(keys_g), VP<float>(acc_g), VP<uint32_t>(cnt_g),
                         VP<uint8_t>(dirty_g), p, VP<uint64_t>(ok), VP<float>(ov),
                         VP<uint32_t>(oc), VP<uint32_t>(on));
  });
  m.def("gpu_gen_vectors", [](intptr_t vec, int64_t n, int dim, uint64_t seed, uint64_t sid,
                              uint64_t idx0, float lo, float span, intptr_t stream) {
    check_dim(dim);
    gpu::gen_vectors(VP<float>(vec), n, dim, seed, sid, idx0, lo, span, stream);
  });
  m.def("cpu_gen_vectors", [](intptr_t vec, int64_t n, int dim, uint64_t seed, uint64_t sid,
                              uint64_t idx0, float lo, float span) {
    check_dim(dim);
    py::gil_scoped_release nogil;
    cpu::gen_vectors(VP<float>(vec), n, dim, seed, sid, idx0, lo, span);
  });
  m.def("gpu_vec_gather", [](intptr_t recs, int rw, intptr_t counts, int nb, uint32_t bcap,
                             intptr_t vec, int dim, intptr_t out, intptr_t stream) {
    check_dim(dim);
    gpu::vec_gather(VP<void>(recs), rw, VP<uint32_t>(counts), nb, bcap, VP<float>(vec), dim,
                    VP<float>(out), stream);
  });
  m.def("cpu_vec_gather", [](intptr_t recs, int rw, intptr_t counts, int nb, uint32_t bcap,
                             intptr_t vec, int dim, intptr_t out) {
    check_dim(dim);
    py::gil_scoped_release nogil;
    cpu::vec_gather(VP<void>(recs), rw, VP<uint32_t>(counts), nb, bcap, VP<float>(vec), dim,
                    VP<float>(out));
  });
}
