// mxstream — pybind11 bindings of the list-window pane arena / counting-sort firing kernels
// (csrc/listwin_hip.hip) and their C++ twins (csrc/listwin_cpu.cpp). Addresses are passed as
// integers (tensor data_ptr()); shapes are checked by the Python caller
// (runtime/list_window_operator.py) before any launch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <tuple>
#include <vector>

#include "mxs_listwin.h"
#include "mxs_runtime.h"

namespace py = pybind11;
using namespace mxs;

namespace {

template <class T>
T* LP(intptr_t p) {
  return reinterpret_cast<T*>(p);
}

LwPanes make_panes(const std::vector<std::tuple<intptr_t, intptr_t, int64_t>>& v) {
  if (v.empty() || v.size() > (size_t)kLwMaxPanes)
    throw std::invalid_argument("list window: 1..64 panes per firing");
  LwPanes w{};
  w.n = (int32_t)v.size();
  for (size_t i = 0; i < v.size(); ++i) {
    w.p[i].keys = LP<const int64_t>(std::get<0>(v[i]));
    w.p[i].vals = LP<const uint64_t>(std::get<1>(v[i]));
    w.p[i].len = std::get<2>(v[i]);
    if (w.p[i].len < 0) throw std::invalid_argument("list window: negative pane length");
  }
  return w;
}

LwRankPanes make_rank_panes(
    const std::vector<std::tuple<intptr_t, intptr_t, intptr_t, intptr_t, int64_t, int64_t, int64_t>>& v) {
  if (v.empty() || v.size() > (size_t)kLwMaxRankPanes)
    throw std::invalid_argument("list window: 1..32 panes per ranked firing");
  LwRankPanes w{};
  w.n = (int32_t)v.size();
  for (size_t i = 0; i < v.size(); ++i) {
    auto& p = w.p[i];
    p.keys = LP<const int64_t>(std::get<0>(v[i]));
    p.vals = LP<const uint64_t>(std::get<1>(v[i]));
    p.ranks = LP<const uint32_t>(std::get<2>(v[i]));
    p.counts = LP<const uint32_t>(std::get<3>(v[i]));
    p.kbase = std::get<4>(v[i]);
    p.ksize = std::get<5>(v[i]);
    p.len = std::get<6>(v[i]);
    if (!p.counts || !p.ranks || p.ksize <= 0 || p.len < 0)
      throw std::invalid_argument("list window: ranked pane without counts / ranks");
  }
  return w;
}

void check_ring(int ring) {
  if (ring < 1 || ring > kLwMaxRing || (ring & (ring - 1)))
    throw std::invalid_argument("list window: ring must be a power of two <= 4096");
}

}  // namespace

void bind_listwin(py::module_& m) {
  m.def("lw_pane_count", [](bool cuda, intptr_t ts, int64_t n, int64_t offset, int64_t pane,
                            int ring, int64_t late_ts, intptr_t counts, intptr_t stream) {
    check_ring(ring);
    if (pane <= 0) throw std::invalid_argument("list window: pane must be positive");
    if (cuda)
      gpu::lw_pane_count(LP<int64_t>(ts), n, offset, pane, ring, late_ts, LP<int64_t>(counts),
                         stream);
    else
      cpu::lw_pane_count(LP<int64_t>(ts), n, offset, pane, ring, late_ts, LP<int64_t>(counts));
  });
  m.def("lw_pane_scatter", [](bool cuda, intptr_t keys, intptr_t ts, intptr_t vals, int64_t n,
                              int64_t offset, int64_t pane, int ring, int64_t late_ts,
                              intptr_t tab, intptr_t cursor, intptr_t stream) {
    check_ring(ring);
    if (pane <= 0) throw std::invalid_argument("list window: pane must be positive");
    if (cuda)
      gpu::lw_pane_scatter(LP<int64_t>(keys), LP<int64_t>(ts), LP<uint64_t>(vals), n, offset,
                           pane, ring, late_ts, LP<int64_t>(tab), LP<int64_t>(cursor), stream);
    else
      cpu::lw_pane_scatter(LP<int64_t>(keys), LP<int64_t>(ts), LP<uint64_t>(vals), n, offset,
                           pane, ring, late_ts, LP<int64_t>(tab), LP<int64_t>(cursor));
  });
  m.def("lw_key_count", [](bool cuda, std::vector<std::tuple<intptr_t, intptr_t, int64_t>> panes,
                           int64_t kmin, int64_t nkeys, intptr_t counts, intptr_t stream) {
    const LwPanes w = make_panes(panes);
    if (cuda)
      gpu::lw_key_count(w, kmin, nkeys, LP<uint32_t>(counts), stream);
    else
      cpu::lw_key_count(w, kmin, nkeys, LP<uint32_t>(counts));
  });
  m.def("lw_scan_scratch_bytes", &gpu::lw_scan_scratch_bytes);
  m.def("lw_scan", [](bool cuda, intptr_t counts, int64_t nkeys, int64_t kmin, intptr_t scratch,
                      intptr_t offs, intptr_t heads, intptr_t head_keys, intptr_t nheads,
                      intptr_t stream) {
    if (nkeys <= 0) throw std::invalid_argument("list window: empty key range");
    if (cuda)
      gpu::lw_scan(LP<uint32_t>(counts), nkeys, kmin, LP<void>(scratch), LP<int64_t>(offs),
                   LP<int64_t>(heads), LP<int64_t>(head_keys), LP<int64_t>(nheads), stream);
    else
      cpu::lw_scan(LP<uint32_t>(counts), nkeys, kmin, LP<int64_t>(offs), LP<int64_t>(heads),
                   LP<int64_t>(head_keys), LP<int64_t>(nheads));
  });
  using RankPaneArg = std::tuple<intptr_t, intptr_t, intptr_t, intptr_t, int64_t, int64_t, int64_t>;
  m.def("lw_rank_prefix", [](bool cuda, std::vector<RankPaneArg> panes, int64_t kmin,
                             int64_t nkeys, intptr_t total, intptr_t pre, intptr_t stream) {
    const LwRankPanes w = make_rank_panes(panes);
    if (cuda)
      gpu::lw_rank_prefix(w, kmin, nkeys, LP<uint32_t>(total), LP<uint32_t>(pre), stream);
    else
      cpu::lw_rank_prefix(w, kmin, nkeys, LP<uint32_t>(total), LP<uint32_t>(pre));
  });
  m.def("lw_rank_scatter", [](bool cuda, std::vector<RankPaneArg> panes, int64_t kmin,
                              int64_t nkeys, intptr_t offs, intptr_t pre, intptr_t out_ord,
                              intptr_t stream) {
    const LwRankPanes w = make_rank_panes(panes);
    if (cuda)
      gpu::lw_rank_scatter(w, kmin, nkeys, LP<int64_t>(offs), LP<uint32_t>(pre),
                           LP<uint64_t>(out_ord), stream);
    else
      cpu::lw_rank_scatter(w, kmin, nkeys, LP<int64_t>(offs), LP<uint32_t>(pre),
                           LP<uint64_t>(out_ord));
  });
  m.def("lw_key_scatter", [](bool cuda,
                             std::vector<std::tuple<intptr_t, intptr_t, int64_t>> panes,
                             int64_t kmin, intptr_t cursor, intptr_t out_ord, intptr_t stream) {
    const LwPanes w = make_panes(panes);
    if (cuda)
      gpu::lw_key_scatter(w, kmin, LP<int64_t>(cursor), LP<uint64_t>(out_ord), stream);
    else
      cpu::lw_key_scatter(w, kmin, LP<int64_t>(cursor), LP<uint64_t>(out_ord));
  });
}
