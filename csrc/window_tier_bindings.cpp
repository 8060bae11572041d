// mxstream — pybind11 binding of the host-DRAM window tier (csrc/window_tier.h), used by
// runtime/window_spill.py HostWindowTier.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "mxs_runtime.h"
#include "window_tier.h"

namespace py = pybind11;

namespace {

template <class T>
using Arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <class T>
py::array_t<T> np_of(const std::vector<T>& v) {
  return py::array_t<T>((py::ssize_t)v.size(), v.data());
}

}  // namespace

void bind_window_tier(py::module_& m) {
  using mxs::WindowTierCore;
  py::class_<WindowTierCore>(m, "WindowTier")
      .def(py::init<int>(), py::arg("agg"))
      .def("copy", [](const WindowTierCore& t) { return WindowTierCore(t); })
      .def_readwrite("prefault", &WindowTierCore::prefault_)
      .def_property_readonly("spare_chunks", &WindowTierCore::spare_chunks)
      .def_property_readonly("nrows", &WindowTierCore::nrows)
      .def_property_readonly("nbytes", &WindowTierCore::nbytes)
      .def_property_readonly("rows_in", &WindowTierCore::rows_in)
      .def("pane_range", [](const WindowTierCore& t) -> py::object {
        int64_t lo, hi;
        if (!t.pane_range(&lo, &hi)) return py::none();
        return py::make_tuple(lo, hi);
      })
      .def("absorb", [](WindowTierCore& t, Arr<uint64_t> key, Arr<int64_t> pane, Arr<int64_t> acc,
                        Arr<int64_t> cnt, Arr<uint8_t> dirty) {
        const size_t n = (size_t)key.size();
        if ((size_t)pane.size() != n || (size_t)acc.size() != n || (size_t)cnt.size() != n ||
            (size_t)dirty.size() != n)
          throw std::invalid_argument("WindowTier.absorb: column lengths differ");
        py::gil_scoped_release nogil;
        t.absorb(key.data(), pane.data(), acc.data(), cnt.data(), dirty.data(), n);
      })
      .def("absorb_presorted", [](WindowTierCore& t, Arr<uint64_t> key, Arr<uint64_t> acc,
                                  Arr<uint32_t> cnt, Arr<uint8_t> dirty, int64_t p0,
                                  Arr<uint32_t> counts) {
        uint64_t n = 0;
        for (py::ssize_t j = 0; j < counts.size(); ++j) n += counts.data()[j];
        if ((uint64_t)key.size() < n || (uint64_t)acc.size() < n || (uint64_t)cnt.size() < n ||
            (uint64_t)dirty.size() < n)
          throw std::invalid_argument("WindowTier.absorb_presorted: columns shorter than counts");
        py::gil_scoped_release nogil;
        t.absorb_presorted(key.data(), acc.data(), cnt.data(), dirty.data(), p0, counts.data(),
                           (int)counts.size());
      })
      // Live rows of panes [p0, p1] into caller buffers (addresses; pinned host memory of the
      // device-merged firing): returns the row count, rows written only when it is <= cap.
      .def("export_rows", [](const WindowTierCore& t, int64_t p0, int64_t p1, intptr_t k,
                             intptr_t a, intptr_t c, size_t cap) {
        py::gil_scoped_release nogil;
        return t.export_rows(p0, p1, reinterpret_cast<uint64_t*>(k), reinterpret_cast<uint64_t*>(a),
                             reinterpret_cast<uint32_t*>(c), cap);
      })
      .def("export_window", [](const WindowTierCore& t, int64_t p0, int64_t p1, intptr_t k,
                               intptr_t a, intptr_t c, size_t r_begin, size_t cap) {
        py::gil_scoped_release nogil;
        return t.export_window(p0, p1, reinterpret_cast<uint64_t*>(k),
                               reinterpret_cast<uint64_t*>(a), reinterpret_cast<uint32_t*>(c),
                               r_begin, cap, true);
      })
      .def("part", [](const WindowTierCore& t, int64_t p0, int64_t p1) {
        std::vector<uint64_t> k;
        std::vector<int64_t> a, c;
        {
          py::gil_scoped_release nogil;
          t.part(p0, p1, &k, &a, &c);
        }
        return py::make_tuple(np_of(k), np_of(a), np_of(c));
      })
      .def("merge_fire", [](const WindowTierCore& t, int64_t p0, int64_t p1, Arr<uint64_t> dk,
                            Arr<int64_t> da, Arr<int64_t> dc, bool only_dev) {
        const size_t n = (size_t)dk.size();
        if ((size_t)da.size() != n || (size_t)dc.size() != n)
          throw std::invalid_argument("WindowTier.merge_fire: column lengths differ");
        std::vector<uint64_t> k;
        std::vector<int64_t> a, c;
        {
          py::gil_scoped_release nogil;
          t.merge_fire(p0, p1, dk.data(), da.data(), dc.data(), n, only_dev, &k, &a, &c);
        }
        return py::make_tuple(np_of(k), np_of(a), np_of(c));
      })
      .def("merge_fire_epilogue",
           [](const WindowTierCore& t, int64_t p0, int64_t p1, Arr<uint64_t> dk, Arr<int64_t> da,
              Arr<int64_t> dc, bool only_dev, std::vector<int32_t> mc, std::vector<double> mk,
              std::vector<int32_t> fc, std::vector<double> fk, int64_t wstart, int64_t wend) {
             const size_t n = (size_t)dk.size();
             if ((size_t)da.size() != n || (size_t)dc.size() != n)
               throw std::invalid_argument("WindowTier.merge_fire_epilogue: column lengths differ");
             const mxs::ExprProg mp = WindowTierCore::prog(mc.data(), mc.size(), mk.data(),
                                                                   mk.size());
             const mxs::ExprProg fp = WindowTierCore::prog(fc.data(), fc.size(), fk.data(),
                                                                   fk.size());
             std::vector<uint64_t> k, ok;
             std::vector<int64_t> a, c, oraw;
             std::vector<double> ov;
             std::vector<int32_t> oc;
             {
               py::gil_scoped_release nogil;
               t.merge_fire(p0, p1, dk.data(), da.data(), dc.data(), n, only_dev, &k, &a, &c);
               t.epilogue(k, a, c, mp, fp, wstart, wend, &ok, &ov, &oraw, &oc);
             }
             return py::make_tuple(np_of(ok), np_of(ov), np_of(oraw), np_of(oc));
           })
      .def("purge", [](WindowTierCore& t, int64_t keep_from) {
        py::gil_scoped_release nogil;
        t.purge(keep_from);
      })
      .def("rows", [](WindowTierCore& t) {
        WindowTierCore::Rows r;
        {
          py::gil_scoped_release nogil;
          r = t.rows();
        }
        py::dict d;
        d["key"] = np_of(r.key);
        d["pane"] = np_of(r.pane);
        d["acc"] = np_of(r.acc);
        d["cnt"] = np_of(r.cnt);
        d["dirty"] = np_of(r.dirty);
        return d;
      })
      .def("clear", &WindowTierCore::clear);
}
