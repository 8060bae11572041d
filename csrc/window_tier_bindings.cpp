// mxstream — pybind11 binding of the host-DRAM window tier (csrc/window_tier.h), used by
// runtime/window_spill.py HostWindowTier.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

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
