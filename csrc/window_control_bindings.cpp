// mxstream — pybind binding of the window operators' host control (csrc/window_control.h): the
// Python KeyedWindowOperator drives its firing, re-firing and purging with the same C++ state
// machine as the C ABI pipeline (csrc/pipeline.cpp).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "window_control.h"

namespace py = pybind11;

void bind_window_control(py::module_& m) {
  using mxs::WindowControl;
  using i128 = WindowControl::i128;
  py::class_<WindowControl>(m, "WindowControl")
      .def(py::init<int64_t, int64_t, int64_t, int64_t>(), py::arg("size"), py::arg("slide"),
           py::arg("offset"), py::arg("lateness"))
      .def_property_readonly("pane", &WindowControl::pane)
      .def_property_readonly("panes_per_window", &WindowControl::panes_per_window)
      .def("pane_of", [](const WindowControl& c, int64_t t) { return c.pane_of((i128)t); })
      .def("pane_start", [](const WindowControl& c, int64_t p) { return c.pane_start((i128)p); })
      .def("last_start", [](const WindowControl& c, int64_t t) { return c.last_start((i128)t); })
      .def("first_start_containing",
           [](const WindowControl& c, int64_t t) { return c.first_start_containing((i128)t); })
      .def("align_up", [](const WindowControl& c, int64_t t) { return c.align_up((i128)t); })
      .def("fired_hi", &WindowControl::fired_hi)
      .def("late_ts", &WindowControl::late_ts, py::arg("wm"), py::arg("event_time") = true)
      .def("pane_base_from_wm", &WindowControl::pane_base_from_wm)
      .def("has_nfs", &WindowControl::has_nfs)
      .def("has_live", &WindowControl::has_live)
      .def("nfs", &WindowControl::nfs)
      .def("min_live", &WindowControl::min_live)
      .def("max_seen", &WindowControl::max_seen)
      .def("set_nfs", &WindowControl::set_nfs)
      .def("set_live", &WindowControl::set_live)
      .def("live_span_with", &WindowControl::live_span_with)
      .def("observe", &WindowControl::observe)
      .def("overlaps_live", &WindowControl::overlaps_live)
      .def("window_panes", &WindowControl::window_panes)
      .def("take_due", &WindowControl::take_due)
      .def("due_count", &WindowControl::due_count)
      .def("refire_windows", &WindowControl::refire_windows)
      .def("purge_range", [](const WindowControl& c, int64_t wm, int64_t ring) {
        const auto r = c.purge_range(wm, ring);
        return py::make_tuple(r.keep_from, r.from, r.stop);
      })
      .def("commit_purge", &WindowControl::commit_purge);
}
