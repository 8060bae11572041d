// mxstream — Python binding of the pinned-slot text file reader (csrc/text_ring.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "mxs_runtime.h"
#include "text_ring.h"

namespace py = pybind11;

void bind_reader(py::module_& m) {
  using mxs::Ready;
  using mxs::TextRingCore;
  py::class_<TextRingCore>(m, "TextFileRing")
      .def(py::init<const std::string&, int64_t, int64_t, std::vector<std::pair<intptr_t, int64_t>>,
                    int64_t, int>(),
           py::arg("path"), py::arg("lo"), py::arg("hi"), py::arg("slots"), py::arg("chunk"),
           py::arg("threads") = 8)
      .def("start", &TextRingCore::start)
      // (slot, nbytes, nlines, end_offset, eof): slot -1 when nothing is ready within timeout_ms;
      // eof when every chunk has been handed out.
      .def("next", [](TextRingCore& r, int timeout_ms) {
        Ready x{-1, 0, 0, 0};
        bool eof = false;
        {
          py::gil_scoped_release nogil;
          if (!r.next(timeout_ms, &x, &eof)) x.slot = -1;
        }
        return py::make_tuple(x.slot, x.nbytes, x.nlines, x.end_off, eof);
      }, py::arg("timeout_ms") = 1000)
      .def("release", &TextRingCore::release)
      .def("close", [](TextRingCore& r) {
        py::gil_scoped_release nogil;
        r.close();
      });
}
