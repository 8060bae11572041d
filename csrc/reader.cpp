// mxstream — Python binding of the pinned-slot text file reader (csrc/text_ring.h).
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <pybind11/functional.h>
#include <pybind11/stl.h>

#include <mutex>
#include <vector>

#include "mxs_runtime.h"
#include "text_ring.h"

namespace py = pybind11;

namespace {

// The reader plus, in mapped mode, the page-locking of its file mapping: the mapping is
// registered read-only once (hipHostRegisterReadOnly) so the copy engine reads the page cache
// directly, and unregistered before the mapping goes away.
class TextFileRing : public mxs::TextRingCore {
 public:
  using mxs::TextRingCore::TextRingCore;
  ~TextFileRing() {
    close();  // the reader thread (which page-locks segments) has stopped
    unregister();
  }
  // 0 on success (or nothing to register), else the hipError_t.
  int register_mapping(unsigned flags) {
    if (registered_ || !map_bytes()) return 0;
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(map_base()), (size_t)map_bytes(),
                                         flags);
    registered_ = e == hipSuccess;
    return (int)e;
  }
  // The mapping page-locked segment by segment by the reader thread (TextRingCore::on_segments).
  void register_segments(int64_t seg, unsigned flags) {
    on_segments(seg, [this, flags](intptr_t p, int64_t len) {
      const hipError_t e = hipHostRegister(reinterpret_cast<void*>(p), (size_t)len, flags);
      if (e == hipSuccess) {
        std::lock_guard<std::mutex> g(seg_mu_);
        segs_.push_back(p);
      }
      return (int)e;
    });
  }
  void unregister() {
    if (registered_) (void)hipHostUnregister(reinterpret_cast<void*>(map_base()));
    registered_ = false;
    std::lock_guard<std::mutex> g(seg_mu_);
    for (intptr_t p : segs_) (void)hipHostUnregister(reinterpret_cast<void*>(p));
    segs_.clear();
  }
  bool registered() const { return registered_; }

 private:
  bool registered_ = false;
  std::mutex seg_mu_;
  std::vector<intptr_t> segs_;
};

}  // namespace

void bind_reader(py::module_& m) {
  using mxs::Ready;
  py::class_<TextFileRing>(m, "TextFileRing")
      .def(py::init<const std::string&, int64_t, int64_t, std::vector<std::pair<intptr_t, int64_t>>,
                    int64_t, int>(),
           py::arg("path"), py::arg("lo"), py::arg("hi"), py::arg("slots"), py::arg("chunk"),
           py::arg("threads") = 8)
      // Mapped mode (csrc/text_ring.h MappedTag): `nslots` virtual slots, chunks handed out as
      // pointers into the file mapping.
      .def_static("mapped", [](const std::string& path, int64_t lo, int64_t hi, int nslots,
                               int64_t chunk, int threads, bool count_lines) {
        return std::unique_ptr<TextFileRing>(new TextFileRing(
            mxs::MappedTag{}, path, lo, hi, nslots, chunk, threads, count_lines));
      }, py::arg("path"), py::arg("lo"), py::arg("hi"), py::arg("nslots"), py::arg("chunk"),
         py::arg("threads") = 8, py::arg("count_lines") = true)
      .def("start", &TextFileRing::start)
      // (slot, nbytes, nlines, end_offset, eof, ptr): slot -1 when nothing is ready within
      // timeout_ms; eof when every chunk has been handed out; ptr: mapped mode's chunk address.
      .def("next", [](TextFileRing& r, int timeout_ms) {
        Ready x{-1, 0, 0, 0, 0};
        bool eof = false;
        {
          py::gil_scoped_release nogil;
          if (!r.next(timeout_ms, &x, &eof)) x.slot = -1;
        }
        return py::make_tuple(x.slot, x.nbytes, x.nlines, x.end_off, eof, x.ptr);
      }, py::arg("timeout_ms") = 1000)
      .def("release", &TextFileRing::release)
      .def_property_readonly("map_base", &TextFileRing::map_base)
      .def_property_readonly("map_bytes", &TextFileRing::map_bytes)
      .def("register_mapping", &TextFileRing::register_mapping, py::arg("flags") = 8u)
      .def("register_segments", &TextFileRing::register_segments, py::arg("seg"),
           py::arg("flags") = 8u)
      .def_property_readonly("segment_bytes", &TextFileRing::segment_bytes)
      .def_property_readonly("registered", &TextFileRing::registered)
      .def("close", [](TextFileRing& r) {
        py::gil_scoped_release nogil;
        r.close();
        r.unregister();
      });
}
