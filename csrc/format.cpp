// mxstream — Python binding of the bulk Java formatter (csrc/javafmt.h): the print sink's
// columnar path (runtime/operators.py PrintSinkOp.process_columns).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <algorithm>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "javafmt.h"
#include "mxs_runtime.h"

namespace py = pybind11;

void bind_format(py::module_& m) {
  // rows i < n of the columns (kind, address): kind 0 = int64 ids into `names` (str), 1 = f64
  // (Double.toString), 2 = int64 (Long.toString). as_tuple: "(f0,f1,...)", else the single
  // column's text. prefixes[sub[i]] is prepended when `sub` (int32 address) is non-zero.
  m.def("java_format_rows", [](std::vector<std::tuple<int, intptr_t>> cols, int64_t n,
                               py::object names, intptr_t sub, std::vector<std::string> prefixes,
                               bool as_tuple) {
    if (cols.empty() || n < 0) throw std::invalid_argument("java_format_rows: no columns");
    if (!as_tuple && cols.size() != 1) throw std::invalid_argument("java_format_rows: arity");
    std::vector<std::string> nm;
    for (auto& c : cols)
      if (std::get<0>(c) == 0) {
        if (names.is_none()) throw std::invalid_argument("java_format_rows: string ids need names");
        if (nm.empty()) nm = names.cast<std::vector<std::string>>();
        break;
      }
    std::vector<std::string> out((size_t)n);
    {
      py::gil_scoped_release nogil;
      const int32_t* sb = reinterpret_cast<const int32_t*>(sub);
      std::string s;
      for (int64_t i = 0; i < n; ++i) {
        s.clear();
        if (sb) {
          const int32_t k = sb[i];
          if (k < 0 || (size_t)k >= prefixes.size())
            throw std::out_of_range("java_format_rows: subtask without prefix");
          s += prefixes[(size_t)k];
        }
        if (as_tuple) s.push_back('(');
        for (size_t j = 0; j < cols.size(); ++j) {
          if (j) s.push_back(',');
          const int kind = std::get<0>(cols[j]);
          const intptr_t a = std::get<1>(cols[j]);
          if (kind == 0) {
            const int64_t id = reinterpret_cast<const int64_t*>(a)[i];
            if (id < 0 || (size_t)id >= nm.size())
              throw std::out_of_range("java_format_rows: string id outside the dictionary");
            s += nm[(size_t)id];
          } else if (kind == 1) {
            mxs::java_double_append(reinterpret_cast<const double*>(a)[i], s);
          } else if (kind == 2) {
            mxs::java_long_append(reinterpret_cast<const int64_t*>(a)[i], s);
          } else {
            throw std::invalid_argument("java_format_rows: unknown column kind");
          }
        }
        if (as_tuple) s.push_back(')');
        out[(size_t)i] = s;
      }
    }
    return out;
  }, py::arg("cols"), py::arg("n"), py::arg("names"), py::arg("sub"), py::arg("prefixes"),
     py::arg("as_tuple") = true);
  // The same rows as ONE bytes object ("line\n" per row), formatted by up to `threads` threads
  // over contiguous row ranges (no Python string per row): the print sink's bulk path for
  // writers that take raw bytes (stdout, files, counters).
  m.def("java_format_bytes", [](std::vector<std::tuple<int, intptr_t>> cols, int64_t n,
                                py::object names, intptr_t sub, std::vector<std::string> prefixes,
                                bool as_tuple, int threads) {
    if (cols.empty() || n < 0) throw std::invalid_argument("java_format_bytes: no columns");
    if (!as_tuple && cols.size() != 1) throw std::invalid_argument("java_format_bytes: arity");
    for (auto& c : cols)
      if (std::get<0>(c) < 0 || std::get<0>(c) > 2)
        throw std::invalid_argument("java_format_bytes: unknown column kind");
    std::vector<std::string> nm;
    for (auto& c : cols)
      if (std::get<0>(c) == 0) {
        if (names.is_none()) throw std::invalid_argument("java_format_bytes: string ids need names");
        nm = names.cast<std::vector<std::string>>();
        break;
      }
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(1, std::min(threads, 64)),
                                                              n / 65536 + 1));
    std::vector<std::string> parts((size_t)T);
    std::vector<std::string> errs((size_t)T);
    {
      py::gil_scoped_release nogil;
      const int32_t* sb = reinterpret_cast<const int32_t*>(sub);
      auto work = [&](int t) {
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        std::string& s = parts[(size_t)t];
        s.reserve((size_t)(hi - lo) * 32);
        for (int64_t i = lo; i < hi; ++i) {
          if (sb) {
            const int32_t k = sb[i];
            if (k < 0 || (size_t)k >= prefixes.size()) {
              errs[(size_t)t] = "java_format_bytes: subtask without prefix";
              return;
            }
            s += prefixes[(size_t)k];
          }
          if (as_tuple) s.push_back('(');
          for (size_t j = 0; j < cols.size(); ++j) {
            if (j) s.push_back(',');
            const int kind = std::get<0>(cols[j]);
            const intptr_t a = std::get<1>(cols[j]);
            if (kind == 0) {
              const int64_t id = reinterpret_cast<const int64_t*>(a)[i];
              if (id < 0 || (size_t)id >= nm.size()) {
                errs[(size_t)t] = "java_format_bytes: string id outside the dictionary";
                return;
              }
              s += nm[(size_t)id];
            } else if (kind == 1) {
              mxs::java_double_append(reinterpret_cast<const double*>(a)[i], s);
            } else {
              mxs::java_long_append(reinterpret_cast<const int64_t*>(a)[i], s);
            }
          }
          if (as_tuple) s.push_back(')');
          s.push_back('\n');
        }
      };
      if (T == 1) {
        work(0);
      } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
      }
    }
    for (auto& e : errs)
      if (!e.empty()) throw std::out_of_range(e);
    size_t total = 0;
    for (auto& p : parts) total += p.size();
    py::bytes out(nullptr, total);
    char* dst = PyBytes_AS_STRING(out.ptr());
    for (auto& p : parts) {
      std::copy(p.begin(), p.end(), dst);
      dst += p.size();
    }
    return out;
  }, py::arg("cols"), py::arg("n"), py::arg("names"), py::arg("sub"), py::arg("prefixes"),
     py::arg("as_tuple") = true, py::arg("threads") = 1);
  m.def("java_double_str", [](double x) {
    std::string s;
    mxs::java_double_append(x, s);
    return s;
  });
}
