// mxstream — host runtime components (C++).
//
//  * StringDict      : interns string keys to dense 64-bit ids and records their Java
//                      String.hashCode (UTF-16), so keyBy on a String field reproduces Flink's key
//                      groups (ComputeCpuMax.java:26 keyBy(0) -> Tuple1<String>.hashCode()).
//  * parse_lines     : vectorised, Java-compatible `line.split(" ")` + Double.parseDouble /
//                      Long.parseLong / LocalDateTime.parse(..).toEpochSecond(+08:00)
//                      (Main.java:21-24, BandwidthMonitor.java:28-30,
//                      BandwidthMonitorWithEventTime.java:33,41).
//  * SocketSource    : background reader thread with Flink SocketTextStreamFunction semantics
//                      ('\n' delimiter, trailing '\r' stripped, remainder flushed at EOF).
//  * write/read_kg_file : keyed-state snapshot files indexed by key group (restore at a
//                      different parallelism re-reads only the owned key-group range).
#include <arpa/inet.h>
#include <netdb.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <fstream>
#include <mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "mxs_common.h"
#include "mxs_log.h"
#include "mxs_runtime.h"
#include "kg_file.h"
#include "socket_reader.h"

namespace py = pybind11;

namespace mxs {
namespace {

// ------------------------------------------------------------------------------------------
// Java String.hashCode over the UTF-16 encoding of UTF-8 input (invalid bytes -> U+FFFD).
// ------------------------------------------------------------------------------------------
int32_t java_string_hash(std::string_view s) {
  return java_hash_utf8(s.data(), (int64_t)s.size());  // mxs_common.h (shared with the GPU)
}

class StringDict {
 public:
  uint64_t intern(std::string_view s) {
    std::lock_guard<std::mutex> g(mu_);
    return intern_locked(s);
  }
  uint64_t intern_locked(std::string_view s) {
    auto it = ids_.find(s);  // no temporary std::string per lookup
    if (it != ids_.end()) return it->second;
    const uint64_t id = strs_.size();
    strs_.emplace_back(s);
    jhash_.push_back(java_string_hash(s));
    ids_.emplace(strs_.back(), id);
    return id;
  }
  std::string get(uint64_t id) const {
    if (id >= strs_.size()) throw std::out_of_range("StringDict id out of range");
    return strs_[id];
  }
  size_t size() const { return strs_.size(); }
  py::array_t<int32_t> jhash_table() const {
    py::array_t<int32_t> a((py::ssize_t)jhash_.size());
    if (!jhash_.empty()) std::memcpy(a.mutable_data(), jhash_.data(), jhash_.size() * 4);
    return a;
  }
  std::vector<std::string> strings() const { return {strs_.begin(), strs_.end()}; }
  std::mutex& mu() { return mu_; }

 private:
  std::mutex mu_;
  // Keys view the interned strings; a deque never relocates its elements, so the views stay valid.
  std::deque<std::string> strs_;
  std::unordered_map<std::string_view, uint64_t> ids_;
  std::vector<int32_t> jhash_;
};

// ------------------------------------------------------------------------------------------
// Java parsing helpers
// ------------------------------------------------------------------------------------------
struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// java.lang.String.split(String) for a single non-regex-metachar separator: every occurrence
// splits, trailing empty strings are removed, "" -> [""].
void java_split(std::string_view line, char sep, std::vector<std::string_view>& out) {
  out.clear();
  if (line.empty()) {  // no match: the array holds the input itself
    out.push_back(line);
    return;
  }
  const char* const b = line.data();
  const char* const e = b + line.size();
  const char* start = b;
  for (const char* q; (q = static_cast<const char*>(std::memchr(start, sep, (size_t)(e - start))));) {
    out.push_back(std::string_view(start, (size_t)(q - start)));
    start = q + 1;
  }
  out.push_back(std::string_view(start, (size_t)(e - start)));
  while (!out.empty() && out.back().empty()) out.pop_back();
}

std::string_view java_trim(std::string_view s) {
  size_t a = 0, b = s.size();
  while (a < b && (unsigned char)s[a] <= ' ') ++a;
  while (b > a && (unsigned char)s[b - 1] <= ' ') --b;
  return s.substr(a, b - a);
}

double java_parse_double(std::string_view raw) {
  std::string_view s = java_trim(raw);
  if (s.empty()) throw ParseError("NumberFormatException: empty String");
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  std::string_view body = s.substr(i);
  if (body == "NaN") return std::nan("");
  if (body == "Infinity") return neg ? -INFINITY : INFINITY;
  // Strip a Java float-type suffix.
  if (!body.empty()) {
    const char c = body.back();
    if (c == 'd' || c == 'D' || c == 'f' || c == 'F') body = body.substr(0, body.size() - 1);
  }
  if (body.empty()) throw ParseError("NumberFormatException: For input string: \"" + std::string(raw) + "\"");
  bool hex = body.size() > 1 && body[0] == '0' && (body[1] == 'x' || body[1] == 'X');
  if (!hex) {
    // Decimal grammar: digits [. digits] [e|E [+-] digits], at least one digit in the mantissa.
    size_t j = 0, nd = 0;
    while (j < body.size() && isdigit((unsigned char)body[j])) ++j, ++nd;
    if (j < body.size() && body[j] == '.') {
      ++j;
      while (j < body.size() && isdigit((unsigned char)body[j])) ++j, ++nd;
    }
    if (nd == 0) throw ParseError("NumberFormatException: For input string: \"" + std::string(raw) + "\"");
    if (j < body.size() && (body[j] == 'e' || body[j] == 'E')) {
      ++j;
      if (j < body.size() && (body[j] == '+' || body[j] == '-')) ++j;
      size_t ne = 0;
      while (j < body.size() && isdigit((unsigned char)body[j])) ++j, ++ne;
      if (ne == 0) throw ParseError("NumberFormatException: For input string: \"" + std::string(raw) + "\"");
    }
    if (j != body.size()) throw ParseError("NumberFormatException: For input string: \"" + std::string(raw) + "\"");
  }
  if (!hex) {
    // Clinger's fast path: a decimal with <= 15 significant digits and no exponent is an exact
    // integer mantissa over an exact power of ten (<= 10^22); one IEEE division of two exact
    // values is correctly rounded, i.e. identical to strtod / Double.parseDouble.
    static const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                    1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                    1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    uint64_t mant = 0;
    int nd = 0, frac = -1;
    bool simple = true;
    for (size_t j = 0; j < body.size(); ++j) {
      const char c = body[j];
      if (c >= '0' && c <= '9') {
        if (mant == 0 && c == '0') {  // leading zeros are not significant
          if (frac >= 0) ++frac;
          continue;
        }
        if (++nd > 15) {
          simple = false;
          break;
        }
        mant = mant * 10 + (uint64_t)(c - '0');
        if (frac >= 0) ++frac;
      } else if (c == '.' && frac < 0) {
        frac = 0;
      } else {
        simple = false;  // exponent: the general path
        break;
      }
    }
    if (simple && (frac < 0 ? 0 : frac) <= 22) {
      const double v = (double)mant / kPow10[frac < 0 ? 0 : frac];
      return neg ? -v : v;
    }
  }
  std::string tmp(body);
  errno = 0;
  char* end = nullptr;
  double v = std::strtod(tmp.c_str(), &end);
  if (end != tmp.c_str() + tmp.size())
    throw ParseError("NumberFormatException: For input string: \"" + std::string(raw) + "\"");
  return neg ? -v : v;
}

int64_t java_parse_long(std::string_view s, int64_t lo, int64_t hi, const char* what) {
  int64_t v = 0;
  const int rc = parse_long_ascii(s.data(), (int64_t)s.size(), lo, hi, &v);
  if (rc == 1) throw ParseError("NumberFormatException: For input string: \"" + std::string(s) + "\"");
  if (rc == 2)
    throw ParseError(std::string("NumberFormatException: ") + what + " overflow \"" + std::string(s) + "\"");
  return v;
}

// LocalDateTime.parse (ISO_LOCAL_DATE_TIME) -> epoch seconds + sub-second millis at an offset.
void parse_iso_local_datetime(std::string_view s, int64_t offset_s, int64_t* epoch_s, int64_t* millis) {
  if (!iso_local_datetime(s.data(), (int64_t)s.size(), offset_s, epoch_s, millis))
    throw ParseError("DateTimeParseException: Text '" + std::string(s) + "' could not be parsed");
}

enum FieldKind : int {
  FK_STR = 0,        // dictionary id (u64)
  FK_DOUBLE = 1,     // Double.parseDouble -> f64
  FK_LONG = 2,       // Long.parseLong -> i64
  FK_TS_INTSEC = 3,  // (int) LocalDateTime.parse(x).toEpochSecond(off) * 1000L  (reference quirk)
  FK_TS_MS = 4,      // exact epoch millis of LocalDateTime.parse(x) at offset
  FK_INT = 5,        // Integer.parseInt -> i64
  FK_RAW_LONG = 6,   // epoch-ms integer field
  FK_ISO_SEC = 7,    // (int) LocalDateTime.parse(x).toEpochSecond(off): int32 seconds
};

// Parse one line's fields into row `li` of the columns. String fields get a thread-local id
// (remapped to the dictionary's ids afterwards). Throws ParseError.
// Open addressing over (hash, id) words with linear probing: field values are short (host
// names, "cpuN"), a lookup is one hash of <= a few words and, on a hit, one compare.
struct LocalDict {
  std::vector<std::string_view> strs;
  std::vector<uint64_t> tab = std::vector<uint64_t>(1024, 0);  // (hash hi 32 | id + 1), 0 = empty
  static uint64_t hash(std::string_view v) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)v.size();
    size_t i = 0;
    for (; i + 8 <= v.size(); i += 8) {
      uint64_t w;
      std::memcpy(&w, v.data() + i, 8);
      h = mix64(h ^ w);
    }
    if (i < v.size()) {
      uint64_t w = 0;
      std::memcpy(&w, v.data() + i, v.size() - i);
      h = mix64(h ^ w);
    }
    return h;
  }
  void grow() {
    std::vector<uint64_t> t(tab.size() * 2, 0);
    const size_t mask = t.size() - 1;
    for (uint64_t x : tab) {
      if (!x) continue;
      size_t j = (size_t)(hash(strs[(uint32_t)x - 1]) & mask);
      while (t[j]) j = (j + 1) & mask;
      t[j] = x;
    }
    tab.swap(t);
  }
  uint32_t intern(std::string_view v) {
    const uint64_t h = hash(v);
    const uint64_t tag = h >> 32 << 32;
    const size_t mask = tab.size() - 1;
    for (size_t j = (size_t)(h & mask);; j = (j + 1) & mask) {
      const uint64_t x = tab[j];
      if (!x) {
        const uint32_t id = (uint32_t)strs.size();
        strs.push_back(v);
        tab[j] = tag | (uint64_t)(id + 1);
        if (2 * strs.size() > tab.size()) grow();
        return id;
      }
      if ((x >> 32 << 32) == tag && strs[(uint32_t)x - 1] == v) return (uint32_t)x - 1;
    }
  }
};

static void parse_line_into(std::string_view line, char sep,
                            const std::vector<std::pair<int, int>>& spec,
                            const std::vector<void*>& ptrs, size_t li, int64_t offset_s,
                            std::vector<std::string_view>& parts, LocalDict& ld) {
  java_split(line, sep, parts);
  for (size_t c = 0; c < spec.size(); ++c) {
    const int fi = spec[c].first;
    if (fi < 0 || (size_t)fi >= parts.size())
      throw ParseError("ArrayIndexOutOfBoundsException: " + std::to_string(fi));
    std::string_view v = parts[fi];
    switch (spec[c].second) {
      case FK_STR: ((uint64_t*)ptrs[c])[li] = ld.intern(v); break;
      case FK_DOUBLE: ((double*)ptrs[c])[li] = java_parse_double(v); break;
      case FK_LONG: ((int64_t*)ptrs[c])[li] = java_parse_long(v, INT64_MIN, INT64_MAX, "long"); break;
      case FK_INT: ((int64_t*)ptrs[c])[li] = java_parse_long(v, INT32_MIN, INT32_MAX, "int"); break;
      case FK_RAW_LONG: ((int64_t*)ptrs[c])[li] = java_parse_long(v, INT64_MIN, INT64_MAX, "long"); break;
      case FK_TS_INTSEC: {
        int64_t es, ms;
        parse_iso_local_datetime(v, offset_s, &es, &ms);
        ((int64_t*)ptrs[c])[li] = (int64_t)(int32_t)(uint32_t)(uint64_t)es * 1000LL;
        break;
      }
      case FK_TS_MS: {
        int64_t es, ms;
        parse_iso_local_datetime(v, offset_s, &es, &ms);
        ((int64_t*)ptrs[c])[li] = es * 1000LL + ms;
        break;
      }
      case FK_ISO_SEC: {
        int64_t es, ms;
        parse_iso_local_datetime(v, offset_s, &es, &ms);
        ((int64_t*)ptrs[c])[li] = (int64_t)(int32_t)(uint32_t)(uint64_t)es;
        break;
      }
      default: throw ParseError("unknown field kind");
    }
  }
}

// Lines of [a, b) of `all` (a starts a line): '\n'-separated, trailing '\r' stripped, a trailing
// newline does not start a line.
static void find_lines(std::string_view all, size_t a, size_t b, std::vector<std::string_view>& out) {
  size_t start = a;
  out.reserve(out.size() + (b - a) / 24 + 16);
  for (const char* q; start < b &&
                      (q = static_cast<const char*>(std::memchr(all.data() + start, '\n', b - start)));) {
    const size_t i = (size_t)(q - all.data());
    std::string_view l = all.substr(start, i - start);
    if (!l.empty() && l.back() == '\r') l.remove_suffix(1);
    out.push_back(l);
    start = i + 1;
  }
  if (start < b) {
    std::string_view l = all.substr(start, b - start);
    if (!l.empty() && l.back() == '\r') l.remove_suffix(1);
    out.push_back(l);
  }
}

// Parse newline-separated lines. Returns (columns, nparsed, error_index, error_message).
//
// threads > 1: the byte buffer is cut into `threads` newline-aligned chunks; each thread finds
// its lines and parses them into its row range, interning string fields into a thread-local
// dictionary. The local dictionaries are then merged into `dict` in chunk order (first
// appearance order over the whole batch) and the string columns remapped -- ids, like every
// column, are identical to the single-threaded parse. An error stops at the lowest failing
// line (nparsed = its index); rows after it are not part of the result.
py::tuple parse_lines(py::bytes data, std::vector<std::pair<int, int>> spec, std::string sep,
                      StringDict& dict, int64_t offset_s, int threads) {
  if (sep.size() != 1) throw std::invalid_argument("separator must be one character");
  char* buf;
  py::ssize_t len;
  if (PYBIND11_BYTES_AS_STRING_AND_SIZE(data.ptr(), &buf, &len)) throw py::error_already_set();
  std::string_view all(buf, (size_t)len);
  const int T = std::max(1, std::min(threads, 64));
  // Newline-aligned chunk bounds.
  std::vector<size_t> cut(T + 1, all.size());
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    size_t c = std::max(cut[t - 1], all.size() * (size_t)t / (size_t)T);
    while (c < all.size() && c > 0 && all[c - 1] != '\n') ++c;
    cut[t] = c;
  }
  std::vector<std::vector<std::string_view>> lines(T);
  {
    py::gil_scoped_release nogil;
    if (T == 1) {
      find_lines(all, 0, all.size(), lines[0]);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] { find_lines(all, cut[t], cut[t + 1], lines[t]); });
      for (auto& x : th) x.join();
    }
  }
  std::vector<size_t> row0(T + 1, 0);
  for (int t = 0; t < T; ++t) row0[t + 1] = row0[t] + lines[t].size();
  const size_t n = row0[T];
  std::vector<py::array> cols;
  std::vector<void*> ptrs;
  for (auto& f : spec) {
    if (f.second == FK_DOUBLE) {
      cols.push_back(py::array_t<double>((py::ssize_t)n));
    } else if (f.second == FK_STR) {
      cols.push_back(py::array_t<uint64_t>((py::ssize_t)n));
    } else {
      cols.push_back(py::array_t<int64_t>((py::ssize_t)n));
    }
    ptrs.push_back(cols.back().mutable_data());
  }
  std::vector<LocalDict> ld(T);
  std::vector<int64_t> terr(T, -1);
  std::vector<std::string> tmsg(T);
  int64_t err_idx = -1;
  std::string err_msg;
  {
    py::gil_scoped_release nogil;
    auto work = [&](int t) {
      std::vector<std::string_view> parts;
      for (size_t k = 0; k < lines[t].size(); ++k) {
        try {
          parse_line_into(lines[t][k], sep[0], spec, ptrs, row0[t] + k, offset_s, parts, ld[t]);
        } catch (const ParseError& e) {
          terr[t] = (int64_t)(row0[t] + k);
          tmsg[t] = e.what();
          return;
        }
      }
    };
    if (T == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t)
      if (terr[t] >= 0) {
        err_idx = terr[t];
        err_msg = tmsg[t];
        break;
      }
    const size_t done = err_idx >= 0 ? (size_t)err_idx : n;
    // Merge the local dictionaries in chunk order, then remap the string columns.
    std::vector<std::vector<uint64_t>> gid(T);
    {
      std::lock_guard<std::mutex> g(dict.mu());
      for (int t = 0; t < T && row0[t] < done; ++t) {
        // Only strings of rows before the error enter the dictionary (as in a serial parse).
        const size_t lim = std::min(done, row0[t + 1]) - row0[t];
        if (lim == lines[t].size()) {
          gid[t].reserve(ld[t].strs.size());
          for (auto v : ld[t].strs) gid[t].push_back(dict.intern_locked(v));
        } else {
          // Partial chunk: intern in first-appearance order over the kept rows only.
          gid[t].assign(ld[t].strs.size(), ~0ull);
          for (size_t k = 0; k < lim; ++k)
            for (size_t c = 0; c < spec.size(); ++c)
              if (spec[c].second == FK_STR) {
                const uint64_t l = ((uint64_t*)ptrs[c])[row0[t] + k];
                if (gid[t][l] == ~0ull) gid[t][l] = dict.intern_locked(ld[t].strs[l]);
              }
        }
      }
    }
    auto remap = [&](int t) {
      const size_t lim = row0[t] < done ? std::min(done, row0[t + 1]) - row0[t] : 0;
      for (size_t c = 0; c < spec.size(); ++c) {
        if (spec[c].second != FK_STR) continue;
        uint64_t* col = (uint64_t*)ptrs[c] + row0[t];
        for (size_t k = 0; k < lim; ++k) col[k] = gid[t][col[k]];
      }
    };
    if (T == 1) {
      remap(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t) th.emplace_back(remap, t);
      for (auto& x : th) x.join();
    }
  }
  py::list out;
  for (auto& c : cols) out.append(c);
  const int64_t done = err_idx >= 0 ? err_idx : (int64_t)n;
  return py::make_tuple(out, done, err_idx, err_msg);
}

// ------------------------------------------------------------------------------------------
// Key-group indexed state files.
// Layout: "MXSKG001" | u64 header_len | header (UTF-8 JSON from Python) | u32 kg_lo | u32 kg_hi |
//         u64 offsets[kg_hi - kg_lo + 2] (row offsets) | columns (each nrows * itemsize, kg-sorted)
// ------------------------------------------------------------------------------------------
void write_kg_file(const std::string& path, const std::string& header, uint32_t kg_lo,
                   uint32_t kg_hi, py::array_t<int32_t, py::array::c_style> kg, py::list columns) {
  const size_t n = (size_t)kg.size();
  const int32_t* kgp = kg.data();
  // Pin every column (contiguous views kept alive here) while holding the GIL, then do the
  // counting sort, the row permutation and the file I/O without it: an asynchronous checkpoint
  // writes from a worker thread while the step loop keeps running Python.
  std::vector<py::array> keep;
  std::vector<std::pair<const char*, size_t>> cols;
  for (auto h : columns) {
    py::array a = py::reinterpret_borrow<py::array>(h);
    if ((size_t)a.size() != n) throw std::invalid_argument("column length mismatch");
    keep.push_back(py::array::ensure(a, py::array::c_style));
    cols.emplace_back((const char*)keep.back().data(), (size_t)keep.back().itemsize());
  }
  py::gil_scoped_release nogil;
  write_kg_columns(path, header, kg_lo, kg_hi, kgp, n, cols);
}

// Returns (header, kg_lo, kg_hi, offsets(np.uint64), raw column bytes for rows in [lo, hi]).
py::tuple read_kg_file(const std::string& path, py::list itemsizes, uint32_t want_lo, uint32_t want_hi) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  char magic[8];
  f.read(magic, 8);
  if (std::memcmp(magic, "MXSKG001", 8) != 0) throw std::runtime_error("bad magic in " + path);
  uint64_t hl;
  f.read((char*)&hl, 8);
  std::string header(hl, '\0');
  f.read(header.data(), (std::streamsize)hl);
  uint32_t lo, hi;
  f.read((char*)&lo, 4);
  f.read((char*)&hi, 4);
  const uint32_t ng = hi - lo + 1;
  std::vector<uint64_t> off(ng + 1);
  f.read((char*)off.data(), (std::streamsize)(off.size() * 8));
  const uint64_t nrows = off[ng];
  const std::streamoff data0 = f.tellg();
  const uint32_t a = std::max(lo, want_lo), b = std::min(hi, want_hi);
  uint64_t r0 = 0, r1 = 0;
  if (a <= b) {
    r0 = off[a - lo];
    r1 = off[b - lo + 1];
  }
  // Each column's rows [r0, r1) straight into a numpy byte array (no intermediate copies), the
  // columns read in parallel with positioned reads and the GIL released.
  py::list cols;
  std::vector<std::tuple<char*, size_t, uint64_t>> jobs;  // (dst, bytes, file offset)
  uint64_t colbase = (uint64_t)data0;
  for (auto h : itemsizes) {
    const size_t isz = h.cast<size_t>();
    py::array_t<uint8_t> a((py::ssize_t)((r1 - r0) * isz));
    jobs.emplace_back((char*)a.mutable_data(), (size_t)((r1 - r0) * isz), colbase + r0 * isz);
    cols.append(a);
    colbase += nrows * isz;
  }
  f.close();
  if (!jobs.empty()) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path);
    std::atomic<bool> bad{false};
    {
      py::gil_scoped_release nogil;
      auto rd = [&](size_t j) {
        auto [dst, n, off] = jobs[j];
        while (n) {
          const ssize_t r = ::pread(fd, dst, n, (off_t)off);
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) {
            bad = true;
            return;
          }
          dst += r;
          n -= (size_t)r;
          off += (uint64_t)r;
        }
      };
      std::vector<std::thread> th;
      for (size_t j = 1; j < jobs.size(); ++j) th.emplace_back(rd, j);
      rd(0);
      for (auto& x : th) x.join();
    }
    ::close(fd);
    if (bad) throw std::runtime_error("short read in " + path);
  }
  py::array_t<uint64_t> offs((py::ssize_t)off.size());
  std::memcpy(offs.mutable_data(), off.data(), off.size() * 8);
  return py::make_tuple(py::bytes(header), lo, hi, offs, cols, (int64_t)(r1 - r0));
}

}  // namespace
}  // namespace mxs

void bind_runtime(py::module_& m) {
  using namespace mxs;
  m.def("java_string_hash", [](const std::string& s) { return java_string_hash(s); });
  m.def("java_parse_double", [](const std::string& s) { return java_parse_double(s); });
  m.def("java_split", [](const std::string& s, const std::string& sep) {
    std::vector<std::string_view> parts;
    java_split(s, sep.at(0), parts);
    std::vector<std::string> out(parts.begin(), parts.end());
    return out;
  });
  m.def("iso_to_epoch_ms", [](const std::string& s, int64_t offset_s) {
    int64_t es, ms;
    parse_iso_local_datetime(s, offset_s, &es, &ms);
    return es * 1000 + ms;
  });
  py::register_exception<ParseError>(m, "ParseError");

  py::class_<StringDict>(m, "StringDict")
      .def(py::init<>())
      .def("intern", [](StringDict& d, const std::string& s) { return d.intern(s); })
      .def("get", &StringDict::get)
      .def("__len__", &StringDict::size)
      .def("jhash_table", &StringDict::jhash_table)
      .def("strings", &StringDict::strings);

  m.def("parse_lines", &parse_lines, py::arg("data"), py::arg("spec"), py::arg("sep"),
        py::arg("dict"), py::arg("offset_s") = 0, py::arg("threads") = 1);

  py::class_<SocketReaderCore>(m, "SocketSource")
      .def(py::init<std::string, int, std::string, int, int64_t, size_t>(), py::arg("host"),
           py::arg("port"), py::arg("delimiter") = "\n", py::arg("max_retry") = 0,
           py::arg("retry_ms") = 500, py::arg("max_queue") = 1 << 22)
      .def("start", &SocketReaderCore::start)
      .def("blocked", &SocketReaderCore::blocked)
      // Returns (joined_lines_bytes, nlines, eof, error).
      .def("poll", [](SocketReaderCore& s, size_t max_lines, int timeout_ms) {
        std::string joined, err;
        size_t n = 0;
        bool eof = false;
        {
          py::gil_scoped_release nogil;
          s.poll(max_lines, timeout_ms, &joined, &n, &eof, &err);
        }
        return py::make_tuple(py::bytes(joined), (int64_t)n, eof, err);
      }, py::arg("max_lines") = 1 << 20, py::arg("timeout_ms") = 100)
      .def("close", [](SocketReaderCore& s) {
        py::gil_scoped_release nogil;
        s.close();
      });

  m.def("write_kg_file", &write_kg_file);
  m.def("read_kg_file", &read_kg_file);
}
