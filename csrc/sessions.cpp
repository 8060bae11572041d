// mxstream — host session-window store (C++).
//
// Event-time session windows (EventTimeSessionWindows.withGap, chapter3/README.md:412-428):
// every element opens [ts, ts + gap); windows that intersect (TimeWindow.intersects, touching
// counts) merge, combining their accumulators (AggregateFunction.merge, chapter2/README.md:145).
// A session fires when the watermark passes end - 1; with allowed lateness it stays until
// end - 1 + lateness, and a late element merged into a fired session fires it again.
//
// Roles:
//  * the CPU engine for session windows (device = cpu), and
//  * the host-DRAM spill tier of the GPU session operator: keys evicted from HBM live here and
//    their records are diverted here (BASELINE config 5, "host-DRAM state spill").
//
// Two tiers inside the store:
//  * hot: key -> sessions map with a due-time heap (elements, merging, firing);
//  * cold: columnar chunks of spilled sessions that already fired and were not modified since
//    (the common case for idle keys: they only wait for their cleanup time). A chunk is one
//    eviction batch; it is dropped as a whole once every row is past cleanup. A record that
//    arrives for a key with cold rows promotes them into the hot map first (rows already past
//    cleanup at that point are discarded, exactly as if they had been cleaned on time).
// Keys that leave the store are reported by fire() so the device spill set can forget them.
//
// Micro-batch semantics (shared with the GPU kernels): a batch's elements of one key are merged
// in timestamp order; a run of elements closer than `gap` becomes one candidate session, which
// is dropped as late only if it is late on its own and merges with no live session.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <climits>

#include "session_shards.h"

namespace py = pybind11;

namespace mxs {
namespace {

using I64Array = py::array_t<int64_t, py::array::c_style>;

template <class T>
py::array_t<T> to_np(const std::vector<T>& v) {
  return py::array_t<T>((py::ssize_t)v.size(), v.data());
}

py::dict columns_dict(const sess::Columns& c) {
  py::dict d;
  d["key"] = to_np(c.key);
  d["start"] = to_np(c.start);
  d["end"] = to_np(c.end);
  d["acc"] = to_np(c.acc);
  d["cnt"] = to_np(c.cnt);
  d["flags"] = to_np(c.flags);
  return d;
}

void same_len(int64_t n, std::initializer_list<int64_t> sizes) {
  for (int64_t s : sizes)
    if (s != n) throw std::invalid_argument("length mismatch");
}

// NumPy adapter of the store core (csrc/session_store.h).
class SessionStore {
 public:
  // shards > 1: key shards worked in parallel by a persistent pool (csrc/session_shards.h)
  SessionStore(int64_t gap, int64_t lateness, int agg, int shards = 1)
      : c_(gap, lateness, agg, shards) {}
  int shards() const { return c_.shards(); }

  // Fold a batch (keys, ts, vals) with the current watermark `wm`; returns late-dropped count.
  int64_t process_np(const I64Array& keys, const I64Array& ts, const I64Array& vals, int64_t wm) {
    same_len(keys.size(), {ts.size(), vals.size()});
    return c_.process(keys.data(), ts.data(), vals.data(), keys.size(), wm);
  }
  // Merge pre-built runs (GPU overflow path): each is a candidate session.
  int64_t merge_runs_np(const I64Array& keys, const I64Array& starts, const I64Array& ends,
                        const I64Array& accs, const I64Array& cnts, int64_t wm) {
    same_len(keys.size(), {starts.size(), ends.size(), accs.size(), cnts.size()});
    return c_.merge_runs(keys.data(), starts.data(), ends.data(), accs.data(), cnts.data(),
                      keys.size(), wm);
  }
  // Arguments by const reference: the call runs without the GIL, so no Python object may be
  // created or released inside it.
  void insert_np(const I64Array& keys, const I64Array& starts, const I64Array& ends,
                 const I64Array& accs, const I64Array& cnts, const I64Array& flags, bool cold) {
    same_len(keys.size(), {starts.size(), ends.size(), accs.size(), cnts.size(), flags.size()});
    c_.insert(keys.data(), starts.data(), ends.data(), accs.data(), cnts.data(), flags.data(),
           keys.size(), cold);
  }
  py::dict extract_np(const I64Array& keys, int64_t wm, int64_t max_sess) {
    std::vector<int64_t> moved;
    py::dict d = columns_dict(c_.extract(keys.data(), keys.size(), wm, max_sess, &moved));
    d["moved"] = to_np(moved);
    return d;
  }
  // extract() laid out for the HBM slot records in one pass (the promote path's assembly):
  // "key" = the distinct keys that got sessions back (ascending), "rec" = [key][max_sess][4]
  // int64 slot records {start, end, acc, cnt | flags << 32} (unused positions zero), "last" =
  // each key's last activity (max end - gap), "moved" = as extract().
  py::dict extract_packed_np(const I64Array& keys, int64_t wm, int64_t max_sess, int64_t gap) {
    std::vector<int64_t> moved, ukey, rec, last;
    {
      py::gil_scoped_release nogil;
      const sess::Columns c = c_.extract(keys.data(), keys.size(), wm, max_sess, &moved);
      const size_t n = c.key.size();
      int64_t pos = 0;
      for (size_t i = 0; i < n; ++i) {
        if (i == 0 || c.key[i] != c.key[i - 1]) {
          ukey.push_back(c.key[i]);
          rec.resize(rec.size() + (size_t)max_sess * 4, 0);
          last.push_back(INT64_MIN);
          pos = 0;
        }
        if (pos >= max_sess) throw std::logic_error("extract_packed: more sessions than a slot");
        int64_t* r = rec.data() + ((ukey.size() - 1) * (size_t)max_sess + (size_t)pos) * 4;
        r[0] = c.start[i];
        r[1] = c.end[i];
        r[2] = c.acc[i];
        r[3] = (int64_t)(((uint64_t)c.cnt[i] & 0xFFFFFFFFull) | ((uint64_t)c.flags[i] << 32));
        last.back() = std::max(last.back(), c.end[i] - gap);
        ++pos;
      }
    }
    py::dict d;
    d["key"] = to_np(ukey);
    d["rec"] = to_np(rec);
    d["last"] = to_np(last);
    d["moved"] = to_np(moved);
    return d;
  }
  // Fire / clean up everything the watermark allows. Returns columns of emitted rows plus the
  // keys that left the store ("released").
  py::dict fire_np(int64_t wm, std::vector<int32_t> map_code, std::vector<double> map_consts,
                   std::vector<int32_t> f_code, std::vector<double> f_consts, bool expire) {
    sess::SessionCore::FireOut o;
    c_.fire(wm, sess::SessionCore::prog(map_code.data(), map_code.size(), map_consts.data(), map_consts.size()),
         sess::SessionCore::prog(f_code.data(), f_code.size(), f_consts.data(), f_consts.size()), o, expire);
    py::dict d;
    d["keys"] = to_np(o.okey);
    d["start"] = to_np(o.ostart);
    d["end"] = to_np(o.oend);
    d["values"] = to_np(o.oval);
    d["raw"] = to_np(o.oraw);
    d["counts"] = to_np(o.ocnt);
    d["refire"] = to_np(o.oref);
    d["released"] = to_np(o.released);
    return d;
  }
  // Cold-chunk expiry alone (GIL released: the GPU operator's spill worker runs it).
  py::array_t<int64_t> expire_cold_np(int64_t wm) {
    std::vector<int64_t> rel;
    {
      py::gil_scoped_release nogil;
      c_.expire_cold(wm, rel);
    }
    return to_np(rel);
  }
  py::array_t<int64_t> spill_set_np(int cap_log2) const {
    py::array_t<int64_t> out((py::ssize_t)1 << cap_log2);
    c_.spill_set(cap_log2, out.mutable_data());
    return out;
  }
  py::array_t<int64_t> key_list_np() const { return to_np(c_.key_list()); }
  py::dict snapshot_np() const { return columns_dict(c_.snapshot()); }
  bool contains(uint64_t key) const { return c_.contains(key); }
  size_t num_keys() const { return c_.num_keys(); }
  size_t num_sessions() const { return c_.num_sessions(); }
  size_t num_cold_rows() const { return c_.num_cold_rows(); }
  size_t bytes() const { return c_.bytes(); }

 private:
  sess::ShardedCore c_;
};

}  // namespace
}  // namespace mxs

void bind_sessions(py::module_& m) {
  using mxs::SessionStore;
  py::class_<SessionStore>(m, "SessionStore")
      .def(py::init<int64_t, int64_t, int, int>(), py::arg("gap"), py::arg("lateness"),
           py::arg("agg"), py::arg("shards") = 1)
      .def_property_readonly("shards", &SessionStore::shards)
      .def("process", &SessionStore::process_np)
      // GIL released: the operator inserts spilled rows from a worker thread while the main
      // thread keeps launching the next step's kernels (the store is not touched concurrently).
      .def("insert", &SessionStore::insert_np, py::arg("keys"), py::arg("starts"),
           py::arg("ends"), py::arg("accs"), py::arg("cnts"), py::arg("flags"),
           py::arg("cold") = false, py::call_guard<py::gil_scoped_release>())
      .def("merge_runs", &SessionStore::merge_runs_np)
      .def("extract", &SessionStore::extract_np)
      .def("extract_packed", &SessionStore::extract_packed_np)
      .def("fire", &SessionStore::fire_np, py::arg("wm"), py::arg("map_code"),
           py::arg("map_consts"), py::arg("f_code"), py::arg("f_consts"),
           py::arg("expire_cold") = true)
      .def("expire_cold", &SessionStore::expire_cold_np)
      .def("spill_set", &SessionStore::spill_set_np)
      .def("contains", &SessionStore::contains)
      .def("num_keys", &SessionStore::num_keys)
      .def("num_sessions", &SessionStore::num_sessions)
      .def("num_cold_rows", &SessionStore::num_cold_rows)
      .def("bytes", &SessionStore::bytes)
      .def("key_list", &SessionStore::key_list_np)
      .def("snapshot", &SessionStore::snapshot_np);
}
