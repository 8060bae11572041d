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
// Micro-batch semantics (shared with the GPU kernels): a batch's elements of one key are merged
// in timestamp order; a run of elements closer than `gap` becomes one candidate session, which
// is dropped as late only if it is late on its own and merges with no live session.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <queue>
#include <unordered_map>
#include <vector>

#include "mxs_common.h"

namespace py = pybind11;

namespace mxs {
namespace {

struct Session {
  int64_t start, end;  // [start, end)
  uint64_t acc;
  uint32_t cnt;
  uint32_t flags;      // bit0: fired, bit1: modified since firing
};

class SessionStore {
 public:
  SessionStore(int64_t gap, int64_t lateness, int agg) : gap_(gap), late_(lateness), agg_(agg) {
    if (gap <= 0) throw std::invalid_argument("session gap must be > 0");
  }

  // Fold a batch (keys, ts, vals) with the current watermark `wm`; returns late-dropped count.
  int64_t process(py::array_t<int64_t, py::array::c_style> keys,
                  py::array_t<int64_t, py::array::c_style> ts,
                  py::array_t<int64_t, py::array::c_style> vals, int64_t wm) {
    const int64_t n = keys.size();
    if (ts.size() != n || vals.size() != n) throw std::invalid_argument("length mismatch");
    const int64_t* k = keys.data();
    const int64_t* t = ts.data();
    const int64_t* v = vals.data();
    std::vector<int64_t> idx(n);
    for (int64_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
      return k[a] != k[b] ? k[a] < k[b] : t[a] < t[b];
    });
    int64_t late = 0;
    int64_t i = 0;
    while (i < n) {
      const uint64_t key = (uint64_t)k[idx[i]];
      int64_t j = i;
      while (j < n && (uint64_t)k[idx[j]] == key) ++j;
      // runs of this key
      int64_t r = i;
      while (r < j) {
        Session c{t[idx[r]], t[idx[r]] + gap_, agg_lift(agg_, (uint64_t)v[idx[r]]), 1u, 0u};
        int64_t q = r + 1;
        while (q < j && t[idx[q]] <= c.end) {  // intersects (touching merges)
          c.end = std::max(c.end, t[idx[q]] + gap_);
          c.acc = agg_combine(agg_, c.acc, agg_lift(agg_, (uint64_t)v[idx[q]]));
          c.cnt += 1;
          ++q;
        }
        late += merge_candidate(key, c, wm);
        r = q;
      }
      i = j;
    }
    return late;
  }

  // Merge pre-built runs (GPU overflow path): each is a candidate session.
  int64_t merge_runs(py::array_t<int64_t, py::array::c_style> keys, py::array_t<int64_t> starts,
                     py::array_t<int64_t> ends, py::array_t<int64_t> accs,
                     py::array_t<int64_t> cnts, int64_t wm) {
    const int64_t n = keys.size();
    int64_t late = 0;
    for (int64_t i = 0; i < n; ++i) {
      Session c{starts.data()[i], ends.data()[i], (uint64_t)accs.data()[i],
                (uint32_t)cnts.data()[i], 0u};
      late += merge_candidate((uint64_t)keys.data()[i], c, wm);
    }
    return late;
  }

  // Insert sessions evicted from HBM (spill). Arrays: key, start, end, acc, cnt, flags.
  void insert(py::array_t<int64_t, py::array::c_style> keys, py::array_t<int64_t> starts,
              py::array_t<int64_t> ends, py::array_t<int64_t> accs, py::array_t<int64_t> cnts,
              py::array_t<int64_t> flags) {
    const int64_t n = keys.size();
    auto K = keys.data();
    auto S = starts.data();
    auto E = ends.data();
    auto A = accs.data();
    auto C = cnts.data();
    auto F = flags.data();
    for (int64_t i = 0; i < n; ++i) {
      auto& vec = m_[(uint64_t)K[i]];
      vec.push_back(Session{S[i], E[i], (uint64_t)A[i], (uint32_t)C[i], (uint32_t)F[i]});
      schedule((uint64_t)K[i]);
    }
  }

  // Fire / clean up everything the watermark allows. Returns columns of emitted rows.
  py::dict fire(int64_t wm, std::vector<int32_t> map_code, std::vector<double> map_consts,
                std::vector<int32_t> f_code, std::vector<double> f_consts) {
    ExprProg mp = prog(map_code, map_consts), fp = prog(f_code, f_consts);
    std::vector<int64_t> okey, ostart, oend, oraw, ocnt, oref;
    std::vector<double> oval;
    while (!heap_.empty() && heap_.top().first <= wm) {
      const uint64_t key = heap_.top().second;
      heap_.pop();
      auto it = m_.find(key);
      if (it == m_.end()) continue;
      auto& vec = it->second;
      std::vector<Session> keep;
      for (auto& s : vec) {
        const int64_t maxts = s.end - 1;
        if (maxts <= wm && (!(s.flags & 1u) || (s.flags & 2u))) {
          double vars[kExprVars] = {0};
          vars[0] = agg_result_f64(agg_, s.acc, s.cnt);
          vars[1] = (double)s.cnt;
          vars[2] = (double)s.start;
          vars[3] = (double)s.end;
          vars[4] = (double)key;
          vars[5] = (double)(int64_t)s.acc;
          vars[6] = mp.ncode ? expr_eval(mp, vars) : vars[0];
          if (!fp.ncode || expr_eval(fp, vars) != 0.0) {
            okey.push_back((int64_t)key);
            ostart.push_back(s.start);
            oend.push_back(s.end);
            oval.push_back(vars[6]);
            oraw.push_back((int64_t)s.acc);
            ocnt.push_back(s.cnt);
            oref.push_back((s.flags & 1u) ? 1 : 0);
          }
          s.flags = 1u;
        }
        if (maxts + late_ > wm || maxts + late_ < maxts) keep.push_back(s);  // not cleaned yet
      }
      if (keep.empty()) {
        m_.erase(it);
      } else {
        vec.swap(keep);
        schedule(key);
      }
    }
    py::dict d;
    d["keys"] = py::array_t<int64_t>((py::ssize_t)okey.size(), okey.data());
    d["start"] = py::array_t<int64_t>((py::ssize_t)ostart.size(), ostart.data());
    d["end"] = py::array_t<int64_t>((py::ssize_t)oend.size(), oend.data());
    d["values"] = py::array_t<double>((py::ssize_t)oval.size(), oval.data());
    d["raw"] = py::array_t<int64_t>((py::ssize_t)oraw.size(), oraw.data());
    d["counts"] = py::array_t<int64_t>((py::ssize_t)ocnt.size(), ocnt.data());
    d["refire"] = py::array_t<int64_t>((py::ssize_t)oref.size(), oref.data());
    return d;
  }

  // Device spill set (open addressing on mix64(key) >> 32, linear probing, empty = ~0) holding
  // every key of this store: records of these keys are diverted from HBM to the host tier.
  py::array_t<int64_t> spill_set(int cap_log2) const {
    const size_t cap = (size_t)1 << cap_log2;
    if (m_.size() * 2 > cap) throw std::invalid_argument("spill set too small");
    py::array_t<int64_t> out((py::ssize_t)cap);
    int64_t* d = out.mutable_data();
    std::fill(d, d + cap, (int64_t)kEmptyKey);
    const uint32_t mask = (uint32_t)(cap - 1);
    for (auto& kv : m_) {
      uint32_t s = (uint32_t)(mix64(kv.first) >> 32) & mask;
      while ((uint64_t)d[s] != kEmptyKey) s = (s + 1) & mask;
      d[s] = (int64_t)kv.first;
    }
    return out;
  }

  bool contains(uint64_t key) const { return m_.count(key) != 0; }
  size_t num_keys() const { return m_.size(); }
  size_t num_sessions() const {
    size_t s = 0;
    for (auto& kv : m_) s += kv.second.size();
    return s;
  }
  size_t bytes() const { return num_sessions() * sizeof(Session) + m_.size() * 48; }

  py::array_t<int64_t> key_list() const {
    std::vector<int64_t> k;
    k.reserve(m_.size());
    for (auto& kv : m_) k.push_back((int64_t)kv.first);
    return py::array_t<int64_t>((py::ssize_t)k.size(), k.data());
  }

  // Snapshot: flat columns (key, start, end, acc, cnt, flags).
  py::dict snapshot() const {
    std::vector<int64_t> k, s, e, a, c, f;
    for (auto& kv : m_)
      for (auto& x : kv.second) {
        k.push_back((int64_t)kv.first);
        s.push_back(x.start);
        e.push_back(x.end);
        a.push_back((int64_t)x.acc);
        c.push_back(x.cnt);
        f.push_back(x.flags);
      }
    py::dict d;
    d["key"] = py::array_t<int64_t>((py::ssize_t)k.size(), k.data());
    d["start"] = py::array_t<int64_t>((py::ssize_t)s.size(), s.data());
    d["end"] = py::array_t<int64_t>((py::ssize_t)e.size(), e.data());
    d["acc"] = py::array_t<int64_t>((py::ssize_t)a.size(), a.data());
    d["cnt"] = py::array_t<int64_t>((py::ssize_t)c.size(), c.data());
    d["flags"] = py::array_t<int64_t>((py::ssize_t)f.size(), f.data());
    return d;
  }

 private:
  static ExprProg prog(const std::vector<int32_t>& code, const std::vector<double>& consts) {
    ExprProg p;
    std::memset(&p, 0, sizeof(p));
    if (code.size() > (size_t)2 * kExprMaxCode || consts.size() > (size_t)kExprMaxConst)
      throw std::invalid_argument("expr program too large");
    for (size_t i = 0; i < code.size(); ++i) p.code[i] = code[i];
    for (size_t i = 0; i < consts.size(); ++i) p.consts[i] = consts[i];
    p.ncode = (int32_t)(code.size() / 2);
    return p;
  }

  // Merge candidate c into key's sessions; returns the number of late-dropped elements.
  int64_t merge_candidate(uint64_t key, Session c, int64_t wm) {
    auto& vec = m_[key];
    Session merged = c;
    bool touched_existing = false;
    std::vector<Session> rest;
    for (auto& s : vec) {
      if (merged.start <= s.end && merged.end >= s.start) {
        merged.start = std::min(merged.start, s.start);
        merged.end = std::max(merged.end, s.end);
        merged.acc = agg_combine(agg_, s.acc, merged.acc);
        merged.cnt += s.cnt;
        merged.flags |= s.flags;
        touched_existing = true;
      } else {
        rest.push_back(s);
      }
    }
    const int64_t maxts = merged.end - 1;
    if (!touched_existing && maxts + late_ <= wm) {
      if (vec.empty()) m_.erase(key);
      return c.cnt;  // late: every window of these elements is already cleaned
    }
    // A fired session that grows (or a new session already past its end within lateness)
    // fires again at the next fire() with the watermark (EventTimeTrigger.onElement).
    if (merged.flags & 1u) merged.flags |= 2u;
    rest.push_back(merged);
    vec.swap(rest);
    schedule(key);
    return 0;
  }

  void schedule(uint64_t key) {
    auto it = m_.find(key);
    if (it == m_.end()) return;
    int64_t t = INT64_MAX;
    for (auto& s : it->second) {
      const int64_t maxts = s.end - 1;
      const int64_t due = ((s.flags & 1u) && !(s.flags & 2u)) ? maxts + late_ : maxts;
      t = std::min(t, due);
    }
    heap_.push({t, key});
  }

  int64_t gap_, late_;
  int agg_;
  std::unordered_map<uint64_t, std::vector<Session>> m_;
  std::priority_queue<std::pair<int64_t, uint64_t>, std::vector<std::pair<int64_t, uint64_t>>,
                      std::greater<>>
      heap_;
};

}  // namespace
}  // namespace mxs

void bind_sessions(py::module_& m) {
  using mxs::SessionStore;
  py::class_<SessionStore>(m, "SessionStore")
      .def(py::init<int64_t, int64_t, int>(), py::arg("gap"), py::arg("lateness"), py::arg("agg"))
      .def("process", &SessionStore::process)
      .def("insert", &SessionStore::insert)
      .def("merge_runs", &SessionStore::merge_runs)
      .def("fire", &SessionStore::fire)
      .def("spill_set", &SessionStore::spill_set)
      .def("contains", &SessionStore::contains)
      .def("num_keys", &SessionStore::num_keys)
      .def("num_sessions", &SessionStore::num_sessions)
      .def("bytes", &SessionStore::bytes)
      .def("key_list", &SessionStore::key_list)
      .def("snapshot", &SessionStore::snapshot);
}
