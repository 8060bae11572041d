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
#include <cstdio>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

#include "session_shards.h"

namespace py = pybind11;

namespace mxs {
namespace {

using I64Array = py::array_t<int64_t, py::array::c_style>;

template <class T>
py::array_t<T> to_np(const std::vector<T>& v) {
  return py::array_t<T>((py::ssize_t)v.size(), v.data());
}
// The vector's buffer handed to NumPy without a copy (the array owns it through a capsule).
template <class T>
py::array_t<T> to_np_move(std::vector<T>&& v) {
  if (v.empty()) return py::array_t<T>(0);
  auto* h = new std::vector<T>(std::move(v));
  py::capsule own(h, [](void* p) { delete static_cast<std::vector<T>*>(p); });
  return py::array_t<T>((py::ssize_t)h->size(), h->data(), own);
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

// The GPU operator's idle-key eviction, off the interpreter (the per-eviction
// Python thread): a persistent C++ worker owned by the store. spill_submit() records a HIP event
// behind the counted D2H of the evicted rows and queues the job; the worker waits for the event
// (blocking sync, no spin), classifies the rows and inserts the hot ones under the store lock,
// copies the cold rows into a chunk WITHOUT the lock, publishes the chunk and expires dead cold
// chunks under the lock again. The main thread never waits for the cold copy: fire() waits only
// for the hot phase of every submitted job (rows that may still fire must be in the map), and
// the calls that read cold rows (extract, snapshot, key counts, ...) join the worker first.
// Results (rows, evicted slots, keys, released keys) are collected by spill_poll / spill_join.
struct SpillJob {
  uint64_t id = 0;
  hipEvent_t ev = nullptr;  // null: the rows are already in host memory (CPU tests)
  const uint8_t* slab = nullptr;
  int64_t ctr_off = 0;      // int32 counters: [7] rows written (may exceed R), [8] slots evicted
  int64_t col_off[6] = {0, 0, 0, 0, 0, 0};  // int64 key, start, end, acc, cnt, flags (R rows)
  int64_t R = 0;
  bool expire = false;
  int64_t expire_wm = INT64_MIN;
};

struct SpillDone {
  uint64_t id = 0;
  int64_t nr = 0, ne = 0, nk = 0;
  int64_t n_hot = 0;       // rows that went to the hot map (not fired-unmodified or key hot)
  int64_t hot_keys = 0;    // hot map size after the insert (0: the all-cold fast path applies)
  double t_populate = 0;   // s: of t_index, the synchronous index page population
  std::vector<int64_t> released;
  double t_wait = 0, t_hot = 0, t_build = 0, t_index = 0, t_publish = 0, t_expire = 0;  // s
  std::exception_ptr err;
};

// NumPy adapter of the store core (csrc/session_store.h).
class SessionStore {
 public:
  // shards > 1: key shards worked in parallel by a persistent pool (csrc/session_shards.h)
  SessionStore(int64_t gap, int64_t lateness, int agg, int shards = 1)
      : c_(gap, lateness, agg, shards) {}
  ~SessionStore() {
    if (th_.joinable()) {
      {
        std::lock_guard<std::mutex> g(qmu_);
        stop_ = true;
      }
      qcv_.notify_all();
      th_.join();
    }
    for (hipEvent_t e : free_ev_) (void)hipEventDestroy(e);
  }
  int shards() const { return c_.shards(); }

  // Fold a batch (keys, ts, vals) with the current watermark `wm`; returns late-dropped count.
  int64_t process_np(const I64Array& keys, const I64Array& ts, const I64Array& vals, int64_t wm) {
    same_len(keys.size(), {ts.size(), vals.size()});
    auto g = joined();
    return c_.process(keys.data(), ts.data(), vals.data(), keys.size(), wm);
  }
  // Merge pre-built runs (GPU overflow path): each is a candidate session.
  int64_t merge_runs_np(const I64Array& keys, const I64Array& starts, const I64Array& ends,
                        const I64Array& accs, const I64Array& cnts, int64_t wm) {
    same_len(keys.size(), {starts.size(), ends.size(), accs.size(), cnts.size()});
    auto g = joined();
    return c_.merge_runs(keys.data(), starts.data(), ends.data(), accs.data(), cnts.data(),
                      keys.size(), wm);
  }
  // Arguments by const reference: the call runs without the GIL, so no Python object may be
  // created or released inside it.
  void insert_np(const I64Array& keys, const I64Array& starts, const I64Array& ends,
                 const I64Array& accs, const I64Array& cnts, const I64Array& flags, bool cold) {
    same_len(keys.size(), {starts.size(), ends.size(), accs.size(), cnts.size(), flags.size()});
    auto g = joined_nogil();
    c_.insert(keys.data(), starts.data(), ends.data(), accs.data(), cnts.data(), flags.data(),
           keys.size(), cold);
  }
  py::dict extract_np(const I64Array& keys, int64_t wm, int64_t max_sess) {
    std::vector<int64_t> moved;
    auto g = joined();
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
      join_all();
      std::lock_guard<std::mutex> g(mu_);
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
  // The promote path's extract straight into caller memory (pinned, reused): promote rows of
  // 8 int64 (csrc/session_store.h extract_rows_into) at `rows` (cap rows) and the keys that left
  // the store at `moved` (moved_cap); `keys` may repeat. Returns (rows, moved, distinct keys).
  std::tuple<int64_t, int64_t, int64_t> extract_rows_into_np(const I64Array& keys, int64_t wm,
                                                             int64_t max_sess, int64_t gap,
                                                             intptr_t rows, int64_t cap,
                                                             intptr_t moved, int64_t moved_cap) {
    py::gil_scoped_release nogil;
    join_all();
    std::lock_guard<std::mutex> g(mu_);
    const auto r = c_.extract_rows_into(keys.data(), keys.size(), wm, max_sess, gap,
                                        reinterpret_cast<int64_t*>(rows), cap,
                                        reinterpret_cast<int64_t*>(moved), moved_cap);
    // The promote kernel writes record `position` of a slot: never past the slot's kSess. Both
    // extract paths bound a key's sessions by max_sess BEFORE the key leaves the store
    // (take_indexed_with's limit; extract() keeps a key with more on the host), so this is an
    // invariant: a violation means the store is already inconsistent, and the keys are gone --
    // no exception could hand the state back, so it stops the process (an assertion).
    const int64_t* w = reinterpret_cast<const int64_t*>(rows);
    for (int64_t i = 0; i < std::get<0>(r); ++i)
      if (w[i * 8 + 7] > max_sess || w[i * 8 + 6] >= w[i * 8 + 7]) {
        std::fprintf(stderr, "mxstream: extract_rows_into: session position out of range "
                             "(row %lld: %lld of %lld, max %lld)\n", (long long)i,
                     (long long)w[i * 8 + 6], (long long)w[i * 8 + 7], (long long)max_sess);
        std::abort();
      }
    return r;
  }
  // The dense cold-row index's counters (csrc/session_store.h IndexStats) summed over shards.
  py::dict index_stats() {
    sess::SessionCore::IndexStats t;
    {
      auto g = joined_nogil();
      t = c_.index_stats();
    }
    py::dict d;
    d["indexed_takes"] = t.indexed;
    d["multi_aborts"] = t.multi;
    d["hot_aborts"] = t.hot;
    d["scans"] = t.scans;
    d["off"] = t.off;
    d["span"] = t.span;
    return d;
  }
  // Fire / clean up everything the watermark allows. Returns columns of emitted rows plus the
  // keys that left the store ("released"). Waits only for the hot phase of queued evictions --
  // of jobs up to `hot_upto` when >= 0 (later ones evicted sessions the GPU fire already saw).
  py::dict fire_np(int64_t wm, std::vector<int32_t> map_code, std::vector<double> map_consts,
                   std::vector<int32_t> f_code, std::vector<double> f_consts, bool expire,
                   int64_t hot_upto) {
    sess::SessionCore::FireOut o;
    {
      py::gil_scoped_release nogil;
      if (expire) join_all();
      else wait_hot(hot_upto);
      std::lock_guard<std::mutex> g(mu_);
      c_.fire(wm, sess::SessionCore::prog(map_code.data(), map_code.size(), map_consts.data(), map_consts.size()),
           sess::SessionCore::prog(f_code.data(), f_code.size(), f_consts.data(), f_consts.size()), o, expire);
    }
    py::dict d;  // the columns' buffers handed over, not copied
    d["keys"] = to_np_move(std::move(o.okey));
    d["start"] = to_np_move(std::move(o.ostart));
    d["end"] = to_np_move(std::move(o.oend));
    d["values"] = to_np_move(std::move(o.oval));
    d["raw"] = to_np_move(std::move(o.oraw));
    d["counts"] = to_np_move(std::move(o.ocnt));
    d["refire"] = to_np_move(std::move(o.oref));
    d["released"] = to_np_move(std::move(o.released));
    return d;
  }
  // Cold-chunk expiry alone (GIL released).
  py::array_t<int64_t> expire_cold_np(int64_t wm) {
    std::vector<int64_t> rel;
    {
      auto g = joined_nogil();
      c_.expire_cold(wm, rel);
    }
    return to_np(rel);
  }
  py::array_t<int64_t> spill_set_np(int cap_log2) {
    py::array_t<int64_t> out((py::ssize_t)1 << cap_log2);
    auto g = joined();
    c_.spill_set(cap_log2, out.mutable_data());
    return out;
  }
  py::array_t<int64_t> key_list_np() {
    auto g = joined();
    return to_np(c_.key_list());
  }
  // extra > 0: every column gets `extra` more rows after the store's, left for the caller to
  // fill (the HBM tier's rows: no concatenation afterwards).
  py::dict snapshot_np(int64_t extra) {
    if (extra < 0) throw std::invalid_argument("extra < 0");
    auto g = joined();
    // The shards build their rows in parallel, then copy them into the numpy columns in
    // parallel, without the GIL (one thread concatenating the shards' vectors and a second copy
    // out to numpy took most of a 10M-row snapshot).
    std::vector<sess::Columns> parts;
    {
      py::gil_scoped_release nogil;
      parts = c_.snapshot_parts();
    }
    std::vector<size_t> offs(parts.size() + 1, 0);
    for (size_t i = 0; i < parts.size(); ++i) offs[i + 1] = offs[i] + parts[i].key.size();
    static const char* names[6] = {"key", "start", "end", "acc", "cnt", "flags"};
    py::dict d;
    int64_t* cols[6];
    for (int c = 0; c < 6; ++c) {
      I64Array a((py::ssize_t)(offs.back() + (size_t)extra));
      cols[c] = a.mutable_data();
      d[names[c]] = a;
    }
    {
      py::gil_scoped_release nogil;
      c_.each([&](int s) {
        const sess::Columns& p = parts[s];
        const std::vector<int64_t>* src[6] = {&p.key, &p.start, &p.end, &p.acc, &p.cnt, &p.flags};
        for (int c = 0; c < 6; ++c)
          if (!src[c]->empty())
            std::memcpy(cols[c] + offs[s], src[c]->data(), src[c]->size() * sizeof(int64_t));
      });
    }
    return d;
  }
  bool contains(uint64_t key) {
    auto g = joined();
    return c_.contains(key);
  }
  size_t num_keys() {
    auto g = joined();
    return c_.num_keys();
  }
  size_t num_sessions() {
    auto g = joined();
    return c_.num_sessions();
  }
  size_t num_cold_rows() {
    auto g = joined();
    return c_.num_cold_rows();
  }
  size_t bytes() {
    auto g = joined();
    return c_.bytes();
  }

  // ---- asynchronous eviction (GPU operator) ---------------------------------------------------
  // stream >= 0: a HIP stream handle whose queued work (the counted D2H into `slab`) must finish
  // before the rows are read; < 0: the rows are already there. Returns the job id (1, 2, ...).
  uint64_t spill_submit(int64_t stream, uintptr_t slab, int64_t ctr_off, std::vector<int64_t> col_off,
                        int64_t R, py::object expire_wm) {
    if (col_off.size() != 6) throw std::invalid_argument("spill_submit: 6 column offsets");
    SpillJob j;
    j.slab = reinterpret_cast<const uint8_t*>(slab);
    j.ctr_off = ctr_off;
    for (int k = 0; k < 6; ++k) j.col_off[k] = col_off[k];
    j.R = R;
    j.expire = !expire_wm.is_none();
    if (j.expire) j.expire_wm = expire_wm.cast<int64_t>();
    py::gil_scoped_release nogil;
    if (stream >= 0) {
      {
        std::lock_guard<std::mutex> g(qmu_);
        if (!free_ev_.empty()) {
          j.ev = free_ev_.back();
          free_ev_.pop_back();
        }
      }
      if (!j.ev && hipEventCreateWithFlags(&j.ev, hipEventDisableTiming | hipEventBlockingSync) !=
                       hipSuccess)
        throw std::runtime_error("spill_submit: hipEventCreate failed");
      if (hipEventRecord(j.ev, reinterpret_cast<hipStream_t>(stream)) != hipSuccess) {
        std::lock_guard<std::mutex> g(qmu_);
        free_ev_.push_back(j.ev);  // the event goes back to the pool, not leaked
        throw std::runtime_error("spill_submit: hipEventRecord failed");
      }
    }
    std::lock_guard<std::mutex> g(qmu_);
    if (!th_.joinable()) th_ = std::thread([this] { worker(); });
    j.id = ++submitted_;
    q_.push_back(j);
    qcv_.notify_all();
    return j.id;
  }
  uint64_t spill_submitted() const { return submitted_; }
  uint64_t spill_completed() {
    std::lock_guard<std::mutex> g(qmu_);
    return completed_;
  }
  // Completed jobs' results (non-blocking); the first failed job's error is raised.
  py::list spill_poll() { return take_results(); }
  // Every submitted job completed (GIL released while waiting), then as spill_poll.
  py::list spill_join() {
    {
      py::gil_scoped_release nogil;
      join_all();
    }
    return take_results();
  }

 private:
  struct Guard {
    std::unique_lock<std::mutex> lk;
  };
  // Join the worker, then hold the store lock for the caller's scope (the GIL is held: for calls
  // that build Python objects under it; the wait itself releases it).
  Guard joined() {
    {
      py::gil_scoped_release nogil;
      join_all();
    }
    return Guard{std::unique_lock<std::mutex>(mu_)};
  }
  Guard joined_nogil() {
    join_all();
    return Guard{std::unique_lock<std::mutex>(mu_)};
  }
  void join_all() {
    std::unique_lock<std::mutex> lk(qmu_);
    dcv_.wait(lk, [&] { return completed_ == submitted_; });
  }
  void wait_hot(int64_t upto = -1) {  // jobs finish their hot phase in id order
    std::unique_lock<std::mutex> lk(qmu_);
    dcv_.wait(lk, [&] { return hot_done_ >= (upto < 0 ? submitted_ : (uint64_t)upto); });
  }
  py::list take_results() {
    std::deque<SpillDone> done;
    {
      std::lock_guard<std::mutex> g(qmu_);
      done.swap(done_);
    }
    if (!done.empty()) {
      // A released key that has hot sessions again (a host fold after the expiry) must stay in
      // the device spill set: dropped from the list here, under the store lock.
      py::gil_scoped_release nogil;
      std::lock_guard<std::mutex> g(mu_);
      if (!c_.hot_free())  // (no hot sessions at all -- the common case: nothing to drop)
        for (auto& d : done) {
          size_t w = 0;
          for (int64_t k : d.released)
            if (!c_.hot((uint64_t)k)) d.released[w++] = k;
          d.released.resize(w);
        }
    }
    py::list out;
    std::exception_ptr err;
    for (auto& d : done) {
      if (d.err && !err) err = d.err;
      py::dict r;
      r["id"] = d.id;
      r["nr"] = d.nr;
      r["ne"] = d.ne;
      r["nk"] = d.nk;
      r["released"] = to_np_move(std::move(d.released));
      r["t_wait"] = d.t_wait;
      r["t_hot"] = d.t_hot;
      r["t_build"] = d.t_build;
      r["t_index"] = d.t_index;
      r["t_publish"] = d.t_publish;
      r["t_expire"] = d.t_expire;
      r["n_hot"] = d.n_hot;
      r["t_populate"] = d.t_populate;
      r["hot_keys"] = d.hot_keys;
      out.append(r);
    }
    if (err) std::rethrow_exception(err);
    return out;
  }
  void worker() {
    using clk = std::chrono::steady_clock;
    auto sec = [](clk::time_point a, clk::time_point b) {
      return std::chrono::duration<double>(b - a).count();
    };
    for (;;) {
      SpillJob j;
      {
        std::unique_lock<std::mutex> lk(qmu_);
        qcv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop_
        j = q_.front();
        q_.pop_front();
      }
      SpillDone d;
      d.id = j.id;
      bool hot_marked = false;
      try {
        const auto t0 = clk::now();
        if (j.ev && hipEventSynchronize(j.ev) != hipSuccess)
          throw std::runtime_error("spill worker: hipEventSynchronize failed");
        const auto t1 = clk::now();
        const int32_t* ctr = reinterpret_cast<const int32_t*>(j.slab + j.ctr_off);
        const int64_t nr_all = ctr[7];
        d.ne = ctr[8];
        int64_t nr = std::min<int64_t>(nr_all, j.R);
        const int64_t* col[6];
        for (int k = 0; k < 6; ++k) col[k] = reinterpret_cast<const int64_t*>(j.slab + j.col_off[k]);
        std::vector<int64_t> tmp[6];
        if (nr_all > j.R) {  // staging overflowed: rows of skipped slots stay zero (cnt == 0)
          for (int64_t i = 0; i < nr; ++i)
            if (col[4][i] > 0)
              for (int k = 0; k < 6; ++k) tmp[k].push_back(col[k][i]);
          for (int k = 0; k < 6; ++k) col[k] = tmp[k].data();
          nr = (int64_t)tmp[0].size();
        }
        d.nr = nr;
        sess::SessionCore::ColdPlan plan;
        sess::SessionCore* one = c_.single();
        // Outside the store lock: every row fired unmodified? (then the insert under the lock
        // is O(1) and the build takes emax and the key count on the pool)
        bool all_fired = one != nullptr;
        for (int64_t i = 0; all_fired && i < nr; ++i) all_fired = col[5][i] == 1;
        {
          std::lock_guard<std::mutex> g(mu_);
          if (nr) {
            if (one) one->insert_hot(col[0], col[1], col[2], col[3], col[4], col[5], nr, true, plan,
                                     all_fired);
            else c_.insert(col[0], col[1], col[2], col[3], col[4], col[5], nr, true);
            if (one) {
              d.n_hot = nr - plan.nc;
              d.hot_keys = one->hot_free() ? 0 : 1;
            }
          }
        }
        {
          std::lock_guard<std::mutex> g(qmu_);
          hot_done_ = j.id;
          hot_marked = true;
        }
        dcv_.notify_all();
        const auto t2 = clk::now();
        if (one && nr) one->build_cold_parallel(col[0], col[1], col[2], col[3], col[4], nr, plan);
        const auto t2b = clk::now();
        if (plan.nkeys >= 0) {
          d.nk = plan.nkeys;
        } else {
          int64_t nk = nr ? 1 : 0;
          for (int64_t i = 1; i < nr; ++i) nk += col[0][i] != col[0][i - 1];
          d.nk = nk;
        }
        // The cold-row index entries of the new chunk, still outside the lock: every other user
        // of the index (extract, promote, expiry) joins this worker first.
        if (one && nr) one->index_cold(plan);
        const auto t3 = clk::now();
        // Expiry: a single store detaches its expired chunks under the lock and reads their keys
        // and frees their memory outside it (the step's host fire waits for this lock).
        std::vector<sess::ColdChunk> gone;
        bool gather_outside = false;
        {
          std::lock_guard<std::mutex> g(mu_);
          if (one && nr) one->publish_cold(plan);
          if (j.expire) {
            if (one) {
              one->detach_expired(j.expire_wm, gone);
              gather_outside = one->hot_free();
              if (!gather_outside) one->released_of(gone, d.released);
            } else {
              c_.expire_cold(j.expire_wm, d.released);
            }
          }
        }
        const auto t4 = clk::now();
        if (!gone.empty()) {
          if (gather_outside) one->released_of(gone, d.released);
          {
            std::lock_guard<std::mutex> g(mu_);
            one->recycle(gone);  // up to the spare limit; the rest stays in `gone`
          }
          gone.clear();  // frees the remaining chunks' memory outside the lock
        }
        const auto t5 = clk::now();
        d.t_wait = sec(t0, t1);
        d.t_hot = sec(t1, t2);
        d.t_build = sec(t2, t2b);
        d.t_index = sec(t2b, t3);
        d.t_publish = sec(t3, t4);
        d.t_expire = sec(t4, t5);
        d.t_populate = plan.t_populate;
      } catch (...) {
        d.err = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> g(qmu_);
        if (j.ev) free_ev_.push_back(j.ev);
        if (!hot_marked) hot_done_ = j.id;
        completed_ = j.id;
        done_.push_back(std::move(d));
      }
      dcv_.notify_all();
    }
  }

  sess::ShardedCore c_;
  std::mutex mu_;  // the store core: the main thread's calls vs the worker's locked phases
  // worker queue state (qmu_)
  std::thread th_;
  std::mutex qmu_;
  std::condition_variable qcv_, dcv_;
  std::deque<SpillJob> q_;
  std::deque<SpillDone> done_;
  std::vector<hipEvent_t> free_ev_;
  uint64_t submitted_ = 0, hot_done_ = 0, completed_ = 0;
  bool stop_ = false;
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
      // GIL released: the rows are read in place (no Python object is touched).
      .def("insert", &SessionStore::insert_np, py::arg("keys"), py::arg("starts"),
           py::arg("ends"), py::arg("accs"), py::arg("cnts"), py::arg("flags"),
           py::arg("cold") = false, py::call_guard<py::gil_scoped_release>())
      .def("merge_runs", &SessionStore::merge_runs_np)
      .def("extract", &SessionStore::extract_np)
      .def("extract_packed", &SessionStore::extract_packed_np)
      .def("extract_rows_into", &SessionStore::extract_rows_into_np)
      .def("index_stats", &SessionStore::index_stats)
      .def("fire", &SessionStore::fire_np, py::arg("wm"), py::arg("map_code"),
           py::arg("map_consts"), py::arg("f_code"), py::arg("f_consts"),
           py::arg("expire_cold") = true, py::arg("hot_upto") = -1)
      .def("expire_cold", &SessionStore::expire_cold_np)
      .def("spill_set", &SessionStore::spill_set_np)
      .def("contains", &SessionStore::contains)
      .def("num_keys", &SessionStore::num_keys)
      .def("num_sessions", &SessionStore::num_sessions)
      .def("num_cold_rows", &SessionStore::num_cold_rows)
      .def("bytes", &SessionStore::bytes)
      .def("key_list", &SessionStore::key_list_np)
      .def("snapshot", &SessionStore::snapshot_np, py::arg("extra") = 0)
      .def("spill_submit", &SessionStore::spill_submit, py::arg("stream"), py::arg("slab"),
           py::arg("ctr_off"), py::arg("col_off"), py::arg("rows"), py::arg("expire_wm") = py::none())
      .def("spill_submitted", &SessionStore::spill_submitted)
      .def("spill_completed", &SessionStore::spill_completed)
      .def("spill_poll", &SessionStore::spill_poll)
      .def("spill_join", &SessionStore::spill_join);
}
