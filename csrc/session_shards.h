// mxstream — the host session store split into key shards worked by a persistent thread pool.
//
// The GPU session operator's host tier (csrc/session_store.h) is touched every step: the
// eviction insert of idle keys (~10^5-10^6 rows), the firing of host-resident sessions, the
// extract of revisited keys. One store does each on one core (3-4 ms per step at config 5,
// BASELINE "host-DRAM state spill"). Keys never interact across sessions, so the store is S
// independent SessionCore shards (shard = top bits of a key mix); every call partitions its
// rows by shard (a stable counting sort, so a key's rows keep their order) and the shards run
// in parallel on a pool of persistent workers (no thread start per call). Results are
// concatenated in shard order, except extract's, which keeps its documented ascending key order.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "session_store.h"
#include "thread_pool.h"

namespace mxs {
namespace sess {

class ShardedCore {
 public:
  ShardedCore(int64_t gap, int64_t lateness, int agg, int shards) {
    int b = 0;
    while ((1 << b) < shards && b < 8) ++b;
    bits_ = b;
    for (int i = 0; i < (1 << b); ++i) {
      sh_.emplace_back(new SessionCore(gap, lateness, agg));
      // shards run in parallel on the pool below: each one alone stays single-threaded
      if ((1 << b) > 1) sh_.back()->max_threads_ = 1;
    }
    if ((1 << b) > 1) {
      const unsigned hw = std::thread::hardware_concurrency();
      const int workers = std::min<int>((1 << b), std::min<int>(hw ? (int)hw : 1, 16)) - 1;
      pool_.reset(new WorkerPool(std::max(0, workers)));
    }
  }
  int shards() const { return (int)sh_.size(); }
  // The one core of an unsharded store (the asynchronous spill worker's phased insert), else null.
  SessionCore* single() { return sh_.size() == 1 ? sh_[0].get() : nullptr; }
  int shard_of(uint64_t key) const {
    return bits_ ? (int)((mix64(key ^ 0x5bd1e9955bd1e995ull) * 0x9e3779b97f4a7c15ull) >> (64 - bits_))
                 : 0;
  }

  // Rows 0..n-1 grouped by shard: idx[off[s] .. off[s + 1]) are shard s's rows, in order.
  void group(const int64_t* keys, int64_t n, std::vector<uint32_t>& idx,
             std::vector<int64_t>& off) const {
    const int S = shards();
    off.assign(S + 1, 0);
    std::vector<uint8_t> sid((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
      sid[i] = (uint8_t)shard_of((uint64_t)keys[i]);
      ++off[sid[i] + 1];
    }
    for (int s = 0; s < S; ++s) off[s + 1] += off[s];
    std::vector<int64_t> cur(off.begin(), off.end() - 1);
    idx.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) idx[cur[sid[i]]++] = (uint32_t)i;
  }
  // Per-shard copies of `ncol` int64 columns.
  struct Split {
    std::vector<int64_t> off;
    std::vector<std::vector<int64_t>> col;  // [ncol] x n, shard-grouped
  };
  Split split(const int64_t* keys, int64_t n, std::initializer_list<const int64_t*> cols) const {
    Split sp;
    std::vector<uint32_t> idx;
    group(keys, n, idx, sp.off);
    for (const int64_t* c : cols) {
      std::vector<int64_t> v((size_t)n);
      for (int64_t j = 0; j < n; ++j) v[j] = c[idx[j]];
      sp.col.push_back(std::move(v));
    }
    return sp;
  }
  void each(const std::function<void(int)>& f) {
    if (pool_) pool_->run(shards(), f);
    else for (int s = 0; s < shards(); ++s) f(s);
  }

  int64_t process(const int64_t* k, const int64_t* t, const int64_t* v, int64_t n, int64_t wm) {
    if (shards() == 1) return sh_[0]->process(k, t, v, n, wm);
    const Split sp = split(k, n, {k, t, v});
    std::vector<int64_t> late(shards(), 0);
    each([&](int s) {
      const int64_t a = sp.off[s], m = sp.off[s + 1] - a;
      if (m) late[s] = sh_[s]->process(&sp.col[0][a], &sp.col[1][a], &sp.col[2][a], m, wm);
    });
    int64_t tot = 0;
    for (int64_t x : late) tot += x;
    return tot;
  }
  int64_t merge_runs(const int64_t* keys, const int64_t* starts, const int64_t* ends,
                     const int64_t* accs, const int64_t* cnts, int64_t n, int64_t wm) {
    if (shards() == 1) return sh_[0]->merge_runs(keys, starts, ends, accs, cnts, n, wm);
    const Split sp = split(keys, n, {keys, starts, ends, accs, cnts});
    std::vector<int64_t> late(shards(), 0);
    each([&](int s) {
      const int64_t a = sp.off[s], m = sp.off[s + 1] - a;
      if (m)
        late[s] = sh_[s]->merge_runs(&sp.col[0][a], &sp.col[1][a], &sp.col[2][a], &sp.col[3][a],
                                     &sp.col[4][a], m, wm);
    });
    int64_t tot = 0;
    for (int64_t x : late) tot += x;
    return tot;
  }
  void insert(const int64_t* K, const int64_t* S, const int64_t* E, const int64_t* A,
              const int64_t* C, const int64_t* F, int64_t n, bool cold) {
    if (shards() == 1) return sh_[0]->insert(K, S, E, A, C, F, n, cold);
    const Split sp = split(K, n, {K, S, E, A, C, F});
    each([&](int s) {
      const int64_t a = sp.off[s], m = sp.off[s + 1] - a;
      if (m)
        sh_[s]->insert(&sp.col[0][a], &sp.col[1][a], &sp.col[2][a], &sp.col[3][a], &sp.col[4][a],
                       &sp.col[5][a], m, cold);
    });
  }
  // Rows grouped by key, keys ascending (each shard's output is; the shards' are merged).
  Columns extract(const int64_t* keys, int64_t n, int64_t wm, int64_t max_sess,
                  std::vector<int64_t>* moved) {
    if (shards() == 1) return sh_[0]->extract(keys, n, wm, max_sess, moved);
    const Split sp = split(keys, n, {keys});
    std::vector<Columns> part(shards());
    std::vector<std::vector<int64_t>> mv(shards());
    each([&](int s) {
      const int64_t a = sp.off[s], m = sp.off[s + 1] - a;
      if (m) part[s] = sh_[s]->extract(&sp.col[0][a], m, wm, max_sess, &mv[s]);
    });
    // k-way merge by key (keys are disjoint between shards, ascending within each)
    Columns out;
    size_t total = 0;
    for (auto& p : part) total += p.key.size();
    for (auto* v : {&out.key, &out.start, &out.end, &out.acc, &out.cnt, &out.flags})
      v->reserve(total);
    std::vector<size_t> pos(shards(), 0);
    for (;;) {
      int best = -1;
      for (int s = 0; s < shards(); ++s)
        if (pos[s] < part[s].key.size() &&
            (best < 0 || (uint64_t)part[s].key[pos[s]] < (uint64_t)part[best].key[pos[best]]))
          best = s;
      if (best < 0) break;
      Columns& p = part[best];
      const int64_t k = p.key[pos[best]];
      while (pos[best] < p.key.size() && p.key[pos[best]] == k) {
        const size_t i = pos[best]++;
        out.key.push_back(p.key[i]);
        out.start.push_back(p.start[i]);
        out.end.push_back(p.end[i]);
        out.acc.push_back(p.acc[i]);
        out.cnt.push_back(p.cnt[i]);
        out.flags.push_back(p.flags[i]);
      }
    }
    for (auto& m : mv) moved->insert(moved->end(), m.begin(), m.end());
    return out;
  }
  SessionCore::IndexStats index_stats() const {
    SessionCore::IndexStats t;
    for (auto& c : sh_) {
      const auto x = c->index_stats();
      t.indexed += x.indexed;
      t.multi += x.multi;
      t.hot += x.hot;
      t.scans += x.scans;
      t.off += x.off;
      t.span += x.span;
    }
    return t;
  }
  // The promote path's extract as promote rows (SessionCore::extract_rows_into).
  std::tuple<int64_t, int64_t, int64_t> extract_rows_into(const int64_t* keys, int64_t n,
                                                          int64_t wm, int64_t max_sess,
                                                          int64_t gap, int64_t* rows, int64_t cap,
                                                          int64_t* moved_out,
                                                          int64_t moved_cap) {
    if (shards() == 1)
      return sh_[0]->extract_rows_into(keys, n, wm, max_sess, gap, rows, cap, moved_out,
                                       moved_cap);
    std::vector<uint64_t> want, bits;
    SessionCore::sort_unique_keys(keys, n, want, bits);
    std::vector<int64_t> moved;
    const Columns c = extract((const int64_t*)want.data(), (int64_t)want.size(), wm, max_sess,
                              &moved);
    const auto r = SessionCore::promote_rows(c, moved, gap, rows, cap, moved_out, moved_cap);
    return {r.first, r.second, (int64_t)want.size()};
  }
  void fire(int64_t wm, const ExprProg& mp, const ExprProg& fp, SessionCore::FireOut& o,
            bool expire_cold = true) {
    if (shards() == 1) return sh_[0]->fire(wm, mp, fp, o, expire_cold);
    std::vector<SessionCore::FireOut> part(shards());
    each([&](int s) { sh_[s]->fire(wm, mp, fp, part[s], expire_cold); });
    for (auto& p : part) {
      auto cat = [](auto& dst, const auto& src) { dst.insert(dst.end(), src.begin(), src.end()); };
      cat(o.okey, p.okey);
      cat(o.ostart, p.ostart);
      cat(o.oend, p.oend);
      cat(o.oraw, p.oraw);
      cat(o.ocnt, p.ocnt);
      cat(o.oref, p.oref);
      cat(o.released, p.released);
      cat(o.oval, p.oval);
    }
  }
  void expire_cold(int64_t wm, std::vector<int64_t>& released) {
    if (shards() == 1) return sh_[0]->expire_cold(wm, released);
    std::vector<std::vector<int64_t>> part(shards());
    each([&](int s) { sh_[s]->expire_cold(wm, part[s]); });
    for (auto& p : part) released.insert(released.end(), p.begin(), p.end());
  }
  void spill_set(int cap_log2, int64_t* d) const {
    const size_t cap = (size_t)1 << cap_log2;
    if (num_keys() * 2 > cap) throw std::invalid_argument("spill set too small");
    std::fill(d, d + cap, (int64_t)kEmptyKey);
    for (auto& s : sh_) s->spill_set_add(cap_log2, d);
  }
  bool contains(uint64_t key) const { return sh_[shard_of(key)]->contains(key); }
  bool hot(uint64_t key) const { return sh_[shard_of(key)]->hot(key); }
  // No shard holds hot (in-memory, not cold-chunk) sessions.
  bool hot_free() const {
    for (auto& s : sh_)
      if (!s->hot_free()) return false;
    return true;
  }
  size_t num_keys() const {
    size_t t = 0;
    for (auto& s : sh_) t += s->num_keys();
    return t;
  }
  size_t num_sessions() const {
    size_t t = 0;
    for (auto& s : sh_) t += s->num_sessions();
    return t;
  }
  size_t num_cold_rows() const {
    size_t t = 0;
    for (auto& s : sh_) t += s->num_cold_rows();
    return t;
  }
  size_t bytes() const {
    size_t t = 0;
    for (auto& s : sh_) t += s->bytes();
    return t;
  }
  std::vector<int64_t> key_list() const {
    std::vector<int64_t> k;
    for (auto& s : sh_) {
      auto p = s->key_list();
      k.insert(k.end(), p.begin(), p.end());
    }
    std::sort(k.begin(), k.end());
    return k;
  }
  // snapshot() of every shard, built by the shards in parallel (shard order, as snapshot()).
  std::vector<Columns> snapshot_parts() {
    std::vector<Columns> part(sh_.size());
    each([&](int s) { part[s] = sh_[s]->snapshot(); });
    return part;
  }

  Columns snapshot() const {
    Columns out;
    for (auto& s : sh_) {
      Columns p = s->snapshot();
      out.key.insert(out.key.end(), p.key.begin(), p.key.end());
      out.start.insert(out.start.end(), p.start.begin(), p.start.end());
      out.end.insert(out.end.end(), p.end.begin(), p.end.end());
      out.acc.insert(out.acc.end(), p.acc.begin(), p.acc.end());
      out.cnt.insert(out.cnt.end(), p.cnt.begin(), p.cnt.end());
      out.flags.insert(out.flags.end(), p.flags.begin(), p.flags.end());
    }
    return out;
  }

 private:
  int bits_ = 0;
  std::vector<std::unique_ptr<SessionCore>> sh_;
  std::unique_ptr<WorkerPool> pool_;
};

}  // namespace sess
}  // namespace mxs
