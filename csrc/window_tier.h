// mxstream — host-DRAM tier of the keyed window state (BASELINE north star: keyed state with
// spill to host DRAM). Rows (key, pane, acc, cnt, dirty) evicted from the HBM
// tables by window_compact arrive as append-only chunks (no re-concatenation of the whole tier
// per eviction); a firing's share of the tier is hash-combined per key over the chunks that
// overlap the window's panes; a purge drops whole chunks below the live range and filters at
// most the chunks that straddle it. No Python in here (csrc/window_tier_bindings.cpp binds it).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <utility>
#include <vector>

#include "mxs_common.h"

namespace mxs {

class WindowTierCore {
 public:
  struct Chunk {
    int64_t pmin = INT64_MAX, pmax = INT64_MIN;
    std::vector<uint64_t> key;
    std::vector<int64_t> pane, acc, cnt;
    std::vector<uint8_t> dirty;
    size_t size() const { return key.size(); }
  };
  struct Rows {
    std::vector<uint64_t> key;
    std::vector<int64_t> pane, acc, cnt;
    std::vector<uint8_t> dirty;
  };

  explicit WindowTierCore(int agg) : agg_(agg) {}

  int agg() const { return agg_; }
  size_t nrows() const { return rows_; }
  size_t nbytes() const { return rows_ * (8 + 8 + 8 + 8 + 1); }
  int64_t rows_in() const { return rows_in_; }
  bool empty() const { return rows_ == 0; }
  // [min pane, max pane] over all rows (false when empty).
  bool pane_range(int64_t* lo, int64_t* hi) const {
    if (!rows_) return false;
    *lo = INT64_MAX;
    *hi = INT64_MIN;
    for (auto& c : chunks_) {
      *lo = std::min(*lo, c.pmin);
      *hi = std::max(*hi, c.pmax);
    }
    return true;
  }

  void absorb(const uint64_t* key, const int64_t* pane, const int64_t* acc, const int64_t* cnt,
              const uint8_t* dirty, size_t n) {
    if (!n) return;
    Chunk c;
    c.key.assign(key, key + n);
    c.pane.assign(pane, pane + n);
    c.acc.assign(acc, acc + n);
    c.cnt.assign(cnt, cnt + n);
    c.dirty.assign(dirty, dirty + n);
    for (size_t i = 0; i < n; ++i) {
      c.pmin = std::min(c.pmin, pane[i]);
      c.pmax = std::max(c.pmax, pane[i]);
    }
    rows_ += n;
    rows_in_ += (int64_t)n;
    chunks_.push_back(std::move(c));
  }

  // The tier's share of the window over panes [p0, p1]: one (key, acc, cnt) per key, keys
  // ascending. Hash aggregation over the overlapping chunks only.
  void part(int64_t p0, int64_t p1, std::vector<uint64_t>* keys, std::vector<int64_t>* acc,
            std::vector<int64_t>* cnt) const {
    keys->clear();
    acc->clear();
    cnt->clear();
    size_t cand = 0;
    for (auto& c : chunks_)
      if (c.pmax >= p0 && c.pmin <= p1) cand += c.size();
    if (!cand) return;
    size_t cap = 16;
    while (cap < 2 * cand) cap <<= 1;
    std::vector<uint64_t> hk(cap, kEmptyKey);
    std::vector<int64_t> ha(cap), hc(cap, 0);
    const size_t mask = cap - 1;
    for (auto& c : chunks_) {
      if (c.pmax < p0 || c.pmin > p1) continue;
      for (size_t i = 0; i < c.size(); ++i) {
        if (c.pane[i] < p0 || c.pane[i] > p1 || !c.cnt[i]) continue;
        const uint64_t k = c.key[i];
        size_t h = (size_t)(mix64(k) >> 32) & mask;
        while (hk[h] != kEmptyKey && hk[h] != k) h = (h + 1) & mask;
        if (hk[h] == kEmptyKey) {
          hk[h] = k;
          ha[h] = c.acc[i];
          hc[h] = c.cnt[i];
        } else {
          ha[h] = (int64_t)agg_combine(agg_, (uint64_t)ha[h], (uint64_t)c.acc[i]);
          hc[h] += c.cnt[i];
        }
      }
    }
    std::vector<std::pair<uint64_t, size_t>> order;
    for (size_t h = 0; h < cap; ++h)
      if (hk[h] != kEmptyKey) order.push_back({hk[h], h});
    std::sort(order.begin(), order.end());
    keys->reserve(order.size());
    acc->reserve(order.size());
    cnt->reserve(order.size());
    for (auto& [k, h] : order) {
      keys->push_back(k);
      acc->push_back(ha[h]);
      cnt->push_back(hc[h]);
    }
  }

  // A tiered firing: the device's rows of the window (dev_*: one per key, no epilogue) combined
  // with this tier's rows of panes [p0, p1] per key, in one hash aggregation. only_dev: a
  // re-firing -- tier rows count only for keys the device fired. Output order: hash order.
  void merge_fire(int64_t p0, int64_t p1, const uint64_t* dk, const int64_t* da,
                  const int64_t* dc, size_t nd, bool only_dev, std::vector<uint64_t>* keys,
                  std::vector<int64_t>* acc, std::vector<int64_t>* cnt) const {
    keys->clear();
    acc->clear();
    cnt->clear();
    size_t cand = nd;
    for (auto& c : chunks_)
      if (c.pmax >= p0 && c.pmin <= p1) cand += c.size();
    size_t cap = 16;
    while (cap < 2 * cand) cap <<= 1;
    std::vector<uint64_t> hk(cap, kEmptyKey);
    std::vector<int64_t> ha(cap), hc(cap, 0);
    const size_t mask = cap - 1;
    auto put = [&](uint64_t k, int64_t a, int64_t c, bool insert) {
      size_t h = (size_t)(mix64(k) >> 32) & mask;
      while (hk[h] != kEmptyKey && hk[h] != k) h = (h + 1) & mask;
      if (hk[h] == kEmptyKey) {
        if (!insert) return;
        hk[h] = k;
        ha[h] = a;
        hc[h] = c;
      } else {
        ha[h] = (int64_t)agg_combine(agg_, (uint64_t)ha[h], (uint64_t)a);
        hc[h] += c;
      }
    };
    for (size_t i = 0; i < nd; ++i) put(dk[i], da[i], dc[i], true);
    for (auto& c : chunks_) {
      if (c.pmax < p0 || c.pmin > p1) continue;
      for (size_t i = 0; i < c.size(); ++i)
        if (c.pane[i] >= p0 && c.pane[i] <= p1 && c.cnt[i])
          put(c.key[i], c.acc[i], c.cnt[i], !only_dev);
    }
    for (size_t h = 0; h < cap; ++h)
      if (hk[h] != kEmptyKey) {
        keys->push_back(hk[h]);
        acc->push_back(ha[h]);
        cnt->push_back(hc[h]);
      }
  }

  // Drop rows of panes < keep_from: whole chunks below it, filtered straddling chunks.
  void purge(int64_t keep_from) {
    std::deque<Chunk> kept;
    for (auto& c : chunks_) {
      if (c.pmax < keep_from) {
        rows_ -= c.size();
        continue;
      }
      if (c.pmin < keep_from) {
        Chunk f;
        for (size_t i = 0; i < c.size(); ++i) {
          if (c.pane[i] < keep_from) continue;
          f.key.push_back(c.key[i]);
          f.pane.push_back(c.pane[i]);
          f.acc.push_back(c.acc[i]);
          f.cnt.push_back(c.cnt[i]);
          f.dirty.push_back(c.dirty[i]);
          f.pmin = std::min(f.pmin, c.pane[i]);
          f.pmax = std::max(f.pmax, c.pane[i]);
        }
        rows_ -= c.size() - f.size();
        if (f.size()) kept.push_back(std::move(f));
        continue;
      }
      kept.push_back(std::move(c));
    }
    chunks_.swap(kept);
  }

  // Every row, merged per (key, pane) (a key evicted, re-inserted and evicted again), ordered by
  // (pane, key). Also compacts the tier to that one chunk.
  Rows rows() {
    Rows out;
    if (!rows_) return out;
    struct R {
      int64_t pane;
      uint64_t key;
      size_t ci, i;
    };
    std::vector<R> idx;
    idx.reserve(rows_);
    for (size_t ci = 0; ci < chunks_.size(); ++ci)
      for (size_t i = 0; i < chunks_[ci].size(); ++i)
        idx.push_back({chunks_[ci].pane[i], chunks_[ci].key[i], ci, i});
    std::sort(idx.begin(), idx.end(), [](const R& a, const R& b) {
      return a.pane != b.pane ? a.pane < b.pane : a.key < b.key;
    });
    Chunk m;
    for (size_t q = 0; q < idx.size(); ++q) {
      const Chunk& c = chunks_[idx[q].ci];
      const size_t i = idx[q].i;
      if (q && idx[q].pane == idx[q - 1].pane && idx[q].key == idx[q - 1].key) {
        m.acc.back() = (int64_t)agg_combine(agg_, (uint64_t)m.acc.back(), (uint64_t)c.acc[i]);
        m.cnt.back() += c.cnt[i];
        m.dirty.back() = std::max(m.dirty.back(), c.dirty[i]);
        continue;
      }
      m.key.push_back(c.key[i]);
      m.pane.push_back(c.pane[i]);
      m.acc.push_back(c.acc[i]);
      m.cnt.push_back(c.cnt[i]);
      m.dirty.push_back(c.dirty[i]);
      m.pmin = std::min(m.pmin, c.pane[i]);
      m.pmax = std::max(m.pmax, c.pane[i]);
    }
    out.key = m.key;
    out.pane = m.pane;
    out.acc = m.acc;
    out.cnt = m.cnt;
    out.dirty = m.dirty;
    chunks_.clear();
    rows_ = m.size();
    if (rows_) chunks_.push_back(std::move(m));
    return out;
  }

  void clear() {
    chunks_.clear();
    rows_ = 0;
  }

 private:
  int agg_;
  std::deque<Chunk> chunks_;
  size_t rows_ = 0;
  int64_t rows_in_ = 0;
};

}  // namespace mxs
