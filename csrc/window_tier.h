// mxstream — host-DRAM tier of the keyed window state (BASELINE north star: keyed state with
// spill to host DRAM). Rows (key, pane, acc, cnt, dirty) evicted from the HBM
// tables by window_compact arrive as append-only chunks (no re-concatenation of the whole tier
// per eviction); a firing's share of the tier is hash-combined per key over the chunks that
// overlap the window's panes; a purge drops whole chunks below the live range and filters at
// most the chunks that straddle it. No Python in here (csrc/window_tier_bindings.cpp binds it).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <utility>
#include <vector>

#include "mxs_common.h"

namespace mxs {

// Allocator whose resize() leaves new elements uninitialised: the tier's columns are always
// written in full right after they grow (an eviction's counting sort scatters every row), and
// std::vector's zero fill was a whole extra single-threaded pass over ~33 bytes a row.
template <class T>
struct NoInitAlloc {
  using value_type = T;
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  T* allocate(size_t n) { return std::allocator<T>().allocate(n); }
  void deallocate(T* p, size_t n) { std::allocator<T>().deallocate(p, n); }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
    else ::new ((void*)p) U(std::forward<A>(a)...);
  }
  bool operator==(const NoInitAlloc&) const { return true; }
  bool operator!=(const NoInitAlloc&) const { return false; }
};
template <class T>
using RowVec = std::vector<T, NoInitAlloc<T>>;

class WindowTierCore {
 public:
  struct Chunk {
    int64_t pmin = INT64_MAX, pmax = INT64_MIN;
    RowVec<uint64_t> key;
    RowVec<int64_t> pane, acc, cnt;
    RowVec<uint8_t> dirty;
    // Lazy purge: rows of panes < live_from are dead (skipped by every reader) until they are
    // half the chunk, then the chunk is filtered. pane_rows[p - pmin] = rows of pane p.
    int64_t live_from = INT64_MIN;
    size_t dead = 0;
    std::vector<size_t> pane_rows;
    // Pane-sorted chunk (every absorbed eviction): rows grouped by pane ascending, pane p's rows
    // at [pane_off[p - pmin], pane_off[p - pmin + 1]), no zero-count rows. A firing's export is
    // then one contiguous segment per chunk (no per-row filter) and a purge only moves
    // live_from: the dead rows are a prefix.
    bool sorted = false;
    std::vector<size_t> pane_off;
    size_t size() const { return key.size(); }
    bool live(size_t i) const { return pane[i] >= live_from; }
    void count_panes() {
      pane_rows.assign(size() ? (size_t)(pmax - pmin + 1) : 0, 0);
      for (int64_t p : pane) ++pane_rows[(size_t)(p - pmin)];
      pane_off.clear();
      if (sorted) {
        pane_off.assign(pane_rows.size() + 1, 0);
        for (size_t j = 0; j < pane_rows.size(); ++j) pane_off[j + 1] = pane_off[j] + pane_rows[j];
      }
    }
    // Rows [lo, hi) of the live rows of panes [p0, p1] (sorted chunks only).
    void segment(int64_t p0, int64_t p1, size_t* lo, size_t* hi) const {
      const int64_t a = std::max(std::max(p0, pmin), live_from);
      const int64_t b = std::min(p1, pmax);
      if (a > b) {
        *lo = *hi = 0;
        return;
      }
      *lo = pane_off[(size_t)(a - pmin)];
      *hi = pane_off[(size_t)(b - pmin) + 1];
    }
  };
  struct Rows {
    std::vector<uint64_t> key;
    std::vector<int64_t> pane, acc, cnt;
    std::vector<uint8_t> dirty;
  };

  explicit WindowTierCore(int agg) : agg_(agg) {}
  // A copy (the frozen tier of an asynchronous snapshot) leaves the spare columns behind.
  WindowTierCore(const WindowTierCore& o)
      : agg_(o.agg_), chunks_(o.chunks_), rows_(o.rows_), rows_in_(o.rows_in_) {}
  ~WindowTierCore() {
    if (pf_.joinable()) pf_.join();
  }

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
      int64_t first = c.pmin;  // lowest live pane (dead rows of a lazy purge excluded)
      if (c.live_from > first) {
        first = c.live_from;
        if (!c.pane_rows.empty())
          while (first < c.pmax && !c.pane_rows[(size_t)(first - c.pmin)]) ++first;
      }
      *lo = std::min(*lo, first);
      *hi = std::max(*hi, c.pmax);
    }
    return true;
  }

  void absorb(const uint64_t* key, const int64_t* pane, const int64_t* acc, const int64_t* cnt,
              const uint8_t* dirty, size_t n) {
    if (!n) return;
    Chunk c;
    for (size_t i = 0; i < n; ++i) {
      c.pmin = std::min(c.pmin, pane[i]);
      c.pmax = std::max(c.pmax, pane[i]);
    }
    if ((uint64_t)(c.pmax - c.pmin) < ((uint64_t)1 << 20)) {
      // A purged or pre-faulted chunk's columns: capacity whose pages are already mapped
      // (fresh columns of a 5M-row eviction page-fault ~190 MB in).
      take_spare(c, n);
      absorb_sorted(c, key, pane, acc, cnt, dirty, n);
      prefault_async(n);
    } else {
      c.key.assign(key, key + n);
      c.pane.assign(pane, pane + n);
      c.acc.assign(acc, acc + n);
      c.cnt.assign(cnt, cnt + n);
      c.dirty.assign(dirty, dirty + n);
    }
    rows_ += c.size();
    rows_in_ += (int64_t)n;
    if (c.size()) chunks_.push_back(std::move(c));
  }

  // An eviction already grouped by pane on the device (window_rows_pane_sort): rows of pane
  // p0 + j are the next counts[j] rows. Threads copy equal row shares; no per-row sort here.
  void absorb_presorted(const uint64_t* key, const uint64_t* acc, const uint32_t* cnt,
                        const uint8_t* dirty, int64_t p0, const uint32_t* counts, int np) {
    size_t n = 0;
    int j0 = -1, j1 = -1;
    for (int j = 0; j < np; ++j)
      if (counts[j]) {
        n += counts[j];
        if (j0 < 0) j0 = j;
        j1 = j;
      }
    if (!n) return;
    Chunk c;
    take_spare(c, n);
    c.pmin = p0 + j0;
    c.pmax = p0 + j1;
    const size_t P = (size_t)(j1 - j0 + 1);
    c.pane_rows.assign(P, 0);
    c.pane_off.assign(P + 1, 0);
    for (size_t p = 0; p < P; ++p) {
      c.pane_rows[p] = counts[j0 + p];
      c.pane_off[p + 1] = c.pane_off[p] + c.pane_rows[p];
    }
    c.key.resize(n);
    c.pane.resize(n);
    c.acc.resize(n);
    c.cnt.resize(n);
    c.dirty.resize(n);
    const size_t T = host_threads(n);
    run_threads(T, [&](size_t t) {
      const size_t lo = n * t / T, hi = n * (t + 1) / T;
      if (lo >= hi) return;
      std::memcpy(c.key.data() + lo, key + lo, (hi - lo) * 8);
      std::memcpy(c.acc.data() + lo, acc + lo, (hi - lo) * 8);
      std::memcpy(c.dirty.data() + lo, dirty + lo, hi - lo);
      for (size_t i = lo; i < hi; ++i) c.cnt[i] = cnt[i];
      // pane column from the segments
      size_t p = (size_t)(std::upper_bound(c.pane_off.begin(), c.pane_off.end(), lo) -
                          c.pane_off.begin()) - 1;
      for (size_t i = lo; i < hi;) {
        const size_t e = std::min(hi, c.pane_off[p + 1]);
        std::fill(c.pane.data() + i, c.pane.data() + e, c.pmin + (int64_t)p);
        i = e;
        ++p;
      }
    });
    c.sorted = true;
    rows_ += n;
    rows_in_ += (int64_t)n;
    chunks_.push_back(std::move(c));
    prefault_async(n);
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
        if (c.pane[i] < p0 || c.pane[i] > p1 || !c.cnt[i] || !c.live(i)) continue;
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

  // Live rows of panes [p0, p1], uncombined (the device-merged tiered firing combines them on
  // the GPU): written to k / a / c when they fit `cap` rows; returns the row count either way.
  // Pane-sorted chunks contribute one contiguous segment each (copied by threads in equal row
  // shares); other chunks are filtered row by row (counted in parallel, then copied to their
  // prefix offsets). Row order is unspecified.
  // Window form: only output rows [r_begin, r_begin + cap) are written (to k[o - r_begin]...),
  // so a large export can go through a ring of fixed pinned slabs piece by piece; the returned
  // total is the whole export's row count. The output order is the same for every window.
  size_t export_rows(int64_t p0, int64_t p1, uint64_t* k, uint64_t* a, uint32_t* c,
                     size_t cap) const {
    return export_window(p0, p1, k, a, c, 0, cap, false);
  }
  size_t export_window(int64_t p0, int64_t p1, uint64_t* k, uint64_t* a, uint32_t* c,
                       size_t r_begin, size_t cap, bool partial) const {
    struct Seg {
      const Chunk* ch;
      size_t lo, hi, out;
    };
    std::vector<Seg> segs;
    std::vector<const Chunk*> src;
    size_t nseg = 0;
    for (auto& ch : chunks_) {
      if (ch.pmax < p0 || ch.pmin > p1 || !ch.size()) continue;
      if (ch.sorted) {
        size_t lo, hi;
        ch.segment(p0, p1, &lo, &hi);
        if (hi > lo) {
          segs.push_back({&ch, lo, hi, nseg});
          nseg += hi - lo;
        }
      } else {
        src.push_back(&ch);
      }
    }
    auto keep = [&](const Chunk& ch, size_t i) {
      return ch.pane[i] >= p0 && ch.pane[i] <= p1 && ch.cnt[i] && ch.live(i);
    };
    std::vector<size_t> cnt(src.size(), 0);
    const size_t Tu = std::max<size_t>(1, std::min<size_t>(src.size(), host_threads(1u << 30)));
    if (!src.empty())
      run_threads(Tu, [&](size_t t) {
        for (size_t j = t; j < src.size(); j += Tu) {
          const Chunk& ch = *src[j];
          size_t m = 0;
          for (size_t i = 0; i < ch.size(); ++i) m += keep(ch, i) ? 1 : 0;
          cnt[j] = m;
        }
      });
    std::vector<size_t> off(src.size() + 1, nseg);
    for (size_t j = 0; j < src.size(); ++j) off[j + 1] = off[j] + cnt[j];
    const size_t total = off.back();
    if (total == 0 || (!partial && total > cap)) return total;
    // the output window [wb, we) of the row order
    const size_t wb = std::min(r_begin, total), we = std::min(total, r_begin + cap);
    if (wb >= we) return total;
    // sorted segments: thread t copies output rows [wb + n * t / T, wb + n * (t + 1) / T) of the
    // window's part that falls in the segments [0, nseg)
    const size_t sb = wb, se = std::min(we, nseg);
    const size_t nwin = se > sb ? se - sb : 0;
    const size_t T = host_threads(nwin);
    if (nwin)
      run_threads(T, [&](size_t t) {
        const size_t r0 = sb + nwin * t / T, r1 = sb + nwin * (t + 1) / T;
        for (const Seg& s : segs) {
          const size_t o0 = std::max(r0, s.out), o1 = std::min(r1, s.out + (s.hi - s.lo));
          if (o0 >= o1) continue;
          const size_t i0 = s.lo + (o0 - s.out), m = o1 - o0;
          std::memcpy(k + (o0 - wb), s.ch->key.data() + i0, m * 8);
          std::memcpy(a + (o0 - wb), s.ch->acc.data() + i0, m * 8);
          const int64_t* cs = s.ch->cnt.data() + i0;
          for (size_t q = 0; q < m; ++q) c[o0 - wb + q] = (uint32_t)cs[q];
        }
      });
    if (!src.empty() && we > nseg)
      run_threads(Tu, [&](size_t t) {
        for (size_t j = t; j < src.size(); j += Tu) {
          if (off[j + 1] <= wb || off[j] >= we) continue;
          const Chunk& ch = *src[j];
          size_t o = off[j];
          for (size_t i = 0; i < ch.size() && o < we; ++i) {
            if (!keep(ch, i)) continue;
            if (o >= wb) {
              k[o - wb] = ch.key[i];
              a[o - wb] = (uint64_t)ch.acc[i];
              c[o - wb] = (uint32_t)ch.cnt[i];
            }
            ++o;
          }
        }
      });
    return total;
  }

  // A tiered firing: the device's rows of the window (dev_*: one per key, no epilogue) combined
  // with this tier's rows of panes [p0, p1] per key. only_dev: a re-firing -- tier rows count
  // only for keys the device fired. Output order: partition order (unspecified).
  //
  // Radix-partitioned parallel hash aggregation (the single-table version spent ~300 ms per
  // firing on cache misses at 10M rows): threads count their share of every source per
  // partition (top bits of mix64(key)), scatter the rows into partition-contiguous buffers, then
  // aggregate partitions independently in cache-sized tables. Device rows of a partition are
  // folded before its tier rows, so only_dev sees every device key first.
  void merge_fire(int64_t p0, int64_t p1, const uint64_t* dk, const int64_t* da,
                  const int64_t* dc, size_t nd, bool only_dev, std::vector<uint64_t>* keys,
                  std::vector<int64_t>* acc, std::vector<int64_t>* cnt) const {
    keys->clear();
    acc->clear();
    cnt->clear();
    struct Src {
      const uint64_t* k;
      const int64_t *a, *c, *pane;
      size_t n;
      bool dev;
      int64_t live_from;
    };
    std::vector<Src> src;
    if (nd) src.push_back({dk, da, dc, nullptr, nd, true, INT64_MIN});
    size_t cand = nd;
    for (auto& c : chunks_)
      if (c.pmax >= p0 && c.pmin <= p1 && c.size()) {
        src.push_back({c.key.data(), c.acc.data(), c.cnt.data(), c.pane.data(), c.size(), false,
                       c.live_from});
        cand += c.size();
      }
    if (!cand) return;
    const int pbits = cand > (1u << 20) ? 8 : 4;
    const size_t P = (size_t)1 << pbits;
    unsigned hw = std::thread::hardware_concurrency();
    const size_t T = cand < (1u << 16) ? 1 : std::max(1u, std::min(hw ? hw : 1u, 16u));
    auto part_of = [&](uint64_t k) { return (size_t)(mix64(k) >> (64 - pbits)); };
    auto keep = [&](const Src& s, size_t i) {
      return s.dev || (s.pane[i] >= p0 && s.pane[i] <= p1 && s.c[i] && s.pane[i] >= s.live_from);
    };
    auto piece = [&](const Src& s, size_t t, size_t* lo, size_t* hi) {
      *lo = s.n * t / T;
      *hi = s.n * (t + 1) / T;
    };
    auto run = [&](auto&& fn) {
      if (T == 1) {
        fn((size_t)0);
        return;
      }
      std::vector<std::thread> th;
      for (size_t t = 0; t < T; ++t) th.emplace_back(fn, t);
      for (auto& x : th) x.join();
    };
    // 1. counts per (thread, partition)
    std::vector<size_t> cnts(T * P, 0);
    run([&](size_t t) {
      size_t* ct = cnts.data() + t * P;
      for (auto& s : src) {
        size_t lo, hi;
        piece(s, t, &lo, &hi);
        for (size_t i = lo; i < hi; ++i)
          if (keep(s, i)) ++ct[part_of(s.k[i])];
      }
    });
    // partition-major offsets: partition p holds thread 0's rows, then thread 1's, ...
    std::vector<size_t> off(T * P), pstart(P + 1, 0);
    size_t tot = 0;
    for (size_t p = 0; p < P; ++p) {
      pstart[p] = tot;
      for (size_t t = 0; t < T; ++t) {
        off[t * P + p] = tot;
        tot += cnts[t * P + p];
      }
    }
    pstart[P] = tot;
    struct Row {
      uint64_t k;
      int64_t a, c;
      uint64_t dev;
    };
    std::vector<Row> rows(tot);
    // 2. scatter
    run([&](size_t t) {
      size_t* o = off.data() + t * P;
      for (auto& s : src) {
        size_t lo, hi;
        piece(s, t, &lo, &hi);
        for (size_t i = lo; i < hi; ++i)
          if (keep(s, i)) rows[o[part_of(s.k[i])]++] = Row{s.k[i], s.a[i], s.c[i], s.dev};
      }
    });
    // 3. aggregate partitions (thread t takes partitions t, t + T, ...)
    std::vector<std::vector<Row>> outp(P);
    run([&](size_t t) {
      std::vector<uint64_t> hk;
      std::vector<int64_t> ha, hc;
      for (size_t p = t; p < P; p += T) {
        const size_t b = pstart[p], e = pstart[p + 1];
        if (b == e) continue;
        size_t cap = 16;
        while (cap < 2 * (e - b)) cap <<= 1;
        hk.assign(cap, kEmptyKey);
        ha.assign(cap, 0);
        hc.assign(cap, 0);
        const size_t mask = cap - 1;
        for (int pass = 0; pass < 2; ++pass) {  // device rows first, then tier rows
          for (size_t i = b; i < e; ++i) {
            const Row& r = rows[i];
            if ((r.dev != 0) != (pass == 0)) continue;
            // (mix64's low bits: the partition took the top ones)
            size_t h = (size_t)mix64(r.k) & mask;
            while (hk[h] != kEmptyKey && hk[h] != r.k) h = (h + 1) & mask;
            if (hk[h] == kEmptyKey) {
              if (!r.dev && only_dev) continue;
              hk[h] = r.k;
              ha[h] = r.a;
              hc[h] = r.c;
            } else {
              ha[h] = (int64_t)agg_combine(agg_, (uint64_t)ha[h], (uint64_t)r.a);
              hc[h] += r.c;
            }
          }
        }
        auto& out = outp[p];
        for (size_t h = 0; h < cap; ++h)
          if (hk[h] != kEmptyKey) out.push_back(Row{hk[h], ha[h], hc[h], 0});
      }
    });
    size_t nout = 0;
    for (auto& o : outp) nout += o.size();
    keys->reserve(nout);
    acc->reserve(nout);
    cnt->reserve(nout);
    for (auto& o : outp)
      for (auto& r : o) {
        keys->push_back(r.k);
        acc->push_back(r.a);
        cnt->push_back(r.c);
      }
  }

  // A traced program from its (op, arg) code list and constants (csrc/mxs_common.h ExprProg).
  static ExprProg prog(const int32_t* code, size_t ncode, const double* consts, size_t nconst) {
    ExprProg p;
    std::memset(&p, 0, sizeof(p));
    if (ncode > (size_t)2 * kExprMaxCode || nconst > (size_t)kExprMaxConst)
      throw std::invalid_argument("expr program too large");
    for (size_t i = 0; i < ncode; ++i) p.code[i] = code[i];
    for (size_t i = 0; i < nconst; ++i) p.consts[i] = consts[i];
    p.ncode = (int32_t)(ncode / 2);
    return p;
  }

  // The window epilogue over merged rows (the host twin of window_fire's fused map/filter):
  // result, traced map, traced filter; kept rows in input order. Threaded over row ranges.
  void epilogue(const std::vector<uint64_t>& keys, const std::vector<int64_t>& acc,
                const std::vector<int64_t>& cnt, const ExprProg& mp, const ExprProg& fp,
                int64_t wstart, int64_t wend, std::vector<uint64_t>* ok,
                std::vector<double>* oval, std::vector<int64_t>* oraw,
                std::vector<int32_t>* ocnt) const {
    const size_t n = keys.size();
    unsigned hw = std::thread::hardware_concurrency();
    const size_t T = n < (1u << 15) ? 1 : std::max(1u, std::min(hw ? hw : 1u, 16u));
    struct Part {
      std::vector<uint64_t> k;
      std::vector<double> v;
      std::vector<int64_t> r;
      std::vector<int32_t> c;
    };
    std::vector<Part> parts(T);
    auto work = [&](size_t t) {
      const size_t lo = n * t / T, hi = n * (t + 1) / T;
      Part& pt = parts[t];
      for (size_t i = lo; i < hi; ++i) {
        double vars[kExprVars] = {0};
        vars[0] = agg_result_f64(agg_, (uint64_t)acc[i], (uint32_t)cnt[i]);
        vars[1] = (double)cnt[i];
        vars[2] = (double)wstart;
        vars[3] = (double)wend;
        vars[4] = (double)keys[i];
        vars[5] = (double)acc[i];
        vars[6] = mp.ncode ? expr_eval(mp, vars) : vars[0];
        if (fp.ncode && expr_eval(fp, vars) == 0.0) continue;
        pt.k.push_back(keys[i]);
        pt.v.push_back(vars[6]);
        pt.r.push_back(acc[i]);
        pt.c.push_back((int32_t)cnt[i]);
      }
    };
    if (T == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (size_t t = 0; t < T; ++t) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
    ok->clear();
    oval->clear();
    oraw->clear();
    ocnt->clear();
    for (auto& pt : parts) {
      ok->insert(ok->end(), pt.k.begin(), pt.k.end());
      oval->insert(oval->end(), pt.v.begin(), pt.v.end());
      oraw->insert(oraw->end(), pt.r.begin(), pt.r.end());
      ocnt->insert(ocnt->end(), pt.c.begin(), pt.c.end());
    }
  }

  // Drop rows of panes < keep_from: whole chunks below it, filtered straddling chunks. A chunk
  // whose rows below live_from are already dead purges from max(keep_from, live_from), so a
  // keep_from lower than an earlier purge's never revives dead rows or rewinds the counts.
  void purge(int64_t keep_from) {
    std::deque<Chunk> kept;
    for (auto& c : chunks_) {
      const int64_t kf = std::max(keep_from, c.live_from);
      if (c.pmax < kf) {
        rows_ -= c.size() - c.dead;
        if (c.sorted) give_spare(std::move(c));
        continue;
      }
      if (c.sorted && c.pmin < kf) {  // dead rows are the prefix below kf's segment
        const size_t below = c.pane_off[(size_t)(kf - c.pmin)];
        rows_ -= below - c.dead;
        c.dead = below;
        c.live_from = kf;
        kept.push_back(std::move(c));
        continue;
      }
      if (c.pmin < kf && !c.pane_rows.empty() && kf <= c.pmax) {
        // rows below kf from the pane histogram; mark them dead unless they are half
        size_t below = 0;
        for (int64_t p = c.pmin; p < kf; ++p) below += c.pane_rows[(size_t)(p - c.pmin)];
        if (2 * below < c.size()) {
          rows_ -= below - c.dead;  // below >= c.dead: kf >= live_from
          c.dead = below;
          c.live_from = kf;
          kept.push_back(std::move(c));
          continue;
        }
      }
      if (c.pmin < kf) {
        Chunk f;
        for (size_t i = 0; i < c.size(); ++i) {
          if (c.pane[i] < kf) continue;
          f.key.push_back(c.key[i]);
          f.pane.push_back(c.pane[i]);
          f.acc.push_back(c.acc[i]);
          f.cnt.push_back(c.cnt[i]);
          f.dirty.push_back(c.dirty[i]);
          f.pmin = std::min(f.pmin, c.pane[i]);
          f.pmax = std::max(f.pmax, c.pane[i]);
        }
        rows_ -= c.size() - c.dead - f.size();
        if (f.size()) {
          if ((uint64_t)(f.pmax - f.pmin) < ((uint64_t)1 << 20)) f.count_panes();
          kept.push_back(std::move(f));
        }
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
        if (chunks_[ci].live(i)) idx.push_back({chunks_[ci].pane[i], chunks_[ci].key[i], ci, i});
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
    out.key.assign(m.key.begin(), m.key.end());
    out.pane.assign(m.pane.begin(), m.pane.end());
    out.acc.assign(m.acc.begin(), m.acc.end());
    out.cnt.assign(m.cnt.begin(), m.cnt.end());
    out.dirty.assign(m.dirty.begin(), m.dirty.end());
    chunks_.clear();
    rows_ = m.size();
    if (rows_ && (uint64_t)(m.pmax - m.pmin) < ((uint64_t)1 << 20)) {
      m.sorted = true;  // ordered by (pane, key)
      m.count_panes();
    }
    if (rows_) chunks_.push_back(std::move(m));
    return out;
  }

  void clear() {
    if (pf_.joinable()) pf_.join();
    chunks_.clear();
    spare_.clear();
    rows_ = 0;
  }
  // Spare chunks held for the next absorb (tests / metrics).
  size_t spare_chunks() {
    std::lock_guard<std::mutex> g(sp_mu_);
    return spare_.size();
  }
  void join_prefault() {
    if (pf_.joinable()) pf_.join();
  }

 private:
  // fn(t) for t in [0, T) on T host threads (the caller runs t = 0).
  template <class F>
  static void run_threads(size_t T, F&& fn) {
    if (T <= 1) {
      fn((size_t)0);
      return;
    }
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; ++t) th.emplace_back(fn, t);
    fn((size_t)0);
    for (auto& x : th) x.join();
  }
  static size_t host_threads(size_t rows, size_t per = (size_t)1 << 18) {
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max<size_t>(1, std::min<size_t>({(size_t)(hw ? hw : 1), (size_t)16,
                                                 rows / per + 1}));
  }
  // Counting sort of an eviction's rows by pane into `c` (zero-count rows dropped): threads
  // histogram their row range per pane, then scatter at (pane, thread) prefix offsets, so the
  // order inside a pane stays the input order.
  void absorb_sorted(Chunk& c, const uint64_t* key, const int64_t* pane, const int64_t* acc,
                     const int64_t* cnt, const uint8_t* dirty, size_t n) {
    const size_t P = (size_t)(c.pmax - c.pmin + 1);
    const size_t T = host_threads(n);
    std::vector<size_t> h(T * P, 0);
    const int64_t pmin = c.pmin;
    run_threads(T, [&](size_t t) {
      size_t* ht = h.data() + t * P;
      for (size_t i = n * t / T, e = n * (t + 1) / T; i < e; ++i)
        if (cnt[i]) ++ht[(size_t)(pane[i] - pmin)];
    });
    std::vector<size_t> off(T * P);
    c.pane_rows.assign(P, 0);
    c.pane_off.assign(P + 1, 0);
    size_t tot = 0;
    for (size_t p = 0; p < P; ++p) {
      c.pane_off[p] = tot;
      for (size_t t = 0; t < T; ++t) {
        off[t * P + p] = tot;
        tot += h[t * P + p];
      }
      c.pane_rows[p] = tot - c.pane_off[p];
    }
    c.pane_off[P] = tot;
    c.key.resize(tot);
    c.pane.resize(tot);
    c.acc.resize(tot);
    c.cnt.resize(tot);
    c.dirty.resize(tot);
    run_threads(T, [&](size_t t) {
      size_t* o = off.data() + t * P;
      for (size_t i = n * t / T, e = n * (t + 1) / T; i < e; ++i) {
        if (!cnt[i]) continue;
        const size_t q = o[(size_t)(pane[i] - pmin)]++;
        c.key[q] = key[i];
        c.pane[q] = pane[i];
        c.acc[q] = acc[i];
        c.cnt[q] = cnt[i];
        c.dirty[q] = dirty[i];
      }
    });
    c.sorted = true;
    // (pmin / pmax may bound panes whose rows were all zero-count: harmless)
  }

  // Spare columns for the next absorb: the spare with the most capacity (an eviction of n rows
  // into fresh columns pays its page faults -- ~10 GB/s of first touch -- on the caller).
  void take_spare(Chunk& c, size_t n) {
    std::lock_guard<std::mutex> g(sp_mu_);
    if (spare_.empty()) return;
    size_t best = 0;
    for (size_t i = 1; i < spare_.size(); ++i)
      if (spare_[i].key.capacity() > spare_[best].key.capacity()) best = i;
    (void)n;
    Chunk& sp = spare_[best];
    c.key.swap(sp.key);
    c.pane.swap(sp.pane);
    c.acc.swap(sp.acc);
    c.cnt.swap(sp.cnt);
    c.dirty.swap(sp.dirty);
    spare_.erase(spare_.begin() + (std::ptrdiff_t)best);
  }
  void give_spare(Chunk&& c) {
    std::lock_guard<std::mutex> g(sp_mu_);
    if (spare_.size() >= kMaxSpare) return;  // freed
    c.key.clear();
    c.pane.clear();
    c.acc.clear();
    c.cnt.clear();
    c.dirty.clear();
    spare_.push_back(std::move(c));
  }
  // After an absorb of n rows: unless a spare already holds 2 n rows, a background thread maps
  // and touches the columns of the next one, so the page faults run beside the stream's next
  // steps instead of inside the next absorb. Evictions grow with the key space: a 1.25 n spare
  // was outgrown often enough to leave 10 ms absorbs in config 4-spill.
  void prefault_async(size_t n) {
    if (!prefault_) return;
    const size_t want = 2 * n;
    {
      std::lock_guard<std::mutex> g(sp_mu_);
      for (auto& sp : spare_)
        if (sp.key.capacity() >= want) return;
      if (spare_.size() >= kMaxSpare) return;
    }
    if (pf_.joinable()) {
      if (!pf_done_.load(std::memory_order_acquire)) return;  // one at a time
      pf_.join();
    }
    pf_done_.store(false, std::memory_order_relaxed);
    pf_ = std::thread([this, want] {
      Chunk c;
      touch(c.key, want);
      touch(c.pane, want);
      touch(c.acc, want);
      touch(c.cnt, want);
      touch(c.dirty, want);
      give_spare(std::move(c));
      pf_done_.store(true, std::memory_order_release);
    });
  }
  template <class V>
  static void touch(V& v, size_t n) {
    v.resize(n);
    auto* b = reinterpret_cast<volatile unsigned char*>(v.data());
    const size_t bytes = n * sizeof(typename V::value_type);
    for (size_t o = 0; o < bytes; o += 4096) b[o] = 0;
  }
  static constexpr size_t kMaxSpare = 3;

 public:
  bool prefault_ = true;  // A/B knob (MXS_TIER_PREFAULT=0 on the Python side)

 private:

  int agg_;

  std::deque<Chunk> chunks_;
  std::mutex sp_mu_;
  std::thread pf_;
  std::atomic<bool> pf_done_{true};
  std::vector<Chunk> spare_;  // purged / pre-faulted chunks whose columns absorb() reuses
  size_t rows_ = 0;
  int64_t rows_in_ = 0;
};

}  // namespace mxs
