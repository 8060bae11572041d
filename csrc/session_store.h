// mxstream — host session-window store core (C++, no Python): shared by the pybind module
// (csrc/sessions.cpp: CPU engine + spill tier of the GPU session operator) and the C ABI
// (csrc/pipeline.cpp: mxs_session_*). Semantics: see csrc/sessions.cpp.
#ifndef MXS_SESSION_STORE_H_
#define MXS_SESSION_STORE_H_

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <queue>
#include <sys/mman.h>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "mxs_common.h"
#include "thread_pool.h"

namespace mxs {
namespace sess {

struct Session {
  int64_t start, end;  // [start, end)
  uint64_t acc;
  uint32_t cnt;
  uint32_t flags;      // bit0: fired, bit1: modified since firing
};

// A growable column of trivially copyable values whose resize does not initialise: an eviction
// of 10^5-10^6 rows into a cold chunk writes every element itself (std::vector's zero fill was a
// whole extra pass over the chunk's ~40 bytes a row).
template <class T>
struct PodVec {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  PodVec() = default;
  PodVec(const PodVec& o) { assign(o); }
  PodVec& operator=(const PodVec& o) {
    if (this != &o) assign(o);
    return *this;
  }
  PodVec(PodVec&& o) noexcept : p(o.p), n(o.n), cap(o.cap) {
    o.p = nullptr;
    o.n = o.cap = 0;
  }
  PodVec& operator=(PodVec&& o) noexcept {
    if (this != &o) {
      std::free(p);
      p = o.p;
      n = o.n;
      cap = o.cap;
      o.p = nullptr;
      o.n = o.cap = 0;
    }
    return *this;
  }
  ~PodVec() { std::free(p); }
  void assign(const PodVec& o) {
    resize(o.n);
    if (o.n) std::memcpy(p, o.p, o.n * sizeof(T));
  }
  void reserve(size_t m) {
    if (m <= cap) return;
    T* q = static_cast<T*>(std::realloc(p, m * sizeof(T)));
    if (!q) throw std::bad_alloc();
    p = q;
    cap = m;
  }
  void resize(size_t m) {  // new elements are NOT initialised
    reserve(m);
    n = m;
  }
  void clear() { n = 0; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  size_t capacity() const { return cap; }
  T* data() { return p; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T* begin() { return p; }
  T* end() { return p + n; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
};

struct ColdChunk {
  PodVec<uint64_t> key;
  PodVec<int64_t> start, end;
  PodVec<uint64_t> acc;
  PodVec<uint32_t> cnt;  // 0 = row gone (promoted or discarded)
  int64_t max_due = INT64_MIN;
  size_t live = 0;
  uint32_t seq = 0;  // identity in the dense cold-row index (SessionCore::loc_), 0 = none
  // Rows by key: promote() looks keys up by binary search or a merge join instead of probing a
  // hash set with every cold row of the store.
  std::vector<uint32_t> by_key;
  uint64_t kmin = ~0ull, kmax = 0;

  // Key range at sealing (O(n)); the sorted row index is built on the first promote() that
  // reaches this chunk, so chunks that are never revisited never pay for it.
  void seal() {
    for (uint64_t k : key) {
      kmin = k < kmin ? k : kmin;
      kmax = k > kmax ? k : kmax;
    }
  }
  void ensure_index() {
    if (by_key.size() == key.size()) return;
    const size_t n = key.size();
    const uint64_t span = n ? kmax - kmin : 0;
    if (n && span < ((uint64_t)1 << 32)) {
      // Keys within 2^32 of each other (dictionary ids, drifting id ranges): stable LSD radix
      // sort of the row ids by (key - kmin), 11-bit digits over the span's bits -- O(n) per
      // pass instead of an O(n log n) comparison sort (the chunks hold 10^5-10^6 rows).
      int bits = 0;
      while (bits < 64 && (span >> bits)) ++bits;
      std::vector<uint32_t> a(n), b(n);
      std::vector<uint32_t> off((size_t)1 << 11);
      for (size_t i = 0; i < n; ++i) a[i] = (uint32_t)i;
      for (int sh = 0; sh < bits || sh == 0; sh += 11) {
        std::fill(off.begin(), off.end(), 0u);
        for (size_t i = 0; i < n; ++i) ++off[((key[a[i]] - kmin) >> sh) & 2047u];
        uint32_t t = 0;
        for (auto& c : off) {
          const uint32_t x = c;
          c = t;
          t += x;
        }
        for (size_t i = 0; i < n; ++i) b[off[((key[a[i]] - kmin) >> sh) & 2047u]++] = a[i];
        a.swap(b);
        if (bits == 0) break;
      }
      by_key.swap(a);
      return;
    }
    // (key, row) pairs sorted contiguously: an index sort with key[] lookups in the comparator
    // was 5x slower (random reads).
    std::vector<std::pair<uint64_t, uint32_t>> kr(n);
    for (size_t i = 0; i < n; ++i) kr[i] = {key[i], (uint32_t)i};
    std::sort(kr.begin(), kr.end());
    by_key.resize(n);
    for (size_t i = 0; i < n; ++i) by_key[i] = kr[i].second;
  }
};

// Session rows as flat columns (key, start, end, acc, cnt, flags).
struct Columns {
  std::vector<int64_t> key, start, end, acc, cnt, flags;
  void add(uint64_t k, int64_t s, int64_t e, uint64_t a, uint32_t c, uint32_t f) {
    key.push_back((int64_t)k);
    start.push_back(s);
    end.push_back(e);
    acc.push_back((int64_t)a);
    cnt.push_back(c);
    flags.push_back(f);
  }
};

class SessionCore {
 public:
  SessionCore(int64_t gap, int64_t lateness, int agg) : gap_(gap), late_(lateness), agg_(agg) {
    if (gap <= 0) throw std::invalid_argument("session gap must be > 0");
  }

  // Fold a batch (keys, ts, vals) with the current watermark `wm`; returns late-dropped count.
  int64_t process(const int64_t* k, const int64_t* t, const int64_t* v, int64_t n, int64_t wm) {
    promote(k, n, wm);
    // Sort the records themselves by (key, ts) (contiguous, no indirect compares): every
    // aggregate is a commutative monoid, so the order of equal (key, ts) records is free.
    struct KTV {
      uint64_t k;
      int64_t t, v;
    };
    std::vector<KTV> r(n);
    for (int64_t i = 0; i < n; ++i) r[i] = KTV{(uint64_t)k[i], t[i], v[i]};
    std::sort(r.begin(), r.end(),
              [](const KTV& a, const KTV& b) { return a.k != b.k ? a.k < b.k : a.t < b.t; });
    int64_t late = 0;
    int64_t i = 0;
    while (i < n) {
      const uint64_t key = r[i].k;
      int64_t j = i;
      while (j < n && r[j].k == key) ++j;
      int64_t q0 = i;
      while (q0 < j) {
        Session c{r[q0].t, r[q0].t + gap_, agg_lift(agg_, (uint64_t)r[q0].v), 1u, 0u};
        int64_t q = q0 + 1;
        while (q < j && r[q].t <= c.end) {  // intersects (touching merges)
          c.end = std::max(c.end, r[q].t + gap_);
          c.acc = agg_combine(agg_, c.acc, agg_lift(agg_, (uint64_t)r[q].v));
          c.cnt += 1;
          ++q;
        }
        late += merge_candidate(key, c, wm);
        q0 = q;
      }
      i = j;
    }
    return late;
  }

  // Merge pre-built runs (GPU overflow path): each is a candidate session.
  int64_t merge_runs(const int64_t* keys, const int64_t* starts, const int64_t* ends,
                     const int64_t* accs, const int64_t* cnts, int64_t n, int64_t wm) {
    promote(keys, n, wm);
    int64_t late = 0;
    for (int64_t i = 0; i < n; ++i) {
      Session c{starts[i], ends[i], (uint64_t)accs[i], (uint32_t)cnts[i], 0u};
      late += merge_candidate((uint64_t)keys[i], c, wm);
    }
    return late;
  }

  // Insert sessions evicted from HBM. Arrays: key, start, end, acc, cnt, flags. With `cold`,
  // fired-and-unmodified sessions of keys without hot state go to one new cold chunk.
  // Three phases, so the asynchronous spill worker (csrc/sessions.cpp) can hold the store's lock
  // only where the store is touched: insert_hot (classify every row, hot rows into the map),
  // build_cold (the cold rows copied into a chunk: no store state), publish_cold (the chunk
  // joins the store).
  struct ColdPlan {
    ColdChunk ch;
    std::vector<uint8_t> isc;  // per row: 1 = goes to the cold chunk
    int64_t nc = 0, emax = INT64_MIN;
    double t_populate = 0;  // s: index_cold's synchronous page population (spill worker timers)
    bool emax_pending = false;  // all-cold fast path: emax (and nkeys) computed by the build
    int64_t nkeys = -1;         // distinct keys of the rows (runs of equal keys), from the build
    bool indexed = false;  // index_cold() ran (the spill worker runs it outside the lock)
  };
  void insert(const int64_t* K, const int64_t* S, const int64_t* E, const int64_t* A,
              const int64_t* C, const int64_t* F, int64_t n, bool cold) {
    ColdPlan p;
    insert_hot(K, S, E, A, C, F, n, cold, p);
    if (cold) {
      build_cold_parallel(K, S, E, A, C, n, p);
      index_cold(p);
      publish_cold(p);
    }
  }
  // all_fired: the caller checked (outside the store lock) that every row has F == 1.
  void insert_hot(const int64_t* K, const int64_t* S, const int64_t* E, const int64_t* A,
                  const int64_t* C, const int64_t* F, int64_t n, bool cold, ColdPlan& p,
                  bool all_fired = false) {
    refresh_hot_filter();
    if (cold && !spare_.empty()) {
      // A dropped chunk's columns: capacity whose pages are already mapped. Fresh columns of a
      // 400K-row eviction cost ~3500 page faults, most of the insert's time.
      p.ch = std::move(spare_.back());
      spare_.pop_back();
    }
    const bool no_hot = m_.empty();
    if (cold && no_hot && all_fired) {
      // The common eviction (config 5) with the rows pre-checked: every row is cold. O(1)
      // under the store lock -- the build (outside it, on the pool) takes emax and the keys.
      p.nc = n;
      p.emax_pending = true;
      return;
    }
    // Row i goes to the cold chunk iff it fired unmodified (F == 1) and its key is not hot --
    // hot already at the call, or made hot by an EARLIER row of this call (the serial rule).
    // (key, first row) of the rows that turn keys hot, sorted by key, behind a bit filter: a
    // cold-eligible row pays one bit test unless its key also has such a row.
    std::vector<std::pair<uint64_t, int64_t>> first_hot;
    std::vector<uint64_t> fh_bits;
    uint64_t fh_mask = 0;
    if (cold) {
      for (int64_t i = 0; i < n; ++i)
        if (F[i] != 1) first_hot.push_back({(uint64_t)K[i], i});
      if (!first_hot.empty()) {
        std::sort(first_hot.begin(), first_hot.end());  // (key, row): the first row leads
        size_t nb = 64;
        while (nb < first_hot.size() * 16) nb <<= 1;
        fh_bits.assign(nb / 64, 0);
        fh_mask = nb - 1;
        for (auto& kv : first_hot) {
          const uint64_t b = mix64(kv.first) & fh_mask;
          fh_bits[b >> 6] |= 1ull << (b & 63);
        }
      }
    }
    auto goes_cold = [&](int64_t i) -> bool {
      if (!cold || F[i] != 1) return false;
      const uint64_t key = (uint64_t)K[i];
      if (!no_hot && is_hot(key)) return false;
      if (!first_hot.empty()) {
        const uint64_t b = mix64(key) & fh_mask;
        if ((fh_bits[b >> 6] >> (b & 63)) & 1ull) {
          auto f = std::lower_bound(first_hot.begin(), first_hot.end(),
                                    std::make_pair(key, (int64_t)INT64_MIN));
          if (f != first_hot.end() && f->first == key && f->second < i) return false;
        }
      }
      return true;
    };
    if (cold && no_hot && first_hot.empty()) {
      // The common eviction (config 5): no hot state and every row fired unmodified -- every
      // row is cold, no per-row classification (build_cold reads isc only when nc < n).
      int64_t em = INT64_MIN;
      for (int64_t i = 0; i < n; ++i) em = E[i] > em ? E[i] : em;
      p.nc = n;
      p.emax = em;
      return;
    }
    if (cold) {
      p.isc.resize((size_t)n);
      int64_t c = 0, em = INT64_MIN;
      for (int64_t i = 0; i < n; ++i) {
        const uint8_t x = goes_cold(i) ? 1 : 0;
        p.isc[i] = x;
        if (x) {
          ++c;
          em = E[i] > em ? E[i] : em;
        }
      }
      p.nc = c;
      p.emax = em;
      if (c == n) return;  // every row cold: nothing for the hot map
    }
    for (int64_t i = 0; i < n; ++i) {
      if (cold && p.isc[i]) continue;
      const uint64_t key = (uint64_t)K[i];
      m_[key].push_back(Session{S[i], E[i], (uint64_t)A[i], (uint32_t)C[i], (uint32_t)F[i]});
      mark_hot(key);
      schedule(key);
    }
  }
  // build_cold with the common all-cold copy split into row blocks on the store's pool (the
  // spill worker's build phase: ~12 MB of column copies per eviction, mostly first-touch page
  // faults of the chunk's fresh columns). Reads the store's pool only: outside the lock.
  void build_cold_parallel(const int64_t* K, const int64_t* S, const int64_t* E, const int64_t* A,
                           const int64_t* C, int64_t n, ColdPlan& p) {
    constexpr int64_t kBlk = 65536;
    if (p.nc != n || n < 2 * kBlk) return build_cold(K, S, E, A, C, n, p);
    if (!pool_) {
      unsigned hw = std::thread::hardware_concurrency();
      pool_.reset(new WorkerPool(std::max(0, std::min<int>(hw ? (int)hw : 1, max_threads_) - 1)));
    }
    ColdChunk& ch = p.ch;
    ch.key.resize(n);
    ch.start.resize(n);
    ch.end.resize(n);
    ch.acc.resize(n);
    ch.cnt.resize(n);
    const int nb = (int)((n + kBlk - 1) / kBlk);
    std::vector<uint64_t> lo((size_t)nb, ~0ull), hi((size_t)nb, 0);
    std::vector<int64_t> em((size_t)nb, INT64_MIN), runs((size_t)nb, 0);
    pool_->run(nb, [&](int b) {
      const int64_t a = (int64_t)b * kBlk, m = std::min(n, a + kBlk) - a;
      std::memcpy(ch.key.data() + a, K + a, (size_t)m * 8);
      std::memcpy(ch.start.data() + a, S + a, (size_t)m * 8);
      std::memcpy(ch.end.data() + a, E + a, (size_t)m * 8);
      std::memcpy(ch.acc.data() + a, A + a, (size_t)m * 8);
      uint64_t l = ~0ull, h = 0;
      int64_t e = INT64_MIN, r = 0;
      for (int64_t i = a; i < a + m; ++i) {
        ch.cnt[i] = (uint32_t)C[i];
        const uint64_t k = (uint64_t)K[i];
        l = k < l ? k : l;
        h = k > h ? k : h;
        e = E[i] > e ? E[i] : e;
        r += i == 0 || K[i] != K[i - 1];  // a new run of equal keys starts here
      }
      lo[(size_t)b] = l;
      hi[(size_t)b] = h;
      em[(size_t)b] = e;
      runs[(size_t)b] = r;
    });
    int64_t e = INT64_MIN, r = 0;
    for (int b = 0; b < nb; ++b) {
      ch.kmin = std::min(ch.kmin, lo[(size_t)b]);
      ch.kmax = std::max(ch.kmax, hi[(size_t)b]);
      e = std::max(e, em[(size_t)b]);
      r += runs[(size_t)b];
    }
    if (p.emax_pending) {
      p.emax = e;
      p.emax_pending = false;
    }
    p.nkeys = r;
  }
  // The classified cold rows into p.ch (touches no store state: runs outside the store lock).
  static void build_cold(const int64_t* K, const int64_t* S, const int64_t* E, const int64_t* A,
                         const int64_t* C, int64_t n, ColdPlan& p) {
    ColdChunk& ch = p.ch;
    if (p.emax_pending) {  // (all-cold fast path: every row is cold)
      int64_t e = INT64_MIN;
      for (int64_t i = 0; i < n; ++i) e = E[i] > e ? E[i] : e;
      p.emax = e;
      p.emax_pending = false;
    }
    const int64_t nc = p.nc;
    ch.key.resize(nc);
    ch.start.resize(nc);
    ch.end.resize(nc);
    ch.acc.resize(nc);
    ch.cnt.resize(nc);
    if (nc == n) {  // the common eviction: every row cold, straight column copies
      std::memcpy(ch.key.data(), K, (size_t)n * 8);
      std::memcpy(ch.start.data(), S, (size_t)n * 8);
      std::memcpy(ch.end.data(), E, (size_t)n * 8);
      std::memcpy(ch.acc.data(), A, (size_t)n * 8);
      for (int64_t i = 0; i < n; ++i) ch.cnt[i] = (uint32_t)C[i];
    } else {
      int64_t o = 0;
      for (int64_t i = 0; i < n; ++i) {
        if (!p.isc[i]) continue;
        ch.key[o] = (uint64_t)K[i];
        ch.start[o] = S[i];
        ch.end[o] = E[i];
        ch.acc[o] = (uint64_t)A[i];
        ch.cnt[o] = (uint32_t)C[i];
        ++o;
      }
    }
    if (nc) ch.seal();
  }
  void publish_cold(ColdPlan& p) {
    ColdChunk& ch = p.ch;
    if (ch.key.empty()) {
      if (ch.key.capacity() && spare_.size() < 4) spare_.push_back(std::move(ch));
      return;
    }
    if (!p.indexed) index_cold(p);
    ch.max_due = std::max(ch.max_due, cleanup_time(p.emax - 1));
    ch.live = ch.key.size();
    cold_rows_ += ch.live;
    if (ch.seq) set_seq_pos(ch.seq, (int32_t)cold_.size());
    cold_.push_back(std::move(ch));
  }

  // Dense cold-row index: loc_[key - loc_base_] = (chunk seq << 32 | row) of the first cold
  // row of the key's run in its chunk (an evicted slot's sessions are adjacent rows), so an
  // extract finds the rows of its wanted keys with one lookup per key instead of a scan of
  // every cold row of the store (config 5 with revisits: ~10^5 wanted keys against ~10^7 cold
  // rows per step). An entry is trusted only after checking that its chunk is still in the
  // store and that its row still holds the key with cnt > 0 (taken rows, expired chunks and
  // reused chunk memory leave stale entries behind). A key with live rows in two chunks (or two
  // runs of one chunk) is marked kMultiLoc and sends the extract that wants it to the scan.
  // The index is one reserved virtual range of kMaxLocSpan entries (no copies as it grows:
  // untouched pages cost nothing); keys outside it (hashed keys) switch it off for good.
  // Runs outside the store lock in the spill worker (every other index user joins the worker
  // first): the chunk is not published yet, so its own rows are checked against `p.ch`.
  void index_cold(ColdPlan& p) {
    p.indexed = true;
    ColdChunk& ch = p.ch;
    ch.seq = 0;
    if (ch.key.empty() || loc_off_) return;
    if (!loc_) {
      void* m = ::mmap(nullptr, kMaxLocSpan * sizeof(uint64_t), PROT_READ | PROT_WRITE,
                       MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
      if (m == MAP_FAILED) {
        loc_off_ = true;
        return;
      }
      // 4 KB pages: huge pages (MADV_HUGEPAGE) populated here stalled the stepping thread by
      // ~3 ms per step in config 5 with revisits (profiles/r5_index_paging.md); opt-in
      if (env_flag("MXS_INDEX_THP", false)) (void)::madvise(m, kMaxLocSpan * sizeof(uint64_t), MADV_HUGEPAGE);
      loc_ = static_cast<uint64_t*>(m);
      // room below the first keys for ids a little older than them
      loc_base_ = ch.kmin > kMaxLocSpan / 8 ? ch.kmin - kMaxLocSpan / 8 : 0;
      pop_lo_ = ch.kmin - loc_base_;
      pop_hi_.store(pop_lo_);
    }
    if (ch.kmin < loc_base_ || ch.kmax - loc_base_ >= kMaxLocSpan) {
      drop_index();
      return;
    }
    ch.seq = next_seq_++;
    // Entries of ids never seen before sit on fresh pages: mapped in one call
    // (MADV_POPULATE_WRITE, Linux 5.14+; an error just leaves them to the faults below) instead
    // of one page fault per 4 KB from the store passes, which the mm lock serialises -- and,
    // for ids above the mapped range (drifting key spaces), ahead of need on a background
    // thread, so the worker's index phase finds its pages mapped.
    if (env_flag("MXS_INDEX_POPULATE", true)) {
      const auto tp0 = std::chrono::steady_clock::now();
      const size_t lo = ch.kmin - loc_base_, hi = ch.kmax - loc_base_ + 1;
      if (lo < pop_lo_) {
        populate(lo, pop_lo_);
        pop_lo_ = lo;
      }
      const size_t ph = pop_hi_.load();
      if (hi > ph) {
        populate(ph, hi);
        size_t cur = pop_hi_.load();
        while (cur < hi && !pop_hi_.compare_exchange_weak(cur, hi)) {
        }
      }
      populate_ahead(hi);
      p.t_populate += std::chrono::duration<double>(std::chrono::steady_clock::now() - tp0).count();
    }
    // Row blocks on the pool, two passes of relaxed (plain) stores -- atomic read-modify-writes
    // serialize every cache miss, key-range tasks re-read the key column per task:
    //  1. every run's first row stores its entry, or kMultiLoc over a live entry of another row;
    //  2. every run's first row reads its entry back: another row's entry there means a second
    //     run of the key in this chunk (its writer lost the race) -> kMultiLoc.
    const uint32_t cur = ch.seq;
    const size_t n = ch.key.size();
    auto entry = [&](uint64_t k) { return loc_ + (k - loc_base_); };
    auto first_of_run = [&](size_t r) { return r == 0 || ch.key[r - 1] != ch.key[r]; };
    auto pass1 = [&](size_t lo, size_t hi) {
      for (size_t r = lo; r < hi; ++r) {
        if (!first_of_run(r)) continue;  // a run's later rows: reached from its first
        const uint64_t k = ch.key[r];
        uint64_t* e = entry(k);
        const uint64_t old = __atomic_load_n(e, __ATOMIC_RELAXED);
        if (old == kMultiLoc) continue;
        uint64_t want = ((uint64_t)cur << 32) | (uint64_t)r;
        if (old != kNoLoc) {
          const uint32_t es = (uint32_t)(old >> 32), er = (uint32_t)old;
          const bool live = es == cur ? (er < n && er != r && ch.key[er] == k && ch.cnt[er])
                                      : live_loc(old, k);
          if (live) want = kMultiLoc;
        }
        __atomic_store_n(e, want, __ATOMIC_RELAXED);
      }
    };
    auto pass2 = [&](size_t lo, size_t hi) {
      for (size_t r = lo; r < hi; ++r) {
        if (!first_of_run(r)) continue;
        uint64_t* e = entry(ch.key[r]);
        const uint64_t v = __atomic_load_n(e, __ATOMIC_RELAXED);
        if (v != kMultiLoc && v != (((uint64_t)cur << 32) | (uint64_t)r))
          __atomic_store_n(e, kMultiLoc, __ATOMIC_RELAXED);
      }
    };
    constexpr size_t kBlk = 32768;
    const int nb = (int)((n + kBlk - 1) / kBlk);
    if (nb <= 1) {
      pass1(0, n);
      pass2(0, n);
      return;
    }
    if (!pool_) {
      unsigned hw = std::thread::hardware_concurrency();
      pool_.reset(new WorkerPool(std::max(0, std::min<int>(hw ? (int)hw : 1, max_threads_) - 1)));
    }
    pool_->run(nb, [&](int b) { pass1((size_t)b * kBlk, std::min(n, (size_t)(b + 1) * kBlk)); });
    pool_->run(nb, [&](int b) { pass2((size_t)b * kBlk, std::min(n, (size_t)(b + 1) * kBlk)); });
  }
  ~SessionCore() { drop_index(); }

  // Hand keys back to the HBM tier: every listed key with at most `max_sess` live sessions
  // leaves the store (hot sessions and cold rows; rows past cleanup at `wm` are dropped).
  // Returns its sessions as columns grouped by key (keys ascending) plus "moved": every listed
  // key that is no longer in the store (its spill-set entry can go). Keys with more sessions
  // than an HBM slot holds stay here.
  Columns extract(const int64_t* keys, int64_t n, int64_t wm, int64_t max_sess,
                  std::vector<int64_t>* moved) {
    // Dense key spans (dictionary ids, drifting id ranges -- every keyed state here is fed by
    // those): the wanted set is a bitmap over [wmin, wmax] and cold rows are grouped by a
    // counting sort on the key offset, O(n + span) instead of sorts and hash probes.
    uint64_t wmin = ~0ull, wmax = 0;
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t k = (uint64_t)keys[i];
      wmin = k < wmin ? k : wmin;
      wmax = k > wmax ? k : wmax;
    }
    const uint64_t wspan = n ? wmax - wmin + 1 : 0;
    // The bitmap (<= 16 MB) pays even for few keys in a wide span: membership tests in a
    // chunk scan stay sequential and cache-resident (a hash-set probe per cold row cost 20 ns).
    const bool dense = n && wspan <= ((uint64_t)1 << 27);
    std::vector<uint64_t> want;
    std::vector<uint64_t> wbits;  // dense: bit (key - wmin) set for wanted keys
    if (dense) {
      wbits.assign((wspan + 63) / 64, 0);
      for (int64_t i = 0; i < n; ++i) {
        const uint64_t o = (uint64_t)keys[i] - wmin;
        wbits[o >> 6] |= 1ull << (o & 63);
      }
      for (size_t w = 0; w < wbits.size(); ++w)
        for (uint64_t b = wbits[w]; b; b &= b - 1)
          want.push_back(wmin + (w << 6) + (uint64_t)__builtin_ctzll(b));
    } else {
      want.assign((const uint64_t*)keys, (const uint64_t*)keys + n);
      std::sort(want.begin(), want.end());
      want.erase(std::unique(want.begin(), want.end()), want.end());
    }
    auto wanted_dense = [&](uint64_t k) {
      const uint64_t o = k - wmin;
      return k >= wmin && o < wspan && ((wbits[o >> 6] >> (o & 63)) & 1ull);
    };
    // Cold rows of the wanted keys come straight out of their chunks (no detour through the hot
    // map); rows already past cleanup at `wm` are dropped, as a promote would.
    std::vector<std::pair<uint64_t, Session>> cold;
    std::vector<uint64_t> wset;  // hash set of `want`, built on first use
    size_t wmask = 0;
    const bool indexed = cold_rows_ && !want.empty() && take_indexed(want, wm, cold);
    if (cold_rows_ && !want.empty() && !indexed) ++ixs_.scans;
    if (cold_rows_ && !want.empty() && !indexed) {
      // Dense keys: the chunks that need a full scan (no row index, or many wanted keys --
      // every chunk of scattered evictions spans the whole id range) are scanned in parallel,
      // one chunk per task; their rows lead `cold` (a key's rows keep their order: they sit in
      // one chunk, and the key sort below is stable).
      std::vector<char> pdone;
      if (dense) {
        std::vector<size_t> scan;
        size_t rows = 0;
        for (size_t ci = 0; ci < cold_.size(); ++ci) {
          const ColdChunk& ch = cold_[ci];
          if (!ch.live || want.back() < ch.kmin || want.front() > ch.kmax) continue;
          auto lo = std::lower_bound(want.begin(), want.end(), ch.kmin);
          auto hi = std::upper_bound(lo, want.end(), ch.kmax);
          const size_t nw = (size_t)(hi - lo), nc = ch.key.size();
          if (lo != hi && (ch.by_key.size() != nc || nw * 20 >= nc)) {
            scan.push_back(ci);
            rows += nc;
          }
        }
        unsigned hw = std::thread::hardware_concurrency();
        const size_t nth = std::min<size_t>({scan.size(), hw ? hw : 1, (size_t)max_threads_,
                                             rows / 65536 + 1});
        if (nth > 1) {
          // Two passes, each one chunk per task: count the kept rows, then write them at their
          // offsets in `cold` (growing per-task vectors cost more in page faults and unmaps
          // than the scan itself).
          pdone.assign(cold_.size(), 0);
          std::vector<size_t> keep(scan.size() + 1, 0), gone(scan.size(), 0);
          auto pfor = [&](auto&& body) {
            std::atomic<size_t> next{0};
            auto work = [&] {
              for (size_t j; (j = next.fetch_add(1)) < scan.size();) body(j);
            };
            std::vector<std::thread> th;
            for (size_t t = 1; t < nth; ++t) th.emplace_back(work);
            work();
            for (auto& t : th) t.join();
          };
          pfor([&](size_t j) {
            const ColdChunk& ch = cold_[scan[j]];
            const uint32_t nc = (uint32_t)ch.key.size();
            size_t k = 0, g = 0;
            for (uint32_t r = 0; r < nc; ++r) {
              if (!ch.cnt[r] || !wanted_dense(ch.key[r])) continue;
              ++g;
              k += cleanup_time(ch.end[r] - 1) > wm;
            }
            keep[j + 1] = k;
            gone[j] = g;
          });
          for (size_t j = 0; j < scan.size(); ++j) keep[j + 1] += keep[j];
          cold.resize(keep[scan.size()]);
          pfor([&](size_t j) {
            ColdChunk& ch = cold_[scan[j]];
            const uint32_t nc = (uint32_t)ch.key.size();
            auto* o = cold.data() + keep[j];
            for (uint32_t r = 0; r < nc; ++r) {
              if (!ch.cnt[r] || !wanted_dense(ch.key[r])) continue;
              if (cleanup_time(ch.end[r] - 1) > wm)
                *o++ = {ch.key[r], Session{ch.start[r], ch.end[r], ch.acc[r], ch.cnt[r], 1u}};
              ch.cnt[r] = 0;
            }
            ch.live -= gone[j];
          });
          for (size_t j = 0; j < scan.size(); ++j) {
            pdone[scan[j]] = 1;
            cold_rows_ -= gone[j];
          }
        }
      }
      for (size_t ci = 0; ci < cold_.size(); ++ci) {
        auto& ch = cold_[ci];
        if (!pdone.empty() && pdone[ci]) continue;  // scanned above
        if (!ch.live || want.back() < ch.kmin || want.front() > ch.kmax) continue;
        auto lo = std::lower_bound(want.begin(), want.end(), ch.kmin);
        auto hi = std::upper_bound(lo, want.end(), ch.kmax);
        if (lo == hi) continue;
        auto take = [&](uint32_t r) {
          if (!ch.cnt[r]) return;
          if (cleanup_time(ch.end[r] - 1) > wm)
            cold.push_back({ch.key[r], Session{ch.start[r], ch.end[r], ch.acc[r], ch.cnt[r], 1u}});
          ch.cnt[r] = 0;
          ch.live -= 1;
          cold_rows_ -= 1;
        };
        const size_t nw = (size_t)(hi - lo), nc = ch.key.size();
        if (dense && (ch.by_key.size() != nc || nw * 20 >= nc)) {
          for (uint32_t r = 0; r < (uint32_t)nc; ++r)
            if (ch.cnt[r] && wanted_dense(ch.key[r])) take(r);
          continue;
        }
        if (ch.by_key.size() != nc && nw * 20 >= nc) {
          // Many wanted keys and no row index yet: one pass over the chunk probing a hash set
          // of the wanted keys (sorting the chunk's 10^5-10^6 rows for an index costs more).
          if (wset.empty()) {
            size_t cap = 16;
            while (cap < 2 * want.size()) cap <<= 1;
            wset.assign(cap, kEmptyKey);
            wmask = cap - 1;
            for (uint64_t k : want) {
              size_t h = (size_t)(mix64(k) >> 32) & wmask;
              while (wset[h] != kEmptyKey && wset[h] != k) h = (h + 1) & wmask;
              wset[h] = k;
            }
          }
          for (uint32_t r = 0; r < (uint32_t)nc; ++r) {
            const uint64_t k = ch.key[r];
            if (!ch.cnt[r] || k < *lo || k > *(hi - 1)) continue;
            size_t h = (size_t)(mix64(k) >> 32) & wmask;
            while (wset[h] != kEmptyKey && wset[h] != k) h = (h + 1) & wmask;
            if (wset[h] == k) take(r);
          }
          continue;
        }
        ch.ensure_index();
        for (auto it = lo; it != hi; ++it) {
          auto p = std::lower_bound(ch.by_key.begin(), ch.by_key.end(), *it,
                                    [&](uint32_t r, uint64_t k) { return ch.key[r] < k; });
          for (; p != ch.by_key.end() && ch.key[*p] == *it; ++p) take(*p);
        }
      }
      if (dense && cold.size() > 1 && wspan <= (uint64_t)4 * cold.size() + 65536) {
        // stable counting sort by key offset (same order as the stable comparison sort)
        std::vector<uint32_t> cnt(wspan + 1, 0);
        for (const auto& c : cold) ++cnt[c.first - wmin + 1];
        for (size_t i = 1; i < cnt.size(); ++i) cnt[i] += cnt[i - 1];
        std::vector<std::pair<uint64_t, Session>> sorted(cold.size());
        for (const auto& c : cold) sorted[cnt[c.first - wmin]++] = c;
        cold.swap(sorted);
      } else if (cold.size() > 1 && cold.size() < ((size_t)1 << 24) && wspan != 0 &&
                 64 - __builtin_clzll(wspan | 1) + 24 <= 64) {
        // Few rows in a wide key span: LSD radix sort of (key offset << 24 | row) words, 11-bit
        // digits (a stable_sort of the 40-byte rows moved ~100 MB for 10^5 rows). The row
        // index in the low bits keeps equal keys in their original order.
        const int kb = 64 - __builtin_clzll(wspan | 1) + 24;
        std::vector<uint64_t> a(cold.size()), b(cold.size());
        for (size_t i = 0; i < cold.size(); ++i) a[i] = ((cold[i].first - wmin) << 24) | i;
        std::vector<uint32_t> off(2048);
        for (int sh = 24; sh < kb; sh += 11) {  // the row bits are already in order
          std::fill(off.begin(), off.end(), 0u);
          for (uint64_t x : a) ++off[(x >> sh) & 2047u];
          uint32_t t = 0;
          for (auto& c : off) {
            const uint32_t y = c;
            c = t;
            t += y;
          }
          for (uint64_t x : a) b[off[(x >> sh) & 2047u]++] = x;
          a.swap(b);
        }
        std::vector<std::pair<uint64_t, Session>> sorted(cold.size());
        for (size_t i = 0; i < a.size(); ++i) sorted[i] = cold[a[i] & 0xFFFFFFu];
        cold.swap(sorted);
      } else if (cold.size() > 1) {
        std::stable_sort(cold.begin(), cold.end(),
                         [](const auto& a, const auto& b) { return a.first < b.first; });
      }
      forget_keys(want);  // every cold row of the wanted keys is gone (moved or turned hot)
    }
    const bool no_hot = m_.empty();
    Columns out;
    for (auto* v : {&out.key, &out.start, &out.end, &out.acc, &out.cnt, &out.flags})
      v->reserve(cold.size() + (no_hot ? 0 : want.size()));
    moved->reserve(moved->size() + want.size());
    size_t c = 0;
    for (uint64_t key : want) {
      const size_t c0 = c;
      while (c < cold.size() && cold[c].first < key) ++c;  // (cannot happen: keys are wanted)
      const size_t cb = c;
      while (c < cold.size() && cold[c].first == key) ++c;
      (void)c0;
      auto it = no_hot ? m_.end() : m_.find(key);
      const int64_t nhot = it == m_.end() ? 0 : (int64_t)it->second.size();
      if (nhot + (int64_t)(c - cb) > max_sess) {  // stays on the host: cold rows turn hot
        auto& vec = m_[key];
        mark_hot(key);
        for (size_t q = cb; q < c; ++q) vec.push_back(cold[q].second);
        schedule(key);
        continue;
      }
      if (it != m_.end()) {
        for (const Session& x : it->second) out.add(key, x.start, x.end, x.acc, x.cnt, x.flags);
        m_.erase(it);  // its heap entries turn stale
      }
      for (size_t q = cb; q < c; ++q) {
        const Session& x = cold[q].second;
        out.add(key, x.start, x.end, x.acc, x.cnt, x.flags);
      }
      moved->push_back((int64_t)key);
    }
    return out;
  }

  // Counters of the dense cold-row index: extracts served by it, sent to the scan by a
  // multi-row key, declined by hot keys (direct promote rows), full scans, index switched off.
  struct IndexStats {
    int64_t indexed = 0, multi = 0, hot = 0, scans = 0, off = 0, span = 0;
  };
  IndexStats index_stats() const {
    IndexStats t = ixs_;
    t.off = loc_off_ ? 1 : 0;
    t.span = loc_ ? (int64_t)kMaxLocSpan : 0;
    return t;
  }

  // The promote path's extract laid out for the HBM slot records in caller memory (pinned,
  // reused): one row of kPromoteRow int64 per returned session {key, start, end, acc,
  // cnt | flags << 32, last activity of the key (max end - gap), position of the session in its
  // key, sessions of the key}; rows of a key are adjacent, position 0 first. `moved` receives
  // the keys that left the store. Returns {rows, moved}.
  static constexpr int kPromoteRow = 8;
  // The keys ascending without duplicates: a copy when they already are, a bitmap over their
  // span for dense ids (the promote path passes a step's diverted record keys as they come,
  // ~10^5 with repeats), a sort otherwise.
  static void sort_unique_keys(const int64_t* keys, int64_t n, std::vector<uint64_t>& out,
                               std::vector<uint64_t>& bits) {
    const uint64_t* k = (const uint64_t*)keys;
    out.clear();
    if (n <= 0) return;
    bool sorted = true;
    uint64_t lo = k[0], hi = k[0];
    for (int64_t i = 1; i < n; ++i) {
      sorted = sorted && k[i - 1] < k[i];
      lo = k[i] < lo ? k[i] : lo;
      hi = k[i] > hi ? k[i] : hi;
    }
    if (sorted) {
      out.assign(k, k + n);
      return;
    }
    const uint64_t span = hi - lo + 1;
    if (span != 0 && span <= ((uint64_t)1 << 28) && span / 64 <= (uint64_t)n * 4) {
      bits.assign((size_t)((span + 63) / 64), 0);
      for (int64_t i = 0; i < n; ++i) {
        const uint64_t o = k[i] - lo;
        bits[o >> 6] |= 1ull << (o & 63);
      }
      for (size_t w = 0; w < bits.size(); ++w)
        for (uint64_t b = bits[w]; b; b &= b - 1)
          out.push_back(lo + (w << 6) + (uint64_t)__builtin_ctzll(b));
      return;
    }
    out.assign(k, k + n);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
  }
  // Returns {rows, moved keys, distinct wanted keys}; `keys` may repeat and come in any order.
  std::tuple<int64_t, int64_t, int64_t> extract_rows_into(const int64_t* keys, int64_t n,
                                                          int64_t wm, int64_t max_sess,
                                                          int64_t gap, int64_t* rows, int64_t cap,
                                                          int64_t* moved_out,
                                                          int64_t moved_cap) {
    std::vector<uint64_t>& want = ix_want_;
    sort_unique_keys(keys, n, want, ix_bits_);
    const int64_t nu = (int64_t)want.size();
    // No hot sessions among the wanted keys and at most max_sess cold rows per key in one
    // place (the revisit shape): the rows go from the chunks straight into `rows`.
    if (max_sess >= 1 && index_usable() && nu > 0) {
      if ((int64_t)want.size() > moved_cap)
        throw std::length_error("extract_rows_into: moved capacity");
      int64_t nk = 0;
      const bool ok = take_indexed_with(
          want, wm, true, (size_t)max_sess,
          [&](size_t total) {
            if ((int64_t)total > cap) throw std::length_error("extract_rows_into: row capacity");
            nk = (int64_t)total;
          },
          [&](size_t o, const ColdChunk& ch, uint32_t r, uint32_t j, uint32_t nkey,
              int64_t last_end) {
            int64_t* w = rows + o * kPromoteRow;
            w[0] = (int64_t)ch.key[r];
            w[1] = ch.start[r];
            w[2] = ch.end[r];
            w[3] = (int64_t)ch.acc[r];
            w[4] = (int64_t)(((uint64_t)ch.cnt[r] & 0xFFFFFFFFull) | (1ull << 32));  // fired
            w[5] = last_end - gap;
            w[6] = j;
            w[7] = nkey;
          });
      if (ok) {
        std::memcpy(moved_out, want.data(), want.size() * sizeof(int64_t));
        return {nk, nu, nu};
      }
    }
    std::vector<int64_t> moved;
    const std::vector<uint64_t> uniq(want);  // (extract reuses the scratch)
    const Columns c = extract((const int64_t*)uniq.data(), nu, wm, max_sess, &moved);
    const auto r = promote_rows(c, moved, gap, rows, cap, moved_out, moved_cap);
    return {r.first, r.second, nu};
  }
  // extract()'s output (keys grouped, ascending) as promote rows + the moved keys.
  static std::pair<int64_t, int64_t> promote_rows(const Columns& c,
                                                  const std::vector<int64_t>& moved, int64_t gap,
                                                  int64_t* rows, int64_t cap, int64_t* moved_out,
                                                  int64_t moved_cap) {
    const size_t m = c.key.size();
    if ((int64_t)m > cap) throw std::length_error("extract_rows_into: row capacity");
    if ((int64_t)moved.size() > moved_cap) throw std::length_error("extract_rows_into: moved capacity");
    for (size_t i = 0; i < m;) {
      size_t j = i;
      int64_t last = INT64_MIN;
      while (j < m && c.key[j] == c.key[i]) last = std::max(last, c.end[j++] - gap);
      for (size_t q = i; q < j; ++q) {
        int64_t* r = rows + q * kPromoteRow;
        r[0] = c.key[q];
        r[1] = c.start[q];
        r[2] = c.end[q];
        r[3] = c.acc[q];
        r[4] = (int64_t)(((uint64_t)c.cnt[q] & 0xFFFFFFFFull) | ((uint64_t)c.flags[q] << 32));
        r[5] = last;
        r[6] = (int64_t)(q - i);
        r[7] = (int64_t)(j - i);
      }
      i = j;
    }
    if (!moved.empty()) std::memcpy(moved_out, moved.data(), moved.size() * sizeof(int64_t));
    return {(int64_t)m, (int64_t)moved.size()};
  }

  // Fire / clean up everything the watermark allows. Returns columns of emitted rows plus the
  // keys that left the store ("released").
  struct FireOut {
    std::vector<int64_t> okey, ostart, oend, oraw, ocnt, oref, released;
    std::vector<double> oval;
  };
  void fire(int64_t wm, const ExprProg& mp, const ExprProg& fp, FireOut& o,
            bool expire_cold = true) {
    auto& okey = o.okey;
    auto& ostart = o.ostart;
    auto& oend = o.oend;
    auto& oraw = o.oraw;
    auto& ocnt = o.ocnt;
    auto& oref = o.oref;
    auto& released = o.released;
    auto& oval = o.oval;
    while (!heap_.empty() && heap_.top().first <= wm) {
      const int64_t due = heap_.top().first;
      const uint64_t key = heap_.top().second;
      heap_.pop();
      auto it = m_.find(key);
      if (it == m_.end() || it->second.due != due) continue;  // stale entry
      it->second.due = INT64_MAX;  // this entry is consumed
      auto& vec = it->second;
      size_t w = 0;  // sessions kept (not cleaned yet), compacted in place: no allocation per key
      for (size_t r = 0; r < vec.size(); ++r) {
        Session& s = vec[r];
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
        if (cleanup_time(maxts) > wm) vec[w++] = s;  // not cleaned yet
      }
      if (w == 0) {
        m_.erase(it);
        released.push_back((int64_t)key);
      } else {
        vec.resize(w);
        schedule(key);
      }
    }
    for (uint64_t key : pending_released_)
      if (m_.find(key) == m_.end()) released.push_back((int64_t)key);
    pending_released_.clear();
    if (expire_cold) this->expire_cold(wm, released);
  }

  // Cold chunks: dropped as a whole once every row is past cleanup at `wm`; their keys without
  // hot sessions leave the store (appended to `released`). Emits no rows, so the GPU operator
  // runs it on its spill worker, off the step's critical path.
  void expire_cold(int64_t wm, std::vector<int64_t>& released) {
    std::vector<ColdChunk> gone;
    detach_expired(wm, gone);
    released_of(gone, released);
    recycle(gone);
  }  // the chunks not kept as spares are freed here
  // The three steps of expire_cold, so that the spill worker holds the store lock only for the
  // first and the last (config 5 at steady state: expiry under the lock stalled the step's host
  // fire by ~2 ms). 1. Under the lock: chunks past cleanup at `wm` leave cold_ for `gone`.
  void detach_expired(int64_t wm, std::vector<ColdChunk>& gone) {
    bool erased = false;
    for (auto it = cold_.begin(); it != cold_.end();) {
      if (it->max_due <= wm) {
        cold_rows_ -= it->live;
        gone.push_back(std::move(*it));
        it = cold_.erase(it);
        erased = true;
      } else {
        ++it;
      }
    }
    if (erased) reindex_chunks();
  }
  // 2. The keys of the detached chunks' live rows that leave the store: a key with hot sessions
  // stays (under the lock unless hot_free(), i.e. no hot state -- the common case, hot state is
  // overflow only -- which makes it a pure function of the detached chunks).
  void released_of(const std::vector<ColdChunk>& gone, std::vector<int64_t>& released) const {
    const bool no_hot = m_.empty();
    size_t rows = 0;
    for (const ColdChunk& ch : gone) rows += ch.key.size();
    if (no_hot && pool_ && rows >= 262144) {
      // Row blocks on the store's pool: count the live rows per block, then each block writes
      // its keys at its offset (the order of the serial loop).
      constexpr size_t kBlk = 65536;
      std::vector<std::pair<const ColdChunk*, size_t>> blocks;
      for (const ColdChunk& ch : gone)
        for (size_t a = 0; a < ch.key.size(); a += kBlk) blocks.push_back({&ch, a});
      std::vector<size_t> cnt(blocks.size() + 1, 0);
      pool_->run((int)blocks.size(), [&](int b) {
        const ColdChunk& ch = *blocks[(size_t)b].first;
        const size_t a = blocks[(size_t)b].second, e = std::min(ch.key.size(), a + kBlk);
        size_t c = 0;
        for (size_t r = a; r < e; ++r) c += ch.cnt[r] != 0;
        cnt[(size_t)b + 1] = c;
      });
      for (size_t b = 0; b < blocks.size(); ++b) cnt[b + 1] += cnt[b];
      const size_t base = released.size();
      released.resize(base + cnt.back());
      pool_->run((int)blocks.size(), [&](int b) {
        const ColdChunk& ch = *blocks[(size_t)b].first;
        const size_t a = blocks[(size_t)b].second, e = std::min(ch.key.size(), a + kBlk);
        int64_t* o = released.data() + base + cnt[(size_t)b];
        for (size_t r = a; r < e; ++r)
          if (ch.cnt[r]) *o++ = (int64_t)ch.key[r];
      });
      return;
    }
    for (const ColdChunk& ch : gone) {
      released.reserve(released.size() + ch.key.size());
      for (size_t r = 0; r < ch.key.size(); ++r)
        if (ch.cnt[r] && (no_hot || !is_hot(ch.key[r]))) released.push_back((int64_t)ch.key[r]);
    }
  }
  bool hot_free() const { return m_.empty(); }
  // 3. Under the lock: the detached chunks' column memory back to the spare list (at most 4
  // kept for the next evictions' chunks); the caller frees the rest (`gone`) after the lock.
  void recycle(std::vector<ColdChunk>& gone) {
    for (ColdChunk& sp : gone) {
      if (spare_.size() >= 4) break;
      if (!sp.key.capacity()) continue;
      sp.key.clear();
      sp.start.clear();
      sp.end.clear();
      sp.acc.clear();
      sp.cnt.clear();
      sp.by_key.clear();
      sp.max_due = INT64_MIN;
      sp.live = 0;
      sp.kmin = ~0ull;
      sp.kmax = 0;
      sp.seq = 0;
      spare_.push_back(std::move(sp));
    }
  }

  // Device spill set (open addressing on mix64(key) >> 32, linear probing, empty = ~0) holding
  // every key of this store: records of these keys are diverted from HBM to the host tier.
  // `d`: 2^cap_log2 entries.
  void spill_set(int cap_log2, int64_t* d) const {
    const size_t cap = (size_t)1 << cap_log2;
    if (num_keys() * 2 > cap) throw std::invalid_argument("spill set too small");
    std::fill(d, d + cap, (int64_t)kEmptyKey);
    spill_set_add(cap_log2, d);
  }
  // This store's keys added to a spill set `d` that may already hold other keys (shards).
  void spill_set_add(int cap_log2, int64_t* d) const {
    const size_t cap = (size_t)1 << cap_log2;
    const uint32_t mask = (uint32_t)(cap - 1);
    auto put = [&](uint64_t key) {
      uint32_t s = (uint32_t)(mix64(key) >> 32) & mask;
      while ((uint64_t)d[s] != kEmptyKey) {
        if ((uint64_t)d[s] == key) return;
        s = (s + 1) & mask;
      }
      d[s] = (int64_t)key;
    };
    for (auto& kv : m_) put(kv.first);
    for (auto& ch : cold_)
      for (size_t r = 0; r < ch.key.size(); ++r)
        if (ch.cnt[r]) put(ch.key[r]);
  }

  bool contains(uint64_t key) const {
    if (m_.count(key)) return true;
    for (auto& ch : cold_)
      for (size_t r = 0; r < ch.key.size(); ++r)
        if (ch.cnt[r] && ch.key[r] == key) return true;
    return false;
  }
  // The key has sessions in the hot map.
  bool hot(uint64_t key) const { return is_hot(key); }
  // Keys (cold rows are one session per key in practice: an upper bound otherwise).
  size_t num_keys() const { return m_.size() + cold_rows_; }
  size_t num_sessions() const {
    size_t s = cold_rows_;
    for (auto& kv : m_) s += kv.second.size();
    return s;
  }
  size_t num_cold_rows() const { return cold_rows_; }
  size_t bytes() const {
    size_t hot = 0;
    for (auto& kv : m_) hot += kv.second.capacity() * sizeof(Session) + 48;
    size_t cold = 0;
    for (auto& ch : cold_) cold += ch.key.size() * (8 + 8 + 8 + 8 + 4);
    return hot + cold;
  }

  std::vector<int64_t> key_list() const {
    std::unordered_set<uint64_t> ks;
    for (auto& kv : m_) ks.insert(kv.first);
    for (auto& ch : cold_)
      for (size_t r = 0; r < ch.key.size(); ++r)
        if (ch.cnt[r]) ks.insert(ch.key[r]);
    std::vector<int64_t> k(ks.begin(), ks.end());
    std::sort(k.begin(), k.end());
    return k;
  }

  // Snapshot: flat columns (key, start, end, acc, cnt, flags) of both tiers.
  Columns snapshot() const {
    Columns out;
    for (auto& kv : m_)
      for (auto& x : kv.second) out.add(kv.first, x.start, x.end, x.acc, x.cnt, x.flags);
    for (auto& ch : cold_)
      for (size_t r = 0; r < ch.key.size(); ++r)
        if (ch.cnt[r]) out.add(ch.key[r], ch.start[r], ch.end[r], ch.acc[r], ch.cnt[r], 1u);
    return out;
  }

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

 private:
  int64_t cleanup_time(int64_t maxts) const {
    const int64_t c = maxts + late_;
    return c < maxts ? INT64_MAX : c;  // overflow: never cleaned before end of input
  }

  // ---- dense cold-row index (index_cold) ----------------------------------------------------
  // (seq >= 1: a real entry is never 0, so fresh zero pages read as kNoLoc)
  static constexpr uint64_t kNoLoc = 0, kMultiLoc = ~0ull;
  static constexpr uint64_t kNoHit = ~0ull;  // take_indexed: (chunk position << 32 | row) or this
  static constexpr uint64_t kMaxLocSpan = (uint64_t)1 << 28;  // 2 GB of virtual index
  int32_t seq_pos(uint32_t seq) const {
    const uint64_t i = (uint64_t)seq - seq_lo_;
    return seq >= seq_lo_ && i < seq_pos_.size() ? seq_pos_[(size_t)i] : -1;
  }
  void set_seq_pos(uint32_t seq, int32_t pos) {
    if (seq_pos_.empty()) seq_lo_ = seq;
    const size_t i = (size_t)(seq - seq_lo_);
    if (i >= seq_pos_.size()) seq_pos_.resize(i + 1, -1);
    seq_pos_[i] = pos;
  }
  // Chunk positions after an erase from cold_ (tens of chunks).
  void reindex_chunks() {
    uint32_t lo = next_seq_;
    for (auto& ch : cold_)
      if (ch.seq) lo = std::min(lo, ch.seq);
    seq_pos_.assign(next_seq_ > lo ? (size_t)(next_seq_ - lo) : 0, -1);
    seq_lo_ = lo;
    for (size_t i = 0; i < cold_.size(); ++i)
      if (cold_[i].seq) seq_pos_[(size_t)(cold_[i].seq - lo)] = (int32_t)i;
  }
  // The entry still names a live cold row of `key`.
  bool live_loc(uint64_t e, uint64_t key) const {
    const int32_t pos = seq_pos((uint32_t)(e >> 32));
    if (pos < 0) return false;
    const ColdChunk& ch = cold_[(size_t)pos];
    const uint32_t r = (uint32_t)e;
    return r < ch.key.size() && ch.key[r] == key && ch.cnt[r];
  }
  bool index_usable() const { return !loc_off_ && loc_ != nullptr; }
  // Map the index pages of entries [a, b) (whole pages).
  void populate(size_t a, size_t b) const {
    if (b <= a) return;
    const uintptr_t x = reinterpret_cast<uintptr_t>(loc_ + a) & ~(uintptr_t)4095;
    const uintptr_t y = reinterpret_cast<uintptr_t>(loc_ + b);
    (void)::madvise(reinterpret_cast<void*>(x), y - x, 23 /* MADV_POPULATE_WRITE */);
  }
  // Entries up to `need`: when the mapped range ends less than pop_ahead_ / 2 above it, one
  // background thread maps the next pop_ahead_ entries (one at a time; joined before the next).
  // (MXS_INDEX_AHEAD_MB: the read-ahead in MB of entries, default 32)
  const size_t pop_ahead_ = (size_t)std::max(1, env_int_("MXS_INDEX_AHEAD_MB", 32)) << 17;
  static int env_int_(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::atoi(e) : dflt;
  }
  void populate_ahead(size_t need) {
    const size_t ph = pop_hi_.load();
    if (need + pop_ahead_ / 2 <= ph || ph >= kMaxLocSpan || pop_busy_.load()) return;
    if (pop_thread_.joinable()) pop_thread_.join();
    const size_t end = std::min(kMaxLocSpan, ph + pop_ahead_);
    pop_busy_.store(true);
    pop_thread_ = std::thread([this, ph, end] {
      populate(ph, end);
      size_t cur = pop_hi_.load();
      while (cur < end && !pop_hi_.compare_exchange_weak(cur, end)) {
      }
      pop_busy_.store(false);
    });
  }
  void drop_index() {
    if (pop_thread_.joinable()) pop_thread_.join();
    if (loc_) ::munmap(loc_, kMaxLocSpan * sizeof(uint64_t));
    loc_ = nullptr;
    loc_off_ = true;
  }
  // The wanted keys (ascending, unique) lost every cold row: their entries are cleared (a
  // multi-row key goes back to the indexed path).
  void forget_keys(const std::vector<uint64_t>& want) {
    if (!index_usable()) return;
    for (uint64_t k : want) {
      const uint64_t o = k - loc_base_;
      if (k >= loc_base_ && o < kMaxLocSpan) loc_[o] = kNoLoc;
    }
  }
  // Cold rows of the wanted keys (ascending, unique) through the index, in key order: `cold`
  // gets the kept ones (rows past cleanup at wm are dropped), every found row leaves its chunk.
  // False (nothing changed) when the index is off or a wanted key has rows in two places (the
  // scan path takes over).
  bool take_indexed(const std::vector<uint64_t>& want, int64_t wm,
                    std::vector<std::pair<uint64_t, Session>>& cold) {
    return take_indexed_with(
        want, wm, false, SIZE_MAX, [&](size_t total) { cold.resize(total); },
        [&](size_t o, const ColdChunk& ch, uint32_t r, uint32_t, uint32_t, int64_t) {
          cold[o] = {ch.key[r], Session{ch.start[r], ch.end[r], ch.acc[r], ch.cnt[r], 1u}};
        });
  }
  // Two passes over blocks of wanted keys on the pool: resolve every key to its live run of
  // cold rows and count the kept rows (nothing changes; a multi-place key, a key with more
  // than max_kept kept rows, or -- with no_hot -- a key with hot sessions aborts), then
  // size(total kept) and emit(offset, chunk, row, position in the key, kept rows of the key,
  // max end of the key's kept rows) each kept row in key order while the found rows leave their
  // chunks.
  template <class Size, class Emit>
  bool take_indexed_with(const std::vector<uint64_t>& want, int64_t wm, bool no_hot,
                         size_t max_kept, Size&& size, Emit&& emit) {
    if (!index_usable()) return false;
    const size_t nw = want.size();
    constexpr size_t kBlk = 8192;
    const size_t nb = (nw + kBlk - 1) / kBlk;
    ix_hit_.resize(nw);
    ix_run_.resize(nw);
    ix_kept_.assign(nb + 1, 0);
    std::atomic<int> abort{0};  // 1 multi, 2 hot, 3 too many sessions
    if (!pool_) {
      unsigned hw = std::thread::hardware_concurrency();
      pool_.reset(new WorkerPool(std::max(0, std::min<int>(hw ? (int)hw : 1, max_threads_) - 1)));
    }
    const uint64_t base = loc_base_;
    const bool check_hot = no_hot && !m_.empty();
    auto blocks = [&](auto&& body) {
      if (nb <= 1) {
        for (size_t b = 0; b < nb; ++b) body(b);
      } else {
        pool_->run((int)nb, [&](int b) { body((size_t)b); });
      }
    };
    blocks([&](size_t b) {
      size_t kept = 0;
      for (size_t i = b * kBlk, e = std::min(nw, i + kBlk); i < e; ++i) {
        const uint64_t k = want[i];
        uint64_t hit = kNoHit;
        uint32_t run = 0;
        const uint64_t o = k - base;
        if (check_hot && is_hot(k)) {
          abort.store(2, std::memory_order_relaxed);
          return;
        }
        if (k >= base && o < kMaxLocSpan) {
          const uint64_t en = loc_[o];
          if (en == kMultiLoc) {
            abort.store(1, std::memory_order_relaxed);
            return;
          }
          if (en != kNoLoc) {
            const int32_t pos = seq_pos((uint32_t)(en >> 32));
            const uint32_t r = (uint32_t)en;
            if (pos >= 0) {
              const ColdChunk& ch = cold_[(size_t)pos];
              if (r < ch.key.size() && ch.key[r] == k && ch.cnt[r]) {
                hit = ((uint64_t)(uint32_t)pos << 32) | r;
                size_t kk = 0;
                for (uint32_t q = r; q < ch.key.size() && ch.key[q] == k; ++q, ++run)
                  kk += ch.cnt[q] && cleanup_time(ch.end[q] - 1) > wm;
                if (kk > max_kept) {
                  abort.store(3, std::memory_order_relaxed);
                  return;
                }
                kept += kk;
              }
            }
          }
        }
        ix_hit_[i] = hit;
        ix_run_[i] = run;
      }
      ix_kept_[b + 1] = kept;
    });
    if (const int a = abort.load()) {
      ++(a == 2 ? ixs_.hot : ixs_.multi);
      return false;
    }
    ++ixs_.indexed;
    for (size_t b = 0; b < nb; ++b) ix_kept_[b + 1] += ix_kept_[b];
    size(ix_kept_[nb]);
    // per block and chunk: rows taken (a shared atomic per chunk ping-pongs between cores)
    const size_t nch = cold_.size();
    ix_gone_.assign(nb * nch, 0);
    blocks([&](size_t b) {
      size_t o = ix_kept_[b];
      uint32_t* gb = ix_gone_.data() + b * nch;
      for (size_t i = b * kBlk, e = std::min(nw, i + kBlk); i < e; ++i) {
        const uint64_t h = ix_hit_[i];
        if (h == kNoHit) continue;
        const size_t pos = (size_t)(h >> 32);
        ColdChunk& ch = cold_[pos];
        const uint32_t r0 = (uint32_t)h, r1 = r0 + ix_run_[i];
        uint32_t nk = 0;
        int64_t last = INT64_MIN;
        for (uint32_t r = r0; r < r1; ++r)
          if (ch.cnt[r] && cleanup_time(ch.end[r] - 1) > wm) {
            ++nk;
            last = std::max(last, ch.end[r]);
          }
        uint32_t j = 0;
        size_t taken = 0;
        for (uint32_t r = r0; r < r1; ++r) {
          if (!ch.cnt[r]) continue;
          if (cleanup_time(ch.end[r] - 1) > wm) emit(o++, ch, r, j++, nk, last);
          ch.cnt[r] = 0;
          ++taken;
        }
        gb[pos] += (uint32_t)taken;
        loc_[want[i] - base] = kNoLoc;
      }
    });
    for (size_t b = 0; b < nb; ++b)
      for (size_t c = 0; c < nch; ++c) {
        const uint32_t g = ix_gone_[b * nch + c];
        cold_[c].live -= g;
        cold_rows_ -= g;
      }
    return true;
  }

  // Move cold rows of `keys` into the hot map (rows past cleanup at `wm` are discarded).
  void promote(const int64_t* keys, int64_t n, int64_t wm) {
    if (cold_rows_ == 0 || n == 0) return;
    std::vector<uint64_t> want((const uint64_t*)keys, (const uint64_t*)keys + n);
    std::sort(want.begin(), want.end());
    want.erase(std::unique(want.begin(), want.end()), want.end());
    forget_keys(want);  // every cold row of these keys leaves below
    auto take = [&](ColdChunk& ch, uint32_t r) {
      if (!ch.cnt[r]) return;
      if (cleanup_time(ch.end[r] - 1) > wm) {
        m_[ch.key[r]].push_back(Session{ch.start[r], ch.end[r], ch.acc[r], ch.cnt[r], 1u});
        mark_hot(ch.key[r]);
        schedule(ch.key[r]);
      } else {
        pending_released_.push_back(ch.key[r]);  // reported by fire() unless it turns hot
      }
      ch.cnt[r] = 0;
      ch.live -= 1;
      cold_rows_ -= 1;
    };
    for (auto& ch : cold_) {
      if (!ch.live || want.back() < ch.kmin || want.front() > ch.kmax) continue;
      auto lo = std::lower_bound(want.begin(), want.end(), ch.kmin);
      auto hi = std::upper_bound(lo, want.end(), ch.kmax);
      if (lo == hi) continue;
      ch.ensure_index();
      const size_t nw = (size_t)(hi - lo), nc = ch.by_key.size();
      auto ckey = [&](uint32_t r) { return ch.key[r]; };
      if (nw * 20 < nc) {  // few wanted keys: binary search each in the chunk's key order
        for (auto it = lo; it != hi; ++it) {
          auto p = std::lower_bound(ch.by_key.begin(), ch.by_key.end(), *it,
                                    [&](uint32_t r, uint64_t k) { return ckey(r) < k; });
          for (; p != ch.by_key.end() && ckey(*p) == *it; ++p) take(ch, *p);
        }
      } else {  // merge join of two sorted sequences
        size_t i = 0;
        for (auto it = lo; it != hi && i < nc; ++it) {
          while (i < nc && ckey(ch.by_key[i]) < *it) ++i;
          for (; i < nc && ckey(ch.by_key[i]) == *it; ++i) take(ch, ch.by_key[i]);
        }
      }
    }
  }

  // Merge candidate c into key's sessions; returns the number of late-dropped elements.
  int64_t merge_candidate(uint64_t key, Session c, int64_t wm) {
    auto found = m_.find(key);
    Session merged = c;
    bool touched_existing = false;
    if (found != m_.end()) {
      // In-place compaction: sessions intersecting the candidate fold into it, the rest stay.
      auto& vec = found->second;
      size_t w = 0;
      for (size_t r = 0; r < vec.size(); ++r) {
        const Session& s = vec[r];
        if (merged.start <= s.end && merged.end >= s.start) {
          merged.start = std::min(merged.start, s.start);
          merged.end = std::max(merged.end, s.end);
          merged.acc = agg_combine(agg_, s.acc, merged.acc);
          merged.cnt += s.cnt;
          merged.flags |= s.flags;
          touched_existing = true;
        } else {
          vec[w++] = s;
        }
      }
      vec.resize(w);
    }
    if (!touched_existing && cleanup_time(merged.end - 1) <= wm) {
      if (found != m_.end() && found->second.empty()) m_.erase(found);
      return c.cnt;  // late: every window of these elements is already cleaned
    }
    // A fired session that grows (or a new session already past its end within lateness)
    // fires again at the next fire() with the watermark (EventTimeTrigger.onElement).
    if (merged.flags & 1u) merged.flags |= 2u;
    if (found == m_.end()) {
      found = m_.emplace(key, Hot()).first;
      mark_hot(key);
    }
    found->second.push_back(merged);
    schedule(key);
    return 0;
  }

  void schedule(uint64_t key) {
    auto it = m_.find(key);
    if (it == m_.end()) return;
    int64_t t = INT64_MAX;
    for (auto& s : it->second) {
      const int64_t maxts = s.end - 1;
      const int64_t due = ((s.flags & 1u) && !(s.flags & 2u)) ? cleanup_time(maxts) : maxts;
      t = std::min(t, due);
    }
    if (t == it->second.due) return;  // the key's heap entry already says t
    it->second.due = t;
    heap_.push({t, key});
  }

  int64_t gap_, late_;
 public:
  // extract's chunk-scan / worker-phase threads (1 inside a sharded store); MXS_STORE_THREADS
  // caps it (the pool shares the process's CPU quota with the stepping thread)
  int max_threads_ = default_threads();
  static bool env_flag(const char* name, bool dflt) {
    const char* e = std::getenv(name);
    return e ? e[0] != '0' : dflt;
  }
  static int default_threads() {
    const char* e = std::getenv("MXS_STORE_THREADS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? std::min(v, 64) : 16;
  }
  std::unique_ptr<WorkerPool> pool_;  // indexed extract's key blocks (created on first use)
 private:
  int agg_;
  // A key's live sessions plus the due time of its one valid heap entry (schedule() pushes only
  // when the due time changes; fire() skips popped entries whose time is not the key's due).
  // A hot key's sessions: up to two inline (nearly every key holds one or two), more on the
  // heap -- an eviction that sends 10^5 keys to the hot map no longer allocates a session
  // buffer per key on top of the map node.
  struct Hot {
    int64_t due = INT64_MAX;
    uint32_t n = 0, cap = 2;
    Session inl[2];
    Session* ext = nullptr;

    Hot() = default;
    Hot(const Hot& o) : due(o.due) { for (const Session& x : o) push_back(x); }
    Hot& operator=(const Hot& o) {
      if (this != &o) {
        n = 0;
        due = o.due;
        for (const Session& x : o) push_back(x);
      }
      return *this;
    }
    Hot(Hot&& o) noexcept : due(o.due), n(o.n), cap(o.cap), ext(o.ext) {
      if (!ext) for (uint32_t i = 0; i < n; ++i) inl[i] = o.inl[i];
      o.ext = nullptr;
      o.n = 0;
      o.cap = 2;
    }
    ~Hot() { delete[] ext; }
    Session* data() { return ext ? ext : inl; }
    const Session* data() const { return ext ? ext : inl; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    size_t capacity() const { return cap; }
    Session& operator[](size_t i) { return data()[i]; }
    Session* begin() { return data(); }
    Session* end() { return data() + n; }
    const Session* begin() const { return data(); }
    const Session* end() const { return data() + n; }
    void resize(size_t w) { n = (uint32_t)(w < n ? w : n); }  // shrink only
    void push_back(const Session& x) {
      if (n == cap) {
        Session* nb = new Session[(size_t)cap * 2];
        for (uint32_t i = 0; i < n; ++i) nb[i] = data()[i];
        delete[] ext;
        ext = nb;
        cap *= 2;
      }
      data()[n++] = x;
    }
  };
  std::unordered_map<uint64_t, Hot> m_;
  // "May be hot" filter over the hot map's keys (one bit per mix64 bucket, set on every hot
  // insert, never cleared; rebuilt when mostly stale): eviction inserts and cold-chunk expiry
  // ask it before probing m_, so the common cold key costs one bit test instead of a hash-map
  // miss.
  static constexpr int kHotBits = 24;
  std::vector<uint64_t> hot_filter_ = std::vector<uint64_t>((size_t)1 << (kHotBits - 6), 0);
  size_t hot_marks_ = 0;
  void mark_hot(uint64_t key) {
    const uint64_t b = mix64(key) >> (64 - kHotBits);
    hot_filter_[b >> 6] |= 1ull << (b & 63);
    ++hot_marks_;
  }
  bool is_hot(uint64_t key) const {
    if (m_.empty()) return false;
    const uint64_t b = mix64(key) >> (64 - kHotBits);
    if (!((hot_filter_[b >> 6] >> (b & 63)) & 1ull)) return false;
    return m_.find(key) != m_.end();
  }
  void refresh_hot_filter() {
    if (hot_marks_ < ((size_t)1 << 20) || hot_marks_ < 4 * m_.size()) return;
    std::fill(hot_filter_.begin(), hot_filter_.end(), 0ull);
    hot_marks_ = 0;
    for (const auto& kv : m_) mark_hot(kv.first);
  }
  std::priority_queue<std::pair<int64_t, uint64_t>, std::vector<std::pair<int64_t, uint64_t>>,
                      std::greater<>>
      heap_;
  std::deque<ColdChunk> cold_;
  std::vector<ColdChunk> spare_;  // emptied chunks whose column capacity is reused
  size_t cold_rows_ = 0;
  uint64_t* loc_ = nullptr;  // dense cold-row index (index_cold): kMaxLocSpan reserved entries
  size_t pop_lo_ = 0;                 // entries [pop_lo_, pop_hi_) have their pages mapped
  std::atomic<size_t> pop_hi_{0};
  std::atomic<bool> pop_busy_{false};
  std::thread pop_thread_;            // the read-ahead mapping (populate_ahead)
  uint64_t loc_base_ = 0;
  bool loc_off_ = false;
  uint32_t next_seq_ = 1, seq_lo_ = 1;
  std::vector<int32_t> seq_pos_;  // chunk seq - seq_lo_ -> position in cold_ (-1: gone)
  std::vector<uint64_t> ix_hit_, ix_want_, ix_bits_;  // take_indexed scratch (kept between calls)
  std::vector<uint32_t> ix_run_, ix_gone_;
  IndexStats ixs_;
  std::vector<size_t> ix_kept_;
  std::vector<uint64_t> pending_released_;
};

}  // namespace sess
}  // namespace mxs

#endif  // MXS_SESSION_STORE_H_
