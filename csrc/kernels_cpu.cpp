// mxstream — host C++ twins of the gfx950 kernels (kernels_hip.hip).
//
// Same arguments, same state layout, same hashing: the CPU engine is the no-GPU execution path
// (BASELINE config 1 runs here) and the reference the GPU kernels are tested against. Events are
// processed in arrival order, so float accumulations match Flink's per-record order exactly.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

#include "mxs_kernels.h"

namespace mxs {
namespace cpu {

// Record at index `idx` of a bucket buffer in either layout (24-byte Rec / 16-byte RecC).
static Rec load_any(const Rec* base, size_t idx, int rec_words) {
  if (rec_words == 3) return base[idx];
  if (rec_words == 1) {
    const RecN& c = reinterpret_cast<const RecN*>(base)[idx];
    Rec r;
    r.key = c.key;
    r.val = (uint64_t)(int64_t)((int32_t)c.vt >> 4);
    r.t = (c.vt & 15u) == kNarrowHoleT ? 0xFFFFFFFFu : (c.vt & 15u);
    r.aux = 0;
    return r;
  }
  const RecC& c = reinterpret_cast<const RecC*>(base)[idx];
  Rec r;
  r.key = c.key;
  r.val = (uint64_t)(int64_t)(int32_t)c.val;
  r.t = c.t;
  r.aux = 0;
  return r;
}

void gen_events(uint64_t* keys, int64_t* ts, uint64_t* vals, int64_t n, uint64_t seed,
                uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
                int64_t ts_span, int64_t disorder, int64_t val_lo, int64_t val_span,
                int32_t val_f64, double zipf_s, uint64_t key_base) {
  const double span_per_event = (double)ts_span / (double)n;
  const uint64_t disorder_p1 = (uint64_t)(disorder + 1);
  const uint64_t base = mix64(seed ^ (stream_id * 0xd1b54a32d192ed03ull));
  for (int64_t i = 0; i < n; ++i) {
    uint64_t key;
    int64_t t, v;
    gen_event(base, idx0 + (uint64_t)i, i, nkeys, ts_base, span_per_event, disorder_p1, val_lo,
              val_span > 0 ? (uint64_t)val_span : 0, zipf_s, key, t, v);
    key += key_base;
    if (val_f64 & 2) reinterpret_cast<int32_t*>(keys)[i] = (int32_t)key;
    else keys[i] = key;
    ts[i] = t;
    vals[i] = (val_f64 & 1) ? f64_bits((double)v) : (uint64_t)v;
  }
}

void partition(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
               const int32_t* jhash_tab, int64_t n, const PartPlan& p, const int32_t* kg_dest,
               uint32_t* cursor, Rec* out, int64_t* stats, uint32_t* late_idx, uint32_t late_cap) {
  int64_t tmax = stats[kStatMaxTs], qmin = stats[kStatMinPane], qmax = stats[kStatMaxPane];
  int64_t nlate = 0, nacc = 0;
  int64_t ovf = 0;
  uint32_t pmask = 0;  // kStatPaneMask, as the GPU partitions report it
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t key = keys[i];
    const int64_t t = ts[i];
    tmax = std::max(tmax, t);
    uint32_t rt = 0;
    if (key >= kTombKey) {  // reserved ids (tombstone / empty-slot / hole markers): reported
      ovf |= 8;
      continue;
    }
    if (p.window_mode) {
      if (p.drop_late && t < p.late_ts) {
        if (late_idx) {
          const int64_t pos = stats[kStatLate] + nlate;
          if (pos < (int64_t)late_cap) late_idx[pos] = (uint32_t)i;
        }
        ++nlate;
        continue;
      }
      int64_t q;
      if (!rel_pane(t, p, &rt, &q)) {
        ovf |= 2;
        continue;
      }
      qmin = std::min(qmin, q);
      qmax = std::max(qmax, q);
      pmask |= 1u << (rt < 31u ? rt : 31u);
    }
    ++nacc;
    const int32_t jh = p.nranks == 1 ? 0 : p.hash_mode ? jhash_tab[key] : java_long_hash((int64_t)key);
    const uint32_t b = bucket_of(key, jh, p, kg_dest);
    const uint32_t pos = cursor[b]++;
    if (pos >= p.bucket_cap) {
      ovf |= 1;
    } else if (p.rec_words == 1) {  // narrow 8-byte record
      RecN& r = reinterpret_cast<RecN*>(out)[(size_t)b * p.bucket_cap + pos];
      if ((int64_t)(int32_t)vals[i] != (int64_t)vals[i]) ovf |= 4;
      if (!narrow_fits(key, (int64_t)vals[i], rt)) ovf |= 16;
      r.key = (uint32_t)key;
      r.vt = ((uint32_t)vals[i] << 4) | (rt & 15u);
    } else if (p.rec_words == 2) {  // compact 16-byte record (int32 value)
      RecC& r = reinterpret_cast<RecC*>(out)[(size_t)b * p.bucket_cap + pos];
      if ((int64_t)(int32_t)vals[i] != (int64_t)vals[i]) ovf |= 4;
      r.key = key;
      r.val = (uint32_t)vals[i];
      r.t = rt;
    } else {
      Rec& r = out[(size_t)b * p.bucket_cap + pos];
      r.key = key;
      r.val = vals[i];
      r.t = rt;
      r.aux = (uint32_t)i;
    }
  }
  stats[kStatMaxTs] = tmax;
  stats[kStatMinPane] = qmin;
  stats[kStatMaxPane] = qmax;
  stats[kStatLate] += nlate;
  stats[kStatAccepted] += nacc;
  stats[kStatOverflow] |= ovf;
  stats[kStatPaneMask] |= pmask;
}

void step_begin(uint32_t* cursor, int nb, int64_t* stats) {
  std::memset(cursor, 0, sizeof(uint32_t) * (size_t)nb);
  for (int j = 0; j < kStatCount; ++j)
    stats[j] = j == kStatMaxTs ? INT64_MIN : j == kStatMinPane ? INT64_MAX
             : j == kStatMaxPane ? INT64_MIN : 0;
}

void step_finish(const int64_t* stats, int64_t* local_maxts, int64_t bound, int32_t event_mode,
                 int64_t proc_now, int64_t* red, const uint32_t* flags, int32_t idle,
                 int32_t fill_word, const uint32_t* cursor, int nb) {
  int64_t lm = std::max(local_maxts[0], stats[kStatMaxTs]);
  local_maxts[0] = lm;
  const int64_t wm = event_mode ? (lm == INT64_MIN ? INT64_MIN : lm - bound) : proc_now;
  const int64_t qmax = stats[kStatMaxPane];
  red[0] = qmax == INT64_MIN ? INT64_MAX : -qmax;
  red[1] = stats[kStatMinPane];
  red[2] = idle ? INT64_MAX : wm;
  red[3] = -(stats[kStatOverflow] & 1);
  if (fill_word && cursor) {
    uint32_t m = 0;
    for (int i = 0; i < nb; ++i) m = std::max(m, cursor[i]);
    red[3] = (stats[kStatOverflow] & 1) ? -((int64_t)1 << 40) : -(int64_t)m;
  }
  red[4] = -((stats[kStatOverflow] >> 1) & 1);
  // Record width a value needs: -2 = 24-byte records, -1 = 16-byte records, 0 = as planned.
  red[5] = (stats[kStatOverflow] & 4) ? -2 : (stats[kStatOverflow] & 16) ? -1 : 0;
  red[6] = flags ? -(int64_t)(flags[0] & 1u) : 0;  // a key found no slot (table full), sticky
  red[7] = -((stats[kStatOverflow] >> 3) & 1);  // the reserved key id ~0 occurred
  for (int j = 0; j < kStatCount; ++j) red[8 + j] = stats[j];
}

static inline uint32_t probe_insert(uint64_t* keys, uint64_t key, uint32_t mask, bool* inserted) {
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    const uint64_t k = keys[s];
    if (k == key) return s;
    if (k == kEmptyKey) {
      keys[s] = key;
      *inserted = true;
      return s;
    }
    s = (s + 1) & mask;
  }
  return kNoSlot;
}

void window_agg(const Rec* recs, const uint32_t* counts, const AggPlan& p, uint64_t* keys_g,
                uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g, uint32_t* occupancy,
                uint32_t* flags) {
  if (p.skip && *p.skip) return;  // incomplete exchange (AggPlan.skip)
  const uint32_t cap = 1u << p.cap_log2, mask = cap - 1;
  const size_t nslots = (size_t)p.nsub << p.cap_log2;
  // Deterministic f64 sums: per-step slot sums in 128-bit fixed point, folded once per slot
  // (the GPU kernel's LDS accumulation + write-back, bit for bit).
  const bool det = p.det && (p.agg == AGG_SUM_F64 || p.agg == AGG_AVG_F64);
  std::vector<unsigned __int128> dsum;
  std::vector<uint32_t> dcnt;
  if (det) {
    dsum.assign((size_t)p.np_step * cap, 0);
    dcnt.assign((size_t)p.np_step * cap, 0);
  }
  for (int sub = 0; sub < p.nsub; ++sub) {
    uint64_t* keys = keys_g + ((size_t)sub << p.cap_log2);
    bool inserted = false;
    for (int src = 0; src < p.nsrc; ++src) {
      uint32_t c = counts[(size_t)src * p.nsub + sub];
      c = std::min(c, p.bucket_cap);
      const size_t seg0 = ((size_t)src * p.nsub + sub) * p.bucket_cap;
      for (uint32_t e = 0; e < c; ++e) {
        const Rec r = load_any(recs, seg0 + e, p.rec_words);
        const int64_t q = (int64_t)r.t - p.p_lo;
        if (q < 0 || q >= p.np_step) continue;
        uint32_t s;
        if (p.dense_bits) {
          if (p.dense_bits < 64 && (r.key >> p.dense_bits)) {  // id outside the dense space
            flags[0] |= 1u;
            continue;
          }
          s = dense_slot(r.key, p.dense_mul, p.dense_bits) & mask;
        } else {
          s = probe_insert(keys, r.key, mask, &inserted);
        }
        if (s == kNoSlot) {
          flags[0] |= 1u;
          continue;
        }
        const int64_t pane = p.pane_base + (int64_t)r.t;
        const size_t gi = (size_t)(pane & (p.ring - 1)) * nslots + ((size_t)sub << p.cap_log2) + s;
        if (det) {
          uint64_t lo, hi;
          if (!f64_to_fx(as_f64(r.val), &lo, &hi)) {
            flags[0] |= 8u;
            continue;
          }
          const size_t li = (size_t)q * cap + s;
          dsum[li] += ((unsigned __int128)hi << 64) | lo;
          dcnt[li] += p.combined ? r.aux : 1u;
        } else {
          const uint64_t v = agg_lift(p.agg, r.val);
          if (p.agg != AGG_COUNT) acc_g[gi] = cnt_g[gi] ? agg_combine(p.agg, acc_g[gi], v) : v;
          cnt_g[gi] += p.combined ? r.aux : 1u;
        }
        if (pane <= p.fired_hi) {
          dirty_g[gi] = 1;
          if (p.dacc && !det) {  // local-global delta ring of late-but-allowed data
            const uint64_t v = agg_lift(p.agg, r.val);
            if (p.agg != AGG_COUNT) p.dacc[gi] = p.dcnt[gi] ? agg_combine(p.agg, p.dacc[gi], v) : v;
            p.dcnt[gi] += p.combined ? r.aux : 1u;
          }
          const size_t slot = ((size_t)sub << p.cap_log2) + s;
          if (p.dlist && !p.slot_mark[slot]) {
            p.slot_mark[slot] = 1;
            p.dlist[(*p.dlist_n)++] = (uint32_t)slot;
          }
        }
      }
    }
    if (det) {
      for (int q = 0; q < p.np_step; ++q)
        for (uint32_t s = 0; s < cap; ++s) {
          const size_t li = (size_t)q * cap + s;
          if (!dcnt[li]) continue;
          const int64_t pane = p.pane_base + p.p_lo + q;
          const size_t gi = (size_t)(pane & (p.ring - 1)) * nslots + ((size_t)sub << p.cap_log2) + s;
          const double d = fx_to_f64((uint64_t)dsum[li], (uint64_t)(dsum[li] >> 64));
          acc_g[gi] = cnt_g[gi] ? f64_bits(as_f64(acc_g[gi]) + d) : f64_bits(d);
          cnt_g[gi] += dcnt[li];
          dsum[li] = 0;
          dcnt[li] = 0;
        }
    }
    if (inserted) {
      uint32_t occ = 0;
      for (uint32_t i = 0; i < cap; ++i) occ += keys[i] != kEmptyKey;
      occupancy[sub] = occ;
    }
  }
}

void window_fire(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                 const uint8_t* dirty_g, const FirePlan& p, uint64_t* out_keys,
                 double* out_vals, uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n) {
  const int64_t nslots = p.nslots;
  uint32_t n = *out_n;
  const int64_t nvisit = p.list ? (int64_t)*p.list_n : nslots;
  for (int64_t v = 0; v < nvisit; ++v) {
    const int64_t s = p.list ? (int64_t)p.list[v] : v;
    bool dirty = !p.only_dirty, have = false;
    uint64_t acc = 0;
    uint32_t cnt = 0;
    for (int j = 0; j < p.npanes; ++j) {
      const size_t gi = (size_t)((p.p0 + j) & (p.ring - 1)) * nslots + s;
      const uint32_t c = cnt_g[gi];
      if (c) {
        acc = have ? agg_combine(p.agg, acc, acc_g[gi]) : acc_g[gi];
        have = true;
        cnt += c;
        if (p.only_dirty && dirty_g[gi]) dirty = true;
      }
    }
    if (!cnt || !dirty) continue;
    const uint64_t key = keys_g[s];
    double vars[kExprVars];
    vars[0] = agg_result_f64(p.agg, acc, cnt);
    vars[1] = (double)cnt;
    vars[2] = p.wstart;
    vars[3] = p.wend;
    vars[4] = (double)key;
    vars[5] = (double)(int64_t)acc;
    vars[6] = p.map.ncode ? expr_eval(p.map, vars) : vars[0];
    vars[7] = 0.0;
    const bool emit = p.filt.ncode ? (expr_eval(p.filt, vars) != 0.0) : true;
    if (!emit) continue;
    if (n < p.out_cap) {
      if (p.key32)
        reinterpret_cast<uint32_t*>(out_keys)[n] = (uint32_t)key;
      else
        out_keys[n] = key;
      out_vals[n] = vars[6];
      if (out_raw) out_raw[n] = acc;
      if (out_cnt) out_cnt[n] = cnt;
    }
    ++n;
  }
  *out_n = n;
}

void rolling(const Rec* recs, const uint32_t* counts, const RollPlan& p, uint64_t* keys_g,
             uint64_t* acc_g, uint32_t* cnt_g, uint32_t* occupancy, uint32_t* flags,
             uint64_t* out_vals) {
  // Ordered per key: records of one sub-table are visited in (src, arrival) order, which is the
  // order Flink's StreamGroupedReduce sees them on one channel.
  const uint32_t cap = 1u << p.cap_log2, mask = cap - 1;
  for (int sub = 0; sub < p.nsub; ++sub) {
    uint64_t* keys = keys_g + ((size_t)sub << p.cap_log2);
    bool inserted = false;
    for (int src = 0; src < p.nsrc; ++src) {
      uint32_t c = std::min(counts[(size_t)src * p.nsub + sub], p.bucket_cap);
      const Rec* seg = recs + ((size_t)src * p.nsub + sub) * p.bucket_cap;
      for (uint32_t e = 0; e < c; ++e) {
        const Rec& r = seg[e];
        const uint32_t s = probe_insert(keys, r.key, mask, &inserted);
        if (s == kNoSlot) {
          flags[0] |= 1u;
          continue;
        }
        const size_t gi = ((size_t)sub << p.cap_log2) + s;
        const uint64_t v = agg_lift(p.agg, r.val);
        acc_g[gi] = cnt_g[gi] ? agg_combine(p.agg, acc_g[gi], v) : v;
        cnt_g[gi] += 1;
        if (p.emit && out_vals) out_vals[r.aux] = p.agg == AGG_COUNT ? cnt_g[gi] : acc_g[gi];
      }
    }
    if (inserted) {
      uint32_t occ = 0;
      for (uint32_t i = 0; i < cap; ++i) occ += keys[i] != kEmptyKey;
      occupancy[sub] = occ;
    }
  }
}

// Rolling keyed state with per-record rows (key, post-update value, src<<32|arrival) in
// per-key arrival order: the twin of rolling_lookup + sort + rolling_scan on the GPU.
void rolling_rows(const Rec* recs, const uint32_t* counts, int nsrc, int nsub, uint32_t bucket_cap,
                  int cap_log2, int agg, uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g,
                  uint32_t* flags, const ExprProg& filt, uint64_t* out_key, uint64_t* out_val,
                  int64_t* out_tag, uint32_t* out_n, uint32_t out_cap, uint32_t count_n) {
  // count_n > 0: tumbling count windows -- emit when a key's open window reaches count_n
  // elements, then start a new one (the GPU rolling_scan's segmented mode).
  const uint32_t mask = (1u << cap_log2) - 1;
  uint32_t n = *out_n;
  for (int sub = 0; sub < nsub; ++sub) {
    uint64_t* keys = keys_g + ((size_t)sub << cap_log2);
    bool inserted = false;
    for (int src = 0; src < nsrc; ++src) {
      const uint32_t c = std::min(counts[(size_t)src * nsub + sub], bucket_cap);
      const Rec* seg = recs + ((size_t)src * nsub + sub) * bucket_cap;
      for (uint32_t e = 0; e < c; ++e) {
        const Rec& r = seg[e];
        if (r.t == 0xFFFFFFFFu) continue;
        const uint32_t s = probe_insert(keys, r.key, mask, &inserted);
        if (s == kNoSlot) {
          flags[0] |= 1u;
          continue;
        }
        const size_t gi = ((size_t)sub << cap_log2) + s;
        const uint64_t v = agg_lift(agg, r.val);
        acc_g[gi] = cnt_g[gi] ? agg_combine(agg, acc_g[gi], v) : v;
        cnt_g[gi] += 1;
        bool emit = !count_n || cnt_g[gi] == count_n;
        if (filt.ncode) {
          double vars[kExprVars] = {0};
          vars[0] = agg_result_f64(agg, acc_g[gi], cnt_g[gi]);
          vars[1] = (double)cnt_g[gi];
          vars[4] = (double)r.key;
          vars[5] = (double)(int64_t)acc_g[gi];
          vars[6] = vars[0];
          emit = expr_eval(filt, vars) != 0.0;
        }
        if (emit) {
          if (n < out_cap) {
            out_key[n] = r.key;
            out_val[n] = agg == AGG_COUNT ? (uint64_t)cnt_g[gi] : acc_g[gi];
            out_tag[n] = ((int64_t)src << 32) | r.aux;
          }
          ++n;
        }
        if (count_n && cnt_g[gi] == count_n) cnt_g[gi] = 0;  // window purged
      }
    }
  }
  *out_n = n;
}

// Worker threads of the CPU twins' embarrassingly parallel loops (set_threads; 1 = serial).
static std::atomic<int> g_threads{1};
void set_threads(int n) { g_threads = std::max(1, std::min(n, 256)); }
int get_threads() { return g_threads; }

template <class F>
static void parallel_for(int64_t n, int64_t min_per_thread, F&& body) {
  const int64_t t = std::min<int64_t>(g_threads, std::max<int64_t>(1, n / min_per_thread));
  if (t <= 1) {
    body(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int64_t k = 0; k < t; ++k)
    th.emplace_back([&, k] { body(n * k / t, n * (k + 1) / t); });
  for (auto& x : th) x.join();
}

void format_rows_len(const FmtArgs& a, int64_t n, int64_t* len, uint32_t* bad) {
  if (a.ncols < 1 || a.ncols > kFmtMaxCols) throw std::invalid_argument("format: column count");
  std::atomic<uint32_t> flag{0};
  parallel_for(n, 1 << 16, [&](int64_t lo, int64_t hi) {
    bool all = true;
    for (int64_t i = lo; i < hi; ++i) {
      bool ok = true;
      len[i] = fmt_row(a, i, nullptr, ok);
      all = all && ok;
    }
    if (!all) flag.fetch_or(1u);
  });
  if (flag.load()) *bad |= 1u;
}

void format_rows_write(const FmtArgs& a, int64_t n, const int64_t* end, char* out) {
  if (a.ncols < 1 || a.ncols > kFmtMaxCols) throw std::invalid_argument("format: column count");
  parallel_for(n, 1 << 16, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      bool ok = true;
      fmt_row(a, i, out + (i ? end[i - 1] : 0), ok);
    }
  });
}

void expr_filter(const double* x, int64_t n, const ExprProg& prog, uint8_t* keep) {
  parallel_for(n, 1 << 16, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      double vars[kExprVars] = {x[i], 0, 0, 0, 0, 0, 0, 0};
      keep[i] = expr_eval(prog, vars) != 0.0;
    }
  });
}

void expr_filter_compact(const double* x, int64_t n, const ExprProg& prog, int64_t* idx,
                         int64_t* total) {
  int64_t c = 0;
  for (int64_t i = 0; i < n; ++i) {
    double vars[kExprVars] = {x[i], 0, 0, 0, 0, 0, 0, 0};
    if (expr_eval(prog, vars) != 0.0) idx[c++] = i;
  }
  total[0] = c;
}

void keygroups(const uint64_t* keys, int64_t n, int hash_mode, const int32_t* jhash, int max_par,
               int32_t* kg) {
  for (int64_t i = 0; i < n; ++i) {
    const int32_t h = hash_mode ? jhash[keys[i]] : java_long_hash((int64_t)keys[i]);
    kg[i] = key_group_of_hash(h, max_par);
  }
}

void table_insert(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2, uint64_t* keys_g,
                  int64_t* slots) {
  const uint32_t mask = (1u << cap_log2) - 1;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t key = keys[i];
    const uint64_t sub = sub_table_of(key, nsub_log2);
    uint64_t* t = keys_g + (sub << cap_log2);
    uint32_t s = slot_hash(key) & mask;
    int64_t found = -1;
    for (uint32_t p = 0; p <= mask; ++p) {
      if (t[s] == key) {
        found = s;
        break;
      }
      if (t[s] == kEmptyKey) {
        t[s] = key;
        found = s;
        break;
      }
      s = (s + 1) & mask;
    }
    slots[i] = found < 0 ? -1 : (int64_t)((sub << cap_log2) | (uint64_t)found);
  }
}

void window_combine(const Rec* recs, const uint32_t* counts, int nbuckets, const AggPlan& p,
                    Rec* out, uint32_t ccap, uint32_t* out_counts, uint32_t* flags) {
  const uint32_t cap = 1u << p.cap_log2, mask = cap - 1;
  std::vector<uint64_t> keys(cap), acc((size_t)cap * p.np_step);
  std::vector<uint32_t> cnt((size_t)cap * p.np_step);
  for (int b = 0; b < nbuckets; ++b) {
    std::fill(keys.begin(), keys.end(), kEmptyKey);
    std::fill(cnt.begin(), cnt.end(), 0u);
    bool inserted = false, ovf = false;
    const uint32_t c = std::min(counts[b], p.bucket_cap);
    for (uint32_t e = 0; e < c; ++e) {
      const Rec r = load_any(recs, (size_t)b * p.bucket_cap + e, p.rec_words);
      const int64_t q = (int64_t)r.t - p.p_lo;
      if (q < 0 || q >= p.np_step) continue;
      const uint32_t s = probe_insert(keys.data(), r.key, mask, &inserted);
      if (s == kNoSlot) {
        ovf = true;
        continue;
      }
      const size_t li = (size_t)q * cap + s;
      const uint64_t v = agg_lift(p.agg, r.val);
      acc[li] = cnt[li] ? agg_combine(p.agg, acc[li], v) : v;
      cnt[li] += 1;
    }
    uint32_t n = 0;
    for (size_t li = 0; li < cnt.size(); ++li) {
      if (!cnt[li]) continue;
      if (n >= ccap) {
        ovf = true;
        break;
      }
      Rec& o = out[(size_t)b * ccap + n++];
      o.key = keys[li & mask];
      o.val = p.agg == AGG_COUNT ? 0 : acc[li];
      o.t = (uint32_t)(p.p_lo + (int64_t)(li >> p.cap_log2));
      o.aux = cnt[li];
    }
    out_counts[b] = n;
    if (ovf) flags[0] |= 2u;
  }
}

void f64_order_bits(const uint64_t* v, int64_t n, uint64_t* o) {
  for (int64_t i = 0; i < n; ++i) o[i] = mxs::f64_order_bits(v[i]);
}

void segment_median_select(const int64_t* heads, int64_t nseg, int64_t total,
                           const uint64_t* ord, double* out) {
  std::vector<uint64_t> v;
  for (int64_t sg = 0; sg < nseg; ++sg) {
    const int64_t a = heads[sg], e = sg + 1 < nseg ? heads[sg + 1] : total, n = e - a;
    if (n <= 0) {
      out[sg] = 0.0;
      continue;
    }
    v.assign(ord + a, ord + e);
    std::nth_element(v.begin(), v.begin() + n / 2, v.end());
    const double hi = as_f64(f64_from_order_bits(v[n / 2]));
    if (n & 1) {
      out[sg] = hi;
    } else {
      const uint64_t lo = *std::max_element(v.begin(), v.begin() + n / 2);
      out[sg] = (hi + as_f64(f64_from_order_bits(lo))) / 2.0;
    }
  }
}

void segment_median(const int64_t* heads, int64_t nseg, int64_t total, const uint64_t* ord,
                    double* out) {
  for (int64_t s = 0; s < nseg; ++s) {
    const int64_t a = heads[s], b = s + 1 < nseg ? heads[s + 1] : total, n = b - a;
    double m = 0.0;
    if (n > 0) {
      const double hi = as_f64(f64_from_order_bits(ord[a + n / 2]));
      m = (n & 1) ? hi : (hi + as_f64(f64_from_order_bits(ord[a + n / 2 - 1]))) / 2.0;
    }
    out[s] = m;
  }
}

void window_compact(uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                    int nsub, int cap_log2, int ring, int64_t p_lo, int np, int64_t cutoff,
                    const CompactOut& out, uint32_t* occupancy) {
  const uint32_t cap = 1u << cap_log2, mask = cap - 1;
  const size_t nslots = (size_t)nsub << cap_log2;
  std::vector<uint64_t> nk(cap), ta(cap);
  std::vector<uint32_t> from(cap), tc(cap);
  std::vector<uint8_t> td(cap);
  for (int sub = 0; sub < nsub; ++sub) {
    const size_t sbase = (size_t)sub << cap_log2;
    std::fill(nk.begin(), nk.end(), kEmptyKey);
    std::fill(from.begin(), from.end(), kNoSlot);
    uint32_t kept = 0;
    for (uint32_t s = 0; s < cap; ++s) {
      const uint64_t k = keys_g[sbase + s];
      if (k == kEmptyKey || k == kTombKey) continue;
      int64_t newest = INT64_MIN;
      for (int j = 0; j < np; ++j) {
        const int64_t p = p_lo + j;
        if (cnt_g[(size_t)(p & (ring - 1)) * nslots + sbase + s]) newest = p;
      }
      if (newest == INT64_MIN) {
        ++out.counters[0];
        continue;
      }
      if (newest <= cutoff) {
        ++out.counters[1];
        for (int j = 0; j < np; ++j) {
          const int64_t p = p_lo + j;
          const size_t gi = (size_t)(p & (ring - 1)) * nslots + sbase + s;
          if (!cnt_g[gi]) continue;
          const uint32_t q = (*out.n)++;
          if (q < out.cap) {
            out.key[q] = k;
            out.pane[q] = p;
            out.acc[q] = acc_g[gi];
            out.cnt[q] = cnt_g[gi];
            out.dirty[q] = dirty_g[gi];
          } else {
            out.counters[2] |= 1u;
          }
        }
        continue;
      }
      bool ins = false;
      const uint32_t t = probe_insert(nk.data(), k, mask, &ins);
      if (t == kNoSlot) {
        out.counters[2] |= 1u;
        continue;
      }
      from[t] = s;
      ++kept;
    }
    for (uint32_t i = 0; i < cap; ++i) keys_g[sbase + i] = nk[i];
    for (int j = 0; j < np; ++j) {
      const size_t pb = (size_t)((p_lo + j) & (ring - 1)) * nslots + sbase;
      for (uint32_t i = 0; i < cap; ++i) {
        ta[i] = acc_g[pb + i];
        tc[i] = cnt_g[pb + i];
        td[i] = dirty_g[pb + i];
      }
      for (uint32_t i = 0; i < cap; ++i) {
        const uint32_t f = from[i];
        acc_g[pb + i] = f == kNoSlot ? 0 : ta[f];
        cnt_g[pb + i] = f == kNoSlot ? 0 : tc[f];
        dirty_g[pb + i] = f == kNoSlot ? 0 : td[f];
      }
    }
    occupancy[sub] = kept;
  }
}

void dirty_clear(const uint32_t* list, const uint32_t* list_n, uint32_t list_cap, int ring,
                 int64_t nslots, uint8_t* dirty_g, uint32_t* slot_mark, int64_t p_lo, int np,
                 uint64_t* dacc, uint32_t* dcnt) {
  const uint32_t n = std::min(*list_n, list_cap);
  np = std::min(np, ring);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t s = list[i];
    slot_mark[s] = 0;
    for (int j = 0; j < np; ++j) {
      const size_t gi = (size_t)((p_lo + j) & (ring - 1)) * nslots + s;
      dirty_g[gi] = 0;
      if (dcnt) {
        dcnt[gi] = 0;
        dacc[gi] = 0;
      }
    }
  }
}

// Local-global window aggregation: rows of a locally fired window -> owner (rank, sub-table)
// buckets as combined records (val = partial accumulator, aux = element count, t = pane 0).
void scatter_partials(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt,
                      const uint32_t* n_in, const ScatPlan& p, const int32_t* jhash,
                      const int32_t* kg_dest, uint32_t* cursor, Rec* out, uint32_t* flags) {
  const uint32_t n = std::min(*n_in, p.n_cap);
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t k = keys[i];
    const int32_t jh = p.hash_mode ? jhash[k] : java_long_hash((int64_t)k);
    const uint32_t dest = (uint32_t)kg_dest[key_group_of_hash(jh, p.max_parallelism)];
    const uint32_t b = (dest << p.nsub_log2) | sub_table_of(k, p.nsub_log2);
    const uint32_t pos = cursor[b]++;
    if (pos >= p.bucket_cap) {
      flags[0] |= 1u;  // more keys than the owner's sub-table holds: table full
      continue;
    }
    Rec& r = out[(size_t)b * p.bucket_cap + pos];
    r.key = k;
    r.val = acc[i];
    r.t = 0;
    r.aux = cnt[i];
  }
}

void bucket_repack(const uint64_t* src, const uint32_t* counts, int nb, uint32_t src_cap,
                   uint32_t dst_cap, int words, uint64_t* dst, uint64_t* xstat) {
  for (int b = 0; b < nb; ++b) {
    const uint32_t c = std::min(counts[b], dst_cap);
    std::memcpy(dst + (size_t)b * dst_cap * words, src + (size_t)b * src_cap * words,
                (size_t)c * words * 8);
    if (xstat) xstat[1] += (uint64_t)c * words * 8;
  }
  if (xstat) xstat[0] += (uint64_t)nb * dst_cap * words * 8;
}

void tier_merge(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt, int64_t n,
                const uint32_t* n_dev, int mode, int agg, uint64_t* tkeys, uint64_t* tacc,
                uint32_t* tcnt, uint8_t* tdirty, uint32_t mask, uint32_t* flags) {
  if (n_dev) n = std::min<int64_t>(n, (int64_t)*n_dev);
  const bool find_only = (mode & 2) != 0, mark = (mode & 1) != 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t k = keys[i];
    if (k >= kTombKey || cnt[i] == 0) continue;
    uint32_t s = (uint32_t)(mix64(k) >> 20) & mask;
    uint32_t found = kNoSlot;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
      if (tkeys[s] == k) {
        found = s;
        break;
      }
      if (tkeys[s] == kEmptyKey) {
        if (!find_only) {
          tkeys[s] = k;
          found = s;
        }
        break;
      }
      s = (s + 1) & mask;
    }
    if (found == kNoSlot) {
      if (!find_only) flags[0] |= 1u;
      continue;
    }
    tacc[found] = agg_combine(agg, tacc[found], acc[i]);
    tcnt[found] += cnt[i];
    if (mark) tdirty[found] = 1;
  }
}

// ---- packed-row exchange (twin of csrc/exchange_hip.hip) ------------------------------------
void xrows_count(const int64_t* dest, int64_t n, int world, uint32_t* counts, uint32_t* bad) {
  for (int d = 0; d < world; ++d) counts[d] = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (dest[i] >= 0 && dest[i] < world) ++counts[dest[i]];
    else *bad |= 1u;
  }
}

void xrows_scatter(const int64_t* dest, int64_t n, int world, uint32_t cap, const XRowCols& c,
                   uint32_t* send, uint32_t* ovf) {
  std::vector<uint32_t> pos((size_t)world, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t d = dest[i];
    if (d < 0 || d >= world) continue;
    const uint32_t p = pos[d]++;
    if (p >= cap) {
      *ovf |= 1u;
      continue;
    }
    uint32_t* row = send + ((size_t)d * cap + p) * (size_t)c.rw;
    int o = 0;
    for (int k = 0; k < c.ncol; ++k) {
      std::memcpy(row + o, c.src[k] + (size_t)i * c.words[k], sizeof(uint32_t) * c.words[k]);
      o += c.words[k];
    }
  }
}

void xrows_unpack(const uint32_t* recv, const uint32_t* rc, int world, uint32_t cap,
                  const XRowCols& c) {
  size_t orow = 0;
  for (int s = 0; s < world; ++s) {
    const uint32_t m = rc[s] < cap ? rc[s] : cap;
    for (uint32_t idx = 0; idx < m; ++idx, ++orow) {
      const uint32_t* row = recv + ((size_t)s * cap + idx) * (size_t)c.rw;
      int o = 0;
      for (int k = 0; k < c.ncol; ++k) {
        std::memcpy(c.dst[k] + orow * c.words[k], row + o, sizeof(uint32_t) * c.words[k]);
        o += c.words[k];
      }
    }
  }
}

}  // namespace cpu
}  // namespace mxs
