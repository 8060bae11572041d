// mxstream — C++ twins of the list-window (process window) kernels (csrc/listwin_hip.hip):
// the same pane arena and counting-sort firing on the host, for the CPU engine and the
// differential tests.
#include <stdexcept>

#include "mxs_listwin.h"

namespace mxs {
namespace cpu {

static int lw_slot(int64_t t, int64_t offset, int64_t pane, int ring, int64_t late_ts) {
  if (t < late_ts) return ring;
  return (int)(lw_floor_div(t - offset, pane) & (int64_t)(ring - 1));
}

void lw_pane_count(const int64_t* ts, int64_t n, int64_t offset, int64_t pane, int ring,
                   int64_t late_ts, int64_t* counts) {
  for (int64_t i = 0; i < n; ++i) counts[lw_slot(ts[i], offset, pane, ring, late_ts)] += 1;
}

void lw_pane_scatter(const int64_t* keys, const int64_t* ts, const uint64_t* vals, int64_t n,
                     int64_t offset, int64_t pane, int ring, int64_t late_ts, const int64_t* tab,
                     int64_t* cursor) {
  for (int64_t i = 0; i < n; ++i) {
    const int r = lw_slot(ts[i], offset, pane, ring, late_ts);
    if (r == ring) continue;
    const int64_t pos = cursor[r]++;
    reinterpret_cast<int64_t*>(tab[r])[pos] = keys[i];
    reinterpret_cast<uint64_t*>(tab[ring + r])[pos] = vals[i];
    uint32_t* kc = reinterpret_cast<uint32_t*>(tab[3 * ring + r]);
    if (kc)
      reinterpret_cast<uint32_t*>(tab[2 * ring + r])[pos] = kc[keys[i] - tab[4 * ring + r]]++;
  }
}

void lw_key_count(const LwPanes& w, int64_t kmin, int64_t nkeys, uint32_t* counts) {
  (void)nkeys;
  for (int q = 0; q < w.n; ++q)
    for (int64_t i = 0; i < w.p[q].len; ++i) counts[w.p[q].keys[i] - kmin] += 1;
}

void lw_scan(const uint32_t* counts, int64_t nkeys, int64_t kmin, int64_t* offs, int64_t* heads,
             int64_t* head_keys, int64_t* nheads) {
  int64_t o = 0, h = 0;
  for (int64_t k = 0; k < nkeys; ++k) {
    offs[k] = o;
    if (counts[k]) {
      heads[h] = o;
      head_keys[h] = kmin + k;
      ++h;
    }
    o += counts[k];
  }
  offs[nkeys] = o;
  *nheads = h;
}

void lw_key_scatter(const LwPanes& w, int64_t kmin, int64_t* cursor, uint64_t* out_ord) {
  for (int q = 0; q < w.n; ++q)
    for (int64_t i = 0; i < w.p[q].len; ++i)
      out_ord[cursor[w.p[q].keys[i] - kmin]++] = f64_order_bits(w.p[q].vals[i]);
}

void lw_rank_prefix(const LwRankPanes& w, int64_t kmin, int64_t nkeys, uint32_t* total,
                    uint32_t* pre) {
  for (int64_t k = 0; k < nkeys; ++k) {
    uint32_t run = 0;
    for (int j = 0; j < w.n; ++j) {
      const int64_t o = kmin + k - w.p[j].kbase;
      pre[(int64_t)j * nkeys + k] = run;
      run += (o >= 0 && o < w.p[j].ksize) ? w.p[j].counts[o] : 0u;
    }
    total[k] = run;
  }
}

void lw_rank_scatter(const LwRankPanes& w, int64_t kmin, int64_t nkeys, const int64_t* offs,
                     const uint32_t* pre, uint64_t* out_ord) {
  for (int j = 0; j < w.n; ++j)
    for (int64_t i = 0; i < w.p[j].len; ++i) {
      const int64_t k = w.p[j].keys[i] - kmin;
      out_ord[offs[k] + pre[(int64_t)j * nkeys + k] + w.p[j].ranks[i]] =
          f64_order_bits(w.p[j].vals[i]);
    }
}

}  // namespace cpu
}  // namespace mxs
