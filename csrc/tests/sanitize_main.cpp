// mxstream — host sanitizer harness. Built by `python -m mxstream.build
// --sanitize` with -fsanitize=address,undefined (and -fno-sanitize-recover) against the C++ twins
// of the kernels, then driven through a few micro-batches of the keyed window pipeline
// (partition -> window_agg -> fire), the vector-metric windows and the table checker, on
// adversarial shapes: tiny sub-tables, late data, bucket counts at capacity, empty batches.
// Exit code 0 and no sanitizer report = pass (tests/test_debug.py).
#include <cstdio>
#include <cstring>
#include <vector>

#include "mxs_check.h"
#include "mxs_kernels.h"
#include "mxs_vector.h"

using namespace mxs;

static int fail(const char* what) {
  std::fprintf(stderr, "sanitize_main: %s\n", what);
  return 1;
}

int main() {
  const int64_t n = 20000;
  const int nsub_log2 = 3, cap_log2 = 9, ring = 8, nsub = 1 << nsub_log2, dim = 32;
  const uint32_t bcap = 4096;
  const size_t nslots = (size_t)nsub << cap_log2;
  std::vector<uint64_t> keys(n), vals(n);
  std::vector<int64_t> ts(n);
  std::vector<int32_t> kg_dest(128, 0);
  std::vector<uint32_t> cursor(nsub);
  std::vector<Rec> recs((size_t)nsub * bcap);
  std::vector<int64_t> stats(kStatCount), red(16), local_maxts(1, INT64_MIN);
  std::vector<uint64_t> keys_g(nslots, kEmptyKey), acc_g(ring * nslots);
  std::vector<uint32_t> cnt_g(ring * nslots), occ(nsub), flags(4), late_idx(1024);
  std::vector<uint8_t> dirty_g(ring * nslots);
  std::vector<float> vec((size_t)n * dim), vacc_g(ring * nslots * dim);
  std::vector<uint64_t> vkeys_g(nslots, kEmptyKey);
  std::vector<uint32_t> vcnt_g(ring * nslots);
  std::vector<uint8_t> vdirty_g(ring * nslots);
  std::vector<uint64_t> out_keys(nslots), out_raw(nslots);
  std::vector<double> out_vals(nslots);
  std::vector<float> out_vec(nslots * dim);
  std::vector<uint32_t> out_cnt(nslots), out_n(1);

  int64_t fired_through = INT64_MIN;
  for (int step = 0; step < 6; ++step) {
    const int64_t m = step == 3 ? 0 : n;  // one empty batch
    cpu::gen_events(keys.data(), ts.data(), vals.data(), m, 7, 0, (uint64_t)step * n, 1500,
                    step * 1000, 1000, 400, 0, 1000, 0, 0.0);
    if (step == 5)
      for (int64_t i = 0; i < m; i += 50) ts[i] -= 4000;  // late data
    cpu::gen_vectors(vec.data(), m, dim, 7, 0, (uint64_t)step * n, -10.0f, 100.0f);
    cpu::step_begin(cursor.data(), nsub, stats.data());
    PartPlan pp;
    std::memset(&pp, 0, sizeof(pp));
    pp.max_parallelism = 128;
    pp.nsub_log2 = nsub_log2;
    pp.nranks = 1;
    pp.window_mode = 1;
    pp.drop_late = 1;
    pp.bucket_cap = bcap;
    pp.late_ts = step >= 2 ? (step - 2) * 1000 : INT64_MIN;
    pp.tbase = -1000;
    pp.pane = 500;
    pp.inv_pane = 1.0 / 500;
    pp.rec_words = 3;
    // Values carry the row index for the vector path; the scalar path sums them.
    for (int64_t i = 0; i < m; ++i) vals[i] = (uint64_t)i;
    cpu::partition(keys.data(), ts.data(), vals.data(), nullptr, m, pp, kg_dest.data(),
                   cursor.data(), recs.data(), stats.data(), late_idx.data(),
                   (uint32_t)late_idx.size());
    cpu::step_finish(stats.data(), local_maxts.data(), 400, 1, 0, red.data(), nullptr);
    if (stats[kStatOverflow]) return fail("bucket overflow");
    const int64_t qmin = stats[kStatMinPane], qmax = stats[kStatMaxPane];
    if (qmin > qmax) continue;
    AggPlan ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.cap_log2 = cap_log2;
    ap.nsub = nsub;
    ap.ring = ring;
    ap.agg = AGG_SUM_I64;
    ap.nsrc = 1;
    ap.bucket_cap = bcap;
    ap.np_step = (int32_t)(qmax - qmin + 1);
    ap.pg = 1;
    ap.pane_base = 0;
    ap.p_lo = qmin;
    ap.fired_hi = fired_through;
    ap.rec_words = 3;
    if (ap.np_step > ring) return fail("ring too small");
    cpu::window_agg(recs.data(), cursor.data(), ap, keys_g.data(), acc_g.data(), cnt_g.data(),
                    dirty_g.data(), occ.data(), flags.data());
    VecAggPlan vp;
    std::memset(&vp, 0, sizeof(vp));
    vp.cap_log2 = cap_log2;
    vp.nsub = nsub;
    vp.ring = ring;
    vp.dim = dim;
    vp.nsrc = 1;
    vp.bucket_cap = bcap;
    vp.np_step = ap.np_step;
    vp.rec_words = 3;
    vp.p_lo = qmin;
    vp.fired_hi = fired_through;
    cpu::vec_window_agg(recs.data(), cursor.data(), vp, vec.data(), vkeys_g.data(),
                        vacc_g.data(), vcnt_g.data(), vdirty_g.data(), occ.data(), flags.data());
    // Fire the oldest pane's window (one pane per window here).
    FirePlan fp;
    std::memset(&fp, 0, sizeof(fp));
    fp.agg = AGG_SUM_I64;
    fp.npanes = 1;
    fp.ring = ring;
    fp.nslots = (int64_t)nslots;
    fp.p0 = qmin;
    fp.out_cap = (uint32_t)nslots;
    out_n[0] = 0;
    cpu::window_fire(keys_g.data(), acc_g.data(), cnt_g.data(), dirty_g.data(), fp,
                     out_keys.data(), out_vals.data(), out_raw.data(), out_cnt.data(),
                     out_n.data());
    VecFirePlan vf;
    std::memset(&vf, 0, sizeof(vf));
    vf.dim = dim;
    vf.npanes = 1;
    vf.ring = ring;
    vf.avg = 1;
    vf.nslots = (int64_t)nslots;
    vf.p0 = qmin;
    vf.out_cap = (uint32_t)nslots;
    uint32_t vn = 0;
    cpu::vec_window_fire(vkeys_g.data(), vacc_g.data(), vcnt_g.data(), vdirty_g.data(), vf,
                         out_keys.data(), out_vec.data(), out_cnt.data(), &vn);
    if (vn != out_n[0]) return fail("vector and scalar windows disagree on live keys");
    fired_through = qmin;
  }
  uint64_t chk[kChkN] = {0, 0, 0, 0};
  cpu::check_table(keys_g.data(), nsub, nsub_log2, cap_log2, chk);
  if (chk[kChkMisplaced] || chk[kChkBrokenChain] || chk[kChkDuplicate] || !chk[kChkLive])
    return fail("table invariant violated");
  std::printf("sanitize_main ok: %llu live keys\n", (unsigned long long)chk[kChkLive]);
  return 0;
}
