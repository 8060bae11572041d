// mxstream — native keyed event-time window pipeline + C ABI (mxs_c.h).
//
// A host without Python (a JNI binding of the Java DataStream API, a C/C++ service) runs the
// reference's BandwidthMonitorWithEventTime shape
// (chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:30-55) through the SAME
// native window step as the Python operator (csrc/window_step.h WindowStep: Flink window
// assignment, bounded-out-of-orderness watermark, late drop, re-firing of late-but-allowed data,
// purge after cleanup time, Long.MAX_VALUE watermark at end of input), on gfx950 (device = 1) or
// the C++ twins (device = 0). tests/test_capi.py replays the chapter3 README golden stream through
// the C ABI. Also here: the rolling-aggregate and session loops of the C ABI.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "mxs_c.h"
#include "window_step.h"
#include "mxs_check.h"
#include "mxs_kernels.h"
#include "session_store.h"

namespace mxs {
namespace {

thread_local std::string g_err;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

int64_t next_pow2(int64_t x) {
  int64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Device-or-host buffers of one pipeline (the rolling loop below).
struct Mem {
  bool gpu = false;
  hipStream_t stream = nullptr;
  std::vector<void*> owned;

  void* alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0) bytes = 8;
    if (gpu) {
      hip_ok(hipMalloc(&p, bytes), "hipMalloc");
    } else {
      p = std::calloc(1, bytes);
      if (!p) throw std::bad_alloc();
    }
    owned.push_back(p);
    return p;
  }
  void release(void* p) {
    if (!p) return;
    owned.erase(std::remove(owned.begin(), owned.end(), p), owned.end());
    if (gpu) (void)hipFree(p);
    else std::free(p);
  }
  void fill(void* p, int byte, size_t bytes) {
    if (gpu) hip_ok(hipMemsetAsync(p, byte, bytes, stream), "hipMemsetAsync");
    else std::memset(p, byte, bytes);
  }
  void to_dev(void* dst, const void* src, size_t bytes) {
    if (gpu) hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream), "H2D");
    else std::memcpy(dst, src, bytes);
  }
  void to_host(void* dst, const void* src, size_t bytes) {
    if (gpu) {
      hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream), "D2H");
      hip_ok(hipStreamSynchronize(stream), "hipStreamSynchronize");
    } else {
      std::memcpy(dst, src, bytes);
    }
  }
  ~Mem() {
    for (void* p : owned) {
      if (gpu) (void)hipFree(p);
      else std::free(p);
    }
  }
};

// runtime/geometry.py state_geometry(max_keys, world = 1) (the rolling loop's tables)
void state_geometry(int64_t max_keys, int* nsub_out, int* cap_log2_out) {
  const double per_rank = (double)max_keys + 64;
  const double load = 0.7;
  int64_t nsub = next_pow2(std::max<int64_t>(1, (int64_t)std::ceil(per_rank / (4096 * load))));
  nsub = std::max<int64_t>(nsub, 256);
  const double need = per_rank / (double)nsub / load;
  int cl = (int)std::ceil(std::log2(std::max(need, 2.0)));
  cl = std::max(6, std::min(12, cl));
  const double mean = per_rank / (double)nsub;
  while (cl < 12 && mean + 4 * std::sqrt(mean) + 8 > (double)(1 << cl) * 0.85) ++cl;
  *nsub_out = (int)nsub;
  *cap_log2_out = cl;
}

}  // namespace

// The C ABI's window pipeline: the SAME native step the Python operator runs
// (csrc/window_step.h WindowStep, one rank, unpipelined), fed from host arrays.
class WindowPipeline {
 public:
  explicit WindowPipeline(const mxs_window_config& c) : gpu_(c.device != 0) {
    if (c.lateness_ms < 0 || c.ooo_bound_ms < 0) throw std::invalid_argument("negative lateness / bound");
    WindowStepConfig w;
    w.size = c.size_ms;
    w.slide = c.slide_ms;
    w.offset = c.offset_ms;
    w.lateness = c.lateness_ms;
    w.agg = c.agg;
    w.gpu = gpu_;
    w.device_index = c.device_index;
    w.max_parallelism = c.max_parallelism > 0 ? c.max_parallelism : 128;
    w.max_keys = std::max<int64_t>(c.max_keys, 1);
    w.batch_capacity = std::max<int64_t>(c.batch_capacity, 1024);
    w.ooo_bound = c.ooo_bound_ms;
    struct One : StepComm {
      void allreduce_min_i64(int64_t*, int, intptr_t) override {}
      void all_to_all(void* r, const void* s, int64_t b, int, intptr_t) override {
        if (r != s) std::memmove(r, s, (size_t)b);
      }
    };
    if (gpu_) {
      hip_ok(hipSetDevice(c.device_index), "hipSetDevice");
      hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    }
    step_.reset(new WindowStep(w, std::make_shared<One>()));
  }
  ~WindowPipeline() {
    step_.reset();
    if (gpu_ && stream_) (void)hipStreamDestroy(stream_);
    for (void* p : in_) (void)hipFree(p);  // device copies of the host batches (GPU only)
  }

  void process(const uint64_t* keys_h, const int64_t* ts_h, const int64_t* vals_h, int64_t n) {
    if (n < 0) throw std::invalid_argument("negative batch size");
    const void *k = keys_h, *t = ts_h, *v = vals_h;
    if (gpu_ && n) {
      if (n > in_cap_) {
        for (void* p : in_) (void)hipFree(p);
        in_.assign(3, nullptr);
        for (auto& p : in_) hip_ok(hipMalloc(&p, (size_t)n * 8), "hipMalloc");
        in_cap_ = n;
      }
      hip_ok(hipMemcpyAsync(in_[0], keys_h, n * 8, hipMemcpyHostToDevice, stream_), "H2D");
      hip_ok(hipMemcpyAsync(in_[1], ts_h, n * 8, hipMemcpyHostToDevice, stream_), "H2D");
      hip_ok(hipMemcpyAsync(in_[2], vals_h, n * 8, hipMemcpyHostToDevice, stream_), "H2D");
      k = in_[0];
      t = in_[1];
      v = in_[2];
    }
    step_->process(k, false, (const int64_t*)t, v, n, (intptr_t)stream_);
    collect();
  }

  void finish() {
    step_->finish((intptr_t)stream_);
    collect();
  }

  int64_t watermark() const { return step_->wm(); }
  int64_t late_dropped() const { return step_->metrics().num_late_records_dropped; }
  int64_t records_in() const { return step_->metrics().num_records_in; }
  std::deque<mxs_window_result> results;

 private:
  void collect() {
    for (const FireRows& r : step_->take(true))
      for (int64_t i = 0; i < r.n; ++i)
        results.push_back({r.start, r.end, ((const uint64_t*)r.keys)[i], r.vals[i], r.raw[i],
                           (uint32_t)r.cnt[i], r.refire ? 1 : 0});
  }

  bool gpu_;
  hipStream_t stream_ = nullptr;
  std::unique_ptr<WindowStep> step_;
  std::vector<void*> in_;
  int64_t in_cap_ = 0;
};

}  // namespace mxs

// ---- C ABI ----------------------------------------------------------------------------------
namespace mxs {
// The single-rank control loop of runtime/rolling_operator.py (KeyedRollingOperator) in C++:
// GPU = _process_direct (rolling_lookup_direct -> sort_pairs over the slot bits -> rolling_heads
// -> rolling_scan, count_n for count windows); CPU = partition (window_mode 0) -> rolling_rows.
class RollingPipeline {
 public:
  explicit RollingPipeline(const mxs_rolling_config& c) : cfg_(c) {
    if (c.agg < AGG_SUM_I64 || c.agg > AGG_AVG_I64) throw std::invalid_argument("unknown aggregate");
    if ((c.agg == AGG_AVG_F64 || c.agg == AGG_AVG_I64) && c.count_window <= 0)
      throw std::invalid_argument("rolling avg is not a Flink rolling aggregate (count windows only)");
    if (c.count_window < 0 || c.count_window >= ((int64_t)1 << 31))
      throw std::invalid_argument("count window size out of range");
    mem_.gpu = c.device != 0;
    if (mem_.gpu) {
      hip_ok(hipSetDevice(c.device_index), "hipSetDevice");
      hip_ok(hipStreamCreateWithFlags(&mem_.stream, hipStreamNonBlocking), "hipStreamCreate");
    }
    state_geometry(std::max<int64_t>(c.max_keys, 1), &nsub_, &cap_log2_);
    nsub_log2_ = 0;
    while ((1 << nsub_log2_) < nsub_) ++nsub_log2_;
    nslots_ = (int64_t)nsub_ << cap_log2_;
    keys_g_ = (uint64_t*)mem_.alloc(nslots_ * 8);
    mem_.fill(keys_g_, 0xFF, nslots_ * 8);
    acc_g_ = (uint64_t*)mem_.alloc(nslots_ * 8);
    mem_.fill(acc_g_, 0, nslots_ * 8);
    cnt_g_ = (uint32_t*)mem_.alloc(nslots_ * 4);
    mem_.fill(cnt_g_, 0, nslots_ * 4);
    flags_ = (uint32_t*)mem_.alloc(16);
    mem_.fill(flags_, 0, 16);
    nbuf_ = (uint32_t*)mem_.alloc(16);
    kg_dest_ = (int32_t*)mem_.alloc(128 * 4);
    mem_.fill(kg_dest_, 0, 128 * 4);
    stats_ = (int64_t*)mem_.alloc(kStatCount * 8);
    grow(std::max<int64_t>(c.batch_capacity, 1024));
  }
  ~RollingPipeline() {
    if (mem_.gpu && mem_.stream) {
      (void)hipStreamSynchronize(mem_.stream);
      (void)hipStreamDestroy(mem_.stream);
    }
  }

  void process(const uint64_t* keys_h, const int64_t* vals_h, int64_t n) {
    if (n < 0) throw std::invalid_argument("negative batch size");
    if (n == 0) return;
    if (n >= ((int64_t)1 << 31)) throw std::invalid_argument("batch too large");
    if (n > cap_) grow(n);
    mem_.to_dev(in_keys_, keys_h, n * 8);
    mem_.to_dev(in_vals_, vals_h, n * 8);
    const ExprProg none{};
    uint32_t hn[4];
    if (mem_.gpu) {
      const intptr_t st = (intptr_t)mem_.stream;
      mem_.fill(nbuf_, 0, 16);
      int shift = 1;
      while (((int64_t)1 << shift) < n) ++shift;
      int nb = 0;
      while (((int64_t)1 << nb) <= nslots_) ++nb;  // bit length of nslots
      gpu::rolling_lookup_direct(in_keys_, in_vals_, (uint32_t)n, nsub_log2_, cap_log2_, keys_g_,
                                 sort_key_, vals_buf_, nbuf_, flags_, shift, st);
      const int nbits = shift + nb;
      const size_t need = gpu::sort_pairs_temp_bytes(n, shift, nbits);
      if (need > temp_bytes_) {
        mem_.release(temp_);
        temp_ = mem_.alloc(need);
        temp_bytes_ = need;
      }
      gpu::sort_pairs(temp_, temp_bytes_, (const uint64_t*)sort_key_, (uint64_t*)sort_out_,
                      vals_buf_, vals_out_, n, shift, nbits, st);
      gpu::rolling_heads(sort_out_, nbuf_, n, heads_, nbuf_ + 1, shift, st);
      mem_.fill(flags_ + 2, 0, 4);  // emitted-row cursor
      gpu::rolling_scan(cfg_.agg, sort_out_, nullptr, vals_out_, nbuf_, heads_, nbuf_ + 1,
                        std::min<int64_t>(n, nslots_), acc_g_, cnt_g_, keys_g_, none, out_key_,
                        out_val_, out_tag_, flags_ + 2, (uint32_t)cap_, shift, shift, st,
                        (uint32_t)cfg_.count_window);
    } else {
      // Keyed (non-window) partition into sub-table buckets, then the sequential twin.
      PartPlan pp;
      std::memset(&pp, 0, sizeof(pp));
      pp.max_parallelism = 128;
      pp.nsub_log2 = nsub_log2_;
      pp.nranks = 1;
      pp.bucket_cap = bcap_;
      pp.pane = 1;
      pp.inv_pane = 1.0;
      pp.rec_words = 3;
      std::vector<int64_t> ts0((size_t)n, 0);
      uint32_t* counts = (uint32_t*)heads_;  // nsub counters (host memory on the CPU path)
      for (;;) {
        cpu::step_begin(counts, nsub_, stats_);
        cpu::partition(in_keys_, ts0.data(), in_vals_, nullptr, n, pp, kg_dest_, counts,
                       (Rec*)sort_key_, stats_, nullptr, 0);
        if (!(stats_[kStatOverflow] & 1)) break;
        bcap_ *= 2;  // a bucket overflowed: larger buckets, same batch again
        alloc_buckets();
        pp.bucket_cap = bcap_;
      }
      flags_[2] = 0;
      cpu::rolling_rows((const Rec*)sort_key_, counts, 1, nsub_, bcap_, cap_log2_, cfg_.agg,
                        keys_g_, acc_g_, cnt_g_, flags_, none, out_key_, out_val_, out_tag_,
                        flags_ + 2, (uint32_t)cap_, (uint32_t)cfg_.count_window);
    }
    mem_.to_host(hn, flags_, 16);
    if (hn[0] & 1) throw std::runtime_error("keyed state table full: a key found no free slot (raise max_keys)");
    if (hn[0] & 4) throw std::invalid_argument("key ids -1 and -2 are reserved");
    const int64_t rows = std::min<int64_t>(hn[2], cap_);
    if (!rows) return;
    std::vector<uint64_t> k((size_t)rows), v((size_t)rows);
    std::vector<int64_t> t((size_t)rows);
    mem_.to_host(k.data(), out_key_, rows * 8);
    mem_.to_host(v.data(), out_val_, rows * 8);
    mem_.to_host(t.data(), out_tag_, rows * 8);
    std::vector<int64_t> order((size_t)rows);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      return (t[a] & 0xFFFFFFFF) < (t[b] & 0xFFFFFFFF);
    });
    for (int64_t j : order)
      rows_.push_back(mxs_rolling_row{k[j], (int64_t)v[j], t[j] & 0xFFFFFFFF});
    records_in_ += n;
  }

  std::deque<mxs_rolling_row> rows_;

 private:
  // sort_key_ doubles as the CPU path's bucketed Rec buffer (nsub x bcap records).
  void alloc_buckets() {
    mem_.release(sort_key_);
    const int64_t recs = mem_.gpu ? cap_ : std::max<int64_t>((int64_t)nsub_ * bcap_, cap_);
    sort_key_ = (int64_t*)mem_.alloc(recs * (mem_.gpu ? 8 : 24));
  }

  void grow(int64_t n) {
    cap_ = std::max<int64_t>(n, cap_);
    bcap_ = std::max<uint32_t>(bcap_, (uint32_t)std::max<int64_t>(64, (int64_t)(1.5 * (double)cap_ / nsub_ + 64)));
    for (void* q : {(void*)in_keys_, (void*)in_vals_, (void*)sort_out_,
                    (void*)vals_buf_, (void*)vals_out_, (void*)heads_, (void*)out_key_,
                    (void*)out_val_, (void*)out_tag_})
      mem_.release(q);
    in_keys_ = (uint64_t*)mem_.alloc(cap_ * 8);
    in_vals_ = (uint64_t*)mem_.alloc(cap_ * 8);
    alloc_buckets();
    sort_out_ = (int64_t*)mem_.alloc(cap_ * 8);
    vals_buf_ = (uint64_t*)mem_.alloc(cap_ * 8);
    vals_out_ = (uint64_t*)mem_.alloc(cap_ * 8);
    heads_ = (uint32_t*)mem_.alloc(std::max<int64_t>(cap_, nsub_) * 4);
    out_key_ = (uint64_t*)mem_.alloc(cap_ * 8);
    out_val_ = (uint64_t*)mem_.alloc(cap_ * 8);
    out_tag_ = (int64_t*)mem_.alloc(cap_ * 8);
  }

  mxs_rolling_config cfg_;
  Mem mem_;
  int nsub_ = 0, cap_log2_ = 0, nsub_log2_ = 0;
  int64_t nslots_ = 0, cap_ = 0, records_in_ = 0;
  uint32_t bcap_ = 0;
  size_t temp_bytes_ = 0;
  void* temp_ = nullptr;
  uint64_t *keys_g_ = nullptr, *acc_g_ = nullptr, *in_keys_ = nullptr, *in_vals_ = nullptr;
  uint64_t *vals_buf_ = nullptr, *vals_out_ = nullptr, *out_key_ = nullptr, *out_val_ = nullptr;
  int64_t *sort_key_ = nullptr, *sort_out_ = nullptr, *out_tag_ = nullptr, *stats_ = nullptr;
  uint32_t *cnt_g_ = nullptr, *flags_ = nullptr, *nbuf_ = nullptr, *heads_ = nullptr;
  int32_t* kg_dest_ = nullptr;
};
}  // namespace mxs

struct mxs_pipeline {
  mxs::WindowPipeline impl;
  explicit mxs_pipeline(const mxs_window_config& c) : impl(c) {}
};

struct mxs_rolling {
  mxs::RollingPipeline impl;
  explicit mxs_rolling(const mxs_rolling_config& c) : impl(c) {}
};

namespace {
template <class F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    mxs::g_err = e.what();
  } catch (...) {
    mxs::g_err = "unknown error";
  }
  return -1;
}
}  // namespace

extern "C" {

void mxs_window_config_default(mxs_window_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->size_ms = 60000;
  c->slide_ms = 60000;
  c->agg = MXS_AGG_SUM_I64;
  c->max_parallelism = 128;
  c->max_keys = 1 << 16;
  c->batch_capacity = 1 << 16;
}

mxs_pipeline* mxs_pipeline_create(const mxs_window_config* cfg) {
  if (!cfg) {
    mxs::g_err = "null config";
    return nullptr;
  }
  mxs_pipeline* p = nullptr;
  if (guard([&] { p = new mxs_pipeline(*cfg); }) != 0) return nullptr;
  return p;
}

void mxs_pipeline_destroy(mxs_pipeline* p) { delete p; }

int mxs_pipeline_process(mxs_pipeline* p, const uint64_t* keys, const int64_t* ts,
                         const int64_t* vals, int64_t n) {
  if (!p || (n > 0 && (!keys || !ts || !vals))) {
    mxs::g_err = "null argument";
    return -1;
  }
  return guard([&] { p->impl.process(keys, ts, vals, n); });
}

int mxs_pipeline_finish(mxs_pipeline* p) {
  if (!p) return -1;
  return guard([&] { p->impl.finish(); });
}

int64_t mxs_pipeline_num_results(const mxs_pipeline* p) {
  return p ? (int64_t)p->impl.results.size() : -1;
}

int64_t mxs_pipeline_take_results(mxs_pipeline* p, mxs_window_result* out, int64_t cap) {
  if (!p || (cap > 0 && !out)) return -1;
  int64_t n = 0;
  while (n < cap && !p->impl.results.empty()) {
    out[n++] = p->impl.results.front();
    p->impl.results.pop_front();
  }
  return n;
}

int64_t mxs_pipeline_watermark(const mxs_pipeline* p) { return p ? p->impl.watermark() : INT64_MIN; }
int64_t mxs_pipeline_late_dropped(const mxs_pipeline* p) { return p ? p->impl.late_dropped() : -1; }
int64_t mxs_pipeline_records_in(const mxs_pipeline* p) { return p ? p->impl.records_in() : -1; }
void mxs_rolling_config_default(mxs_rolling_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->agg = MXS_AGG_SUM_I64;
  c->max_keys = 1 << 16;
  c->batch_capacity = 1 << 16;
}

mxs_rolling* mxs_rolling_create(const mxs_rolling_config* cfg) {
  if (!cfg) {
    mxs::g_err = "null config";
    return nullptr;
  }
  mxs_rolling* r = nullptr;
  if (guard([&] { r = new mxs_rolling(*cfg); }) != 0) return nullptr;
  return r;
}

void mxs_rolling_destroy(mxs_rolling* r) { delete r; }

int mxs_rolling_process(mxs_rolling* r, const uint64_t* keys, const int64_t* vals, int64_t n) {
  if (!r || (n > 0 && (!keys || !vals))) {
    mxs::g_err = "null argument";
    return -1;
  }
  return guard([&] { r->impl.process(keys, vals, n); });
}

int64_t mxs_rolling_num_rows(const mxs_rolling* r) { return r ? (int64_t)r->impl.rows_.size() : -1; }

int64_t mxs_rolling_take_rows(mxs_rolling* r, mxs_rolling_row* out, int64_t cap) {
  if (!r || (cap > 0 && !out)) return -1;
  int64_t n = 0;
  while (n < cap && !r->impl.rows_.empty()) {
    out[n++] = r->impl.rows_.front();
    r->impl.rows_.pop_front();
  }
  return n;
}

// ---- sessions ---------------------------------------------------------------------------------
struct mxs_session {
  explicit mxs_session(const mxs_session_config& c)
      : store(c.gap_ms, c.lateness_ms, c.agg), bound(c.ooo_bound_ms), agg(c.agg) {
    if (c.lateness_ms < 0 || c.ooo_bound_ms < 0) throw std::invalid_argument("negative lateness / bound");
    if (c.agg < 0 || c.agg > MXS_AGG_AVG_I64) throw std::invalid_argument("unknown aggregate");
  }
  void fire_at(int64_t w) {
    wm = w;
    if (wm == INT64_MIN) return;
    mxs::sess::SessionCore::FireOut o;
    const mxs::ExprProg none = mxs::sess::SessionCore::prog(nullptr, 0, nullptr, 0);
    store.fire(wm, none, none, o);
    for (size_t i = 0; i < o.okey.size(); ++i)
      results.push_back(mxs_session_result{(uint64_t)o.okey[i], o.ostart[i], o.oend[i], o.oval[i],
                                           o.oraw[i], (uint32_t)o.ocnt[i], (int32_t)o.oref[i]});
  }
  void process(const uint64_t* k, const int64_t* t, const int64_t* v, int64_t n) {
    // Same micro-batch order as the Python operator: fold against the old watermark, then fire
    // at the advanced one (late data may re-open fired sessions without moving it).
    late += store.process((const int64_t*)k, t, v, n, wm);
    for (int64_t i = 0; i < n; ++i) maxts = std::max(maxts, t[i]);
    const int64_t w = maxts == INT64_MIN ? INT64_MIN : maxts - bound;
    fire_at(std::max(wm, w));
  }
  mxs::sess::SessionCore store;
  int64_t bound, wm = INT64_MIN, maxts = INT64_MIN, late = 0;
  int32_t agg;
  std::deque<mxs_session_result> results;
};

void mxs_session_config_default(mxs_session_config* cfg) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->gap_ms = 5000;
  cfg->agg = MXS_AGG_SUM_I64;
}

mxs_session* mxs_session_create(const mxs_session_config* cfg) {
  if (!cfg) {
    mxs::g_err = "null config";
    return nullptr;
  }
  mxs_session* s = nullptr;
  if (guard([&] { s = new mxs_session(*cfg); }) != 0) return nullptr;
  return s;
}

void mxs_session_destroy(mxs_session* s) { delete s; }

int mxs_session_process(mxs_session* s, const uint64_t* keys, const int64_t* ts,
                        const int64_t* vals, int64_t n) {
  if (!s || (n > 0 && (!keys || !ts || !vals))) {
    mxs::g_err = "null argument";
    return -1;
  }
  return guard([&] { s->process(keys, ts, vals, n); });
}

int mxs_session_finish(mxs_session* s) {
  if (!s) return -1;
  return guard([&] { s->fire_at(INT64_MAX); });
}

int64_t mxs_session_num_results(const mxs_session* s) { return s ? (int64_t)s->results.size() : -1; }

int64_t mxs_session_take_results(mxs_session* s, mxs_session_result* out, int64_t cap) {
  if (!s || (cap > 0 && !out)) return -1;
  int64_t n = 0;
  while (n < cap && !s->results.empty()) {
    out[n++] = s->results.front();
    s->results.pop_front();
  }
  return n;
}

int64_t mxs_session_watermark(const mxs_session* s) { return s ? s->wm : INT64_MIN; }
int64_t mxs_session_late_dropped(const mxs_session* s) { return s ? s->late : -1; }

const char* mxs_last_error(void) { return mxs::g_err.c_str(); }
const char* mxs_version(void) { return "mxstream-native 0.1 (gfx950)"; }

}  // extern "C"
