// mxstream — the keyed window operator's step, native: ONE C++ implementation of the per-rank
// micro-batch loop of an event-/processing-time window (keyBy partition, watermark valve, pane
// aggregation, firing, late re-firing, purge, host-DRAM spill tier) shared by the Python-bound
// operator (runtime/window_operator.py KeyedWindowOperator, through the pybind class WindowStep)
// and the C ABI pipeline (csrc/pipeline.cpp, csrc/mxs_c.h). The Python layer only converts
// arguments and wraps the fired rows; every phase of a step -- front, settle, aggregate, fire,
// purge, spill -- runs here, with the GIL released.
//
// Reference semantics: chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:30-55
// (bounded-out-of-orderness watermark, keyBy, sliding event-time window, reduce, map, filter),
// chapter3/README.md:209-228 (allowed lateness), BandwidthMonitor.java:32-40 (processing time).
//
// Step shape (one process() call, pipelined mode "stream"):
//
//   S0:  gen/ingest(i+1) | front(i+1): step_begin + partition + step_finish [+ MIN all-reduce]
//        -> reduced vector to pinned host memory (event)              <- the step's host sync
//        back(i): [combine + exchange] window_agg, re-fire, fire, purge, spill check
//   copy stream: fired rows -> pinned slabs (device-counted copy), resolved by take()
//
// Collectives (world > 1) go through StepComm: the Python binding forwards them to the rank's
// torch.distributed process group (RCCL over xGMI on the GPU box, gloo / loopback on the CPU).
#ifndef MXS_WINDOW_STEP_H_
#define MXS_WINDOW_STEP_H_

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "mxs_kernels.h"
#include "mxs_vector.h"
#include "window_control.h"
#include "window_tier.h"

namespace mxs {

// A buffer owned by the step: device memory on a GPU, host memory on the CPU twin, or page-locked
// host memory (pinned = true). Shared with the tensor views handed to Python, so a regrow never
// frees memory a view still reads.
struct MemBlock {
  void* p = nullptr;
  size_t bytes = 0;
  int kind = 0;  // 0 host, 1 device, 2 pinned host
  ~MemBlock();
};
using Buf = std::shared_ptr<MemBlock>;
Buf mem_alloc(size_t bytes, int kind, bool zero = true);

template <class T>
inline T* P(const Buf& b) {
  return b ? reinterpret_cast<T*>(b->p) : nullptr;
}

// Collectives of the keyBy exchange (world > 1). Buffers are the step's own; `elem` is the element
// size in bytes of the all-to-all (every rank sends bytes / world to each peer).
struct StepComm {
  int world = 1, rank = 0;
  virtual ~StepComm() = default;
  virtual void allreduce_min_i64(int64_t* buf, int n, intptr_t stream) = 0;
  virtual void all_to_all(void* recv, const void* send, int64_t bytes, int elem,
                          intptr_t stream) = 0;
};

struct WindowStepConfig {
  int64_t size = 60000, slide = 60000, offset = 0, lateness = 0;
  int32_t agg = AGG_SUM_I64;
  bool gpu = false;
  int device_index = 0;
  int parallelism = 0, max_parallelism = 128;
  int hash_mode = 0;
  const int32_t* jhash = nullptr;  // key id -> Java String.hashCode (hash_mode 1; caller-owned)
  ExprProg map{}, filt{};
  int64_t max_keys = 1 << 20, batch_capacity = 1 << 20;
  double bucket_slack = 1.5;
  int cap_log2 = -1;               // -1: automatic geometry
  bool event_time = true;
  int64_t ooo_bound = 0;
  bool side_output_late = false;
  int64_t late_capacity = 1 << 16;
  bool external_watermark = false;
  int combine = -1, compact = -1, narrow = -1;  // -1: automatic
  bool dense_keys = false;
  int pipeline = 0;                // 0 off, 1 "stream" (one stream, deferred order), 2 two streams
  int exchange = 0;                // 0 auto, 1 records, 2 partials (local-global)
  int idle_timeout_steps = -1;
  bool deterministic = false;
  bool spill = false;
  double spill_load = 0.8;
  int spill_check_steps = 8;
  int spill_keep_panes = -1;
  bool emit_kv = false;
  int latency_fire = 0;
  int64_t window_keys = -1;
  // Vector windows (runtime/vector_window_operator.py): dim > 0 keeps one f32 vector per (key,
  // pane) and fires the per-key sum / average vector (csrc/vector_hip.hip, MFMA).
  int dim = 0;
  bool vec_avg = true;
  bool vec_has_threshold = false;
  double vec_threshold = 0.0;
  int vec_mode = 0;
};

// One firing (or a batched group of firings) whose rows are on their way to a host slab.
struct FireBatch {
  std::vector<int64_t> wins;     // window starts, in firing order
  bool kv = false, only_dirty = false, bounds = false, vec = false;
  int64_t seq = 0;
  Buf slab;                      // host memory holding every column (views keep it alive)
  int64_t flags_off = 0, bounds_off = 0, ncap = 0;
  int64_t col_off[4] = {0, 0, 0, 0};
  int col_esz[4] = {8, 8, 8, 4};
  int ncols = 4;
  hipEvent_t ev = nullptr;       // the copy's completion (null: already on the host)
  // resolved (host) row bounds: per window, cumulative
  std::vector<uint32_t> hb;
};

// A resolved window result (rows are views into `slab`).
struct FireRows {
  int64_t start = 0, end = 0;
  bool refire = false, kv = false, vec = false;
  int64_t seq = 0;
  int64_t n = 0;
  Buf slab;
  const void* keys = nullptr;
  const double* vals = nullptr;
  const float* vecs = nullptr;
  const int64_t* raw = nullptr;
  const int32_t* cnt = nullptr;
};

// Native stage timing: with timing on, each phase of a step (partition, combine,
// all_to_all, window_agg, fire) is bracketed by HIP events on its stream (GPU) or the host clock
// (CPU); take_stages() returns the resolved (stage, ms) samples. The hook, when set by the Python
// module, also opens a named range (roctx with MXS_ROCTX=1, Chrome trace spans) per phase.
using StageRangeHook = void (*)(const char* name, bool push);
extern StageRangeHook g_stage_range_hook;
struct StageSample {
  const char* name;
  hipEvent_t a, b;
  double ms;
};

struct StepMetrics {
  int64_t num_records_in = 0, num_late_records_dropped = 0, num_records_out = 0, num_fires = 0;
  int64_t current_watermark = INT64_MIN, steps = 0, bucket_regrows = 0, ring_regrows = 0;
  int64_t compact_fallbacks = 0, latency_fires = 0, combine_regrows = 0, a2a_bytes = 0;
  int64_t payload_bytes = 0, merge_compactions = 0, async_evictions = 0, dropped_keys = 0;
  int64_t spilled_keys = 0, spilled_rows = 0;
};

class WindowStep {
 public:
  WindowStep(const WindowStepConfig& cfg, std::shared_ptr<StepComm> comm);
  ~WindowStep();
  WindowStep(const WindowStep&) = delete;
  WindowStep& operator=(const WindowStep&) = delete;

  // ---- entry points (stream: the caller's HIP stream, S0) ---------------------------------
  // keys: int64 (or int32 dictionary ids, key32), ts: int64, vals: int64 (the f64 bit pattern of
  // float aggregates; the batch row for vector windows, whose vectors are `vecs` [n x dim]).
  void process(const void* keys, bool key32, const int64_t* ts, const void* vals, int64_t n,
               intptr_t stream, const float* vecs = nullptr);
  void flush(intptr_t stream);
  void advance_watermark(int64_t wm, intptr_t stream);
  void finish(intptr_t stream);
  // Firings in order. block = false: stop at the first whose copy is still running.
  std::vector<FireRows> take(bool block);
  bool has_results() const { return !done_.empty() || !queue_.empty(); }
  // After process(): true when its firings should be resolved now (unpipelined, or a
  // latency-bounded firing), false when they may stay in flight until a later call.
  bool block_hint() const { return block_hint_; }

  // ---- control -----------------------------------------------------------------------------
  void mark_idle(bool idle) { idle_marked_ = idle; }
  bool idle() const {
    return idle_marked_ || (cfg_.idle_timeout_steps >= 0 && empty_steps_ >= cfg_.idle_timeout_steps);
  }
  void set_proc_time(int64_t now) { proc_now_ = now; }  // processing time of the next batch
  // Table maintenance at a step boundary: drop keys without live data and (spill) move keys
  // whose newest pane <= cutoff to the host tier. Returns {dropped, evicted, rows} (-1: async).
  std::vector<int64_t> compact_state(bool has_cutoff, int64_t cutoff, bool wait, intptr_t stream);
  void sync_state(intptr_t stream);  // pending half applied, streams drained, evictions landed
  void drain_all();
  // Device-side invariant check of the hashed table (MXS_DEBUG); throws on a violation.
  void check_table(intptr_t stream);

  // ---- state (checkpoint / restore / introspection) ------------------------------------------
  WindowControl& ctl() { return ctl_; }
  StepMetrics& metrics() { return m_; }
  const StepMetrics& metrics() const { return m_; }
  const WindowStepConfig& cfg() const { return cfg_; }
  int64_t wm() const { return wm_; }
  void set_wm(int64_t w) { wm_ = w; m_.current_watermark = w; }
  int world() const { return world_; }
  int nsub() const { return nsub_; }
  int nsub_log2() const { return nsub_log2_; }
  int cap_log2() const { return cap_log2_; }
  int64_t nslots() const { return nslots_; }
  int64_t ring() const { return ring_; }
  int rec_w() const { return rec_w_; }
  int dense_bits() const { return dense_bits_; }
  uint32_t dense_mul() const { return dense_mul_; }
  bool local_global() const { return local_global_; }
  bool exchanging() const { return exchanging_; }
  bool combine() const { return combine_; }
  int nbuckets() const { return nbuckets_; }
  int64_t bucket_cap() const { return bucket_cap_; }
  int64_t batch_capacity() const { return batch_capacity_; }
  bool pipeline() const { return pipeline_ != 0; }
  int fire_group() const { return fire_group_; }
  bool has_tier() const { return tier_ != nullptr; }
  WindowTierCore* tier() { return tier_.get(); }
  bool use_dlist() const { return dlist_ != nullptr; }
  bool async_fire() const { return async_fire_; }
  bool two_level() const { return scratch_ != nullptr; }
  void set_ccap_hint(uint32_t c) { ccap_hint_ = c; }
  void set_timing(bool on) { timing_ = on; }
  // The key id -> Java hash table (hash_mode 1) moves when the string dictionary grows.
  void set_jhash(const int32_t* j) { cfg_.jhash = j; }
  std::vector<std::pair<std::string, double>> take_stages();
  int64_t ring_m() const { return ring_m_; }
  int64_t nslots_o() const { return nslots_o_; }
  int nsub_o() const { return nsub_o_; }
  int nsub_o_log2() const { return nsub_o_log2_; }
  int cap_log2_o() const { return cap_log2_o_; }
  // Named state buffers (keys_g, acc_g, cnt_g, dirty_g, occ, dacc_g, dcnt_g, vacc_g, keys_m,
  // acc_m, cnt_m, dirty_m, occ_m, dlist, dlist_n, slot_mark, flags, kg_dest, out_keys, ...).
  Buf buffer(const std::string& name) const;
  // Replace the ring by `ring` panes (restore), state zeroed.
  void reset_state(int64_t ring);
  // Late side output of event-time steps: the dropped elements' batch row indices.
  std::vector<std::vector<uint32_t>>& late_side() { return late_side_; }
  // Local-global: rebuild the owners' merged values of fired, not yet cleaned windows (restore).
  void rebuild_merge_ring(intptr_t stream);

 private:
  struct Front {
    const void* keys = nullptr;
    bool key32 = false;
    const int64_t* ts = nullptr;
    const void* vals = nullptr;
    const float* vecs = nullptr;
    int64_t n = 0;
    int par = 0, cpar = 0;
    int64_t old_wm = INT64_MIN, pane_base = 0, proc_now = 0;
    int rw = 3;
    bool idle = false;
    hipEvent_t ev = nullptr;
  };
  struct Back {
    int par = 0, cpar = 0;
    int64_t n = 0, old_wm = INT64_MIN, pane_base = 0;
    int rw = 3;
    bool has_data = false;
    int64_t qmin = 0, np_step = 0, pg = 1, gmin = 0, gmax = -1, fired_hi = INT64_MIN;
    bool has_new_wm = false;
    int64_t new_wm = 0;
    uint32_t ccap = 0, hard = 0;
    hipEvent_t chk_ev = nullptr;
    int64_t maxb = 0;
    int64_t fill = 0;      // largest bucket fill (over all ranks with the records exchange)
    int64_t accepted = 0;  // records this rank's partition kept
    uint32_t pmask = 0;
    int64_t np_act = 0, seq = 0;
    const float* vecs = nullptr;
  };

  // geometry / buffers
  void geometry(int64_t max_keys);
  void init_owner_tables(int64_t max_keys);
  void alloc_buckets(int64_t capacity, double slack);
  void alloc_state(int64_t ring);
  void grow_ring(int64_t need);
  bool two_level_ok() const;
  int rank_of_kg(int kg) const;
  // step phases
  Front front(const void* keys, bool key32, const int64_t* ts, const void* vals,
              const float* vecs, int64_t n);
  void launch_front(Front& f);
  Back settle(Front& f);
  void back_begin(Back& b);
  void back_finish(Back& b);
  int64_t due_windows(const Back& b);
  int64_t pane_base(const int64_t* ts, int64_t n);
  // combine (records exchange with the sender-side combiner)
  void combine_begin(Back& b);
  void combine_finish(Back& b, const Rec** recs, const uint32_t** counts, uint32_t* bcap);
  void exchange_records(Back& b, uint32_t* xcap_out);
  void aggregate(const Rec* recs, const uint32_t* counts, AggPlan& ap, const Back* b);
  bool agg_pack_ok(int rw) const;
  // firing
  void fire_ready(int64_t wm, int64_t seq);
  void refire(int64_t pmin, int64_t pmax, int64_t old_wm, int64_t seq);
  void fire_list(const std::vector<int64_t>& starts, bool only_dirty, int64_t seq);
  void fire_many(const std::vector<int64_t>& starts, bool only_dirty, int64_t seq);
  bool refire_fused(const std::vector<int64_t>& starts, const std::vector<FireWin>& wins,
                    int64_t seq);
  void fire_window(int64_t s, bool only_dirty, int64_t seq);
  void fire_window_partials(int64_t s, int64_t p0, int64_t p1, bool only_dirty, bool emit,
                            int64_t seq);
  void fire_window_tiered(int64_t s, int64_t p0, int64_t p1, bool only_dirty, int64_t seq);
  void fire_window_vector(int64_t s, int64_t p0, int64_t p1, bool only_dirty, int64_t seq);
  void maybe_compact_merge();
  void purge(int64_t wm);
  void zero_panes(int64_t r, int64_t k);
  // host rows
  void queue_counted(FireBatch&& fb, const std::vector<std::pair<const void*, int>>& cols,
                     int64_t cap, const uint32_t* n_dev, bool with_bounds,
                     const uint32_t* bounds_dev, int nwin, hipEvent_t* busy);
  void queue_sync(FireBatch&& fb, const std::vector<std::pair<const void*, int>>& cols,
                  int64_t n, std::vector<uint32_t> hb);
  uint32_t fired_count();  // host sync: rows of the last single fire (checks the flags)
  void check_fire_flags(const uint32_t* hf);
  Buf take_slab(size_t bytes);
  void claim(hipEvent_t* ev);
  void claim_flags();
  // spill tier
  void maybe_spill();
  void land_evictions();
  struct TierTab;
  void tier_rows(int64_t p0, int64_t p1, Buf* k, Buf* a, Buf* c, int64_t* n);
  void tier_combine(const uint32_t* n_dev, int dev_mode, int tier_mode, int64_t p0, int64_t p1);
  // plumbing
  void memset_async(const Buf& b, int byte, size_t off, size_t bytes);
  void copy_d2d(void* dst, const void* src, size_t bytes);
  void to_host_sync(void* dst, const void* src, size_t bytes);
  hipEvent_t new_event();
  void recycle(hipEvent_t e);
  void record(hipEvent_t ev, hipStream_t s);
  void host_wait(hipEvent_t ev);
  hipStream_t st() const { return cur_; }
  intptr_t sti() const { return (intptr_t)cur_; }
  struct StreamScope;
  struct Stage;
  bool timing_ = false;
  std::vector<StageSample> stages_;

  WindowStepConfig cfg_;
  std::shared_ptr<StepComm> comm_;
  WindowControl ctl_;
  StepMetrics m_;
  int world_ = 1, rank_ = 0, parallelism_ = 1, part_ranks_ = 1;
  bool gpu_ = false, local_global_ = false, exchanging_ = false, combine_ = false;
  bool async_fire_ = false, debug_ = false, sparse_panes_ = true, fused_refire_ = true;
  bool agg_pack_env_ = true, evict_pane_sort_ = true, tier_bg_ = false;
  int force_split_ = 0;
  int pipeline_ = 0;
  int nsub_ = 0, nsub_log2_ = 0, cap_log2_ = 0, dense_bits_ = 0, rec_w_ = 3, nbuckets_ = 0;
  uint32_t dense_mul_ = 0;
  int64_t nslots_ = 0, ring_ = 4, bucket_cap_ = 0, batch_capacity_ = 0;
  double slack_ = 1.5;
  int fire_group_ = 1;
  int64_t orows_ = 0;
  int64_t wm_ = INT64_MIN;
  bool idle_marked_ = false;
  int64_t empty_steps_ = 0, proc_now_ = 0;
  int par_ = 0;
  hipStream_t cur_ = nullptr, s0_ = nullptr, s1_ = nullptr, copy_ = nullptr;
  // state
  Buf keys_g_, acc_g_, cnt_g_, dirty_g_, dacc_g_, dcnt_g_, vacc_g_, occ_, flags_, kg_dest_;
  Buf local_maxts_, dlist_, dlist_n_, slot_mark_, late_idx_, minbuf_, hflags_, wide_;
  bool block_hint_ = true;
  Buf send_[2], red_[2], hred_[2];
  // Bucket cursors and partition stats rotate over three sets (cpar): a step's step_finish
  // resets the next step's set, last read by the state half of the step two before (queued
  // ahead, or waited for through ev_consumed_) -- the next step launches no step_begin.
  Buf cursor_[3], stats_[3];
  int cpar_ = 0;
  bool refire_cleared_ = false;  // the last refire()'s fused kernel cleared its listed slots
  // Device bytes the fused re-firing's staging may take to skip its list-length read
  // (MXS_REFIRE_STAGE_MB, default 8 GiB of the 288 GB HBM).
  int64_t refire_stage_budget_ = (int64_t)8192 << 20;
  bool fused_reset_ = true;  // MXS_STEP_RESET=0: a step_begin launch per step (A/B)
  bool debug_exchange_ = false;  // MXS_DEBUG_EXCHANGE=1: one stderr line per records exchange
  bool cready_[3] = {false, false, false};
  Buf recv_, recv_counts_, scratch_, scratch_cursor_, comb_send_, comb_recv_, comb_counts_;
  Buf chk_, hchk_;
  Buf out_keys_, out_vals_, out_raw_, out_cnt_, fire_bounds_, hbounds_, out_vec_;
  Buf stage_[5];
  Buf rout_[10];
  int64_t rout_cap_ = 0;
  bool rout_kv_ = false;
  Buf send_vec_, recv_vec_;
  // local-global owner side
  int nsub_o_ = 0, nsub_o_log2_ = 0, cap_log2_o_ = 0;
  int64_t nslots_o_ = 0, ring_m_ = 1, fbcap_ = 0, mfires_ = 0;
  Buf keys_m_, acc_m_, cnt_m_, dirty_m_, occ_m_, fsend_, frecv_, fcursor_, frecv_counts_, part_n_;
  Buf fxsend_, fmax_, xsend_, comb_x_;
  // plan caches
  PartPlan pplan_{};
  bool pplan_ok_ = false;
  int64_t pplan_key_[5] = {0, 0, 0, 0, 0};
  uint32_t ccap_hint_ = 0;
  hipEvent_t ev_consumed_[2] = {nullptr, nullptr}, ev_part_[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> ev_pool_, free_ev_;
  hipEvent_t ready_ev_ = nullptr;
  Buf evict_slab_;
  std::unique_ptr<Back> pending_;
  hipEvent_t out_busy_ = nullptr, rout_busy_ = nullptr, tout_busy_ = nullptr;
  std::deque<FireBatch> queue_;   // firings whose rows may still be in flight, in order
  std::deque<FireRows> done_;
  std::vector<Buf> slabs_;        // host slab pool (reused once no view holds a slab)
  std::vector<std::vector<uint32_t>> late_side_;
  int64_t dirty_lo_ = 0;
  uint32_t dirty_mask_ = 0;
  // spill tier
  std::unique_ptr<WindowTierCore> tier_;
  Buf sp_key_, sp_pane_, sp_acc_, sp_cnt_, sp_dirty_, sp_ctr_, sp_skey_, sp_sacc_, sp_scnt_,
      sp_sdirty_, sp_pcount_;
  int64_t sp_cap_ = 0;
  struct Eviction {
    Buf slab;
    hipEvent_t ev = nullptr;
    int64_t ctr_off = 0, pc_off = 0, off[5] = {0, 0, 0, 0, 0}, cap = 0;
    bool presorted = false;
    int64_t p_lo = 0, np = 0;
  };
  std::unique_ptr<Eviction> evict_pending_;
  hipEvent_t evict_busy_ = nullptr;
  int64_t occ_prev_ = -1;
  Buf tt_[8];
  int64_t tt_size_ = 0;
  Buf tier_slabs_[4];
  hipEvent_t tier_slab_ev_[4] = {nullptr, nullptr, nullptr, nullptr};
  Buf tier_k_, tier_a_, tier_c_;
  int64_t tier_dev_cap_ = 0;
};

}  // namespace mxs

#endif  // MXS_WINDOW_STEP_H_
