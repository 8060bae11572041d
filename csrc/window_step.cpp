// mxstream — the keyed window operator's native step (csrc/window_step.h). Every phase of a
// micro-batch -- front (partition + watermark valve), settle (the step's one host sync), the state
// half (combine / exchange / window_agg), firing (batched, fused re-firing, local-global partials,
// tiered, vector), purge and the host-DRAM spill tier -- is driven from here; the gfx950 kernels
// (kernels_hip.hip, vector_hip.hip) or their C++ twins (kernels_cpu.cpp) do the work.
//
// Reference: chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:30-55;
// chapter3/README.md:209-228 (allowed lateness); SURVEY.md §3.4-3.5 (window semantics).
#include "window_step.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <thread>

#include "mxs_check.h"

namespace mxs {

namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

int64_t next_pow2(int64_t x) {
  int64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

int bit_length(uint64_t x) {
  int b = 0;
  while (x) {
    ++b;
    x >>= 1;
  }
  return b;
}

bool env_on(const char* name, bool def) {
  const char* v = std::getenv(name);
  if (!v || !*v) return def;
  return std::strcmp(v, "0") != 0;
}

int env_int(const char* name, int def) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : def;
}

// runtime/geometry.py state_geometry: LDS-sized hash sub-tables for one rank.
void state_geometry(int64_t max_keys, int world, int cap_log2, int* nsub_out, int* cl_out) {
  const int64_t per_rank =
      (int64_t)((double)max_keys / world * (world > 1 ? 1.3 : 1.0)) + 64;
  if (cap_log2 >= 0 && cap_log2 < 9) {  // explicit small tables (tests): load <= 0.5
    *nsub_out = (int)next_pow2(std::max<int64_t>(
        1, (int64_t)std::ceil((double)per_rank / ((double)(1 << cap_log2) * 0.5))));
    *cl_out = cap_log2;
    return;
  }
  const double load = 0.7;
  int64_t nsub = next_pow2(std::max<int64_t>(
      1, (int64_t)std::ceil((double)per_rank / ((double)(1 << 12) * load))));
  nsub = std::max<int64_t>(nsub, next_pow2(std::max(1, 256 / world)));
  const double need = (double)per_rank / (double)nsub / load;
  int cl = (int)std::ceil(std::log2(std::max(need, 2.0)));
  cl = std::max(6, std::min(12, cl));
  const double mean = (double)per_rank / (double)nsub;
  while (cl < 12 && mean + 4 * std::sqrt(mean) + 8 > (double)(1 << cl) * 0.85) ++cl;
  *nsub_out = (int)nsub;
  *cl_out = cl;
}

constexpr int kRedWords = 16;
constexpr int64_t kAggSlice = 131072;  // records per workgroup of a split sub-table
}  // namespace

// ---- memory --------------------------------------------------------------------------------
MemBlock::~MemBlock() {
  if (!p) return;
  if (kind == 1) (void)hipFree(p);
  else if (kind == 2) (void)hipHostFree(p);
  else std::free(p);
}

Buf mem_alloc(size_t bytes, int kind, bool zero) {
  auto b = std::make_shared<MemBlock>();
  bytes = std::max<size_t>(bytes, 16);
  bytes = (bytes + 255) & ~(size_t)255;
  b->bytes = bytes;
  b->kind = kind;
  if (kind == 1) {
    hip_ok(hipMalloc(&b->p, bytes), "hipMalloc");
    if (zero) {
      hip_ok(hipMemset(b->p, 0, bytes), "hipMemset");
      hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    }
  } else if (kind == 2) {
    hip_ok(hipHostMalloc(&b->p, bytes, hipHostMallocDefault), "hipHostMalloc");
    if (zero) std::memset(b->p, 0, bytes);
  } else {
    if (posix_memalign(&b->p, 256, bytes) != 0) throw std::bad_alloc();
    if (zero) std::memset(b->p, 0, bytes);
  }
  return b;
}

StageRangeHook g_stage_range_hook = nullptr;

// One timed phase of a step (see StageSample); a no-op unless timing or a range hook is on.
struct WindowStep::Stage {
  WindowStep* w;
  const char* name;
  hipEvent_t a = nullptr;
  std::chrono::steady_clock::time_point t0;
  Stage(WindowStep* s, const char* n) : w(s), name(n) {
    if (g_stage_range_hook) g_stage_range_hook(n, true);
    if (!w->timing_) return;
    if (w->gpu_) {
      hip_ok(hipEventCreate(&a), "hipEventCreate");
      hip_ok(hipEventRecord(a, w->cur_), "hipEventRecord");
    } else {
      t0 = std::chrono::steady_clock::now();
    }
  }
  ~Stage() {
    if (g_stage_range_hook) g_stage_range_hook(name, false);
    if (!w->timing_) return;
    if (w->gpu_) {
      hipEvent_t b = nullptr;
      if (hipEventCreate(&b) == hipSuccess && hipEventRecord(b, w->cur_) == hipSuccess)
        w->stages_.push_back({name, a, b, 0.0});
    } else {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      w->stages_.push_back({name, nullptr, nullptr, ms});
    }
  }
};

std::vector<std::pair<std::string, double>> WindowStep::take_stages() {
  std::vector<std::pair<std::string, double>> out;
  std::vector<StageSample> keep;
  for (auto& s : stages_) {
    if (s.a) {
      if (hipEventQuery(s.b) != hipSuccess) {
        keep.push_back(s);
        continue;
      }
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, s.a, s.b);
      (void)hipEventDestroy(s.a);
      (void)hipEventDestroy(s.b);
      out.emplace_back(s.name, (double)ms);
    } else {
      out.emplace_back(s.name, s.ms);
    }
  }
  stages_.swap(keep);
  return out;
}

// The state half of a step on the operator's second stream (pipeline mode 2), restored after.
struct WindowStep::StreamScope {
  WindowStep* w;
  hipStream_t saved;
  StreamScope(WindowStep* s, bool use_s1) : w(s), saved(s->cur_) {
    if (use_s1 && s->s1_) s->cur_ = s->s1_;
  }
  ~StreamScope() { w->cur_ = saved; }
};

// ---- construction ----------------------------------------------------------------------------
WindowStep::WindowStep(const WindowStepConfig& c, std::shared_ptr<StepComm> comm)
    : cfg_(c), comm_(std::move(comm)), ctl_(c.size, c.slide, c.offset, c.lateness) {
  gpu_ = c.gpu;
  world_ = comm_ ? comm_->world : 1;
  rank_ = comm_ ? comm_->rank : 0;
  if (c.agg < AGG_SUM_I64 || c.agg > AGG_AVG_I64) throw std::invalid_argument("unknown aggregate");
  if (c.ooo_bound < 0) throw std::invalid_argument("negative out-of-orderness bound");
  if (gpu_) hip_ok(hipSetDevice(c.device_index), "hipSetDevice");
  const bool vec = c.dim > 0;
  parallelism_ = c.parallelism > 0 ? c.parallelism : world_;
  const bool det = c.deterministic && (c.agg == AGG_SUM_F64 || c.agg == AGG_AVG_F64);
  cfg_.deterministic = det;
  // ---- keyBy exchange strategy (G > 1): "partials" = local-global aggregation (a rank folds
  // its own events into a table of the whole key space; a fired window's partial rows cross ONE
  // all-to-all to the key's owner); "records" = every step's records cross to the key's owner.
  const bool lg_ok = world_ > 1 && !vec && !det;
  if (c.exchange == 2 && world_ > 1 && !lg_ok)
    throw std::invalid_argument("exchange='partials' needs deterministic=False and a plain reduce");
  local_global_ = lg_ok && c.exchange != 1;
  exchanging_ = world_ > 1 && !local_global_;
  part_ranks_ = exchanging_ ? world_ : 1;

  // ---- state geometry ----
  if (c.dense_keys) {
    if (exchanging_ || vec)
      throw std::invalid_argument("dense_keys needs one destination (G = 1 or exchange='partials')");
    int bits = std::max(4, bit_length((uint64_t)std::max<int64_t>(c.max_keys - 1, 0)));
    if (bits > 32) throw std::invalid_argument("dense_keys: ids must fit 32 bits");
    int cl = c.cap_log2 < 0 ? std::min(12, bits) : std::min(c.cap_log2, bits);
    cl = std::min(cl, std::max(5, bits - 8));
    nsub_ = 1 << (bits - cl);
    cap_log2_ = cl;
    dense_bits_ = bits;
    dense_mul_ = (uint32_t)((0x9E3779B1ull & ((1ull << bits) - 1)) | 1ull);
  } else {
    state_geometry(c.max_keys, part_ranks_, c.cap_log2, &nsub_, &cap_log2_);
  }
  nsub_log2_ = bit_length((uint64_t)nsub_) - 1;
  if ((int64_t)nsub_ * part_ranks_ > 16384)
    throw std::invalid_argument("key space too large for the bucket histogram; raise cap_log2");
  nslots_ = (int64_t)nsub_ << cap_log2_;
  const int64_t pane = ctl_.pane();
  ring_ = std::max<int64_t>(4, next_pow2(ctl_.panes_per_window() + 2 + (c.lateness + pane - 1) / pane +
                                         (std::max(c.ooo_bound, c.slide) + pane - 1) / pane));
  const int dk = gpu_ ? 1 : 0;
  keys_g_ = mem_alloc(nslots_ * 8, dk, false);
  if (dense_bits_) {
    // The key of every slot: the inverse bijection (dense slots are never "inserted").
    uint64_t inv = 1, m = dense_mul_, mask = (dense_bits_ == 64) ? ~0ull : ((1ull << dense_bits_) - 1);
    for (int i = 0; i < 6; ++i) inv = inv * (2 - m * inv);  // Newton: inverse mod 2^64
    std::vector<uint64_t> k((size_t)nslots_);
    for (int64_t s = 0; s < nslots_; ++s) k[(size_t)s] = ((uint64_t)s * inv) & mask;
    if (gpu_) hip_ok(hipMemcpy(keys_g_->p, k.data(), nslots_ * 8, hipMemcpyHostToDevice), "H2D keys");
    else std::memcpy(keys_g_->p, k.data(), nslots_ * 8);
  } else if (gpu_) {
    hip_ok(hipMemset(keys_g_->p, 0xFF, nslots_ * 8), "hipMemset");
  } else {
    std::memset(keys_g_->p, 0xFF, nslots_ * 8);
  }
  alloc_state(ring_);
  occ_ = mem_alloc(nsub_ * 4, dk);
  flags_ = mem_alloc(16, dk);
  kg_dest_ = mem_alloc(cfg_.max_parallelism * 4, dk);
  {
    std::vector<int32_t> kgd(cfg_.max_parallelism);
    for (int kg = 0; kg < cfg_.max_parallelism; ++kg) kgd[kg] = rank_of_kg(kg);
    if (gpu_) hip_ok(hipMemcpy(kg_dest_->p, kgd.data(), kgd.size() * 4, hipMemcpyHostToDevice), "H2D");
    else std::memcpy(kg_dest_->p, kgd.data(), kgd.size() * 4);
  }
  nbuckets_ = part_ranks_ << nsub_log2_;
  combine_ = (c.combine < 0 ? exchanging_ : (c.combine > 0 && exchanging_)) && !det && !vec;
  // Pipelining: the partition of batch i+1 is enqueued before the state half of batch i.
  pipeline_ = (c.pipeline && !c.external_watermark && (c.pipeline == 1 || !local_global_)) ? c.pipeline : 0;
  if (gpu_) {
    // the caller's stream is S0; the copy stream and (mode 2) the state stream are the step's own
    if (pipeline_ == 2) hip_ok(hipStreamCreateWithFlags(&s1_, hipStreamNonBlocking), "stream");
  }
  slack_ = c.bucket_slack;
  alloc_buckets(c.batch_capacity, c.bucket_slack);
  for (int p = 0; p < (pipeline_ ? 2 : 1); ++p) {
    red_[p] = mem_alloc(kRedWords * 8, dk);
    hred_[p] = mem_alloc(kRedWords * 8, gpu_ ? 2 : 0);
  }
  for (int p = 0; p < 3; ++p) {
    stats_[p] = mem_alloc(kStatCount * 8, dk);
    const int64_t init[kStatCount] = {INT64_MIN, INT64_MAX, INT64_MIN, 0, 0, 0, 0, 0};
    if (gpu_) hip_ok(hipMemcpy(stats_[p]->p, init, sizeof(init), hipMemcpyHostToDevice), "H2D");
    else std::memcpy(stats_[p]->p, init, sizeof(init));
  }
  hchk_ = mem_alloc(16, gpu_ ? 2 : 0);
  hflags_ = mem_alloc(16, gpu_ ? 2 : 0);
  chk_ = mem_alloc(16, dk);
  local_maxts_ = mem_alloc(8, dk);
  minbuf_ = mem_alloc(8, dk);
  {
    const int64_t mn = INT64_MIN;
    if (gpu_) hip_ok(hipMemcpy(local_maxts_->p, &mn, 8, hipMemcpyHostToDevice), "H2D");
    else std::memcpy(local_maxts_->p, &mn, 8);
  }
  if (local_global_)
    init_owner_tables(c.window_keys > 0 ? c.window_keys : (c.spill ? 4 * c.max_keys : c.max_keys));
  // Batched firing: up to fire_group due windows per launch group (one window's rows never
  // exceed nslots, so the output holds the group's rows).
  fire_group_ = vec ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>(64, ((int64_t)1 << 21) / nslots_));
  orows_ = nslots_ * fire_group_;
  if (local_global_) orows_ = std::max(orows_, nslots_o_);
  out_keys_ = mem_alloc(orows_ * 8, dk, false);
  out_vals_ = mem_alloc(orows_ * 8, dk, false);
  out_raw_ = mem_alloc(orows_ * 8, dk, false);
  out_cnt_ = mem_alloc(orows_ * 4, dk, false);
  fire_bounds_ = mem_alloc(((std::max(fire_group_, 32) + 3) & ~3) * 4, dk);
  hbounds_ = mem_alloc(std::max(fire_group_, 32) * 4, gpu_ ? 2 : 0);
  async_fire_ = gpu_ && env_on("MXS_ASYNC_FIRE", true);
  if (async_fire_ && env_on("MXS_COPY_STREAM", true))
    hip_ok(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking), "stream");
  if (gpu_) slabs_.push_back(mem_alloc((size_t)orows_ * 28 + 4 * 256, 2, false));
  if (c.side_output_late) late_idx_ = mem_alloc(c.late_capacity * 4, dk);
  // Touched-slot list (allowed lateness): re-firings visit only slots that received late data.
  if (c.lateness > 0 && !vec) {
    dlist_ = mem_alloc(nslots_ * 4, dk, false);
    dlist_n_ = mem_alloc(16, dk);
    slot_mark_ = mem_alloc(nslots_ * 4, dk);
  }
  comb_counts_ = mem_alloc(nbuckets_ * 4, dk);
  ccap_hint_ = 1u << cap_log2_;
  // Record width: 16-byte records (int32 values) for integer aggregates on the GPU; 8-byte ones
  // (32-bit key id, 28-bit value, 4-bit pane) for one destination or <= 512 exchange buckets. A
  // value that does not fit widens the format for good (the step is redone).
  const bool int_agg = c.agg == AGG_SUM_I64 || c.agg == AGG_MIN_I64 || c.agg == AGG_MAX_I64 ||
                       c.agg == AGG_COUNT || c.agg == AGG_AVG_I64;
  bool compact = c.compact < 0 ? (gpu_ && int_agg) : (c.compact > 0 && int_agg);
  bool narrow = c.narrow < 0 ? (compact && gpu_) : c.narrow > 0;
  const bool narrow_x = env_on("MXS_NARROW_EXCHANGE", true);
  narrow = narrow && compact && !vec &&
           (!exchanging_ || (narrow_x && (part_ranks_ << nsub_log2_) <= 512));
  rec_w_ = narrow ? 1 : compact ? 2 : 3;
  debug_ = env_on("MXS_DEBUG", false);
  sparse_panes_ = env_on("MXS_SPARSE_PANES", true);
  fused_refire_ = env_on("MXS_FUSED_REFIRE", true);
  agg_pack_env_ = env_on("MXS_AGG_PACK", true);
  force_split_ = env_int("MXS_AGG_FORCE_SPLIT", 0);
  refire_stage_budget_ = (int64_t)env_int("MXS_REFIRE_STAGE_MB", 8192) << 20;
  fused_reset_ = env_on("MXS_STEP_RESET", true);
  debug_exchange_ = env_on("MXS_DEBUG_EXCHANGE", false);
  evict_pane_sort_ = env_on("MXS_EVICT_PANE_SORT", true);
  if (c.spill) {
    if (dense_bits_ || vec) throw std::invalid_argument("spill needs hashed keys and a plain reduce");
    if (det)
      throw std::invalid_argument("deterministic=True does not combine with spill=True");
    tier_.reset(new WindowTierCore(c.agg));
    tier_->prefault_ = env_on("MXS_TIER_PREFAULT", true);
  }
  if (vec) {
    vacc_g_ = mem_alloc((size_t)ring_ * nslots_ * c.dim * 4, dk);
    out_vec_ = mem_alloc((size_t)nslots_ * c.dim * 4, dk, false);
  }
  if (gpu_) hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

WindowStep::~WindowStep() {
  if (gpu_) {
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
    if (s1_) (void)hipStreamDestroy(s1_);
    if (copy_) (void)hipStreamDestroy(copy_);
  }
}

int WindowStep::rank_of_kg(int kg) const {
  const int sub = kg * parallelism_ / cfg_.max_parallelism;
  return sub * world_ / parallelism_;
}

void WindowStep::alloc_state(int64_t ring) {
  const int dk = gpu_ ? 1 : 0;
  acc_g_ = mem_alloc((size_t)(cfg_.dim > 0 ? 1 : ring * nslots_) * 8, dk);
  cnt_g_ = mem_alloc((size_t)ring * nslots_ * 4, dk);
  dirty_g_ = mem_alloc((size_t)ring * nslots_, dk);
  if (local_global_ && cfg_.lateness > 0) {
    dacc_g_ = mem_alloc((size_t)ring * nslots_ * 8, dk);
    dcnt_g_ = mem_alloc((size_t)ring * nslots_ * 4, dk);
  }
}

void WindowStep::init_owner_tables(int64_t max_keys) {
  // The owner side of a local-global fire: the merge table of this rank's key share (one slice
  // per fired, not yet cleaned window) and the fire exchange buffers. A bucket (owner, owner
  // sub-table) holds at most one row per key of that sub-table: capacity = the sub-table's.
  state_geometry(max_keys, world_, cfg_.cap_log2, &nsub_o_, &cap_log2_o_);
  nsub_o_log2_ = bit_length((uint64_t)nsub_o_) - 1;
  if ((int64_t)nsub_o_ * world_ > 16384)
    throw std::invalid_argument("key space too large for the fire exchange; raise cap_log2");
  nslots_o_ = (int64_t)nsub_o_ << cap_log2_o_;
  ring_m_ = next_pow2((cfg_.lateness + cfg_.slide - 1) / cfg_.slide + 2);
  const int dk = gpu_ ? 1 : 0;
  keys_m_ = mem_alloc(nslots_o_ * 8, dk, false);
  memset_async(keys_m_, 0xFF, 0, nslots_o_ * 8);
  acc_m_ = mem_alloc(ring_m_ * nslots_o_ * 8, dk);
  cnt_m_ = mem_alloc(ring_m_ * nslots_o_ * 4, dk);
  dirty_m_ = mem_alloc(ring_m_ * nslots_o_, dk);
  occ_m_ = mem_alloc(nsub_o_ * 4, dk);
  fbcap_ = (int64_t)1 << cap_log2_o_;
  const int64_t nbf = (int64_t)world_ << nsub_o_log2_;
  fsend_ = mem_alloc(nbf * fbcap_ * 24, dk, false);
  fxsend_ = mem_alloc(nbf * fbcap_ * 24, dk, false);
  fmax_ = mem_alloc(16, dk);
  frecv_ = mem_alloc(nbf * fbcap_ * 24, dk, false);
  fcursor_ = mem_alloc(nbf * 4, dk);
  frecv_counts_ = mem_alloc(nbf * 4, dk);
  part_n_ = mem_alloc(16, dk);
}

bool WindowStep::two_level_ok() const {
  return gpu_ && part_ranks_ == 1 && nbuckets_ > 512 && nbuckets_ <= 512 * 32 &&
         env_on("MXS_TWO_LEVEL", true);
}

void WindowStep::alloc_buckets(int64_t capacity, double slack) {
  drain_all();
  batch_capacity_ = capacity;
  slack_ = slack;
  const double per = (double)capacity / nbuckets_;
  // The GPU partition pads every workgroup's run to whole 8-record groups (<= 7 holes per bucket
  // and workgroup, <= 1024 workgroups): capacity is a multiple of 8 with that slack.
  const int64_t nblk = std::min<int64_t>(1024, std::max<int64_t>(1, (capacity + 65535) / 65536));
  const int64_t cap = (int64_t)(per * slack + 6 * std::sqrt(std::max(per, 1.0)) + 64) + 8 * nblk;
  bucket_cap_ = (cap + 7) & ~(int64_t)7;
  const size_t words = (size_t)nbuckets_ * bucket_cap_ * 3;
  const int dk = gpu_ ? 1 : 0;
  for (int p = 0; p < (pipeline_ ? 2 : 1); ++p) send_[p] = mem_alloc(words * 8, dk, false);
  for (int p = 0; p < 3; ++p) {
    cursor_[p] = mem_alloc(nbuckets_ * 4, dk);
    cready_[p] = false;  // (fresh buffers: the next front runs its step_begin)
  }
  recv_ = exchanging_ && !combine_ ? mem_alloc(words * 8, dk, false) : nullptr;
  recv_counts_ = exchanging_ ? mem_alloc(nbuckets_ * 4, dk) : nullptr;
  scratch_ = scratch_cursor_ = nullptr;
  xsend_ = nullptr;  // the exchange's repack buffer follows the bucket capacity
  if (two_level_ok()) {
    scratch_ = mem_alloc((size_t)nbuckets_ * bucket_cap_ * 8, dk, false);
    scratch_cursor_ = mem_alloc(512 * 4, dk);
  }
  pplan_ok_ = false;
  for (auto& e : ev_consumed_) e = nullptr;
}

void WindowStep::grow_ring(int64_t need) {
  // Re-lay the pane ring so `need` consecutive panes fit (rare; keeps absolute pane ids).
  drain_all();
  const int64_t nr = next_pow2(need), old = ring_;
  Buf oacc = acc_g_, ocnt = cnt_g_, odirty = dirty_g_, odacc = dacc_g_, odcnt = dcnt_g_,
      ovacc = vacc_g_;
  alloc_state(nr);
  const int64_t D = cfg_.dim;
  if (D > 0) vacc_g_ = mem_alloc((size_t)nr * nslots_ * D * 4, gpu_ ? 1 : 0);
  if (ctl_.has_live())
    for (int64_t p = ctl_.min_live(); p <= ctl_.max_seen(); ++p) {
      const int64_t so = (p & (old - 1)) * nslots_, sn = (p & (nr - 1)) * nslots_;
      if (D > 0) copy_d2d(P<float>(vacc_g_) + sn * D, P<float>(ovacc) + so * D, nslots_ * D * 4);
      else copy_d2d(P<uint64_t>(acc_g_) + sn, P<uint64_t>(oacc) + so, nslots_ * 8);
      copy_d2d(P<uint32_t>(cnt_g_) + sn, P<uint32_t>(ocnt) + so, nslots_ * 4);
      copy_d2d(P<uint8_t>(dirty_g_) + sn, P<uint8_t>(odirty) + so, nslots_);
      if (dacc_g_ && odacc) {
        copy_d2d(P<uint64_t>(dacc_g_) + sn, P<uint64_t>(odacc) + so, nslots_ * 8);
        copy_d2d(P<uint32_t>(dcnt_g_) + sn, P<uint32_t>(odcnt) + so, nslots_ * 4);
      }
    }
  if (gpu_) hip_ok(hipStreamSynchronize(cur_), "sync");
  ring_ = nr;
  ++m_.ring_regrows;
}

void WindowStep::reset_state(int64_t ring) {
  drain_all();
  if (ring != ring_) {
    ring_ = ring;
    alloc_state(ring);
    if (cfg_.dim > 0) vacc_g_ = mem_alloc((size_t)ring * nslots_ * cfg_.dim * 4, gpu_ ? 1 : 0);
  } else {
    memset_async(acc_g_, 0, 0, acc_g_->bytes);
    memset_async(cnt_g_, 0, 0, cnt_g_->bytes);
    memset_async(dirty_g_, 0, 0, dirty_g_->bytes);
    if (vacc_g_) memset_async(vacc_g_, 0, 0, vacc_g_->bytes);
    if (dacc_g_) {
      memset_async(dacc_g_, 0, 0, dacc_g_->bytes);
      memset_async(dcnt_g_, 0, 0, dcnt_g_->bytes);
    }
  }
  if (!dense_bits_) memset_async(keys_g_, 0xFF, 0, nslots_ * 8);
  if (dlist_) {
    memset_async(dlist_n_, 0, 0, 16);
    memset_async(slot_mark_, 0, 0, slot_mark_->bytes);
  }
  memset_async(occ_, 0, 0, occ_->bytes);
  pending_.reset();
  evict_pending_.reset();
  queue_.clear();
  done_.clear();
  if (tier_) tier_->clear();
  drain_all();
}

Buf WindowStep::buffer(const std::string& n) const {
  if (n == "keys_g") return keys_g_;
  if (n == "acc_g") return acc_g_;
  if (n == "cnt_g") return cnt_g_;
  if (n == "dirty_g") return dirty_g_;
  if (n == "vacc_g") return vacc_g_;
  if (n == "dacc_g") return dacc_g_;
  if (n == "dcnt_g") return dcnt_g_;
  if (n == "occ") return occ_;
  if (n == "flags") return flags_;
  if (n == "kg_dest") return kg_dest_;
  if (n == "dlist") return dlist_;
  if (n == "dlist_n") return dlist_n_;
  if (n == "slot_mark") return slot_mark_;
  if (n == "keys_m") return keys_m_;
  if (n == "acc_m") return acc_m_;
  if (n == "cnt_m") return cnt_m_;
  if (n == "dirty_m") return dirty_m_;
  if (n == "occ_m") return occ_m_;
  if (n == "out_keys") return out_keys_;
  if (n == "out_vals") return out_vals_;
  if (n == "out_raw") return out_raw_;
  if (n == "out_cnt") return out_cnt_;
  if (n == "scratch") return scratch_;
  if (n == "send") return send_[0];
  if (n == "cursor") return cursor_[0];
  throw std::invalid_argument("WindowStep: no buffer named " + n);
}

// ---- plumbing ----------------------------------------------------------------------------------
void WindowStep::memset_async(const Buf& b, int byte, size_t off, size_t bytes) {
  if (!b || !bytes) return;
  if (gpu_) hip_ok(hipMemsetAsync((char*)b->p + off, byte, bytes, cur_), "hipMemsetAsync");
  else std::memset((char*)b->p + off, byte, bytes);
}

void WindowStep::copy_d2d(void* dst, const void* src, size_t bytes) {
  if (!bytes) return;
  if (gpu_) hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, cur_), "D2D");
  else std::memmove(dst, src, bytes);
}

void WindowStep::to_host_sync(void* dst, const void* src, size_t bytes) {
  if (!bytes) return;
  if (gpu_) {
    hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, cur_), "D2H");
    hip_ok(hipStreamSynchronize(cur_), "hipStreamSynchronize");
  } else {
    std::memcpy(dst, src, bytes);
  }
}

hipEvent_t WindowStep::new_event() {
  if (!free_ev_.empty()) {
    hipEvent_t e = free_ev_.back();
    free_ev_.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  ev_pool_.push_back(e);
  return e;
}

void WindowStep::recycle(hipEvent_t e) {
  // An event whose work has completed goes back to the pool; a busy marker naming it is cleared
  // (the copy it guards is done, nothing needs to wait for it any more).
  if (!e) return;
  for (hipEvent_t* b : {&out_busy_, &rout_busy_, &tout_busy_, &evict_busy_})
    if (*b == e) *b = nullptr;
  free_ev_.push_back(e);
}

void WindowStep::record(hipEvent_t ev, hipStream_t s) { hip_ok(hipEventRecord(ev, s), "hipEventRecord"); }

// The step's host waits poll the event (a blocking wait sleeps in the driver and wakes tens of
// microseconds late -- time the pipelined step cannot hide; profiles/r2_host_sync.md).
void WindowStep::host_wait(hipEvent_t ev) {
  if (!ev) return;
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) hip_ok(e, "hipEventQuery");
  }
}

void WindowStep::claim_flags() {
  // Every counted copy in flight reads the flags words (row count, overflow bits) when it runs
  // on the copy stream: whatever fire resets them next waits for all of them first, whichever
  // output columns they copy (plain, re-firing or tiered).
  claim(&out_busy_);
  claim(&rout_busy_);
  claim(&tout_busy_);
}

void WindowStep::claim(hipEvent_t* ev) {
  if (*ev) {
    hip_ok(hipStreamWaitEvent(cur_, *ev, 0), "hipStreamWaitEvent");
    *ev = nullptr;
  }
}

void WindowStep::drain_all() {
  if (!gpu_) return;
  if (cur_) hip_ok(hipStreamSynchronize(cur_), "sync");
  if (s1_) hip_ok(hipStreamSynchronize(s1_), "sync");
  if (copy_) hip_ok(hipStreamSynchronize(copy_), "sync");
  hip_ok(hipDeviceSynchronize(), "sync");
}

Buf WindowStep::take_slab(size_t bytes) {
  // A free slab (no FireRows view holds it) of at least `bytes`; reused, else a new one.
  const int kind = gpu_ ? 2 : 0;
  int smallest_free = -1;
  for (size_t i = 0; i < slabs_.size(); ++i) {
    if (slabs_[i].use_count() != 1) continue;
    if (slabs_[i]->bytes >= bytes) return slabs_[i];
    if (smallest_free < 0 || slabs_[i]->bytes < slabs_[(size_t)smallest_free]->bytes)
      smallest_free = (int)i;
  }
  if (slabs_.size() >= 8 && smallest_free >= 0) slabs_.erase(slabs_.begin() + smallest_free);
  Buf b = mem_alloc((size_t)next_pow2((int64_t)std::max<size_t>(bytes, 1 << 16)), kind, false);
  slabs_.push_back(b);
  return b;
}

// ---- entry points ------------------------------------------------------------------------------
void WindowStep::process(const void* keys, bool key32, const int64_t* ts, const void* vals,
                         int64_t n, intptr_t stream, const float* vecs) {
  cur_ = s0_ = (hipStream_t)stream;
  block_hint_ = !pipeline_;
  if (n > batch_capacity_ && world_ == 1 && pending_) {
    // The buffers are reallocated for this batch: the queued state half reads the old ones.
    flush(stream);
  }
  if (!pipeline_) {
    Front f = front(keys, key32, ts, vals, vecs, n);
    Back b = settle(f);
    back_begin(b);
    back_finish(b);
    return;
  }
  std::unique_ptr<Back> prev = std::move(pending_);
  if (prev) {
    StreamScope sc(this, true);
    back_begin(*prev);  // combiner + its tiny all-reduce, before S0's partition
  }
  Front f = front(keys, key32, ts, vals, vecs, n);  // partition of this batch (S0)
  if (prev) back_finish(*prev);
  Back b = settle(f);  // the step's one host sync (S1 / the queued state half keep working)
  if (cfg_.latency_fire > 0) {
    const int64_t due = due_windows(b);
    if (due > 0 && due <= cfg_.latency_fire) {
      // Latency-bounded firing: this batch's firings leave in this call.
      {
        StreamScope sc(this, true);
        back_begin(b);
      }
      back_finish(b);
      ++m_.latency_fires;
      block_hint_ = true;
      return;
    }
  }
  pending_.reset(new Back(b));
}

void WindowStep::flush(intptr_t stream) {
  cur_ = s0_ = (hipStream_t)stream;
  std::unique_ptr<Back> prev = std::move(pending_);
  if (prev) {
    {
      StreamScope sc(this, true);
      back_begin(*prev);
    }
    back_finish(*prev);
  }
}

void WindowStep::advance_watermark(int64_t wm, intptr_t stream) {
  flush(stream);
  if (wm <= wm_) return;
  wm_ = wm;
  m_.current_watermark = wm;
  StreamScope sc(this, true);
  fire_ready(wm, m_.steps);
  purge(wm);
}

void WindowStep::finish(intptr_t stream) {
  if (cfg_.event_time) advance_watermark(INT64_MAX, stream);
  else flush(stream);
}

void WindowStep::sync_state(intptr_t stream) {
  cur_ = s0_ = (hipStream_t)stream;
  if (pending_) flush(stream);
  drain_all();
  land_evictions();
}

int64_t WindowStep::due_windows(const Back& b) {
  return ctl_.due_count(b.has_data, b.has_data ? b.gmin : 0, b.has_data ? b.gmax : 0, b.fired_hi,
                        b.has_new_wm, b.has_new_wm ? b.new_wm : 0);
}

// ---- front: partition + watermark valve ----------------------------------------------------------
int64_t WindowStep::pane_base(const int64_t* ts, int64_t n) {
  // Base pane of the step, identical on every rank (records carry pane - base).
  if (wm_ > INT64_MIN) return ctl_.pane_base_from_wm(wm_);
  // No watermark yet: the global minimum timestamp (one MIN all-reduce, first steps only).
  int64_t m = INT64_MAX;
  if (gpu_) {
    gpu::fill_u64(P<uint64_t>(minbuf_), 1, (uint64_t)INT64_MAX, (intptr_t)cur_);
    if (n) gpu::min_i64(ts, n, P<int64_t>(minbuf_), (intptr_t)cur_);
  } else {
    for (int64_t i = 0; i < n; ++i) m = std::min(m, ts[i]);
    *P<int64_t>(minbuf_) = m;
  }
  if (world_ > 1) comm_->allreduce_min_i64(P<int64_t>(minbuf_), 1, (intptr_t)cur_);
  to_host_sync(&m, minbuf_->p, 8);
  int64_t base = m != INT64_MAX ? ctl_.pane_of(m) : 0;
  if (ctl_.has_live()) base = std::min(base, ctl_.min_live());
  return base;
}

WindowStep::Front WindowStep::front(const void* keys, bool key32, const int64_t* ts,
                                    const void* vals, const float* vecs, int64_t n) {
  // A batch past the capacity: one rank regrows alone (process() drained the pending state
  // half first); with peers the regrow is agreed through the step's reduced vector (settle).
  if (n > batch_capacity_ && world_ == 1) {
    flush((intptr_t)cur_);
    alloc_buckets(n, slack_);
  }
  Front f;
  f.par = par_;
  if (pipeline_) par_ ^= 1;
  f.cpar = cpar_;
  cpar_ = (cpar_ + 1) % 3;
  empty_steps_ = n == 0 ? empty_steps_ + 1 : 0;
  f.keys = keys;
  f.key32 = key32;
  f.ts = ts;
  f.vals = vals;
  f.vecs = vecs;
  f.n = n;
  f.old_wm = wm_;
  f.idle = idle();
  f.pane_base = pane_base(ts, n);
  f.proc_now = cfg_.event_time ? 0 : proc_now_;
  launch_front(f);
  return f;
}

void WindowStep::launch_front(Front& f) {
  const int p = f.par;
  if (gpu_ && ev_consumed_[p]) {
    // send[p] / cursor[p] are still read by the state half of the step before last
    hip_ok(hipStreamWaitEvent(cur_, ev_consumed_[p], 0), "wait");
  }
  f.rw = rec_w_;
  const bool two_level = rec_w_ == 1 && scratch_ != nullptr;
  bool key32 = f.key32;
  // int32 key ids (the columnar sources' dictionary ids) are read as they are by the compact GPU
  // partition; widened to int64 for the other paths.
  const void* keys_in = f.keys;
  if (key32 && gpu_ &&
      (!(((rec_w_ == 1 || rec_w_ == 2) && nbuckets_ <= 512) || two_level) ||
       (int64_t)nbuckets_ * bucket_cap_ >= ((int64_t)1 << 32))) {
    if (!wide_ || (int64_t)wide_->bytes < f.n * 8) wide_ = mem_alloc((size_t)f.n * 8, 1, false);
    gpu::widen_i32((const int32_t*)f.keys, f.n, P<int64_t>(wide_), (intptr_t)cur_);
    keys_in = wide_->p;
    key32 = false;
  }
  const int64_t key[5] = {bucket_cap_, rec_w_, cfg_.event_time ? 1 : 0, key32 ? 1 : 0,
                          two_level ? 1 : 0};
  if (!pplan_ok_ || std::memcmp(key, pplan_key_, sizeof(key)) != 0) {
    std::memset(&pplan_, 0, sizeof(pplan_));
    pplan_.max_parallelism = cfg_.max_parallelism;
    pplan_.nsub_log2 = nsub_log2_;
    pplan_.nranks = part_ranks_;
    pplan_.window_mode = 1;
    pplan_.drop_late = cfg_.event_time ? 1 : 0;
    pplan_.hash_mode = cfg_.hash_mode;
    pplan_.bucket_cap = (uint32_t)bucket_cap_;
    pplan_.pane = ctl_.pane();
    pplan_.inv_pane = 1.0 / (double)ctl_.pane();
    pplan_.rec_words = rec_w_;
    pplan_.dense_bits = dense_bits_;
    pplan_.dense_mul = dense_mul_;
    pplan_.key32 = key32 ? 1 : 0;
    if (two_level) {
      pplan_.scratch = P<uint64_t>(scratch_);
      pplan_.scratch_cursor = P<uint32_t>(scratch_cursor_);
    }
    std::memcpy(pplan_key_, key, sizeof(key));
    pplan_ok_ = true;
  }
  pplan_.late_ts = ctl_.late_ts(f.old_wm, cfg_.event_time);
  pplan_.tbase = ctl_.pane_start(f.pane_base);
  if (f.n >= ((int64_t)1 << 32)) throw std::invalid_argument("batch too large (2^32 events)");
  const int nb = nbuckets_;
  const int cp = f.cpar, cn = (f.cpar + 1) % 3;
  // (G > 1) a batch past the capacity is not partitioned: red[4] = -(n << 1) asks every rank to
  // regrow to n and redo the step (settle), so the bucket geometry stays the same on all ranks.
  const bool over = f.n > batch_capacity_;
  uint32_t* cur = P<uint32_t>(cursor_[cp]);
  Rec* send = P<Rec>(send_[p]);
  int64_t* stats = P<int64_t>(stats_[cp]);
  int64_t* red = P<int64_t>(red_[p]);
  uint32_t* li = P<uint32_t>(late_idx_);
  const uint32_t lcap = late_idx_ ? (uint32_t)cfg_.late_capacity : 0u;
  const int64_t bound = cfg_.ooo_bound;
  const int32_t ev = cfg_.event_time ? 1 : 0;
  Stage stage(this, "partition");
  if (gpu_) {
    const intptr_t s = (intptr_t)cur_;
    if (!cready_[cp]) gpu::step_begin(cur, nb, stats, s);  // (else reset by the last step_finish)
    cready_[cp] = false;  // a redo of this step resets them again
    if (f.n && !over)
      gpu::partition((const uint64_t*)keys_in, f.ts, (const uint64_t*)f.vals, cfg_.jhash, f.n,
                     pplan_, P<int32_t>(kg_dest_), cur, send, stats, li, lcap, s);
    gpu::step_finish(stats, P<int64_t>(local_maxts_), bound, ev, f.proc_now, red,
                     P<uint32_t>(flags_), s, f.idle ? 1 : 0,
                     world_ == 1 ? P<int64_t>(hred_[p]) : nullptr, exchanging_ ? 1 : 0, cur, nb,
                     fused_reset_ ? P<uint32_t>(cursor_[cn]) : nullptr,
                     fused_reset_ ? P<int64_t>(stats_[cn]) : nullptr);
    cready_[cn] = fused_reset_;
    if (over) gpu::fill_u64((uint64_t*)(red + 4), 1, (uint64_t)(-(f.n << 1)), s);
  } else {
    cpu::step_begin(cur, nb, stats);
    std::vector<uint64_t> wide;
    const void* keys = f.keys;
    if (f.n && key32) {  // int32 key ids: sign-extended copy for the CPU kernel
      wide.resize((size_t)f.n);
      const int32_t* k32 = (const int32_t*)f.keys;
      for (int64_t i = 0; i < f.n; ++i) wide[(size_t)i] = (uint64_t)(int64_t)k32[i];
      keys = wide.data();
    }
    if (f.n && !over)
      cpu::partition((const uint64_t*)keys, f.ts, (const uint64_t*)f.vals, cfg_.jhash, f.n, pplan_,
                     P<int32_t>(kg_dest_), cur, send, stats, li, lcap);
    cpu::step_finish(stats, P<int64_t>(local_maxts_), bound, ev, f.proc_now, red,
                     P<uint32_t>(flags_), f.idle ? 1 : 0, exchanging_ ? 1 : 0, cur, nb);
    if (over) red[4] = -(f.n << 1);
  }
  // Watermark valve + pane range + every overflow flag: ONE MIN all-reduce per step.
  int64_t dbg_before[8] = {0};
  if (debug_exchange_ && gpu_) {
    hip_ok(hipStreamSynchronize(cur_), "sync");
    hip_ok(hipMemcpy(dbg_before, red, 64, hipMemcpyDeviceToHost), "D2H");
  }
  if (world_ > 1) comm_->allreduce_min_i64(red, 8, (intptr_t)cur_);
  if (debug_exchange_ && gpu_) {
    int64_t after[8];
    hip_ok(hipStreamSynchronize(cur_), "sync");
    hip_ok(hipMemcpy(after, red, 64, hipMemcpyDeviceToHost), "D2H");
    std::fprintf(stderr, "[mxs front] rank %d world %d stream %p red3 %lld -> %lld red2 %lld -> %lld\n",
                 rank_, world_, (void*)cur_, (long long)dbg_before[3], (long long)after[3],
                 (long long)dbg_before[2], (long long)after[2]);
  }
  if (gpu_) {
    if (world_ > 1)
      hip_ok(hipMemcpyAsync(hred_[p]->p, red, kRedWords * 8, hipMemcpyDeviceToHost, cur_), "D2H");
    if (!ev_part_[p]) ev_part_[p] = new_event();
    record(ev_part_[p], cur_);
    f.ev = ev_part_[p];
  } else {
    std::memcpy(hred_[p]->p, red, kRedWords * 8);
    f.ev = nullptr;
  }
}

WindowStep::Back WindowStep::settle(Front& f) {
  // The step's host sync: overflow handling (redo), watermark and pane bookkeeping.
  const int64_t* host = nullptr;
  for (;;) {
    if (f.ev) host_wait(f.ev);
    host = P<int64_t>(hred_[f.par]);
    if (host[4] == -1)
      throw std::runtime_error("event timestamp outside the representable pane range "
                               "(more than 2^32 panes ahead of the watermark)");
    if (host[6]) throw std::runtime_error("keyed state table full: a key found no free slot (raise max_keys)");
    if (host[7]) throw std::invalid_argument("key ids -1 and -2 are reserved (the state tables' markers)");
    const int need_rw = -host[5] == 1 ? 2 : -host[5] == 2 ? 3 : rec_w_;
    if (host[4] < -1) {
      // Some rank's batch exceeds the capacity (word 4 = -(largest such batch << 1)): every
      // rank regrows to it -- the same bucket geometry everywhere -- and redoes the step.
      ++m_.bucket_regrows;
      alloc_buckets(std::max<int64_t>(batch_capacity_, (-host[4]) >> 1), slack_);
    } else if (need_rw > rec_w_) {
      // A record does not fit the format: wider records from now on.
      rec_w_ = need_rw;
      ++m_.compact_fallbacks;
    } else if (exchanging_ ? -host[3] >= ((int64_t)1 << 40) : host[3] != 0) {
      // A bucket overflowed somewhere: grow the fixed bucket capacity and redo the step. (With
      // the records exchange the word carries the largest fill over the ranks instead.)
      ++m_.bucket_regrows;
      alloc_buckets(batch_capacity_, slack_ * 2);
    } else {
      break;
    }
    drain_all();
    launch_front(f);
  }
  const int64_t qmax = -host[0], qmin = host[1];
  int64_t wm_global = host[2];
  if (wm_global == INT64_MAX) wm_global = f.old_wm;  // every partition idle: the watermark holds
  const int64_t* stv = host + 8;
  m_.num_records_in += f.n;
  m_.num_late_records_dropped += stv[kStatLate];
  if (cfg_.side_output_late && stv[kStatLate]) {
    const int64_t nl = std::min<int64_t>(stv[kStatLate], cfg_.late_capacity);
    std::vector<uint32_t> idx((size_t)nl);
    to_host_sync(idx.data(), late_idx_->p, nl * 4);
    late_side_.push_back(std::move(idx));
  }
  Back b;
  b.par = f.par;
  b.cpar = f.cpar;
  b.n = f.n;
  b.old_wm = f.old_wm;
  b.rw = f.rw;
  b.pane_base = f.pane_base;
  b.maxb = stv[kStatMaxBucket];
  b.fill = exchanging_ ? -host[3] : stv[kStatMaxBucket];
  b.accepted = stv[kStatAccepted];
  b.seq = m_.steps + 1;
  b.vecs = f.vecs;
  if (qmin <= qmax) {
    const int64_t gmin = f.pane_base + qmin, gmax = f.pane_base + qmax;
    const int64_t span = ctl_.live_span_with(gmin, gmax);
    if (span > ring_) grow_ring(span);
    // live range += [gmin, gmax]; the fire cursor moves back to the first not-yet-due window
    // holding new data (due windows receiving data re-fire)
    ctl_.observe(gmin, gmax, f.old_wm);
    b.fired_hi = ctl_.fired_hi();
    const int64_t cap = (int64_t)1 << cap_log2_;
    int64_t lds_budget = 150 * 1024 - cap * 8 - (dlist_ ? cap * 4 + cap / 8 + 16 : 0);
    b.has_data = true;
    b.qmin = qmin;
    b.np_step = gmax - gmin + 1;
    // Sparse pane rows: the aggregation visits only the panes that received records. Own
    // records only: the exchanged / combined paths keep the dense range.
    const uint32_t pm = (uint32_t)(stv[kStatPaneMask] & 0xFFFFFFFF);
    b.pmask = (pm && !(pm >> 31) && gpu_ && !exchanging_ && !combine_ && sparse_panes_) ? pm : 0u;
    b.np_act = b.pmask ? __builtin_popcount(b.pmask) : b.np_step;
    if (dense_bits_) lds_budget += cap * 8;  // no LDS key table for dense ids
    const int64_t per_pane = cfg_.deterministic ? 20 : (agg_pack_ok(b.rw) ? 8 : 12);
    b.pg = std::max<int64_t>(1, std::min<int64_t>(b.np_act, lds_budget / (cap * per_pane)));
    b.gmin = gmin;
    b.gmax = gmax;
  }
  ++m_.steps;
  if (!cfg_.external_watermark) {
    b.has_new_wm = true;
    b.new_wm = std::max(f.old_wm, wm_global);
    wm_ = b.new_wm;
    m_.current_watermark = b.new_wm;
  }
  return b;
}

bool WindowStep::agg_pack_ok(int rw) const {
  // Mirror of the launcher's packed (sum, count) LDS accumulator condition.
  int64_t per_wg = (int64_t)part_ranks_ * bucket_cap_;
  if (force_split_ > 1 && dense_bits_ && part_ranks_ == 1 && !dlist_)
    per_wg = (bucket_cap_ + force_split_ - 1) / force_split_;
  return (cfg_.agg == AGG_SUM_I64 || cfg_.agg == AGG_AVG_I64) && rw <= 2 && !combine_ &&
         per_wg < 65536 && agg_pack_env_;
}

// ---- state half --------------------------------------------------------------------------------
void WindowStep::back_begin(Back& b) {
  if (!b.has_data) return;
  if (gpu_ && ev_part_[b.par]) hip_ok(hipStreamWaitEvent(cur_, ev_part_[b.par], 0), "wait");
  if (combine_) {
    Stage stage(this, "combine");
    combine_begin(b);
  }
}

void WindowStep::back_finish(Back& b) {
  StreamScope sc(this, true);
  if (b.has_data) {
    const Rec* recs = exchanging_ ? P<Rec>(recv_) : P<Rec>(send_[b.par]);
    const uint32_t* counts = exchanging_ ? P<uint32_t>(recv_counts_) : P<uint32_t>(cursor_[b.cpar]);
    uint32_t bcap = (uint32_t)bucket_cap_;
    int combined = 0;
    if (combine_) {
      Stage stage(this, "all_to_all");
      combine_finish(b, &recs, &counts, &bcap);
      combined = 1;
    } else if (exchanging_) {
      Stage stage(this, "all_to_all");
      exchange_records(b, &bcap);
    }
    if (gpu_ && exchanging_) {
      if (!ev_consumed_[b.par]) ev_consumed_[b.par] = new_event();
      record(ev_consumed_[b.par], cur_);
    }
    const bool sparse = b.pmask && !combined;
    AggPlan ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.cap_log2 = cap_log2_;
    ap.nsub = nsub_;
    ap.ring = (int32_t)ring_;
    ap.agg = cfg_.agg;
    ap.nsrc = part_ranks_;
    ap.bucket_cap = bcap;
    ap.np_step = (int32_t)(sparse ? b.np_act : b.np_step);
    ap.pg = (int32_t)b.pg;
    ap.pane_base = b.pane_base;
    ap.p_lo = b.qmin;
    ap.fired_hi = b.fired_hi;
    ap.combined = combined;
    ap.rec_words = combined ? 3 : b.rw;
    ap.pmask = sparse ? b.pmask : 0u;
    ap.dense_bits = dense_bits_;
    ap.dense_mul = dense_mul_;
    ap.det = cfg_.deterministic ? 1 : 0;
    // Hot keys: a sub-table holding more than kAggSlice records is shared by several workgroups.
    ap.split = combined ? 1 : (int32_t)std::min<int64_t>(64, std::max<int64_t>(1, (b.maxb + kAggSlice - 1) / kAggSlice));
    if (force_split_ > 1 && ap.split == 1 && !combined) ap.split = -force_split_;
    if (dlist_) {
      ap.dlist = P<uint32_t>(dlist_);
      ap.dlist_n = P<uint32_t>(dlist_n_);
      ap.slot_mark = P<uint32_t>(slot_mark_);
    }
    if (dacc_g_) {
      ap.dacc = P<uint64_t>(dacc_g_);
      ap.dcnt = P<uint32_t>(dcnt_g_);
    }
    {
      Stage stage(this, "window_agg");
      aggregate(recs, counts, ap, &b);
    }
    if (gpu_ && !exchanging_) {
      if (!ev_consumed_[b.par]) ev_consumed_[b.par] = new_event();
      record(ev_consumed_[b.par], cur_);
    }
    if (debug_) check_table((intptr_t)cur_);
    // Late-but-allowed data: re-fire already-passed windows that are not cleaned yet.
    if (b.gmin <= b.fired_hi) {
      const int64_t fr = b.fired_hi - b.pane_base;
      if (b.pmask && fr >= 0 && fr < 31) {
        dirty_lo_ = b.pane_base;
        dirty_mask_ = b.pmask & (uint32_t)((1ull << (fr + 1)) - 1);
      } else {
        dirty_lo_ = 0;
        dirty_mask_ = 0;
      }
      refire(b.gmin, std::min(b.gmax, b.fired_hi), b.old_wm, b.seq);
      dirty_lo_ = 0;
      dirty_mask_ = 0;
    }
  }
  if (b.has_new_wm) {
    Stage stage(this, "fire");
    fire_ready(b.new_wm, b.seq);
    purge(b.new_wm);
  }
  if (tier_ && m_.steps % std::max(1, cfg_.spill_check_steps) == 0) maybe_spill();
}

void WindowStep::aggregate(const Rec* recs, const uint32_t* counts, AggPlan& ap, const Back* b) {
  if (ap.np_step > ap.ring) throw std::invalid_argument("step touches more panes than the ring holds");
  if (cfg_.dim > 0) {
    VecAggPlan vp;
    std::memset(&vp, 0, sizeof(vp));
    vp.cap_log2 = ap.cap_log2;
    vp.nsub = ap.nsub;
    vp.ring = (int32_t)ring_;
    vp.dim = cfg_.dim;
    vp.nsrc = ap.nsrc;
    vp.bucket_cap = ap.bucket_cap;
    vp.np_step = ap.np_step;
    vp.positional = world_ > 1 ? 1 : 0;
    vp.rec_words = ap.rec_words;
    vp.mode = cfg_.vec_mode;
    vp.pane_base = ap.pane_base;
    vp.p_lo = ap.p_lo;
    vp.fired_hi = ap.fired_hi;
    const float* vec = world_ > 1 ? P<float>(recv_vec_) : (b ? b->vecs : nullptr);
    if (gpu_)
      gpu::vec_window_agg(recs, counts, vp, vec, P<uint64_t>(keys_g_), P<float>(vacc_g_),
                          P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_), P<uint32_t>(occ_),
                          P<uint32_t>(flags_), (intptr_t)cur_);
    else
      cpu::vec_window_agg(recs, counts, vp, vec, P<uint64_t>(keys_g_), P<float>(vacc_g_),
                          P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_), P<uint32_t>(occ_),
                          P<uint32_t>(flags_));
    return;
  }
  if (gpu_)
    gpu::window_agg(recs, counts, ap, P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                    P<uint8_t>(dirty_g_), P<uint32_t>(occ_), P<uint32_t>(flags_), (intptr_t)cur_);
  else
    cpu::window_agg(recs, counts, ap, P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                    P<uint8_t>(dirty_g_), P<uint32_t>(occ_), P<uint32_t>(flags_));
}

void WindowStep::exchange_records(Back& b, uint32_t* xcap_out) {
  // G > 1 without the combiner: the buckets are repacked to a stride of the largest fill over
  // all ranks (all-reduced with the step's MIN vector), then ONE equal-split all-to-all moves
  // nbuckets x that stride records of rw words -- not the partition's fixed capacity (which
  // carries 1.5x slack): no padding crosses xGMI beyond the fill spread between buckets.
  const int rw = b.rw;
  const uint32_t xcap = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(b.fill, bucket_cap_));
  if (!xsend_) xsend_ = mem_alloc((size_t)nbuckets_ * bucket_cap_ * 24, gpu_ ? 1 : 0, false);
  if (gpu_)
    gpu::bucket_repack(P<uint64_t>(send_[b.par]), P<uint32_t>(cursor_[b.cpar]), nbuckets_,
                       (uint32_t)bucket_cap_, xcap, rw, P<uint64_t>(xsend_), nullptr, (intptr_t)cur_);
  else
    cpu::bucket_repack(P<uint64_t>(send_[b.par]), P<uint32_t>(cursor_[b.cpar]), nbuckets_,
                       (uint32_t)bucket_cap_, xcap, rw, P<uint64_t>(xsend_), nullptr);
  const int64_t words = (int64_t)nbuckets_ * xcap * rw;
  if (debug_exchange_)
    std::fprintf(stderr, "[mxs exchange] rank %d step %lld rw %d fill %lld bucket_cap %lld xcap %u "
                 "nbuckets %d words %lld\n", rank_, (long long)m_.steps, rw, (long long)b.fill,
                 (long long)bucket_cap_, xcap, nbuckets_, (long long)words);
  if (cfg_.dim > 0) {
    const int64_t need = (int64_t)nbuckets_ * xcap * cfg_.dim;
    if (!send_vec_ || (int64_t)send_vec_->bytes < need * 4) {
      send_vec_ = mem_alloc(need * 4, gpu_ ? 1 : 0);
      recv_vec_ = mem_alloc(need * 4, gpu_ ? 1 : 0);
    }
    if (gpu_)
      gpu::vec_gather(xsend_->p, rw, P<uint32_t>(cursor_[b.cpar]), nbuckets_, xcap, b.vecs,
                      cfg_.dim, P<float>(send_vec_), (intptr_t)cur_);
    else
      cpu::vec_gather(xsend_->p, rw, P<uint32_t>(cursor_[b.cpar]), nbuckets_, xcap, b.vecs,
                      cfg_.dim, P<float>(send_vec_));
    comm_->all_to_all(recv_vec_->p, send_vec_->p, need * 4, 4, (intptr_t)cur_);
    m_.a2a_bytes += need * 4;
    m_.payload_bytes += b.accepted * cfg_.dim * 4;
  }
  comm_->all_to_all(recv_->p, xsend_->p, words * 8, 8, (intptr_t)cur_);
  comm_->all_to_all(recv_counts_->p, cursor_[b.cpar]->p, (int64_t)nbuckets_ * 4, 4, (intptr_t)cur_);
  m_.a2a_bytes += words * 8;
  m_.payload_bytes += b.accepted * rw * 8;
  *xcap_out = xcap;
}

// ---- records exchange with the sender-side combiner -------------------------------------------
void WindowStep::combine_begin(Back& b) {
  // Pre-aggregate every send bucket to one record per (key, pane); the global overflow flag and
  // largest fill go through one small MIN all-reduce into pinned memory (read by combine_finish).
  const int64_t cap = (int64_t)1 << cap_log2_;
  const int64_t hard = std::min<int64_t>(bucket_cap_, cap * b.np_step);
  const int64_t ccap = std::min<int64_t>(hard, std::max<int64_t>(64, ((int64_t)ccap_hint_ + 7) & ~7));
  if (!comb_send_ || (int64_t)comb_send_->bytes < (int64_t)nbuckets_ * ccap * 24) {
    drain_all();
    comb_send_ = mem_alloc((size_t)nbuckets_ * ccap * 24, gpu_ ? 1 : 0, false);
    comb_recv_ = mem_alloc((size_t)nbuckets_ * ccap * 24, gpu_ ? 1 : 0, false);
  }
  memset_async(flags_, 0, 4, 4);
  AggPlan cp;
  std::memset(&cp, 0, sizeof(cp));
  cp.cap_log2 = cap_log2_;
  cp.nsub = nbuckets_;
  cp.ring = (int32_t)ring_;
  cp.agg = cfg_.agg;
  cp.nsrc = 1;
  cp.bucket_cap = (uint32_t)bucket_cap_;
  cp.np_step = (int32_t)b.np_step;
  cp.pg = (int32_t)b.pg;
  cp.p_lo = b.qmin;
  cp.rec_words = b.rw;
  cp.split = 1;
  // chk = [-(overflow bit), -(largest combined bucket)] (window_combine writes both)
  if (gpu_) {
    gpu::window_combine(P<Rec>(send_[b.par]), P<uint32_t>(cursor_[b.cpar]), nbuckets_, cp,
                        P<Rec>(comb_send_), (uint32_t)ccap, P<uint32_t>(comb_counts_),
                        P<uint32_t>(flags_) + 1, (intptr_t)cur_);
    gpu::combine_check(P<uint32_t>(flags_) + 1, P<uint32_t>(comb_counts_), nbuckets_,
                       P<int64_t>(chk_), (intptr_t)cur_);
  } else {
    cpu::window_combine(P<Rec>(send_[b.par]), P<uint32_t>(cursor_[b.cpar]), nbuckets_, cp,
                        P<Rec>(comb_send_), (uint32_t)ccap, P<uint32_t>(comb_counts_),
                        P<uint32_t>(flags_) + 1);
    const uint32_t* cc = P<uint32_t>(comb_counts_);
    uint32_t mx = 0;
    for (int i = 0; i < nbuckets_; ++i) mx = std::max(mx, cc[i]);
    int64_t sum = 0;
    for (int i = 0; i < nbuckets_; ++i) sum += cc[i];
    P<int64_t>(chk_)[0] = -(int64_t)(P<uint32_t>(flags_)[1] & 2u);
    P<int64_t>(chk_)[1] = -(int64_t)mx;
    P<int64_t>(chk_)[2] = sum;
  }
  if (world_ > 1) comm_->allreduce_min_i64(P<int64_t>(chk_), 2, (intptr_t)cur_);
  b.ccap = (uint32_t)ccap;
  b.hard = (uint32_t)hard;
  if (gpu_) {
    hip_ok(hipMemcpyAsync(hchk_->p, chk_->p, 24, hipMemcpyDeviceToHost, cur_), "D2H");
    if (!b.chk_ev) b.chk_ev = new_event();
    record(b.chk_ev, cur_);
  } else {
    std::memcpy(hchk_->p, chk_->p, 24);
    b.chk_ev = nullptr;
  }
}

void WindowStep::combine_finish(Back& b, const Rec** recs, const uint32_t** counts, uint32_t* bcap) {
  // The combined buckets cross ONE all-to-all at a stride of the largest combined fill over all
  // ranks: the all-reduced check (overflow bit, largest fill) is read first -- a short host wait
  // on the combine, while the next batch's partition keeps the GPU busy -- an overflow is redone
  // with twice the capacity right here, and the buckets are repacked to the fill (no padding
  // crosses xGMI beyond the fill spread between buckets).
  int64_t ovf = 0, fill = 0;
  for (;;) {
    if (b.chk_ev) host_wait(b.chk_ev);
    ovf = -P<int64_t>(hchk_)[0];
    fill = -P<int64_t>(hchk_)[1];
    if (!ovf) break;
    if (b.ccap >= b.hard)
      throw std::runtime_error("window_combine: a send bucket exceeds its sub-table capacity");
    ccap_hint_ = b.ccap * 2;
    ++m_.combine_regrows;
    combine_begin(b);
  }
  m_.payload_bytes += P<int64_t>(hchk_)[2] * 24;
  // next step's combined capacity: this step's global fill + 10 % (an overflow is redone above)
  ccap_hint_ = (uint32_t)std::max<int64_t>(64, (int64_t)(fill * 1.10) + 16);
  const uint32_t x = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(fill, b.ccap));
  if (!comb_x_ || comb_x_->bytes < (size_t)nbuckets_ * x * 24)
    comb_x_ = mem_alloc((size_t)nbuckets_ * b.ccap * 24, gpu_ ? 1 : 0, false);
  if (gpu_)
    gpu::bucket_repack(P<uint64_t>(comb_send_), P<uint32_t>(comb_counts_), nbuckets_, b.ccap, x, 3,
                       P<uint64_t>(comb_x_), nullptr, (intptr_t)cur_);
  else
    cpu::bucket_repack(P<uint64_t>(comb_send_), P<uint32_t>(comb_counts_), nbuckets_, b.ccap, x, 3,
                       P<uint64_t>(comb_x_), nullptr);
  const int64_t bytes = (int64_t)nbuckets_ * x * 24;
  comm_->all_to_all(comb_recv_->p, comb_x_->p, bytes, 8, (intptr_t)cur_);
  comm_->all_to_all(recv_counts_->p, comb_counts_->p, (int64_t)nbuckets_ * 4, 4, (intptr_t)cur_);
  m_.a2a_bytes += bytes;
  *recs = P<Rec>(comb_recv_);
  *counts = P<uint32_t>(recv_counts_);
  *bcap = x;
}

// ---- firing --------------------------------------------------------------------------------
void WindowStep::check_fire_flags(const uint32_t* hf) {
  if (hf[0] & 1u) throw std::runtime_error("keyed state table full: a key found no free slot (raise max_keys)");
  if (hf[0] & 8u)
    throw std::invalid_argument("deterministic f64 sum: a value is NaN, infinite or |x| >= 2^63");
}

uint32_t WindowStep::fired_count() {
  uint32_t hf[4];
  to_host_sync(hf, flags_->p, 16);
  check_fire_flags(hf);
  return hf[2];
}

void WindowStep::fire_ready(int64_t wm, int64_t seq) {
  const std::vector<int64_t> due = ctl_.take_due(wm);
  fire_list(due, false, seq);
}

void WindowStep::refire(int64_t pmin, int64_t pmax, int64_t old_wm, int64_t seq) {
  refire_cleared_ = false;
  fire_list(ctl_.refire_windows(pmin, pmax, old_wm), true, seq);
  if (dlist_ && refire_cleared_) {
    memset_async(dlist_n_, 0, 0, 4);  // the fused re-firing cleared the slots itself
  } else if (dlist_) {
    if (gpu_)
      gpu::dirty_clear(P<uint32_t>(dlist_), P<uint32_t>(dlist_n_), (uint32_t)nslots_, (int)ring_,
                       nslots_, P<uint8_t>(dirty_g_), P<uint32_t>(slot_mark_), pmin,
                       (int)(pmax - pmin + 1), (intptr_t)cur_, P<uint64_t>(dacc_g_),
                       P<uint32_t>(dcnt_g_));
    else
      cpu::dirty_clear(P<uint32_t>(dlist_), P<uint32_t>(dlist_n_), (uint32_t)nslots_, (int)ring_,
                       nslots_, P<uint8_t>(dirty_g_), P<uint32_t>(slot_mark_), pmin,
                       (int)(pmax - pmin + 1), P<uint64_t>(dacc_g_), P<uint32_t>(dcnt_g_));
    memset_async(dlist_n_, 0, 0, 4);
  } else {
    for (int64_t p = pmin; p <= pmax; ++p)
      memset_async(dirty_g_, 0, (size_t)((p & (ring_ - 1)) * nslots_), nslots_);
  }
}

void WindowStep::fire_list(const std::vector<int64_t>& starts, bool only_dirty, int64_t seq) {
  const bool batched = !local_global_ && !tier_ && cfg_.dim == 0;
  if (starts.size() > 1 && batched) {
    fire_many(starts, only_dirty, seq);
    return;
  }
  for (int64_t s : starts) fire_window(s, only_dirty, seq);
}

// Queue a firing whose rows stay on the device until the copy kernel moves them (row count read
// on the device): fixed words (flags [+ bounds]) first, then every column at capacity `cap`.
void WindowStep::queue_counted(FireBatch&& fb, const std::vector<std::pair<const void*, int>>& cols,
                               int64_t cap, const uint32_t* n_dev, bool with_bounds,
                               const uint32_t* bounds_dev, int nwin, hipEvent_t* busy) {
  D2HBatch bt;
  std::memset(&bt, 0, sizeof(bt));
  int64_t off = 0;
  auto add = [&](const void* src, int64_t bytes, int64_t esz) {
    if (bt.n >= kD2HMax) throw std::logic_error("queue_counted: too many copies");
    bt.c[bt.n].src = src;
    bt.c[bt.n].bytes = bytes;
    bt.c[bt.n].dst_off = off;
    bt.c[bt.n].esz = esz;
    ++bt.n;
    const int64_t o = off;
    off += (bytes + 255) & ~(int64_t)255;
    return o;
  };
  fb.flags_off = add(flags_->p, 16, 0);
  if (with_bounds) fb.bounds_off = add(bounds_dev, (((int64_t)nwin + 3) & ~(int64_t)3) * 4, 0);
  fb.ncap = cap;
  fb.ncols = (int)cols.size();
  for (size_t i = 0; i < cols.size(); ++i) {
    fb.col_esz[i] = cols[i].second;
    fb.col_off[i] = add(cols[i].first, cap * cols[i].second, cols[i].second);
  }
  fb.slab = take_slab((size_t)off);
  hipStream_t st = cur_;
  if (copy_) {
    // (an event can be recorded again once a wait on it has been enqueued)
    if (!ready_ev_) ready_ev_ = new_event();
    record(ready_ev_, cur_);
    hip_ok(hipStreamWaitEvent(copy_, ready_ev_, 0), "wait");
    st = copy_;
  }
  const int e = gpu::d2h_kernel(fb.slab->p, bt.c, bt.n, (intptr_t)st, n_dev, copy_ ? 64 : 1024);
  if (e != 0) throw std::runtime_error("gpu_d2h_counted failed (hipError " + std::to_string(e) + ")");
  fb.ev = new_event();
  record(fb.ev, st);
  if (busy) *busy = fb.ev;
  queue_.push_back(std::move(fb));
  // keep the event pool bounded: events of resolved batches are recycled in take()
}

void WindowStep::queue_sync(FireBatch&& fb, const std::vector<std::pair<const void*, int>>& cols,
                            int64_t n, std::vector<uint32_t> hb) {
  // Rows already counted on the host: one copy of the first n rows of every column.
  int64_t off = 0;
  std::vector<int64_t> offs;
  for (auto& c : cols) {
    offs.push_back(off);
    off += (n * c.second + 255) & ~(int64_t)255;
  }
  fb.slab = take_slab((size_t)std::max<int64_t>(off, 256));
  for (size_t i = 0; i < cols.size(); ++i) {
    if (gpu_)
      hip_ok(hipMemcpyAsync((char*)fb.slab->p + offs[i], cols[i].first, n * cols[i].second,
                            hipMemcpyDeviceToHost, cur_), "D2H");
    else
      std::memcpy((char*)fb.slab->p + offs[i], cols[i].first, n * cols[i].second);
    fb.col_off[i] = offs[i];
    fb.col_esz[i] = cols[i].second;
  }
  if (gpu_) hip_ok(hipStreamSynchronize(cur_), "sync");
  fb.ncols = (int)cols.size();
  fb.ncap = n;
  fb.ev = nullptr;
  fb.hb = std::move(hb);
  queue_.push_back(std::move(fb));
}

std::vector<FireRows> WindowStep::take(bool block) {
  std::vector<FireRows> out;
  while (!done_.empty()) {
    out.push_back(std::move(done_.front()));
    done_.pop_front();
  }
  while (!queue_.empty()) {
    FireBatch& fb = queue_.front();
    if (fb.ev) {
      if (!block && hipEventQuery(fb.ev) == hipErrorNotReady) break;
      host_wait(fb.ev);
      const uint32_t* hf = (const uint32_t*)((char*)fb.slab->p + fb.flags_off);
      check_fire_flags(hf);
      if (fb.bounds) {
        const uint32_t* hb = (const uint32_t*)((char*)fb.slab->p + fb.bounds_off);
        fb.hb.assign(hb, hb + fb.wins.size());
      } else {
        fb.hb.assign(1, hf[2]);
      }
    }
    const int64_t n = std::min<int64_t>(fb.hb.empty() ? 0 : fb.hb.back(), fb.ncap);
    if (n > 0) m_.num_records_out += n;
    int64_t lo = 0;
    for (size_t w = 0; w < fb.wins.size() && n > 0; ++w) {
      const int64_t hi = std::min<int64_t>(w < fb.hb.size() ? fb.hb[w] : n, n);
      if (hi > lo) {
        FireRows r;
        r.start = fb.wins[w];
        r.end = WindowControl::clamp64((__int128)fb.wins[w] + ctl_.size());
        r.refire = fb.only_dirty;
        r.kv = fb.kv;
        r.vec = fb.vec;
        r.seq = fb.seq;
        r.n = hi - lo;
        r.slab = fb.slab;
        const char* base = (const char*)fb.slab->p;
        r.keys = base + fb.col_off[0] + lo * fb.col_esz[0];
        if (fb.vec) {
          r.vecs = (const float*)(base + fb.col_off[1]) + lo * cfg_.dim;
          r.cnt = (const int32_t*)(base + fb.col_off[2]) + lo;
        } else {
          r.vals = (const double*)(base + fb.col_off[1]) + lo;
          if (!fb.kv) {
            r.raw = (const int64_t*)(base + fb.col_off[2]) + lo;
            r.cnt = (const int32_t*)(base + fb.col_off[3]) + lo;
          }
        }
        out.push_back(std::move(r));
      }
      lo = hi;
    }
    recycle(fb.ev);
    queue_.pop_front();
  }
  return out;
}

void WindowStep::fire_window(int64_t s, bool only_dirty, int64_t seq) {
  // Only panes inside the live span exist in the ring; older / newer panes of the window never
  // held data and their ring slots belong to other panes (aliasing).
  if (gpu_) claim_flags();
  const auto pr = ctl_.window_panes(s);
  const int64_t p0 = pr.first, p1 = pr.second;
  if (p1 < p0) return;
  if (cfg_.dim > 0) return fire_window_vector(s, p0, p1, only_dirty, seq);
  if (local_global_) return fire_window_partials(s, p0, p1, only_dirty, true, seq);
  if (tier_) {
    land_evictions();
    int64_t lo, hi;
    if (tier_->pane_range(&lo, &hi) && lo <= p1 && hi >= p0)
      return fire_window_tiered(s, p0, p1, only_dirty, seq);
  }
  memset_async(flags_, 0, 8, 4);  // out_n
  const bool kv = cfg_.emit_kv && dense_bits_;
  FirePlan fp;
  std::memset(&fp, 0, sizeof(fp));
  fp.agg = cfg_.agg;
  fp.npanes = (int32_t)(p1 - p0 + 1);
  fp.ring = (int32_t)ring_;
  fp.only_dirty = only_dirty ? 1 : 0;
  fp.nslots = nslots_;
  fp.p0 = p0;
  fp.wstart = (double)s;
  fp.wend = (double)s + (double)ctl_.size();
  fp.out_cap = (uint32_t)orows_;
  fp.map = cfg_.map;
  fp.filt = cfg_.filt;
  if (only_dirty && dlist_) {
    fp.list = P<uint32_t>(dlist_);
    fp.list_n = P<uint32_t>(dlist_n_);
  }
  fp.key32 = kv ? 1 : 0;
  uint32_t* on = P<uint32_t>(flags_) + 2;
  if (gpu_)
    gpu::window_fire(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                     P<uint8_t>(dirty_g_), fp, P<uint64_t>(out_keys_), P<double>(out_vals_),
                     kv ? nullptr : P<uint64_t>(out_raw_), kv ? nullptr : P<uint32_t>(out_cnt_), on,
                     (intptr_t)cur_);
  else
    cpu::window_fire(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                     P<uint8_t>(dirty_g_), fp, P<uint64_t>(out_keys_), P<double>(out_vals_),
                     kv ? nullptr : P<uint64_t>(out_raw_), kv ? nullptr : P<uint32_t>(out_cnt_), on);
  ++m_.num_fires;
  FireBatch fb;
  fb.wins = {s};
  fb.kv = kv;
  fb.only_dirty = only_dirty;
  fb.seq = seq;
  std::vector<std::pair<const void*, int>> cols;
  if (kv) cols = {{out_keys_->p, 4}, {out_vals_->p, 8}};
  else cols = {{out_keys_->p, 8}, {out_vals_->p, 8}, {out_raw_->p, 8}, {out_cnt_->p, 4}};
  if (async_fire_) {
    queue_counted(std::move(fb), cols, orows_, on, false, nullptr, 1, &out_busy_);
    return;
  }
  const uint32_t n = (uint32_t)std::min<int64_t>(fired_count(), orows_);
  if (n == 0) return;
  queue_sync(std::move(fb), cols, n, {n});
}

void WindowStep::fire_many(const std::vector<int64_t>& starts, bool only_dirty, int64_t seq) {
  // Batched firing: a group of due windows is evaluated by one native call (one fire launch per
  // window at a shared cursor, the cursor recorded after each window), then ONE copy of the
  // group's rows to a host slab -- a watermark jump over many slides (5 min / 5 s windows: 60 per
  // element) no longer costs two host round trips per window.
  const bool kv = cfg_.emit_kv && dense_bits_;
  FirePlan base;
  std::memset(&base, 0, sizeof(base));
  base.agg = cfg_.agg;
  base.npanes = 1;
  base.ring = (int32_t)ring_;
  base.only_dirty = only_dirty ? 1 : 0;
  base.nslots = nslots_;
  base.out_cap = (uint32_t)orows_;
  base.map = cfg_.map;
  base.filt = cfg_.filt;
  base.key32 = kv ? 1 : 0;
  if (only_dirty && dlist_) {
    base.list = P<uint32_t>(dlist_);
    base.list_n = P<uint32_t>(dlist_n_);
  }
  std::vector<int64_t> ws;
  std::vector<FireWin> wins;
  for (int64_t s : starts) {
    const auto pr = ctl_.window_panes(s);
    if (pr.second >= pr.first) {
      ws.push_back(s);
      FireWin w;
      w.p0 = pr.first;
      w.npanes = (int32_t)(pr.second - pr.first + 1);
      w.wstart = (double)s;
      w.wend = (double)s + (double)ctl_.size();
      if (w.npanes > base.ring) throw std::invalid_argument("window_fire_many: window panes exceed the ring");
      wins.push_back(w);
    }
  }
  if (gpu_ && only_dirty && dlist_ && wins.size() > 1 && wins.size() <= 32 && fused_refire_) {
    if (refire_fused(ws, wins, seq)) return;
  }
  if (gpu_ && !stage_[0]) {
    const int64_t n = orows_;
    stage_[0] = mem_alloc(n * 8, 1, false);
    stage_[1] = mem_alloc(n * 8, 1, false);
    stage_[2] = mem_alloc(n * 8, 1, false);
    stage_[3] = mem_alloc(n * 4, 1, false);
    stage_[4] = mem_alloc(std::max(fire_group_, 32) * 4, 1);
  }
  if (gpu_) claim_flags();
  const int g = fire_group_;
  for (size_t i = 0; i < wins.size(); i += g) {
    const int k = (int)std::min<size_t>(g, wins.size() - i);
    std::vector<int64_t> chunk(ws.begin() + i, ws.begin() + i + k);
    uint32_t* on = P<uint32_t>(flags_) + 2;
    uint32_t* bounds = P<uint32_t>(fire_bounds_);
    if (gpu_) {
      claim_flags();  // the previous chunk's copy may still read out_* and the flags
      FireStage st{P<uint64_t>(stage_[0]), P<double>(stage_[1]),
                   kv ? nullptr : P<uint64_t>(stage_[2]), kv ? nullptr : P<uint32_t>(stage_[3]),
                   P<uint32_t>(stage_[4]), (uint32_t)nslots_};
      gpu::window_fire_many(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                            P<uint8_t>(dirty_g_), base, wins.data() + i, k, st, P<uint64_t>(out_keys_),
                            P<double>(out_vals_), kv ? nullptr : P<uint64_t>(out_raw_),
                            kv ? nullptr : P<uint32_t>(out_cnt_), on, bounds, (intptr_t)cur_);
    } else {
      *on = 0;
      for (int j = 0; j < k; ++j) {
        FirePlan p = base;
        p.p0 = wins[i + j].p0;
        p.npanes = wins[i + j].npanes;
        p.wstart = wins[i + j].wstart;
        p.wend = wins[i + j].wend;
        cpu::window_fire(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                         P<uint8_t>(dirty_g_), p, P<uint64_t>(out_keys_), P<double>(out_vals_),
                         kv ? nullptr : P<uint64_t>(out_raw_), kv ? nullptr : P<uint32_t>(out_cnt_), on);
        bounds[j] = *on;
      }
    }
    m_.num_fires += k;
    FireBatch fb;
    fb.wins = chunk;
    fb.kv = kv;
    fb.only_dirty = only_dirty;
    fb.bounds = true;
    fb.seq = seq;
    std::vector<std::pair<const void*, int>> cols;
    if (kv) cols = {{out_keys_->p, 4}, {out_vals_->p, 8}};
    else cols = {{out_keys_->p, 8}, {out_vals_->p, 8}, {out_raw_->p, 8}, {out_cnt_->p, 4}};
    if (async_fire_) {
      queue_counted(std::move(fb), cols, orows_, bounds + (k - 1), true, bounds, k, &out_busy_);
      continue;
    }
    std::vector<uint32_t> hb((size_t)k);
    uint32_t hf[4];
    to_host_sync(hf, flags_->p, 16);
    to_host_sync(hb.data(), bounds, (size_t)k * 4);
    check_fire_flags(hf);
    const int64_t n = std::min<int64_t>(hb.back(), orows_);
    if (n == 0) continue;
    queue_sync(std::move(fb), cols, n, std::move(hb));
  }
}

bool WindowStep::refire_fused(const std::vector<int64_t>& starts, const std::vector<FireWin>& wins,
                              int64_t seq) {
  // Every re-fired window of the step in ONE pass over the touched-slot list (each listed slot's
  // union of panes loaded once), packed in window order into the re-firing's own output columns
  // and copied on the copy stream. The touched-slot count is read first (one small wait on the
  // aggregation): each window's staging region is sized to it.
  const int k = (int)wins.size();
  const bool kv = cfg_.emit_kv && dense_bits_;
  // Staging regions sized for the whole slot table (the list never exceeds it) when the two
  // buffer sets fit the budget: no host wait on the aggregation for the list length (a ~0.1 ms
  // GPU bubble per re-firing step in config 4); past the budget, the count is read first.
  const int64_t full = ((int64_t)nslots_ + 3) & ~(int64_t)3;
  const int64_t row_bytes = kv ? 16 : 28;
  int64_t region = full;
  if ((int64_t)k * full * row_bytes * 2 > refire_stage_budget_) {
    uint32_t n_list = 0;
    to_host_sync(&n_list, dlist_n_->p, 4);
    if (n_list == 0) {
      m_.num_fires += k;
      return true;
    }
    region = ((int64_t)n_list + 3) & ~(int64_t)3;
  }
  const int64_t rows_cap = k * region;
  claim_flags();  // earlier copies read the staging / columns and the flags
  if (!rout_[0] || rout_cap_ < rows_cap || rout_kv_ != kv) {
    const int64_t cap = std::max<int64_t>(rows_cap, 1 << 16);
    for (int j = 0; j < 2; ++j) {
      rout_[4 * j + 0] = mem_alloc(cap * 8, 1, false);
      rout_[4 * j + 1] = mem_alloc(cap * 8, 1, false);
      rout_[4 * j + 2] = kv ? nullptr : mem_alloc(cap * 8, 1, false);
      rout_[4 * j + 3] = kv ? nullptr : mem_alloc(cap * 4, 1, false);
    }
    rout_[8] = mem_alloc(32 * 4, 1);
    rout_[9] = mem_alloc(36 * 4, 1);
    rout_cap_ = cap;
    rout_kv_ = kv;
  }
  FirePlan base;
  std::memset(&base, 0, sizeof(base));
  base.agg = cfg_.agg;
  base.npanes = 1;
  base.ring = (int32_t)ring_;
  base.only_dirty = 1;
  base.nslots = nslots_;
  base.out_cap = (uint32_t)orows_;
  base.map = cfg_.map;
  base.filt = cfg_.filt;
  base.key32 = kv ? 1 : 0;
  base.list = P<uint32_t>(dlist_);
  base.list_n = P<uint32_t>(dlist_n_);
  // The re-firing clears the listed slots' dirty bytes and marks itself (no dirty_clear launch;
  // the fused path runs only without the local-global delta ring, which dirty_clear also resets)
  base.clear_mark = dacc_g_ ? nullptr : P<uint32_t>(slot_mark_);
  FireStage st{P<uint64_t>(rout_[0]), P<double>(rout_[1]), P<uint64_t>(rout_[2]),
               P<uint32_t>(rout_[3]), P<uint32_t>(rout_[8]), (uint32_t)region};
  uint32_t* bnd = P<uint32_t>(rout_[9]);
  memset_async(flags_, 0, 12, 4);
  const bool ok = gpu::window_refire_many(
      P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_), base,
      wins.data(), k, st, P<uint64_t>(rout_[4]), P<double>(rout_[5]), P<uint64_t>(rout_[6]),
      P<uint32_t>(rout_[7]), bnd + 32, bnd, P<uint32_t>(flags_) + 3, (intptr_t)cur_, dirty_lo_,
      dirty_mask_);
  if (!ok) return false;
  refire_cleared_ = base.clear_mark != nullptr;
  FireBatch fb;
  fb.wins = starts;
  fb.kv = kv;
  fb.only_dirty = true;
  fb.bounds = true;
  fb.seq = seq;
  std::vector<std::pair<const void*, int>> cols;
  if (kv) cols = {{rout_[4]->p, 4}, {rout_[5]->p, 8}};
  else cols = {{rout_[4]->p, 8}, {rout_[5]->p, 8}, {rout_[6]->p, 8}, {rout_[7]->p, 4}};
  queue_counted(std::move(fb), cols, rows_cap, bnd + (k - 1), true, bnd, k, &rout_busy_);
  m_.num_fires += k;
  return true;
}

void WindowStep::fire_window_partials(int64_t s, int64_t p0, int64_t p1, bool only_dirty,
                                      bool emit, int64_t seq) {
  // Local-global fire of window [s, s + size): local partials -> owner -> emit.
  //  1. local fire without epilogue: one row (key, partial acc, count) per local key with data
  //     in the window; a re-firing reads the delta ring of the late data instead (listed slots);
  //  2. scatter_partials: rows -> combined records in (owner rank, owner sub-table) buckets;
  //  3. ONE equal-split all-to-all of the buckets (+ their counts);
  //  4. the owner folds the G partials per key into the window's merge slice (window_agg,
  //     combined records; a first fire resets the slice, a re-firing adds the deltas) and fires
  //     it with the fused map/filter epilogue. The slice lives until the window is cleaned.
  const bool delta = only_dirty && dacc_g_;
  memset_async(part_n_, 0, 0, 4);
  FirePlan fp;
  std::memset(&fp, 0, sizeof(fp));
  fp.agg = cfg_.agg;
  fp.npanes = (int32_t)(p1 - p0 + 1);
  fp.ring = (int32_t)ring_;
  fp.only_dirty = only_dirty ? 1 : 0;
  fp.nslots = nslots_;
  fp.p0 = p0;
  fp.wstart = (double)s;
  fp.wend = (double)s + (double)ctl_.size();
  fp.out_cap = (uint32_t)orows_;
  if (only_dirty && dlist_) {
    fp.list = P<uint32_t>(dlist_);
    fp.list_n = P<uint32_t>(dlist_n_);
  }
  const uint64_t* acc = delta ? P<uint64_t>(dacc_g_) : P<uint64_t>(acc_g_);
  const uint32_t* cnt = delta ? P<uint32_t>(dcnt_g_) : P<uint32_t>(cnt_g_);
  if (gpu_)
    gpu::window_fire(P<uint64_t>(keys_g_), acc, cnt, P<uint8_t>(dirty_g_), fp, P<uint64_t>(out_keys_),
                     P<double>(out_vals_), P<uint64_t>(out_raw_), P<uint32_t>(out_cnt_),
                     P<uint32_t>(part_n_), (intptr_t)cur_);
  else
    cpu::window_fire(P<uint64_t>(keys_g_), acc, cnt, P<uint8_t>(dirty_g_), fp, P<uint64_t>(out_keys_),
                     P<double>(out_vals_), P<uint64_t>(out_raw_), P<uint32_t>(out_cnt_),
                     P<uint32_t>(part_n_));
  const uint64_t* pk = P<uint64_t>(out_keys_);
  const uint64_t* pa = P<uint64_t>(out_raw_);
  const uint32_t* pc = P<uint32_t>(out_cnt_);
  int64_t n_cap = orows_;
  if (!delta && tier_) {
    land_evictions();
    int64_t lo, hi;
    if (tier_->pane_range(&lo, &hi) && lo <= p1 && hi >= p0) {
      // spilled keys: this rank's tier rows of the window join its local partials
      tier_combine(P<uint32_t>(part_n_), 0, 0, p0, p1);
      memset_async(part_n_, 0, 0, 4);
      FirePlan tp = fp;
      tp.npanes = 1;
      tp.ring = 1;
      tp.p0 = 0;
      tp.only_dirty = 0;
      tp.list = nullptr;
      tp.list_n = nullptr;
      tp.nslots = tt_size_;
      tp.out_cap = (uint32_t)(tt_size_ / 2);
      if (gpu_)
        gpu::window_fire(P<uint64_t>(tt_[0]), P<uint64_t>(tt_[1]), P<uint32_t>(tt_[2]),
                         P<uint8_t>(tt_[3]), tp, P<uint64_t>(tt_[4]), P<double>(tt_[5]),
                         P<uint64_t>(tt_[6]), P<uint32_t>(tt_[7]), P<uint32_t>(part_n_), (intptr_t)cur_);
      else
        cpu::window_fire(P<uint64_t>(tt_[0]), P<uint64_t>(tt_[1]), P<uint32_t>(tt_[2]),
                         P<uint8_t>(tt_[3]), tp, P<uint64_t>(tt_[4]), P<double>(tt_[5]),
                         P<uint64_t>(tt_[6]), P<uint32_t>(tt_[7]), P<uint32_t>(part_n_));
      pk = P<uint64_t>(tt_[4]);
      pa = P<uint64_t>(tt_[6]);
      pc = P<uint32_t>(tt_[7]);
      n_cap = tt_size_ / 2;
    }
  }
  memset_async(fcursor_, 0, 0, fcursor_->bytes);
  ScatPlan sp{};
  sp.max_parallelism = cfg_.max_parallelism;
  sp.nranks = world_;
  sp.nsub_log2 = nsub_o_log2_;
  sp.hash_mode = cfg_.hash_mode;
  sp.bucket_cap = (uint32_t)fbcap_;
  sp.n_cap = (uint32_t)n_cap;
  if (gpu_)
    gpu::scatter_partials(pk, pa, pc, P<uint32_t>(part_n_), sp, cfg_.jhash, P<int32_t>(kg_dest_),
                          P<uint32_t>(fcursor_), P<Rec>(fsend_), P<uint32_t>(flags_), (intptr_t)cur_);
  else
    cpu::scatter_partials(pk, pa, pc, P<uint32_t>(part_n_), sp, cfg_.jhash, P<int32_t>(kg_dest_),
                          P<uint32_t>(fcursor_), P<Rec>(fsend_), P<uint32_t>(flags_));
  // The owners' buckets hold at most one row per key of an owner sub-table (fbcap = its slot
  // count); the all-to-all moves a stride of the largest fill over the ranks instead (one
  // 1-word MIN all-reduce and a host read per fired window), repacked on the device.
  const int nbf = world_ << nsub_o_log2_;
  if (gpu_) {
    gpu::neg_max_u32(P<uint32_t>(fcursor_), nbf, P<int64_t>(fmax_), (intptr_t)cur_);
    hip_ok(hipMemcpyAsync(P<int64_t>(fmax_) + 1, part_n_->p, 4, hipMemcpyDeviceToDevice, cur_), "D2D");
  } else {
    const uint32_t* fc = P<uint32_t>(fcursor_);
    uint32_t mx = 0;
    for (int i = 0; i < nbf; ++i) mx = std::max(mx, fc[i]);
    P<int64_t>(fmax_)[0] = -(int64_t)mx;
    P<int64_t>(fmax_)[1] = *P<uint32_t>(part_n_);
  }
  comm_->allreduce_min_i64(P<int64_t>(fmax_), 1, (intptr_t)cur_);
  int64_t hx[2];
  to_host_sync(hx, fmax_->p, 16);
  const uint32_t fx = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(-hx[0], fbcap_));
  if (gpu_)
    gpu::bucket_repack(P<uint64_t>(fsend_), P<uint32_t>(fcursor_), nbf, (uint32_t)fbcap_, fx, 3,
                       P<uint64_t>(fxsend_), nullptr, (intptr_t)cur_);
  else
    cpu::bucket_repack(P<uint64_t>(fsend_), P<uint32_t>(fcursor_), nbf, (uint32_t)fbcap_, fx, 3,
                       P<uint64_t>(fxsend_), nullptr);
  comm_->all_to_all(frecv_->p, fxsend_->p, (int64_t)nbf * fx * 24, 8, (intptr_t)cur_);
  comm_->all_to_all(frecv_counts_->p, fcursor_->p, (int64_t)nbf * 4, 4, (intptr_t)cur_);
  m_.a2a_bytes += (int64_t)nbf * fx * 24;
  m_.payload_bytes += (hx[1] & 0xFFFFFFFF) * 24;
  const int64_t widx = WindowControl::fdiv((__int128)s - cfg_.offset, cfg_.slide);
  const int64_t so = (widx & (ring_m_ - 1)) * nslots_o_;
  if (!only_dirty) {  // the slice's previous window is cleaned: reuse it
    memset_async(acc_m_, 0, so * 8, nslots_o_ * 8);
    memset_async(cnt_m_, 0, so * 4, nslots_o_ * 4);
    memset_async(dirty_m_, 0, so, nslots_o_);
  }
  AggPlan mp;
  std::memset(&mp, 0, sizeof(mp));
  mp.cap_log2 = cap_log2_o_;
  mp.nsub = nsub_o_;
  mp.ring = (int32_t)ring_m_;
  mp.agg = cfg_.agg;
  mp.nsrc = world_;
  mp.bucket_cap = fx;
  mp.np_step = 1;
  mp.pg = 1;
  mp.pane_base = widx;
  mp.p_lo = 0;
  mp.fired_hi = only_dirty ? widx : INT64_MIN;
  mp.combined = 1;
  mp.rec_words = 3;
  mp.det = cfg_.deterministic ? 1 : 0;
  mp.split = 1;
  if (gpu_)
    gpu::window_agg(P<Rec>(frecv_), P<uint32_t>(frecv_counts_), mp, P<uint64_t>(keys_m_),
                    P<uint64_t>(acc_m_), P<uint32_t>(cnt_m_), P<uint8_t>(dirty_m_), P<uint32_t>(occ_m_),
                    P<uint32_t>(flags_), (intptr_t)cur_);
  else
    cpu::window_agg(P<Rec>(frecv_), P<uint32_t>(frecv_counts_), mp, P<uint64_t>(keys_m_),
                    P<uint64_t>(acc_m_), P<uint32_t>(cnt_m_), P<uint8_t>(dirty_m_), P<uint32_t>(occ_m_),
                    P<uint32_t>(flags_));
  if (!emit) return;  // restore: rebuild the merged value of an already fired window
  memset_async(flags_, 0, 8, 4);
  FirePlan op;
  std::memset(&op, 0, sizeof(op));
  op.agg = cfg_.agg;
  op.npanes = 1;
  op.ring = (int32_t)ring_m_;
  op.only_dirty = only_dirty ? 1 : 0;
  op.nslots = nslots_o_;
  op.p0 = widx;
  op.wstart = (double)s;
  op.wend = (double)s + (double)ctl_.size();
  op.out_cap = (uint32_t)orows_;
  op.map = cfg_.map;
  op.filt = cfg_.filt;
  uint32_t* on = P<uint32_t>(flags_) + 2;
  if (gpu_)
    gpu::window_fire(P<uint64_t>(keys_m_), P<uint64_t>(acc_m_), P<uint32_t>(cnt_m_),
                     P<uint8_t>(dirty_m_), op, P<uint64_t>(out_keys_), P<double>(out_vals_),
                     P<uint64_t>(out_raw_), P<uint32_t>(out_cnt_), on, (intptr_t)cur_);
  else
    cpu::window_fire(P<uint64_t>(keys_m_), P<uint64_t>(acc_m_), P<uint32_t>(cnt_m_),
                     P<uint8_t>(dirty_m_), op, P<uint64_t>(out_keys_), P<double>(out_vals_),
                     P<uint64_t>(out_raw_), P<uint32_t>(out_cnt_), on);
  if (only_dirty) memset_async(dirty_m_, 0, so, nslots_o_);
  ++m_.num_fires;
  maybe_compact_merge();
  FireBatch fb;
  fb.wins = {s};
  fb.only_dirty = only_dirty;
  fb.seq = seq;
  std::vector<std::pair<const void*, int>> cols = {
      {out_keys_->p, 8}, {out_vals_->p, 8}, {out_raw_->p, 8}, {out_cnt_->p, 4}};
  if (async_fire_) {
    queue_counted(std::move(fb), cols, orows_, on, false, nullptr, 1, &out_busy_);
    return;
  }
  const uint32_t n = (uint32_t)std::min<int64_t>(fired_count(), orows_);
  if (n == 0) return;
  queue_sync(std::move(fb), cols, n, {n});
}

void WindowStep::maybe_compact_merge() {
  // The owner's merge table keeps a key while any merge slice (a fired window inside its allowed
  // lateness) holds a value for it. Keys whose slices were all recycled are dead; with a
  // drifting key space they would fill the table, so every 16 partial fires the fullest
  // sub-table is checked and, above 0.6 load, window_compact drops the dead keys and rehashes
  // the live ones with their slices (every ring position is a "live pane"; nothing is evicted).
  if (++mfires_ % 16) return;
  std::vector<uint32_t> occ((size_t)nsub_o_);
  to_host_sync(occ.data(), occ_m_->p, (size_t)nsub_o_ * 4);
  const uint32_t mx = occ.empty() ? 0 : *std::max_element(occ.begin(), occ.end());
  if (mx <= 0.6 * (double)((int64_t)1 << cap_log2_o_)) return;
  Buf ctr = mem_alloc(16, gpu_ ? 1 : 0);
  Buf dummy = mem_alloc(64, gpu_ ? 1 : 0);
  CompactOut o{};
  o.key = P<uint64_t>(dummy);
  o.pane = P<int64_t>(dummy);
  o.acc = P<uint64_t>(dummy);
  o.cnt = P<uint32_t>(dummy);
  o.dirty = P<uint8_t>(dummy);
  o.n = P<uint32_t>(ctr) + 3;
  o.cap = 1;
  o.counters = P<uint32_t>(ctr);
  if (gpu_)
    gpu::window_compact(P<uint64_t>(keys_m_), P<uint64_t>(acc_m_), P<uint32_t>(cnt_m_),
                        P<uint8_t>(dirty_m_), nsub_o_, cap_log2_o_, (int)ring_m_, 0, (int)ring_m_,
                        INT64_MIN, o, P<uint32_t>(occ_m_), (intptr_t)cur_);
  else
    cpu::window_compact(P<uint64_t>(keys_m_), P<uint64_t>(acc_m_), P<uint32_t>(cnt_m_),
                        P<uint8_t>(dirty_m_), nsub_o_, cap_log2_o_, (int)ring_m_, 0, (int)ring_m_,
                        INT64_MIN, o, P<uint32_t>(occ_m_));
  uint32_t hc[4];
  to_host_sync(hc, ctr->p, 16);
  if (hc[2]) throw std::runtime_error("merge table compaction: live keys do not fit");
  ++m_.merge_compactions;
}

void WindowStep::fire_window_vector(int64_t s, int64_t p0, int64_t p1, bool only_dirty, int64_t seq) {
  memset_async(flags_, 0, 8, 4);
  VecFirePlan vp;
  std::memset(&vp, 0, sizeof(vp));
  vp.dim = cfg_.dim;
  vp.npanes = (int32_t)(p1 - p0 + 1);
  vp.ring = (int32_t)ring_;
  vp.only_dirty = only_dirty ? 1 : 0;
  vp.nslots = nslots_;
  vp.p0 = p0;
  vp.avg = cfg_.vec_avg ? 1 : 0;
  vp.use_thr = cfg_.vec_has_threshold ? 1 : 0;
  vp.thr = (float)cfg_.vec_threshold;
  vp.out_cap = (uint32_t)nslots_;
  uint32_t* on = P<uint32_t>(flags_) + 2;
  if (gpu_)
    gpu::vec_window_fire(P<uint64_t>(keys_g_), P<float>(vacc_g_), P<uint32_t>(cnt_g_),
                         P<uint8_t>(dirty_g_), vp, P<uint64_t>(out_keys_), P<float>(out_vec_),
                         P<uint32_t>(out_cnt_), on, (intptr_t)cur_);
  else
    cpu::vec_window_fire(P<uint64_t>(keys_g_), P<float>(vacc_g_), P<uint32_t>(cnt_g_),
                         P<uint8_t>(dirty_g_), vp, P<uint64_t>(out_keys_), P<float>(out_vec_),
                         P<uint32_t>(out_cnt_), on);
  const uint32_t n = (uint32_t)std::min<int64_t>(fired_count(), nslots_);
  ++m_.num_fires;
  if (n == 0) return;
  FireBatch fb;
  fb.wins = {s};
  fb.vec = true;
  fb.only_dirty = only_dirty;
  fb.seq = seq;
  // keys (8), vectors (dim f32 per row), counts (4)
  int64_t off = 0;
  const int64_t ok = off;
  off += ((int64_t)n * 8 + 255) & ~(int64_t)255;
  const int64_t ov = off;
  off += ((int64_t)n * cfg_.dim * 4 + 255) & ~(int64_t)255;
  const int64_t oc = off;
  off += ((int64_t)n * 4 + 255) & ~(int64_t)255;
  fb.slab = take_slab((size_t)off);
  auto cp = [&](int64_t o, const void* src, size_t bytes) {
    if (gpu_) hip_ok(hipMemcpyAsync((char*)fb.slab->p + o, src, bytes, hipMemcpyDeviceToHost, cur_), "D2H");
    else std::memcpy((char*)fb.slab->p + o, src, bytes);
  };
  cp(ok, out_keys_->p, (size_t)n * 8);
  cp(ov, out_vec_->p, (size_t)n * cfg_.dim * 4);
  cp(oc, out_cnt_->p, (size_t)n * 4);
  if (gpu_) hip_ok(hipStreamSynchronize(cur_), "sync");
  fb.col_off[0] = ok;
  fb.col_off[1] = ov;
  fb.col_off[2] = oc;
  fb.col_esz[0] = 8;
  fb.col_esz[1] = cfg_.dim * 4;
  fb.col_esz[2] = 4;
  fb.ncols = 3;
  fb.ncap = n;
  fb.hb = {n};
  queue_.push_back(std::move(fb));
}

void WindowStep::zero_panes(int64_t r, int64_t k) {
  // Reset k consecutive pane slabs starting at ring position r (pane-major state).
  const size_t so = (size_t)(r * nslots_), ns = (size_t)(k * nslots_);
  if (gpu_) {  // one launch for the three slabs
    if (cfg_.dim > 0) gpu::zero_panes(vacc_g_->p, cfg_.dim * 4, P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_), so, ns, (intptr_t)cur_);
    else gpu::zero_panes(acc_g_->p, 8, P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_), so, ns, (intptr_t)cur_);
    return;
  }
  if (cfg_.dim > 0) memset_async(vacc_g_, 0, so * cfg_.dim * 4, ns * cfg_.dim * 4);
  else memset_async(acc_g_, 0, so * 8, ns * 8);
  memset_async(cnt_g_, 0, so * 4, ns * 4);
  memset_async(dirty_g_, 0, so, ns);
}

void WindowStep::purge(int64_t wm) {
  if (!ctl_.has_live()) return;
  // keep_from: first pane of the earliest window not cleaned; panes [p, stop) are zeroed (at
  // most one ring of them)
  const auto r = ctl_.purge_range(wm, ring_);
  if (tier_) {
    land_evictions();
    tier_->purge(r.keep_from);
  }
  int64_t p = r.from;
  const int64_t stop = r.stop;
  while (p < stop) {  // at most two runs of consecutive ring positions (wrap-around)
    const int64_t rp = p & (ring_ - 1);
    const int64_t k = std::min(stop - p, ring_ - rp);
    zero_panes(rp, k);
    p += k;
  }
  ctl_.commit_purge(r.keep_from);
}

// ---- host-DRAM spill tier ------------------------------------------------------------------------
void WindowStep::maybe_spill() {
  const int64_t cap = (int64_t)1 << cap_log2_;
  std::vector<uint32_t> occ((size_t)nsub_);
  to_host_sync(occ.data(), occ_->p, (size_t)nsub_ * 4);
  const int64_t o = occ.empty() ? 0 : *std::max_element(occ.begin(), occ.end());
  // Compact above spill_load, or earlier when the fullest sub-table's growth since the last
  // check (twice over) would fill it first.
  const int64_t prev = occ_prev_;
  occ_prev_ = o;
  const int64_t growth = prev >= 0 ? std::max<int64_t>(0, o - prev) : 0;
  if (!ctl_.has_live() || (o <= cfg_.spill_load * cap && o + 2 * growth <= 0.95 * cap)) return;
  const int64_t keep = cfg_.spill_keep_panes > 0 ? cfg_.spill_keep_panes : ctl_.panes_per_window();
  compact_state(true, ctl_.max_seen() - keep, false, (intptr_t)cur_);
  occ_prev_ = -1;  // the compacted occupancy is not read back (asynchronous)
}

std::vector<int64_t> WindowStep::compact_state(bool has_cutoff, int64_t cutoff_pane, bool wait,
                                               intptr_t stream) {
  // Drop keys without live data and (with the spill tier) move keys whose newest data pane is
  // <= cutoff_pane to host DRAM. wait = false (the spill check inside a step, GPU): the evicted
  // rows go to a pinned slab by the counted copy kernel on the copy stream, with no host sync;
  // the tier absorbs them at the next point that reads it (land_evictions).
  if (stream) cur_ = (hipStream_t)stream;
  if (dense_bits_) return {0, 0, 0};
  if (has_cutoff && !tier_) throw std::invalid_argument("evicting keys needs the spill tier (spill=True)");
  land_evictions();
  drain_all();
  int64_t p_lo = 0, np = 0;
  if (ctl_.has_live()) {
    p_lo = ctl_.min_live();
    np = std::min<int64_t>(ring_, ctl_.max_seen() - ctl_.min_live() + 1);
  }
  const int64_t cutoff = has_cutoff ? cutoff_pane : INT64_MIN;
  const bool async = gpu_ && !wait && copy_ && tier_;
  int64_t rows_cap;
  if (cutoff == INT64_MIN) {
    rows_cap = 1;
  } else if (async) {
    rows_cap = (nslots_ * std::max<int64_t>(np, 1) + 15) & ~(int64_t)15;
  } else {
    std::vector<uint32_t> occ((size_t)nsub_);
    to_host_sync(occ.data(), occ_->p, (size_t)nsub_ * 4);
    int64_t tot = 0;
    for (uint32_t x : occ) tot += x;
    rows_cap = std::max<int64_t>(1, tot * std::max<int64_t>(np, 1));
  }
  const int dk = gpu_ ? 1 : 0;
  if (!sp_key_ || sp_cap_ < rows_cap) {
    sp_key_ = mem_alloc(rows_cap * 8, dk, false);
    sp_pane_ = mem_alloc(rows_cap * 8, dk, false);
    sp_acc_ = mem_alloc(rows_cap * 8, dk, false);
    sp_cnt_ = mem_alloc(rows_cap * 4, dk, false);
    sp_dirty_ = mem_alloc(rows_cap, dk, false);
    sp_ctr_ = mem_alloc(16, dk);
    sp_skey_ = nullptr;
    sp_cap_ = rows_cap;
  }
  if (async && evict_busy_) claim(&evict_busy_);  // the last copy read the rows
  memset_async(sp_ctr_, 0, 0, 16);
  CompactOut o{};
  o.key = P<uint64_t>(sp_key_);
  o.pane = P<int64_t>(sp_pane_);
  o.acc = P<uint64_t>(sp_acc_);
  o.cnt = P<uint32_t>(sp_cnt_);
  o.dirty = P<uint8_t>(sp_dirty_);
  o.n = P<uint32_t>(sp_ctr_) + 3;
  o.cap = (uint32_t)sp_cap_;
  o.counters = P<uint32_t>(sp_ctr_);
  if (gpu_)
    gpu::window_compact(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                        P<uint8_t>(dirty_g_), nsub_, cap_log2_, (int)ring_, p_lo, (int)np, cutoff,
                        o, P<uint32_t>(occ_), (intptr_t)cur_);
  else
    cpu::window_compact(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_),
                        P<uint8_t>(dirty_g_), nsub_, cap_log2_, (int)ring_, p_lo, (int)np, cutoff,
                        o, P<uint32_t>(occ_));
  if (async) {
    const int64_t ncap = sp_cap_;
    std::unique_ptr<Eviction> ev(new Eviction());
    D2HBatch bt;
    std::memset(&bt, 0, sizeof(bt));
    int64_t off = 0;
    auto add = [&](const void* src, int64_t bytes, int64_t esz) {
      bt.c[bt.n].src = src;
      bt.c[bt.n].bytes = bytes;
      bt.c[bt.n].dst_off = off;
      bt.c[bt.n].esz = esz;
      ++bt.n;
      const int64_t r = off;
      off += (bytes + 255) & ~(int64_t)255;
      return r;
    };
    ev->ctr_off = add(sp_ctr_->p, 16, 0);
    ev->cap = ncap;
    if (evict_pane_sort_ && np > 0 && np <= 64) {
      // Rows grouped by pane on the device: the tier takes them with memcpy instead of a host
      // counting sort (csrc/window_tier.h absorb_presorted).
      if (!sp_skey_) {
        sp_skey_ = mem_alloc(ncap * 8, 1, false);
        sp_sacc_ = mem_alloc(ncap * 8, 1, false);
        sp_scnt_ = mem_alloc(ncap * 4, 1, false);
        sp_sdirty_ = mem_alloc(ncap, 1, false);
        sp_pcount_ = mem_alloc(128 * 4, 1);
      }
      gpu::window_rows_pane_sort(P<uint64_t>(sp_key_), P<int64_t>(sp_pane_), P<uint64_t>(sp_acc_),
                                 P<uint32_t>(sp_cnt_), P<uint8_t>(sp_dirty_), P<uint32_t>(sp_ctr_) + 3,
                                 (uint32_t)ncap, p_lo, (int)np, P<uint64_t>(sp_skey_),
                                 P<uint64_t>(sp_sacc_), P<uint32_t>(sp_scnt_), P<uint8_t>(sp_sdirty_),
                                 P<uint32_t>(sp_pcount_), (intptr_t)cur_);
      ev->pc_off = add(sp_pcount_->p, 128 * 4, 0);
      ev->off[0] = add(sp_skey_->p, ncap * 8, 8);
      ev->off[1] = add(sp_sacc_->p, ncap * 8, 8);
      ev->off[2] = add(sp_scnt_->p, ncap * 4, 4);
      ev->off[3] = add(sp_sdirty_->p, (ncap + 15) & ~(int64_t)15, 1);
      ev->presorted = true;
      ev->p_lo = p_lo;
      ev->np = np;
    } else {
      ev->off[0] = add(sp_key_->p, ncap * 8, 8);
      ev->off[1] = add(sp_pane_->p, ncap * 8, 8);
      ev->off[2] = add(sp_acc_->p, ncap * 8, 8);
      ev->off[3] = add(sp_cnt_->p, ncap * 4, 4);
      ev->off[4] = add(sp_dirty_->p, (ncap + 15) & ~(int64_t)15, 1);
    }
    // the eviction's pinned slab, reused while large enough (sizes grow with the key space)
    if (!evict_slab_ || evict_slab_->bytes < (size_t)off || evict_slab_.use_count() > 1)
      evict_slab_ = mem_alloc((size_t)off, 2, false);
    ev->slab = evict_slab_;
    if (!ready_ev_) ready_ev_ = new_event();
    record(ready_ev_, cur_);
    hip_ok(hipStreamWaitEvent(copy_, ready_ev_, 0), "wait");
    const int e = gpu::d2h_kernel(ev->slab->p, bt.c, bt.n, (intptr_t)copy_, P<uint32_t>(sp_ctr_) + 3, 64);
    if (e != 0) throw std::runtime_error("eviction copy failed");
    ev->ev = new_event();
    record(ev->ev, copy_);
    evict_busy_ = ev->ev;
    evict_pending_ = std::move(ev);
    ++m_.async_evictions;
    return {-1, -1, -1};
  }
  uint32_t ctr[4];
  to_host_sync(ctr, sp_ctr_->p, 16);
  if (ctr[2]) throw std::runtime_error("window_compact: eviction rows overflowed (internal error)");
  const int64_t n = ctr[3];
  if (n && tier_) {
    std::vector<uint64_t> k((size_t)n);
    std::vector<int64_t> pn((size_t)n), a((size_t)n), c((size_t)n);
    std::vector<uint32_t> c32((size_t)n);
    std::vector<uint8_t> d((size_t)n);
    to_host_sync(k.data(), sp_key_->p, n * 8);
    to_host_sync(pn.data(), sp_pane_->p, n * 8);
    to_host_sync(a.data(), sp_acc_->p, n * 8);
    to_host_sync(c32.data(), sp_cnt_->p, n * 4);
    to_host_sync(d.data(), sp_dirty_->p, n);
    for (int64_t i = 0; i < n; ++i) c[(size_t)i] = c32[(size_t)i];
    tier_->absorb(k.data(), pn.data(), a.data(), c.data(), d.data(), (size_t)n);
  }
  m_.dropped_keys += ctr[0];
  m_.spilled_keys += ctr[1];
  m_.spilled_rows += n;
  return {(int64_t)ctr[0], (int64_t)ctr[1], n};
}

void WindowStep::land_evictions() {
  // Absorb an asynchronous eviction's rows into the tier (its copy has long completed when this
  // runs: the next spill check, a firing over tier panes or a purge).
  std::unique_ptr<Eviction> ev = std::move(evict_pending_);
  if (!ev) return;
  host_wait(ev->ev);
  recycle(ev->ev);  // the copy has completed
  const char* base = (const char*)ev->slab->p;
  const uint32_t* ctr = (const uint32_t*)(base + ev->ctr_off);
  if (ctr[2]) throw std::runtime_error("window_compact: eviction rows overflowed (internal error)");
  const int64_t n = std::min<int64_t>(ctr[3], ev->cap);
  if (n && tier_) {
    if (ev->presorted) {
      const uint32_t* counts = (const uint32_t*)(base + ev->pc_off);
      int64_t tot = 0;
      for (int64_t j = 0; j < ev->np; ++j) tot += counts[j];
      if (tot != n)
        throw std::runtime_error("window_rows_pane_sort: pane counts do not add up (internal error)");
      tier_->absorb_presorted((const uint64_t*)(base + ev->off[0]), (const uint64_t*)(base + ev->off[1]),
                              (const uint32_t*)(base + ev->off[2]), (const uint8_t*)(base + ev->off[3]),
                              ev->p_lo, counts, (int)ev->np);
    } else {
      std::vector<int64_t> c((size_t)n);
      const uint32_t* c32 = (const uint32_t*)(base + ev->off[3]);
      for (int64_t i = 0; i < n; ++i) c[(size_t)i] = c32[i];
      tier_->absorb((const uint64_t*)(base + ev->off[0]), (const int64_t*)(base + ev->off[1]),
                    (const int64_t*)(base + ev->off[2]), c.data(), (const uint8_t*)(base + ev->off[4]),
                    (size_t)n);
    }
  }
  // (Touched-slot lists and dirty bytes are empty here: every step's re-firings cleared them
  // before this step boundary, so no slot id survives the rehash.)
  m_.dropped_keys += ctr[0];
  m_.spilled_keys += ctr[1];
  m_.spilled_rows += n;
}

void WindowStep::tier_rows(int64_t p0, int64_t p1, Buf* k, Buf* a, Buf* c, int64_t* n) {
  // The tier's live rows of panes [p0, p1] on the device, piece by piece through a ring of four
  // fixed page-locked slabs (the pinned memory never grows with the tier).
  *n = 0;
  const size_t bound = tier_->nrows();
  if (bound == 0) return;
  if (!gpu_) {
    const int64_t cap = (int64_t)bound;
    if (!tier_k_ || tier_dev_cap_ < cap) {
      tier_k_ = mem_alloc(cap * 8, 0, false);
      tier_a_ = mem_alloc(cap * 8, 0, false);
      tier_c_ = mem_alloc(cap * 4, 0, false);
      tier_dev_cap_ = cap;
    }
    *n = (int64_t)tier_->export_rows(p0, p1, P<uint64_t>(tier_k_), P<uint64_t>(tier_a_),
                                     P<uint32_t>(tier_c_), bound);
    *k = tier_k_;
    *a = tier_a_;
    *c = tier_c_;
    return;
  }
  const int64_t pr = (int64_t)1 << 22;
  int64_t total = -1, r = 0;
  int i = 0;
  while (total < 0 || r < total) {
    const int si = i % 4;
    if (!tier_slabs_[si]) tier_slabs_[si] = mem_alloc((size_t)pr * 20, 2, false);
    if (tier_slab_ev_[si]) {
      host_wait(tier_slab_ev_[si]);  // this slab's previous piece has reached the device
    }
    char* base = (char*)tier_slabs_[si]->p;
    const int64_t got = (int64_t)tier_->export_window(p0, p1, (uint64_t*)base, (uint64_t*)(base + 8 * pr),
                                                      (uint32_t*)(base + 16 * pr), (size_t)r, (size_t)pr, true);
    if (total < 0) {
      if (got == 0) return;
      total = got;
      if (!tier_k_ || tier_dev_cap_ < total) {
        tier_k_ = mem_alloc(total * 8, 1, false);
        tier_a_ = mem_alloc(total * 8, 1, false);
        tier_c_ = mem_alloc(total * 4, 1, false);
        tier_dev_cap_ = total;
      }
    } else if (got != total) {
      throw std::runtime_error("tier export: the tier changed between pieces (internal error)");
    }
    const int64_t m = std::min(pr, total - r);
    hip_ok(hipMemcpyAsync(P<uint64_t>(tier_k_) + r, base, m * 8, hipMemcpyHostToDevice, cur_), "H2D");
    hip_ok(hipMemcpyAsync(P<uint64_t>(tier_a_) + r, base + 8 * pr, m * 8, hipMemcpyHostToDevice, cur_), "H2D");
    hip_ok(hipMemcpyAsync(P<uint32_t>(tier_c_) + r, base + 16 * pr, m * 4, hipMemcpyHostToDevice, cur_), "H2D");
    if (!tier_slab_ev_[si]) tier_slab_ev_[si] = new_event();
    record(tier_slab_ev_[si], cur_);
    r += m;
    ++i;
  }
  *k = tier_k_;
  *a = tier_a_;
  *c = tier_c_;
  *n = total;
}

void WindowStep::tier_combine(const uint32_t* n_dev, int dev_mode, int tier_mode, int64_t p0, int64_t p1) {
  // tier_merge of the device rows in out_keys / out_raw / out_cnt (count n_dev on the device)
  // and the tier's rows of panes [p0, p1] into the transient combine table tt_[0..3]; outputs
  // tt_[4..7] hold >= half the table's rows.
  Buf tk, ta, tc;
  int64_t n_t = 0;
  tier_rows(p0, p1, &tk, &ta, &tc, &n_t);
  const int64_t need = next_pow2(std::max<int64_t>(1024, 2 * (orows_ + n_t)));
  const int dk = gpu_ ? 1 : 0;
  if (!tt_[0] || tt_size_ < need) {
    if (gpu_) claim(&tout_busy_);
    tt_[0] = mem_alloc(need * 8, dk, false);
    tt_[1] = mem_alloc(need * 8, dk, false);
    tt_[2] = mem_alloc(need * 4, dk, false);
    tt_[3] = mem_alloc(need, dk, false);
    tt_[4] = mem_alloc(need / 2 * 8, dk, false);
    tt_[5] = mem_alloc(need / 2 * 8, dk, false);
    tt_[6] = mem_alloc(need / 2 * 8, dk, false);
    tt_[7] = mem_alloc(need / 2 * 4, dk, false);
    tt_size_ = need;
  }
  if (gpu_) claim(&tout_busy_);  // the previous tiered firing's copy reads the outputs
  const int64_t size = tt_size_;
  memset_async(tt_[0], 0xFF, 0, size * 8);
  const uint64_t ident = agg_identity(cfg_.agg);
  if (gpu_) {
    if (ident == 0) memset_async(tt_[1], 0, 0, size * 8);
    else gpu::fill_u64(P<uint64_t>(tt_[1]), size, ident, (intptr_t)cur_);
  } else {
    std::fill(P<uint64_t>(tt_[1]), P<uint64_t>(tt_[1]) + size, ident);
  }
  memset_async(tt_[2], 0, 0, size * 4);
  memset_async(tt_[3], 0, 0, size);
  auto merge = [&](const uint64_t* k, const uint64_t* a, const uint32_t* c, int64_t n,
                   const uint32_t* nd, int mode) {
    if (gpu_)
      gpu::tier_merge(k, a, c, n, nd, mode, cfg_.agg, P<uint64_t>(tt_[0]), P<uint64_t>(tt_[1]),
                      P<uint32_t>(tt_[2]), P<uint8_t>(tt_[3]), (uint32_t)(size - 1), P<uint32_t>(flags_),
                      (intptr_t)cur_);
    else
      cpu::tier_merge(k, a, c, n, nd, mode, cfg_.agg, P<uint64_t>(tt_[0]), P<uint64_t>(tt_[1]),
                      P<uint32_t>(tt_[2]), P<uint8_t>(tt_[3]), (uint32_t)(size - 1), P<uint32_t>(flags_));
  };
  merge(P<uint64_t>(out_keys_), P<uint64_t>(out_raw_), P<uint32_t>(out_cnt_), orows_, n_dev, dev_mode);
  if (n_t) merge(P<uint64_t>(tk), P<uint64_t>(ta), P<uint32_t>(tc), n_t, nullptr, tier_mode);
}

void WindowStep::fire_window_tiered(int64_t s, int64_t p0, int64_t p1, bool only_dirty, int64_t seq) {
  // Window [s, s + size) with part of its state in the host tier, merged on the device:
  //  1. the device fires its rows of the window without the epilogue (count stays on the device);
  //  2. the tier's live rows of panes [p0, p1] are exported uncombined and copied H2D;
  //  3. tier_merge combines both per key into a transient table (a re-firing marks the
  //     device's dirty keys and folds tier rows of those keys only);
  //  4. window_fire over the table (one pane) with the fused map/filter epilogue.
  if (gpu_) claim_flags();
  memset_async(flags_, 0, 8, 4);
  FirePlan fp;
  std::memset(&fp, 0, sizeof(fp));
  fp.agg = cfg_.agg;
  fp.npanes = (int32_t)(p1 - p0 + 1);
  fp.ring = (int32_t)ring_;
  fp.only_dirty = only_dirty ? 1 : 0;
  fp.nslots = nslots_;
  fp.p0 = p0;
  fp.wstart = (double)s;
  fp.wend = (double)s + (double)ctl_.size();
  fp.out_cap = (uint32_t)orows_;
  if (only_dirty && dlist_) {
    fp.list = P<uint32_t>(dlist_);
    fp.list_n = P<uint32_t>(dlist_n_);
  }
  uint32_t* on = P<uint32_t>(flags_) + 2;
  if (gpu_)
    gpu::window_fire(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_),
                     fp, P<uint64_t>(out_keys_), P<double>(out_vals_), P<uint64_t>(out_raw_),
                     P<uint32_t>(out_cnt_), on, (intptr_t)cur_);
  else
    cpu::window_fire(P<uint64_t>(keys_g_), P<uint64_t>(acc_g_), P<uint32_t>(cnt_g_), P<uint8_t>(dirty_g_),
                     fp, P<uint64_t>(out_keys_), P<double>(out_vals_), P<uint64_t>(out_raw_),
                     P<uint32_t>(out_cnt_), on);
  ++m_.num_fires;
  tier_combine(on, only_dirty ? 1 : 0, only_dirty ? 2 : 0, p0, p1);
  memset_async(flags_, 0, 8, 4);
  FirePlan tp = fp;
  tp.npanes = 1;
  tp.ring = 1;
  tp.p0 = 0;
  tp.list = nullptr;
  tp.list_n = nullptr;
  tp.nslots = tt_size_;
  tp.out_cap = (uint32_t)(tt_size_ / 2);
  tp.map = cfg_.map;
  tp.filt = cfg_.filt;
  if (gpu_)
    gpu::window_fire(P<uint64_t>(tt_[0]), P<uint64_t>(tt_[1]), P<uint32_t>(tt_[2]), P<uint8_t>(tt_[3]),
                     tp, P<uint64_t>(tt_[4]), P<double>(tt_[5]), P<uint64_t>(tt_[6]), P<uint32_t>(tt_[7]),
                     on, (intptr_t)cur_);
  else
    cpu::window_fire(P<uint64_t>(tt_[0]), P<uint64_t>(tt_[1]), P<uint32_t>(tt_[2]), P<uint8_t>(tt_[3]),
                     tp, P<uint64_t>(tt_[4]), P<double>(tt_[5]), P<uint64_t>(tt_[6]), P<uint32_t>(tt_[7]),
                     on);
  FireBatch fb;
  fb.wins = {s};
  fb.only_dirty = only_dirty;
  fb.seq = seq;
  std::vector<std::pair<const void*, int>> cols = {
      {tt_[4]->p, 8}, {tt_[5]->p, 8}, {tt_[6]->p, 8}, {tt_[7]->p, 4}};
  if (async_fire_) {
    queue_counted(std::move(fb), cols, tt_size_ / 2, on, false, nullptr, 1, &tout_busy_);
    return;
  }
  const uint32_t n = (uint32_t)std::min<int64_t>(fired_count(), tt_size_ / 2);
  if (n == 0) return;
  queue_sync(std::move(fb), cols, n, {n});
}

// ---- checks / restore helpers -------------------------------------------------------------------
void WindowStep::check_table(intptr_t stream) {
  if (dense_bits_) return;
  Buf st = mem_alloc(kChkN * 8, gpu_ ? 1 : 0);
  uint64_t h[kChkN];
  if (gpu_) {
    gpu::check_table(P<uint64_t>(keys_g_), nsub_, nsub_log2_, cap_log2_, P<uint64_t>(st), stream);
    hip_ok(hipMemcpyAsync(h, st->p, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream), "D2H");
    hip_ok(hipStreamSynchronize((hipStream_t)stream), "sync");
  } else {
    cpu::check_table(P<uint64_t>(keys_g_), nsub_, nsub_log2_, cap_log2_, P<uint64_t>(st));
    std::memcpy(h, st->p, sizeof(h));
  }
  if (h[kChkMisplaced] || h[kChkBrokenChain] || h[kChkDuplicate])
    throw std::runtime_error("keyed state table invariant violated after step " +
                             std::to_string(m_.steps) + ": misplaced " + std::to_string(h[kChkMisplaced]) +
                             ", broken chains " + std::to_string(h[kChkBrokenChain]) + ", duplicates " +
                             std::to_string(h[kChkDuplicate]));
}

void WindowStep::rebuild_merge_ring(intptr_t stream) {
  // Local-global with allowed lateness, after a restore: the owners' merged values of the windows
  // that fired but are not cleaned are recomputed from the restored state -- the same collective
  // exchange as a fire, without the emit. Every rank runs the same window sequence.
  cur_ = (hipStream_t)stream;
  memset_async(keys_m_, 0xFF, 0, keys_m_->bytes);
  memset_async(acc_m_, 0, 0, acc_m_->bytes);
  memset_async(cnt_m_, 0, 0, cnt_m_->bytes);
  memset_async(dirty_m_, 0, 0, dirty_m_->bytes);
  memset_async(occ_m_, 0, 0, occ_m_->bytes);
  if (cfg_.lateness <= 0 || !ctl_.has_nfs() || !ctl_.has_live() || wm_ == INT64_MIN) return;
  int64_t s = std::max(ctl_.align_up((__int128)wm_ - ctl_.size() - cfg_.lateness + 2),
                       ctl_.first_start_containing(ctl_.pane_start(ctl_.min_live())));
  while (s < ctl_.nfs()) {
    const int64_t p0 = std::max(ctl_.pane_of(s), ctl_.min_live());
    const int64_t p1 = std::min(ctl_.pane_of(s) + ctl_.panes_per_window() - 1, ctl_.max_seen());
    if (p1 >= p0) fire_window_partials(s, p0, p1, false, false, 0);
    s += cfg_.slide;
  }
}

}  // namespace mxs
