// mxstream — CDNA4 (gfx950) kernels for the keyed streaming engine.
//
// Design (MI355X-first, see docs/DESIGN.md):
//   * partition  : keyBy + window assignment + late check in ONE pass. Each 512-thread workgroup
//                  builds an LDS histogram over (dest rank, sub-table) buckets for its chunk,
//                  reserves one run per bucket with a single global atomic, then scatters
//                  24-byte records into fixed-capacity buckets. The send buffer is therefore
//                  already dest-contiguous with equal splits: the RCCL all-to-all needs no
//                  host-side count exchange.
//   * window_agg : one 1024-thread workgroup OWNS one hash sub-table for the whole launch. The
//                  sub-table's keys and the step's pane deltas live in LDS (ds_cmpst_b64 insert,
//                  ds_add_u64 / ds_add_f64 / ds_max_i64 accumulation), so there is not a single
//                  global atomic per event; the deltas are written back with plain coalesced
//                  read-modify-writes (ownership makes them race-free).
//   * window_fire: pane-major state => each firing sweeps contiguous slot ranges; the window
//                  result, the traced map/filter epilogue (ExprProg) and wave-ballot compaction
//                  are fused into the sweep.
// Replaces the per-record Flink operators used by the reference: keyBy
// (chapter2/.../ComputeCpuMax.java:26), WindowOperator + ReducingState
// (chapter3/.../BandwidthMonitor.java:32-37, BandwidthMonitorWithEventTime.java:45-47),
// AggregatingState (chapter2/.../ComputeCpuAvg.java:27-59).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "mxs_kernels.h"

namespace mxs {
namespace {

#define HIP_CHECK(x)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                  \
  } while (0)

constexpr int kWave = 64;
// Partition variants (scripts/kbench.py A/B, profiles/): 0 plain scatter, 1 + non-temporal
// input loads, 2/3 + non-temporal stores (3x slower: rejected), 4/5 staged write-combined
// scatter (5 = with non-temporal loads; production when nb <= 512).

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t w = __shfl_xor(v, o);
    v = v > w ? v : w;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t w = __shfl_xor(v, o);
    v = v < w ? v : w;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Order-preserving map double <-> int64 so f64 min/max use the native ds_min_i64/ds_max_i64.
__device__ __forceinline__ int64_t f64_ord(uint64_t bits) {
  return (int64_t)(bits ^ ((uint64_t)((int64_t)bits >> 63) & 0x7FFFFFFFFFFFFFFFull));
}
__device__ __forceinline__ uint64_t f64_unord(int64_t o) {
  return (uint64_t)o ^ ((uint64_t)(o >> 63) & 0x7FFFFFFFFFFFFFFFull);
}

// ------------------------------------------------------------------------------------------
// Synthetic source: SoA (key, ts, val) batch from a counter-based RNG (device-side so the
// benchmark measures the engine, not PCIe).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void gen_one(uint64_t base, uint64_t idx, int64_t i, uint64_t nkeys,
                                        int64_t ts_base, double span_per_event,
                                        uint64_t disorder_p1, int64_t val_lo, uint64_t val_span,
                                        int32_t mode, double zipf_s, uint64_t& key, int64_t& t,
                                        uint64_t& v) {
  int64_t x;
  gen_event(base, idx, i, nkeys, ts_base, span_per_event, disorder_p1, val_lo, val_span, zipf_s,
            key, t, x);
  v = (mode & 1) ? f64_bits((double)x) : (uint64_t)x;
}

// Two consecutive events per lane: every column is written with 16-byte stores (8-byte int32
// key pairs), so a wave moves whole 1 KiB lines per store instruction. Event i is a pure function
// of (seed, stream, idx0 + i), independent of the launch shape.
__global__ __launch_bounds__(256) void gen_events_kernel(
    uint64_t* __restrict__ keys, int64_t* __restrict__ ts, uint64_t* __restrict__ vals,
    int64_t n, uint64_t seed, uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
    double span_per_event, uint64_t disorder_p1, int64_t val_lo, uint64_t val_span,
    int32_t mode, double zipf_s, uint64_t key_base) {
  // mode bit 0: values as f64 bits; bit 1: int32 key ids (the columnar sources' dictionary ids)
  // zipf_s > 0: skewed keys (key_of_draw: power law, rank 0 hottest); 0: uniform.
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t npairs = n >> 1;
  const uint64_t base = mix64(seed ^ (stream_id * 0xd1b54a32d192ed03ull));  // rng64's stream word
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += stride) {
    const int64_t i = 2 * p;
    uint64_t k0, k1, v0, v1;
    int64_t t0, t1;
    gen_one(base, idx0 + (uint64_t)i, i, nkeys, ts_base, span_per_event, disorder_p1, val_lo,
            val_span, mode, zipf_s, k0, t0, v0);
    gen_one(base, idx0 + (uint64_t)i + 1, i + 1, nkeys, ts_base, span_per_event, disorder_p1,
            val_lo, val_span, mode, zipf_s, k1, t1, v1);
    k0 += key_base;  // (a drifting key window: no separate add pass over the column)
    k1 += key_base;
    if (mode & 4) {  // a column not 16-byte aligned (a sliced tensor): scalar stores
      if (mode & 2) {
        reinterpret_cast<int32_t*>(keys)[i] = (int32_t)k0;
        reinterpret_cast<int32_t*>(keys)[i + 1] = (int32_t)k1;
      } else {
        keys[i] = k0;
        keys[i + 1] = k1;
      }
      ts[i] = t0;
      ts[i + 1] = t1;
      vals[i] = v0;
      vals[i + 1] = v1;
      continue;
    }
    if (mode & 2) {
      reinterpret_cast<uint2*>(keys)[p] = make_uint2((uint32_t)k0, (uint32_t)k1);
    } else {
      reinterpret_cast<ulonglong2*>(keys)[p] = make_ulonglong2(k0, k1);
    }
    reinterpret_cast<longlong2*>(ts)[p] = make_longlong2(t0, t1);
    reinterpret_cast<ulonglong2*>(vals)[p] = make_ulonglong2(v0, v1);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {  // odd tail
    const int64_t i = n - 1;
    uint64_t k, v;
    int64_t t;
    gen_one(mix64(seed ^ (stream_id * 0xd1b54a32d192ed03ull)), idx0 + (uint64_t)i, i, nkeys,
            ts_base, span_per_event, disorder_p1, val_lo, val_span, mode, zipf_s, k, t, v);
    k += key_base;
    if (mode & 2) reinterpret_cast<int32_t*>(keys)[i] = (int32_t)k;
    else keys[i] = k;
    ts[i] = t;
    vals[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// Fired rows -> pinned host slab by a kernel (16-byte vector stores into mapped host memory):
// the DMA path (hipMemcpyAsync D2H) stalled the host for 7-9 ms at one firing in some runs
// (profiles/r2_fire_d2h.md); a kernel copy has no lazily initialised engine behind it.
// ------------------------------------------------------------------------------------------
// With b.n_dev the row count stays on the device: copies with esz > 0 move only the rows the
// producer counted (the fire needs no host round trip for its count before the copy).
__global__ __launch_bounds__(256) void d2h_copy_kernel(unsigned char* __restrict__ dst, D2HBatch b) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t rows = b.n_dev ? (int64_t)*b.n_dev : -1;
  for (int k = 0; k < b.n; ++k) {
    const v4u* __restrict__ s = reinterpret_cast<const v4u*>(b.c[k].src);
    v4u* __restrict__ d = reinterpret_cast<v4u*>(dst + b.c[k].dst_off);
    int64_t bytes = b.c[k].bytes;
    if (rows >= 0 && b.c[k].esz > 0) {
      const int64_t want = (rows * b.c[k].esz + 15) & ~(int64_t)15;
      bytes = want < bytes ? want : bytes;
    }
    const int64_t n16 = bytes >> 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
      d[i] = __builtin_nontemporal_load(&s[i]);
  }
}

// ------------------------------------------------------------------------------------------
// Partition: keyBy (Flink key groups -> dest rank) x sub-table, window assignment, late drop.
// ------------------------------------------------------------------------------------------
// Per-element partition decision; identical code runs in pass A (histogram) and pass B
// (scatter) so both passes agree without storing per-element bucket ids.
// kind: 0 = keep, 1 = late (dropped), 2 = unrepresentable pane (overflow), 3 = reserved key id
// (~0 is the tables' empty-slot marker and the partition's hole marker: reported, never stored)
struct PartEval {
  int kind;
  uint32_t bucket;
  uint32_t t;
};

// ONE = true: compiled for a single rank (no key-group hashing at all; bucket = sub-table).
template <bool ONE = false>
__device__ __forceinline__ PartEval part_eval(uint64_t key, int64_t ts, const int32_t* jhash_tab,
                                              const PartPlan& p, const int32_t* kg_dest) {
  PartEval e;
  e.kind = 0;
  e.t = 0;
  e.bucket = 0;
  if (key >= kTombKey) {  // ~1 / ~0: tombstone and empty-slot markers of the tables
    e.kind = 3;
    return e;
  }
  if (p.window_mode) {
    if (p.drop_late && ts < p.late_ts) {
      e.kind = 1;
      return e;
    }
    int64_t q;
    if (!rel_pane(ts, p, &e.t, &q)) {
      e.kind = 2;
      return e;
    }
  }
  if constexpr (ONE) {
    e.bucket = sub_of(key, p);
  } else {
    const int32_t jh = p.nranks == 1 ? 0 : p.hash_mode ? jhash_tab[key] : java_long_hash((int64_t)key);
    e.bucket = bucket_of(key, jh, p, kg_dest);
  }
  return e;
}

// Block-wide reduction helpers (one global atomic per workgroup instead of one per wave).
__device__ __forceinline__ int64_t block_reduce_i64(int64_t v, int64_t* red, int op) {
  // op: 0 = max, 1 = min, 2 = sum. `red` = kMaxWaves int64 of LDS.
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o);
    v = op == 0 ? (v > w ? v : w) : op == 1 ? (v < w ? v : w) : op == 3 ? (v | w) : v + w;
  }
  const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) red[wid] = v;
  __syncthreads();
  v = red[0];
  for (int i = 1; i < nw; ++i) {
    const int64_t w = red[i];
    v = op == 0 ? (v > w ? v : w) : op == 1 ? (v < w ? v : w) : op == 3 ? (v | w) : v + w;
  }
  return v;
}

// Relative pane -> kStatPaneMask bit (bit 31: pane >= 31, mask unusable).
__device__ __forceinline__ uint32_t pane_bit(uint32_t q) { return 1u << (q < 31u ? q : 31u); }

// ILP factor: each thread issues kPartU independent loads before it consumes any, so 16 waves
// per CU keep ~16 x 64 x kPartU loads in flight (the loop was latency-bound at one chain).
constexpr int kPartU = 8;
// The plain-scatter kernel keeps key, ts and value of every unrolled element live across
// part_eval: at 1024 threads (<= 128 VGPRs) 8 elements spilled to scratch, 4 do not.
constexpr int kPlainU = 4;

// Input-stream loads: V&1 = non-temporal (streamed once; keep L2 for the scatter's open lines).
template <int V, class T>
__device__ __forceinline__ T ldin(const T* p) {
  if (V & 1) return __builtin_nontemporal_load(p);
  return *p;
}

// Key column load: 64-bit keys, or int32 dictionary ids (PartPlan.key32) sign-extended so the
// reserved markers -1 / -2 stay detectable.
template <int V, bool K32>
__device__ __forceinline__ uint64_t ldkey(const uint64_t* keys, int64_t i) {
  if constexpr (K32) return (uint64_t)(int64_t)ldin<V>(&reinterpret_cast<const int32_t*>(keys)[i]);
  else return ldin<V>(&keys[i]);
}

// Two consecutive events per lane (PAIR partition variant): keys as one 8-byte (int32 ids) or
// 16-byte load, ts and values as one 16-byte load each -- half the load instructions of the
// one-event-per-lane form and 1 KB of contiguous bytes per wave-wide ts / value load.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <int V, typename T>
__device__ __forceinline__ T ldvec(const T* p) {
  if (V & 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int V, bool K32>
__device__ __forceinline__ void ldkey2(const uint64_t* keys, int64_t i, uint64_t& k0, uint64_t& k1) {
  if constexpr (K32) {
    const u32x2_t w = ldvec<V>(reinterpret_cast<const u32x2_t*>(reinterpret_cast<const int32_t*>(keys) + i));
    k0 = (uint64_t)(int64_t)(int32_t)w.x;
    k1 = (uint64_t)(int64_t)(int32_t)w.y;
  } else {
    const u32x4_t w = ldvec<V>(reinterpret_cast<const u32x4_t*>(keys + i));
    k0 = (uint64_t)w.x | ((uint64_t)w.y << 32);
    k1 = (uint64_t)w.z | ((uint64_t)w.w << 32);
  }
}
template <int V>
__device__ __forceinline__ void ld64x2(const void* base, int64_t i, uint64_t& a, uint64_t& b) {
  const u32x4_t w = ldvec<V>(reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint64_t*>(base) + i));
  a = (uint64_t)w.x | ((uint64_t)w.y << 32);
  b = (uint64_t)w.z | ((uint64_t)w.w << 32);
}

template <int V>
__global__ __launch_bounds__(1024) void partition_kernel(
    const uint64_t* __restrict__ keys, const int64_t* __restrict__ ts,
    const uint64_t* __restrict__ vals, const int32_t* __restrict__ jhash_tab, int64_t n,
    int64_t chunk, PartPlan plan, const int32_t* __restrict__ kg_dest,
    uint32_t* __restrict__ cursor, Rec* __restrict__ out, int64_t* __restrict__ stats,
    uint32_t* __restrict__ late_idx, uint32_t late_cap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lhist[];  // nb u32 | 16 x i64 scratch
  const int nb = plan.nranks << plan.nsub_log2;
  int64_t* lred = (int64_t*)(lhist + ((nb + 3) & ~3));
  for (int b = threadIdx.x; b < nb; b += blockDim.x) lhist[b] = 0;
  __syncthreads();

  const int64_t start = (int64_t)blockIdx.x * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;
  const int64_t bstep = (int64_t)blockDim.x * kPlainU;
  int64_t tmax = INT64_MIN, qmin = INT64_MAX, qmax = INT64_MIN, nlate = 0, nacc = 0;
  uint32_t pmask = 0;
  int bad = 0;  // stats overflow bits: 2 unrepresentable pane, 8 reserved key

  // Pass A: histogram + stats.
  for (int64_t i0 = start + threadIdx.x; i0 < end; i0 += bstep) {
    uint64_t k[kPlainU];
    int64_t t[kPlainU];
#pragma unroll
    for (int u = 0; u < kPlainU; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < end) {
        k[u] = ldin<V>(&keys[i]);
        t[u] = ldin<V>(&ts[i]);
      }
    }
#pragma unroll
    for (int u = 0; u < kPlainU; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i >= end) break;
      tmax = t[u] > tmax ? t[u] : tmax;
      const PartEval e = part_eval(k[u], t[u], jhash_tab, plan, kg_dest);
      if (e.kind) {
        if (e.kind >= 2) {
          bad |= e.kind == 2 ? 2 : 8;
          continue;
        }
        ++nlate;
        if (late_idx) {
          const unsigned long long pos = atomicAdd((unsigned long long*)&stats[kStatLate], 1ull);
          if (pos < late_cap) late_idx[pos] = (uint32_t)i;
        }
        continue;
      }
      ++nacc;
      qmin = (int64_t)e.t < qmin ? (int64_t)e.t : qmin;
      qmax = (int64_t)e.t > qmax ? (int64_t)e.t : qmax;
      pmask |= pane_bit(e.t);
      atomicAdd(&lhist[e.bucket], 1u);
    }
  }
  __syncthreads();

  // Reserve one run per bucket: one global atomic per (workgroup, non-empty bucket). With
  // 64K events per workgroup a run averages >= 32 records, so the scatter below writes runs.
  bool overflow = false;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const uint32_t c = lhist[b];
    if (c) {
      const uint32_t base = atomicAdd(&cursor[b], c);
      if (base + c > plan.bucket_cap) overflow = true;
      lhist[b] = base;
    }
  }
  __syncthreads();

  bool wide = false;   // a value does not fit a 16-byte record
  bool nwide = false;  // a record does not fit the 8-byte format
  // Pass B: scatter records into their bucket runs.
  const uint32_t bcap = plan.bucket_cap;
  for (int64_t i0 = start + threadIdx.x; i0 < end; i0 += bstep) {
    uint64_t k[kPlainU], v[kPlainU];
    int64_t t[kPlainU];
#pragma unroll
    for (int u = 0; u < kPlainU; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < end) {
        k[u] = ldin<V>(&keys[i]);
        t[u] = ldin<V>(&ts[i]);
        v[u] = ldin<V>(&vals[i]);
      }
    }
#pragma unroll
    for (int u = 0; u < kPlainU; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i >= end) break;
      const PartEval e = part_eval(k[u], t[u], jhash_tab, plan, kg_dest);
      if (e.kind) continue;
      const uint32_t pos = atomicAdd(&lhist[e.bucket], 1u);
      if (pos < bcap && !(plan.ablate & 1u) && plan.rec_words == 1) {
        // 8-byte record (one destination, more buckets than the staged kernel takes): 32-bit key
        // id, 28-bit value, 4-bit pane; a record that does not fit flags bit 16 (widen, redo).
        if (!narrow_fits(k[u], (int64_t)v[u], e.t)) nwide = true;
        ((uint2*)out)[(size_t)e.bucket * bcap + pos] =
            make_uint2((uint32_t)k[u], ((uint32_t)v[u] << 4) | (e.t & 15u));
      } else if (pos < bcap && !(plan.ablate & 1u) && plan.rec_words == 2) {
        // 16-byte record: one vector store (int32 value; wider values flag bit 2).
        if ((int64_t)(int32_t)v[u] != (int64_t)v[u]) wide = true;
        ((uint4*)out)[(size_t)e.bucket * bcap + pos] =
            make_uint4((uint32_t)k[u], (uint32_t)(k[u] >> 32), (uint32_t)v[u], e.t);
      } else if (pos < bcap && !(plan.ablate & 1u)) {
        Rec* dst = &out[(size_t)e.bucket * bcap + pos];
        if (V & 2) {
          __builtin_nontemporal_store(k[u], &dst->key);
          __builtin_nontemporal_store(v[u], &dst->val);
          __builtin_nontemporal_store(((uint64_t)(uint32_t)i << 32) | e.t, (uint64_t*)&dst->t);
        } else {
          Rec r;
          r.key = k[u];
          r.val = v[u];
          r.t = e.t;
          r.aux = (uint32_t)i;
          *dst = r;
        }
      }
    }
  }

  // Block stats -> one global atomic per workgroup and statistic.
  tmax = block_reduce_i64(tmax, lred, 0);
  qmin = block_reduce_i64(qmin, lred, 1);
  qmax = block_reduce_i64(qmax, lred, 0);
  nacc = block_reduce_i64(nacc, lred, 2);
  pmask = (uint32_t)block_reduce_i64(pmask, lred, 3);
  if (!late_idx) nlate = block_reduce_i64(nlate, lred, 2);
  const int64_t flags = block_reduce_i64(overflow ? 1 : 0, lred, 0) |
                        block_reduce_i64(bad & 2, lred, 0) | block_reduce_i64(bad & 8, lred, 0) |
                        block_reduce_i64(wide ? 4 : 0, lred, 0) |
                        block_reduce_i64(nwide ? 16 : 0, lred, 0);
  if (threadIdx.x == 0) {
    atomicMax((long long*)&stats[kStatMaxTs], (long long)tmax);
    if (nacc) {
      atomicMin((long long*)&stats[kStatMinPane], (long long)qmin);
      atomicMax((long long*)&stats[kStatMaxPane], (long long)qmax);
      atomicAdd((unsigned long long*)&stats[kStatAccepted], (unsigned long long)nacc);
      if (pmask) atomicOr((unsigned long long*)&stats[kStatPaneMask], (unsigned long long)pmask);
    }
    if (!late_idx && nlate) atomicAdd((unsigned long long*)&stats[kStatLate], (unsigned long long)nlate);
    if (flags) atomicOr((unsigned long long*)&stats[kStatOverflow], (unsigned long long)flags);
  }
}

// ------------------------------------------------------------------------------------------
// Staged partition (nb <= 512): write-combined scatter.
//
// The plain scatter writes 24-byte records into nb open runs per workgroup; on gfx950 the
// partially written 128-B lines are evicted by the input stream long before they fill
// (measured: 4.6x HBM write amplification). Here every round of kStageR records is counting-
// sorted by bucket in LDS; each bucket keeps its partial tail group (< 8 records) in an LDS
// carry buffer and only complete 8-record groups (192 B = three aligned 64-B sectors) are
// written. Per-workgroup runs are reserved in multiples of 8 and the final partial group is
// padded with hole records (t = kHoleT), which window_agg skips.
// ------------------------------------------------------------------------------------------
constexpr int kStageU = 2;                  // events per thread per round
constexpr int kStageR = 1024 * kStageU;     // records per round
constexpr int kStageMaxNb = 512;
constexpr uint32_t kHoleT = 0xFFFFFFFFu;

__device__ __forceinline__ void lds_store_rec(Rec* dst, const Rec& r) {
  uint64_t* d = (uint64_t*)dst;
  d[0] = r.key;
  d[1] = r.val;
  d[2] = ((uint64_t)r.aux << 32) | r.t;
}

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* wsum) {
  // 1024-thread exclusive scan; wsum = 17 u32 of LDS. Returns this thread's exclusive prefix.
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < 16; ++w) {
      const uint32_t t = wsum[w];
      wsum[w] = acc;
      acc += t;
    }
    wsum[16] = acc;
  }
  __syncthreads();
  return wsum[wid] + x - v;
}

template <int V>
__global__ __launch_bounds__(1024) void partition_staged_kernel(
    const uint64_t* __restrict__ keys, const int64_t* __restrict__ ts,
    const uint64_t* __restrict__ vals, const int32_t* __restrict__ jhash_tab, int64_t n,
    int64_t chunk, PartPlan plan, const int32_t* __restrict__ kg_dest,
    uint32_t* __restrict__ cursor, Rec* __restrict__ out, int64_t* __restrict__ stats,
    uint32_t* __restrict__ late_idx, uint32_t late_cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  const int nb = plan.nranks << plan.nsub_log2;
  Rec* carry = (Rec*)psm;                                   // [kStageMaxNb][8]
  Rec* rbuf = carry + kStageMaxNb * 8;                      // [kStageR]
  uint32_t* run_base = (uint32_t*)(rbuf + kStageR);          // [kStageMaxNb]
  uint32_t* lcnt = run_base + kStageMaxNb;                   // records appended per bucket
  uint32_t* rcnt = lcnt + kStageMaxNb;                       // this round's count per bucket
  uint32_t* roff = rcnt + kStageMaxNb;                       // this round's offsets
  uint32_t* wsum = roff + kStageMaxNb;                       // 17 scan words (+pad)
  int64_t* lred = (int64_t*)(wsum + 20);                     // 16 x i64

  for (int b = threadIdx.x; b < kStageMaxNb; b += blockDim.x) {
    run_base[b] = 0;
    lcnt[b] = 0;
    rcnt[b] = 0;
  }
  __syncthreads();

  const int64_t start = (int64_t)blockIdx.x * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;
  int64_t tmax = INT64_MIN, qmin = INT64_MAX, qmax = INT64_MIN, nlate = 0, nacc = 0;
  uint32_t pmask = 0;
  int bad = 0;  // stats overflow bits: 2 unrepresentable pane, 8 reserved key

  // Pass A: histogram (into run_base) + stats.
  for (int64_t i0 = start + threadIdx.x; i0 < end; i0 += (int64_t)blockDim.x * kPartU) {
    uint64_t k[kPartU];
    int64_t t[kPartU];
#pragma unroll
    for (int u = 0; u < kPartU; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < end) {
        k[u] = ldin<V>(&keys[i]);
        t[u] = ldin<V>(&ts[i]);
      }
    }
#pragma unroll
    for (int u = 0; u < kPartU; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i >= end) break;
      tmax = t[u] > tmax ? t[u] : tmax;
      const PartEval e = part_eval(k[u], t[u], jhash_tab, plan, kg_dest);
      if (e.kind) {
        if (e.kind >= 2) {
          bad |= e.kind == 2 ? 2 : 8;
          continue;
        }
        ++nlate;
        if (late_idx) {
          const unsigned long long pos = atomicAdd((unsigned long long*)&stats[kStatLate], 1ull);
          if (pos < late_cap) late_idx[pos] = (uint32_t)i;
        }
        continue;
      }
      ++nacc;
      qmin = (int64_t)e.t < qmin ? (int64_t)e.t : qmin;
      pmask |= pane_bit(e.t);
      qmax = (int64_t)e.t > qmax ? (int64_t)e.t : qmax;
      atomicAdd(&run_base[e.bucket], 1u);
    }
  }
  __syncthreads();

  // Reserve this workgroup's run per bucket, rounded up to whole 8-record groups so every
  // group written below covers aligned 64-B sectors (bucket_cap is a multiple of 8).
  bool overflow = false;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const uint32_t c = (run_base[b] + 7u) & ~7u;
    uint32_t base = 0;
    if (c) {
      base = atomicAdd(&cursor[b], c);
      if (base + c > plan.bucket_cap) overflow = true;
    }
    run_base[b] = base;
  }
  const uint32_t bcap = plan.bucket_cap;
  if (threadIdx.x == 0) wsum[18] = 0;
  __syncthreads();
  if (overflow) wsum[18] = 1;
  __syncthreads();
  const bool any_ovf = wsum[18] != 0;

  // Pass B: rounds of kStageR records -> LDS sort by bucket -> whole-group writes.
  for (int64_t r0 = start; r0 < end; r0 += kStageR) {
    uint32_t bk[kStageU], rk[kStageU];
    Rec rec[kStageU];
    bool keep[kStageU];
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int64_t i = r0 + (int64_t)u * blockDim.x + threadIdx.x;
      keep[u] = false;
      if (i < end) {
        const uint64_t k = ldin<V>(&keys[i]);
        const int64_t t = ldin<V>(&ts[i]);
        const uint64_t v = ldin<V>(&vals[i]);
        const PartEval e = part_eval(k, t, jhash_tab, plan, kg_dest);
        if (!e.kind) {
          keep[u] = true;
          bk[u] = e.bucket;
          rec[u].key = k;
          rec[u].val = v;
          rec[u].t = e.t;
          rec[u].aux = (uint32_t)i;
          rk[u] = atomicAdd(&rcnt[e.bucket], 1u);
        }
      }
    }
    __syncthreads();
    const uint32_t myc = threadIdx.x < (unsigned)nb ? rcnt[threadIdx.x] : 0u;
    const uint32_t off = block_exclusive_scan(myc, wsum);
    if (threadIdx.x < (unsigned)nb) roff[threadIdx.x] = off;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kStageU; ++u)
      if (keep[u]) lds_store_rec(&rbuf[roff[bk[u]] + rk[u]], rec[u]);
    __syncthreads();
    // Flush: one thread per bucket writes its complete groups (carry first, then this round).
    if (threadIdx.x < (unsigned)nb && !any_ovf) {
      const int b = threadIdx.x;
      const uint32_t nc = lcnt[b] & 7u;      // records waiting in carry[b]
      const uint32_t nr = rcnt[b];
      const uint32_t tot = nc + nr;
      const uint32_t groups = tot >> 3;
      const uint32_t first = lcnt[b] - nc;   // run offset of carry[b][0]
      Rec* dstb = out + (size_t)b * bcap + run_base[b] + first;
      const Rec* src_r = rbuf + roff[b];
      for (uint32_t g = 0; g < groups; ++g) {
        uint4* d = (uint4*)(dstb + g * 8);   // 192 B = 12 x 16 B
#pragma unroll
        for (int q = 0; q < 12; ++q) {
          // 16-B chunk q of the group: records are 24 B, chunk spans record idx = q*16/24.
          const uint32_t byte = q * 16;
          const uint32_t j = g * 8 + byte / 24;  // record index within (carry ++ round)
          const uint32_t ob = byte % 24;         // 0, 16 or 8
          const Rec* ra = j < nc ? &carry[b * 8 + j] : &src_r[j - nc];
          const uint64_t* rw = (const uint64_t*)ra;
          uint4 v;
          if (ob == 0) {
            v = make_uint4((uint32_t)rw[0], (uint32_t)(rw[0] >> 32), (uint32_t)rw[1], (uint32_t)(rw[1] >> 32));
          } else if (ob == 16) {
            const uint32_t j2 = j + 1;
            const Rec* rb = j2 < nc ? &carry[b * 8 + j2] : &src_r[j2 - nc];
            const uint64_t* rw2 = (const uint64_t*)rb;
            v = make_uint4((uint32_t)rw[2], (uint32_t)(rw[2] >> 32), (uint32_t)rw2[0], (uint32_t)(rw2[0] >> 32));
          } else {  // ob == 8
            v = make_uint4((uint32_t)rw[1], (uint32_t)(rw[1] >> 32), (uint32_t)rw[2], (uint32_t)(rw[2] >> 32));
          }
          d[q] = v;
        }
      }
      // Keep the remainder (< 8 records) in the carry buffer. When no group was written the
      // carried records stay in place; otherwise every remaining record comes from rbuf, so
      // the copy never reads a carry slot it has already overwritten.
      const uint32_t rem = tot - groups * 8;
      for (uint32_t j = 0; j < rem; ++j) {
        const uint32_t jj = groups * 8 + j;
        if (jj < nc) continue;  // groups == 0: already at carry[b * 8 + jj] with jj == j
        const uint64_t* rw = (const uint64_t*)&src_r[jj - nc];
        uint64_t* cw = (uint64_t*)&carry[b * 8 + j];
        cw[0] = rw[0];
        cw[1] = rw[1];
        cw[2] = rw[2];
      }
      lcnt[b] += nr;
      rcnt[b] = 0;
    }
    __syncthreads();
  }
  // Final partial groups, padded with holes.
  if (threadIdx.x < (unsigned)nb && !any_ovf) {
    const int b = threadIdx.x;
    const uint32_t nc = lcnt[b] & 7u;
    if (nc) {
      Rec* dst = out + (size_t)b * bcap + run_base[b] + (lcnt[b] - nc);
      for (uint32_t j = 0; j < 8; ++j) {
        Rec r;
        if (j < nc) {
          r = carry[b * 8 + j];
        } else {
          r.key = kEmptyKey;
          r.val = 0;
          r.t = kHoleT;
          r.aux = kHoleT;
        }
        dst[j] = r;
      }
    }
  }

  // Block stats -> one global atomic per workgroup and statistic.
  tmax = block_reduce_i64(tmax, lred, 0);
  qmin = block_reduce_i64(qmin, lred, 1);
  qmax = block_reduce_i64(qmax, lred, 0);
  nacc = block_reduce_i64(nacc, lred, 2);
  pmask = (uint32_t)block_reduce_i64(pmask, lred, 3);
  if (!late_idx) nlate = block_reduce_i64(nlate, lred, 2);
  const int64_t flags = (any_ovf ? 1 : 0) | block_reduce_i64(bad & 2, lred, 0) |
                        block_reduce_i64(bad & 8, lred, 0);
  if (threadIdx.x == 0) {
    atomicMax((long long*)&stats[kStatMaxTs], (long long)tmax);
    if (nacc) {
      atomicMin((long long*)&stats[kStatMinPane], (long long)qmin);
      atomicMax((long long*)&stats[kStatMaxPane], (long long)qmax);
      atomicAdd((unsigned long long*)&stats[kStatAccepted], (unsigned long long)nacc);
      if (pmask) atomicOr((unsigned long long*)&stats[kStatPaneMask], (unsigned long long)pmask);
    }
    if (!late_idx && nlate) atomicAdd((unsigned long long*)&stats[kStatLate], (unsigned long long)nlate);
    if (flags) atomicOr((unsigned long long*)&stats[kStatOverflow], (unsigned long long)flags);
  }
}

constexpr size_t kStagedLds = (size_t)kStageMaxNb * 8 * sizeof(Rec) + (size_t)kStageR * sizeof(Rec) +
                              (size_t)kStageMaxNb * 4 * 4 + 20 * 4 + 16 * 8;
static_assert(kStagedLds <= 160 * 1024, "staged partition LDS image exceeds 160 KiB");

// ------------------------------------------------------------------------------------------
// Compact staged partition (16-byte RecC, integer window aggregates). Differences from the
// 24-byte staged kernel, each measured (profiles/README.md):
//  * pass A reads only the keys (the bucket is a function of the key); late / unrepresentable
//    records are counted into the reservation and their slots filled with holes at the end, so
//    pass B alone reads ts/val (32 B of input per event instead of 40 B);
//  * a record is one 16-byte vector; the LDS image (~42 KB) lets two workgroups share a CU;
//  * cooperative flush: after the per-round LDS counting sort every thread writes one sorted
//    record to its bucket run (runs are contiguous, so a wave's stores coalesce and the partial
//    sectors at run ends are completed by the next round while still in L2). This beat the
//    carry/whole-group flush of the 24-byte kernel by ~3 % end to end.
// A value outside int32 sets stats overflow bit 2: the host redoes the step with 24-byte records.
// ------------------------------------------------------------------------------------------
constexpr int kCU = 2;                   // events per thread per round (production)
constexpr int kCG = 4;                   // reservation granularity (records per 64-byte sector)
constexpr int kCMaxNb = 512;
constexpr int kKgLdsMax = 4096;          // max parallelism whose kg -> rank table goes to LDS
constexpr size_t compact_lds(int cu) {
  return (size_t)1024 * cu * sizeof(RecC) + (size_t)kCMaxNb * 6 * 4 + 20 * 4 + 16 * 8 +
         (size_t)1024 * cu * 2 + (size_t)kKgLdsMax * 4;
}
constexpr size_t kCompactLds = compact_lds(kCU);
static_assert(kCompactLds <= 80 * 1024, "compact partition must fit two workgroups per CU");
constexpr int kCUProd = 4;               // production round: 4096 records, one group per CU
static_assert(compact_lds(kCUProd) <= 160 * 1024, "compact partition LDS exceeds 160 KiB");
// LDS image of a round of 1024 * cu records of rb bytes (8-byte RecN rounds fit 8192 records).
constexpr size_t compact_lds_rb(int cu, int rb) {
  return (size_t)1024 * cu * rb + (size_t)kCMaxNb * 6 * 4 + 20 * 4 + 16 * 8 +
         (size_t)1024 * cu * 2 + (size_t)kKgLdsMax * 4;
}
static_assert(compact_lds_rb(8, 8) <= 160 * 1024, "8K-record RecN rounds exceed 160 KiB");

// RB = 16: RecC records; RB = 8: RecN records (one destination, see RecN).
template <int V, int CU = kCU, bool ONE = false, int RB = 16, bool K32 = false, bool PAIR = false>
__global__ __launch_bounds__(1024) void partition_compact_kernel(
    const uint64_t* __restrict__ keys, const int64_t* __restrict__ ts,
    const uint64_t* __restrict__ vals, const int32_t* __restrict__ jhash_tab, int64_t n,
    int64_t chunk, PartPlan plan, const int32_t* __restrict__ kg_dest,
    uint32_t* __restrict__ cursor, RecC* __restrict__ out, int64_t* __restrict__ stats,
    uint32_t* __restrict__ late_idx, uint32_t late_cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char csm[];
  const int nb = plan.nranks << plan.nsub_log2;
  using RT = typename std::conditional<RB == 8, uint2, uint4>::type;
  RT* rbuf = (RT*)csm;                                         // [(1024 * CU)] sorted round
  uint32_t* run_base = (uint32_t*)(rbuf + (1024 * CU));                // [kCMaxNb]
  uint32_t* resv = run_base + kCMaxNb;                         // reserved records per bucket
  uint32_t* lcnt = resv + kCMaxNb;                             // records written per bucket
  uint32_t* rcnt = lcnt + kCMaxNb;                             // this round's count per bucket
  uint32_t* roff = rcnt + kCMaxNb;                             // this round's offsets
  uint32_t* wsum = roff + kCMaxNb;                             // 17 scan words (+pad)
  int64_t* lred = (int64_t*)(wsum + 20);                       // 16 x i64
  uint16_t* sbk = (uint16_t*)(lred + 16);                      // [(1024 * CU)] bucket of rbuf[j]
  uint32_t* dbase = (uint32_t*)(sbk + (1024 * CU));                    // [kCMaxNb] round's dest - offset
  int32_t* skg = (int32_t*)(dbase + kCMaxNb);                  // [kKgLdsMax] key group -> rank

  for (int b = threadIdx.x; b < kCMaxNb; b += blockDim.x) {
    run_base[b] = 0;
    lcnt[b] = 0;
    rcnt[b] = 0;
  }
  // G > 1: the key-group -> rank table lives in LDS. A global load per record inside the round
  // made the in-order vmcnt wait for the next round's prefetched (key, ts, value) loads too.
  const bool kg_lds = !ONE && plan.nranks > 1 && plan.max_parallelism <= kKgLdsMax;
  if (kg_lds)
    for (int g = threadIdx.x; g < plan.max_parallelism; g += blockDim.x) skg[g] = kg_dest[g];
  __syncthreads();
  const int64_t start = (int64_t)blockIdx.x * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;

  // Event u of a thread's group: lane-strided, or (PAIR) two consecutive events per lane.
  auto ev_at = [&](int64_t base, int u) -> int64_t {
    if constexpr (PAIR)
      return base + (int64_t)(u >> 1) * 2 * blockDim.x + 2 * (int64_t)threadIdx.x + (u & 1);
    else
      return base + (int64_t)u * blockDim.x + threadIdx.x;
  };
  // Pass A: bucket histogram from the keys alone.
  auto bucket_a = [&](uint64_t key) -> uint32_t {
    if constexpr (ONE) {
      return sub_of(key, plan);
    } else {
      key = key < kTombKey ? key : 0;  // reserved ids: any bucket (their slot becomes a hole)
      const int32_t jh = plan.nranks == 1 ? 0
                         : plan.hash_mode ? jhash_tab[key] : java_long_hash((int64_t)key);
      return kg_lds ? bucket_of(key, jh, plan, skg) : bucket_of(key, jh, plan, kg_dest);
    }
  };
  for (int64_t i0 = start; i0 < end; i0 += (int64_t)blockDim.x * kPartU) {
    uint64_t k[kPartU];
    if (i0 + (int64_t)blockDim.x * kPartU <= end) {
      // Full iteration (all but a group's last): no per-lane bounds checks.
#pragma unroll
      for (int u = 0; u < kPartU; u += (PAIR ? 2 : 1)) {
        if constexpr (PAIR) ldkey2<V, K32>(keys, ev_at(i0, u), k[u], k[u + 1]);
        else k[u] = ldkey<V, K32>(keys, ev_at(i0, u));
      }
#pragma unroll
      for (int u = 0; u < kPartU; ++u) atomicAdd(&run_base[bucket_a(k[u])], 1u);
      continue;
    }
    if constexpr (PAIR) {
#pragma unroll
      for (int u = 0; u < kPartU; u += 2) {
        const int64_t i = ev_at(i0, u);
        if (i + 1 < end) ldkey2<V, K32>(keys, i, k[u], k[u + 1]);
        else if (i < end) k[u] = ldkey<V, K32>(keys, i);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kPartU; ++u) {
        const int64_t i = ev_at(i0, u);
        if (i < end) k[u] = ldkey<V, K32>(keys, i);
      }
    }
#pragma unroll
    for (int u = 0; u < kPartU; ++u) {
      const int64_t i = ev_at(i0, u);
      if (i >= end) continue;
      atomicAdd(&run_base[bucket_a(k[u])], 1u);
    }
  }
  __syncthreads();
  bool overflow = false;
  uint32_t mb = 0;  // largest bucket fill seen by this group (the last reserver sees the total)
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const uint32_t c = (run_base[b] + (kCG - 1)) & ~(uint32_t)(kCG - 1);
    uint32_t base = 0;
    if (c) {
      base = atomicAdd(&cursor[b], c);
      if (base + c > plan.bucket_cap) overflow = true;
      mb = base + c > mb ? base + c : mb;
    }
    run_base[b] = base;
    resv[b] = c;
  }
  if (threadIdx.x == 0) {
    wsum[18] = 0;
    wsum[19] = 0;
  }
  __syncthreads();
  if (overflow) wsum[18] = 1;
  if (mb) atomicMax(&wsum[19], mb);
  __syncthreads();
  const bool any_ovf = wsum[18] != 0;
  // Max bucket fill of the step (stats): the host splits an oversized sub-table's aggregation
  // over several workgroups (hot keys, AggPlan.split).
  if (threadIdx.x == 0 && wsum[19])
    atomicMax((unsigned long long*)&stats[kStatMaxBucket], (unsigned long long)wsum[19]);
  const uint32_t bcap = plan.bucket_cap;

  int64_t tmax = INT64_MIN, nlate = 0, nacc = 0;
  uint32_t qmin32 = 0xFFFFFFFFu, qmax32 = 0;  // relative panes are u32: 32-bit min/max per event
  uint32_t pmask = 0;  // kStatPaneMask
  int64_t flags = 0;
  const bool pane32 = plan.window_mode && plan.pane > 0 && plan.pane < ((int64_t)1 << 31);
  const uint32_t pane_u = (uint32_t)plan.pane;
  // Pass B: rounds of (1024 * CU) records -> LDS counting sort by bucket -> cooperative run writes.
  // Software-pipelined: the next round's (key, ts, value) loads are issued before this round's
  // LDS sort and flush, so the HBM latency is not exposed once per round (16 rounds/group).
  uint64_t nk[CU], nv[CU];
  int64_t nt[CU];
  auto load_round = [&](int64_t base) {
    if constexpr (PAIR) {
#pragma unroll
      for (int u = 0; u < CU; u += 2) {
        const int64_t i = ev_at(base, u);
        if (i + 1 < end) {
          ldkey2<V, K32>(keys, i, nk[u], nk[u + 1]);
          uint64_t t0, t1;
          ld64x2<V>(ts, i, t0, t1);
          nt[u] = (int64_t)t0;
          nt[u + 1] = (int64_t)t1;
          ld64x2<V>(vals, i, nv[u], nv[u + 1]);
        } else if (i < end) {
          nk[u] = ldkey<V, K32>(keys, i);
          nt[u] = ldin<V>(&ts[i]);
          nv[u] = ldin<V>(&vals[i]);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int64_t i = ev_at(base, u);
        if (i < end) {
          nk[u] = ldkey<V, K32>(keys, i);
          nt[u] = ldin<V>(&ts[i]);
          nv[u] = ldin<V>(&vals[i]);
        }
      }
    }
  };
  load_round(start);
  for (int64_t r0 = start; r0 < end; r0 += (1024 * CU)) {
    uint32_t bk[CU], rk[CU];
    RT rec[CU];
    bool keep[CU];
    uint64_t ck[CU], cv[CU];
    int64_t ct[CU];
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      ck[u] = nk[u];
      ct[u] = nt[u];
      cv[u] = nv[u];
    }
    load_round(r0 + (1024 * CU));
    // Fast path: a full round whose events in this wave are all ordinary (valid key, not late,
    // relative pane in 32 bits) -- decided by one wave vote, then evaluated without per-lane
    // branches (PMC: the general path spent as many SALU as VALU instructions on exec-mask
    // bookkeeping). Record-width misfits only set flag bits (the host redoes the step).
    // (8-byte records only: the 16-byte kernels spill with both paths compiled in.)
    bool simple = RB == 8 && r0 + (1024 * CU) <= end && pane32 && !(plan.ablate & 8u);
    if (simple) {
      bool ok = true;
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int64_t d = ct[u] - plan.tbase;
        ok = ok && ck[u] < kTombKey && !(plan.drop_late && ct[u] < plan.late_ts) && d >= 0 &&
             d < ((int64_t)1 << 31);
      }
      simple = __all(ok);
    }
    if (RB == 8 && simple) {
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const uint64_t k = ck[u];
        const int64_t t = ct[u];
        const uint64_t v = cv[u];
        tmax = t > tmax ? t : tmax;
        const uint32_t du = (uint32_t)(t - plan.tbase);
        uint32_t q = (uint32_t)((double)du * plan.inv_pane);
        const uint32_t qp = q * pane_u;
        q = qp > du ? q - 1u : (du - qp >= pane_u ? q + 1u : q);
        qmin32 = q < qmin32 ? q : qmin32;
        pmask |= pane_bit(q);
        qmax32 = q > qmax32 ? q : qmax32;
        flags |= (int64_t)(int32_t)v != (int64_t)v ? 4 : 0;  // needs 24-byte records
        uint32_t b;
        if constexpr (ONE) {
          b = sub_of(k, plan);
        } else {
          const int32_t jh = plan.nranks == 1 ? 0
                             : plan.hash_mode ? jhash_tab[k] : java_long_hash((int64_t)k);
          b = kg_lds ? bucket_of(k, jh, plan, skg) : bucket_of(k, jh, plan, kg_dest);
        }
        keep[u] = true;
        bk[u] = b;
        if constexpr (RB == 8) {
          flags |= narrow_fits(k, (int64_t)v, q) ? 0 : 16;  // needs 16-byte records
          rec[u] = make_uint2((uint32_t)k, ((uint32_t)v << 4) | (q & 15u));
        } else {
          rec[u] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)v, q);
        }
        rk[u] = atomicAdd(&rcnt[b], 1u);
      }
    } else
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const int64_t i = ev_at(r0, u);
      keep[u] = false;
      if (i < end) {
        const uint64_t k = ck[u];
        const int64_t t = ct[u];
        const uint64_t v = cv[u];
        tmax = t > tmax ? t : tmax;
        const PartEval e = ONE      ? part_eval<true>(k, t, jhash_tab, plan, kg_dest)
                           : kg_lds ? part_eval(k, t, jhash_tab, plan, skg)
                                    : part_eval(k, t, jhash_tab, plan, kg_dest);
        if (e.kind == 1) {
          ++nlate;
          if (late_idx) {
            const unsigned long long pos = atomicAdd((unsigned long long*)&stats[kStatLate], 1ull);
            if (pos < late_cap) late_idx[pos] = (uint32_t)i;
          }
        } else if (e.kind >= 2) {
          flags |= e.kind == 2 ? 2 : 8;
        } else {
          if ((int64_t)(int32_t)v != (int64_t)v) flags |= 4;  // needs 24-byte records
          qmin32 = e.t < qmin32 ? e.t : qmin32;
          pmask |= pane_bit(e.t);
          qmax32 = e.t > qmax32 ? e.t : qmax32;
          keep[u] = true;
          bk[u] = e.bucket;
          if constexpr (RB == 8) {
            if (!narrow_fits(k, (int64_t)v, e.t)) flags |= 16;  // needs 16-byte records
            rec[u] = make_uint2((uint32_t)k, ((uint32_t)v << 4) | (e.t & 15u));
          } else {
            rec[u] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)v, e.t);
          }
          rk[u] = atomicAdd(&rcnt[e.bucket], 1u);
        }
      }
    }
    __syncthreads();
    const uint32_t myc = threadIdx.x < (unsigned)nb ? rcnt[threadIdx.x] : 0u;
    const uint32_t off = block_exclusive_scan(myc, wsum);
    if (threadIdx.x < (unsigned)nb) {
      roff[threadIdx.x] = off;
      // Record j of this round (bucket b) goes to out[b * bcap + run_base[b] + lcnt[b] + j -
      // roff[b]]: one per-bucket base (mod 2^32) so the flush does one LDS lookup per record.
      dbase[threadIdx.x] = threadIdx.x * bcap + run_base[threadIdx.x] + lcnt[threadIdx.x] - off;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < CU; ++u)
      if (keep[u]) {
        const uint32_t j = roff[bk[u]] + rk[u];
        rbuf[j] = rec[u];
        sbk[j] = (uint16_t)bk[u];
      }
    __syncthreads();
    const uint32_t nrec = wsum[16];
    nacc += threadIdx.x == 0 ? nrec : 0u;
    if (!any_ovf) {
      RT* outr = (RT*)out;
      for (uint32_t j = threadIdx.x; j < nrec; j += blockDim.x) outr[dbase[sbk[j]] + j] = rbuf[j];
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)nb) {
      lcnt[threadIdx.x] += rcnt[threadIdx.x];
      rcnt[threadIdx.x] = 0;
    }
    __syncthreads();
  }
  // Tail: holes in the reserved slots that no record filled (padding to a whole sector, and the
  // slots counted for late / dropped records in pass A).
  if (threadIdx.x < (unsigned)nb && !any_ovf) {
    const int b = threadIdx.x;
    RT* dst = (RT*)out + (size_t)b * bcap + run_base[b];
    RT hole;
    if constexpr (RB == 8) hole = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    else hole = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, kHoleT);
    for (uint32_t w = lcnt[b]; w < resv[b]; ++w) dst[w] = hole;
  }

  int64_t qmin = qmin32 == 0xFFFFFFFFu && qmax32 == 0 ? INT64_MAX : (int64_t)qmin32;
  int64_t qmax = qmin == INT64_MAX ? INT64_MIN : (int64_t)qmax32;
  tmax = block_reduce_i64(tmax, lred, 0);
  qmin = block_reduce_i64(qmin, lred, 1);
  qmax = block_reduce_i64(qmax, lred, 0);
  pmask = (uint32_t)block_reduce_i64(pmask, lred, 3);
  if (!late_idx) nlate = block_reduce_i64(nlate, lred, 2);
  flags = (any_ovf ? 1 : 0) | block_reduce_i64(flags & 2, lred, 0) |
          block_reduce_i64(flags & 4, lred, 0) | block_reduce_i64(flags & 8, lred, 0) |
          (RB == 8 ? block_reduce_i64(flags & 16, lred, 0) : 0);
  if (threadIdx.x == 0) {
    atomicMax((long long*)&stats[kStatMaxTs], (long long)tmax);
    if (nacc) {
      atomicMin((long long*)&stats[kStatMinPane], (long long)qmin);
      atomicMax((long long*)&stats[kStatMaxPane], (long long)qmax);
      atomicAdd((unsigned long long*)&stats[kStatAccepted], (unsigned long long)nacc);
      if (pmask) atomicOr((unsigned long long*)&stats[kStatPaneMask], (unsigned long long)pmask);
    }
    if (!late_idx && nlate) atomicAdd((unsigned long long*)&stats[kStatLate], (unsigned long long)nlate);
    if (flags) atomicOr((unsigned long long*)&stats[kStatOverflow], (unsigned long long)flags);
  }
}

// Step prologue: zero the bucket cursors and reset the stats block (one launch instead of two
// memsets + a host copy).
__global__ __launch_bounds__(256) void step_begin_kernel(uint32_t* __restrict__ cursor, int nb,
                                                         int64_t* __restrict__ stats) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x)
    cursor[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x < kStatCount) {
    const int j = threadIdx.x;
    stats[j] = j == kStatMaxTs ? INT64_MIN : j == kStatMinPane ? INT64_MAX
             : j == kStatMaxPane ? INT64_MIN : 0;
  }
}

// Step epilogue: fold this batch into the source partition's watermark and build the vector
// the watermark valve all-reduces (MIN): [-max pane, min pane, wm, -bucket ovf, -pane ovf] plus
// a copy of the raw stats for the host (red[8..15]).
__global__ void step_finish_kernel(const int64_t* __restrict__ stats, int64_t* __restrict__ local_maxts,
                                   int64_t bound, int32_t event_mode, int64_t proc_now,
                                   int64_t* __restrict__ red, const uint32_t* __restrict__ flags,
                                   int32_t idle, int64_t* __restrict__ host_red, int32_t fill_word,
                                   const uint32_t* __restrict__ cursor, int nb,
                                   uint32_t* __restrict__ next_cursor,
                                   int64_t* __restrict__ next_stats) {
  // A later step's cursors and stats (distinct buffers): step_begin's work, in this launch.
  if (next_cursor) {
    for (int i = threadIdx.x; i < nb; i += blockDim.x) next_cursor[i] = 0;
    if (threadIdx.x < kStatCount) {
      const int j = threadIdx.x;
      next_stats[j] = j == kStatMaxTs ? INT64_MIN : j == kStatMinPane ? INT64_MAX
                    : j == kStatMaxPane ? INT64_MIN : 0;
    }
  }
  // fill_word: the largest bucket fill, from the cursors (every partition variant fills them)
  __shared__ uint32_t fmax[64];
  if (fill_word) {
    uint32_t m = 0;
    for (int i = threadIdx.x; i < nb; i += 64) m = cursor[i] > m ? cursor[i] : m;
    fmax[threadIdx.x] = m;
    __syncthreads();
    for (int s = 32; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s && fmax[threadIdx.x + s] > fmax[threadIdx.x])
        fmax[threadIdx.x] = fmax[threadIdx.x + s];
      __syncthreads();
    }
  }
  // One lane per word of the reduced vector (16 words).
  const int j = threadIdx.x;
  if (j >= 16) return;
  int64_t lm = local_maxts[0];
  const int64_t bm = stats[kStatMaxTs];
  lm = bm > lm ? bm : lm;
  if (j == 0) local_maxts[0] = lm;
  const int64_t wm = event_mode ? (lm == INT64_MIN ? INT64_MIN : lm - bound) : proc_now;
  const int64_t ovf = stats[kStatOverflow];
  int64_t v;
  switch (j) {
    case 0: {
      const int64_t qmax = stats[kStatMaxPane];
      v = qmax == INT64_MIN ? INT64_MAX : -qmax;
      break;
    }
    case 1: v = stats[kStatMinPane]; break;
    case 2: v = idle ? INT64_MAX : wm; break;  // an idle partition has no say in the MIN
    case 3:
      v = !fill_word ? -(ovf & 1) : (ovf & 1) ? -((int64_t)1 << 40) : -(int64_t)fmax[0];
      break;
    case 4: v = -((ovf >> 1) & 1); break;
    // Record width a value needs: -2 = 24-byte records, -1 = 16-byte records, 0 = as planned.
    case 5: v = (ovf & 4) ? -2 : (ovf & 16) ? -1 : 0; break;
    case 6: v = flags ? -(int64_t)(flags[0] & 1u) : 0; break;  // a key found no slot, sticky
    case 7: v = -((ovf >> 3) & 1); break;  // the reserved key id ~0 occurred
    default: v = stats[j - 8]; break;
  }
  red[j] = v;
  if (host_red) host_red[j] = v;  // vector store into the mapped pinned buffer
}

__global__ __launch_bounds__(256) void combine_check_kernel(const uint32_t* __restrict__ flags,
                                                            const uint32_t* __restrict__ counts,
                                                            int nb, int64_t* __restrict__ chk) {
  __shared__ uint32_t mx[256];
  __shared__ uint64_t sm[256];
  uint32_t m = 0;
  uint64_t sum = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    m = counts[i] > m ? counts[i] : m;
    sum += counts[i];
  }
  mx[threadIdx.x] = m;
  sm[threadIdx.x] = sum;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      if (mx[threadIdx.x + s] > mx[threadIdx.x]) mx[threadIdx.x] = mx[threadIdx.x + s];
      sm[threadIdx.x] += sm[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    chk[0] = -(int64_t)(flags[0] & 2u);
    chk[1] = -(int64_t)mx[0];
    chk[2] = (int64_t)sm[0];  // records combined on this rank (payload accounting; not reduced)
  }
}

// One workgroup per bucket: the bucket's records (words u64 each) copied as 16-byte vectors where
// the whole run is 16-byte aligned (rec words even or stride-aligned), else word by word.
__global__ __launch_bounds__(256) void bucket_repack_kernel(const uint64_t* __restrict__ src,
                                                            const uint32_t* __restrict__ counts,
                                                            uint32_t src_cap, uint32_t dst_cap,
                                                            int words, uint64_t* __restrict__ dst,
                                                            unsigned long long* __restrict__ xstat) {
  const int b = blockIdx.x;
  const uint32_t c = counts[b] < dst_cap ? counts[b] : dst_cap;
  const uint64_t* s = src + (size_t)b * src_cap * words;
  uint64_t* d = dst + (size_t)b * dst_cap * words;
  const size_t nw = (size_t)c * words;
  if (!(((uintptr_t)s | (uintptr_t)d) & 15)) {
    const size_t nv = nw / 2;
    const uint4* s4 = (const uint4*)s;
    uint4* d4 = (uint4*)d;
    for (size_t i = threadIdx.x; i < nv; i += blockDim.x) d4[i] = s4[i];
    if ((nw & 1) && threadIdx.x == 0) d[nw - 1] = s[nw - 1];
  } else {
    for (size_t i = threadIdx.x; i < nw; i += blockDim.x) d[i] = s[i];
  }
  if (xstat && threadIdx.x == 0) {
    atomicAdd(&xstat[1], (unsigned long long)nw * 8ull);
    atomicAdd(&xstat[0], (unsigned long long)dst_cap * words * 8ull);
  }
}

__global__ __launch_bounds__(256) void neg_max_u32_kernel(const uint32_t* __restrict__ counts, int nb,
                                                          int64_t* __restrict__ out) {
  __shared__ uint32_t mx[256];
  uint32_t m = 0;
  for (int i = threadIdx.x; i < nb; i += 256) m = counts[i] > m ? counts[i] : m;
  mx[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s && mx[threadIdx.x + s] > mx[threadIdx.x]) mx[threadIdx.x] = mx[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = -(int64_t)mx[0];
}

__global__ __launch_bounds__(256) void widen_i32_kernel(const int32_t* __restrict__ in, int64_t n,
                                                        int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int64_t)in[i];
}

// Grid-stride zeroing of three byte ranges in one launch (the purge of a run of pane slabs).
__global__ __launch_bounds__(256) void zero3_kernel(uint4* __restrict__ a, int64_t na,
                                                    uint4* __restrict__ b, int64_t nb,
                                                    uint4* __restrict__ c, int64_t nc) {
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb + nc; i += stride) {
    if (i < na) a[i] = z;
    else if (i < na + nb) b[i - na] = z;
    else c[i - na - nb] = z;
  }
}

__global__ __launch_bounds__(256) void fill_u64_kernel(uint64_t* __restrict__ p, int64_t n, uint64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// ------------------------------------------------------------------------------------------
// LDS hash sub-table helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_probe_insert(uint64_t* skeys, uint64_t key, uint32_t mask,
                                                     int* inserted) {
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    // Relaxed workgroup-scope atomic load, not a volatile read: the volatile cast made the
    // access generic (flat_load ... sc0 sc1 + s_waitcnt vmcnt(0)), which waited for every
    // record load in flight before each probe.
    const uint64_t k = __hip_atomic_load(&skeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == key) return s;
    if (k == kEmptyKey) {
      const uint64_t prev = atomicCAS((unsigned long long*)&skeys[s], (unsigned long long)kEmptyKey,
                                      (unsigned long long)key);
      if (prev == kEmptyKey) {
        *inserted = 1;
        return s;
      }
      if (prev == key) return s;
    }
    s = (s + 1) & mask;
  }
  return kNoSlot;
}

// lds_probe_insert with four slots per step: the four relaxed 64-bit loads of s..s+3 are
// independent, so a probe costs one LDS round trip per four slots instead of one per slot --
// and a wave's lanes, which wait for the longest probe among them, do ~4x fewer dependent
// rounds (hashed window_agg: 160 us per 16.7M events with the one-slot loop). Same slot order
// and CAS protocol as the one-slot loop: a slot read as empty but taken meanwhile fails its CAS
// and the scan goes on, so the table layout is unchanged.
__device__ __forceinline__ uint32_t lds_probe_insert4(uint64_t* skeys, uint64_t key,
                                                      uint32_t mask, int* inserted) {
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; i += 4) {
    uint64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      k[u] = __hip_atomic_load(&skeys[(s + u) & mask], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i + u > mask) return kNoSlot;  // every slot seen
      const uint32_t j = (s + u) & mask;
      if (k[u] == key) return j;
      if (k[u] == kEmptyKey) {
        const uint64_t prev = atomicCAS((unsigned long long*)&skeys[j],
                                        (unsigned long long)kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey) {
          *inserted = 1;
          return j;
        }
        if (prev == key) return j;
      }
    }
    s = (s + 4) & mask;
  }
  return kNoSlot;
}

// 32-bit key ids (8-byte RecN records) in a table private to one kernel (the sender-side
// combiner): slots in aligned groups of four, one 16-byte LDS read per group, groups probed
// linearly. Half the LDS bytes per key and one read instruction per four slots (PMC of the G = 8
// records path: combiner bank-conflict cycles 1.65x its active LDS cycles with 64-bit keys).
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t lds_probe_insert_g4(uint32_t* sk, uint32_t key, uint32_t mask,
                                                        int* inserted) {
  uint32_t g = slot_hash((uint64_t)key) & mask & ~3u;
  for (uint32_t i = 0; i <= mask; i += 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(&sk[g]);
    const uint32_t k[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k[u] == key) return g + u;
      if (k[u] == kEmpty32) {
        const uint32_t prev = atomicCAS(&sk[g + u], kEmpty32, key);
        if (prev == kEmpty32) {
          *inserted = 1;
          return g + u;
        }
        if (prev == key) return g + u;
      }
    }
    g = (g + 4) & mask;
  }
  return kNoSlot;
}

template <int AGG>
__device__ __forceinline__ int64_t lds_identity() {
  if (AGG == AGG_MIN_I64 || AGG == AGG_MIN_F64) return INT64_MAX;
  if (AGG == AGG_MAX_I64 || AGG == AGG_MAX_F64) return INT64_MIN;
  return 0;
}

template <int AGG>
__device__ __forceinline__ void lds_accumulate(uint64_t* a, uint64_t v) {
  if (AGG == AGG_SUM_I64 || AGG == AGG_AVG_I64) {
    atomicAdd((unsigned long long*)a, (unsigned long long)v);
  } else if (AGG == AGG_SUM_F64 || AGG == AGG_AVG_F64) {
    atomicAdd((double*)a, as_f64(v));
  } else if (AGG == AGG_MIN_I64) {
    atomicMin((long long*)a, (long long)v);
  } else if (AGG == AGG_MAX_I64) {
    atomicMax((long long*)a, (long long)v);
  } else if (AGG == AGG_MIN_F64) {
    atomicMin((long long*)a, (long long)f64_ord(v));
  } else if (AGG == AGG_MAX_F64) {
    atomicMax((long long*)a, (long long)f64_ord(v));
  }
  // AGG_COUNT: the count array carries it.
}

template <int AGG>
__device__ __forceinline__ uint64_t lds_export(uint64_t a) {
  if (AGG == AGG_MIN_F64 || AGG == AGG_MAX_F64) return f64_unord((int64_t)a);
  if (AGG == AGG_COUNT) return 0;
  return a;
}

// ------------------------------------------------------------------------------------------
// Keyed window aggregation: one workgroup per sub-table.
// LDS image (dynamic, 16-B aligned): keys[cap] u64 | acc[pg][cap] u64 | cnt[pg][cap] u32 | flag
// ------------------------------------------------------------------------------------------
constexpr int kAggU = 4;  // 8 measured equal (162.7 vs 162.1 us, profiles/r1_window_agg_ab.md)

// Record load for both layouts: RW = 3 (24-byte Rec) or 2 (16-byte RecC, int32 value).
template <int RW>
__device__ __forceinline__ Rec load_rec(const void* base, size_t idx) {
  if (RW == 3) return ((const Rec*)base)[idx];
  if (RW == 1) {  // narrow 8-byte record
    const uint2 c = ((const uint2*)base)[idx];
    Rec r;
    r.key = c.x;
    r.val = (uint64_t)(int64_t)((int32_t)c.y >> 4);
    r.t = (c.y & 15u) == kNarrowHoleT ? 0xFFFFFFFFu : (c.y & 15u);
    r.aux = 0;
    return r;
  }
  const uint4 c = ((const uint4*)base)[idx];
  Rec r;
  r.key = (uint64_t)c.x | ((uint64_t)c.y << 32);
  r.val = (uint64_t)(int64_t)(int32_t)c.z;
  r.t = c.w;
  r.aux = 0;
  return r;
}

// Materialise a loaded record in registers at this point (empty asm that "modifies" every
// field). Without it LLVM narrowed the 16-byte record load and sank the key half into the
// per-record branch, where its s_waitcnt vmcnt(0) also waited for the other records in flight.
template <int RW>
__device__ __forceinline__ void pin_rec(Rec& r) {
  asm volatile("" : "+v"(r.key), "+v"(r.val), "+v"(r.t), "+v"(r.aux));
}

// Packed (sum, count) accumulator for integer sums of int32 values (PK = true): one LDS word
// P = sum_i (v_i + 2^48) mod 2^64 holds both the 48-bit signed sum and the 16-bit count, so a
// record costs one LDS atomic instead of two and a pane row 8 bytes instead of 12. Exact while
// |sum| < 2^47 and count < 2^16, guaranteed by the host (int32 values, < 65536 records per
// sub-table and step). An untouched slot stays 0 (a touched one cannot be 0: |sum| < 2^47).
constexpr uint64_t kPkOne = 1ull << 48;
__device__ __forceinline__ int64_t pk_sum(uint64_t p) {
  return (int64_t)(p << 16) >> 16;
}
__device__ __forceinline__ uint32_t pk_cnt(uint64_t p) {
  return (uint32_t)((p - (uint64_t)pk_sum(p)) >> 48);
}

// DENSE: directly addressed dense key ids (AggPlan.dense_bits): no LDS key table, no probe.
constexpr uint32_t kAggSliceMin = 131072;  // records per workgroup of a split sub-table

// V (8-byte packed path only, A/B via MXS_AGG_V): bit 0 = eight record loads in flight per
// thread instead of four; bit 1 = at most 64 VGPRs (launch bounds of eight waves per SIMD), so two
// 1024-thread workgroups fit one CU when their LDS images do.
template <int AGG, int RW, bool PK = false, bool DENSE = false, bool DET = false, int V = 0>
__global__ __launch_bounds__(1024, (V & 2) ? 8 : 1) void window_agg_kernel(
    const void* __restrict__ recs, const uint32_t* __restrict__ counts, AggPlan p,
    uint64_t* __restrict__ keys_g, uint64_t* __restrict__ acc_g, uint32_t* __restrict__ cnt_g,
    uint8_t* __restrict__ dirty_g, uint32_t* __restrict__ occupancy, uint32_t* __restrict__ flags) {
  static_assert(!PK || ((AGG == AGG_SUM_I64 || AGG == AGG_AVG_I64) && RW <= 2),
                "packed accumulators: integer sum/avg of 8/16-byte records only");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // Split sub-tables (AggPlan.split, hot keys): workgroup `slice` of `split` takes an equal
  // share of the sub-table's records; the shares merge into the state with atomic adds.
  if (p.skip && *p.skip) return;  // incomplete exchange: redone by the host (AggPlan.skip)
  // split < 0: every sub-table over -split workgroups (forced, AggPlan.split).
  const int split = p.split < 0 ? -p.split : p.split;  // launcher: 1 unless the layout allows it
  const int sub = split > 1 ? (int)blockIdx.x / split : (int)blockIdx.x;
  const int slice = split > 1 ? (int)blockIdx.x % split : 0;
  int nact = 1;
  if (split > 1) {
    uint32_t ca = counts[sub];
    ca = ca < p.bucket_cap ? ca : p.bucket_cap;
    nact = p.split < 0 ? split : (int)((ca + kAggSliceMin - 1) / kAggSliceMin);
    nact = nact < 1 ? 1 : nact > split ? split : nact;
    if (slice >= nact) return;  // workgroup-uniform: before any barrier
  }
  const bool shared_sub = nact > 1;
  const uint32_t cap = 1u << p.cap_log2;
  const uint32_t mask = cap - 1;
  uint64_t* skeys = (uint64_t*)smem;                   // unused when DENSE
  uint64_t* sacc = DENSE ? (uint64_t*)smem : skeys + cap;
  // DET: two words per slot (128-bit fixed-point sum, f64_to_fx), see AggPlan.det.
  uint32_t* scnt = (uint32_t*)(sacc + (size_t)p.pg * cap * (DET ? 2 : 1));  // unused when PK
  int* sflag = (int*)(scnt + (PK ? 0 : (size_t)p.pg * cap));  // [0] inserted, [1] ovf, [2] occ

  const size_t sbase = (size_t)sub << p.cap_log2;
  const size_t nslots = (size_t)p.nsub << p.cap_log2;
  if constexpr (!DENSE)
    for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) skeys[i] = keys_g[sbase + i];
  if (threadIdx.x < 4) sflag[threadIdx.x] = 0;
  // Touched-slot list (late-but-allowed data): an LDS bitmap dedupes the sub-table's slots
  // across pane passes and an LDS buffer collects them; one global atomic per workgroup at the
  // end reserves the run in the list (a per-wave atomic on one global counter and a returning
  // global atomic per late row made the late steps of config 4 4.7x slower).
  uint32_t* sdl_hdr = (uint32_t*)(sflag + 4);  // [0] listed slots, [1] list base
  uint32_t* sbit = sdl_hdr + 4;                // [cap / 32] listed bits
  uint32_t* sdl = sbit + (cap >> 5);           // [cap] listed slot offsets
  if (p.dlist) {
    if (threadIdx.x < 4) sdl_hdr[threadIdx.x] = 0;
    for (uint32_t i = threadIdx.x; i < (cap >> 5); i += blockDim.x) sbit[i] = 0;
  }

  // Sparse pane rows (AggPlan.pmask): LDS row j of the step holds relative pane srel[j].
  __shared__ int32_t srel[32];
  const bool sparse = p.pmask != 0u && !(p.pmask >> 31);
  if (sparse && threadIdx.x == 0) {
    int j = 0;
    for (int b = 0; b < 31; ++b)
      if (p.pmask >> b & 1u) srel[j++] = b;
  }
  int inserted = 0;
  bool ovf = false, fxbad = false;
  for (int pg0 = 0; pg0 < p.np_step; pg0 += p.pg) {
    const int npg = (p.np_step - pg0) < p.pg ? (p.np_step - pg0) : p.pg;
    for (uint32_t i = threadIdx.x; i < (uint32_t)npg * cap; i += blockDim.x) {
      if (DET) {
        sacc[2 * i] = 0;
        sacc[2 * i + 1] = 0;
      } else {
        sacc[i] = PK ? 0ull : (uint64_t)lds_identity<AGG>();
      }
      if (!PK) scnt[i] = 0;
    }
    __syncthreads();
    const int64_t q0 = p.p_lo + pg0;  // relative pane of LDS row 0
    for (int src = 0; src < p.nsrc; ++src) {
      uint32_t c = counts[(size_t)src * p.nsub + sub];
      c = c < p.bucket_cap ? c : p.bucket_cap;
      const size_t seg0 = ((size_t)src * p.nsub + sub) * p.bucket_cap;
      // This workgroup's share [e_lo, c) of the segment (all of it unless split).
      const uint32_t e_lo = shared_sub ? (uint32_t)((uint64_t)c * slice / nact) : 0u;
      if (shared_sub) c = (uint32_t)((uint64_t)c * (slice + 1) / nact);
      // kU independent record loads in flight per thread before the LDS work.
      constexpr int kU = (V & 1) ? 8 : kAggU;
      for (uint32_t e0 = e_lo + threadIdx.x; e0 < c; e0 += blockDim.x * kU) {
        Rec rr[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t e = e0 + u * blockDim.x;
          // Branch-free: a load under `if (e < c)` made the compiler wait for each load at the
          // branch join (s_waitcnt vmcnt(0) after every load: no loads in flight at all).
          // Lanes past the end re-read the last record and skip it below.
          rr[u] = load_rec<RW>(recs, seg0 + (e < c ? e : c - 1));
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) pin_rec<RW>(rr[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t e = e0 + u * blockDim.x;
          if (e >= c) break;
          const Rec& r = rr[u];
          if (r.t == 0xFFFFFFFFu) continue;  // hole record (staged partition padding)
          const int64_t q = sparse ? (r.t < 31u ? (int64_t)__popc(p.pmask & ((1u << r.t) - 1u)) - pg0 : -1)
                                   : (int64_t)r.t - q0;
          if (q < 0 || q >= npg) continue;
          uint32_t s;
          if constexpr (DENSE) {
            if (r.key >> p.dense_bits) {  // id outside the dense key space: table full
              ovf = true;
              continue;
            }
            s = dense_slot(r.key, p.dense_mul, p.dense_bits) & mask;
          } else {
            s = lds_probe_insert4(skeys, r.key, mask, &inserted);
            if (s == kNoSlot) {
              ovf = true;
              continue;
            }
          }
          const uint32_t li = (uint32_t)q * cap + s;
          if (DET) {
            uint64_t lo, hi;
            if (!f64_to_fx(as_f64(r.val), &lo, &hi)) {
              fxbad = true;
              continue;
            }
            // 128-bit add from two 64-bit LDS atomics: the carry out of the low word goes into
            // the high word (two's complement, so the final sum is order-independent).
            const uint64_t old = atomicAdd((unsigned long long*)&sacc[2 * li], (unsigned long long)lo);
            atomicAdd((unsigned long long*)&sacc[2 * li + 1],
                      (unsigned long long)(hi + (old + lo < old ? 1ull : 0ull)));
            atomicAdd(&scnt[li], p.combined ? r.aux : 1u);
          } else if (PK) {
            atomicAdd((unsigned long long*)&sacc[li], (unsigned long long)(r.val + kPkOne));
          } else {
            lds_accumulate<AGG>(&sacc[li], r.val);
            atomicAdd(&scnt[li], p.combined ? r.aux : 1u);
          }
        }
      }
    }
    __syncthreads();
    // Write back the deltas of touched slots (this workgroup owns these slots: plain RMW).
    // kWB slots per thread per batch: all their state loads are issued before the first
    // combine, so the read-modify-write costs one memory latency per batch instead of one per
    // slot (a slot-at-a-time loop serialised 8 dependent HBM round trips per thread).
    constexpr int kWB = (V & 2) ? 4 : 8;  // V bit 1: fewer registers (64-VGPR variant)
    const uint32_t nrow = (uint32_t)npg * cap;
    for (uint32_t i0 = threadIdx.x; i0 < nrow; i0 += blockDim.x * kWB) {
      uint32_t dc[kWB], oc[kWB];
      uint64_t oa[kWB];
      size_t gi[kWB];
#pragma unroll
      for (int w = 0; w < kWB; ++w) {
        const uint32_t i = i0 + (uint32_t)w * blockDim.x;
        dc[w] = i < nrow ? (PK ? pk_cnt(sacc[i]) : scnt[i]) : 0u;
        oc[w] = 0;
        oa[w] = 0;
        gi[w] = 0;
        if (dc[w]) {
          const int64_t pane = p.pane_base + (sparse ? (int64_t)srel[pg0 + (i >> p.cap_log2)]
                                                     : q0 + (int64_t)(i >> p.cap_log2));
          gi[w] = (size_t)(pane & (p.ring - 1)) * nslots + sbase + (i & mask);
          if (!shared_sub) {
            oc[w] = cnt_g[gi[w]];
            if (AGG != AGG_COUNT) oa[w] = acc_g[gi[w]];
          }
        }
      }
      bool late[kWB];
#pragma unroll
      for (int w = 0; w < kWB; ++w) {
        late[w] = false;
        if (!dc[w]) continue;
        const uint32_t i = i0 + (uint32_t)w * blockDim.x;
        const uint64_t d = DET ? f64_bits(fx_to_f64(sacc[2 * i], sacc[2 * i + 1]))
                           : PK ? (uint64_t)pk_sum(sacc[i]) : lds_export<AGG>(sacc[i]);
        if (shared_sub) {
          // Additive aggregates only (launcher): an empty slot's accumulator is 0.
          if (AGG != AGG_COUNT) atomicAdd((unsigned long long*)&acc_g[gi[w]], (unsigned long long)d);
          atomicAdd(&cnt_g[gi[w]], dc[w]);
        } else {
          if (AGG != AGG_COUNT) acc_g[gi[w]] = oc[w] ? agg_combine(AGG, oa[w], d) : d;
          cnt_g[gi[w]] = oc[w] + dc[w];
        }
        if (p.pane_base + (sparse ? (int64_t)srel[pg0 + (i >> p.cap_log2)]
                                  : q0 + (int64_t)(i >> p.cap_log2)) <= p.fired_hi) {
          dirty_g[gi[w]] = 1;
          late[w] = true;
          if (p.dacc) {  // local-global delta ring (this workgroup owns the slot: plain RMW)
            const uint32_t odc = p.dcnt[gi[w]];
            if (AGG != AGG_COUNT) p.dacc[gi[w]] = odc ? agg_combine(AGG, p.dacc[gi[w]], d) : d;
            p.dcnt[gi[w]] = odc + dc[w];
          }
        }
      }
      if (p.dlist) {
#pragma unroll
        for (int w = 0; w < kWB; ++w) {
          if (!late[w]) continue;
          const uint32_t s = (i0 + (uint32_t)w * blockDim.x) & mask;
          const uint32_t bit = 1u << (s & 31u);
          if (!(atomicOr(&sbit[s >> 5], bit) & bit)) sdl[atomicAdd(&sdl_hdr[0], 1u)] = s;
        }
      }
    }
    __syncthreads();
  }
  if (inserted) sflag[0] = 1;
  if (ovf) sflag[1] = 1;
  if (fxbad) sflag[3] = 1;
  __syncthreads();
  if (threadIdx.x == 0 && sflag[3]) atomicOr(&flags[0], 8u);  // DET: value outside fixed point
  if (p.dlist && sdl_hdr[0]) {
    if (threadIdx.x == 0) sdl_hdr[1] = atomicAdd(p.dlist_n, sdl_hdr[0]);
    __syncthreads();
    const uint32_t nl = sdl_hdr[0], base = sdl_hdr[1];
    for (uint32_t j = threadIdx.x; j < nl; j += blockDim.x) p.dlist[base + j] = (uint32_t)(sbase + sdl[j]);
  }
  if (sflag[0]) {
    for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
      const uint64_t k = skeys[i];
      keys_g[sbase + i] = k;
      if (k != kEmptyKey) atomicAdd(&sflag[2], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) occupancy[sub] = (uint32_t)sflag[2];
  }
  if (threadIdx.x == 0 && sflag[1]) atomicOr(&flags[0], 1u);
}

// ------------------------------------------------------------------------------------------
// Experiment (profiles/r2_direct_atomics.md): pane accumulation by global atomics straight from
// the source columns (dense ids, one rank), no partition. mode 0: sum + count atomics; 1: sum
// atomic only; 2: no atomics (loads + pane/slot math only, a checksum keeps it alive).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void direct_agg_probe_kernel(
    const uint64_t* __restrict__ keys, const int64_t* __restrict__ ts,
    const uint64_t* __restrict__ vals, int64_t n, int64_t tbase, int64_t pane, int ring,
    int64_t nslots, uint32_t mul, int bits, int64_t pane_base, uint64_t* __restrict__ acc_g,
    uint32_t* __restrict__ cnt_g, int mode, uint64_t* __restrict__ sink) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint64_t chk = 0;
  const double inv = 1.0 / (double)pane;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t k = __builtin_nontemporal_load(&keys[i]);
    const int64_t t = __builtin_nontemporal_load(&ts[i]);
    const uint64_t v = __builtin_nontemporal_load(&vals[i]);
    const int64_t q = (int64_t)((double)(t - tbase) * inv);
    const int64_t p = pane_base + q;
    const size_t gi = (size_t)(p & (ring - 1)) * nslots + dense_slot(k, mul, bits);
    if (mode == 0) {
      atomicAdd((unsigned long long*)&acc_g[gi], (unsigned long long)v);
      atomicAdd(&cnt_g[gi], 1u);
    } else if (mode == 1) {
      atomicAdd((unsigned long long*)&acc_g[gi], (unsigned long long)v);
    } else {
      chk += gi ^ v;
    }
  }
  if (mode == 2 && chk == 0x1234567) sink[0] = chk;
}

// ------------------------------------------------------------------------------------------
// Keyed-window table maintenance for the host-DRAM spill tier (hashed keys): one workgroup per
// sub-table. A key with no data in the live panes is dropped (the tables never delete keys
// otherwise); a key whose newest data pane is <= cutoff is evicted: its live (pane, acc, cnt,
// dirty) rows go to the host tier. The kept keys are re-inserted into a fresh LDS table (no
// tombstones: window_agg's probe stays a plain linear probe) and each live pane's slice is
// permuted through LDS to the new positions.
// LDS: old keys | new keys | pane acc [cap] u64, then from-slot | pane cnt [cap] u32, dirty [cap].
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void window_compact_kernel(
    uint64_t* __restrict__ keys_g, uint64_t* __restrict__ acc_g, uint32_t* __restrict__ cnt_g,
    uint8_t* __restrict__ dirty_g, int cap_log2, int ring, int64_t nslots, int64_t p_lo, int np,
    int64_t cutoff, CompactOut out, uint32_t* __restrict__ occupancy) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t cap = 1u << cap_log2, mask = cap - 1;
  const size_t sbase = (size_t)blockIdx.x << cap_log2;
  uint64_t* sold = (uint64_t*)smem;
  uint64_t* snew = sold + cap;
  uint64_t* sacc = snew + cap;
  uint32_t* sfrom = (uint32_t*)(sacc + cap);
  uint32_t* scnt = sfrom + cap;
  uint8_t* sdirty = (uint8_t*)(scnt + cap);
  uint32_t* sc = (uint32_t*)(sdirty + cap);  // [0] dropped, [1] evicted, [2] overflow, [3] kept
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
    sold[i] = keys_g[sbase + i];
    snew[i] = kEmptyKey;
    sfrom[i] = kNoSlot;
  }
  if (threadIdx.x < 6) sc[threadIdx.x] = 0;
  __syncthreads();
  // Evicted keys' rows: counted and placed inside the block first (LDS cursor sc[4], the slot's
  // run start + 1 kept in scnt[s], which the permutation below overwrites), then ONE device-scope
  // atomic reserves the block's run in the output (a same-address atomic per row serialises
  // across the XCDs).
  for (uint32_t s = threadIdx.x; s < cap; s += blockDim.x) scnt[s] = 0;
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < cap; s += blockDim.x) {
    const uint64_t k = sold[s];
    if (k == kEmptyKey || k == kTombKey) continue;
    int64_t newest = INT64_MIN;
    uint32_t nrows = 0;
    for (int j = 0; j < np; ++j) {
      const int64_t p = p_lo + j;
      if (cnt_g[(size_t)(p & (ring - 1)) * nslots + sbase + s]) {
        newest = p;
        ++nrows;
      }
    }
    if (newest == INT64_MIN) {
      atomicAdd(&sc[0], 1u);
      continue;
    }
    if (newest <= cutoff) {
      atomicAdd(&sc[1], 1u);
      scnt[s] = atomicAdd(&sc[4], nrows) + 1u;
      continue;
    }
    int ins = 0;
    const uint32_t t = lds_probe_insert(snew, k, mask, &ins);
    if (t == kNoSlot) {
      atomicOr(&sc[2], 1u);
      continue;
    }
    sfrom[t] = s;
    atomicAdd(&sc[3], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) sc[5] = sc[4] ? atomicAdd(out.n, sc[4]) : 0u;
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < cap; s += blockDim.x) {
    const uint32_t o1 = scnt[s];
    if (!o1) continue;
    const uint64_t k = sold[s];
    uint32_t q = sc[5] + o1 - 1;
    for (int j = 0; j < np; ++j) {
      const int64_t p = p_lo + j;
      const size_t gi = (size_t)(p & (ring - 1)) * nslots + sbase + s;
      const uint32_t c = cnt_g[gi];
      if (!c) continue;
      if (q < out.cap) {
        out.key[q] = k;
        out.pane[q] = p;
        out.acc[q] = acc_g[gi];
        out.cnt[q] = c;
        out.dirty[q] = dirty_g[gi];
      } else {
        atomicOr(&sc[2], 1u);
      }
      ++q;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) keys_g[sbase + i] = snew[i];
  for (int j = 0; j < np; ++j) {
    const size_t pb = (size_t)((p_lo + j) & (ring - 1)) * nslots + sbase;
    for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
      sacc[i] = acc_g[pb + i];
      scnt[i] = cnt_g[pb + i];
      sdirty[i] = dirty_g[pb + i];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
      const uint32_t f = sfrom[i];
      const bool has = f != kNoSlot;
      acc_g[pb + i] = has ? sacc[f] : 0ull;
      cnt_g[pb + i] = has ? scnt[f] : 0u;
      dirty_g[pb + i] = has ? sdirty[f] : (uint8_t)0;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    occupancy[blockIdx.x] = sc[3];
    atomicAdd(&out.counters[0], sc[0]);
    atomicAdd(&out.counters[1], sc[1]);
    if (sc[2]) atomicOr(&out.counters[2], 1u);
  }
}

// ------------------------------------------------------------------------------------------
// Evicted window rows grouped by pane on the device (host-DRAM tier, csrc/window_tier.h): the
// tier keeps every chunk pane-sorted, and a host counting sort of a 5M-row eviction cost 42 ms
// per eviction on the box (55 % of config 4-spill's timed host time, profiles/r4q_*). Two
// passes over the compaction's n rows (count read on the device): per-pane counts (LDS
// histogram, one global atomic per pane and workgroup), then each workgroup reserves its
// per-pane runs and scatters its rows through an LDS cursor. The pane column is not written:
// the counts carry it. Row order inside a pane is unspecified (the tier's merges are
// order-free).
// ------------------------------------------------------------------------------------------
constexpr int kPaneSortMax = 64;

__global__ __launch_bounds__(256) void pane_sort_hist_kernel(const int64_t* __restrict__ pane,
                                                             const uint32_t* __restrict__ n_dev,
                                                             uint32_t cap, int64_t p_lo, int np,
                                                             uint32_t* __restrict__ gcount) {
  __shared__ uint32_t h[kPaneSortMax];
  if (threadIdx.x < kPaneSortMax) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t n = *n_dev < cap ? *n_dev : cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int64_t j = pane[i] - p_lo;
    if (j >= 0 && j < np) atomicAdd(&h[j], 1u);
  }
  __syncthreads();
  if ((int)threadIdx.x < np && h[threadIdx.x]) atomicAdd(&gcount[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void pane_sort_scatter_kernel(
    const uint64_t* __restrict__ key, const int64_t* __restrict__ pane,
    const uint64_t* __restrict__ acc, const uint32_t* __restrict__ cnt,
    const uint8_t* __restrict__ dirty, const uint32_t* __restrict__ n_dev, uint32_t cap,
    int64_t p_lo, int np, const uint32_t* __restrict__ gcount, uint32_t* __restrict__ gcur,
    uint64_t* __restrict__ okey, uint64_t* __restrict__ oacc, uint32_t* __restrict__ ocnt,
    uint8_t* __restrict__ odirty) {
  __shared__ uint32_t h[kPaneSortMax], base[kPaneSortMax];
  if (threadIdx.x < kPaneSortMax) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t n = *n_dev < cap ? *n_dev : cap;
  const uint32_t step = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const int64_t j = pane[i] - p_lo;
    if (j >= 0 && j < np) atomicAdd(&h[j], 1u);
  }
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int j = 0; j < np; ++j) {
      base[j] = s;
      s += gcount[j];
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < np && h[threadIdx.x])
    base[threadIdx.x] += atomicAdd(&gcur[threadIdx.x], h[threadIdx.x]);
  __syncthreads();
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const int64_t j = pane[i] - p_lo;
    if (j < 0 || j >= np) continue;
    const uint32_t q = atomicAdd(&base[j], 1u);
    okey[q] = key[i];
    oacc[q] = acc[i];
    ocnt[q] = cnt[i];
    odirty[q] = dirty[i];
  }
}

// ------------------------------------------------------------------------------------------
// Sender-side combiner (G > 1): one workgroup per send bucket (dest rank, sub-table) folds its raw
// records into a fresh LDS table of that sub-table's geometry and writes one pre-aggregated
// record per (key, pane): val = exported accumulator, aux = element count. The all-to-all then
// moves ~#distinct (key, pane) records instead of every event (sum/min/max/count/avg are all
// associative, so the receiver's window_agg result is unchanged).
// ------------------------------------------------------------------------------------------
// PK: packed (sum, count) words for integer sums of int32 values (see kPkOne): one LDS atomic
// per record instead of two, and no count array (the launcher checks bucket_cap < 2^16).
template <int AGG, int RW, bool PK = false>
__global__ __launch_bounds__(1024) void window_combine_kernel(
    const void* __restrict__ recs, const uint32_t* __restrict__ counts, AggPlan p,
    Rec* __restrict__ out, uint32_t ccap, uint32_t* __restrict__ out_counts,
    uint32_t* __restrict__ flags) {
  static_assert(!PK || ((AGG == AGG_SUM_I64 || AGG == AGG_AVG_I64) && RW <= 2),
                "packed combiner: integer sum/avg of 8/16-byte records only");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // KN: 8-byte RecN records carry 32-bit key ids -- 32-bit LDS keys, four-slot groups.
  constexpr bool KN = RW == 1 && PK;
  const int b = blockIdx.x;
  const uint32_t cap = 1u << p.cap_log2;
  const uint32_t mask = cap - 1;
  uint64_t* skeys = (uint64_t*)smem;
  uint32_t* skeys32 = (uint32_t*)smem;
  uint64_t* sacc = KN ? (uint64_t*)(skeys32 + cap) : skeys + cap;
  uint32_t* scnt = (uint32_t*)(sacc + (size_t)p.pg * cap);      // unused when PK
  uint32_t* sflag = scnt + (PK ? 0 : (size_t)p.pg * cap);  // [0] records written, [1] overflow
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
    if constexpr (KN) skeys32[i] = kEmpty32;
    else skeys[i] = kEmptyKey;
  }
  if (threadIdx.x < 2) sflag[threadIdx.x] = 0;
  uint32_t c = counts[b];
  c = c < p.bucket_cap ? c : p.bucket_cap;
  const size_t seg0 = (size_t)b * p.bucket_cap;
  Rec* dst = out + (size_t)b * ccap;
  int inserted = 0;
  bool ovf = false;
  for (int pg0 = 0; pg0 < p.np_step; pg0 += p.pg) {
    const int npg = (p.np_step - pg0) < p.pg ? (p.np_step - pg0) : p.pg;
    for (uint32_t i = threadIdx.x; i < (uint32_t)npg * cap; i += blockDim.x) {
      sacc[i] = PK ? 0ull : (uint64_t)lds_identity<AGG>();
      if (!PK) scnt[i] = 0;
    }
    __syncthreads();
    const int64_t q0 = p.p_lo + pg0;
    for (uint32_t e0 = threadIdx.x; e0 < c; e0 += blockDim.x * kAggU) {
      Rec rr[kAggU];
#pragma unroll
      for (int u = 0; u < kAggU; ++u) {
        const uint32_t e = e0 + u * blockDim.x;
        rr[u] = load_rec<RW>(recs, seg0 + (e < c ? e : c - 1));  // branch-free (see window_agg)
      }
#pragma unroll
      for (int u = 0; u < kAggU; ++u) pin_rec<RW>(rr[u]);
#pragma unroll
      for (int u = 0; u < kAggU; ++u) {
        const uint32_t e = e0 + u * blockDim.x;
        if (e >= c) break;
        const Rec& r = rr[u];
        if (r.t == 0xFFFFFFFFu) continue;  // hole record (staged partition padding)
        const int64_t q = (int64_t)r.t - q0;
        if (q < 0 || q >= npg) continue;
        uint32_t s;
        if constexpr (KN) {
          // (an id equal to the empty marker cannot be combined: the step goes out raw)
          s = (uint32_t)r.key != kEmpty32 ? lds_probe_insert_g4(skeys32, (uint32_t)r.key, mask,
                                                                &inserted)
                                          : kNoSlot;
        } else {
          s = lds_probe_insert4(skeys, r.key, mask, &inserted);
        }
        if (s == kNoSlot) {
          ovf = true;
          continue;
        }
        const uint32_t li = (uint32_t)q * cap + s;
        if (PK) {
          atomicAdd((unsigned long long*)&sacc[li], (unsigned long long)(r.val + kPkOne));
        } else {
          lds_accumulate<AGG>(&sacc[li], r.val);
          atomicAdd(&scnt[li], 1u);
        }
      }
    }
    __syncthreads();
    // Compact the touched (slot, pane) cells into the bucket's output run (one LDS atomic per
    // wave).
    for (uint32_t i0 = 0; i0 < (uint32_t)npg * cap; i0 += blockDim.x) {
      const uint32_t i = i0 + threadIdx.x;
      const bool have = i < (uint32_t)npg * cap && (PK ? sacc[i] != 0ull : scnt[i] != 0);
      const unsigned long long m = __ballot(have);
      uint32_t wb = 0;
      if (lane_id() == 0 && m) wb = atomicAdd(&sflag[0], (uint32_t)__popcll(m));
      wb = __shfl(wb, 0);
      if (have) {
        const uint32_t pos = wb + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        if (pos < ccap) {
          Rec o;
          o.key = KN ? (uint64_t)skeys32[i & mask] : skeys[i & mask];
          o.val = PK ? (uint64_t)pk_sum(sacc[i]) : lds_export<AGG>(sacc[i]);
          o.t = (uint32_t)(q0 + (int64_t)(i >> p.cap_log2));
          o.aux = PK ? pk_cnt(sacc[i]) : scnt[i];
          dst[pos] = o;
        } else {
          ovf = true;
        }
      }
    }
    __syncthreads();
  }
  if (ovf) sflag[1] = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    out_counts[b] = sflag[0] < ccap ? sflag[0] : ccap;
    if (sflag[1]) atomicOr(&flags[0], 2u);  // bit1: combiner overflow (send raw this step)
  }
}

// ------------------------------------------------------------------------------------------
// Window firing: sweep slots (pane-major => coalesced), combine the window's panes, evaluate
// the fused map/filter epilogue and compact the emitted rows with one atomic per wave.
// The epilogue VM keeps its operand stack and variables in per-lane LDS columns (a runtime-
// indexed private array would live in scratch memory).
// ------------------------------------------------------------------------------------------
struct LdsCol {
  double* base;
  int stride;
  __device__ __forceinline__ double get(int i) const { return base[i * stride]; }
  __device__ __forceinline__ void set(int i, double x) { base[i * stride] = x; }
};

// Epilogue variables in registers (a switch over named values: no runtime-indexed array).
struct RegVars {
  double v0, v1, v2, v3, v4, v5, v6;
  __device__ __forceinline__ double get(int i) const {
    switch (i) {
      case 0: return v0;
      case 1: return v1;
      case 2: return v2;
      case 3: return v3;
      case 4: return v4;
      case 5: return v5;
      default: return v6;
    }
  }
};

constexpr int kFireThreads = 1024;
constexpr int kFireU = 4;  // slots per thread per round (ILP)
constexpr int kFireP = 8;  // panes whose counts are loaded together
constexpr int kFireMultiThreads = 256;

// One window's sweep, shared by the single-window kernel (T = 1024, the whole grid on one window)
// and the batched kernel (T = 256, blockIdx.y = window): the window fields (p0, npanes, wstart,
// wend) come as arguments so the plan itself stays in the kernel-argument segment.
template <int T, int U>
__device__ __forceinline__ void fire_window_body(
    const uint64_t* __restrict__ keys_g, const uint64_t* __restrict__ acc_g,
    const uint32_t* __restrict__ cnt_g, const uint8_t* __restrict__ dirty_g, const FirePlan& p,
    int64_t p0, int npanes, double wstart, double wend, uint64_t* __restrict__ out_keys,
    double* __restrict__ out_vals, uint64_t* __restrict__ out_raw, uint32_t* __restrict__ out_cnt,
    uint32_t* __restrict__ out_n, uint32_t out_cap, double* fsm, int64_t bx, int64_t gx) {
  // LDS: [kExprVars + depth][T] f64 VM columns | T/64 wave counts | block base
  LdsCol vars{fsm + threadIdx.x, T};
  LdsCol stack{fsm + kExprVars * T + threadIdx.x, T};
  const int depth = p.map.depth > p.filt.depth ? p.map.depth : p.filt.depth;
  uint32_t* wcnt = (uint32_t*)(fsm + (size_t)(kExprVars + depth) * T);
  const int wid = threadIdx.x >> 6, nw = T >> 6;
  const int64_t nslots = p.nslots;
  const int64_t per_round = (int64_t)T * U;
  const bool chain_only = (!p.map.ncode || p.map.chain) && (!p.filt.ncode || p.filt.chain);
  // Slot-list mode (re-firings): visit only the listed slots.
  const int64_t nvisit = p.list ? (int64_t)*p.list_n : nslots;
  // Rounds are block-uniform, so every lane reaches the barriers and the ballots.
  for (int64_t base = bx * per_round; base < nvisit; base += gx * per_round) {
    bool emit[U];
    uint64_t acc[U], key[U];
    uint32_t cnt[U];
    double val[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = base + (int64_t)u * T + threadIdx.x;
      emit[u] = false;
      acc[u] = 0;
      key[u] = 0;
      cnt[u] = 0;
      val[u] = 0.0;
      if (v < nvisit) {
        const int64_t s = p.list ? (int64_t)p.list[v] : v;
        bool dirty = !p.only_dirty;
        bool have = false;
        // Panes in groups of kFireP: the group's count loads are all in flight before the first
        // is used (a window of 60 panes -- 5 min / 5 s -- was 60 serial memory round trips per
        // slot, and a small table has too few slots to hide them).
        for (int j0 = 0; j0 < npanes; j0 += kFireP) {
          uint32_t cg[kFireP];
#pragma unroll
          for (int q = 0; q < kFireP; ++q) {
            const int j = j0 + q < npanes ? j0 + q : npanes - 1;
            const uint32_t c = cnt_g[(size_t)((p0 + j) & (p.ring - 1)) * nslots + s];
            cg[q] = j0 + q < npanes ? c : 0u;
          }
          // The group's accumulator loads are issued together as well (predicated on a
          // non-zero count), then combined: one memory round trip per group, not per pane.
          uint64_t ag[kFireP];
#pragma unroll
          for (int q = 0; q < kFireP; ++q) {
            const size_t gi = (size_t)((p0 + j0 + q) & (p.ring - 1)) * nslots + s;
            ag[q] = cg[q] ? acc_g[gi] : 0ull;
          }
#pragma unroll
          for (int q = 0; q < kFireP; ++q) {
            if (!cg[q]) continue;
            acc[u] = have ? agg_combine(p.agg, acc[u], ag[q]) : ag[q];
            have = true;
            cnt[u] += cg[q];
            if (p.only_dirty && dirty_g[(size_t)((p0 + j0 + q) & (p.ring - 1)) * nslots + s])
              dirty = true;
          }
        }
        if (cnt[u] && dirty) {
          key[u] = keys_g[s];
          const double v0 = agg_result_f64(p.agg, acc[u], cnt[u]);
          val[u] = v0;
          emit[u] = true;
          if ((p.map.ncode || p.filt.ncode) && !(p.ablate & 1u) && chain_only) {
            // Register-only epilogue (plan-uniform branch): no LDS stack / variable columns.
            const RegVars rv{v0, (double)cnt[u], wstart, wend, (double)key[u],
                             (double)(int64_t)acc[u], 0.0};
            if (p.map.ncode) val[u] = expr_eval_chain(p.map, rv);
            if (p.filt.ncode) {
              RegVars rf = rv;
              rf.v6 = val[u];
              emit[u] = expr_eval_chain(p.filt, rf) != 0.0;
            }
          } else if ((p.map.ncode || p.filt.ncode) && !(p.ablate & 1u)) {
            vars.set(0, v0);
            vars.set(1, (double)cnt[u]);
            vars.set(2, wstart);
            vars.set(3, wend);
            vars.set(4, (double)key[u]);
            vars.set(5, (double)(int64_t)acc[u]);
            if (p.map.ncode) val[u] = expr_eval_t(p.map, stack, vars);
            vars.set(6, val[u]);
            if (p.filt.ncode) emit[u] = expr_eval_t(p.filt, stack, vars) != 0.0;
          }
        }
      }
    }
    // Block-level compaction: wave ballots -> LDS prefix over waves -> ONE global atomic per
    // round (a per-wave atomic on one counter serialises ~65K times at 4M slots).
    uint32_t mine = 0;
    unsigned long long masks[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      masks[u] = __ballot(emit[u]);
      mine += (uint32_t)__popcll(masks[u]);
    }
    __syncthreads();
    if (lane_id() == 0) wcnt[wid] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (int w = 0; w < nw; ++w) {
        const uint32_t c = wcnt[w];
        wcnt[w] = tot;
        tot += c;
      }
      wcnt[nw] = tot ? atomicAdd(out_n, tot) : 0u;
    }
    __syncthreads();
    uint32_t pos = wcnt[nw] + wcnt[wid];
    const unsigned long long lt = (1ull << lane_id()) - 1ull;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (emit[u]) {
        const uint32_t q = pos + (uint32_t)__popcll(masks[u] & lt);
        if (q < out_cap) {
          if (p.key32)
            reinterpret_cast<uint32_t*>(out_keys)[q] = (uint32_t)key[u];
          else
            out_keys[q] = key[u];
          out_vals[q] = val[u];
          if (out_raw) out_raw[q] = acc[u];
          if (out_cnt) out_cnt[q] = cnt[u];
        }
      }
      pos += (uint32_t)__popcll(masks[u]);
    }
  }
}

__global__ __launch_bounds__(kFireThreads) void window_fire_kernel(
    const uint64_t* __restrict__ keys_g, const uint64_t* __restrict__ acc_g,
    const uint32_t* __restrict__ cnt_g, const uint8_t* __restrict__ dirty_g, FirePlan p,
    uint64_t* __restrict__ out_keys, double* __restrict__ out_vals, uint64_t* __restrict__ out_raw,
    uint32_t* __restrict__ out_cnt, uint32_t* __restrict__ out_n) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  fire_window_body<kFireThreads, kFireU>(keys_g, acc_g, cnt_g, dirty_g, p, p.p0, p.npanes,
                                         p.wstart, p.wend, out_keys, out_vals, out_raw, out_cnt,
                                         out_n, p.out_cap, fsm, blockIdx.x, gridDim.x);
}

// Batched firing: blockIdx.y = window of the pack. Window w appends to its own region
// [w * region, (w + 1) * region) of the staging columns at its own counter win_n[w] (a window
// emits at most one row per slot, so region = nslots never overflows); fire_pack_kernel then
// lays the regions out back to back in window order. A 5 min / 5 s window over a 2K-key table
// is 8 workgroups of 256 slots; 32 windows fill the chip where one window's sweep had ONE
// 1024-thread workgroup and 52 us of serial pane loads.
constexpr int kFireMultiMax = 32;  // windows per launch (kernel-argument segment)
struct FireWinPack {
  FireWin w[kFireMultiMax];
  int n;
};

template <int U>
__global__ __launch_bounds__(kFireMultiThreads) void window_fire_multi_kernel(
    const uint64_t* __restrict__ keys_g, const uint64_t* __restrict__ acc_g,
    const uint32_t* __restrict__ cnt_g, const uint8_t* __restrict__ dirty_g, FirePlan p,
    FireWinPack pack, int w0, FireStage st) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  const int y = blockIdx.y;
  const FireWin& w = pack.w[y];
  const size_t o = (size_t)(w0 + y) * st.region;
  fire_window_body<kFireMultiThreads, U>(
      keys_g, acc_g, cnt_g, dirty_g, p, w.p0, w.npanes, w.wstart, w.wend, st.keys + o,
      st.vals + o, st.raw ? st.raw + o : nullptr, st.cnt ? st.cnt + o : nullptr,
      st.win_n + w0 + y, st.region, fsm, blockIdx.x, gridDim.x);
}


// Fused re-firing of several windows over ONE touched-slot list (allowed lateness): late data of
// a step lands in a few panes, and every already-fired window containing them re-fires. One
// thread per listed slot loads the union of the windows' panes once (<= kRefireP panes: count,
// then accumulator and dirty byte where the count is non-zero, all in flight together) and
// evaluates every window from registers -- the per-window sweep read each slot's panes once per
// window (3 re-fired windows of 6 panes: 18 random (count, acc, dirty) triples per slot, here 8).
// Window w appends to staging region w at counter win_n[w] (block-level compaction per window);
// fire_pack_kernel lays the regions out in window order.
constexpr int kRefireP = 16;
constexpr int kRefireThreads = 256;

__global__ __launch_bounds__(kRefireThreads) void window_refire_multi_kernel(
    const uint64_t* __restrict__ keys_g, const uint64_t* __restrict__ acc_g,
    const uint32_t* __restrict__ cnt_g, uint8_t* __restrict__ dirty_g, FirePlan p,
    FireWinPack pack, int64_t u0, int nu, uint32_t dmask, FireStage st) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  constexpr int T = kRefireThreads;
  LdsCol vars{fsm + threadIdx.x, T};
  LdsCol stack{fsm + kExprVars * T + threadIdx.x, T};
  const int depth = p.map.depth > p.filt.depth ? p.map.depth : p.filt.depth;
  uint32_t* wcnt = (uint32_t*)(fsm + (size_t)(kExprVars + depth) * T);
  const int wid = threadIdx.x >> 6, nw = T >> 6;
  const int64_t nslots = p.nslots;
  const bool chain_only = (!p.map.ncode || p.map.chain) && (!p.filt.ncode || p.filt.chain);
  const int64_t nvisit = (int64_t)*p.list_n;
  for (int64_t base = (int64_t)blockIdx.x * T; base < nvisit; base += (int64_t)gridDim.x * T) {
    const int64_t v = base + threadIdx.x;
    const bool live = v < nvisit;
    const int64_t s = live ? (int64_t)p.list[v] : 0;
    uint32_t cg[kRefireP];
    uint64_t ag[kRefireP];
    uint32_t dirt = 0;
#pragma unroll
    for (int q = 0; q < kRefireP; ++q)
      cg[q] = (live && q < nu) ? cnt_g[(size_t)((u0 + q) & (p.ring - 1)) * nslots + s] : 0u;
#pragma unroll
    for (int q = 0; q < kRefireP; ++q) {
      const size_t gi = (size_t)((u0 + q) & (p.ring - 1)) * nslots + s;
      ag[q] = cg[q] ? acc_g[gi] : 0ull;
      // dirty bytes only in the panes that received late data this step (dmask: every other
      // pane's dirty bytes are clear -- dirty_clear ran after the previous re-firing)
      if (cg[q] && (dmask >> q & 1u) && dirty_g[gi]) dirt |= 1u << q;
    }
    const uint64_t key = live ? keys_g[s] : 0ull;
    for (int w = 0; w < pack.n; ++w) {  // block-uniform: every lane reaches the barriers
      const FireWin& fw = pack.w[w];
      const int off = (int)(fw.p0 - u0);
      uint64_t acc = 0;
      uint32_t cnt = 0;
      bool have = false, dirty = false;
#pragma unroll
      for (int q = 0; q < kRefireP; ++q) {
        if (q < off || q >= off + fw.npanes || !cg[q]) continue;
        acc = have ? agg_combine(p.agg, acc, ag[q]) : ag[q];
        have = true;
        cnt += cg[q];
        dirty = dirty || (dirt >> q & 1u);
      }
      bool emit = false;
      double val = 0.0;
      if (cnt && dirty) {
        const double v0 = agg_result_f64(p.agg, acc, cnt);
        val = v0;
        emit = true;
        if ((p.map.ncode || p.filt.ncode) && chain_only) {
          const RegVars rv{v0, (double)cnt, fw.wstart, fw.wend, (double)key, (double)(int64_t)acc,
                           0.0};
          if (p.map.ncode) val = expr_eval_chain(p.map, rv);
          if (p.filt.ncode) {
            RegVars rf = rv;
            rf.v6 = val;
            emit = expr_eval_chain(p.filt, rf) != 0.0;
          }
        } else if (p.map.ncode || p.filt.ncode) {
          vars.set(0, v0);
          vars.set(1, (double)cnt);
          vars.set(2, fw.wstart);
          vars.set(3, fw.wend);
          vars.set(4, (double)key);
          vars.set(5, (double)(int64_t)acc);
          if (p.map.ncode) val = expr_eval_t(p.map, stack, vars);
          vars.set(6, val);
          if (p.filt.ncode) emit = expr_eval_t(p.filt, stack, vars) != 0.0;
        }
      }
      const unsigned long long m = __ballot(emit);
      __syncthreads();
      if (lane_id() == 0) wcnt[wid] = (uint32_t)__popcll(m);
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int i = 0; i < nw; ++i) {
          const uint32_t c = wcnt[i];
          wcnt[i] = tot;
          tot += c;
        }
        wcnt[nw] = tot ? atomicAdd(&st.win_n[w], tot) : 0u;
      }
      __syncthreads();
      if (emit) {
        const uint32_t q = wcnt[nw] + wcnt[wid] + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        if (q < st.region) {
          const size_t o = (size_t)w * st.region;
          if (p.key32)
            reinterpret_cast<uint32_t*>(st.keys + o)[q] = (uint32_t)key;
          else
            st.keys[o + q] = key;
          st.vals[o + q] = val;
          if (st.raw) st.raw[o + q] = acc;
          if (st.cnt) st.cnt[o + q] = cnt;
        }
      }
    }
    if (p.clear_mark && live) {
      // dirty_clear's work for this slot, by the thread that just read its dirty bytes: the
      // panes that held them (dmask panes with a count; dirty bytes are set only with data)
#pragma unroll
      for (int q = 0; q < kRefireP; ++q)
        if (dirt >> q & 1u) dirty_g[(size_t)((u0 + q) & (p.ring - 1)) * nslots + s] = 0;
      p.clear_mark[s] = 0u;
    }
  }
}

// Regions -> contiguous rows in window order; bounds[w] = rows of windows 0..w, *out_n = total.
// A window with more rows than its region sets bit 16 of *ovf (when given): its rows past the
// region were not staged (the fused re-firing's regions are the stage split k ways).
__global__ __launch_bounds__(256) void fire_pack_kernel(FireStage st, int k, int key32,
                                                        uint64_t* __restrict__ out_keys,
                                                        double* __restrict__ out_vals,
                                                        uint64_t* __restrict__ out_raw,
                                                        uint32_t* __restrict__ out_cnt,
                                                        uint32_t* __restrict__ bounds,
                                                        uint32_t* __restrict__ out_n,
                                                        uint32_t* __restrict__ ovf) {
  const int w = blockIdx.y;
  __shared__ uint32_t s_off;
  if (threadIdx.x < 64) {  // wave 0: prefix of the earlier windows' row counts
    uint32_t c = 0;
    for (int j = threadIdx.x; j < w; j += 64) {
      const uint32_t x = st.win_n[j];
      c += x < st.region ? x : st.region;
    }
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    if (threadIdx.x == 0) s_off = c;
  }
  __syncthreads();
  const uint32_t off = s_off;
  uint32_t n = st.win_n[w];
  n = n < st.region ? n : st.region;
  const size_t src = (size_t)w * st.region;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    if (key32)
      reinterpret_cast<uint32_t*>(out_keys)[off + i] =  // region w's compact keys start at
          reinterpret_cast<const uint32_t*>(st.keys + src)[i];  // its first 64-bit word
    else
      out_keys[off + i] = st.keys[src + i];
    out_vals[off + i] = st.vals[src + i];
    if (out_raw) out_raw[off + i] = st.raw[src + i];
    if (out_cnt) out_cnt[off + i] = st.cnt[src + i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    bounds[w] = off + n;
    if (w == k - 1) *out_n = off + n;
    if (ovf && st.win_n[w] > st.region) atomicOr(ovf, 16u);
  }
}

// ------------------------------------------------------------------------------------------
// Local-global window aggregation (G > 1): every rank folds its own events into a local table
// of the whole key space (no per-event exchange); when a window fires, the rows of the local
// fire (key, partial accumulator, count) travel to the key's owner rank as combined records.
// One workgroup scatters kScatU * 1024 rows: LDS histogram over the (owner, sub-table) buckets,
// one global cursor atomic per touched bucket, then the writes. The row count comes from the
// fire's device counter, so no host round trip sits between the local fire and the exchange.
// ------------------------------------------------------------------------------------------
// Reset the touched-slot list after a step's re-firings: every listed slot's dirty bytes (all
// ring panes) and its mark.
__global__ __launch_bounds__(256) void dirty_clear_kernel(const uint32_t* __restrict__ list,
                                                          const uint32_t* __restrict__ list_n,
                                                          uint32_t list_cap, int ring, int64_t nslots,
                                                          uint8_t* __restrict__ dirty_g,
                                                          uint32_t* __restrict__ slot_mark,
                                                          int64_t p_lo, int np,
                                                          uint64_t* __restrict__ dacc,
                                                          uint32_t* __restrict__ dcnt) {
  uint32_t n = *list_n;
  n = n < list_cap ? n : list_cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = list[i];
    slot_mark[s] = 0u;
    for (int j = 0; j < np; ++j) {
      const size_t gi = (size_t)((p_lo + j) & (ring - 1)) * nslots + s;
      dirty_g[gi] = 0;
      if (dcnt) {
        dcnt[gi] = 0u;
        dacc[gi] = 0ull;
      }
    }
  }
}

constexpr int kScatThreads = 1024;
constexpr int kScatU = 8;

__global__ __launch_bounds__(kScatThreads) void scatter_partials_kernel(
    const uint64_t* __restrict__ keys, const uint64_t* __restrict__ acc,
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ n_in, ScatPlan p,
    const int32_t* __restrict__ jhash, const int32_t* __restrict__ kg_dest,
    uint32_t* __restrict__ cursor, Rec* __restrict__ out, uint32_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) uint32_t scm[];
  const int nb = p.nranks << p.nsub_log2;
  uint32_t* lcnt = scm;       // [nb] rows of this group per bucket
  uint32_t* lbase = scm + nb;  // [nb] the group's base in each bucket
  uint32_t n = *n_in;
  n = n < p.n_cap ? n : p.n_cap;
  const uint32_t r0 = blockIdx.x * (uint32_t)(kScatThreads * kScatU);
  if (r0 >= n) return;  // workgroup-uniform
  for (int b = threadIdx.x; b < nb; b += kScatThreads) lcnt[b] = 0;
  __syncthreads();
  uint32_t bk[kScatU], rk[kScatU];
  uint64_t kk[kScatU];
#pragma unroll
  for (int u = 0; u < kScatU; ++u) {
    const uint32_t i = r0 + (uint32_t)u * kScatThreads + threadIdx.x;
    bk[u] = 0xFFFFFFFFu;
    if (i < n) {
      const uint64_t k = keys[i];
      kk[u] = k;
      const int32_t jh = p.hash_mode ? jhash[k] : java_long_hash((int64_t)k);
      const uint32_t dest = (uint32_t)kg_dest[key_group_of_hash(jh, p.max_parallelism)];
      bk[u] = (dest << p.nsub_log2) | sub_table_of(k, p.nsub_log2);
      rk[u] = atomicAdd(&lcnt[bk[u]], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += kScatThreads) {
    const uint32_t c = lcnt[b];
    lbase[b] = c ? atomicAdd(&cursor[b], c) : 0u;
  }
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int u = 0; u < kScatU; ++u) {
    if (bk[u] == 0xFFFFFFFFu) continue;
    const uint32_t i = r0 + (uint32_t)u * kScatThreads + threadIdx.x;
    const uint32_t pos = lbase[bk[u]] + rk[u];
    if (pos >= p.bucket_cap) {
      ovf = true;
      continue;
    }
    Rec r;
    r.key = kk[u];
    r.val = acc[i];
    r.t = 0;
    r.aux = cnt[i];
    out[(size_t)bk[u] * p.bucket_cap + pos] = r;
  }
  if (ovf) atomicOr(&flags[0], 1u);
}

// Stateless predicate (chapter1 filter `usage > 90`, Main.java:31) over one f64 column.
__global__ __launch_bounds__(256) void expr_filter_kernel(const double* __restrict__ x, int64_t n,
                                                          ExprProg prog, uint8_t* __restrict__ keep) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  LdsCol vars{fsm + threadIdx.x, 256};
  LdsCol stack{fsm + kExprVars * 256 + threadIdx.x, 256};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    vars.set(0, x[i]);
    keep[i] = expr_eval_t(prog, stack, vars) != 0.0;
  }
}

// Order-preserving filter compaction (chapter1 `filter(usage > 90)`, Main.java:31):
// the indices of the rows that pass, in input order. Three launches, no atomics on the data path:
//   1. filter_mask  : a workgroup owns a tile of kFcItems x 256 rows (row = tile + j*256 + tid);
//                     each wave ballots its lanes' predicates into one 64-bit word per item j
//                     (words in row order: j-major, wave-minor) and the tile count is written;
//   2. filter_scan  : one workgroup turns the tile counts into exclusive offsets (+ the total);
//   3. filter_write : each kept row's position = tile offset + popcount of the tile's earlier
//                     words + popcount of its own word's lower lanes.
// Tile constants kFcItems / kFcWords / kFcTile: mxs_kernels.h (shared with csrc/ingest_hip.hip).

__global__ __launch_bounds__(256) void filter_mask_kernel(const double* __restrict__ x, int64_t n,
                                                          ExprProg prog,
                                                          uint64_t* __restrict__ masks,
                                                          uint32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  LdsCol vars{fsm + threadIdx.x, 256};
  LdsCol stack{fsm + kExprVars * 256 + threadIdx.x, 256};
  __shared__ uint32_t wcnt[kFcWords];
  const int64_t tile = (int64_t)blockIdx.x * kFcTile;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < kFcItems; ++j) {
    const int64_t i = tile + j * 256 + threadIdx.x;
    bool keep = false;
    if (i < n) {
      vars.set(0, x[i]);
      keep = expr_eval_t(prog, stack, vars) != 0.0;
    }
    const uint64_t m = __ballot(keep);
    if (lane == 0) {
      masks[(size_t)blockIdx.x * kFcWords + j * 4 + wave] = m;
      wcnt[j * 4 + wave] = (uint32_t)__popcll(m);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kFcWords; ++w) c += wcnt[w];
    counts[blockIdx.x] = c;
  }
}

// Line starts of a text batch (GPU ingest): positions i < n with i == 0 or buf[i-1] == '\n', in
// order -- the same tile ballots as filter_mask_kernel, then filter_scan / filter_write.
__global__ __launch_bounds__(256) void line_start_mask_kernel(const uint8_t* __restrict__ buf,
                                                              int64_t n,
                                                              uint64_t* __restrict__ masks,
                                                              uint32_t* __restrict__ counts) {
  // 16 bytes per thread (one 16-byte load when the batch is 16-byte aligned): bit k of `bits`
  // = position base + k starts a line (the byte before it is '\n'); four lanes' 16 bits make the
  // 64-bit mask word of positions [64w, 64w + 64) -- the layout filter_write_kernel reads.
  // One byte per thread ran at ~0.8 TB/s.
  __shared__ uint32_t wcnt[kFcWords];
  const int64_t base = (int64_t)blockIdx.x * kFcTile + (int64_t)threadIdx.x * 16;
  uint32_t bits = 0;
  if (base < n) {
    const bool prev_nl = base == 0 || buf[base - 1] == (uint8_t)'\n';
    uint8_t by[16];
    if (base + 16 <= n && ((uintptr_t)(buf + base) & 15) == 0) {
      const uint4 v = *reinterpret_cast<const uint4*>(buf + base);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) by[k] = (uint8_t)(w[k >> 2] >> ((k & 3) * 8));
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) by[k] = base + k < n ? buf[base + k] : (uint8_t)0;
    }
    bits = prev_nl ? 1u : 0u;
#pragma unroll
    for (int k = 1; k < 16; ++k) bits |= (by[k - 1] == (uint8_t)'\n' ? 1u : 0u) << k;
    if (base + 16 > n) bits &= (1u << (n - base)) - 1u;  // positions past the end
  }
  const int lane = threadIdx.x & 63;
  const uint64_t v1 = (uint64_t)__shfl_down(bits, 1), v2 = (uint64_t)__shfl_down(bits, 2),
                 v3 = (uint64_t)__shfl_down(bits, 3);
  if ((lane & 3) == 0) {
    const uint64_t word = (uint64_t)bits | v1 << 16 | v2 << 32 | v3 << 48;
    masks[(size_t)blockIdx.x * kFcWords + (threadIdx.x >> 2)] = word;
    wcnt[threadIdx.x >> 2] = (uint32_t)__popcll(word);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kFcWords; ++w) c += wcnt[w];
    counts[blockIdx.x] = c;
  }
}

// Exclusive scan of `nt` tile counts by one 1024-thread workgroup (chunks of 1024, carried).
__global__ __launch_bounds__(1024) void filter_scan_kernel(const uint32_t* __restrict__ counts,
                                                           int64_t nt, int64_t* __restrict__ offs,
                                                           int64_t* __restrict__ total) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nt; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nt ? (int64_t)counts[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan in LDS
      const int64_t add = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < nt) offs[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) total[0] = carry;
}

__global__ __launch_bounds__(256) void filter_write_kernel(const uint64_t* __restrict__ masks,
                                                           const int64_t* __restrict__ offs,
                                                           int64_t n, int64_t* __restrict__ idx,
                                                           int64_t cap) {
  // cap: idx holds this many entries (line starts sized by a bound; the count is exact anyway)
  __shared__ uint32_t wpre[kFcWords];
  const uint64_t* tm = masks + (size_t)blockIdx.x * kFcWords;
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kFcWords; ++w) {
      wpre[w] = c;
      c += (uint32_t)__popcll(tm[w]);
    }
  }
  __syncthreads();
  const int64_t tile = (int64_t)blockIdx.x * kFcTile, off = offs[blockIdx.x];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int j = 0; j < kFcItems; ++j) {
    const int w = j * 4 + wave;
    const uint64_t m = tm[w];
    const int64_t i = tile + j * 256 + threadIdx.x;
    const int64_t q = off + wpre[w] + __popcll(m & below);
    if (((m >> lane) & 1ull) && i < n && q < cap) idx[q] = i;
  }
}

// ------------------------------------------------------------------------------------------
// Rolling keyed state (StreamGroupedReduce / keyed ValueState): per-record post-update values
// in arrival order per key (ComputeCpuMax.java:26 `keyBy(0).max(2)` emits on every record).
//   1. rolling_lookup : one workgroup per received (src, sub) bucket; find/insert the key in the
//                       HBM hash table (global CAS), write sort key (slot<<40 | src<<32 | aux)
//                       and the value, compacted.
//   2. sort (one radix sort of the 64-bit keys: key-major, then channel, then arrival)
//   3. rolling_heads  : segment starts (first record of every key) compacted.
//   4. rolling_scan   : one wave per key segment: ordered inclusive scan with shuffles, seeded
//                       by the stored state, traced filter epilogue, ballot-compacted output,
//                       state written back once per key.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t global_probe_insert(uint64_t* keys, uint64_t key, uint32_t mask) {
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    const uint64_t k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return s;
    if (k == kEmptyKey) {
      const uint64_t prev = atomicCAS((unsigned long long*)&keys[s], (unsigned long long)kEmptyKey,
                                      (unsigned long long)key);
      if (prev == kEmptyKey || prev == key) return s;
    }
    s = (s + 1) & mask;
  }
  return kNoSlot;
}

constexpr uint32_t kLookupChunk = 8192;  // records per workgroup (grid = buckets x chunks)

__global__ __launch_bounds__(256) void rolling_lookup_kernel(
    const Rec* __restrict__ recs, const uint32_t* __restrict__ counts, int nsrc, int nsub,
    uint32_t bucket_cap, int cap_log2, uint64_t* __restrict__ keys_g,
    int64_t* __restrict__ sort_key, uint64_t* __restrict__ vals_out, uint32_t* __restrict__ n_out,
    uint32_t* __restrict__ flags, int abits, int shift) {
  const int b = blockIdx.y;  // = src * nsub + sub
  const int src = b / nsub, sub = b % nsub;
  uint32_t c = counts[b];
  c = c < bucket_cap ? c : bucket_cap;
  const uint32_t lo = blockIdx.x * kLookupChunk;
  if (lo >= c) return;  // whole workgroup exits together
  const uint32_t hi = lo + kLookupChunk < c ? lo + kLookupChunk : c;
  const size_t seg = (size_t)b * bucket_cap;
  __shared__ uint32_t base;
  if (threadIdx.x == 0) base = atomicAdd(n_out, hi - lo);
  __syncthreads();
  uint64_t* keys = keys_g + ((size_t)sub << cap_log2);
  const uint32_t mask = (1u << cap_log2) - 1;
  for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) {
    const Rec r = recs[seg + e];
    int64_t sk = INT64_MAX;  // holes and overflow sort last and are ignored
    if (r.t != 0xFFFFFFFFu) {
      const uint32_t s = global_probe_insert(keys, r.key, mask);
      if (s == kNoSlot) {
        atomicOr(&flags[0], 1u);
      } else {
        const uint64_t slot = ((uint64_t)sub << cap_log2) | s;
        sk = (int64_t)((slot << shift) | ((uint64_t)src << abits) | r.aux);
      }
    }
    sort_key[base + (e - lo)] = sk;
    vals_out[base + (e - lo)] = r.val;
  }
}

// Single-rank lookup straight from the source columns (no partition pass): the
// sort key is slot << shift | arrival index, and record i lands at position i, so the batch is
// already in arrival order. A stable radix sort over the slot bits alone then yields the same
// (slot, arrival) order as the full-key sort of the partitioned path, in ~2 passes instead of ~5.
__global__ __launch_bounds__(256) void rolling_lookup_direct_kernel(
    const uint64_t* __restrict__ keys, const uint64_t* __restrict__ vals, uint32_t n,
    int nsub_log2, int cap_log2, uint64_t* __restrict__ keys_g, int64_t* __restrict__ sort_key,
    uint64_t* __restrict__ vals_out, uint32_t* __restrict__ n_out, uint32_t* __restrict__ flags,
    int shift) {
  if (blockIdx.x == 0 && threadIdx.x == 0) n_out[0] = n;
  const uint32_t mask = (1u << cap_log2) - 1;
  // Four records per thread per round: their column loads and first-probe table reads are all
  // issued before any is consumed (the table read is the long-latency step; most records hit
  // their home slot, the rest fall back to the full insert-or-find probe).
  constexpr int U = 4;
  for (uint32_t base = blockIdx.x * blockDim.x * U; base < n; base += gridDim.x * blockDim.x * U) {
    uint64_t key[U], v[U], home[U], k0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * blockDim.x + threadIdx.x;
      key[u] = i < n ? keys[i] : 0;
      v[u] = i < n ? vals[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * blockDim.x + threadIdx.x;
      home[u] = (sub_table_of(key[u], nsub_log2) << cap_log2) | (slot_hash(key[u]) & mask);
      k0[u] = i < n ? __hip_atomic_load(&keys_g[home[u]], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT)
                    : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * blockDim.x + threadIdx.x;
      if (i >= n) continue;
      if (key[u] >= kTombKey) {  // reserved ids (table markers): flagged, never stored
        atomicOr(&flags[0], 4u);
        sort_key[i] = INT64_MAX;
        vals_out[i] = v[u];
        continue;
      }
      uint64_t slot;
      if (k0[u] == key[u]) {
        slot = home[u];
      } else {
        const uint64_t sub = sub_table_of(key[u], nsub_log2);
        const uint32_t s = global_probe_insert(keys_g + (sub << cap_log2), key[u], mask);
        slot = s == kNoSlot ? ~0ull : ((sub << cap_log2) | s);
      }
      int64_t sk = INT64_MAX;
      if (slot == ~0ull) {
        atomicOr(&flags[0], 1u);
      } else {
        sk = (int64_t)((slot << shift) | i);
      }
      sort_key[i] = sk;
      vals_out[i] = v[u];
    }
  }
}

// Segment starts of a (slot << shift)-sorted key array (first record of every slot), compacted.
// A workgroup owns a chunk of kHeadsChunk records: it counts the chunk's heads, reserves their
// run with ONE device-scope atomic (a same-address atomic per wave serialises across the 8 XCDs:
// it made this kernel 3 ms at 16M records), then writes them through an LDS cursor. The list is
// unordered across chunks; its consumers treat segments independently.
constexpr uint32_t kHeadsChunk = 16384;

__device__ __forceinline__ bool seg_head_at(const int64_t* __restrict__ sk, uint32_t i, uint32_t n,
                                            int shift) {
  if (i >= n) return false;
  const int64_t k = sk[i];
  return k != INT64_MAX && (i == 0 || (sk[i - 1] >> shift) != (k >> shift));
}

__global__ __launch_bounds__(256) void seg_heads_kernel(const int64_t* __restrict__ sk,
                                                        const uint32_t* __restrict__ n_in,
                                                        uint32_t* __restrict__ heads,
                                                        uint32_t* __restrict__ n_heads, int shift) {
  __shared__ uint32_t s_w[4], s_base, s_cur;
  const uint32_t n = *n_in;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  for (uint32_t c0 = blockIdx.x * kHeadsChunk; c0 < n; c0 += gridDim.x * kHeadsChunk) {
    const uint32_t c1 = c0 + kHeadsChunk < n ? c0 + kHeadsChunk : n;
    uint32_t cnt = 0;
    for (uint32_t i = c0 + threadIdx.x; i < c1; i += 256) cnt += seg_head_at(sk, i, n, shift);
    for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d);
    if (lane == 0) s_w[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
      s_base = tot ? atomicAdd(n_heads, tot) : 0u;
      s_cur = 0;
    }
    __syncthreads();
    for (uint32_t i0 = c0; i0 < c1; i0 += 256) {  // block-uniform trip count
      const uint32_t i = i0 + threadIdx.x;
      const bool h = i < c1 && seg_head_at(sk, i, n, shift);
      const unsigned long long m = __ballot(h);
      if (m) {
        uint32_t wb = 0;
        if (lane == 0) wb = s_base + atomicAdd(&s_cur, (uint32_t)__popcll(m));
        wb = __shfl(wb, 0);
        if (h) heads[wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
      }
    }
    __syncthreads();  // s_w / s_base / s_cur are reused by the next chunk
  }
}

template <int AGG>
__device__ __forceinline__ uint64_t roll_combine(uint64_t a, uint64_t b) {
  return agg_combine(AGG, a, b);
}

template <int AGG>
__global__ __launch_bounds__(256) void rolling_scan_kernel(
    const int64_t* __restrict__ sk, const int64_t* __restrict__ perm,
    const uint64_t* __restrict__ vals, const uint32_t* __restrict__ n_in,
    const uint32_t* __restrict__ heads, const uint32_t* __restrict__ n_heads,
    uint64_t* __restrict__ acc_g, uint32_t* __restrict__ cnt_g, const uint64_t* __restrict__ keys_g,
    ExprProg filt, uint64_t* __restrict__ out_key, uint64_t* __restrict__ out_val,
    int64_t* __restrict__ out_tag, uint32_t* __restrict__ out_n, uint32_t out_cap, int abits,
    int shift, uint32_t count_n) {
  // count_n > 0: tumbling count windows (countWindow(n), PurgingTrigger(CountTrigger(n))): the
  // scan is segmented at every n-th element of a key (per-key ordinal % n == 0 starts a window),
  // only the element completing a window emits, and the state keeps the open window.
  extern __shared__ __attribute__((aligned(16))) double rsm[];  // VM columns [8 + depth][256]
  LdsCol vars{rsm + threadIdx.x, 256};
  LdsCol stack{rsm + kExprVars * 256 + threadIdx.x, 256};
  const uint32_t n = *n_in, nh = *n_heads;
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t h = wave; h < nh; h += nwaves) {  // wave-uniform loop
    const uint32_t start = heads[h];
    const uint64_t slot = (uint64_t)(sk[start] >> shift);
    uint32_t end = start + 1;
    // Segment end: next record with a different slot (scan forward a wave at a time).
    for (;;) {
      const uint32_t i = end + lane;
      const bool same = i < n && (uint64_t)(sk[i] >> shift) == slot && sk[i] != INT64_MAX;
      const unsigned long long m = __ballot(!same);
      if (m) {
        end += (uint32_t)__ffsll((long long)m) - 1;
        break;
      }
      end += 64;
    }
    const uint32_t c0 = cnt_g[slot];
    uint64_t carry = c0 ? acc_g[slot] : 0;
    bool have = c0 != 0;
    const uint64_t key = keys_g[slot];
    uint32_t cnt = c0;
    for (uint32_t b0 = start; b0 < end; b0 += 64) {
      const uint32_t i = b0 + lane;
      const bool in = i < end;
      // perm == nullptr: values were sorted along with the keys.
      uint64_t v = in ? agg_lift(AGG, vals[perm ? perm[i] : i]) : 0;
      // Inclusive wave scan (Hillis-Steele) over the ordered chunk; with count windows a
      // segmented scan (f: a window starts at or before this lane within the chunk).
      int f = count_n && (cnt + (uint32_t)lane) % count_n == 0;
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(v, o);
        const int g = __shfl_up(f, o);
        if (lane >= o && in && !f) {
          v = roll_combine<AGG>(y, v);
          f = g;
        }
      }
      const uint64_t post = have && !f ? roll_combine<AGG>(carry, v) : v;
      const uint32_t pcount = count_n ? count_n : cnt + (uint32_t)(lane + 1);
      const uint32_t nin = (end - b0) < 64 ? (end - b0) : 64;
      bool emit = in && (!count_n || (cnt + (uint32_t)lane + 1) % count_n == 0);
      if (in && filt.ncode) {
        vars.set(0, agg_result_f64(AGG, post, pcount));
        vars.set(1, (double)pcount);
        vars.set(4, (double)key);
        vars.set(5, (double)(int64_t)post);
        vars.set(6, agg_result_f64(AGG, post, pcount));
        emit = expr_eval_t(filt, stack, vars) != 0.0;
      }
      const unsigned long long m = __ballot(emit);
      uint32_t wb = 0;
      if (lane == 0 && m) wb = atomicAdd(out_n, (uint32_t)__popcll(m));
      wb = __shfl(wb, 0);
      if (emit) {
        const uint32_t q = wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (q < out_cap) {
          out_key[q] = key;
          out_val[q] = AGG == AGG_COUNT ? (uint64_t)pcount : post;
          const int64_t k = sk[i];
          const int64_t srcv = (k >> abits) & (((int64_t)1 << (shift - abits)) - 1);
          out_tag[q] = (srcv << 32) | (k & (((int64_t)1 << abits) - 1));  // src << 32 | arrival
        }
      }
      carry = __shfl(post, (int)nin - 1);
      have = true;
      cnt += nin;
    }
    if (lane == 0) {
      if (AGG != AGG_COUNT) acc_g[slot] = carry;
      cnt_g[slot] = count_n ? cnt % count_n : cnt;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Session windows on the GPU (BASELINE config 5). Per key slot: up to kSess sessions (SoA:
// start, end, acc, cnt, flags) + due time (min over sessions of maxTs, or cleanup time once
// fired) + last activity (LRU for the host-DRAM spill). Keys evicted to host DRAM are recorded
// in a device spill set; their records are diverted to the host SessionStore (csrc/sessions.cpp).
// ------------------------------------------------------------------------------------------
constexpr int kSess = 4;
// kTombKey (mxs_common.h): evicted slot, probing continues past it

struct SessArgs {
  int64_t gap, lateness, wm, tbase;
  int32_t agg, cap_log2;
  int64_t nslots;
  int32_t tbits;  // sort key = slot << tbits | (ts - tbase)
  int32_t st;     // element stride of sk / vals: 1 (two arrays) or 2 (interleaved (key, value))
};

__device__ __forceinline__ bool set_contains(const uint64_t* set, uint32_t mask, uint64_t key) {
  uint32_t s = (uint32_t)(mix64(key) >> 32) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    const uint64_t k = set[s];
    if (k == key) return true;
    if (k == kEmptyKey) return false;
    s = (s + 1) & mask;
  }
  return false;
}

__device__ __forceinline__ void set_insert(uint64_t* set, uint32_t mask, uint64_t key) {
  uint32_t s = (uint32_t)(mix64(key) >> 32) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    const uint64_t prev = atomicCAS((unsigned long long*)&set[s], (unsigned long long)kEmptyKey,
                                    (unsigned long long)key);
    if (prev == kEmptyKey || prev == key) return;
    s = (s + 1) & mask;
  }
}

// Insert-or-find with tombstone reuse. Linear-probing invariant: a key sits before the first
// empty slot of its chain, so the probe runs to the key or the first empty slot and claims the
// first tombstone seen on the way (else that empty slot). A lost CAS means another key was
// inserted there: restart (each restart is someone else's progress). `inserted` counts claimed
// empty slots only (tombstone reuse does not shorten the empty-slot budget).
// kScope: __HIP_MEMORY_SCOPE_AGENT for a table in global memory, _WORKGROUP for one staged in
// LDS (the same code then compiles to ds_read / ds_cmpst).
template <int kScope = __HIP_MEMORY_SCOPE_AGENT>
__device__ __forceinline__ uint32_t sess_probe_insert(uint64_t* keys, uint64_t key, uint32_t mask,
                                                      uint32_t* inserted) {
  const uint32_t s0 = slot_hash(key) & mask;
  for (;;) {
    uint32_t s = s0, tomb = kNoSlot, target = kNoSlot;
    for (uint32_t i = 0; i <= mask; ++i) {
      const uint64_t k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, kScope);
      if (k == key) return s;
      if (k == kTombKey) {
        if (tomb == kNoSlot) tomb = s;
      } else if (k == kEmptyKey) {
        target = s;
        break;
      }
      s = (s + 1) & mask;
    }
    const bool use_tomb = tomb != kNoSlot;
    if (use_tomb) target = tomb;
    if (target == kNoSlot) return kNoSlot;  // full: no empty slot, no tombstone
    const uint64_t expect = use_tomb ? kTombKey : kEmptyKey;
    const uint64_t prev = atomicCAS((unsigned long long*)&keys[target], (unsigned long long)expect,
                                    (unsigned long long)key);
    if (prev == expect) {
      // every new key counts (into an empty slot or a reused tombstone): the host derives the
      // live-key count from inserts - evictions (session_operator occupancy bookkeeping)
      if (inserted) atomicAdd(inserted, 1u);
      return target;
    }
    if (prev == key) return target;
  }
}

// sess_probe_insert reporting whether THIS call claimed the slot for the key.
template <int kScope = __HIP_MEMORY_SCOPE_AGENT>
__device__ __forceinline__ uint32_t sess_probe_claim(uint64_t* keys, uint64_t key, uint32_t mask,
                                                     bool* claimed) {
  const uint32_t s0 = slot_hash(key) & mask;
  for (;;) {
    uint32_t s = s0, tomb = kNoSlot, target = kNoSlot;
    for (uint32_t i = 0; i <= mask; ++i) {
      const uint64_t k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, kScope);
      if (k == key) return s;
      if (k == kTombKey) {
        if (tomb == kNoSlot) tomb = s;
      } else if (k == kEmptyKey) {
        target = s;
        break;
      }
      s = (s + 1) & mask;
    }
    const bool use_tomb = tomb != kNoSlot;
    if (use_tomb) target = tomb;
    if (target == kNoSlot) return kNoSlot;
    const uint64_t expect = use_tomb ? kTombKey : kEmptyKey;
    const uint64_t prev = atomicCAS((unsigned long long*)&keys[target], (unsigned long long)expect,
                                    (unsigned long long)key);
    if (prev == expect) {
      *claimed = true;
      return target;
    }
    if (prev == key) return target;
  }
}

// Read-only probe: the key's slot, or kNoSlot (first empty slot reached / table scanned).
template <int kScope = __HIP_MEMORY_SCOPE_AGENT>
__device__ __forceinline__ uint32_t sess_find(const uint64_t* keys, uint64_t key, uint32_t mask) {
  // Four independent loads per round (tombstones make the session tables' chains long; a
  // wave waits for its longest chain, so rounds -- not slots -- set the cost).
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; i += 4) {
    uint64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = __hip_atomic_load(&keys[(s + u) & mask], __ATOMIC_RELAXED, kScope);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i + u > mask) return kNoSlot;
      if (k[u] == key) return (s + u) & mask;
      if (k[u] == kEmptyKey) return kNoSlot;
    }
    s = (s + 4) & mask;
  }
  return kNoSlot;
}

// RW: record width of the bucketed input (3 = 24-byte Rec, 2 = 16-byte RecC, load_rec).
template <int RW>
__global__ __launch_bounds__(256) void session_lookup_kernel(
    const void* __restrict__ recs, const uint32_t* __restrict__ counts, int nsrc, int nsub,
    uint32_t bucket_cap, int cap_log2, uint64_t* __restrict__ keys_g,
    uint64_t* __restrict__ spill_set, uint32_t spill_mask, int32_t spill_any,
    int64_t* __restrict__ sort_key, uint64_t* __restrict__ vals_out, uint32_t* __restrict__ n_out,
    Rec* __restrict__ host_recs, uint32_t* __restrict__ n_host, uint32_t host_cap,
    uint32_t* __restrict__ n_inserted, int tbits) {
  const int b = blockIdx.y;
  const int sub = b % nsub;
  uint32_t c = counts[b];
  c = c < bucket_cap ? c : bucket_cap;
  const uint32_t lo = blockIdx.x * kLookupChunk;
  if (lo >= c) return;
  const uint32_t hi = lo + kLookupChunk < c ? lo + kLookupChunk : c;
  const size_t seg = (size_t)b * bucket_cap;
  __shared__ uint32_t base;
  if (threadIdx.x == 0) base = atomicAdd(n_out, hi - lo);
  __syncthreads();
  uint64_t* keys = keys_g + ((size_t)sub << cap_log2);
  const uint32_t mask = (1u << cap_log2) - 1;
  for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) {
    const Rec r = load_rec<RW>(recs, seg + e);
    int64_t sk = INT64_MAX;
    if (r.t != 0xFFFFFFFFu) {
      // Resident keys are found in the slot table (a key is never resident and spilled at once),
      // so only keys missing from it pay the spill-set probe.
      uint32_t s = sess_find(keys, r.key, mask);
      bool to_host = s == kNoSlot && spill_any && set_contains(spill_set, spill_mask, r.key);
      if (!to_host && s == kNoSlot) {
        s = sess_probe_insert(keys, r.key, mask, n_inserted);
        if (s == kNoSlot) {  // sub-table full: the key lives in host DRAM from now on
          to_host = true;
          set_insert(spill_set, spill_mask, r.key);
        }
      }
      if (to_host) {
        const uint32_t q = atomicAdd(n_host, 1u);
        if (q < host_cap) host_recs[q] = r;
      } else {
        const uint64_t slot = ((uint64_t)sub << cap_log2) | s;
        sk = (int64_t)((slot << tbits) | r.t);
      }
    }
    sort_key[base + (e - lo)] = sk;
    vals_out[base + (e - lo)] = r.val;
  }
}

// LDS variant (sub-tables of <= 8192 slots): one workgroup owns one sub-table for the whole
// step -- its keys are staged in LDS, probed/inserted with ds_read/ds_cmpst, written back once.
// Records of every source rank for that sub-table are handled by the same workgroup.
constexpr int kSessLookupBlock = 512;
constexpr int kSessLookupLdsMaxLog2 = 12;  // 32 KB of keys

template <int RW>
__global__ __launch_bounds__(kSessLookupBlock) void session_lookup_lds_kernel(
    const void* __restrict__ recs, const uint32_t* __restrict__ counts, int nsrc, int nsub,
    uint32_t bucket_cap, int cap_log2, uint64_t* __restrict__ keys_g,
    uint64_t* __restrict__ spill_set, uint32_t spill_mask, int32_t spill_any,
    int64_t* __restrict__ sort_key, uint64_t* __restrict__ vals_out, uint32_t* __restrict__ n_out,
    Rec* __restrict__ host_recs, uint32_t* __restrict__ n_host, uint32_t host_cap,
    uint32_t* __restrict__ n_inserted, int tbits) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lkeys[];
  __shared__ uint32_t base, lins;
  const int sub = blockIdx.x;
  const uint32_t cap = 1u << cap_log2, mask = cap - 1;
  uint64_t* gkeys = keys_g + ((size_t)sub << cap_log2);
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) lkeys[i] = gkeys[i];
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int src = 0; src < nsrc; ++src) {
      const uint32_t c = counts[src * nsub + sub];
      tot += c < bucket_cap ? c : bucket_cap;
    }
    base = tot ? atomicAdd(n_out, tot) : 0u;
    lins = 0;
  }
  __syncthreads();
  uint32_t off = base;
  for (int src = 0; src < nsrc; ++src) {
    const int b = src * nsub + sub;
    uint32_t c = counts[b];
    c = c < bucket_cap ? c : bucket_cap;
    const size_t seg = (size_t)b * bucket_cap;
    for (uint32_t e = threadIdx.x; e < c; e += blockDim.x) {
      const Rec r = load_rec<RW>(recs, seg + e);
      int64_t sk = INT64_MAX;
      if (r.t != 0xFFFFFFFFu) {
        uint32_t s = sess_find<__HIP_MEMORY_SCOPE_WORKGROUP>(lkeys, r.key, mask);
        bool to_host = s == kNoSlot && spill_any && set_contains(spill_set, spill_mask, r.key);
        if (!to_host && s == kNoSlot) {
          s = sess_probe_insert<__HIP_MEMORY_SCOPE_WORKGROUP>(lkeys, r.key, mask, &lins);
          if (s == kNoSlot) {  // sub-table full: the key lives in host DRAM from now on
            to_host = true;
            set_insert(spill_set, spill_mask, r.key);
          }
        }
        if (to_host) {
          const uint32_t q = atomicAdd(n_host, 1u);
          if (q < host_cap) host_recs[q] = r;
        } else {
          const uint64_t slot = ((uint64_t)sub << cap_log2) | s;
          sk = (int64_t)((slot << tbits) | r.t);
        }
      }
      sort_key[off + e] = sk;
      vals_out[off + e] = r.val;
    }
    off += c;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) gkeys[i] = lkeys[i];
  if (threadIdx.x == 0 && n_inserted && lins) atomicAdd(n_inserted, lins);
}

// Fused lookup + LDS-staged segmented sort (the session fold's replacement for a device-wide
// radix sort). Records arrive bucketed by sub-table, so the global (slot, ts) order is just every
// sub-table's records in (local slot, ts) order: one workgroup per sub-table
//   1. looks its records up in the LDS-staged slot table (insert / divert exactly as
//      session_lookup_lds) and keeps (local slot << 32 | t) per record in LDS, in arrival order;
//   2. writes the table back, then counts records per local slot (u16 LDS histogram in the
//      table's space), scans the counts and scatters record indices into slot segments;
//   3. ranks every record inside its slot segment by (t, arrival index) -- segments are short
//      (a few records per key and step), a hot key's long segment costs O(len^2) LDS reads in
//      its own workgroup only -- and writes (slot << tbits | t, value) at
//      block base + segment start + rank.
// The output equals a stable sort of session_lookup's keys with the holes removed, so
// session_merge runs on it unchanged. LDS: max(cap*8, cap*2 + m*2) + m*8 bytes for m records.
constexpr int kSessSortBlock = 1024;
constexpr int kLsRegs = 16;  // record values kept in registers per thread (m <= 16K: all of them)

template <int RW>
__global__ __launch_bounds__(kSessSortBlock) void session_lookup_sort_kernel(
    const void* __restrict__ recs, const uint32_t* __restrict__ counts, int nsrc, int nsub,
    uint32_t bucket_cap, int cap_log2, uint64_t* __restrict__ keys_g,
    uint64_t* __restrict__ spill_set, uint32_t spill_mask, int32_t spill_any,
    int64_t* __restrict__ sort_out, uint64_t* __restrict__ vals_out, uint32_t* __restrict__ n_out,
    Rec* __restrict__ host_recs, uint32_t* __restrict__ n_host, uint32_t host_cap,
    uint32_t* __restrict__ n_inserted, int tbits, uint32_t m_cap, const int64_t* __restrict__ skip,
    uint32_t skip_mask, uint64_t* __restrict__ heads_out, uint32_t* __restrict__ n_heads,
    int pair) {
  extern __shared__ __attribute__((aligned(16))) uint64_t slds[];
  // Launched before the host has read the step's partition flags: any flagged word of the
  // reduced vector (bucket overflow, unrepresentable span, reserved key) means the step is
  // redone -- nothing is looked up, inserted or counted (the merge then sees 0 records).
  if (skip) {
    int64_t any = 0;
    for (int w = 0; w < 32; ++w)
      if (skip_mask >> w & 1u) any |= skip[w];
    if (any) return;
  }
  __shared__ uint32_t s_base, s_lins, s_kept, s_m, s_hbase, s_hcnt;
  __shared__ uint32_t s_src_off[65];
  const int sub = blockIdx.x;
  const uint32_t cap = 1u << cap_log2, mask = cap - 1;
  const uint32_t regA = (cap * 8 > cap * 2 + m_cap * 2 ? cap * 8 : cap * 2 + m_cap * 2);
  uint64_t* lkeys = slds;                                              // phase 1: slot table
  uint16_t* cur = reinterpret_cast<uint16_t*>(slds);                   // phase 2: per-slot cursors
  // (u16 cursors, two per 32-bit word: the atomics add 1 << 16 * (slot & 1) to the word; a
  // block holds < 65536 records, so a half never carries into the other)
  uint32_t* cur32 = reinterpret_cast<uint32_t*>(slds);
  uint16_t* idxl = cur + cap;                                          // phase 2: slot segments
  uint64_t* rk = slds + regA / 8;                                      // (slot << 32 | t) per record
  uint64_t* gkeys = keys_g + ((size_t)sub << cap_log2);
  // per slot, 2 bits: key claimed this step (1 resident, 2 spilled); 1 KB of static LDS
  __shared__ uint32_t sflag[(1u << kSessLookupLdsMaxLog2) / 16];
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) lkeys[i] = gkeys[i];
  for (uint32_t i = threadIdx.x; i < (cap + 15) / 16; i += blockDim.x) sflag[i] = 0;
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int src = 0; src < nsrc; ++src) {
      s_src_off[src] = tot;
      const uint32_t c = counts[src * nsub + sub];
      tot += c < bucket_cap ? c : bucket_cap;
    }
    s_src_off[nsrc] = tot;
    s_m = tot;
    s_lins = 0;
    s_kept = 0;
  }
  __syncthreads();
  const uint32_t m = s_m;  // the launcher sized m_cap >= nsrc * bucket_cap >= m
  // Phase 1: lookup / insert / divert; rk[i] = (local slot << 32 | t) or ~0 (not folded here).
  // Records are visited by arrival index i = k * blockDim + tid, the same thread-to-record map as
  // phase 3, so each thread keeps the values of its first kLsRegs records in registers and phase
  // 3 writes them without re-reading the bucket (an uncoalesced gather).
  uint32_t kept = 0;
  auto rec_at = [&](uint32_t i) -> Rec {
    int src = 0;
    while (src + 1 < nsrc && i >= s_src_off[src + 1]) ++src;
    return load_rec<RW>(recs, (size_t)(src * nsub + sub) * bucket_cap + (i - s_src_off[src]));
  };
  // 1a: insert-or-find every record's key in the LDS table. Only the thread that claims a slot
  //     for a key new to the table probes the device spill set (once per key instead of once per
  //     record of every key still missing: those global probes made the kernel latency-bound)
  //     and flags the slot: 1 resident, 2 spilled (records go to the host tier), 3 table full.
  auto lookup = [&](uint32_t i) -> uint64_t {
    const Rec r = rec_at(i);
    uint64_t v = ~0ull;
    if (r.t != 0xFFFFFFFFu) {
      uint32_t sl = sess_find<__HIP_MEMORY_SCOPE_WORKGROUP>(lkeys, r.key, mask);
      if (sl == kNoSlot) {
        bool claimed = false;
        sl = sess_probe_claim<__HIP_MEMORY_SCOPE_WORKGROUP>(lkeys, r.key, mask, &claimed);
        if (sl == kNoSlot) {  // sub-table full: the key lives in host DRAM from now on
          set_insert(spill_set, spill_mask, r.key);
          const uint32_t q = atomicAdd(n_host, 1u);
          if (q < host_cap) host_recs[q] = r;
        } else if (claimed) {
          const uint32_t f = (spill_any && set_contains(spill_set, spill_mask, r.key)) ? 2u : 1u;
          atomicOr(&sflag[sl >> 4], f << ((sl & 15u) * 2));
        }
      }
      if (sl != kNoSlot) v = ((uint64_t)sl << 32) | r.t;
    }
    rk[i] = v;
    return r.val;
  };
  uint64_t vreg[kLsRegs];
#pragma unroll
  for (int k = 0; k < kLsRegs; ++k) {
    const uint32_t i = k * kSessSortBlock + threadIdx.x;
    vreg[k] = i < m ? lookup(i) : 0ull;
  }
  for (uint32_t i = kLsRegs * kSessSortBlock + threadIdx.x; i < m; i += kSessSortBlock) lookup(i);
  __syncthreads();
  // 1b: records of keys found in the spill set go to the host tier; the rest are kept.
  for (uint32_t i = threadIdx.x; i < m; i += kSessSortBlock) {
    const uint64_t v = rk[i];
    if (v == ~0ull) continue;
    const uint32_t sl = (uint32_t)(v >> 32);
    if (((sflag[sl >> 4] >> ((sl & 15u) * 2)) & 3u) == 2u) {
      const uint32_t q = atomicAdd(n_host, 1u);
      if (q < host_cap) host_recs[q] = rec_at(i);
      rk[i] = ~0ull;
    } else {
      ++kept;
    }
  }
  if (kept) atomicAdd(&s_kept, kept);
  __syncthreads();
  // Spilled keys leave the table again (tombstones, reusable); new resident keys are counted.
  uint32_t ins = 0;
  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
    const uint32_t f = (sflag[i >> 4] >> ((i & 15u) * 2)) & 3u;
    if (f == 2) lkeys[i] = kTombKey;
    ins += f == 1;
    gkeys[i] = f == 2 ? kTombKey : lkeys[i];
  }
  if (ins) atomicAdd(&s_lins, ins);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (n_inserted && s_lins) atomicAdd(n_inserted, s_lins);
    s_base = s_kept ? atomicAdd(n_out, s_kept) : 0u;
  }
  __syncthreads();
  // Phase 2: per-slot counts -> exclusive offsets -> segments of record indices.
  for (uint32_t i = threadIdx.x; i < cap / 2; i += blockDim.x) cur32[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
    const uint64_t v = rk[i];
    if (v != ~0ull) {
      const uint32_t sl = (uint32_t)(v >> 32);
      atomicAdd(&cur32[sl >> 1], 1u << ((sl & 1u) * 16));
    }
  }
  __syncthreads();
  // Block-wide exclusive scan of cap (<= 4096) u16 counts: each thread sums a run of cap/T,
  // wave prefix with shuffles, wave totals through LDS.
  {
    __shared__ uint32_t s_wave[kSessSortBlock / 64], s_nz[kSessSortBlock / 64];
    const uint32_t per = (cap + kSessSortBlock - 1) / kSessSortBlock;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < cap ? lo + per : cap;
    uint32_t run = 0, nz = 0;
    for (uint32_t i = lo; i < hi; ++i) {
      const uint32_t c = cur[i];
      run += c;
      nz += c != 0u;
    }
    uint32_t incl = run;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (lane_id() >= d) incl += y;
    }
    for (int d = 32; d >= 1; d >>= 1) nz += __shfl_xor(nz, d);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 63) s_wave[w] = incl;
    if (lane_id() == 0) s_nz[w] = nz;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0, segs = 0;
      for (int i = 0; i < kSessSortBlock / 64; ++i) {
        const uint32_t c = s_wave[i];
        s_wave[i] = t;
        t += c;
        segs += s_nz[i];
      }
      // One device-scope atomic per workgroup reserves its segment-list run (a same-address
      // atomic per wave serialises across the XCDs: 3x the kernel time at 16M records).
      s_hbase = (heads_out && segs) ? atomicAdd(n_heads, segs) : 0u;
      s_hcnt = 0;
    }
    __syncthreads();
    uint32_t o = s_wave[w] + incl - run;
    for (uint32_t i = lo; i < hi; ++i) {
      const uint32_t c = cur[i];
      cur[i] = (uint16_t)o;
      o += c;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
    const uint64_t v = rk[i];
    if (v != ~0ull) {
      const uint32_t sl = (uint32_t)(v >> 32), sh = (sl & 1u) * 16;
      const uint32_t pos = (atomicAdd(&cur32[sl >> 1], 1u << sh) >> sh) & 0xFFFFu;
      idxl[pos] = (uint16_t)i;
    }
  }
  __syncthreads();
  // Phase 3: rank inside the slot segment [end(slot - 1), end(slot)) by (t, arrival index).
  // The record ranked first in its segment also lists the segment (output position | length <<
  // 32) for session_merge_heads: the merge then runs one lane per key instead of one per record.
  const uint64_t sub_slot0 = (uint64_t)sub << cap_log2;
  auto place = [&](uint32_t i, uint64_t v, uint64_t val, bool& head, uint64_t& hv) {
    const uint32_t sl = (uint32_t)(v >> 32), t = (uint32_t)v;
    const uint32_t end = cur[sl], start = sl ? cur[sl - 1] : 0u;
    uint32_t rank = 0;
    for (uint32_t q = start; q < end; ++q) {
      const uint32_t j = idxl[q];
      const uint32_t tj = (uint32_t)rk[j];
      rank += (tj < t || (tj == t && j < i)) ? 1u : 0u;
    }
    const uint32_t out = s_base + start + rank;
    const int64_t key = (int64_t)(((sub_slot0 | sl) << tbits) | t);
    if (pair) {
      // one 16-byte store of the (key, value) pair: half the partial-line write requests of
      // two scattered 8-byte stores, and the merge reads the pair with one 16-byte load
      reinterpret_cast<longlong2*>(sort_out)[out] = make_longlong2(key, (long long)val);
    } else {
      sort_out[out] = key;
      vals_out[out] = val;
    }
    head = rank == 0;
    hv = (uint64_t)(s_base + start) | ((uint64_t)(end - start) << 32);
  };
#pragma unroll
  for (int k = 0; k < kLsRegs + 1; ++k) {
   // k < kLsRegs: the record's value is in vreg[k]; k == kLsRegs: every remaining record (values
   // re-read from the bucket)
   for (uint32_t i0 = k * kSessSortBlock; i0 < (k < kLsRegs ? (k + 1) * kSessSortBlock : m) &&
                                          i0 < m; i0 += kSessSortBlock) {  // block-uniform
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t v = i < m ? rk[i] : ~0ull;
    bool head = false;
    uint64_t hv = 0;
    if (v != ~0ull) place(i, v, k < kLsRegs ? vreg[k] : rec_at(i).val, head, hv);
    if (heads_out) {
      const unsigned long long hm = __ballot(head);
      if (hm) {
        uint32_t wb = 0;
        if (lane_id() == 0) wb = s_hbase + atomicAdd(&s_hcnt, (uint32_t)__popcll(hm));
        wb = __shfl(wb, 0);
        if (head) heads_out[wb + (uint32_t)__popcll(hm & ((1ull << lane_id()) - 1ull))] = hv;
      }
    }
   }
  }
}

struct __attribute__((aligned(32))) SessRec {
  int64_t start, end;  // [start, end)
  uint64_t acc;
  uint32_t cnt;        // 0 = free
  uint32_t flags;      // bit0 fired, bit1 modified since firing
};
static_assert(sizeof(SessRec) == 32, "SessRec layout");

// A slot's sessions in registers: fixed positions, valid iff cnt != 0. Every index below is a
// compile-time constant (unrolled loops), so the state never spills to scratch.
struct SessState {
  int64_t start[kSess], end[kSess];
  uint64_t acc[kSess];
  uint32_t cnt[kSess], flags[kSess];
};

__device__ __forceinline__ int sess_count(const SessState& st) {
  int n = 0;
#pragma unroll
  for (int j = 0; j < kSess; ++j) n += st.cnt[j] != 0;
  return n;
}

// Merge candidate run (cs, ce, ca, cc) into the slot's sessions.
// Returns: 0 merged/inserted, 1 late-dropped, 2 overflow (all kSess positions hold sessions
// that do not intersect the candidate; the state is unchanged).
__device__ __forceinline__ int sess_merge(SessState& st, int64_t cs, int64_t ce, uint64_t ca,
                                          uint32_t cc, const SessArgs& a) {
  int64_t ms = cs, me = ce;
  uint64_t macc = ca;
  uint32_t mcnt = cc, mflags = 0;
  bool touched = false, any_free = false;
#pragma unroll
  for (int j = 0; j < kSess; ++j) {
    if (st.cnt[j] && ms <= st.end[j] && me >= st.start[j]) {
      ms = ms < st.start[j] ? ms : st.start[j];
      me = me > st.end[j] ? me : st.end[j];
      macc = agg_combine(a.agg, st.acc[j], macc);
      mcnt += st.cnt[j];
      mflags |= st.flags[j];
      touched = true;
    }
    any_free |= st.cnt[j] == 0;
  }
  if (!touched && (me - 1) + a.lateness <= a.wm) return 1;
  if (!touched && !any_free) return 2;
  if (mflags & 1u) mflags |= 2u;
  // Sessions absorbed into the merged one leave; the merged one takes the first free position.
  bool placed = false;
#pragma unroll
  for (int j = 0; j < kSess; ++j) {
    const bool absorbed = st.cnt[j] && ms <= st.end[j] && me >= st.start[j];
    if (absorbed) st.cnt[j] = 0;
    if (!placed && st.cnt[j] == 0) {
      st.start[j] = ms;
      st.end[j] = me;
      st.acc[j] = macc;
      st.cnt[j] = mcnt;
      st.flags[j] = mflags;
      placed = true;
    }
  }
  return 0;
}

__device__ __forceinline__ int64_t sess_due(const SessState& st, int64_t lateness) {
  int64_t t = INT64_MAX;
#pragma unroll
  for (int j = 0; j < kSess; ++j) {
    if (!st.cnt[j]) continue;
    const int64_t maxts = st.end[j] - 1;
    const int64_t due = ((st.flags[j] & 1u) && !(st.flags[j] & 2u)) ? maxts + lateness : maxts;
    t = due < t ? due : t;
  }
  return t;
}

// A slot's kSess sessions are one 128-byte AoS record (one cache line): loads and stores are
// four 32-byte accesses instead of 20 scattered ones.
__device__ __forceinline__ void sess_load(SessState& st, const SessRec* r) {
#pragma unroll
  for (int j = 0; j < kSess; ++j) {
    const SessRec x = r[j];
    st.start[j] = x.start;
    st.end[j] = x.end;
    st.acc[j] = x.acc;
    st.cnt[j] = x.cnt;
    st.flags[j] = x.flags;
  }
}

__device__ __forceinline__ void sess_clear(SessState& st) {
#pragma unroll
  for (int j = 0; j < kSess; ++j) {
    st.start[j] = st.end[j] = 0;
    st.acc[j] = 0;
    st.cnt[j] = st.flags[j] = 0;
  }
}

__device__ __forceinline__ void sess_store(const SessState& st, SessRec* r) {
#pragma unroll
  for (int j = 0; j < kSess; ++j) {
    SessRec x;
    x.start = st.start[j];
    x.end = st.end[j];
    x.acc = st.acc[j];
    x.cnt = st.cnt[j];
    x.flags = st.cnt[j] ? st.flags[j] : 0u;
    r[j] = x;
  }
}

// Per-key fold state shared by the thread-per-segment and wave-per-segment merge kernels.
// Per-slot (due, last) words are interleaved: slot_due points at word 0 of a 16-byte pair per
// slot, slot_last at word 1 (session_operator.py allocates one (nslots, 2) tensor).
constexpr int64_t kSlotMeta = 2;

struct SessOut {
  SessRec* sess;
  int64_t* slot_due;
  int64_t* slot_last;
  uint64_t* late_cnt;
  const uint64_t* keys;  // the slot table's keys (read for the overflow list)
  int64_t* ovf_slots;    // (slot, key) pairs
  uint32_t* n_ovf;
  int64_t* ovf_rows;
  uint32_t* n_ovf_runs;
  uint32_t ovf_cap;
};

// Merge one candidate run into the key's sessions (or route it to the host tier on overflow).
__device__ __forceinline__ void sess_commit(SessState& st, bool& overflow, uint64_t& late,
                                            int64_t slot, int64_t ps, int64_t pe, uint64_t pa,
                                            uint32_t pc, const SessArgs& a, const SessOut& o) {
  const int res = overflow ? 2 : sess_merge(st, ps, pe, pa, pc, a);
  if (res == 1) {
    late += pc;
  } else if (res == 2) {
    // More than kSess live sessions: this run (and every later run of the key) goes to the
    // host store, which takes the key over after the step.
    overflow = true;
    const uint32_t q = atomicAdd(o.n_ovf_runs, 1u);
    if (q < o.ovf_cap) {
      o.ovf_rows[q] = slot;
      o.ovf_rows[o.ovf_cap + q] = ps;
      o.ovf_rows[2 * (size_t)o.ovf_cap + q] = pe;
      o.ovf_rows[3 * (size_t)o.ovf_cap + q] = (int64_t)pa;
      o.ovf_rows[4 * (size_t)o.ovf_cap + q] = pc;
    }
  }
}

__device__ __forceinline__ void sess_finish(const SessState& st, int64_t slot, int64_t last_ts,
                                            uint64_t late, bool overflow, const SessArgs& a,
                                            const SessOut& o) {
  sess_store(st, o.sess + slot * kSess);
  // (due, last) of the slot share one 16-byte word: one read and one store per merged key
  longlong2* meta = reinterpret_cast<longlong2*>(o.slot_due) + slot;
  const long long prev_last = meta->y;
  *meta = make_longlong2(sess_due(st, a.lateness), last_ts > prev_last ? last_ts : prev_last);
  if (late) atomicAdd((unsigned long long*)o.late_cnt, (unsigned long long)late);
  if (overflow) {
    // The host evicts these keys and re-merges their overflow runs. The key rides along: a
    // pipelined step may evict the slot (idle) before the host reads the list.
    const uint32_t q = atomicAdd(o.n_ovf, 1u);
    o.ovf_slots[2 * (size_t)q] = slot;
    o.ovf_slots[2 * (size_t)q + 1] = (int64_t)o.keys[slot];
  }
}

constexpr uint32_t kSessLongSeg = 96;  // segments longer than this go to the wave kernel

// One key's records [i, j) (ts order): runs split at gaps > gap, each run merged into the key's
// sessions, state written back once.
__device__ __forceinline__ void sess_merge_segment(const int64_t* __restrict__ sk,
                                                   const uint64_t* __restrict__ vals, uint32_t i,
                                                   uint32_t j, int64_t slot, const SessArgs& a,
                                                   const SessOut& o) {
  const int64_t tmask = ((int64_t)1 << a.tbits) - 1;
  SessState st;
  sess_load(st, o.sess + slot * kSess);
  uint64_t late = 0;
  bool overflow = false;
  bool pv = false;
  int64_t ps = 0, pe = 0;
  uint64_t pa = 0;
  uint32_t pc = 0;
  int64_t ts = 0;
  for (uint32_t r = i; r < j; ++r) {
    ts = a.tbase + (sk[(size_t)r * a.st] & tmask);
    const uint64_t v = agg_lift(a.agg, vals[(size_t)r * a.st]);
    if (pv && ts <= pe) {
      pe = ts + a.gap;
      pa = agg_combine(a.agg, pa, v);
      pc += 1;
    } else {
      if (pv) sess_commit(st, overflow, late, slot, ps, pe, pa, pc, a, o);
      ps = ts;
      pe = ts + a.gap;
      pa = v;
      pc = 1;
      pv = true;
    }
  }
  sess_commit(st, overflow, late, slot, ps, pe, pa, pc, a, o);
  sess_finish(st, slot, ts, late, overflow, a, o);
}

// Thread per key segment (sorted by slot, then ts): the thread at a segment head walks its
// records serially, splitting runs at ts gaps > gap. Typical session workloads have a few records
// per key and step, where a wave per key would idle most lanes. Long segments are queued for
// session_merge_long_kernel.
__global__ __launch_bounds__(256) void session_merge_small_kernel(
    const int64_t* __restrict__ sk,
    const uint64_t* __restrict__ vals, const uint32_t* __restrict__ n_in, SessArgs a, SessOut o,
    uint32_t* __restrict__ long_heads, uint32_t* __restrict__ n_long) {
  const uint32_t n = *n_in;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int64_t k = sk[i];
    if (k == INT64_MAX) continue;
    const int64_t slot = k >> a.tbits;
    if (i > 0 && (sk[i - 1] >> a.tbits) == slot) continue;  // not a segment head
    uint32_t j = i + 1;
    while (j < n && j - i <= kSessLongSeg) {
      const int64_t kj = sk[j];
      if (kj == INT64_MAX || (kj >> a.tbits) != slot) break;
      ++j;
    }
    if (j - i > kSessLongSeg) {
      long_heads[atomicAdd(n_long, 1u)] = i;
      continue;
    }
    sess_merge_segment(sk, vals, i, j, slot, a, o);
  }
}

// Dense variant over the segment list written by session_lookup_sort (position | length << 32):
// every lane owns a key, none scans for segment heads.
__global__ __launch_bounds__(256) void session_merge_heads_kernel(
    const int64_t* __restrict__ sk, const uint64_t* __restrict__ vals,
    const uint64_t* __restrict__ heads, const uint32_t* __restrict__ n_heads, SessArgs a,
    SessOut o, uint32_t* __restrict__ long_heads, uint32_t* __restrict__ n_long) {
  const uint32_t nh = *n_heads;
  for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += gridDim.x * blockDim.x) {
    const uint64_t hv = heads[h];
    const uint32_t i = (uint32_t)hv, len = (uint32_t)(hv >> 32);
    if (len > kSessLongSeg) {
      long_heads[atomicAdd(n_long, 1u)] = i;
      continue;
    }
    sess_merge_segment(sk, vals, i, i + len, sk[(size_t)i * a.st] >> a.tbits, a, o);
  }
}

// One wave per long key segment: lanes find the runs of their 64-record chunk (ts gaps > gap
// split runs) and their accumulators with shuffles; lane 0 folds the runs in ts order.
__global__ __launch_bounds__(256) void session_merge_long_kernel(
    const int64_t* __restrict__ sk,
    const uint64_t* __restrict__ vals, const uint32_t* __restrict__ n_in,
    const uint32_t* __restrict__ heads, const uint32_t* __restrict__ n_heads, SessArgs a,
    SessOut o) {
  const uint32_t n = *n_in, nh = *n_heads;
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t h = wave; h < nh; h += nwaves) {
    const uint32_t start = heads[h];
    const int64_t slot = sk[(size_t)start * a.st] >> a.tbits;
    const int64_t tmask = ((int64_t)1 << a.tbits) - 1;
    SessState st;
    sess_load(st, o.sess + slot * kSess);
    uint64_t late = 0;
    bool overflow = false;
    int64_t last_ts = INT64_MIN;
    // Lane 0's pending run: a run ending on a chunk's last lane may continue in the next chunk,
    // so runs are committed only once the following run starts more than `gap` later.
    bool pv = false;
    int64_t ps = 0, pe = 0;
    uint64_t pa = 0;
    uint32_t pc = 0;
    for (uint32_t b0 = start;; b0 += 64) {
      const uint32_t i = b0 + lane;
      const int64_t ki = i < n ? sk[(size_t)i * a.st] : INT64_MAX;
      const bool in = ki != INT64_MAX && (ki >> a.tbits) == slot;
      const unsigned long long inm = __ballot(in);
      if (!inm) break;
      const int64_t ts = in ? a.tbase + (ki & tmask) : 0;
      const uint64_t v = in ? agg_lift(a.agg, vals[(size_t)i * a.st]) : 0;
      const int64_t prev_ts = __shfl_up(ts, 1);
      const bool head = in && (lane == 0 || ts > prev_ts + a.gap);
      // Segmented inclusive scan of (acc, cnt) over runs.
      uint64_t acc = v;
      uint32_t cnt = in ? 1u : 0u;
      const unsigned long long hm = __ballot(head);
      const unsigned long long below = hm & ((lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1ull));
      const int run0 = 63 - __clzll(below);
      for (int off = 1; off < 64; off <<= 1) {
        const uint64_t ya = __shfl_up(acc, off);
        const uint32_t yc = __shfl_up(cnt, off);
        if (in && lane - off >= run0) {
          acc = agg_combine(a.agg, ya, acc);
          cnt += yc;
        }
      }
      // Run ends: next lane is a head or out of range.
      const bool next_head = __shfl_down(head ? 1 : 0, 1) != 0;
      const bool next_in = __shfl_down(in ? 1 : 0, 1) != 0;
      const bool run_end = in && (lane == 63 || !next_in || next_head);
      const unsigned long long em = __ballot(run_end);
      const int64_t chunk_last = __shfl(ts, 63 - __clzll(inm));
      last_ts = chunk_last > last_ts ? chunk_last : last_ts;
      unsigned long long rem = em;
      while (rem) {
        const int e = __ffsll((long long)rem) - 1;
        rem &= rem - 1;
        const unsigned long long hb = hm & ((e == 63) ? ~0ull : ((1ull << (e + 1)) - 1ull));
        const int r0 = 63 - __clzll(hb);
        const int64_t cs = __shfl(ts, r0);
        const int64_t ce = __shfl(ts, e) + a.gap;
        const uint64_t ca = __shfl(acc, e);
        const uint32_t cc = __shfl(cnt, e);
        if (lane == 0) {
          if (pv && cs <= pe) {  // continues the pending run across the chunk boundary
            pe = ce > pe ? ce : pe;
            pa = agg_combine(a.agg, pa, ca);
            pc += cc;
          } else {
            if (pv) sess_commit(st, overflow, late, slot, ps, pe, pa, pc, a, o);
            ps = cs;
            pe = ce;
            pa = ca;
            pc = cc;
            pv = true;
          }
        }
      }
      if (__popcll(inm) < 64) break;
    }
    if (lane == 0) {
      if (pv) sess_commit(st, overflow, late, slot, ps, pe, pa, pc, a, o);
      sess_finish(st, slot, last_ts, late, overflow, a, o);
    }
  }
}

// Fire due sessions: one lane per slot whose due time has passed.
__global__ __launch_bounds__(256) void session_fire_kernel(
    SessArgs a, const uint64_t* __restrict__ keys_g, SessRec* __restrict__ sess, int64_t* __restrict__ slot_due, ExprProg map, ExprProg filt,
    uint64_t* __restrict__ out_key, int64_t* __restrict__ out_start, int64_t* __restrict__ out_end,
    double* __restrict__ out_val, uint64_t* __restrict__ out_raw, uint32_t* __restrict__ out_cnt,
    uint32_t* __restrict__ out_n, uint32_t out_cap) {
  extern __shared__ __attribute__((aligned(16))) double ssm[];
  LdsCol vars{ssm + threadIdx.x, 256};
  LdsCol stack{ssm + kExprVars * 256 + threadIdx.x, 256};
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < a.nslots;
       base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t slot = base + threadIdx.x;
    const bool due = slot < a.nslots && slot_due[slot * kSlotMeta] <= a.wm;
    if (!__ballot(due)) continue;
    SessState st;
    sess_clear(st);
    if (due) sess_load(st, sess + slot * kSess);
    const uint64_t key = due ? keys_g[slot] : 0;
#pragma unroll
    for (int j = 0; j < kSess; ++j) {
      bool emit = false;
      double val = 0.0;
      if (due && st.cnt[j]) {
        const int64_t maxts = st.end[j] - 1;
        if (maxts <= a.wm && (!(st.flags[j] & 1u) || (st.flags[j] & 2u))) {
          const double v0 = agg_result_f64(a.agg, st.acc[j], st.cnt[j]);
          val = v0;
          emit = true;
          if (map.ncode || filt.ncode) {
            vars.set(0, v0);
            vars.set(1, (double)st.cnt[j]);
            vars.set(2, (double)st.start[j]);
            vars.set(3, (double)st.end[j]);
            vars.set(4, (double)key);
            vars.set(5, (double)(int64_t)st.acc[j]);
            if (map.ncode) val = expr_eval_t(map, stack, vars);
            vars.set(6, val);
            if (filt.ncode) emit = expr_eval_t(filt, stack, vars) != 0.0;
          }
          st.flags[j] = 1u;
        }
      }
      const unsigned long long m = __ballot(emit);
      if (m) {
        uint32_t wb = 0;
        if (lane_id() == 0) wb = atomicAdd(out_n, (uint32_t)__popcll(m));
        wb = __shfl(wb, 0);
        if (emit) {
          const uint32_t q = wb + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
          if (q < out_cap) {
            out_key[q] = key;
            out_start[q] = st.start[j];
            out_end[q] = st.end[j];
            out_val[q] = val;
            out_raw[q] = st.acc[j];
            out_cnt[q] = st.cnt[j];
          }
        }
      }
    }
    if (due) {
      // Drop sessions past cleanup (maxTs + lateness <= wm).
#pragma unroll
      for (int j = 0; j < kSess; ++j)
        if (st.cnt[j] && (st.end[j] - 1) + a.lateness <= a.wm) st.cnt[j] = 0;
      sess_store(st, sess + slot * kSess);
      slot_due[slot * kSlotMeta] = sess_due(st, a.lateness);
    }
  }
}

// Evict (spill) slots idle since before `idle_before` (or listed in `slots`): pack their key and
// sessions into staging rows, tombstone the slot and insert the key into the spill set.
constexpr int kEvictBlock = 1024;

__global__ __launch_bounds__(kEvictBlock) void session_evict_kernel(
    SessArgs a, uint64_t* __restrict__ keys_g, SessRec* __restrict__ sess, int64_t* __restrict__ slot_due,
    int64_t* __restrict__ slot_last, int64_t idle_before, const int64_t* __restrict__ slots,
    uint32_t nslots_list, uint64_t* __restrict__ spill_set, uint32_t spill_mask,
    int64_t* __restrict__ st_key, int64_t* __restrict__ st_start, int64_t* __restrict__ st_end,
    int64_t* __restrict__ st_acc, int64_t* __restrict__ st_cnt, int64_t* __restrict__ st_flags,
    uint32_t* __restrict__ n_rows, uint32_t row_cap, uint32_t* __restrict__ n_evicted) {
  const int64_t total = slots ? (int64_t)nslots_list : a.nslots;
  const int lane = lane_id();
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < total;
       base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    int64_t slot = -1;
    uint64_t key = kEmptyKey;
    bool take = false;
    if (i < total) {
      slot = slots ? slots[i] : i;
      key = keys_g[slot];
      take = key != kEmptyKey && key != kTombKey && (slots || slot_last[slot * kSlotMeta] < idle_before);
    }
    SessState st;
    sess_clear(st);
    if (take) sess_load(st, sess + slot * kSess);
    const int nst = sess_count(st);
    // Block-aggregated row allocation: one global atomic per block iteration (same-address
    // atomics serialize at L2; per-wave atomics made this kernel atomic-bound).
    __shared__ uint32_t wsum[kEvictBlock / 64];
    __shared__ uint32_t bdone;
    const int wid = threadIdx.x >> 6;
    uint32_t x = take ? (uint32_t)nst : 0u;
    uint32_t incl = x;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    if (threadIdx.x == 0) bdone = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t run = 0;
      for (int w = 0; w < kEvictBlock / 64; ++w) {
        const uint32_t t = wsum[w];
        wsum[w] = run;
        run += t;
      }
      const uint32_t base = run ? atomicAdd(n_rows, run) : 0u;
      for (int w = 0; w < kEvictBlock / 64; ++w) wsum[w] += base;
    }
    __syncthreads();
    const uint32_t q = wsum[wid] + incl - x;
    bool done = false;
    if (take && nst == 0) {  // no live session: free the slot, the key is not spilled
      done = true;
    } else if (take && q + nst <= row_cap) {
      uint32_t r = q;
#pragma unroll
      for (int j = 0; j < kSess; ++j) {
        if (st.cnt[j]) {
          st_key[r] = (int64_t)key;
          st_start[r] = st.start[j];
          st_end[r] = st.end[j];
          st_acc[r] = (int64_t)st.acc[j];
          st_cnt[r] = st.cnt[j];
          st_flags[r] = st.flags[j];
          ++r;
        }
      }
      SessState empty;
      sess_clear(empty);
      sess_store(empty, sess + slot * kSess);
      set_insert(spill_set, spill_mask, key);
      done = true;
    }  // else: staging full, the key stays resident this round
    if (done) {
      slot_due[slot * kSlotMeta] = INT64_MAX;
      slot_last[slot * kSlotMeta] = INT64_MIN;
      keys_g[slot] = kTombKey;
    }
    const unsigned long long dm = __ballot(done);
    if (lane == 0 && dm) atomicAdd(&bdone, (uint32_t)__popcll(dm));
    __syncthreads();
    if (threadIdx.x == 0 && bdone) atomicAdd(n_evicted, bdone);
    __syncthreads();  // wsum / bdone are rewritten by the next iteration
  }
}

// Forget keys that left the host store (tombstones: probing continues past them).
__global__ __launch_bounds__(256) void set_erase_kernel(uint64_t* __restrict__ set, uint32_t mask,
                                                        const int64_t* __restrict__ keys,
                                                        int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = (uint64_t)keys[i];
    uint32_t s = (uint32_t)(mix64(key) >> 32) & mask;
    for (uint32_t p = 0; p <= mask; ++p) {
      const uint64_t k = set[s];
      if (k == key) {
        set[s] = kTombKey;
        break;
      }
      if (k == kEmptyKey) break;
      s = (s + 1) & mask;
    }
  }
}

// Grow / compact the device spill set without a host round trip: every live key of the old
// set (not empty, not a tombstone) is re-inserted into the fresh, larger set. The old set holds
// exactly the host store's keys (inserted by the lookup/evict kernels, erased on release), so
// the result equals a rebuild from the store, including keys whose host insert is still queued.
// Batch insert into / membership probe of a device key set (open addressing on mix64 >> 32,
// linear probing, kEmptyKey empty, kTombKey erased) -- the rolling spill tier's set of keys that
// live in host DRAM. The probe writes one byte per key and counts hits with one device-scope
// atomic per workgroup.
__global__ __launch_bounds__(256) void set_insert_kernel(uint64_t* __restrict__ set, uint32_t mask,
                                                         const int64_t* __restrict__ keys,
                                                         int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    set_insert(set, mask, (uint64_t)keys[i]);
}

__global__ __launch_bounds__(256) void set_probe_kernel(const uint64_t* __restrict__ set,
                                                        uint32_t mask,
                                                        const int64_t* __restrict__ keys, int64_t n,
                                                        uint8_t* __restrict__ hit,
                                                        uint32_t* __restrict__ n_hit) {
  __shared__ uint32_t s_hits;
  if (threadIdx.x == 0) s_hits = 0;
  __syncthreads();
  uint32_t h = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool in = set_contains(set, mask, (uint64_t)keys[i]);
    hit[i] = in ? 1 : 0;
    h += in;
  }
  for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d);
  if (lane_id() == 0 && h) atomicAdd(&s_hits, h);
  __syncthreads();
  if (threadIdx.x == 0 && s_hits) atomicAdd(n_hit, s_hits);
}

__global__ __launch_bounds__(256) void set_rehash_kernel(const uint64_t* __restrict__ old,
                                                         int64_t n_old, uint64_t* __restrict__ neu,
                                                         uint32_t new_mask) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_old;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = old[i];
    if (k < kTombKey) set_insert(neu, new_mask, k);
  }
}

// Rebuild the slot table without tombstones: every live slot is re-inserted into fresh arrays
// (same sub-table, new position) with its sessions, due time and last activity.
__global__ __launch_bounds__(256) void session_rehash_kernel(
    SessArgs a, const uint64_t* __restrict__ keys_o, const SessRec* __restrict__ sess_o,
    const int64_t* __restrict__ due_o, const int64_t* __restrict__ last_o,
    uint64_t* __restrict__ keys_n, SessRec* __restrict__ sess_n, int64_t* __restrict__ due_n,
    int64_t* __restrict__ last_n, uint32_t* __restrict__ inserted) {
  // Inserted keys are counted per workgroup (a device-scope atomic per key on one counter
  // serialised across the XCDs: 7.4 ms for 5.5M keys).
  __shared__ uint32_t s_ins;
  if (threadIdx.x == 0) s_ins = 0;
  __syncthreads();
  const uint32_t mask = (1u << a.cap_log2) - 1;
  uint32_t ins = 0;
  for (int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; slot < a.nslots;
       slot += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys_o[slot];
    if (key == kEmptyKey || key == kTombKey) continue;
    const int64_t sub = slot >> a.cap_log2;
    uint64_t* keys = keys_n + (sub << a.cap_log2);
    bool claimed = false;
    const uint32_t s = sess_probe_claim(keys, key, mask, &claimed);
    ins += claimed;
    const int64_t ns = (sub << a.cap_log2) | s;  // never kNoSlot: the old table held the key
#pragma unroll
    for (int j = 0; j < kSess; ++j) sess_n[ns * kSess + j] = sess_o[slot * kSess + j];
    due_n[ns * kSlotMeta] = due_o[slot * kSlotMeta];
    last_n[ns * kSlotMeta] = last_o[slot * kSlotMeta];
  }
  for (int d = 32; d >= 1; d >>= 1) ins += __shfl_xor(ins, d);
  if (lane_id() == 0 && ins) atomicAdd(&s_ins, ins);
  __syncthreads();
  if (threadIdx.x == 0 && s_ins && inserted) atomicAdd(inserted, s_ins);
}

// ------------------------------------------------------------------------------------------
// Checkpoint support (K17): key group of every exported key, and re-insertion of restored keys.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void keygroup_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                       int hash_mode,
                                                       const int32_t* __restrict__ jhash,
                                                       int max_par, int32_t* __restrict__ kg) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    const int32_t h = hash_mode ? jhash[k] : java_long_hash((int64_t)k);
    kg[i] = key_group_of_hash(h, max_par);
  }
}

// Insert keys into a fresh sub-table layout (sub = top nsub_log2 bits of mix64, linear probing on
// the low bits -- the same placement window_agg / the lookups use). slot = -1 if the sub-table is
// full.
__global__ __launch_bounds__(256) void table_insert_kernel(const uint64_t* __restrict__ keys,
                                                           int64_t n, int nsub_log2, int cap_log2,
                                                           uint64_t* __restrict__ keys_g,
                                                           int64_t* __restrict__ slots) {
  const uint32_t mask = (1u << cap_log2) - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    const uint64_t sub = sub_table_of(key, nsub_log2);
    const uint32_t s = global_probe_insert(keys_g + (sub << cap_log2), key, mask);
    slots[i] = s == kNoSlot ? -1 : (int64_t)((sub << cap_log2) | s);
  }
}

// Session slot table insert for keys promoted back from host DRAM: the same tombstone-reusing
// probe as the session lookup (sess_probe_insert), so a sub-table whose free slots are all
// tombstones still takes the key. slot = -1 only if the sub-table has neither.
__global__ __launch_bounds__(256) void session_slot_insert_kernel(
    const uint64_t* __restrict__ keys, int64_t n, int nsub_log2, int cap_log2,
    uint64_t* __restrict__ keys_g, int64_t* __restrict__ slots, uint32_t* __restrict__ inserted) {
  const uint32_t mask = (1u << cap_log2) - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    const uint64_t sub = sub_table_of(key, nsub_log2);
    const uint32_t s = sess_probe_insert(keys_g + (sub << cap_log2), key, mask, inserted);
    slots[i] = s == kNoSlot ? -1 : (int64_t)((sub << cap_log2) | s);
  }
}

// Promoted keys' slot records (host store -> HBM): rec rows [key][kSess][4] go to the slots the
// insert found; a key without a slot (sub-table full) is counted in n_bad and stays on the host.
__global__ __launch_bounds__(256) void session_promote_kernel(
    const int64_t* __restrict__ slots, const int64_t* __restrict__ rec,
    const int64_t* __restrict__ last, int64_t n, int64_t* __restrict__ sess,
    int64_t* __restrict__ slot_due, int64_t* __restrict__ slot_last, uint32_t* __restrict__ n_bad) {
  constexpr int W = kSess * 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = slots[i];
    if (s < 0) {
      atomicAdd(n_bad, 1u);
      continue;
    }
#pragma unroll
    for (int j = 0; j < W; ++j) sess[s * W + j] = rec[i * W + j];
    slot_due[s * kSlotMeta] = INT64_MIN;  // the next fire sweep recomputes the due time
    slot_last[s * kSlotMeta] = last[i];
  }
}

// Promoted keys from host promote rows (SessionStore.extract_rows_into): one row of 8 int64
// {key, start, end, acc, cnt | flags << 32, last activity, position, sessions of the key} per
// session, a key's rows adjacent with position 0 first. Phase 0 (position-0 rows, one per key:
// no two threads insert the same key) finds or inserts the key's slot, writes record 0 and
// zeroes the records the key does not fill; phase 1 writes the other positions into the slot
// their position-0 row found. slots[i] = -1 (phase 0: counted in n_bad) when the sub-table is
// full.
__global__ __launch_bounds__(256) void session_promote_rows_kernel(
    const int64_t* __restrict__ rows, int64_t n, int nsub_log2, int cap_log2, int phase,
    uint64_t* __restrict__ keys_g, int64_t* __restrict__ slots, int64_t* __restrict__ sess,
    int64_t* __restrict__ slot_due, int64_t* __restrict__ slot_last,
    uint32_t* __restrict__ inserted, uint32_t* __restrict__ n_bad) {
  constexpr int W = kSess * 4;
  const uint32_t mask = (1u << cap_log2) - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t* r = rows + i * 8;
    const int64_t pos = r[6], nsess = r[7];
    if ((phase == 0) != (pos == 0)) continue;
    int64_t s;
    if (phase == 0) {
      const uint64_t key = (uint64_t)r[0];
      const uint64_t sub = sub_table_of(key, nsub_log2);
      const uint32_t s32 = sess_probe_insert(keys_g + (sub << cap_log2), key, mask, inserted);
      if (s32 == kNoSlot) {
        slots[i] = -1;
        atomicAdd(n_bad, 1u);
        continue;
      }
      s = (int64_t)((sub << cap_log2) | s32);
      slots[i] = s;
      for (int j = (int)nsess * 4; j < W; ++j) sess[s * W + j] = 0;
      slot_due[s * kSlotMeta] = INT64_MIN;  // the next fire sweep recomputes the due time
      slot_last[s * kSlotMeta] = r[5];
    } else {
      s = slots[i - pos];
      slots[i] = s;
      if (s < 0) continue;
    }
    int64_t* o = sess + s * W + pos * 4;
    o[0] = r[1];
    o[1] = r[2];
    o[2] = r[3];
    o[3] = r[4];
  }
}

// ------------------------------------------------------------------------------------------
// Median of `process` windows (ComputeCpuMiddle.java:36-47): elements are radix-
// sorted by (key, order-preserving value bits); one thread per key segment reads the middle
// element(s). Java Collections.sort order on Double: -0.0 < 0.0, NaN last (all NaN equal).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void f64_order_bits_kernel(const uint64_t* __restrict__ v,
                                                             int64_t n, uint64_t* __restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    o[i] = f64_order_bits(v[i]);
}

__global__ __launch_bounds__(256) void segment_median_kernel(const int64_t* __restrict__ heads,
                                                             int64_t nseg, int64_t total,
                                                             const uint64_t* __restrict__ ord,
                                                             double* __restrict__ out) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg;
       s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = heads[s], b = s + 1 < nseg ? heads[s + 1] : total;
    const int64_t n = b - a;
    double m = 0.0;
    if (n > 0) {
      const double hi = as_f64(f64_from_order_bits(ord[a + n / 2]));
      m = (n & 1) ? hi : (hi + as_f64(f64_from_order_bits(ord[a + n / 2 - 1]))) / 2.0;
    }
    out[s] = m;
  }
}

// Median of every segment of *unsorted* order-preserving f64 bits (segments = a key's values
// after the list window's counting sort by key, csrc/listwin_hip.hip). One wave per segment: a
// segment of up to kMedLds values is staged in the wave's LDS slice and radix-selected there (8
// byte passes, 256-bin LDS histogram; the lower middle element from one more pass); a longer
// one is resolved by two radix selects over global memory.
constexpr int kMedLds = 2048;

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ uint64_t wave_radix_select(const uint64_t* __restrict__ v, int64_t n, int64_t k,
                                      uint32_t* hist, int lane) {
  uint64_t prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = lane; i < 256; i += 64) hist[i] = 0;
    wave_lds_sync();
    for (int64_t i = lane; i < n; i += 64) {
      const uint64_t x = v[i];
      if ((x & mask) == prefix) atomicAdd(&hist[(x >> shift) & 255u], 1u);
    }
    wave_lds_sync();
    // Lane l owns bins 4l..4l+3: find the bin holding the k-th candidate.
    uint32_t c[4], tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = hist[lane * 4 + j];
      tot += c[j];
    }
    uint32_t incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    const uint32_t excl = incl - tot;
    int found = -1;
    int64_t kk = k - excl;
    if (k >= excl && k < incl) {
      for (int j = 0; j < 4; ++j) {
        if (kk < c[j]) {
          found = lane * 4 + j;
          break;
        }
        kk -= c[j];
      }
    }
    const unsigned long long who = __ballot(found >= 0);
    const int src = who ? __ffsll((long long)who) - 1 : 0;
    const int bin = __shfl(found, src);
    k = __shfl(kk, src);
    prefix |= (uint64_t)bin << shift;
    mask |= (uint64_t)255 << shift;
    wave_lds_sync();
  }
  return prefix;
}

__global__ __launch_bounds__(256) void segment_median_select_kernel(
    const int64_t* __restrict__ heads, int64_t nseg, int64_t total, const uint64_t* __restrict__ ord,
    double* __restrict__ out) {
  __shared__ uint64_t buf[4][kMedLds];
  __shared__ uint32_t hbuf[4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t* b = buf[w];
  for (int64_t s = (int64_t)blockIdx.x * 4 + w; s < nseg; s += (int64_t)gridDim.x * 4) {
    const int64_t a = heads[s], e = s + 1 < nseg ? heads[s + 1] : total;
    const int64_t n = e - a;
    uint64_t hi_bits = 0, lo_bits = 0;
    if (n <= 0) {
      if (lane == 0) out[s] = 0.0;
      continue;
    }
    if (n <= kMedLds) {
      // Segment staged in LDS once, then a radix select of the upper middle element (8 byte
      // passes over LDS, 256-bin histogram) -- a full bitonic sort of the segment did ~10x more
      // LDS traffic -- and the lower middle one from one more pass: the largest element below
      // it, unless enough elements tie with it.
      for (int i = lane; i < n; i += 64) b[i] = ord[a + i];
      wave_lds_sync();
      hi_bits = wave_radix_select(b, n, n / 2, hbuf[w], lane);
      if (n & 1) {
        lo_bits = hi_bits;
      } else {
        uint32_t less = 0;
        uint64_t below = 0;
        bool any = false;
        for (int i = lane; i < n; i += 64) {
          const uint64_t x = b[i];
          if (x < hi_bits) {
            ++less;
            if (!any || x > below) below = x;
            any = true;
          }
        }
        for (int o = 32; o >= 1; o >>= 1) {
          less += __shfl_xor(less, o);
          const uint64_t ob = __shfl_xor(below, o);
          const bool oa = __shfl_xor((int)any, o) != 0;
          if (oa && (!any || ob > below)) below = ob;
          any = any || oa;
        }
        // sorted[n/2 - 1] is hi itself when fewer than n/2 elements are below it
        lo_bits = less < (uint32_t)(n / 2) ? hi_bits : below;
      }
      wave_lds_sync();
    } else {
      uint32_t* hist = reinterpret_cast<uint32_t*>(b);
      hi_bits = wave_radix_select(ord + a, n, n / 2, hist, lane);
      lo_bits = (n & 1) ? hi_bits : wave_radix_select(ord + a, n, n / 2 - 1, hist, lane);
    }
    if (lane == 0) {
      const double hi = as_f64(f64_from_order_bits(hi_bits));
      out[s] = (n & 1) ? hi : (hi + as_f64(f64_from_order_bits(lo_bits))) / 2.0;
    }
  }
}

int grid_for(int64_t n, int block, int max_blocks) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return (int)(g < max_blocks ? g : max_blocks);
}

}  // namespace

namespace gpu {

// hipDeviceScheduleSpin: host threads spin (instead of yielding / sleeping) in every
// synchronisation; set before the device's context exists (bench.py MXS_SPIN=1).
int set_spin_schedule() { return (int)hipSetDeviceFlags(hipDeviceScheduleSpin); }

int h2d_async(void* dst, const void* src, size_t bytes, intptr_t stream) {
  return (int)hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
}

int host_register(void* p, size_t bytes) {
  return (int)hipHostRegister(p, bytes, hipHostRegisterDefault);
}

int host_unregister(void* p) { return (int)hipHostUnregister(p); }

int d2h_async(void* dst, const void* src, size_t bytes, intptr_t stream) {
  return (int)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream);
}

int d2h_kernel(void* dst_host, const D2HCopy* copies, int n, intptr_t stream,
               const uint32_t* n_dev, int max_blocks) {
  // Device-side address of the pinned host slab (mapped host memory).
  void* dd = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dd, dst_host, 0);
  if (e != hipSuccess || !dd) return (int)(e != hipSuccess ? e : hipErrorInvalidValue);
  D2HBatch b{};
  if (n < 1 || n > kD2HMax) return (int)hipErrorInvalidValue;
  b.n = n;
  b.n_dev = n_dev;
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    b.c[i] = copies[i];
    if ((copies[i].bytes & 15) || (copies[i].dst_off & 15) || ((uintptr_t)copies[i].src & 15))
      return (int)hipErrorInvalidValue;  // 16-byte granules only (the caller pads)
    total += copies[i].bytes;
  }
  // max_blocks: a copy overlapping compute on a side stream is PCIe-bound; a small grid leaves
  // the CUs to the compute stream.
  const int grid = grid_for(total / 16, 256 * 4, max_blocks < 1 ? 1 : max_blocks > 1024 ? 1024 : max_blocks);
  hipLaunchKernelGGL(d2h_copy_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (unsigned char*)dd, b);
  return (int)hipGetLastError();
}

int h2d_kernel(void* dst_dev, const void* src_host, int64_t bytes, intptr_t stream,
               int max_blocks) {
  // The copy kernel reading a mapped pinned host buffer over PCIe (every CU's loads in flight
  // at once) instead of the SDMA engine: the text batches of the file/socket sources.
  void* sd = nullptr;
  hipError_t e = hipHostGetDevicePointer(&sd, const_cast<void*>(src_host), 0);
  if (e != hipSuccess || !sd) return (int)(e != hipSuccess ? e : hipErrorInvalidValue);
  if (bytes <= 0) return 0;
  if ((bytes & 15) || ((uintptr_t)sd & 15) || ((uintptr_t)dst_dev & 15))
    return (int)hipErrorInvalidValue;  // 16-byte granules only (the caller pads)
  D2HBatch b{};
  b.n = 1;
  b.c[0].src = sd;
  b.c[0].dst_off = 0;
  b.c[0].bytes = bytes;
  b.c[0].esz = 0;
  const int grid = grid_for(bytes / 16, 256 * 4, max_blocks < 1 ? 1 : max_blocks > 2048 ? 2048 : max_blocks);
  hipLaunchKernelGGL(d2h_copy_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (unsigned char*)dst_dev, b);
  return (int)hipGetLastError();
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void gen_events(uint64_t* keys, int64_t* ts, uint64_t* vals, int64_t n, uint64_t seed,
                uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
                int64_t ts_span, int64_t disorder, int64_t val_lo, int64_t val_span,
                int32_t val_f64, double zipf_s, intptr_t stream, uint64_t key_base) {
  if (n <= 0) return;
  // mode bit 2: scalar stores (a column that is not 16-byte aligned; int32 keys need 8 bytes)
  const uintptr_t kmis = (uintptr_t)keys & ((val_f64 & 2) ? 7 : 15);
  const int32_t mode = val_f64 | ((kmis | (((uintptr_t)ts | (uintptr_t)vals) & 15)) ? 4 : 0);
  hipLaunchKernelGGL(gen_events_kernel, dim3(grid_for((n + 1) / 2, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, keys, ts, vals, n, seed, stream_id, idx0, nkeys, ts_base,
                     (double)ts_span / (double)n, (uint64_t)(disorder + 1), val_lo,
                     (uint64_t)(val_span > 0 ? val_span : 0), mode, zipf_s, key_base);
  HIP_CHECK(hipGetLastError());
}

void step_begin(uint32_t* cursor, int nb, int64_t* stats, intptr_t stream) {
  hipLaunchKernelGGL(step_begin_kernel, dim3(grid_for(nb, 256, 64)), dim3(256), 0,
                     (hipStream_t)stream, cursor, nb, stats);
  HIP_CHECK(hipGetLastError());
}

void step_finish(const int64_t* stats, int64_t* local_maxts, int64_t bound, int32_t event_mode,
                 int64_t proc_now, int64_t* red, const uint32_t* flags, intptr_t stream,
                 int32_t idle, int64_t* host_red, int32_t fill_word, const uint32_t* cursor,
                 int nb, uint32_t* next_cursor, int64_t* next_stats) {
  hipLaunchKernelGGL(step_finish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, stats,
                     local_maxts, bound, event_mode, proc_now, red, flags, idle, host_red,
                     fill_word && cursor ? 1 : 0, cursor, nb, next_stats ? next_cursor : nullptr,
                     next_cursor ? next_stats : nullptr);
  HIP_CHECK(hipGetLastError());
}

void combine_check(const uint32_t* flags, const uint32_t* counts, int nb, int64_t* chk,
                   intptr_t stream) {
  hipLaunchKernelGGL(combine_check_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, flags,
                     counts, nb, chk);
  HIP_CHECK(hipGetLastError());
}

void bucket_repack(const uint64_t* src, const uint32_t* counts, int nb, uint32_t src_cap,
                   uint32_t dst_cap, int words, uint64_t* dst, uint64_t* xstat, intptr_t stream) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(bucket_repack_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, src,
                     counts, src_cap, dst_cap, words, dst, (unsigned long long*)xstat);
  HIP_CHECK(hipGetLastError());
}

void neg_max_u32(const uint32_t* counts, int nb, int64_t* out, intptr_t stream) {
  hipLaunchKernelGGL(neg_max_u32_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, counts, nb,
                     out);
  HIP_CHECK(hipGetLastError());
}

void widen_i32(const int32_t* in, int64_t n, int64_t* out, intptr_t stream) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(widen_i32_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in,
                     n, out);
  HIP_CHECK(hipGetLastError());
}

void zero_panes(void* acc, int acc_bytes, uint32_t* cnt, uint8_t* dirty, int64_t so, int64_t n,
                intptr_t stream) {
  if (n <= 0) return;
  // slabs are nslots-multiples of 64 slots: every range below is a whole number of 16 bytes
  uint8_t* a = (uint8_t*)acc + so * acc_bytes;
  uint8_t* b = (uint8_t*)(cnt + so);
  uint8_t* c = dirty + so;
  const int64_t na = n * acc_bytes / 16, nb = n * 4 / 16, nc = n / 16;
  if ((((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) || (n & 15)) {
    HIP_CHECK(hipMemsetAsync(a, 0, n * acc_bytes, (hipStream_t)stream));
    HIP_CHECK(hipMemsetAsync(b, 0, n * 4, (hipStream_t)stream));
    HIP_CHECK(hipMemsetAsync(c, 0, n, (hipStream_t)stream));
    return;
  }
  const int64_t tot = na + nb + nc;
  const int64_t blocks = std::min<int64_t>(2048, (tot + 255) / 256);
  hipLaunchKernelGGL(zero3_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (uint4*)a, na, (uint4*)b, nb, (uint4*)c, nc);
  HIP_CHECK(hipGetLastError());
}

void fill_u64(uint64_t* p, int64_t n, uint64_t v, intptr_t stream) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(fill_u64_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p,
                     n, v);
  HIP_CHECK(hipGetLastError());
}

int getenv_int(const char* name, int def) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : def;
}

// One compact-partition instantiation: LDS attribute set once, one group per 64K events.
template <bool ONE, int RB, bool K32, bool PAIR>
void launch_compact(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
                    const int32_t* jhash_tab, int64_t n, int64_t chunk, int blocks,
                    const PartPlan& plan, const int32_t* kg_dest, uint32_t* cursor, Rec* out,
                    int64_t* stats, uint32_t* late_idx, uint32_t late_cap, intptr_t stream) {
  if constexpr (RB == 8) {
    // MXS_PART_CU8=1: 8192-record rounds (half the rounds, barriers and per-round scans of a
    // workgroup's 64K events; A/B knob)
    static const bool cu8 = getenv_int("MXS_PART_CU8", 0) != 0;
    if (cu8) {
      auto k8 = partition_compact_kernel<1, 8, ONE, RB, K32, PAIR>;
      static bool attr8 = false;
      if (!attr8) {
        HIP_CHECK(hipFuncSetAttribute((const void*)k8, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)compact_lds_rb(8, 8)));
        attr8 = true;
      }
      const size_t lds8 = compact_lds_rb(8, 8) - (ONE ? (size_t)kKgLdsMax * 4 : 0);
      hipLaunchKernelGGL(k8, dim3(blocks), dim3(1024), lds8, (hipStream_t)stream, keys, ts, vals,
                         jhash_tab, n, chunk, plan, kg_dest, cursor, reinterpret_cast<RecC*>(out),
                         stats, late_idx, late_cap);
      HIP_CHECK(hipGetLastError());
      return;
    }
  }
  auto kfn = partition_compact_kernel<1, kCUProd, ONE, RB, K32, PAIR>;
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)compact_lds(kCUProd)));
    attr = true;
  }
  // One rank: no key-group hashing and no LDS kg table.
  const size_t lds = compact_lds(kCUProd) - (ONE ? (size_t)kKgLdsMax * 4 : 0);
  hipLaunchKernelGGL(kfn, dim3(blocks), dim3(1024), lds, (hipStream_t)stream, keys, ts, vals,
                     jhash_tab, n, chunk, plan, kg_dest, cursor, reinterpret_cast<RecC*>(out),
                     stats, late_idx, late_cap);
  HIP_CHECK(hipGetLastError());
}

static const bool kPairEnv = getenv_int("MXS_PAIR", 1) != 0;  // A/B knobs (profiles)
static const bool kFastEnv = getenv_int("MXS_PART_FAST", 1) != 0;


// ------------------------------------------------------------------------------------------
// Two-level partition, level 2 (8-byte records, one destination, > 512 buckets): one workgroup
// per coarse bucket splits its records into the 2^L fine buckets it owns (fine = the low L bits
// of the sub-table). The plain scatter wrote every record into one of 4096 open runs per
// workgroup -- partially written lines evicted long before they filled; here a workgroup has
// 2^L open runs, each wave writes its records as <= 2^L contiguous pieces (wave ballot per
// distinct fine bucket, one LDS atomic per piece), and no global atomic is needed: the fine
// buckets' cursors are this workgroup's LDS counters. Holes of the coarse staging are dropped.
// ------------------------------------------------------------------------------------------
constexpr int kSplitThreads = 1024;

// RB = 8: narrow RecN (hole: pane nibble 15); RB = 24: Rec (hole: t == kHoleT).
template <int RB>
struct SplitRec;
template <>
struct SplitRec<8> {
  uint2 r;
  __device__ __forceinline__ void load(const void* base, size_t i) {
    const unsigned long long w =
        __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(base) + i);
    r = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
  }
  __device__ __forceinline__ void hole() { r = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu); }
  __device__ __forceinline__ bool live() const { return (r.y & 15u) != kNarrowHoleT; }
  __device__ __forceinline__ uint64_t key() const { return (uint64_t)r.x; }
  __device__ __forceinline__ void store(void* base, size_t i) const {
    reinterpret_cast<uint2*>(base)[i] = r;
  }
};
template <>
struct SplitRec<24> {
  uint64_t w0, w1, w2;  // key | val | aux << 32 | t
  __device__ __forceinline__ void load(const void* base, size_t i) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(base) + 3 * i;
    w0 = __builtin_nontemporal_load(q);
    w1 = __builtin_nontemporal_load(q + 1);
    w2 = __builtin_nontemporal_load(q + 2);
  }
  __device__ __forceinline__ void hole() { w0 = w1 = w2 = ~0ull; }
  __device__ __forceinline__ bool live() const { return (uint32_t)w2 != kHoleT; }
  __device__ __forceinline__ uint64_t key() const { return w0; }
  __device__ __forceinline__ void store(void* base, size_t i) const {
    uint64_t* d = reinterpret_cast<uint64_t*>(base) + 3 * i;
    d[0] = w0;
    d[1] = w1;
    d[2] = w2;
  }
};

template <>
struct SplitRec<16> {  // RecC: key lo | key hi | int32 value | t (hole: t == kHoleT)
  uint4 r;
  __device__ __forceinline__ void load(const void* base, size_t i) {
    const u32x4_t w = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(base) + i);
    r = make_uint4(w.x, w.y, w.z, w.w);
  }
  __device__ __forceinline__ void hole() { r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, kHoleT); }
  __device__ __forceinline__ bool live() const { return r.w != kHoleT; }
  __device__ __forceinline__ uint64_t key() const { return (uint64_t)r.x | ((uint64_t)r.y << 32); }
  __device__ __forceinline__ void store(void* base, size_t i) const {
    reinterpret_cast<uint4*>(base)[i] = r;
  }
};

template <int RB>
__global__ __launch_bounds__(kSplitThreads) void partition_split_kernel(
    const void* __restrict__ coarse, const uint32_t* __restrict__ coarse_n, uint32_t ccap,
    PartPlan plan, int L, uint32_t* __restrict__ cursor, void* __restrict__ out,
    int64_t* __restrict__ stats) {
  __shared__ uint32_t scnt[32];
  __shared__ uint32_t sovf;
  const uint32_t c = blockIdx.x;
  const uint32_t nf = 1u << L, fmask = nf - 1u;
  if (threadIdx.x < nf) scnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) sovf = 0;
  __syncthreads();
  uint32_t n = coarse_n[c];
  n = n < ccap ? n : ccap;
  const size_t src0 = (size_t)c * ccap;
  const uint32_t bcap = plan.bucket_cap;
  const unsigned long long lt = (1ull << lane_id()) - 1ull;
  bool ovf = false;
  for (uint32_t base = 0; base < n; base += kSplitThreads * 4) {
    SplitRec<RB> r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t e = base + u * kSplitThreads + threadIdx.x;
      if (e < n)
        r[u].load(coarse, src0 + e);
      else
        r[u].hole();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool live = r[u].live();
      const uint32_t f = live ? sub_of(r[u].key(), plan) & fmask : 0xFFFFFFFFu;
      // One piece per distinct fine bucket in the wave: its lanes write contiguously.
      unsigned long long todo = __ballot(live);
      while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const uint32_t fl = __shfl(f, leader);
        const unsigned long long m = __ballot(live && f == fl);
        uint32_t b = 0;
        if (lane_id() == leader) b = atomicAdd(&scnt[fl], (uint32_t)__popcll(m));
        b = __shfl(b, leader);
        if (live && f == fl) {
          const uint32_t pos = b + (uint32_t)__popcll(m & lt);
          if (pos < bcap)
            r[u].store(out, (size_t)((c << L) | fl) * bcap + pos);
          else
            ovf = true;
        }
        todo &= ~m;
      }
    }
  }
  if (ovf) sovf = 1;
  __syncthreads();
  if (threadIdx.x < nf) cursor[(c << L) | threadIdx.x] = scnt[threadIdx.x];
  if (threadIdx.x == 0 && sovf)
    atomicOr((unsigned long long*)&stats[kStatOverflow], 1ull);  // bucket overflow: redo
}

template <bool ONE, int RB>
void dispatch_compact(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
                      const int32_t* jhash_tab, int64_t n, const PartPlan& plan,
                      const int32_t* kg_dest, uint32_t* cursor, Rec* out, int64_t* stats,
                      uint32_t* late_idx, uint32_t late_cap, intptr_t stream) {
  // 4096-record rounds, up to 64K events per workgroup (one group per CU: 86 KB of LDS),
  // i.e. one workgroup per CU at 16M events. Against 2048-record rounds / 32K events at two
  // groups per CU (kbench, profiles/r1_partition_rounds.md): 227 -> 198 us. Longer bucket
  // runs per group and bigger rounds cut the partial-sector writes and the per-group
  // reservation work; fewer, larger groups beat the higher occupancy.
  const int64_t per = std::min<int64_t>(65536, std::max<int64_t>(4096, (n + 255) / 256));
  const int blocks = grid_for(n, per, 4096);
  int64_t chunk = (n + blocks - 1) / blocks;
  // PAIR loads (two events per lane, 16-byte ts / value loads) need even group boundaries and
  // 16-byte aligned columns (8-byte for int32 keys); a misaligned view takes the lane-strided
  // kernel.
  const bool pair = ((uintptr_t)ts % 16 == 0) && ((uintptr_t)vals % 16 == 0) &&
                    ((uintptr_t)keys % (plan.key32 ? 8 : 16) == 0) && kPairEnv;
  if (pair) chunk = (chunk + 1) & ~(int64_t)1;
  PartPlan pl = plan;
  if (!kFastEnv) pl.ablate |= 8u;  // wave-vote fast path off
#define MXS_COMPACT(K32_, PAIR_)                                                                \
  launch_compact<ONE, RB, K32_, PAIR_>(keys, ts, vals, jhash_tab, n, chunk, blocks, pl,          \
                                       kg_dest, cursor, out, stats, late_idx, late_cap, stream)
  if (plan.key32) {
    if (pair) MXS_COMPACT(true, true);
    else MXS_COMPACT(true, false);
  } else {
    if (pair) MXS_COMPACT(false, true);
    else MXS_COMPACT(false, false);
  }
#undef MXS_COMPACT
}

void partition(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
               const int32_t* jhash_tab, int64_t n, const PartPlan& plan, const int32_t* kg_dest,
               uint32_t* cursor, Rec* out, int64_t* stats, uint32_t* late_idx, uint32_t late_cap,
               intptr_t stream) {
  const int nb = plan.nranks << plan.nsub_log2;
  if (plan.rec_words == 1) {
    // Narrow 8-byte records. Up to 512 buckets the LDS-staged compact kernel; more (e.g. 4096
    // dense sub-tables of a 10M-key window) the plain scatter (one destination). Several
    // destinations (the records exchange): the compact kernel's general bucket path, which
    // halves the all-to-all bytes of 16-byte records.
    if ((uint64_t)nb * plan.bucket_cap >= (1ull << 32))
      throw std::invalid_argument("partition: 8-byte record buffer above 2^32 records");
    if (plan.nranks != 1) {
      if (nb > kCMaxNb)
        throw std::invalid_argument("partition: 8-byte records to several ranks need <= 512 buckets");
      if (n <= 0) return;
      dispatch_compact<false, 8>(keys, ts, vals, jhash_tab, n, plan, kg_dest, cursor, out, stats,
                                 late_idx, late_cap, stream);
      return;
    }
    if (n <= 0) return;
    if (nb > kCMaxNb && plan.scratch && plan.scratch_cursor && nb <= kCMaxNb * 32) {
      // Two-level: compact staged partition into 512 coarse buckets, then the split kernel.
      int L = 0;
      while ((nb >> L) > kCMaxNb) ++L;
      PartPlan pc = plan;
      pc.nsub_log2 = plan.nsub_log2 - L;
      pc.bucket_cap = plan.bucket_cap << L;
      hipStream_t st = (hipStream_t)stream;
      HIP_CHECK(hipMemsetAsync(plan.scratch_cursor, 0, sizeof(uint32_t) * (nb >> L), st));
      dispatch_compact<true, 8>(keys, ts, vals, jhash_tab, n, pc, kg_dest, plan.scratch_cursor,
                                (Rec*)plan.scratch, stats, late_idx, late_cap, stream);
      hipLaunchKernelGGL(partition_split_kernel<8>, dim3(nb >> L), dim3(kSplitThreads), 0, st,
                         (const void*)plan.scratch, plan.scratch_cursor, pc.bucket_cap, plan, L,
                         cursor, (void*)out, stats);
      HIP_CHECK(hipGetLastError());
      return;
    }
    if (nb > kCMaxNb) {
      if (plan.key32)
        throw std::invalid_argument("partition: int32 keys need <= 512 buckets");
      partition_variant(keys, ts, vals, jhash_tab, n, plan, kg_dest, cursor, out, stats,
                        late_idx, late_cap, stream, 1);
      return;
    }
    dispatch_compact<true, 8>(keys, ts, vals, jhash_tab, n, plan, kg_dest, cursor, out, stats,
                              late_idx, late_cap, stream);
    return;
  }
  if (plan.rec_words == 2 && nb > kCMaxNb && plan.scratch && plan.scratch_cursor &&
      nb <= kCMaxNb * 32 && (uint64_t)nb * plan.bucket_cap < (1ull << 32)) {
    // Two-level 16-byte partition (session records, more than 512 buckets): the compact staged
    // kernel into 512 coarse buckets (one LDS counting sort per 4096-record round, contiguous
    // run writes), then one workgroup per coarse bucket splits it into its 2^L fine buckets.
    if (n <= 0) return;
    int L = 0;
    while ((nb >> L) > kCMaxNb) ++L;
    PartPlan pc = plan;
    pc.nsub_log2 = plan.nsub_log2 - L;
    pc.bucket_cap = plan.bucket_cap << L;
    if (pc.nsub_log2 < 0) throw std::invalid_argument("two-level partition: too few sub-tables");
    hipStream_t st = (hipStream_t)stream;
    HIP_CHECK(hipMemsetAsync(plan.scratch_cursor, 0, sizeof(uint32_t) * (nb >> L), st));
    if (plan.nranks == 1)
      dispatch_compact<true, 16>(keys, ts, vals, jhash_tab, n, pc, kg_dest, plan.scratch_cursor,
                                 (Rec*)plan.scratch, stats, late_idx, late_cap, stream);
    else
      dispatch_compact<false, 16>(keys, ts, vals, jhash_tab, n, pc, kg_dest, plan.scratch_cursor,
                                  (Rec*)plan.scratch, stats, late_idx, late_cap, stream);
    hipLaunchKernelGGL(partition_split_kernel<16>, dim3(nb >> L), dim3(kSplitThreads), 0, st,
                       (const void*)plan.scratch, plan.scratch_cursor, pc.bucket_cap, plan, L,
                       cursor, (void*)out, stats);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (plan.rec_words == 2 && nb <= kCMaxNb && (uint64_t)nb * plan.bucket_cap < (1ull << 32)) {
    if (n <= 0) return;
    if (plan.nranks == 1)
      dispatch_compact<true, 16>(keys, ts, vals, jhash_tab, n, plan, kg_dest, cursor, out, stats,
                                 late_idx, late_cap, stream);
    else
      dispatch_compact<false, 16>(keys, ts, vals, jhash_tab, n, plan, kg_dest, cursor, out, stats,
                                  late_idx, late_cap, stream);
    return;
  }
  if (plan.key32)
    throw std::invalid_argument("partition: int32 keys need compact records (<= 512 buckets)");
  if (plan.rec_words == 3 && nb > kStageMaxNb && plan.scratch && plan.scratch_cursor &&
      nb <= kStageMaxNb * 32 && (uint64_t)nb * plan.bucket_cap < (1ull << 32)) {
    // Two-level 24-byte partition (session / generic records): the write-combined staged
    // kernel into 512 coarse buckets, then the split kernel into the fine buckets.
    if (n <= 0) return;
    int L = 0;
    while ((nb >> L) > kStageMaxNb) ++L;
    PartPlan pc = plan;
    pc.nsub_log2 = plan.nsub_log2 - L;
    pc.bucket_cap = plan.bucket_cap << L;
    if (pc.nsub_log2 < 0) throw std::invalid_argument("two-level partition: too few sub-tables");
    hipStream_t st = (hipStream_t)stream;
    HIP_CHECK(hipMemsetAsync(plan.scratch_cursor, 0, sizeof(uint32_t) * (nb >> L), st));
    partition_variant(keys, ts, vals, jhash_tab, n, pc, kg_dest, plan.scratch_cursor,
                      (Rec*)plan.scratch, stats, late_idx, late_cap, stream, 5);
    hipLaunchKernelGGL(partition_split_kernel<24>, dim3(nb >> L), dim3(kSplitThreads), 0, st,
                       (const void*)plan.scratch, plan.scratch_cursor, pc.bucket_cap, plan, L,
                       cursor, (void*)out, stats);
    HIP_CHECK(hipGetLastError());
    return;
  }
  // Write-combined staged scatter when the LDS carry buffers fit (<= 512 buckets); otherwise
  // the plain scatter. Both stream their inputs with non-temporal loads (kbench A/B).
  partition_variant(keys, ts, vals, jhash_tab, n, plan, kg_dest, cursor, out, stats, late_idx,
                    late_cap, stream, nb <= kStageMaxNb ? 5 : 1);
}

void partition_variant(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
                       const int32_t* jhash_tab, int64_t n, const PartPlan& plan,
                       const int32_t* kg_dest, uint32_t* cursor, Rec* out, int64_t* stats,
                       uint32_t* late_idx, uint32_t late_cap, intptr_t stream, int variant) {
  if (n <= 0) return;
  const int nb = plan.nranks << plan.nsub_log2;
  if (nb > 16384) throw std::runtime_error("partition: too many buckets (max 16384)");
  // 64K events per 1024-thread workgroup: one workgroup per CU at 16M events, bucket runs of
  // >= 32 records, and nb global reservations per workgroup instead of per 8K events.
  int blocks = grid_for(n, 65536, 1024);
  const int64_t chunk = (n + blocks - 1) / blocks;
  const size_t lds = (size_t)((nb + 3) & ~3) * 4 + 16 * 8;
  hipStream_t st = (hipStream_t)stream;
#define MXS_PART(VV)                                                                          \
  case VV: {                                                                                  \
    static bool attr = false;                                                                 \
    if (!attr) {                                                                              \
      HIP_CHECK(hipFuncSetAttribute((const void*)partition_kernel<VV>,                         \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));   \
      attr = true;                                                                            \
    }                                                                                         \
    hipLaunchKernelGGL(partition_kernel<VV>, dim3(blocks), dim3(1024), lds, st, keys, ts, vals, \
                       jhash_tab, n, chunk, plan, kg_dest, cursor, out, stats, late_idx,       \
                       late_cap);                                                              \
    break;                                                                                    \
  }
#define MXS_PART_STAGED(VV, TV)                                                               \
  case VV: {                                                                                  \
    if (nb > kStageMaxNb) throw std::runtime_error("staged partition needs <= 512 buckets");  \
    static bool attr = false;                                                                 \
    if (!attr) {                                                                              \
      HIP_CHECK(hipFuncSetAttribute((const void*)partition_staged_kernel<TV>,                  \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStagedLds)); \
      attr = true;                                                                            \
    }                                                                                         \
    hipLaunchKernelGGL(partition_staged_kernel<TV>, dim3(blocks), dim3(1024), kStagedLds, st,   \
                       keys, ts, vals, jhash_tab, n, chunk, plan, kg_dest, cursor, out, stats, \
                       late_idx, late_cap);                                                    \
    break;                                                                                    \
  }
#define MXS_PART_COMPACT(VV, CUV, EPB)                                                         \
  case VV: {                                                                                  \
    if (plan.rec_words != 2 || nb > kCMaxNb) throw std::runtime_error("compact variant: plan"); \
    static bool attr = false;                                                                 \
    if (!attr) {                                                                              \
      HIP_CHECK(hipFuncSetAttribute((const void*)partition_compact_kernel<1, CUV>,             \
                                    hipFuncAttributeMaxDynamicSharedMemorySize,                \
                                    (int)compact_lds(CUV)));                                   \
      attr = true;                                                                            \
    }                                                                                         \
    const int cb = grid_for(n, EPB, 2048);                                                    \
    const int64_t cchunk = (n + cb - 1) / cb;                                                 \
    hipLaunchKernelGGL((partition_compact_kernel<1, CUV>), dim3(cb), dim3(1024),               \
                       compact_lds(CUV), st, keys, ts, vals, jhash_tab, n, cchunk, plan,       \
                       kg_dest, cursor, reinterpret_cast<RecC*>(out), stats, late_idx,         \
                       late_cap);                                                              \
    break;                                                                                    \
  }
  switch (variant) {
    MXS_PART(0) MXS_PART(1) MXS_PART(2) MXS_PART(3)
    MXS_PART_STAGED(4, 0) MXS_PART_STAGED(5, 1)
    MXS_PART_COMPACT(10, 2, 32768) MXS_PART_COMPACT(11, 3, 32768) MXS_PART_COMPACT(12, 4, 32768)
    MXS_PART_COMPACT(13, 3, 49152) MXS_PART_COMPACT(14, 4, 65536)
    MXS_PART_COMPACT(15, 2, 65536) MXS_PART_COMPACT(16, 3, 65536)
    MXS_PART_COMPACT(17, 4, 131072)
    default: throw std::runtime_error("partition: unknown variant");
  }
#undef MXS_PART
#undef MXS_PART_STAGED
#undef MXS_PART_COMPACT
  HIP_CHECK(hipGetLastError());
}

// Packed (sum, count) accumulators apply: integer sum/avg over 16-byte records, raw events
// (not combiner output) and fewer than 2^16 records per sub-table and step. MXS_AGG_PACK=0
// turns them off (A/B switch).
static bool agg_pack_ok(const AggPlan& p) {
  static const bool enabled = [] {
    const char* e = std::getenv("MXS_AGG_PACK");
    return !(e && e[0] == '0');
  }();
  // records one workgroup folds: a forced split (AggPlan.split < 0, dense ids, one source, no
  // touched-slot list: the launcher's split condition) gives each a 1/-split share
  uint64_t per_wg = (uint64_t)p.nsrc * p.bucket_cap;
  if (p.split < -1 && p.dense_bits && p.nsrc == 1 && !p.dlist)
    per_wg = (p.bucket_cap + (uint64_t)(-p.split) - 1) / (uint64_t)(-p.split);
  return enabled && (p.agg == AGG_SUM_I64 || p.agg == AGG_AVG_I64) && p.rec_words <= 2 &&
         !p.combined && per_wg < 65536;
}

template <int AGG, int RW, bool PK, bool DENSE, bool DET = false, int V = 0>
static void launch_agg_v(const Rec* recs, const uint32_t* counts, const AggPlan& p,
                         uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                         uint32_t* occ, uint32_t* flags, size_t lds, hipStream_t s) {
  // dynamic LDS + the kernel's static sparse-pane table (srel, 128 B) stay <= 160 KiB
  constexpr size_t kAggDynMax = 160 * 1024 - 512;
  if (lds > kAggDynMax) throw std::runtime_error("window_agg: LDS image exceeds 160 KiB");
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)window_agg_kernel<AGG, RW, PK, DENSE, DET, V>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kAggDynMax));
    attr = true;
  }
  // Split only what the kernel's atomic merge supports: dense ids (no LDS key table to share),
  // one source segment, additive integer aggregates, no touched-slot list.
  AggPlan q = p;
  const bool split_ok = DENSE && p.nsrc == 1 && !p.dlist &&
                        (AGG == AGG_SUM_I64 || AGG == AGG_AVG_I64 || AGG == AGG_COUNT);
  q.split = split_ok && (p.split > 1 || p.split < -1) ? p.split : 1;
  const int nsplit = q.split < 0 ? -q.split : q.split;
  hipLaunchKernelGGL((window_agg_kernel<AGG, RW, PK, DENSE, DET, V>), dim3(p.nsub * nsplit), dim3(1024),
                     lds, s, (const void*)recs, counts, q, keys_g, acc_g, cnt_g, dirty_g, occ,
                     flags);
}

template <int AGG, bool DENSE>
static void launch_agg_d(const Rec* recs, const uint32_t* counts, const AggPlan& p,
                         uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                         uint32_t* occ, uint32_t* flags, hipStream_t s) {
  const size_t cap = (size_t)1 << p.cap_log2;
  const size_t keys_lds = DENSE ? 0 : cap * 8;  // dense ids need no LDS key table
  const size_t list_lds = p.dlist ? 16 + cap / 8 + cap * 4 : 0;
  if constexpr (AGG == AGG_SUM_F64 || AGG == AGG_AVG_F64) {
    if (p.det) {  // deterministic sums: 16-byte fixed-point accumulators, 24-byte records
      if (p.rec_words != 3) throw std::invalid_argument("window_agg: deterministic sums need 24-byte records");
      const size_t lds_det = keys_lds + (size_t)p.pg * cap * 20 + 16 + list_lds;
      launch_agg_v<AGG, 3, false, DENSE, true>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g,
                                               occ, flags, lds_det, s);
      return;
    }
  }
  if constexpr (AGG == AGG_SUM_I64 || AGG == AGG_AVG_I64) {
    if (agg_pack_ok(p)) {
      const size_t lds_pk = keys_lds + (size_t)p.pg * cap * 8 + 16 + list_lds;
      // Default: the 64-VGPR build (V = 2) when two workgroups' LDS images fit a CU -- that is
      // what its register cap buys (hashed 1M-key step 135 -> 119 us); otherwise the default
      // build (its larger write-back batches). MXS_AGG_V forces a variant (A/B).
      static const int v_env = [] {
        const char* e = std::getenv("MXS_AGG_V");
        return e ? std::atoi(e) & 3 : -1;
      }();
      const int v = v_env >= 0 ? v_env : (2 * (lds_pk + 512) <= 160 * 1024 ? 2 : 0);
      if (p.rec_words == 1) {
        switch (v) {
          case 1: launch_agg_v<AGG, 1, true, DENSE, false, 1>(recs, counts, p, keys_g, acc_g, cnt_g,
                                                              dirty_g, occ, flags, lds_pk, s); break;
          case 2: launch_agg_v<AGG, 1, true, DENSE, false, 2>(recs, counts, p, keys_g, acc_g, cnt_g,
                                                              dirty_g, occ, flags, lds_pk, s); break;
          case 3: launch_agg_v<AGG, 1, true, DENSE, false, 3>(recs, counts, p, keys_g, acc_g, cnt_g,
                                                              dirty_g, occ, flags, lds_pk, s); break;
          default: launch_agg_v<AGG, 1, true, DENSE>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g,
                                                     occ, flags, lds_pk, s);
        }
      } else
        launch_agg_v<AGG, 2, true, DENSE>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g, occ,
                                          flags, lds_pk, s);
      return;
    }
  }
  const size_t lds = keys_lds + (size_t)p.pg * cap * 12 + 16 + list_lds;
  if (p.rec_words == 1)
    launch_agg_v<AGG, 1, false, DENSE>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g, occ, flags,
                                       lds, s);
  else if (p.rec_words == 2)
    launch_agg_v<AGG, 2, false, DENSE>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g, occ, flags,
                                       lds, s);
  else
    launch_agg_v<AGG, 3, false, DENSE>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g, occ, flags,
                                       lds, s);
}

template <int AGG>
static void launch_agg(const Rec* recs, const uint32_t* counts, const AggPlan& p,
                       uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                       uint32_t* occ, uint32_t* flags, size_t, hipStream_t s) {
  if (p.dense_bits)
    launch_agg_d<AGG, true>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g, occ, flags, s);
  else
    launch_agg_d<AGG, false>(recs, counts, p, keys_g, acc_g, cnt_g, dirty_g, occ, flags, s);
}

void window_agg(const Rec* recs, const uint32_t* counts, const AggPlan& plan, uint64_t* keys_g,
                uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g, uint32_t* occupancy,
                uint32_t* flags, intptr_t stream) {
  if (plan.np_step <= 0 || plan.nsub <= 0) return;
  const size_t cap = (size_t)1 << plan.cap_log2;
  // (conservative LDS size; launch_agg_d sizes each variant exactly and checks the limit)
  const size_t lds = cap * 8 + (size_t)plan.pg * cap * (plan.det ? 20 : 12) + 16 +
                     (plan.dlist ? 16 + cap / 8 + cap * 4 : 0);  // touched-slot bitmap + buffer
  if (plan.rec_words < 3 && plan.combined)
    throw std::invalid_argument("window_agg: combined records are 24-byte records");
  hipStream_t s = (hipStream_t)stream;
  switch (plan.agg) {
#define MXS_A(A) case A: launch_agg<A>(recs, counts, plan, keys_g, acc_g, cnt_g, dirty_g, occupancy, flags, lds, s); break;
    MXS_A(AGG_SUM_I64) MXS_A(AGG_SUM_F64) MXS_A(AGG_MIN_I64) MXS_A(AGG_MAX_I64)
    MXS_A(AGG_MIN_F64) MXS_A(AGG_MAX_F64) MXS_A(AGG_COUNT) MXS_A(AGG_AVG_F64) MXS_A(AGG_AVG_I64)
#undef MXS_A
    default: throw std::runtime_error("window_agg: unknown aggregate");
  }
  HIP_CHECK(hipGetLastError());
}

// Tiered firing: combine rows per key into a global open-addressing table with atomics (see
// mxs_kernels.h tier_merge). One row per lane; the probe is linear from the key's hash.
__device__ __forceinline__ void tier_atomic_combine(int agg, uint64_t* p, uint64_t v) {
  switch (agg) {
    case AGG_SUM_I64:
    case AGG_AVG_I64:
    case AGG_COUNT:
      atomicAdd((unsigned long long*)p, (unsigned long long)v);
      return;
    case AGG_SUM_F64:
    case AGG_AVG_F64:
      atomicAdd((double*)p, as_f64(v));
      return;
    case AGG_MIN_I64:
      atomicMin((long long*)p, (long long)v);
      return;
    case AGG_MAX_I64:
      atomicMax((long long*)p, (long long)v);
      return;
    default: {  // f64 min / max: compare-and-swap on the bit pattern
      uint64_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (true) {
        const uint64_t nv = agg_combine(agg, old, v);
        if (nv == old) return;
        const uint64_t prev = atomicCAS((unsigned long long*)p, (unsigned long long)old,
                                        (unsigned long long)nv);
        if (prev == old) return;
        old = prev;
      }
    }
  }
}

__global__ __launch_bounds__(256) void tier_merge_kernel(
    const uint64_t* __restrict__ keys, const uint64_t* __restrict__ acc,
    const uint32_t* __restrict__ cnt, int64_t n, const uint32_t* __restrict__ n_dev, int mode,
    int agg, uint64_t* __restrict__ tkeys, uint64_t* __restrict__ tacc,
    uint32_t* __restrict__ tcnt, uint8_t* __restrict__ tdirty, uint32_t mask,
    uint32_t* __restrict__ flags) {
  if (n_dev) {
    const int64_t d = (int64_t)*n_dev;
    n = d < n ? d : n;
  }
  const bool find_only = (mode & 2) != 0, mark = (mode & 1) != 0;
  bool full = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t k = keys[i];
    const uint32_t c = cnt[i];
    if (k >= kTombKey || c == 0) continue;
    uint32_t s = (uint32_t)(mix64(k) >> 20) & mask;
    uint32_t found = kNoSlot;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
      const uint64_t cur = __hip_atomic_load(&tkeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == k) {
        found = s;
        break;
      }
      if (cur == kEmptyKey) {
        if (find_only) break;
        const uint64_t prev = atomicCAS((unsigned long long*)&tkeys[s],
                                        (unsigned long long)kEmptyKey, (unsigned long long)k);
        if (prev == kEmptyKey || prev == k) {
          found = s;
          break;
        }
      }
      s = (s + 1) & mask;
    }
    if (found == kNoSlot) {
      full = full || !find_only;
      continue;
    }
    tier_atomic_combine(agg, &tacc[found], acc[i]);
    atomicAdd(&tcnt[found], c);
    if (mark) tdirty[found] = 1;
  }
  if (full) atomicOr(&flags[0], 1u);
}

void window_fire(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                 const uint8_t* dirty_g, const FirePlan& plan, uint64_t* out_keys,
                 double* out_vals, uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n,
                 intptr_t stream) {
  if (plan.nslots <= 0) return;
  const int depth = plan.map.depth > plan.filt.depth ? plan.map.depth : plan.filt.depth;
  const size_t lds = (size_t)(kExprVars + depth) * kFireThreads * sizeof(double) + 17 * 4;
  if (lds > 160 * 1024) throw std::runtime_error("window_fire: epilogue stack too deep for LDS");
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)window_fire_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(window_fire_kernel, dim3(grid_for(plan.nslots, kFireThreads * kFireU, 1024)),
                     dim3(kFireThreads), lds,
                     (hipStream_t)stream, keys_g, acc_g, cnt_g, dirty_g, plan, out_keys, out_vals,
                     out_raw, out_cnt, out_n);
  HIP_CHECK(hipGetLastError());
}

void window_fire_many(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                      const uint8_t* dirty_g, const FirePlan& base, const FireWin* wins, int k,
                      const FireStage& st, uint64_t* out_keys, double* out_vals, uint64_t* out_raw,
                      uint32_t* out_cnt, uint32_t* out_n, uint32_t* bounds, intptr_t stream) {
  if (k <= 0 || base.nslots <= 0) return;
  if (st.region < (uint32_t)base.nslots)
    throw std::invalid_argument("window_fire_many: staging region smaller than the table");
  const int depth = base.map.depth > base.filt.depth ? base.map.depth : base.filt.depth;
  const size_t lds = (size_t)(kExprVars + depth) * kFireMultiThreads * sizeof(double) + 8 * 4;
  hipStream_t s = (hipStream_t)stream;
  HIP_CHECK(hipMemsetAsync(st.win_n, 0, sizeof(uint32_t) * k, s));
  const int64_t nvisit = base.nslots;
  const bool big = nvisit >= 65536;
  const int gx = grid_for(nvisit, kFireMultiThreads * (big ? 4 : 1), big ? 256 : 1024);
  for (int w0 = 0; w0 < k; w0 += kFireMultiMax) {
    FireWinPack pack{};
    pack.n = k - w0 < kFireMultiMax ? k - w0 : kFireMultiMax;
    for (int i = 0; i < pack.n; ++i) pack.w[i] = wins[w0 + i];
    if (big)
      hipLaunchKernelGGL(window_fire_multi_kernel<4>, dim3(gx, pack.n), dim3(kFireMultiThreads),
                         lds, s, keys_g, acc_g, cnt_g, dirty_g, base, pack, w0, st);
    else
      hipLaunchKernelGGL(window_fire_multi_kernel<1>, dim3(gx, pack.n), dim3(kFireMultiThreads),
                         lds, s, keys_g, acc_g, cnt_g, dirty_g, base, pack, w0, st);
    HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(fire_pack_kernel, dim3(grid_for(nvisit, 256 * 4, 64), k), dim3(256), 0, s,
                     st, k, base.key32, out_keys, out_vals, out_raw, out_cnt, bounds, out_n,
                     nullptr);
  HIP_CHECK(hipGetLastError());
}

bool window_refire_many(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                        const uint8_t* dirty_g, const FirePlan& base, const FireWin* wins, int k,
                        const FireStage& st, uint64_t* out_keys, double* out_vals,
                        uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n, uint32_t* bounds,
                        uint32_t* ovf, intptr_t stream, int64_t dlo, uint32_t dmask_abs) {
  if (k <= 0 || k > kFireMultiMax || !base.list || !base.list_n || base.nslots <= 0) return false;
  int64_t u0 = wins[0].p0, u1 = wins[0].p0 + wins[0].npanes;
  for (int i = 1; i < k; ++i) {
    u0 = wins[i].p0 < u0 ? wins[i].p0 : u0;
    u1 = wins[i].p0 + wins[i].npanes > u1 ? wins[i].p0 + wins[i].npanes : u1;
  }
  if (u1 - u0 > kRefireP || u1 - u0 > base.ring) return false;
  // Panes that may hold dirty bytes (late data of this step), union-relative; 0 = unknown: all.
  uint32_t dmask = 0;
  for (int64_t q = 0; q < u1 - u0; ++q) {
    const int64_t b = u0 + q - dlo;
    if (!dmask_abs || (b >= 0 && b < 31 && (dmask_abs >> b & 1u))) dmask |= 1u << q;
  }
  const int depth = base.map.depth > base.filt.depth ? base.map.depth : base.filt.depth;
  const size_t lds = (size_t)(kExprVars + depth) * kRefireThreads * sizeof(double) + 8 * 4;
  hipStream_t s = (hipStream_t)stream;
  HIP_CHECK(hipMemsetAsync(st.win_n, 0, sizeof(uint32_t) * k, s));
  FireWinPack pack{};
  pack.n = k;
  for (int i = 0; i < k; ++i) pack.w[i] = wins[i];
  // The list length stays on the device: a grid for the list's capacity (nslots), rounds of
  // 256 slots per workgroup; workgroups past the list end exit at once.
  hipLaunchKernelGGL(window_refire_multi_kernel, dim3(grid_for(base.nslots, kRefireThreads * 4, 2048)),
                     dim3(kRefireThreads), lds, s, keys_g, acc_g, cnt_g,
                     const_cast<uint8_t*>(dirty_g), base, pack, u0,
                     (int)(u1 - u0), dmask, st);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(fire_pack_kernel, dim3(grid_for(base.nslots / k, 256 * 4, 64), k), dim3(256),
                     0, s, st, k, base.key32, out_keys, out_vals, out_raw, out_cnt, bounds, out_n,
                     ovf);
  HIP_CHECK(hipGetLastError());
  return true;
}

void direct_agg_probe(const uint64_t* keys, const int64_t* ts, const uint64_t* vals, int64_t n,
                      int64_t tbase, int64_t pane, int ring, int64_t nslots, uint32_t mul,
                      int bits, int64_t pane_base, uint64_t* acc_g, uint32_t* cnt_g, int mode,
                      uint64_t* sink, int grid, intptr_t stream) {
  hipLaunchKernelGGL(direct_agg_probe_kernel, dim3(grid > 0 ? grid : grid_for(n, 256 * 4, 16384)),
                     dim3(256), 0, (hipStream_t)stream, keys, ts, vals, n, tbase, pane, ring,
                     nslots, mul, bits, pane_base, acc_g, cnt_g, mode, sink);
  HIP_CHECK(hipGetLastError());
}

void window_compact(uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                    int nsub, int cap_log2, int ring, int64_t p_lo, int np, int64_t cutoff,
                    const CompactOut& out, uint32_t* occupancy, intptr_t stream) {
  if (nsub <= 0) return;
  if (cap_log2 > 12 || np > ring || np < 0)
    throw std::invalid_argument("window_compact: sub-table > 4096 slots or bad pane range");
  const size_t cap = (size_t)1 << cap_log2;
  const size_t lds = cap * (8 * 3 + 4 * 2 + 1) + 32;
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)window_compact_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int64_t nslots = (int64_t)nsub << cap_log2;
  hipLaunchKernelGGL(window_compact_kernel, dim3(nsub), dim3(1024), lds, (hipStream_t)stream,
                     keys_g, acc_g, cnt_g, dirty_g, cap_log2, ring, nslots, p_lo, np, cutoff, out,
                     occupancy);
  HIP_CHECK(hipGetLastError());
}

void window_rows_pane_sort(const uint64_t* key, const int64_t* pane, const uint64_t* acc,
                           const uint32_t* cnt, const uint8_t* dirty, const uint32_t* n_dev,
                           uint32_t cap, int64_t p_lo, int np, uint64_t* okey, uint64_t* oacc,
                           uint32_t* ocnt, uint8_t* odirty, uint32_t* counts, intptr_t stream) {
  if (np <= 0 || np > kPaneSortMax)
    throw std::invalid_argument("window_rows_pane_sort: 1..64 panes");
  hipStream_t s = (hipStream_t)stream;
  // counts[0, 64): rows per pane (read by the host with the rows), [64, 128): scatter cursors
  HIP_CHECK(hipMemsetAsync(counts, 0, 2 * kPaneSortMax * sizeof(uint32_t), s));
  if (cap == 0) return;
  const uint32_t want = (cap + 256 * 8 - 1) / (256 * 8);
  const uint32_t blocks = want < 2048 ? (want ? want : 1) : 2048;
  hipLaunchKernelGGL(pane_sort_hist_kernel, dim3(blocks), dim3(256), 0, s, pane, n_dev, cap, p_lo,
                     np, counts);
  hipLaunchKernelGGL(pane_sort_scatter_kernel, dim3(blocks), dim3(256), 0, s, key, pane, acc, cnt,
                     dirty, n_dev, cap, p_lo, np, counts, counts + kPaneSortMax, okey, oacc, ocnt,
                     odirty);
  HIP_CHECK(hipGetLastError());
}

void dirty_clear(const uint32_t* list, const uint32_t* list_n, uint32_t list_cap, int ring,
                 int64_t nslots, uint8_t* dirty_g, uint32_t* slot_mark, int64_t p_lo, int np,
                 intptr_t stream, uint64_t* dacc, uint32_t* dcnt) {
  if (list_cap == 0) return;
  np = np < ring ? np : ring;
  hipLaunchKernelGGL(dirty_clear_kernel, dim3(grid_for(list_cap, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, list, list_n, list_cap, ring, nslots, dirty_g, slot_mark,
                     p_lo, np, dacc, dcnt);
  HIP_CHECK(hipGetLastError());
}

void scatter_partials(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt,
                      const uint32_t* n_in, const ScatPlan& plan, const int32_t* jhash,
                      const int32_t* kg_dest, uint32_t* cursor, Rec* out, uint32_t* flags,
                      intptr_t stream) {
  if (plan.n_cap == 0) return;
  const int nb = plan.nranks << plan.nsub_log2;
  if (nb > 16384) throw std::invalid_argument("scatter_partials: more than 16384 buckets");
  const size_t lds = (size_t)nb * 2 * sizeof(uint32_t);
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)scatter_partials_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int64_t per = (int64_t)kScatThreads * kScatU;
  const int grid = (int)((plan.n_cap + per - 1) / per);
  hipLaunchKernelGGL(scatter_partials_kernel, dim3(grid), dim3(kScatThreads), lds,
                     (hipStream_t)stream, keys, acc, cnt, n_in, plan, jhash, kg_dest, cursor, out,
                     flags);
  HIP_CHECK(hipGetLastError());
}

void expr_filter(const double* x, int64_t n, const ExprProg& prog, uint8_t* keep,
                 intptr_t stream) {
  if (n <= 0) return;
  const size_t lds = (size_t)(kExprVars + prog.depth) * 256 * sizeof(double);
  hipLaunchKernelGGL(expr_filter_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), lds,
                     (hipStream_t)stream, x, n, prog, keep);
  HIP_CHECK(hipGetLastError());
}

void line_starts(const uint8_t* buf, int64_t n, void* scratch, int64_t* idx, int64_t* total,
                 intptr_t stream, int64_t cap) {
  if (n <= 0) {
    HIP_CHECK(hipMemsetAsync(total, 0, 8, (hipStream_t)stream));
    return;
  }
  const int64_t nt = (n + kFcTile - 1) / kFcTile;
  uint64_t* masks = (uint64_t*)scratch;
  int64_t* offs = (int64_t*)(masks + nt * kFcWords);
  uint32_t* counts = (uint32_t*)(offs + nt);
  hipLaunchKernelGGL(line_start_mask_kernel, dim3((uint32_t)nt), dim3(256), 0,
                     (hipStream_t)stream, buf, n, masks, counts);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(filter_scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, counts, nt,
                     offs, total);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(filter_write_kernel, dim3((uint32_t)nt), dim3(256), 0, (hipStream_t)stream,
                     masks, offs, n, idx, cap);
  HIP_CHECK(hipGetLastError());
}

void compact_from_masks(const uint64_t* masks, const uint32_t* counts, int64_t nt, int64_t n,
                        int64_t* offs, int64_t* idx, int64_t* total, intptr_t stream) {
  hipLaunchKernelGGL(filter_scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, counts, nt,
                     offs, total);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(filter_write_kernel, dim3((uint32_t)nt), dim3(256), 0, (hipStream_t)stream,
                     masks, offs, n, idx, INT64_MAX);
  HIP_CHECK(hipGetLastError());
}

int64_t filter_compact_scratch_bytes(int64_t n) {
  const int64_t nt = (n + kFcTile - 1) / kFcTile;
  return nt * (kFcWords * 8 + 4 + 8);
}

void expr_filter_compact(const double* x, int64_t n, const ExprProg& prog, void* scratch,
                         int64_t* idx, int64_t* total, intptr_t stream) {
  if (n <= 0) {
    HIP_CHECK(hipMemsetAsync(total, 0, 8, (hipStream_t)stream));
    return;
  }
  const int64_t nt = (n + kFcTile - 1) / kFcTile;
  uint64_t* masks = (uint64_t*)scratch;
  int64_t* offs = (int64_t*)(masks + nt * kFcWords);
  uint32_t* counts = (uint32_t*)(offs + nt);
  const size_t lds = (size_t)(kExprVars + prog.depth) * 256 * sizeof(double);
  hipLaunchKernelGGL(filter_mask_kernel, dim3((uint32_t)nt), dim3(256), lds, (hipStream_t)stream,
                     x, n, prog, masks, counts);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(filter_scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, counts, nt,
                     offs, total);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(filter_write_kernel, dim3((uint32_t)nt), dim3(256), 0, (hipStream_t)stream,
                     masks, offs, n, idx, INT64_MAX);
  HIP_CHECK(hipGetLastError());
}

void rolling(const Rec*, const uint32_t*, const RollPlan&, uint64_t*, uint64_t*, uint32_t*,
             uint32_t*, uint32_t*, uint64_t*, intptr_t) {
  throw std::runtime_error("gpu::rolling: use rolling_lookup / rolling_heads / rolling_scan");
}

static void check_roll_layout(int abits, int shift) {
  if (abits < 1 || abits > 32 || shift < abits || shift > 40)
    throw std::invalid_argument("rolling sort-key layout out of range");
}

void rolling_lookup(const Rec* recs, const uint32_t* counts, int nsrc, int nsub,
                    uint32_t bucket_cap, int cap_log2, uint64_t* keys_g, int64_t* sort_key,
                    uint64_t* vals_out, uint32_t* n_out, uint32_t* flags, int abits, int shift,
                    intptr_t stream) {
  if (nsrc * nsub <= 0) return;
  check_roll_layout(abits, shift);
  const uint32_t chunks = (bucket_cap + kLookupChunk - 1) / kLookupChunk;
  hipLaunchKernelGGL(rolling_lookup_kernel, dim3(chunks, nsrc * nsub), dim3(256), 0,
                     (hipStream_t)stream,
                     recs, counts, nsrc, nsub, bucket_cap, cap_log2, keys_g, sort_key, vals_out,
                     n_out, flags, abits, shift);
  HIP_CHECK(hipGetLastError());
}

void rolling_lookup_direct(const uint64_t* keys, const uint64_t* vals, uint32_t n, int nsub_log2,
                           int cap_log2, uint64_t* keys_g, int64_t* sort_key, uint64_t* vals_out,
                           uint32_t* n_out, uint32_t* flags, int shift, intptr_t stream) {
  check_roll_layout(shift, shift);
  if ((uint64_t)n > (1ull << shift))
    throw std::invalid_argument("rolling_lookup_direct: arrival index does not fit the shift");
  hipLaunchKernelGGL(rolling_lookup_direct_kernel, dim3(grid_for(n > 0 ? (n + 3) / 4 : 1, 256, 8192)),
                     dim3(256), 0, (hipStream_t)stream, keys, vals, n, nsub_log2, cap_log2, keys_g,
                     sort_key, vals_out, n_out, flags, shift);
  HIP_CHECK(hipGetLastError());
}

void rolling_heads(const int64_t* sk, const uint32_t* n_in, int64_t n_cap, uint32_t* heads,
                   uint32_t* n_heads, int shift, intptr_t stream) {
  hipLaunchKernelGGL(seg_heads_kernel, dim3(grid_for((n_cap + 63) / 64, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, sk, n_in, heads, n_heads, shift);
  HIP_CHECK(hipGetLastError());
}

template <int AGG>
static void launch_roll(const int64_t* sk, const int64_t* perm, const uint64_t* vals,
                        const uint32_t* n_in, const uint32_t* heads, const uint32_t* n_heads,
                        uint64_t* acc_g, uint32_t* cnt_g, const uint64_t* keys_g,
                        const ExprProg& filt, uint64_t* ok, uint64_t* ov, int64_t* ot,
                        uint32_t* on, uint32_t cap, int grid, size_t lds, int abits, int shift,
                        uint32_t count_n, hipStream_t s) {
  hipLaunchKernelGGL(rolling_scan_kernel<AGG>, dim3(grid), dim3(256), lds, s, sk, perm, vals, n_in,
                     heads, n_heads, acc_g, cnt_g, keys_g, filt, ok, ov, ot, on, cap, abits, shift,
                     count_n);
}

void rolling_scan(int agg, const int64_t* sk, const int64_t* perm, const uint64_t* vals,
                  const uint32_t* n_in, const uint32_t* heads, const uint32_t* n_heads,
                  int64_t max_segments, uint64_t* acc_g, uint32_t* cnt_g, const uint64_t* keys_g,
                  const ExprProg& filt, uint64_t* out_key, uint64_t* out_val, int64_t* out_tag,
                  uint32_t* out_n, uint32_t out_cap, int abits, int shift, intptr_t stream,
                  uint32_t count_n) {
  check_roll_layout(abits, shift);
  const int grid = grid_for(max_segments * 64, 256, 4096);
  const size_t lds = (size_t)(kExprVars + filt.depth) * 256 * sizeof(double);
  hipStream_t s = (hipStream_t)stream;
  switch (agg) {
#define MXS_R(A) case A: launch_roll<A>(sk, perm, vals, n_in, heads, n_heads, acc_g, cnt_g, keys_g, filt, out_key, out_val, out_tag, out_n, out_cap, grid, lds, abits, shift, count_n, s); break;
    MXS_R(AGG_SUM_I64) MXS_R(AGG_SUM_F64) MXS_R(AGG_MIN_I64) MXS_R(AGG_MAX_I64)
    MXS_R(AGG_MIN_F64) MXS_R(AGG_MAX_F64) MXS_R(AGG_COUNT)
    MXS_R(AGG_AVG_I64) MXS_R(AGG_AVG_F64)
#undef MXS_R
    default: throw std::runtime_error("rolling_scan: unsupported aggregate");
  }
  HIP_CHECK(hipGetLastError());
}


static SessArgs make_sess_args(int64_t gap, int64_t lateness, int64_t wm, int64_t tbase, int agg,
                               int cap_log2, int64_t nslots, int tbits = 32, int st = 1) {
  SessArgs a;
  a.st = st;
  a.tbits = tbits;
  a.gap = gap;
  a.lateness = lateness;
  a.wm = wm;
  a.tbase = tbase;
  a.agg = agg;
  a.cap_log2 = cap_log2;
  a.nslots = nslots;
  return a;
}

void session_lookup(const void* recs, const uint32_t* counts, int nsrc, int nsub, uint32_t bcap,
                    int cap_log2, uint64_t* keys_g, uint64_t* spill_set, uint32_t spill_mask,
                    int spill_any, int64_t* sk, uint64_t* vals, uint32_t* n_out, Rec* host_recs,
                    uint32_t* n_host, uint32_t host_cap, uint32_t* n_inserted, int tbits,
                    intptr_t stream, int rec_words) {
  if (nsrc * nsub <= 0) return;
  if (tbits < 1 || tbits > 32) throw std::invalid_argument("session_lookup: tbits out of range");
  if (rec_words != 2 && rec_words != 3)
    throw std::invalid_argument("session_lookup: 16- or 24-byte records");
  if (cap_log2 <= kSessLookupLdsMaxLog2) {
    const size_t lds = (size_t)sizeof(uint64_t) << cap_log2;
    hipLaunchKernelGGL(rec_words == 2 ? session_lookup_lds_kernel<2> : session_lookup_lds_kernel<3>,
                       dim3(nsub), dim3(kSessLookupBlock), lds,
                       (hipStream_t)stream, recs, counts, nsrc, nsub, bcap, cap_log2, keys_g,
                       spill_set, spill_mask, spill_any, sk, vals, n_out, host_recs, n_host,
                       host_cap, n_inserted, tbits);
  } else {
    const uint32_t chunks = (bcap + kLookupChunk - 1) / kLookupChunk;
    hipLaunchKernelGGL(rec_words == 2 ? session_lookup_kernel<2> : session_lookup_kernel<3>,
                       dim3(chunks, nsrc * nsub), dim3(256), 0,
                       (hipStream_t)stream, recs, counts, nsrc, nsub, bcap, cap_log2, keys_g,
                       spill_set, spill_mask, spill_any, sk, vals, n_out, host_recs, n_host,
                       host_cap, n_inserted, tbits);
  }
  HIP_CHECK(hipGetLastError());
}

size_t session_lookup_sort_lds(int cap_log2, uint32_t m_cap) {
  const size_t cap = (size_t)1 << cap_log2;
  const size_t a = cap * 8 > cap * 2 + (size_t)m_cap * 2 ? cap * 8 : cap * 2 + (size_t)m_cap * 2;
  return a + (size_t)m_cap * 8;
}

bool session_lookup_sort(const void* recs, const uint32_t* counts, int nsrc, int nsub,
                         uint32_t bcap, int cap_log2, uint64_t* keys_g, uint64_t* spill_set,
                         uint32_t spill_mask, int spill_any, int64_t* sort_out, uint64_t* vals_out,
                         uint32_t* n_out, Rec* host_recs, uint32_t* n_host, uint32_t host_cap,
                         uint32_t* n_inserted, int tbits, intptr_t stream, const int64_t* skip,
                         uint32_t skip_mask, uint64_t* heads_out, uint32_t* n_heads, int pair,
                         int rec_words) {
  if (rec_words != 2 && rec_words != 3)
    throw std::invalid_argument("session_lookup_sort: 16- or 24-byte records");
  if (nsrc * nsub <= 0) return true;
  if (pair && ((uintptr_t)sort_out & 15))
    throw std::invalid_argument("session_lookup_sort: pair output must be 16-byte aligned");
  if (tbits < 1 || tbits > 32) throw std::invalid_argument("session_lookup_sort: tbits out of range");
  const uint64_t m64 = (uint64_t)nsrc * bcap;
  if (nsrc > 64 || cap_log2 > kSessLookupLdsMaxLog2 || m64 > 65535) return false;
  const uint32_t m_cap = ((uint32_t)m64 + 7) & ~7u;
  const size_t lds = session_lookup_sort_lds(cap_log2, m_cap);
  if (lds > 156 * 1024) return false;  // static LDS (slot flags, offsets, counters) takes the rest
  auto kfn = rec_words == 2 ? session_lookup_sort_kernel<2> : session_lookup_sort_kernel<3>;
  static bool attr[2] = {false, false};
  if (!attr[rec_words - 2]) {
    // dynamic + the kernel's static LDS (slot flags, segment offsets, scan scratch) <= 160 KiB
    HIP_CHECK(hipFuncSetAttribute((const void*)kfn,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024));
    attr[rec_words - 2] = true;
  }
  hipLaunchKernelGGL(kfn, dim3(nsub), dim3(kSessSortBlock), lds,
                     (hipStream_t)stream, recs, counts, nsrc, nsub, bcap, cap_log2, keys_g,
                     spill_set, spill_mask, spill_any, sort_out, vals_out, n_out, host_recs,
                     n_host, host_cap, n_inserted, tbits, m_cap, skip, skip_mask, heads_out,
                     n_heads, pair);
  HIP_CHECK(hipGetLastError());
  return true;
}

void session_heads(const int64_t* sk, const uint32_t* n_in, int64_t n_cap, uint32_t* heads,
                   uint32_t* n_heads, intptr_t stream) {
  hipLaunchKernelGGL(seg_heads_kernel, dim3(grid_for((n_cap + 63) / 64, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, sk, n_in, heads, n_heads, 32);
  HIP_CHECK(hipGetLastError());
}

void session_merge(const int64_t* sk, const uint64_t* vals, const uint32_t* n_in,
                   uint32_t* long_heads, uint32_t* n_long, int64_t n_cap, int tbits, int64_t gap,
                   int64_t lateness, int64_t wm, int64_t tbase, int agg, int cap_log2,
                   int64_t nslots, int64_t* sess, int64_t* slot_due, int64_t* slot_last,
                   uint64_t* late_cnt, const uint64_t* keys_g, int64_t* ovf_slots,
                   uint32_t* n_ovf, int64_t* ovf_rows, uint32_t* n_ovf_runs, uint32_t ovf_cap,
                   intptr_t stream) {
  const SessArgs a = make_sess_args(gap, lateness, wm, tbase, agg, cap_log2, nslots, tbits);
  const SessOut o{reinterpret_cast<SessRec*>(sess), slot_due, slot_last, late_cnt, keys_g,
                  ovf_slots, n_ovf, ovf_rows, n_ovf_runs, ovf_cap};
  hipLaunchKernelGGL(session_merge_small_kernel, dim3(grid_for(n_cap, 256, 16384)), dim3(256), 0,
                     (hipStream_t)stream, sk, vals, n_in, a, o, long_heads, n_long);
  HIP_CHECK(hipGetLastError());
  // Long segments (hot keys): a wave each; the count stays on the device (grid-stride waves).
  hipLaunchKernelGGL(session_merge_long_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, sk,
                     vals, n_in, long_heads, n_long, a, o);
  HIP_CHECK(hipGetLastError());
}

void session_merge_heads(const int64_t* sk, const uint64_t* vals, const uint32_t* n_in,
                         const uint64_t* heads, const uint32_t* n_heads, int64_t head_cap,
                         uint32_t* long_heads, uint32_t* n_long, int tbits, int64_t gap,
                         int64_t lateness, int64_t wm, int64_t tbase, int agg, int cap_log2,
                         int64_t nslots, int64_t* sess, int64_t* slot_due, int64_t* slot_last,
                         uint64_t* late_cnt, const uint64_t* keys_g, int64_t* ovf_slots,
                         uint32_t* n_ovf, int64_t* ovf_rows, uint32_t* n_ovf_runs,
                         uint32_t ovf_cap, intptr_t stream, int pair) {
  // pair: session_lookup_sort wrote interleaved (sort key, value) pairs at sk (vals unused)
  const SessArgs a = make_sess_args(gap, lateness, wm, tbase, agg, cap_log2, nslots, tbits,
                                    pair ? 2 : 1);
  if (pair) vals = reinterpret_cast<const uint64_t*>(sk) + 1;
  const SessOut o{reinterpret_cast<SessRec*>(sess), slot_due, slot_last, late_cnt, keys_g,
                  ovf_slots, n_ovf, ovf_rows, n_ovf_runs, ovf_cap};
  hipLaunchKernelGGL(session_merge_heads_kernel, dim3(grid_for(head_cap, 256, 16384)), dim3(256),
                     0, (hipStream_t)stream, sk, vals, heads, n_heads, a, o, long_heads, n_long);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(session_merge_long_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, sk,
                     vals, n_in, long_heads, n_long, a, o);
  HIP_CHECK(hipGetLastError());
}

void session_fire(int64_t gap, int64_t lateness, int64_t wm, int agg, int cap_log2,
                  int64_t nslots, const uint64_t* keys_g, int64_t* sess, int64_t* slot_due,
                  const ExprProg& map, const ExprProg& filt, uint64_t* out_key, int64_t* out_start,
                  int64_t* out_end, double* out_val, uint64_t* out_raw, uint32_t* out_cnt,
                  uint32_t* out_n, uint32_t out_cap, intptr_t stream) {
  const SessArgs a = make_sess_args(gap, lateness, wm, 0, agg, cap_log2, nslots);
  const int depth = map.depth > filt.depth ? map.depth : filt.depth;
  const size_t lds = (size_t)(kExprVars + depth) * 256 * sizeof(double);
  hipLaunchKernelGGL(session_fire_kernel, dim3(grid_for(nslots, 256, 8192)), dim3(256), lds,
                     (hipStream_t)stream, a, keys_g, reinterpret_cast<SessRec*>(sess),
                     slot_due, map, filt, out_key, out_start, out_end, out_val, out_raw, out_cnt,
                     out_n, out_cap);
  HIP_CHECK(hipGetLastError());
}

void session_evict(int64_t nslots, int cap_log2, uint64_t* keys_g, int64_t* sess,
                   int64_t* slot_due, int64_t* slot_last, int64_t idle_before, const int64_t* slots,
                   uint32_t nslots_list, uint64_t* spill_set, uint32_t spill_mask, int64_t* st_key,
                   int64_t* st_start, int64_t* st_end, int64_t* st_acc, int64_t* st_cnt,
                   int64_t* st_flags, uint32_t* n_rows, uint32_t row_cap, uint32_t* n_evicted,
                   intptr_t stream) {
  const SessArgs a = make_sess_args(0, 0, 0, 0, 0, cap_log2, nslots);
  const int64_t total = slots ? (int64_t)nslots_list : nslots;
  if (total <= 0) return;
  hipLaunchKernelGGL(session_evict_kernel, dim3(grid_for(total, kEvictBlock, 2048)),
                     dim3(kEvictBlock), 0,
                     (hipStream_t)stream, a, keys_g, reinterpret_cast<SessRec*>(sess),
                     slot_due, slot_last, idle_before, slots, nslots_list, spill_set, spill_mask,
                     st_key, st_start, st_end, st_acc, st_cnt, st_flags, n_rows, row_cap,
                     n_evicted);
  HIP_CHECK(hipGetLastError());
}

void session_rehash(int64_t nslots, int cap_log2, const uint64_t* keys_o, const int64_t* sess_o,
                    const int64_t* due_o, const int64_t* last_o, uint64_t* keys_n, int64_t* sess_n,
                    int64_t* due_n, int64_t* last_n, uint32_t* inserted, intptr_t stream) {
  const SessArgs a = make_sess_args(0, 0, 0, 0, 0, cap_log2, nslots);
  hipLaunchKernelGGL(session_rehash_kernel, dim3(grid_for(nslots, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, a, keys_o, reinterpret_cast<const SessRec*>(sess_o), due_o,
                     last_o, keys_n, reinterpret_cast<SessRec*>(sess_n), due_n, last_n, inserted);
  HIP_CHECK(hipGetLastError());
}

void set_rehash(const uint64_t* old, int64_t n_old, uint64_t* neu, uint32_t new_mask,
                intptr_t stream) {
  if (n_old <= 0) return;
  hipLaunchKernelGGL(set_rehash_kernel, dim3(grid_for(n_old, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, old, n_old, neu, new_mask);
  HIP_CHECK(hipGetLastError());
}

void set_insert_keys(uint64_t* set, uint32_t mask, const int64_t* keys, int64_t n,
                     intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(set_insert_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, set, mask, keys, n);
  HIP_CHECK(hipGetLastError());
}

void set_probe(const uint64_t* set, uint32_t mask, const int64_t* keys, int64_t n, uint8_t* hit,
               uint32_t* n_hit, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(set_probe_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, set, mask, keys, n, hit, n_hit);
  HIP_CHECK(hipGetLastError());
}

void set_erase(uint64_t* set, uint32_t mask, const int64_t* keys, int64_t n, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(set_erase_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, set, mask, keys, n);
  HIP_CHECK(hipGetLastError());
}

void keygroups(const uint64_t* keys, int64_t n, int hash_mode, const int32_t* jhash, int max_par,
               int32_t* kg, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(keygroup_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, keys, n, hash_mode, jhash, max_par, kg);
  HIP_CHECK(hipGetLastError());
}

void table_insert(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2, uint64_t* keys_g,
                  int64_t* slots, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(table_insert_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, keys, n, nsub_log2, cap_log2, keys_g, slots);
  HIP_CHECK(hipGetLastError());
}

void session_promote(const int64_t* slots, const int64_t* rec, const int64_t* last, int64_t n,
                     int64_t* sess, int64_t* slot_due, int64_t* slot_last, uint32_t* n_bad,
                     intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(session_promote_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, slots, rec, last, n, sess, slot_due, slot_last, n_bad);
  HIP_CHECK(hipGetLastError());
}

void session_promote_rows(const int64_t* rows, int64_t n, int nsub_log2, int cap_log2,
                          uint64_t* keys_g, int64_t* slots, int64_t* sess, int64_t* slot_due,
                          int64_t* slot_last, uint32_t* inserted, uint32_t* n_bad,
                          intptr_t stream) {
  if (n <= 0) return;
  for (int phase = 0; phase < 2; ++phase)
    hipLaunchKernelGGL(session_promote_rows_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, rows, n, nsub_log2, cap_log2, phase, keys_g, slots,
                       sess, slot_due, slot_last, inserted, n_bad);
  HIP_CHECK(hipGetLastError());
}

void session_slot_insert(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2,
                         uint64_t* keys_g, int64_t* slots, uint32_t* inserted, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(session_slot_insert_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, keys, n, nsub_log2, cap_log2, keys_g, slots, inserted);
  HIP_CHECK(hipGetLastError());
}

template <int AGG>
static void launch_combine(const Rec* recs, const uint32_t* counts, int nbuckets,
                           const AggPlan& p, Rec* out, uint32_t ccap, uint32_t* out_counts,
                           uint32_t* flags, size_t lds, hipStream_t s) {
  if constexpr (AGG == AGG_SUM_I64 || AGG == AGG_AVG_I64) {
    // packed accumulators: int32 values (8/16-byte records), < 2^16 records per bucket
    AggPlan q = p;
    q.combined = 0;
    if (p.rec_words <= 2 && agg_pack_ok(q)) {
      static bool attr_pk = false;
      if (!attr_pk) {
        HIP_CHECK(hipFuncSetAttribute((const void*)window_combine_kernel<AGG, 1, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        HIP_CHECK(hipFuncSetAttribute((const void*)window_combine_kernel<AGG, 2, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_pk = true;
      }
      const size_t cap = (size_t)1 << p.cap_log2;
      const size_t lds_pk = cap * (p.rec_words == 1 ? 4 : 8) + (size_t)p.pg * cap * 8 + 16;
      if (p.rec_words == 1)
        hipLaunchKernelGGL((window_combine_kernel<AGG, 1, true>), dim3(nbuckets), dim3(1024),
                           lds_pk, s, (const void*)recs, counts, p, out, ccap, out_counts, flags);
      else
        hipLaunchKernelGGL((window_combine_kernel<AGG, 2, true>), dim3(nbuckets), dim3(1024),
                           lds_pk, s, (const void*)recs, counts, p, out, ccap, out_counts, flags);
      return;
    }
  }
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)window_combine_kernel<AGG, 3>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute((const void*)window_combine_kernel<AGG, 2>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute((const void*)window_combine_kernel<AGG, 1>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (p.rec_words == 1)
    hipLaunchKernelGGL((window_combine_kernel<AGG, 1>), dim3(nbuckets), dim3(1024), lds, s,
                       (const void*)recs, counts, p, out, ccap, out_counts, flags);
  else if (p.rec_words == 2)
    hipLaunchKernelGGL((window_combine_kernel<AGG, 2>), dim3(nbuckets), dim3(1024), lds, s,
                       (const void*)recs, counts, p, out, ccap, out_counts, flags);
  else
    hipLaunchKernelGGL((window_combine_kernel<AGG, 3>), dim3(nbuckets), dim3(1024), lds, s,
                       (const void*)recs, counts, p, out, ccap, out_counts, flags);
}

void window_combine(const Rec* recs, const uint32_t* counts, int nbuckets, const AggPlan& p,
                    Rec* out, uint32_t ccap, uint32_t* out_counts, uint32_t* flags,
                    intptr_t stream) {
  if (nbuckets <= 0) return;
  const size_t cap = (size_t)1 << p.cap_log2;
  const size_t lds = cap * 8 + (size_t)p.pg * cap * 12 + 16;
  if (lds > 160 * 1024) throw std::invalid_argument("window_combine: LDS image exceeds 160 KiB");
  hipStream_t s = (hipStream_t)stream;
  switch (p.agg) {
#define MXS_C(A) case A: launch_combine<A>(recs, counts, nbuckets, p, out, ccap, out_counts, flags, lds, s); break;
    MXS_C(AGG_SUM_I64) MXS_C(AGG_SUM_F64) MXS_C(AGG_MIN_I64) MXS_C(AGG_MAX_I64)
    MXS_C(AGG_MIN_F64) MXS_C(AGG_MAX_F64) MXS_C(AGG_COUNT) MXS_C(AGG_AVG_F64) MXS_C(AGG_AVG_I64)
#undef MXS_C
    default: throw std::runtime_error("window_combine: unsupported aggregate");
  }
  HIP_CHECK(hipGetLastError());
}

void f64_order_bits(const uint64_t* v, int64_t n, uint64_t* o, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(f64_order_bits_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, v, n, o);
  HIP_CHECK(hipGetLastError());
}

void segment_median_select(const int64_t* heads, int64_t nseg, int64_t total, const uint64_t* ord,
                           double* out, intptr_t stream) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(segment_median_select_kernel, dim3(grid_for(nseg, 4, 16384)), dim3(256), 0,
                     (hipStream_t)stream, heads, nseg, total, ord, out);
  HIP_CHECK(hipGetLastError());
}

void segment_median(const int64_t* heads, int64_t nseg, int64_t total, const uint64_t* ord,
                    double* out, intptr_t stream) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(segment_median_kernel, dim3(grid_for(nseg, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, heads, nseg, total, ord, out);
  HIP_CHECK(hipGetLastError());
}

void tier_merge(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt, int64_t n,
                const uint32_t* n_dev, int mode, int agg, uint64_t* tkeys, uint64_t* tacc,
                uint32_t* tcnt, uint8_t* tdirty, uint32_t mask, uint32_t* flags, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(tier_merge_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, keys, acc, cnt, n, n_dev, mode, agg, tkeys, tacc, tcnt,
                     tdirty, mask, flags);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
