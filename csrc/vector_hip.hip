// mxstream — vector-metric keyed windows on gfx950: per (key, pane) sums of D-float metric
// vectors (e.g. one usage value per CPU core of a host), reduced on the MATRIX cores.
//
// Reference shape: ComputeCpuAvg.java:27-59 (keyBy(host).timeWindow(1 min).aggregate(avg)) with
// the per-event scalar generalised to a D-vector — the "batched metric-vector reduce" of
// BASELINE.json's north star.
//
// Why MFMA: after the keyBy partition every workgroup owns one hash sub-table. It counting-sorts
// a round of up to 16 Ki records by (pane, slot) in LDS, so equal keys form runs. A wave then
// takes 32 sorted records at a time and computes their per-run (segment) sums as ONE GEMM:
//
//     C[32 segments x 32 metrics] = A[32 segments x 32 records] (one-hot: record k in segment r)
//                                 * B[32 records x 32 metrics]  (the records' metric vectors)
//
// with v_mfma_f32_32x32x16_bf16 (2 k-steps). B is split into three bf16 terms (hi + mid + lo
// reproduces every f32 exactly, A is exactly 0/1), so the three MFMAs per k-step accumulate in
// f32 and the result equals an f32 segmented sum up to summation order. Only the populated rows
// of C (one per run, ~3 per tile at 16 events/key/step) are flushed to HBM, with 128-byte
// contiguous no-return atomics (two 128-B row segments per wave instruction — the full-rate
// atomic shape). Compared with per-record LDS/HBM atomics, hot keys (long runs) never serialise
// on one address; the VALU variant (mode 1: lanes walk the sorted run sequentially) is kept for
// the A/B in scripts/kbench_vector.py.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "mxs_vector.h"

namespace mxs {
namespace {

#define VHIP_CHECK(x)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                  \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kVThreads = 1024;              // 16 waves per workgroup, one workgroup per CU
constexpr int kVWaves = kVThreads / 64;
constexpr int kVPer = 16;                    // records per thread per round
constexpr int kVLoad = 4;                    // record loads in flight per thread
constexpr int kVRound = kVThreads * kVPer;   // 16 Ki records per LDS round
constexpr int kVHist = 4096;                 // (pane, slot) histogram entries per pane group
constexpr uint32_t kHole = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t vprobe_insert(uint64_t* skeys, uint64_t key, uint32_t mask,
                                                  int* inserted) {
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    // Relaxed workgroup-scope atomic load (a volatile read compiles to a generic flat load that
    // waits for all outstanding global loads; see lds_probe_insert in kernels_hip.hip).
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

// Block-wide exclusive scan of one uint32 per thread (1024 threads); wsum = 17 words of LDS,
// wsum[16] = total.
__device__ __forceinline__ uint32_t vblock_scan(uint32_t v, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
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
    for (int w = 0; w < kVWaves; ++w) {
      const uint32_t t = wsum[w];
      wsum[w] = acc;
      acc += t;
    }
    wsum[16] = acc;
  }
  __syncthreads();
  return wsum[wid] + x - v;
}

__device__ __forceinline__ void split3(float v, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)v;
  const float r1 = v - (float)hi;
  mid = (__bf16)r1;
  lo = (__bf16)(r1 - (float)mid);
}

template <int RW>
__device__ __forceinline__ void vload_rec(const void* base, size_t idx, uint64_t& key, uint32_t& val,
                                          uint32_t& t) {
  if (RW == 2) {
    const uint4 c = ((const uint4*)base)[idx];
    key = (uint64_t)c.x | ((uint64_t)c.y << 32);
    val = c.z;
    t = c.w;
  } else {
    const Rec r = ((const Rec*)base)[idx];
    key = r.key;
    val = (uint32_t)r.val;
    t = r.t;
  }
}

__device__ __forceinline__ size_t vslot_index(uint32_t cc, const VecAggPlan& p, int64_t q0,
                                              size_t nslots, size_t sbase, uint32_t mask) {
  const int64_t pane = p.pane_base + q0 + (cc >> p.cap_log2);
  return (size_t)(pane & (p.ring - 1)) * nslots + sbase + (cc & mask);
}

// ------------------------------------------------------------------------------------------
// vec_window_agg: one 1024-thread workgroup per sub-table.
// LDS: skeys[cap] u64 | hist[kVHist] u32 | srow[kVRound] u32 | sseg[kVRound] u16 |
//      segtab[kVWaves][32] u32 | wsum[20] u32 | flags[4] i32
// ------------------------------------------------------------------------------------------
template <int MODE, int RW>
__global__ __launch_bounds__(kVThreads) void vec_window_agg_kernel(
    const void* __restrict__ recs, const uint32_t* __restrict__ counts, VecAggPlan p,
    const float* __restrict__ vec, uint64_t* __restrict__ keys_g, float* __restrict__ acc_g,
    uint32_t* __restrict__ cnt_g, uint8_t* __restrict__ dirty_g, uint32_t* __restrict__ occupancy,
    uint32_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int sub = blockIdx.x;
  const uint32_t cap = 1u << p.cap_log2;
  const uint32_t mask = cap - 1;
  uint64_t* skeys = (uint64_t*)smem;
  uint32_t* hist = (uint32_t*)(skeys + cap);
  uint32_t* srow = hist + kVHist;
  uint16_t* sseg = (uint16_t*)(srow + kVRound);
  uint32_t* segtab = (uint32_t*)(sseg + kVRound);
  uint32_t* wsum = segtab + kVWaves * 32;
  int* sflag = (int*)(wsum + 20);

  const int D = p.dim;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const size_t sbase = (size_t)sub << p.cap_log2;
  const size_t nslots = (size_t)p.nsub << p.cap_log2;
  for (uint32_t i = threadIdx.x; i < cap; i += kVThreads) skeys[i] = keys_g[sbase + i];
  if (threadIdx.x < 4) sflag[threadIdx.x] = 0;
  const int pg = (int)(kVHist >> p.cap_log2);  // panes per group
  int inserted = 0;
  bool ovf = false;
  __syncthreads();

  for (int pg0 = 0; pg0 < p.np_step; pg0 += pg) {
    const int npg = (p.np_step - pg0) < pg ? (p.np_step - pg0) : pg;
    const uint32_t nh = (uint32_t)npg << p.cap_log2;
    const int64_t q0 = p.p_lo + pg0;
    for (int src = 0; src < p.nsrc; ++src) {
      uint32_t c = counts[(size_t)src * p.nsub + sub];
      c = c < p.bucket_cap ? c : p.bucket_cap;
      const size_t seg0 = ((size_t)src * p.nsub + sub) * p.bucket_cap;
      for (uint32_t r0 = 0; r0 < c; r0 += kVRound) {
        for (uint32_t i = threadIdx.x; i < nh; i += kVThreads) hist[i] = 0;
        __syncthreads();
        // 1. slot lookup + (pane, slot) histogram; the rank inside a bin comes from the atomic.
        uint32_t ck[kVPer], rowk[kVPer];
        uint64_t kk[kVLoad];
        uint32_t vv[kVLoad], tt[kVLoad];
#pragma unroll
        for (int u = 0; u < kVPer; ++u) {
          if (u % kVLoad == 0) {
            // kVLoad branch-free record loads in flight, pinned in registers before the probes
            // (a load per record under `if (e < c)` waited on vmcnt(0) each time).
#pragma unroll
            for (int j = 0; j < kVLoad; ++j) {
              const uint32_t e = r0 + (uint32_t)(u + j) * kVThreads + threadIdx.x;
              vload_rec<RW>(recs, seg0 + (e < c ? e : c - 1), kk[j], vv[j], tt[j]);
            }
#pragma unroll
            for (int j = 0; j < kVLoad; ++j) asm volatile("" : "+v"(kk[j]), "+v"(vv[j]), "+v"(tt[j]));
          }
          ck[u] = kHole;
          rowk[u] = 0;
          const uint32_t e = r0 + (uint32_t)u * kVThreads + threadIdx.x;
          if (e >= c) continue;
          const uint64_t key = kk[u % kVLoad];
          const uint32_t val = vv[u % kVLoad], t = tt[u % kVLoad];
          if (t == kHole) continue;
          const int64_t q = (int64_t)t - q0;
          if (q < 0 || q >= npg) continue;
          const uint32_t s = vprobe_insert(skeys, key, mask, &inserted);
          if (s == kNoSlot) {
            ovf = true;
            continue;
          }
          const uint32_t cc = ((uint32_t)q << p.cap_log2) | s;
          const uint32_t rk = atomicAdd(&hist[cc], 1u);
          ck[u] = (cc << 16) | rk;
          rowk[u] = p.positional ? (uint32_t)(seg0 + e) : val;
        }
        __syncthreads();
        // 2. exclusive scan of the histogram (each thread owns a contiguous run of bins) and the
        //    element counts of the touched (pane, slot) pairs (plain RMW: this group owns them).
        const uint32_t per = (nh + kVThreads - 1) / kVThreads;
        const uint32_t b0 = threadIdx.x * per < nh ? threadIdx.x * per : nh;
        const uint32_t b1 = b0 + per < nh ? b0 + per : nh;
        uint32_t tsum = 0;
        for (uint32_t b = b0; b < b1; ++b) tsum += hist[b];
        uint32_t run = vblock_scan(tsum, wsum);
        const uint32_t nrec = wsum[16];
        for (uint32_t b = b0; b < b1; ++b) {
          const uint32_t n_b = hist[b];
          hist[b] = run;
          run += n_b;
          if (!n_b) continue;
          const int64_t pane = p.pane_base + q0 + (b >> p.cap_log2);
          const size_t gi = (size_t)(pane & (p.ring - 1)) * nslots + sbase + (b & mask);
          cnt_g[gi] += n_b;
          if (pane <= p.fired_hi) dirty_g[gi] = 1;
        }
        __syncthreads();
        // 3. scatter into (pane, slot) order.
#pragma unroll
        for (int u = 0; u < kVPer; ++u) {
          if (ck[u] == kHole) continue;
          const uint32_t cc = ck[u] >> 16;
          const uint32_t pos = hist[cc] + (ck[u] & 0xFFFFu);
          srow[pos] = rowk[u];
          sseg[pos] = (uint16_t)cc;
        }
        __syncthreads();
        // 4. per 32-record tile: segment ids by ballot, segmented sum, flush one row per run.
        const uint32_t ntiles = (nrec + 31) >> 5;
        for (uint32_t tile = wid; tile < ntiles; tile += kVWaves) {
          const uint32_t base = tile << 5;
          const uint32_t idx = base + r;
          const bool valid = idx < nrec;
          const uint32_t cs = valid ? sseg[idx] : 0xFFFFFFFFu;
          const uint32_t cprev = (valid && r > 0) ? sseg[idx - 1] : 0xFFFFFFFEu;
          const bool head = valid && (r == 0 || cs != cprev);
          const uint64_t hm = __ballot(head) & 0xFFFFFFFFull;
          const int nseg = __popcll(hm);
          const int segid = valid ? __popcll(hm & ((2ull << r) - 1)) - 1 : -1;
          if (head && h == 0) segtab[wid * 32 + segid] = cs;
          __builtin_amdgcn_wave_barrier();
          if (MODE == 0) {
            // A fragment (one-hot): lane (r, h), element j of k-step s is A[r][16s + 8h + j].
            bf16x8 a[2];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const int sk = __shfl(segid, 16 * s + 8 * h + j);
                a[s][j] = (__bf16)(sk == r ? 1.0f : 0.0f);
              }
            for (int n = 0; n < (D >> 5); ++n) {
              f32x16 acc = {};
              // Both k-steps' 16 loads issued before the first MFMA (rows re-read from LDS per n).
              float v[2][8];
#pragma unroll
              for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const uint32_t k = base + 16 * s + 8 * h + j;
                  v[s][j] = k < nrec ? vec[(size_t)srow[k] * D + 32 * n + r] : 0.0f;
                }
#pragma unroll
              for (int s = 0; s < 2; ++s) {
                bf16x8 bh, bm, bl;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  __bf16 x, y, z;
                  split3(v[s][j], x, y, z);
                  bh[j] = x;
                  bm[j] = y;
                  bl[j] = z;
                }
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], bl, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], bm, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], bh, acc, 0, 0, 0);
              }
              // C/D map of 32x32: col = lane & 31 (metric), row = (i&3) + 8*(i>>2) + 4*h (segment).
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
                if (row < nseg) {
                  const size_t gi = vslot_index(segtab[wid * 32 + row], p, q0, nslots, sbase, mask);
                  atomicAdd(&acc_g[gi * D + 32 * n + r], acc[i]);
                }
              }
            }
          } else {
            // VALU variant: half-wave h walks records 16h .. 16h+15 of the tile in order, lane r
            // holds metric r of the current run and flushes it when the run ends.
            for (int n = 0; n < (D >> 5); ++n) {
              float sum = 0.0f;
              int cur = -1;
              for (int j = 0; j < 16; ++j) {
                const uint32_t k = base + 16 * h + j;
                const int sk = __shfl(segid, 16 * h + j);
                if (k >= nrec) break;
                if (sk != cur) {
                  if (cur >= 0) {
                    const size_t gi = vslot_index(segtab[wid * 32 + cur], p, q0, nslots, sbase, mask);
                    atomicAdd(&acc_g[gi * D + 32 * n + r], sum);
                  }
                  cur = sk;
                  sum = 0.0f;
                }
                sum += vec[(size_t)srow[k] * D + 32 * n + r];
              }
              if (cur >= 0) {
                const size_t gi = vslot_index(segtab[wid * 32 + cur], p, q0, nslots, sbase, mask);
                atomicAdd(&acc_g[gi * D + 32 * n + r], sum);
              }
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
      }
    }
  }
  if (inserted) sflag[0] = 1;
  if (ovf) sflag[1] = 1;
  __syncthreads();
  if (sflag[0]) {
    for (uint32_t i = threadIdx.x; i < cap; i += kVThreads) {
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
// vec_window_fire: 256 slots per workgroup iteration. Pass A: a half-wave per slot (32 lanes =
// 32 metrics per load) sums the window's panes, applies avg and the alert predicate, and records a
// live flag; a block scan turns the flags into output offsets with ONE output-cursor atomic per
// 256 slots (same-address atomics serialise at L2: one per 8 slots cost 2.8 ms on 2M slots).
// Pass B: the live slots' vectors are recomputed (only alerts are re-read) and written.
// ------------------------------------------------------------------------------------------
constexpr int kVFThreads = 256;
constexpr int kVFHalves = kVFThreads / 32;
constexpr int kVFIter = 256;  // slots per workgroup iteration

__device__ __forceinline__ uint32_t vf_window(const VecFirePlan& p, const uint64_t* keys_g,
                                              const uint32_t* cnt_g, const uint8_t* dirty_g,
                                              int64_t s, bool* dirty) {
  uint32_t cnt = 0;
  *dirty = false;
  if (s >= p.nslots || keys_g[s] == kEmptyKey) return 0;
  for (int q = 0; q < p.npanes; ++q) {
    const size_t gi = (size_t)((p.p0 + q) & (p.ring - 1)) * p.nslots + s;
    cnt += cnt_g[gi];
    if (p.only_dirty) *dirty |= dirty_g[gi] != 0;
  }
  return cnt;
}

// Result vector of slot s in res[0 .. D/32) (lane r holds metrics r, 32 + r, ...); returns the
// max over metrics (half-wave reduction).
__device__ __forceinline__ float vf_result(const VecFirePlan& p, const float* acc_g,
                                           const uint32_t* cnt_g, int64_t s, uint32_t cnt, int r,
                                           float* res) {
  const int D = p.dim;
#pragma unroll
  for (int n = 0; n < 8; ++n) res[n] = 0.0f;
  for (int q = 0; q < p.npanes; ++q) {
    const size_t gi = (size_t)((p.p0 + q) & (p.ring - 1)) * p.nslots + s;
    if (!cnt_g[gi]) continue;
#pragma unroll
    for (int n = 0; n < 8; ++n)
      if (32 * n < D) res[n] += acc_g[gi * D + 32 * n + r];
  }
  float mx = -INFINITY;
#pragma unroll
  for (int n = 0; n < 8; ++n)
    if (32 * n < D) {
      if (p.avg) res[n] = res[n] / (float)cnt;
      mx = res[n] > mx ? res[n] : mx;
    }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    const float w = __shfl_xor(mx, o);
    mx = w > mx ? w : mx;
  }
  return mx;
}

__global__ __launch_bounds__(kVFThreads) void vec_window_fire_kernel(
    const uint64_t* __restrict__ keys_g, const float* __restrict__ acc_g,
    const uint32_t* __restrict__ cnt_g, const uint8_t* __restrict__ dirty_g, VecFirePlan p,
    uint64_t* __restrict__ out_keys, float* __restrict__ out_vec, uint32_t* __restrict__ out_cnt,
    uint32_t* __restrict__ out_n) {
  __shared__ uint32_t live[kVFIter];
  __shared__ uint32_t scnt[kVFIter];
  __shared__ uint32_t wsum[kVFThreads / 64 + 1];
  __shared__ uint32_t obase;
  const int r = threadIdx.x & 31;
  const int half = threadIdx.x >> 5;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int D = p.dim;
  float res[8];
  for (int64_t s0 = (int64_t)blockIdx.x * kVFIter; s0 < p.nslots;
       s0 += (int64_t)gridDim.x * kVFIter) {
    // Pass A1: thread per slot (coalesced key / count reads) -> element count in LDS.
    {
      bool dirty;
      const uint32_t cnt = vf_window(p, keys_g, cnt_g, dirty_g, s0 + threadIdx.x, &dirty);
      scnt[threadIdx.x] = (cnt > 0 && (!p.only_dirty || dirty)) ? cnt : 0u;
    }
    __syncthreads();
    // Pass A2: alert predicate on the live slots' result vectors (half-wave per slot).
    for (int j = half; j < kVFIter; j += kVFHalves) {
      const uint32_t cnt = scnt[j];
      bool ok = cnt > 0;
      if (ok && p.use_thr) ok = vf_result(p, acc_g, cnt_g, s0 + j, cnt, r, res) > p.thr;
      if (r == 0) live[j] = ok ? 1u : 0u;
    }
    __syncthreads();
    // Block exclusive scan of the 256 flags (one per thread) + one cursor atomic.
    const uint32_t f = live[threadIdx.x];
    uint32_t x = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t acc = 0;
      for (int w = 0; w < kVFThreads / 64; ++w) {
        const uint32_t t = wsum[w];
        wsum[w] = acc;
        acc += t;
      }
      obase = acc ? atomicAdd(out_n, acc) : 0u;
    }
    __syncthreads();
    const uint32_t myoff = wsum[wid] + x - f;
    __syncthreads();
    live[threadIdx.x] = f ? myoff + 1 : 0u;  // 1-based offset, 0 = not emitted
    __syncthreads();
    // Pass B: write the live slots.
    for (int j = half; j < kVFIter; j += kVFHalves) {
      const uint32_t l = live[j];
      if (!l) continue;
      const int64_t s = s0 + j;
      const uint32_t o = obase + l - 1;
      if (o >= p.out_cap) continue;
      const uint32_t cnt = scnt[j];
      vf_result(p, acc_g, cnt_g, s, cnt, r, res);
      if (r == 0) {
        out_keys[o] = keys_g[s];
        out_cnt[o] = cnt;
      }
#pragma unroll
      for (int n = 0; n < 8; ++n)
        if (32 * n < D) out_vec[(size_t)o * D + 32 * n + r] = res[n];
    }
    __syncthreads();
  }
}

// Synthetic metric vectors: vec[i*D + d] uniform in [lo, lo + span) from a counter-based RNG
// (row i of the batch = event idx0 + i of the stream, so CPU and GPU generate the same data).
// One thread per 4 consecutive metrics of a row: one 16-byte store.
__global__ __launch_bounds__(256) void gen_vectors_kernel(float* __restrict__ vec, int64_t n, int D,
                                                          uint64_t seed, uint64_t stream_id,
                                                          uint64_t idx0, float lo, float span) {
  const int q = D >> 2;  // float4 per row
  const int64_t total = n * (int64_t)q;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t row = i / q;
    const int d = (int)(i - row * q) * 4;
    const uint64_t ev = idx0 + (uint64_t)row;
    float4 v;
    v.x = gen_vector_value(seed, stream_id, ev, d, lo, span);
    v.y = gen_vector_value(seed, stream_id, ev, d + 1, lo, span);
    v.z = gen_vector_value(seed, stream_id, ev, d + 2, lo, span);
    v.w = gen_vector_value(seed, stream_id, ev, d + 3, lo, span);
    ((float4*)vec)[i] = v;
  }
}

// G > 1: copy each bucket record's metric vector into the send layout (vector j <-> record j),
// so the all-to-all moves vectors next to their records and the receiver reads positionally.
__global__ __launch_bounds__(256) void vec_gather_kernel(const void* __restrict__ recs, int rec_words,
                                                         const uint32_t* __restrict__ counts,
                                                         int nb, uint32_t bcap,
                                                         const float* __restrict__ vec, int D,
                                                         float* __restrict__ out) {
  const int64_t total = (int64_t)nb * bcap;
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 32);
  const int r = threadIdx.x & 31;
  for (int64_t j = (int64_t)blockIdx.x * (blockDim.x / 32) + (threadIdx.x >> 5); j < total; j += stride) {
    const int b = (int)(j / bcap);
    const uint32_t e = (uint32_t)(j - (int64_t)b * bcap);
    if (e >= counts[b]) continue;
    uint32_t row, t;
    if (rec_words == 2) {
      const uint4 c = ((const uint4*)recs)[j];
      row = c.z;
      t = c.w;
    } else {
      const Rec rr = ((const Rec*)recs)[j];
      row = (uint32_t)rr.val;
      t = rr.t;
    }
    if (t == kHole) continue;
    for (int d = r; d < D; d += 32) out[j * D + d] = vec[(size_t)row * D + d];
  }
}

int vgrid(int64_t n, int per, int max_blocks) {
  int64_t b = (n + per - 1) / per;
  if (b < 1) b = 1;
  if (b > max_blocks) b = max_blocks;
  return (int)b;
}

template <int MODE, int RW>
void launch_vagg(const void* recs, const uint32_t* counts, const VecAggPlan& p, const float* vec,
                 uint64_t* keys_g, float* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                 uint32_t* occ, uint32_t* flags, size_t lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    VHIP_CHECK(hipFuncSetAttribute((const void*)vec_window_agg_kernel<MODE, RW>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((vec_window_agg_kernel<MODE, RW>), dim3(p.nsub), dim3(kVThreads), lds, s,
                     recs, counts, p, vec, keys_g, acc_g, cnt_g, dirty_g, occ, flags);
}

}  // namespace

namespace gpu {

size_t vec_window_agg_lds(int cap_log2) {
  return ((size_t)8 << cap_log2) + (size_t)kVHist * 4 + (size_t)kVRound * 6 + kVWaves * 32 * 4 +
         24 * 4;
}

void vec_window_agg(const void* recs, const uint32_t* counts, const VecAggPlan& p,
                    const float* vec, uint64_t* keys_g, float* acc_g, uint32_t* cnt_g,
                    uint8_t* dirty_g, uint32_t* occupancy, uint32_t* flags, intptr_t stream) {
  if (p.np_step <= 0 || p.nsub <= 0) return;
  const size_t lds = vec_window_agg_lds(p.cap_log2);
  if (lds > 160 * 1024) throw std::runtime_error("vec_window_agg: LDS image exceeds 160 KiB");
  hipStream_t s = (hipStream_t)stream;
  const int key = p.mode * 2 + (p.rec_words == 2 ? 0 : 1);
  switch (key) {
    case 0: launch_vagg<0, 2>(recs, counts, p, vec, keys_g, acc_g, cnt_g, dirty_g, occupancy, flags, lds, s); break;
    case 1: launch_vagg<0, 3>(recs, counts, p, vec, keys_g, acc_g, cnt_g, dirty_g, occupancy, flags, lds, s); break;
    case 2: launch_vagg<1, 2>(recs, counts, p, vec, keys_g, acc_g, cnt_g, dirty_g, occupancy, flags, lds, s); break;
    case 3: launch_vagg<1, 3>(recs, counts, p, vec, keys_g, acc_g, cnt_g, dirty_g, occupancy, flags, lds, s); break;
    default: throw std::invalid_argument("vec_window_agg: mode must be 0 (MFMA) or 1 (VALU)");
  }
  VHIP_CHECK(hipGetLastError());
}

void vec_window_fire(const uint64_t* keys_g, const float* acc_g, const uint32_t* cnt_g,
                     const uint8_t* dirty_g, const VecFirePlan& p, uint64_t* out_keys,
                     float* out_vec, uint32_t* out_cnt, uint32_t* out_n, intptr_t stream) {
  if (p.nslots <= 0) return;
  hipLaunchKernelGGL(vec_window_fire_kernel, dim3(vgrid(p.nslots, kVFIter, 2048)),
                     dim3(kVFThreads), 0, (hipStream_t)stream, keys_g, acc_g, cnt_g, dirty_g, p,
                     out_keys, out_vec, out_cnt, out_n);
  VHIP_CHECK(hipGetLastError());
}

void gen_vectors(float* vec, int64_t n, int dim, uint64_t seed, uint64_t stream_id, uint64_t idx0,
                 float lo, float span, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gen_vectors_kernel, dim3(vgrid(n * (dim / 4), 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, vec, n, dim, seed, stream_id, idx0, lo, span);
  VHIP_CHECK(hipGetLastError());
}

void vec_gather(const void* recs, int rec_words, const uint32_t* counts, int nb, uint32_t bcap,
                const float* vec, int dim, float* out, intptr_t stream) {
  const int64_t total = (int64_t)nb * bcap;
  if (total <= 0) return;
  hipLaunchKernelGGL(vec_gather_kernel, dim3(vgrid(total, 8, 8192)), dim3(256), 0,
                     (hipStream_t)stream, recs, rec_words, counts, nb, bcap, vec, dim, out);
  VHIP_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
