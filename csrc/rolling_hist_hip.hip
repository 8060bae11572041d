// mxstream — sort-free keyed rolling COUNT for small key spaces (gfx950).
//
// BASELINE config 2 ("keyed ValueState counter", 10k keys) and any `keyBy(..)` counter whose
// state table fits in LDS: every record emits its key's post-update count in arrival order
// (StreamGroupedReduce / ValueState semantics, chapter2/src/main/java/me/zjy/ComputeCpuMax.java:26,
// golden chapter2/README.md:62-66). The general path (kernels_hip.hip rolling_lookup_direct ->
// radix sort -> rolling_heads -> rolling_scan) sorts the whole batch by slot; with <= 16K slots a
// counting formulation needs no sort at all:
//
//   1. hist   (one 1024-thread workgroup per chunk of <= 64K records): find/insert every key in
//             the HBM hash table, write its slot as u16, LDS histogram of the chunk's slots,
//             histogram written out (part[chunk][slot]).
//   2. group + prefix: per slot, an exclusive scan over the chunks seeded by the stored count
//             (two launches: 16-chunk group totals, then the per-chunk prefixes); the final count
//             is written back to the state table here.
//   3. emit   (one 512-thread workgroup per chunk): the chunk's running counts start from its
//             exclusive prefix in LDS; records are ranked a 512-record tile at a time. Within a
//             tile, every record writes its thread id to owner[slot]; the write that lands names
//             the slot for the tile (no atomics, no hash table). Every record ORs its lane bit
//             into its owner's per-wave 64-bit lane mask; a record's rank is then
//             popcount(masks of earlier waves) + popcount(own wave's mask below its lane) --
//             arrival order without a sort or a serial chain between waves. The last record of a
//             slot in the tile advances the running count (applied after the next tile's first
//             barrier; two mask buffers alternate, so a tile costs two barriers). The traced
//             filter epilogue and the wave-ballot row compaction are fused.
//
// Per record: 8 B key read + 2 B slot write (hist), 2 B slot read (emit) instead of the sort
// path's 32 B in / 32 B out per pass. Output rows are unordered (the host restores arrival order
// by tag, exactly as for the sort path); values are bit-identical to the C++ twin rolling_rows.
#include <hip/hip_runtime.h>

#include <cstdlib>
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

constexpr int kHistThreads = 1024;
constexpr int kTileWaves = 8;
constexpr int kTile = kTileWaves * 64;  // records per tile = threads of the emit workgroup
constexpr uint16_t kNoSlot16 = 0xFFFF;
constexpr uint32_t kChunkMin = kTile, kChunkMax = 65536;
constexpr int kGroup = 16;  // chunks per group in the cross-chunk scan

struct Geo {
  uint32_t chunk, nb, ngroups;
};

Geo geometry(uint32_t n) {
  // >= 256 chunks when the batch allows it (one workgroup per CU), tiles of whole 512 records.
  uint64_t c = ((uint64_t)n + 255) / 256;
  c = (c + kTile - 1) / kTile * kTile;
  if (c < kChunkMin) c = kChunkMin;
  if (c > kChunkMax) c = kChunkMax;
  Geo g;
  g.chunk = (uint32_t)c;
  g.nb = n ? (uint32_t)(((uint64_t)n + c - 1) / c) : 0;
  g.ngroups = (g.nb + kGroup - 1) / kGroup;
  return g;
}

struct RollVars {  // filter variables of the rolling epilogue (rolling_scan's numbering)
  double v0, v1, v4, v5;
  __device__ __forceinline__ double get(int i) const {
    switch (i) {
      case 0: return v0;
      case 1: return v1;
      case 4: return v4;
      case 5: return v5;
      case 6: return v0;
      default: return 0.0;
    }
  }
};

// Insert-or-find by linear probing, eight slots per round trip: the chain is contiguous, so one
// batch of independent loads covers what would otherwise be up to eight dependent L2 reads (the
// tail of the probe-length distribution, not its mean, sets a wave's latency).
// The probe reads are plain (L2-cacheable) loads, not device-scope atomic loads: the table is
// insert-only (a slot goes EMPTY -> key once), so a stale line can only show EMPTY where a key
// now sits, and the device-scope CAS on that slot returns the real occupant (our key: found;
// another key: probing continues after it). Device-scope loads of a 128 KB table hammered by
// every CU are served past the per-XCD L2s.
// A chain filter decoded once per workgroup into registers: the per-record evaluation is then an
// unrolled sequence of uniform branches with hoisted operands, instead of re-reading the program
// (op, arg) pairs from kernel-argument memory and branching on them for every record.
constexpr int kChainOps = 8;
struct ChainRegs {
  int n;  // binops; -1 = longer than kChainOps (use expr_eval_chain)
  int v0;
  int op[kChainOps], src[kChainOps];  // src < 0: constant c[k]
  double c[kChainOps];
  // `x % c` by an integer constant 2 <= c < 2^32: round-up magic multiplier (m, l) for an exact
  // u32 remainder when x is an integer in [0, 2^32) -- counts and key ids always are -- in 7
  // integer ops instead of the library f64 fmod (frexp/ldexp/division: ~80 us per 16.7M rows).
  uint32_t mag[kChainOps], dc[kChainOps];
  int ml[kChainOps];
  // Integer mode: the chain starts from a count variable and only takes remainders by those
  // constants and compares with integer constants (`count % N == 0`, `count >= 1000`): the
  // running value stays an exact u32/0-1 integer, so no f64 op is needed at all.
  bool intmode;
  int64_t ci[kChainOps];
};

__device__ __forceinline__ ChainRegs decode_chain(const ExprProg& p) {
  ChainRegs r;
  r.n = (p.ncode - 1) / 2;
  r.v0 = p.code[1];
  r.intmode = false;
  if (r.n > kChainOps) {
    r.n = -1;
    return r;
  }
  bool im_all = r.v0 == 0 || r.v0 == 1 || r.v0 == 5 || r.v0 == 6;  // count-valued for COUNT
#pragma unroll
  for (int k = 0; k < kChainOps; ++k) {
    const int i = 1 + 2 * k;  // operand pair i, binop pair i + 1
    const bool on = k < r.n;
    const int pop = on ? p.code[2 * i] : OP_CONST;
    const int parg = on ? p.code[2 * i + 1] : 0;
    r.op[k] = on ? p.code[2 * (i + 1)] : OP_ADD;
    r.src[k] = pop == OP_CONST ? -1 : parg;
    r.c[k] = pop == OP_CONST && on ? p.consts[parg] : 0.0;
    const double c = r.c[k];
    const bool im = on && r.op[k] == OP_MOD && pop == OP_CONST && c >= 2.0 && c < 4294967296.0 &&
                    c == trunc(c);
    r.dc[k] = im ? (uint32_t)c : 0u;  // 0 = no integer fast path
    r.ml[k] = im ? 32 - __clz((int)(r.dc[k] - 1)) : 1;
    r.mag[k] = im ? (uint32_t)(((uint64_t)((1ull << r.ml[k]) - r.dc[k]) << 32) / r.dc[k] + 1) : 0u;
    const bool cmp = r.op[k] >= OP_LT && r.op[k] <= OP_NE && pop == OP_CONST && c == trunc(c) &&
                     fabs(c) < 9007199254740992.0;
    r.ci[k] = cmp ? (int64_t)c : 0;
    if (on && !im && !cmp) im_all = false;
  }
  r.intmode = im_all;
  return r;
}

// Integer-mode chain (ChainRegs::intmode) on a count.
__device__ __forceinline__ bool eval_chain_int(const ChainRegs& r, uint32_t count) {
  int64_t x = count;  // stays in [0, 2^32): remainders of a u32 or 0/1 compare results
#pragma unroll
  for (int k = 0; k < kChainOps; ++k) {
    if (k >= r.n) break;
    const int64_t c = r.ci[k];
    switch (r.op[k]) {
      case OP_MOD: {
        const uint32_t u = (uint32_t)x;
        const uint32_t t = __umulhi(r.mag[k], u);
        const uint32_t q = (t + ((u - t) >> 1)) >> (r.ml[k] - 1);
        x = u - q * r.dc[k];
        break;
      }
      case OP_LT: x = x < c; break;
      case OP_LE: x = x <= c; break;
      case OP_GT: x = x > c; break;
      case OP_GE: x = x >= c; break;
      case OP_EQ: x = x == c; break;
      default: x = x != c; break;  // OP_NE
    }
  }
  return x != 0;
}

template <class Vars>
__device__ __forceinline__ double eval_chain_regs(const ChainRegs& r, const ExprProg& p,
                                                  const Vars& vars) {
  if (r.n < 0) return expr_eval_chain(p, vars);
  double x = vars.get(r.v0);
#pragma unroll
  for (int k = 0; k < kChainOps; ++k) {
    if (k >= r.n) break;
    if (r.dc[k] && x >= 0.0 && x < 4294967296.0 && x == trunc(x)) {
      // fmod(x, c) for integers is the integer remainder, +0 included (x >= 0).
      const uint32_t u = (uint32_t)x;
      const uint32_t t = __umulhi(r.mag[k], u);
      const uint32_t q = (t + ((u - t) >> 1)) >> (r.ml[k] - 1);
      x = (double)(u - q * r.dc[k]);
      continue;
    }
    const double b = r.src[k] < 0 ? r.c[k] : vars.get(r.src[k]);
    x = expr_binop(r.op[k], x, b);
  }
  return x;
}

__device__ __forceinline__ uint32_t probe_insert(uint64_t* keys, uint64_t key, uint32_t mask) {
  constexpr uint32_t W = 8;
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t done = 0; done <= mask;) {
    uint64_t k[W];
#pragma unroll
    for (uint32_t j = 0; j < W; ++j) k[j] = keys[(s + j) & mask];  // plain: see below
    uint32_t j = 0;
    for (; j < W; ++j) {
      if (k[j] == key) return (s + j) & mask;
      if (k[j] == kEmptyKey) break;
    }
    if (j < W) {  // first empty slot of the chain: claim it (or meet a racing insert of key)
      const uint32_t t = (s + j) & mask;
      const uint64_t prev = atomicCAS((unsigned long long*)&keys[t], (unsigned long long)kEmptyKey,
                                      (unsigned long long)key);
      if (prev == kEmptyKey || prev == key) return t;
      s = (t + 1) & mask;  // another key took it: continue after it
      done += j + 1;
    } else {
      s = (s + W) & mask;
      done += W;
    }
  }
  return kNoSlot;
}

__global__ __launch_bounds__(kHistThreads) void rolling_hist_count_kernel(
    const uint64_t* __restrict__ keys, uint32_t n, uint32_t chunk, int nsub_log2, int cap_log2,
    uint64_t* __restrict__ keys_g, uint16_t* __restrict__ slot16, uint32_t* __restrict__ part,
    uint32_t nslots, uint32_t* __restrict__ flags, int dense, uint32_t ablate) {
  extern __shared__ uint32_t hcnt[];
  for (uint32_t s = threadIdx.x; s < nslots; s += kHistThreads) hcnt[s] = 0;
  __syncthreads();
  const uint32_t lo = blockIdx.x * chunk;
  const uint32_t hi = n - lo < chunk ? n : lo + chunk;
  const uint32_t mask = (1u << cap_log2) - 1;
  // Eight records per thread per round: the key loads and first-probe table reads are all in
  // flight before any is consumed (most records hit their home slot).
  constexpr int U = 8, W = 4;
  auto finish = [&](uint32_t i, uint32_t slot) {
    slot16[i] = slot == kNoSlot ? kNoSlot16 : (uint16_t)slot;
    if (slot != kNoSlot && !(ablate & 2u)) atomicAdd(&hcnt[slot], 1u);
  };
  if (dense) {  // dictionary ids: slot = key, no table probe (keys_g is filled by the prefix pass)
    for (uint32_t base = lo; base < hi; base += kHistThreads * U) {
      uint64_t key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * kHistThreads + threadIdx.x;
        key[u] = i < hi ? keys[i] : 0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * kHistThreads + threadIdx.x;
        if (i >= hi) continue;
        const bool ok = key[u] < nslots;
        if (!ok) atomicOr(&flags[0], 16u);
        finish(i, ok ? (uint32_t)key[u] : kNoSlot);
      }
    }
  }
  for (uint32_t base = dense ? hi : lo; base < hi; base += kHistThreads * U) {
    uint64_t key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * kHistThreads + threadIdx.x;
      key[u] = i < hi ? keys[i] : 0;
    }
    // Round 1: a 4-slot window from every record's home slot, all 32 loads in flight at once
    // (plain loads: a stale EMPTY only sends the record to the CAS path below).
    uint64_t k[U][W];
    uint32_t home[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * kHistThreads + threadIdx.x;
      home[u] = slot_hash(key[u]) & mask;
      const uint64_t* tab = keys_g + ((size_t)sub_table_of(key[u], nsub_log2) << cap_log2);
#pragma unroll
      for (int j = 0; j < W; ++j) k[u][j] = i < hi ? tab[(home[u] + j) & mask] : 0;
    }
    uint32_t pend = 0;  // records whose key was not met in the window (insert or long chain)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = base + u * kHistThreads + threadIdx.x;
      if (i >= hi) continue;
      if (key[u] >= kTombKey) {  // reserved ids (table markers): flagged, never stored
        atomicOr(&flags[0], 4u);
        finish(i, kNoSlot);
        continue;
      }
      uint32_t hit = kNoSlot;
#pragma unroll
      for (int j = W - 1; j >= 0; --j)
        if (k[u][j] == key[u]) hit = (home[u] + j) & mask;
      if (hit == kNoSlot && (ablate & 1u)) hit = home[u];
      if (hit != kNoSlot)
        finish(i, (sub_table_of(key[u], nsub_log2) << cap_log2) | hit);
      else
        pend |= 1u << u;
    }
    // Round 2: the lane's pending records one at a time -- the wave iterates max-over-lanes
    // times (usually once) instead of once per unrolled record.
    while (pend) {
      const int u = __ffs(pend) - 1;
      pend &= pend - 1;
      uint64_t kk = 0;
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j == u) kk = key[j];
      const uint32_t sub = sub_table_of(kk, nsub_log2);
      const uint32_t sl = probe_insert(keys_g + ((size_t)sub << cap_log2), kk, mask);
      if (sl == kNoSlot) atomicOr(&flags[0], 1u);
      finish(base + u * kHistThreads + threadIdx.x, sl == kNoSlot ? kNoSlot : (sub << cap_log2) | sl);
    }
  }
  __syncthreads();
  uint32_t* out = part + (size_t)blockIdx.x * nslots;
  for (uint32_t s = threadIdx.x; s < nslots; s += kHistThreads) out[s] = hcnt[s];
}

// tot row 0 = the stored counts, row g+1 = group g's total (chunks [16g, 16g+16)).
__global__ __launch_bounds__(256) void rolling_hist_group_kernel(const uint32_t* __restrict__ part,
                                                                 uint32_t nb, uint32_t nslots,
                                                                 const uint32_t* __restrict__ cnt_g,
                                                                 uint32_t* __restrict__ tot) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
  if (s >= nslots) return;
  const uint32_t b0 = g * kGroup, b1 = b0 + kGroup < nb ? b0 + kGroup : nb;
  uint32_t t = 0;
#pragma unroll 4
  for (uint32_t b = b0; b < b1; ++b) t += part[(size_t)b * nslots + s];
  tot[(size_t)(g + 1) * nslots + s] = t;
  if (g == 0) tot[s] = cnt_g[s];
}

// part[b][s] <- stored count + everything of chunks < b (exclusive); the last group writes the
// final counts (it reads tot, not cnt_g, so no other thread's read races the write).
__global__ __launch_bounds__(256) void rolling_hist_prefix_kernel(uint32_t* __restrict__ part,
                                                                  uint32_t nb, uint32_t nslots,
                                                                  const uint32_t* __restrict__ tot,
                                                                  uint32_t* __restrict__ cnt_g,
                                                                  uint64_t* __restrict__ keys_g,
                                                                  int dense) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
  if (s >= nslots) return;
  uint32_t base = 0;
  for (uint32_t r = 0; r <= g; ++r) base += tot[(size_t)r * nslots + s];
  const uint32_t b0 = g * kGroup, b1 = b0 + kGroup < nb ? b0 + kGroup : nb;
  uint32_t p[kGroup];
#pragma unroll
  for (int j = 0; j < kGroup; ++j) p[j] = b0 + j < b1 ? part[(size_t)(b0 + j) * nslots + s] : 0;
#pragma unroll
  for (int j = 0; j < kGroup; ++j) {
    if (b0 + j < b1) part[(size_t)(b0 + j) * nslots + s] = base;
    base += p[j];
  }
  if (g == gridDim.y - 1) {
    cnt_g[s] = base;
    if (dense && base) keys_g[s] = s;  // dense slots hold their own key id
  }
}

// Select path of the emit pass (a filtered counter whose filter passes few counts, e.g.
// `count % 1000 == 0`, config 2): instead of ranking every record of the chunk, find the few
// records whose post-update count passes. Limits of the chunk-local lists (over them, or for a
// slot with more than kSelMaxRun records in the chunk, the chunk takes the ranking path).
constexpr uint32_t kSelSlots = 1024;   // distinct slots with a passing count in the chunk
constexpr uint32_t kSelRecs = 8192;    // records of those slots in the chunk
constexpr uint32_t kSelMaxRun = 512;   // records of one such slot in the chunk
constexpr uint32_t kSelNone = 0xFFFFFFFFu;

__global__ __launch_bounds__(kTile) void rolling_hist_emit_kernel(
    const uint16_t* __restrict__ slot16, uint32_t n, uint32_t chunk,
    const uint32_t* __restrict__ part, uint32_t nslots, const uint64_t* __restrict__ keys_g,
    const uint32_t* __restrict__ cnt_g, ExprProg filt, int need_key, int dense,
    uint64_t* __restrict__ out_key,
    uint64_t* __restrict__ out_val, int64_t* __restrict__ out_tag, uint32_t* __restrict__ out_n,
    uint32_t out_cap, uint32_t ablate) {
  // LDS (<= 160 KB at 16K slots): run[nslots] u32 | owner[nslots] u16 | lane masks
  // m64[2][kTileWaves][kTile] u64, wave-major so a wave's 64 lanes touch 64 different owners'
  // words (owner-major rows would put every owner on the same 4 of the 64 banks).
  // A tile's distinct slots are named without atomics: every record writes its thread id to
  // owner[slot] and, after the barrier, reads back the one write that landed -- the same id for
  // all records of that slot in the tile. Stale owner entries are never read (a slot's entry is
  // written in every tile that reads it), so the array is never cleared.
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* run = lds;
  uint16_t* owner = (uint16_t*)(lds + nslots);
  uint64_t* m64 = (uint64_t*)(lds + nslots + nslots / 2);
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t lo = blockIdx.x * chunk;
  const uint32_t hi = n - lo < chunk ? n : lo + chunk;
  const uint32_t* pre = part + (size_t)blockIdx.x * nslots;
  const uint64_t below = (1ull << lane) - 1ull;
  const ChainRegs chain = decode_chain(filt);
  // The filter on a post-update count of a slot (the rolling epilogue's variables).
  auto passes = [&](uint32_t pcount, uint32_t slot) -> bool {
    if (ablate & 64u) return pcount % 100000u == 0;  // timing reference only
    if (chain.intmode && !(ablate & 128u)) return eval_chain_int(chain, pcount);
    const double key = !need_key ? 0.0 : dense ? (double)slot : (double)keys_g[slot];
    const RollVars rv{(double)pcount, (double)pcount, key, (double)pcount};
    return eval_chain_regs(chain, filt, rv) != 0.0;
  };
  if (filt.ncode && !(ablate & (16u | 256u))) {
    // ---- select path --------------------------------------------------------------------
    // 1. per slot: its records in this chunk take counts pre+1 .. pre+h (h from the next
    //    chunk's prefix); a slot with a passing count among them joins the distinct list.
    // 2. every record of a listed slot drops its chunk-local index into the slot's bucket.
    // 3. a bucket entry's rank = entries of its bucket with a smaller index (buckets are
    //    short): count = pre + rank + 1, emitted when it passes. Rows are unordered (tagged).
    // LDS: aidx[nslots] (over run[]), the lists (over the lane masks).
    uint32_t* aidx = lds;
    uint32_t* L = (uint32_t*)m64;
    uint32_t* dslot = L;
    uint32_t* dlo = L + kSelSlots;
    uint32_t* dh = L + 2 * kSelSlots;
    uint32_t* doff = L + 3 * kSelSlots;
    uint32_t* dfill = L + 4 * kSelSlots;
    uint16_t* bucket = (uint16_t*)(L + 5 * kSelSlots);
    uint16_t* bslot = bucket + kSelRecs;
    uint32_t* sc = L + 5 * kSelSlots + kSelRecs;  // [0] distinct, [1] records, [2] over
    // the chunk's end counts: the next chunk's prefixes, or the slots' totals for the last
    const uint32_t* nxt = blockIdx.x + 1 < gridDim.x ? pre + nslots : cnt_g;
    for (uint32_t s = tid; s < nslots; s += kTile) aidx[s] = kSelNone;
    if (tid < 4) sc[tid] = 0;
    __syncthreads();
    for (uint32_t s = tid; s < nslots; s += kTile) {
      const uint32_t p0 = pre[s];
      const uint32_t p1 = nxt[s];
      const uint32_t h = p1 - p0;
      if (!h) continue;
      if (h > kSelMaxRun) {  // a hot slot: its bucket would be too long to rank by counting
        sc[2] = 1u;
        continue;
      }
      bool any = false;
      for (uint32_t c = p0 + 1; c <= p1 && !any; ++c) any = passes(c, s);
      if (!any) continue;
      const uint32_t d = atomicAdd(&sc[0], 1u);
      const uint32_t at = atomicAdd(&sc[1], h);
      if (d >= kSelSlots || at + h > kSelRecs) {
        sc[2] = 1u;
        continue;
      }
      aidx[s] = d;
      dslot[d] = s;
      dlo[d] = p0;
      dh[d] = h;
      doff[d] = at;
      dfill[d] = 0;
    }
    __syncthreads();
    const bool sel = sc[2] == 0u;
    if (sel) {
      const uint32_t nd = sc[0];
      if (nd) {
        for (uint32_t i = lo + tid; i < hi; i += kTile) {
          const uint32_t slot = slot16[i];
          if (slot == kNoSlot16) continue;
          const uint32_t d = aidx[slot];
          if (d == kSelNone) continue;
          const uint32_t q = doff[d] + atomicAdd(&dfill[d], 1u);
          bucket[q] = (uint16_t)(i - lo);
          bslot[q] = (uint16_t)d;
        }
        __syncthreads();
        const uint32_t nrec = sc[1];
        for (uint32_t base = 0; base < nrec; base += kTile) {  // block-uniform trip count
          const uint32_t e = base + tid;
          bool emit = false;
          uint32_t slot = 0, pcount = 0, li = 0;
          if (e < nrec) {
            const uint32_t d = bslot[e];
            li = bucket[e];
            const uint32_t b0 = doff[d], b1 = b0 + dh[d];
            uint32_t rank = 0;
            for (uint32_t j = b0; j < b1; ++j) rank += bucket[j] < li;
            slot = dslot[d];
            pcount = dlo[d] + rank + 1;
            emit = passes(pcount, slot);
          }
          const unsigned long long m = __ballot(emit);
          if (m) {  // wave-uniform
            uint32_t wb = 0;
            if (lane == 0) wb = atomicAdd(out_n, (uint32_t)__popcll(m));
            wb = __shfl(wb, 0);
            if (emit) {
              const uint32_t q = wb + (uint32_t)__popcll(m & below);
              if (q < out_cap) {
                out_key[q] = dense ? slot : keys_g[slot];
                out_val[q] = pcount;
                out_tag[q] = (int64_t)(lo + li);
              }
            }
          }
        }
      }
      return;  // block-uniform
    }
    __syncthreads();  // the ranking path below reuses the LDS
  }
  for (uint32_t s = tid; s < nslots; s += kTile) run[s] = pre[s];
  for (uint32_t e = tid; e < 2 * kTile * kTileWaves; e += kTile) m64[e] = 0;
  if (!filt.ncode && blockIdx.x == 0 && tid == 0) atomicAdd(out_n, n);  // rows = records
  __syncthreads();
  uint32_t pend_slot = kNoSlot, pend_cnt = 0;  // running-count update of the previous tile
  bool was_owner = false;                        // this thread's masks of the previous tile
  uint32_t buf = 0;
  // One tile: rank the records of [t0, t0 + kTile) (block-uniform call: every thread reaches
  // the barriers). `slot` was loaded a tile earlier.
  auto tile = [&](uint32_t t0, uint32_t slot) {
    const uint32_t i = t0 + tid;
    const bool valid = i < hi && slot != kNoSlot16;
    uint64_t* M = m64 + (size_t)buf * kTile * kTileWaves;
    if (valid) owner[slot] = (uint16_t)((ablate & 4u) ? (slot & (kTile - 1)) : tid);
    __syncthreads();  // A: owners settled; the previous tile's readers are done
    if (pend_slot != kNoSlot) run[pend_slot] = pend_cnt;
    pend_slot = kNoSlot;
    if (was_owner) {  // recycle the previous tile's mask buffer for the tile after this one
      uint64_t* col = m64 + (size_t)(buf ^ 1) * kTile * kTileWaves + tid;
#pragma unroll
      for (int j = 0; j < kTileWaves; ++j) col[j * kTile] = 0;
    }
    uint32_t id = 0;
    if (valid) {
      id = owner[slot];
      if (!(ablate & 8u)) atomicOr((unsigned long long*)&M[(size_t)w * kTile + id], 1ull << lane);
    }
    was_owner = valid && id == tid;
    __syncthreads();  // B: lane masks complete
    bool emit = false;
    uint32_t pcount = 0;
    if (valid) {
      const uint64_t* col = M + id;
      uint64_t r[kTileWaves];
#pragma unroll
      for (int j = 0; j < kTileWaves; ++j) r[j] = (ablate & 32u) ? 0 : col[j * kTile];
      uint32_t before = 0;
      uint64_t later = 0;
#pragma unroll
      for (int j = 0; j < kTileWaves; ++j) {  // compile-time indices only (no scratch array)
        if ((uint32_t)j < w) before += (uint32_t)__popcll(r[j]);
        if ((uint32_t)j == w) {
          before += (uint32_t)__popcll(r[j] & below);
          later |= (r[j] >> lane) >> 1;
        }
        if ((uint32_t)j > w) later |= r[j];
      }
      pcount = run[slot] + before + 1;
      if (!later) {  // last record of this slot in the tile
        pend_slot = slot;
        pend_cnt = pcount;
      }
      emit = !(ablate & 16u);
      if (filt.ncode && !(ablate & 16u)) emit = passes(pcount, slot);
    }
    buf ^= 1;
    if (!filt.ncode) {  // every record emits: its row index is its arrival index (no atomics)
      if (valid && i < out_cap) {
        out_key[i] = dense ? slot : keys_g[slot];
        out_val[i] = pcount;
        out_tag[i] = (int64_t)i;
      }
      return;
    }
    const unsigned long long m = __ballot(emit);
    if (m) {  // wave-uniform
      uint32_t wb = 0;
      if (lane == 0) wb = atomicAdd(out_n, (uint32_t)__popcll(m));
      wb = __shfl(wb, 0);
      if (emit) {
        const uint32_t q = wb + (uint32_t)__popcll(m & below);
        if (q < out_cap) {
          out_key[q] = dense ? slot : keys_g[slot];
          out_val[q] = pcount;
          out_tag[q] = (int64_t)i;  // src 0 << 32 | arrival index
        }
      }
    }
  };
  auto load = [&](uint32_t t0) { return t0 + tid < hi ? (uint32_t)slot16[t0 + tid] : kNoSlot16; };
  // Four tiles per iteration: the next group's slots are loaded before this group's four tiles
  // run, and only the back-edge copy waits for them (four tiles of work later).
  constexpr int G = 4;
  uint32_t cur[G];
#pragma unroll
  for (int j = 0; j < G; ++j) cur[j] = load(lo + j * kTile);
  // Retire the prologue loads here: with them pending on the loop's entry edge the wait-count
  // pass merges that state into the header and waits for every in-flight load each iteration.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  for (uint32_t t0 = lo; t0 < hi; t0 += G * kTile) {  // block-uniform bounds
    uint32_t nxt[G];
#pragma unroll
    for (int j = 0; j < G; ++j) nxt[j] = load(t0 + (G + j) * kTile);
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (t0 + j * kTile < hi) tile(t0 + j * kTile, cur[j]);
#pragma unroll
    for (int j = 0; j < G; ++j) cur[j] = nxt[j];
  }
}

}  // namespace

namespace gpu {

size_t rolling_hist_scratch_bytes(int64_t n, int64_t nslots) {
  const Geo g = geometry((uint32_t)n);
  const size_t words = (size_t)g.nb * nslots + (size_t)(g.ngroups + 1) * nslots;
  return words * 4 + (((size_t)n * 2 + 15) & ~(size_t)15) + 16;
}

bool rolling_hist_supported(int agg, uint32_t count_n, int64_t nslots, const ExprProg& filt) {
  return agg == AGG_COUNT && count_n == 0 && nslots >= 64 && nslots <= kRollHistMaxSlots &&
         (filt.ncode == 0 || filt.chain);
}

void rolling_hist(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2, uint64_t* keys_g,
                  uint32_t* cnt_g, void* scratch, size_t scratch_bytes, const ExprProg& filt,
                  uint64_t* out_key, uint64_t* out_val, int64_t* out_tag, uint32_t* out_n,
                  uint32_t out_cap, uint32_t* flags, int dense, intptr_t stream) {
  const int64_t nslots = (int64_t)1 << (nsub_log2 + cap_log2);
  if (!rolling_hist_supported(AGG_COUNT, 0, nslots, filt))
    throw std::invalid_argument("rolling_hist: state table too large or filter not a chain");
  if (n < 0 || n >= (int64_t)1 << 32) throw std::invalid_argument("rolling_hist: batch size");
  if (n == 0) return;
  if (scratch_bytes < rolling_hist_scratch_bytes(n, nslots))
    throw std::invalid_argument("rolling_hist: scratch buffer too small");
  const Geo g = geometry((uint32_t)n);
  uint32_t* part = (uint32_t*)scratch;
  uint32_t* tot = part + (size_t)g.nb * nslots;
  uint16_t* slot16 = (uint16_t*)(tot + (size_t)(g.ngroups + 1) * nslots);
  int need_key = 0;
  for (int i = 0; i < filt.ncode; ++i)
    if (filt.code[2 * i] == OP_VAR && filt.code[2 * i + 1] == 4) need_key = 1;
  hipStream_t s = (hipStream_t)stream;
  // MXS_RH_ABLATE (timing experiments only; results are wrong when set, except 128 and 256): 1
  // no probe past the home window, 2 no histogram atomics, 4 owner = slot % 512, 8 no lane-mask
  // ORs, 16 no filter evaluation and no rows, 32 no lane-mask reads, 64 filter hard-coded as
  // count % 100000 == 0, 128 no integer-mode chain (f64 evaluation of the decoded chain), 256 no
  // select path (every filtered chunk ranks all its records).
  static const uint32_t ablate = [] {
    const char* e = std::getenv("MXS_RH_ABLATE");
    return e ? (uint32_t)std::strtoul(e, nullptr, 0) : 0u;
  }();
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)rolling_hist_count_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute((const void*)rolling_hist_emit_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const uint32_t ns = (uint32_t)nslots;
  hipLaunchKernelGGL(rolling_hist_count_kernel, dim3(g.nb), dim3(kHistThreads), ns * 4, s, keys,
                     (uint32_t)n, g.chunk, nsub_log2, cap_log2, keys_g, slot16, part, ns, flags,
                     dense, ablate);
  const dim3 sg((ns + 255) / 256, g.ngroups);
  hipLaunchKernelGGL(rolling_hist_group_kernel, sg, dim3(256), 0, s, part, g.nb, ns, cnt_g, tot);
  hipLaunchKernelGGL(rolling_hist_prefix_kernel, sg, dim3(256), 0, s, part, g.nb, ns, tot, cnt_g,
                     keys_g, dense);
  const size_t lds = (size_t)ns * 6 + (size_t)2 * kTile * kTileWaves * 8;  // 160 KB at 16K
  hipLaunchKernelGGL(rolling_hist_emit_kernel, dim3(g.nb), dim3(kTile), lds, s, slot16,
                     (uint32_t)n, g.chunk, part, ns, keys_g, cnt_g, filt, need_key, dense, out_key,
                     out_val, out_tag, out_n, out_cap, ablate);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
