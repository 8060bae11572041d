// mxstream — pane arena and counting-sort firing of `process` (list-state) windows on gfx950
// (declarations and the design: csrc/mxs_listwin.h; C++ twins: csrc/listwin_cpu.cpp).
//
// ComputeCpuMiddle.java:34-48 keeps every element of a (host, 1-min window) and takes the
// median. The elements of a batch are appended to their pane's device buffer (block-aggregated
// cursors: one global atomic per touched pane per workgroup). A firing counts the window's
// elements per dense key id, scans the counts (order-preserving, so segments come out in key
// order) and scatters the values into their key segments as order bits; the per-segment median
// selection (segment_median_select, csrc/kernels_hip.hip) never needs a comparison sort of the
// whole window.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "mxs_listwin.h"

namespace mxs {
namespace {

#define LW_CHECK(x)                                                                         \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                  \
  } while (0)

int grid_of(int64_t n, int per_block, int cap) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

__device__ __forceinline__ int lw_slot(int64_t t, int64_t offset, int64_t pane, int ring,
                                       int64_t late_ts) {
  if (t < late_ts) return ring;  // late: dropped (counted in the extra bin)
  return (int)(lw_floor_div(t - offset, pane) & (int64_t)(ring - 1));
}

constexpr int kLwBlock = 256;
constexpr int kLwItems = 16;  // elements per thread per tile (4096-element tiles)

__global__ __launch_bounds__(kLwBlock) void lw_pane_count_kernel(const int64_t* __restrict__ ts,
                                                                 int64_t n, int64_t offset,
                                                                 int64_t pane, int ring,
                                                                 int64_t late_ts,
                                                                 int64_t* __restrict__ counts) {
  extern __shared__ uint32_t hist[];  // ring + 1 bins
  for (int i = threadIdx.x; i <= ring; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&hist[lw_slot(ts[i], offset, pane, ring, late_ts)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i <= ring; i += blockDim.x)
    if (hist[i]) atomicAdd((unsigned long long*)&counts[i], (unsigned long long)hist[i]);
}

// A tile of kLwBlock * kLwItems elements: LDS counts per ring slot -> one global cursor atomic
// per touched slot -> every element's position = slot base + its LDS rank.
__global__ __launch_bounds__(kLwBlock) void lw_pane_scatter_kernel(
    const int64_t* __restrict__ keys, const int64_t* __restrict__ ts,
    const uint64_t* __restrict__ vals, int64_t n, int64_t offset, int64_t pane, int ring,
    int64_t late_ts, const int64_t* __restrict__ tab, int64_t* __restrict__ cursor) {
  extern __shared__ uint32_t sm[];
  uint32_t* cnt = sm;                                         // ring + 1
  unsigned long long* base = (unsigned long long*)(sm + ((ring + 2) & ~1));  // ring
  const int64_t tile = (int64_t)kLwBlock * kLwItems;
  for (int64_t t0 = (int64_t)blockIdx.x * tile; t0 < n; t0 += (int64_t)gridDim.x * tile) {
    for (int i = threadIdx.x; i <= ring; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    int slot[kLwItems];
#pragma unroll
    for (int u = 0; u < kLwItems; ++u) {
      const int64_t i = t0 + (int64_t)u * kLwBlock + threadIdx.x;
      slot[u] = i < n ? lw_slot(ts[i], offset, pane, ring, late_ts) : ring;
      if (i < n && slot[u] < ring) atomicAdd(&cnt[slot[u]], 1u);
    }
    __syncthreads();
    for (int r = threadIdx.x; r < ring; r += blockDim.x) {
      const uint32_t c = cnt[r];
      base[r] = c ? atomicAdd((unsigned long long*)&cursor[r], (unsigned long long)c) : 0ull;
      cnt[r] = 0;  // reused as the tile's rank cursor
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kLwItems; ++u) {
      const int64_t i = t0 + (int64_t)u * kLwBlock + threadIdx.x;
      if (i < n && slot[u] < ring) {
        const int r = slot[u];
        const unsigned long long pos = base[r] + atomicAdd(&cnt[r], 1u);
        const int64_t key = keys[i];
        reinterpret_cast<int64_t*>(tab[r])[pos] = key;
        reinterpret_cast<uint64_t*>(tab[ring + r])[pos] = vals[i];
        uint32_t* kc = reinterpret_cast<uint32_t*>(tab[3 * ring + r]);
        if (kc)  // rank of the element among its key's elements of this pane
          reinterpret_cast<uint32_t*>(tab[2 * ring + r])[pos] =
              atomicAdd(&kc[key - tab[4 * ring + r]], 1u);
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kLwBlock) void lw_key_count_kernel(LwPanes w, int64_t kmin,
                                                                uint32_t* __restrict__ counts) {
  const LwPane& p = w.p[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.len;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&counts[p.keys[i] - kmin], 1u);
}

__global__ __launch_bounds__(kLwBlock) void lw_key_scatter_kernel(LwPanes w, int64_t kmin,
                                                                  int64_t* __restrict__ cursor,
                                                                  uint64_t* __restrict__ out) {
  const LwPane& p = w.p[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.len;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long pos =
        atomicAdd((unsigned long long*)&cursor[p.keys[i] - kmin], 1ull);
    out[pos] = f64_order_bits(p.vals[i]);
  }
}

// Per key of the window: the panes' counts -> each pane's prefix and the total.
__global__ __launch_bounds__(kLwBlock) void lw_rank_prefix_kernel(LwRankPanes w, int64_t kmin,
                                                                  int64_t nkeys,
                                                                  uint32_t* __restrict__ total,
                                                                  uint32_t* __restrict__ pre) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t key = kmin + k;
    uint32_t run = 0;
    for (int j = 0; j < w.n; ++j) {
      const LwRankPane& p = w.p[j];
      const int64_t o = key - p.kbase;
      pre[(int64_t)j * nkeys + k] = run;
      run += (o >= 0 && o < p.ksize) ? p.counts[o] : 0u;
    }
    total[k] = run;
  }
}

// Placement without atomics: segment start + earlier panes' count of the key + rank.
__global__ __launch_bounds__(kLwBlock) void lw_rank_scatter_kernel(LwRankPanes w, int64_t kmin,
                                                                   int64_t nkeys,
                                                                   const int64_t* __restrict__ offs,
                                                                   const uint32_t* __restrict__ pre,
                                                                   uint64_t* __restrict__ out) {
  const LwRankPane& p = w.p[blockIdx.y];
  const uint32_t* pj = pre + (int64_t)blockIdx.y * nkeys;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.len;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = p.keys[i] - kmin;
    out[offs[k] + pj[k] + p.ranks[i]] = f64_order_bits(p.vals[i]);
  }
}

// ---- order-preserving scan of the key counts ---------------------------------------------
// Block-wide exclusive scan of one value per thread (1024 threads): wave shuffles + wave totals.
template <class T>
__device__ __forceinline__ T block_excl_scan(T v, T* wsum, T* total) {
  T incl = v;
  for (int d = 1; d < 64; d <<= 1) {
    const T y = __shfl_up(incl, d);
    if ((int)(threadIdx.x & 63) >= d) incl += y;
  }
  const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 63) wsum[wv] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    T t = 0;
    for (int i = 0; i < nw; ++i) {
      const T c = wsum[i];
      wsum[i] = t;
      t += c;
    }
    *total = t;
  }
  __syncthreads();
  const T r = wsum[wv] + incl - v;
  __syncthreads();
  return r;
}

constexpr int kScanThreads = 1024;
constexpr int kScanPer = kLwScanTile / kScanThreads;  // 4 keys per thread

// Pass 1: per tile, the element total and the number of non-empty keys.
__global__ __launch_bounds__(kScanThreads) void lw_tile_sums_kernel(
    const uint32_t* __restrict__ counts, int64_t nkeys, uint64_t* __restrict__ tsum,
    uint32_t* __restrict__ tne) {
  __shared__ uint64_t ws[16];
  __shared__ uint32_t wn[16];
  __shared__ uint64_t tot;
  __shared__ uint32_t totn;
  const int64_t k0 = (int64_t)blockIdx.x * kLwScanTile + (int64_t)threadIdx.x * kScanPer;
  uint64_t s = 0;
  uint32_t ne = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    const uint32_t c = k0 + j < nkeys ? counts[k0 + j] : 0u;
    s += c;
    ne += c ? 1u : 0u;
  }
  block_excl_scan<uint64_t>(s, ws, &tot);
  block_excl_scan<uint32_t>(ne, wn, &totn);
  if (threadIdx.x == 0) {
    tsum[blockIdx.x] = tot;
    tne[blockIdx.x] = totn;
  }
}

// Pass 2 (one workgroup): exclusive scan of the tile totals (<= kScanThreads * 4 tiles).
__global__ __launch_bounds__(kScanThreads) void lw_tile_scan_kernel(uint64_t* __restrict__ tsum,
                                                                    uint32_t* __restrict__ tne,
                                                                    int64_t ntiles,
                                                                    int64_t* __restrict__ offs_end,
                                                                    int64_t nkeys,
                                                                    int64_t* __restrict__ nheads) {
  __shared__ uint64_t ws[16];
  __shared__ uint32_t wn[16];
  __shared__ uint64_t tot;
  __shared__ uint32_t totn;
  const int64_t t0 = (int64_t)threadIdx.x * 4;
  uint64_t s[4];
  uint32_t e[4];
  uint64_t ss = 0;
  uint32_t se = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s[j] = t0 + j < ntiles ? tsum[t0 + j] : 0ull;
    e[j] = t0 + j < ntiles ? tne[t0 + j] : 0u;
    ss += s[j];
    se += e[j];
  }
  uint64_t bs = block_excl_scan<uint64_t>(ss, ws, &tot);
  uint32_t be = block_excl_scan<uint32_t>(se, wn, &totn);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (t0 + j < ntiles) {
      tsum[t0 + j] = bs;
      tne[t0 + j] = be;
    }
    bs += s[j];
    be += e[j];
  }
  if (threadIdx.x == 0) {
    offs_end[nkeys] = (int64_t)tot;
    *nheads = (int64_t)totn;
  }
}

// Pass 3: per tile, exclusive offsets of every key and the (start, key) of non-empty keys in
// key order.
__global__ __launch_bounds__(kScanThreads) void lw_tile_write_kernel(
    const uint32_t* __restrict__ counts, int64_t nkeys, int64_t kmin,
    const uint64_t* __restrict__ tsum, const uint32_t* __restrict__ tne, int64_t* __restrict__ offs,
    int64_t* __restrict__ heads, int64_t* __restrict__ head_keys) {
  __shared__ uint64_t ws[16];
  __shared__ uint32_t wn[16];
  __shared__ uint64_t tot;
  __shared__ uint32_t totn;
  const int64_t k0 = (int64_t)blockIdx.x * kLwScanTile + (int64_t)threadIdx.x * kScanPer;
  uint32_t c[kScanPer];
  uint64_t s = 0;
  uint32_t ne = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    c[j] = k0 + j < nkeys ? counts[k0 + j] : 0u;
    s += c[j];
    ne += c[j] ? 1u : 0u;
  }
  uint64_t o = tsum[blockIdx.x] + block_excl_scan<uint64_t>(s, ws, &tot);
  uint32_t h = tne[blockIdx.x] + block_excl_scan<uint32_t>(ne, wn, &totn);
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    if (k0 + j < nkeys) {
      offs[k0 + j] = (int64_t)o;
      if (c[j]) {
        heads[h] = (int64_t)o;
        head_keys[h] = kmin + k0 + j;
        ++h;
      }
    }
    o += c[j];
  }
}

}  // namespace

namespace gpu {

void lw_pane_count(const int64_t* ts, int64_t n, int64_t offset, int64_t pane, int ring,
                   int64_t late_ts, int64_t* counts, intptr_t stream) {
  if (n <= 0) return;
  if (ring < 1 || ring > kLwMaxRing || (ring & (ring - 1)))
    throw std::invalid_argument("lw_pane_count: ring must be a power of two <= 4096");
  const size_t lds = sizeof(uint32_t) * (size_t)(ring + 1);
  hipLaunchKernelGGL(lw_pane_count_kernel, dim3(grid_of(n, kLwBlock * 16, 2048)), dim3(kLwBlock),
                     lds, (hipStream_t)stream, ts, n, offset, pane, ring, late_ts, counts);
  LW_CHECK(hipGetLastError());
}

void lw_pane_scatter(const int64_t* keys, const int64_t* ts, const uint64_t* vals, int64_t n,
                     int64_t offset, int64_t pane, int ring, int64_t late_ts, const int64_t* tab,
                     int64_t* cursor, intptr_t stream) {
  if (n <= 0) return;
  if (ring < 1 || ring > kLwMaxRing || (ring & (ring - 1)))
    throw std::invalid_argument("lw_pane_scatter: ring must be a power of two <= 4096");
  const size_t lds = sizeof(uint32_t) * (size_t)((ring + 2) & ~1) + sizeof(uint64_t) * ring;
  hipLaunchKernelGGL(lw_pane_scatter_kernel, dim3(grid_of(n, kLwBlock * kLwItems, 4096)),
                     dim3(kLwBlock), lds, (hipStream_t)stream, keys, ts, vals, n, offset, pane,
                     ring, late_ts, tab, cursor);
  LW_CHECK(hipGetLastError());
}

void lw_key_count(const LwPanes& w, int64_t kmin, int64_t nkeys, uint32_t* counts,
                  intptr_t stream) {
  if (w.n <= 0 || w.n > kLwMaxPanes) throw std::invalid_argument("lw_key_count: 1..64 panes");
  (void)nkeys;
  int64_t mx = 0;
  for (int i = 0; i < w.n; ++i) mx = w.p[i].len > mx ? w.p[i].len : mx;
  if (mx <= 0) return;
  hipLaunchKernelGGL(lw_key_count_kernel, dim3(grid_of(mx, kLwBlock * 8, 4096), w.n),
                     dim3(kLwBlock), 0, (hipStream_t)stream, w, kmin, counts);
  LW_CHECK(hipGetLastError());
}

int64_t lw_scan_scratch_bytes(int64_t nkeys) {
  const int64_t nt = (nkeys + kLwScanTile - 1) / kLwScanTile;
  return nt * (int64_t)(sizeof(uint64_t) + sizeof(uint32_t)) + 64;
}

void lw_scan(const uint32_t* counts, int64_t nkeys, int64_t kmin, void* scratch, int64_t* offs,
             int64_t* heads, int64_t* head_keys, int64_t* nheads, intptr_t stream) {
  if (nkeys <= 0) throw std::invalid_argument("lw_scan: empty key range");
  const int64_t nt = (nkeys + kLwScanTile - 1) / kLwScanTile;
  if (nt > (int64_t)kScanThreads * 4)
    throw std::invalid_argument("lw_scan: more than 16 Mi keys");
  uint64_t* tsum = reinterpret_cast<uint64_t*>(scratch);
  uint32_t* tne = reinterpret_cast<uint32_t*>(tsum + nt);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(lw_tile_sums_kernel, dim3(nt), dim3(kScanThreads), 0, s, counts, nkeys, tsum,
                     tne);
  hipLaunchKernelGGL(lw_tile_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, tsum, tne, nt, offs,
                     nkeys, nheads);
  hipLaunchKernelGGL(lw_tile_write_kernel, dim3(nt), dim3(kScanThreads), 0, s, counts, nkeys,
                     kmin, tsum, tne, offs, heads, head_keys);
  LW_CHECK(hipGetLastError());
}

void lw_key_scatter(const LwPanes& w, int64_t kmin, int64_t* cursor, uint64_t* out_ord,
                    intptr_t stream) {
  if (w.n <= 0 || w.n > kLwMaxPanes) throw std::invalid_argument("lw_key_scatter: 1..64 panes");
  int64_t mx = 0;
  for (int i = 0; i < w.n; ++i) mx = w.p[i].len > mx ? w.p[i].len : mx;
  if (mx <= 0) return;
  hipLaunchKernelGGL(lw_key_scatter_kernel, dim3(grid_of(mx, kLwBlock * 8, 4096), w.n),
                     dim3(kLwBlock), 0, (hipStream_t)stream, w, kmin, cursor, out_ord);
  LW_CHECK(hipGetLastError());
}

void lw_rank_prefix(const LwRankPanes& w, int64_t kmin, int64_t nkeys, uint32_t* total,
                    uint32_t* pre, intptr_t stream) {
  if (w.n <= 0 || w.n > kLwMaxRankPanes) throw std::invalid_argument("lw_rank_prefix: 1..32 panes");
  if (nkeys <= 0) return;
  hipLaunchKernelGGL(lw_rank_prefix_kernel, dim3(grid_of(nkeys, kLwBlock, 4096)), dim3(kLwBlock),
                     0, (hipStream_t)stream, w, kmin, nkeys, total, pre);
  LW_CHECK(hipGetLastError());
}

void lw_rank_scatter(const LwRankPanes& w, int64_t kmin, int64_t nkeys, const int64_t* offs,
                     const uint32_t* pre, uint64_t* out_ord, intptr_t stream) {
  if (w.n <= 0 || w.n > kLwMaxRankPanes) throw std::invalid_argument("lw_rank_scatter: 1..32 panes");
  int64_t mx = 0;
  for (int i = 0; i < w.n; ++i) mx = w.p[i].len > mx ? w.p[i].len : mx;
  if (mx <= 0) return;
  hipLaunchKernelGGL(lw_rank_scatter_kernel, dim3(grid_of(mx, kLwBlock * 8, 4096), w.n),
                     dim3(kLwBlock), 0, (hipStream_t)stream, w, kmin, nkeys, offs, pre, out_ord);
  LW_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
