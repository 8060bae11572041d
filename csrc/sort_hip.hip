// mxstream — device radix sort of (64-bit key, 64-bit value) pairs over a bit range (gfx950).
//
// The keyed-state passes (rolling on hashed / large key spaces, the session fold's fallback, the
// kernels.sort_pairs op) order a step's records by (slot, arrival or event time). Sorting the
// value column along with the key and only over the bits in use (slot bits + time bits, ~35 of
// 64) avoids both a 64-bit sort and a permutation gather.
//
// Hand-written LSD radix sort, 8-bit digits, three launches per digit pass:
//   1. radix_hist    : one 256-thread workgroup per 4096-key tile; every wave splits its 64 keys
//                      into digit peer groups with 8 ballots (no per-key LDS atomics, so a
//                      constant digit -- the top pass over partly used bits -- costs the same as
//                      a uniform one); group leaders add the group size to the tile's LDS
//                      histogram, written digit-major: hist[digit][tile].
//   2. radix_scan    : one workgroup per digit scans that digit's row over the tiles (exclusive)
//                      and writes the digit total.
//   3. radix_scatter : the tile again, in memory order (wave, item, lane): the same ballot split
//                      ranks every key inside its wave and digit (running per-wave digit counts
//                      in LDS keep the order stable), the per-wave counts are prefixed across the
//                      tile's waves, keys are placed in LDS in sorted order and written out as
//                      contiguous per-digit runs at digit prefix + tile offset; the values follow
//                      through the same LDS positions.
// Stable (equal digits keep their input order in every pass), so the passes compose into a
// stable sort of the selected bits. Buffers ping-pong between the output and the temporary so
// that the last pass lands in the output; the input is never written.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "mxs_kernels.h"

namespace mxs {
namespace gpu {
namespace {

constexpr int kRadixBits = 8;
constexpr int kBins = 1 << kRadixBits;
constexpr int kSortBlock = 256;                       // 4 waves of 64
constexpr int kSortWaves = kSortBlock / 64;
constexpr int kItems = 16;                            // keys per thread
constexpr int kTile = kSortBlock * kItems;            // 4096 keys per workgroup
constexpr int kWaveSpan = 64 * kItems;                // a wave's contiguous 1024 keys

#define SORT_CHECK(x)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess)                                                                      \
      throw std::runtime_error(std::string("radix sort: ") + hipGetErrorString(e_));          \
  } while (0)

__device__ __forceinline__ uint32_t sort_lane() { return threadIdx.x & 63u; }

// Lanes of the wave holding the same digit as this lane (restricted to `valid` lanes).
__device__ __forceinline__ uint64_t digit_peers(uint32_t dig, int nb, uint64_t valid) {
  uint64_t peers = valid;
  for (int b = 0; b < nb; ++b) {
    const bool bit = (dig >> b) & 1u;
    const uint64_t bb = __ballot(bit);
    peers &= bit ? bb : ~bb;
  }
  return peers;
}

__global__ __launch_bounds__(kSortBlock) void radix_hist_kernel(
    const uint64_t* __restrict__ keys, uint32_t n, int shift, int nb,
    uint32_t* __restrict__ hist, uint32_t ntiles) {
  __shared__ uint32_t h[kBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = sort_lane(), w = threadIdx.x >> 6;
  const uint32_t mask = (1u << nb) - 1u;
  const uint32_t base = blockIdx.x * kTile + w * kWaveSpan;
  uint64_t k[kItems];
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const uint32_t i = base + j * 64 + lane;
    k[j] = i < n ? keys[i] : 0;
  }
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const uint32_t i = base + j * 64 + lane;
    const bool valid = i < n;
    const uint64_t vm = __ballot(valid);
    if (!vm) break;  // wave-uniform
    const uint32_t dig = (uint32_t)(k[j] >> shift) & mask;
    const uint64_t peers = digit_peers(dig, nb, vm);
    if (valid && (peers & ((1ull << lane) - 1ull)) == 0)
      atomicAdd(&h[dig], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix, *total the sum.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave,
                                                         uint32_t* total) {
  const uint32_t lane = sort_lane(), w = threadIdx.x >> 6;
  uint32_t incl = v;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) s_wave[w] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kSortWaves; ++i) {
    const uint32_t c = s_wave[i];
    before += (uint32_t)i < w ? c : 0u;
    all += c;
  }
  __syncthreads();  // s_wave may be reused by the caller
  *total = all;
  return before + incl - v;
}

__global__ __launch_bounds__(kSortBlock) void radix_scan_kernel(uint32_t* __restrict__ hist,
                                                                uint32_t ntiles,
                                                                uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_wave[kSortWaves];
  uint32_t* row = hist + (size_t)blockIdx.x * ntiles;
  const uint32_t per = (ntiles + kSortBlock - 1) / kSortBlock;
  const uint32_t lo = threadIdx.x * per;
  const uint32_t hi = lo + per < ntiles ? lo + per : ntiles;
  uint32_t run = 0;
  for (uint32_t i = lo; i < hi; ++i) run += row[i];
  uint32_t total;
  uint32_t o = block_exclusive_scan(run, s_wave, &total);
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = row[i];
    row[i] = o;
    o += c;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = total;
}

__global__ __launch_bounds__(kSortBlock) void radix_scatter_kernel(
    const uint64_t* __restrict__ kin, const uint64_t* __restrict__ vin,
    uint64_t* __restrict__ kout, uint64_t* __restrict__ vout, uint32_t n, int shift, int nb,
    const uint32_t* __restrict__ hist, uint32_t ntiles, const uint32_t* __restrict__ totals) {
  __shared__ uint64_t buf[kTile];                 // keys, then values, in tile-sorted order
  __shared__ uint32_t wcnt[kSortWaves][kBins];    // per-wave running digit counts -> offsets
  __shared__ uint32_t gbase[kBins];               // global position of tile-local position 0
  __shared__ uint32_t tstart[kBins];              // tile-local start of every digit
  __shared__ uint32_t s_wave[kSortWaves];
  const uint32_t lane = sort_lane(), w = threadIdx.x >> 6, t = threadIdx.x;
  const uint32_t mask = (1u << nb) - 1u;
  const uint32_t tile0 = blockIdx.x * kTile;
  const uint32_t base = tile0 + w * kWaveSpan;
#pragma unroll
  for (int q = 0; q < kSortWaves; ++q) wcnt[q][t] = 0;
  uint64_t k[kItems];
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const uint32_t i = base + j * 64 + lane;
    k[j] = i < n ? kin[i] : 0;
  }
  __syncthreads();
  uint16_t pos[kItems];
  uint8_t dg[kItems];
  // Stable rank inside (wave, digit): keys of one wave are visited in memory order (item j, then
  // lane), and the wave's running digit count is read before its group leader bumps it (LDS
  // operations of one wave complete in issue order).
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const uint32_t i = base + j * 64 + lane;
    const bool valid = i < n;
    const uint64_t vm = __ballot(valid);
    const uint32_t dig = (uint32_t)(k[j] >> shift) & mask;
    uint32_t r = 0;
    if (vm) {
      const uint64_t peers = digit_peers(dig, nb, vm);
      const uint64_t lt = peers & ((1ull << lane) - 1ull);
      const uint32_t before = valid ? wcnt[w][dig] : 0u;
      if (valid && lt == 0) wcnt[w][dig] = before + (uint32_t)__popcll(peers);
      r = before + (uint32_t)__popcll(lt);
    }
    pos[j] = (uint16_t)r;
    dg[j] = (uint8_t)dig;
  }
  __syncthreads();
  // Thread t = digit t: per-wave counts -> exclusive offsets across the tile's waves, the digit's
  // tile count -> tile-local start (block scan), global base from the digit prefix and the tile's
  // offset inside the digit's row.
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < kSortWaves; ++q) {
    const uint32_t c = wcnt[q][t];
    wcnt[q][t] = cnt;
    cnt += c;
  }
  uint32_t tile_total;
  const uint32_t ts = block_exclusive_scan(cnt, s_wave, &tile_total);
  uint32_t all;
  const uint32_t dpre = block_exclusive_scan(totals[t], s_wave, &all);
  tstart[t] = ts;
  gbase[t] = dpre + hist[(size_t)t * ntiles + blockIdx.x] - ts;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const uint32_t i = base + j * 64 + lane;
    if (i < n) {
      const uint32_t p = tstart[dg[j]] + wcnt[w][dg[j]] + pos[j];
      buf[p] = k[j];
      pos[j] = (uint16_t)p;
    }
  }
  __syncthreads();
  // Sorted positions q = t + 256 * r leave in order; each thread keeps its positions' global
  // destinations for the value pass (registers instead of a per-position digit array in LDS:
  // 4 KB less LDS, one more workgroup per CU).
  const uint32_t m = n - tile0 < (uint32_t)kTile ? n - tile0 : (uint32_t)kTile;
  uint32_t dst[kItems];
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
    const uint32_t q = t + r * kSortBlock;
    dst[r] = 0;
    if (q < m) {
      const uint64_t key = buf[q];
      dst[r] = gbase[(uint32_t)(key >> shift) & mask] + q;
      kout[dst[r]] = key;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const uint32_t i = base + j * 64 + lane;
    if (i < n) buf[pos[j]] = vin[i];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
    const uint32_t q = t + r * kSortBlock;
    if (q < m) vout[dst[r]] = buf[q];
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline int num_passes(int begin_bit, int end_bit) {
  return (end_bit - begin_bit + kRadixBits - 1) / kRadixBits;
}

}  // namespace

size_t sort_pairs_temp_bytes(int64_t n, int begin_bit, int end_bit) {
  // The kernels index in uint32 (tile base + in-tile offset): the last tile must end below 2^32.
  if (n < 0 || n > ((int64_t)1 << 32) - kTile) throw std::invalid_argument("sort_pairs: n out of range");
  if (begin_bit < 0 || end_bit > 64 || begin_bit >= end_bit)
    throw std::invalid_argument("sort_pairs: bad bit range");
  const size_t ntiles = (size_t)((n + kTile - 1) / kTile);
  size_t bytes = align256(ntiles * kBins * 4) + align256(kBins * 4);
  if (num_passes(begin_bit, end_bit) > 1) bytes += 2 * align256((size_t)n * 8);
  return bytes;
}

void sort_pairs(void* temp, size_t temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                const uint64_t* vals_in, uint64_t* vals_out, int64_t n, int begin_bit, int end_bit,
                intptr_t stream) {
  if (n <= 0) return;
  const size_t need = sort_pairs_temp_bytes(n, begin_bit, end_bit);
  if (need > temp_bytes) throw std::runtime_error("sort_pairs: temporary buffer too small");
  if (keys_in == keys_out || vals_in == vals_out)
    throw std::invalid_argument("sort_pairs: input and output must differ");
  const hipStream_t s = (hipStream_t)stream;
  const uint32_t un = (uint32_t)n;
  const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
  char* p = static_cast<char*>(temp);
  uint32_t* hist = reinterpret_cast<uint32_t*>(p);
  p += align256((size_t)ntiles * kBins * 4);
  uint32_t* totals = reinterpret_cast<uint32_t*>(p);
  p += align256(kBins * 4);
  uint64_t* tk = reinterpret_cast<uint64_t*>(p);
  uint64_t* tv = reinterpret_cast<uint64_t*>(p + align256((size_t)n * 8));
  const int passes = num_passes(begin_bit, end_bit);
  const uint64_t* src_k = keys_in;
  const uint64_t* src_v = vals_in;
  for (int ps = 0; ps < passes; ++ps) {
    const int shift = begin_bit + ps * kRadixBits;
    const int nb = end_bit - shift < kRadixBits ? end_bit - shift : kRadixBits;
    // The last pass writes the output; earlier passes alternate so that holds.
    const bool to_out = ((passes - 1 - ps) & 1) == 0;
    uint64_t* dk = to_out ? keys_out : tk;
    uint64_t* dv = to_out ? vals_out : tv;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(ntiles), dim3(kSortBlock), 0, s, src_k, un, shift,
                       nb, hist, ntiles);
    hipLaunchKernelGGL(radix_scan_kernel, dim3(kBins), dim3(kSortBlock), 0, s, hist, ntiles,
                       totals);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(ntiles), dim3(kSortBlock), 0, s, src_k, src_v,
                       dk, dv, un, shift, nb, hist, ntiles, totals);
    src_k = dk;
    src_v = dv;
  }
  SORT_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
