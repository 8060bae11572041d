// mxstream — LDS line tiles for the gfx950 text parse kernels (csrc/ingest_hip.hip,
// csrc/parse_hip.hip).
//
// A parse kernel gives every thread one line. Read straight from HBM, a wave's byte loads touch
// 64 different lines ~48 bytes apart -- every load instruction fans out over dozens of cache
// lines and each line is re-read once per byte, so the parse ran at ~0.2 TB/s. Here a
// 256-thread workgroup owns a tile of 256 consecutive lines; their bytes (one contiguous range
// of the batch) are staged into LDS with coalesced 16-byte loads (one pass over HBM), and every
// thread splits and parses its line from LDS. Tiles whose bytes exceed the LDS budget (very long
// lines) parse from global memory with the same code.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxs {

constexpr int kTileLines = 256;         // lines per workgroup (one per thread)
constexpr int kTileLdsBytes = 24 * 1024;  // up to ~96-byte lines; 6 workgroups per CU fit LDS

// Text in LDS: byte i of the batch lives at p[i - base] for i in the staged range.
struct LdsText {
  const char* p;
  int64_t base;
  __device__ __forceinline__ char operator[](int64_t i) const { return p[i - base]; }
};
__device__ __forceinline__ const char* text_at(const LdsText& t, int64_t i) { return t.p + (i - t.base); }

// Bytes [lo, hi) of `text` fit an LDS tile of `cap` bytes (stage_line_tile's condition).
__device__ __forceinline__ bool tile_fits_lds(const char* text, int64_t lo, int64_t hi, int cap) {
  const int64_t nb = hi - lo;
  const int pad = (int)((uintptr_t)(text + lo) & 15);
  return nb > 0 && nb + pad <= cap;
}

// Stage bytes [lo, hi) of `text` into `lds` (16-byte aligned, cap bytes): unaligned head and
// tail bytes one per thread, the aligned body as 16-byte loads/stores. Returns the LdsText view,
// or p == nullptr when the range does not fit (the caller parses from global memory). Every
// thread of the workgroup must call it (it ends with a barrier).
__device__ __forceinline__ LdsText stage_line_tile(const char* __restrict__ text, int64_t lo,
                                                   int64_t hi, char* lds, int cap) {
  const int64_t nb = hi - lo;
  const int pad = (int)((uintptr_t)(text + lo) & 15);
  if (nb <= 0 || nb + pad > cap) return LdsText{nullptr, lo};
  int head = (16 - pad) & 15;
  if (head > nb) head = (int)nb;
  const int64_t nbody = (nb - head) >> 4;
  const int64_t tail0 = head + (nbody << 4);
  const char* src = text + lo;
  char* dst = lds + pad;
  const int t = threadIdx.x;
  if (t < head) dst[t] = src[t];
  const uint4* s4 = reinterpret_cast<const uint4*>(src + head);
  uint4* d4 = reinterpret_cast<uint4*>(dst + head);  // lds + 16: aligned
  for (int64_t k = t; k < nbody; k += blockDim.x) d4[k] = s4[k];
  if (t < nb - tail0) dst[tail0 + t] = src[tail0 + t];
  __syncthreads();
  return LdsText{dst, lo};
}

}  // namespace mxs
