// mxstream — device pane arena of `process` (list-state) windows: ComputeCpuMiddle.java:34-48
// keeps every element of a (key, window) and hands the Iterable to the window function. Here the
// elements live per pane (pane = gcd(size, slide)) in device append buffers; a firing gathers
// the window's panes with a counting sort by dense key id (histogram -> scan -> scatter, no
// comparison sort) and the per-key median is selected per segment (segment_median_select).
//
// Kernels (csrc/listwin_hip.hip) and their C++ twins (csrc/listwin_cpu.cpp):
//   lw_pane_count    elements per ring slot of the batch (+ late count in slot `ring`)
//   lw_pane_scatter  append the batch's elements to their pane buffers (cursor per slot)
//   lw_key_count     elements per key over a window's panes
//   lw_scan          counts -> exclusive offsets, and the ascending list of non-empty keys with
//                    their segment starts (order-preserving; tiles + one-workgroup tile scan)
//   lw_key_scatter   values of the window's panes into their key segments as f64 order bits
#pragma once
#include <cstdint>

#include "mxs_common.h"

namespace mxs {

// One pane of a window: device (or host) buffers of its `len` elements.
struct LwPane {
  const int64_t* keys;
  const uint64_t* vals;  // f64 bit patterns
  int64_t len;
};

constexpr int kLwMaxPanes = 64;      // panes per window in one launch
constexpr int kLwScanTile = 4096;    // keys per scan tile
constexpr int kLwMaxRing = 4096;     // ring slots of the pane arena

struct LwPanes {
  LwPane p[kLwMaxPanes];
  int32_t n;
};

// Arena targets of a batch scatter: a table (device memory for the GPU launch) of 5 * ring
// words -- [r] the key buffer of ring slot r, [ring + r] its value buffer, [2 ring + r] its
// per-element rank buffer (u32), [3 ring + r] its per-key element counts (u32, over the slot's
// key range), [4 ring + r] the first key of that range -- and a fill cursor per slot. The
// append records each element's rank among its key's elements in the pane (the atomic count),
// so a firing places every element without atomics: segment start + earlier panes' counts of
// the key + rank. A slot with a null count array (key range too wide) records no ranks.

// One pane of a ranked firing.
struct LwRankPane {
  const int64_t* keys;
  const uint64_t* vals;
  const uint32_t* ranks;
  const uint32_t* counts;  // per key of [kbase, kbase + ksize)
  int64_t kbase, ksize, len;
};
constexpr int kLwMaxRankPanes = 32;
struct LwRankPanes {
  LwRankPane p[kLwMaxRankPanes];
  int32_t n;
};

namespace gpu {
void lw_pane_count(const int64_t* ts, int64_t n, int64_t offset, int64_t pane, int ring,
                   int64_t late_ts, int64_t* counts, intptr_t stream);
void lw_pane_scatter(const int64_t* keys, const int64_t* ts, const uint64_t* vals, int64_t n,
                     int64_t offset, int64_t pane, int ring, int64_t late_ts, const int64_t* tab,
                     int64_t* cursor, intptr_t stream);
void lw_key_count(const LwPanes& w, int64_t kmin, int64_t nkeys, uint32_t* counts,
                  intptr_t stream);
int64_t lw_scan_scratch_bytes(int64_t nkeys);
void lw_scan(const uint32_t* counts, int64_t nkeys, int64_t kmin, void* scratch, int64_t* offs,
             int64_t* heads, int64_t* head_keys, int64_t* nheads, intptr_t stream);
void lw_key_scatter(const LwPanes& w, int64_t kmin, int64_t* cursor, uint64_t* out_ord,
                    intptr_t stream);
// Ranked firing: total per-key counts of the window and each pane's prefix (pre[j * nkeys + k]),
// then the placement scatter.
void lw_rank_prefix(const LwRankPanes& w, int64_t kmin, int64_t nkeys, uint32_t* total,
                    uint32_t* pre, intptr_t stream);
void lw_rank_scatter(const LwRankPanes& w, int64_t kmin, int64_t nkeys, const int64_t* offs,
                     const uint32_t* pre, uint64_t* out_ord, intptr_t stream);
}  // namespace gpu

namespace cpu {
void lw_pane_count(const int64_t* ts, int64_t n, int64_t offset, int64_t pane, int ring,
                   int64_t late_ts, int64_t* counts);
void lw_pane_scatter(const int64_t* keys, const int64_t* ts, const uint64_t* vals, int64_t n,
                     int64_t offset, int64_t pane, int ring, int64_t late_ts, const int64_t* tab,
                     int64_t* cursor);
void lw_key_count(const LwPanes& w, int64_t kmin, int64_t nkeys, uint32_t* counts);
void lw_scan(const uint32_t* counts, int64_t nkeys, int64_t kmin, int64_t* offs, int64_t* heads,
             int64_t* head_keys, int64_t* nheads);
void lw_key_scatter(const LwPanes& w, int64_t kmin, int64_t* cursor, uint64_t* out_ord);
void lw_rank_prefix(const LwRankPanes& w, int64_t kmin, int64_t nkeys, uint32_t* total,
                    uint32_t* pre);
void lw_rank_scatter(const LwRankPanes& w, int64_t kmin, int64_t nkeys, const int64_t* offs,
                     const uint32_t* pre, uint64_t* out_ord);
}  // namespace cpu

// Java floorDiv for the pane of a timestamp.
MXS_HD int64_t lw_floor_div(int64_t a, int64_t b) {
  const int64_t q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

}  // namespace mxs
