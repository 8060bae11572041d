// mxstream — keyed-state invariant checker: GPU kernel (check_hip.hip) and C++
// twin (check_cpu.cpp) over the open-addressing slot tables every keyed operator uses.
//
// For every live slot s of sub-table `sub` holding key k:
//   * placement : k belongs to this sub-table (sub_table_of(k) == sub; partition rule);
//   * chain     : linear probing from k's home slot (slot_hash(k) & mask) reaches s without passing
//                 an empty slot (otherwise lookups of k would stop early and re-insert it);
//   * unique    : no slot between the home slot and s holds k (a duplicate live key).
// Tombstones (session tables) count as occupied for the chain rule, as in the probe loops.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "mxs_common.h"

namespace mxs {

// kTombKey (mxs_common.h): session tables' deleted-slot marker

enum CheckStat { kChkLive = 0, kChkMisplaced = 1, kChkBrokenChain = 2, kChkDuplicate = 3, kChkN = 4 };

// Violations of one live slot (bit 0 misplaced, 1 broken chain, 2 duplicate).
MXS_HD uint32_t check_slot(const uint64_t* keys, uint32_t s, uint32_t mask, int nsub_log2,
                           uint32_t sub) {
  const uint64_t k = keys[s];
  uint32_t bad = 0;
  if (nsub_log2 > 0 && sub_table_of(k, nsub_log2) != sub) bad |= 1u;
  uint32_t i = slot_hash(k) & mask;
  for (uint32_t step = 0; step <= mask && i != s; ++step) {
    const uint64_t x = keys[i];
    if (x == kEmptyKey) {
      bad |= 2u;
      break;
    }
    if (x == k) {
      bad |= 4u;
      break;
    }
    i = (i + 1) & mask;
  }
  return bad;
}

namespace gpu {
void check_table(const uint64_t* keys_g, int nsub, int nsub_log2, int cap_log2, uint64_t* stats,
                 intptr_t stream);
// out[0] = min(out[0], min(x[0..n))) (caller initialises out[0]); used by the native pipeline
// for the first step's pane base.
void min_i64(const int64_t* x, int64_t n, int64_t* out, intptr_t stream);
}
namespace cpu {
// C++ twin (header-only so the sanitizer harness links it without the Python bindings).
inline void check_table(const uint64_t* keys_g, int nsub, int nsub_log2, int cap_log2,
                        uint64_t* stats) {
  const uint32_t cap = 1u << cap_log2, mask = cap - 1;
  for (int sub = 0; sub < nsub; ++sub) {
    const uint64_t* keys = keys_g + ((size_t)sub << cap_log2);
    for (uint32_t s = 0; s < cap; ++s) {
      const uint64_t k = keys[s];
      if (k == kEmptyKey || k == kTombKey) continue;
      ++stats[kChkLive];
      const uint32_t bad = check_slot(keys, s, mask, nsub_log2, (uint32_t)sub);
      stats[kChkMisplaced] += bad & 1u;
      stats[kChkBrokenChain] += (bad >> 1) & 1u;
      stats[kChkDuplicate] += (bad >> 2) & 1u;
    }
  }
}
}  // namespace cpu

}  // namespace mxs
