// mxstream — vector-metric keyed windows: plans and launchers (GPU: vector_hip.hip, CPU twin:
// vector_cpu.cpp).
//
// Per (key, pane) f32 sums of D-float metric vectors, state acc[ring][slot][D] next to the usual
// keys[slot] / cnt[ring][slot] / dirty[ring][slot] of the scalar window operator. The records
// come from the regular keyBy partition pass with val = the event's row in the batch (G = 1), or,
// after the G > 1 exchange of records and vectors, the record's position (positional mode).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "mxs_kernels.h"

namespace mxs {

struct VecAggPlan {
  int32_t cap_log2;     // slots per sub-table (2^6 .. 2^12)
  int32_t nsub;
  int32_t ring;
  int32_t dim;          // D: multiple of 32, <= 256
  int32_t nsrc;
  uint32_t bucket_cap;
  int32_t np_step;
  int32_t positional;   // 0: vector row = record.val; 1: vector row = record position
  int32_t rec_words;    // 2 (RecC) or 3 (Rec)
  int32_t mode;         // GPU: 0 = MFMA segmented sum, 1 = VALU segmented sum (A/B only)
  int64_t pane_base;
  int64_t p_lo;
  int64_t fired_hi;
};

struct VecFirePlan {
  int32_t dim;
  int32_t npanes;
  int32_t ring;
  int32_t only_dirty;
  int32_t avg;          // 1: result = sum / count
  int32_t use_thr;      // 1: emit only windows whose max metric result > thr
  float thr;
  int64_t nslots;
  int64_t p0;
  uint32_t out_cap;
};

// Synthetic metric value d of event `row` (shared by the GPU generator and its CPU twin).
MXS_HD float gen_vector_value(uint64_t seed, uint64_t stream_id, uint64_t row, int d, float lo,
                              float span) {
  const uint64_t x = rng64(seed ^ 0x5EC7ull, stream_id, row * 1024u + (uint64_t)d);
  return lo + span * (float)((double)(x >> 40) * (1.0 / 16777216.0));
}

namespace gpu {
size_t vec_window_agg_lds(int cap_log2);
void vec_window_agg(const void* recs, const uint32_t* counts, const VecAggPlan& p,
                    const float* vec, uint64_t* keys_g, float* acc_g, uint32_t* cnt_g,
                    uint8_t* dirty_g, uint32_t* occupancy, uint32_t* flags, intptr_t stream);
void vec_window_fire(const uint64_t* keys_g, const float* acc_g, const uint32_t* cnt_g,
                     const uint8_t* dirty_g, const VecFirePlan& p, uint64_t* out_keys,
                     float* out_vec, uint32_t* out_cnt, uint32_t* out_n, intptr_t stream);
void gen_vectors(float* vec, int64_t n, int dim, uint64_t seed, uint64_t stream_id, uint64_t idx0,
                 float lo, float span, intptr_t stream);
void vec_gather(const void* recs, int rec_words, const uint32_t* counts, int nb, uint32_t bcap,
                const float* vec, int dim, float* out, intptr_t stream);
}  // namespace gpu

namespace cpu {
void vec_window_agg(const void* recs, const uint32_t* counts, const VecAggPlan& p,
                    const float* vec, uint64_t* keys_g, float* acc_g, uint32_t* cnt_g,
                    uint8_t* dirty_g, uint32_t* occupancy, uint32_t* flags);
void vec_window_fire(const uint64_t* keys_g, const float* acc_g, const uint32_t* cnt_g,
                     const uint8_t* dirty_g, const VecFirePlan& p, uint64_t* out_keys,
                     float* out_vec, uint32_t* out_cnt, uint32_t* out_n);
void gen_vectors(float* vec, int64_t n, int dim, uint64_t seed, uint64_t stream_id, uint64_t idx0,
                 float lo, float span);
void vec_gather(const void* recs, int rec_words, const uint32_t* counts, int nb, uint32_t bcap,
                const float* vec, int dim, float* out);
}  // namespace cpu

}  // namespace mxs
