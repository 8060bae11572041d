// mxstream — CPU twins of the vector-metric window kernels (csrc/vector_hip.hip). Same state
// layout and record formats as the GPU; sums are f32 in arrival order (the GPU sums the same
// values in (pane, slot)-sorted order, so results agree up to f32 rounding).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "mxs_vector.h"

namespace mxs {
namespace cpu {

namespace {
inline void load_vrec(const void* base, size_t idx, int rec_words, uint64_t& key, uint32_t& val,
                      uint32_t& t) {
  if (rec_words == 2) {
    const RecC r = ((const RecC*)base)[idx];
    key = r.key;
    val = r.val;
    t = r.t;
  } else {
    const Rec r = ((const Rec*)base)[idx];
    key = r.key;
    val = (uint32_t)r.val;
    t = r.t;
  }
}

inline uint32_t vprobe(uint64_t* keys, uint64_t key, uint32_t mask, bool* inserted) {
  uint32_t s = slot_hash(key) & mask;
  for (uint32_t i = 0; i <= mask; ++i) {
    const uint64_t k = keys[s];
    if (k == key) return s;
    if (k == kEmptyKey) {
      keys[s] = key;
      *inserted = true;
      return s;
    }
    s = (s + 1) & mask;
  }
  return kNoSlot;
}
}  // namespace

void vec_window_agg(const void* recs, const uint32_t* counts, const VecAggPlan& p,
                    const float* vec, uint64_t* keys_g, float* acc_g, uint32_t* cnt_g,
                    uint8_t* dirty_g, uint32_t* occupancy, uint32_t* flags) {
  const uint32_t cap = 1u << p.cap_log2, mask = cap - 1;
  const size_t nslots = (size_t)p.nsub << p.cap_log2;
  const int D = p.dim;
  for (int sub = 0; sub < p.nsub; ++sub) {
    uint64_t* keys = keys_g + ((size_t)sub << p.cap_log2);
    bool inserted = false;
    for (int src = 0; src < p.nsrc; ++src) {
      const uint32_t c = std::min(counts[(size_t)src * p.nsub + sub], p.bucket_cap);
      const size_t seg0 = ((size_t)src * p.nsub + sub) * p.bucket_cap;
      for (uint32_t e = 0; e < c; ++e) {
        uint64_t key;
        uint32_t val, t;
        load_vrec(recs, seg0 + e, p.rec_words, key, val, t);
        if (t == 0xFFFFFFFFu) continue;
        const int64_t q = (int64_t)t - p.p_lo;
        if (q < 0 || q >= p.np_step) continue;
        const uint32_t s = vprobe(keys, key, mask, &inserted);
        if (s == kNoSlot) {
          flags[0] |= 1u;
          continue;
        }
        const int64_t pane = p.pane_base + (int64_t)t;
        const size_t gi = (size_t)(pane & (p.ring - 1)) * nslots + ((size_t)sub << p.cap_log2) + s;
        const size_t row = p.positional ? seg0 + e : (size_t)val;
        const float* v = vec + row * D;
        float* a = acc_g + gi * D;
        for (int d = 0; d < D; ++d) a[d] += v[d];
        cnt_g[gi] += 1;
        if (pane <= p.fired_hi) dirty_g[gi] = 1;
      }
    }
    if (inserted) {
      uint32_t occ = 0;
      for (uint32_t i = 0; i < cap; ++i) occ += keys[i] != kEmptyKey;
      occupancy[sub] = occ;
    }
  }
}

void vec_window_fire(const uint64_t* keys_g, const float* acc_g, const uint32_t* cnt_g,
                     const uint8_t* dirty_g, const VecFirePlan& p, uint64_t* out_keys,
                     float* out_vec, uint32_t* out_cnt, uint32_t* out_n) {
  const int D = p.dim;
  std::vector<float> res(D);
  uint32_t n = *out_n;
  for (int64_t s = 0; s < p.nslots; ++s) {
    if (keys_g[s] == kEmptyKey) continue;
    uint32_t cnt = 0;
    bool dirty = false;
    std::fill(res.begin(), res.end(), 0.0f);
    for (int q = 0; q < p.npanes; ++q) {
      const size_t gi = (size_t)((p.p0 + q) & (p.ring - 1)) * p.nslots + s;
      if (!cnt_g[gi]) continue;
      cnt += cnt_g[gi];
      if (dirty_g[gi]) dirty = true;
      for (int d = 0; d < D; ++d) res[d] += acc_g[gi * D + d];
    }
    if (!cnt || (p.only_dirty && !dirty)) continue;
    float mx = -INFINITY;
    for (int d = 0; d < D; ++d) {
      if (p.avg) res[d] = res[d] / (float)cnt;
      mx = std::max(mx, res[d]);
    }
    if (p.use_thr && !(mx > p.thr)) continue;
    if (n < p.out_cap) {
      out_keys[n] = keys_g[s];
      out_cnt[n] = cnt;
      std::memcpy(out_vec + (size_t)n * D, res.data(), sizeof(float) * D);
    }
    ++n;
  }
  *out_n = n;
}

void gen_vectors(float* vec, int64_t n, int dim, uint64_t seed, uint64_t stream_id, uint64_t idx0,
                 float lo, float span) {
  for (int64_t i = 0; i < n; ++i)
    for (int d = 0; d < dim; ++d)
      vec[i * dim + d] = gen_vector_value(seed, stream_id, idx0 + (uint64_t)i, d, lo, span);
}

void vec_gather(const void* recs, int rec_words, const uint32_t* counts, int nb, uint32_t bcap,
                const float* vec, int dim, float* out) {
  for (int b = 0; b < nb; ++b) {
    const uint32_t c = std::min(counts[b], bcap);
    for (uint32_t e = 0; e < c; ++e) {
      const size_t j = (size_t)b * bcap + e;
      uint64_t key;
      uint32_t row, t;
      load_vrec(recs, j, rec_words, key, row, t);
      if (t == 0xFFFFFFFFu) continue;
      std::memcpy(out + j * dim, vec + (size_t)row * dim, sizeof(float) * dim);
    }
  }
}

}  // namespace cpu
}  // namespace mxs
