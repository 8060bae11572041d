// mxstream — C++ twins of the device text ingest (csrc/ingest_hip.hip): the same per-line code
// (csrc/ingest.h), the same dictionary table and the same id assignment (first occurrence in
// (line, field) order), so the CPU engine and the GPU produce identical columns and ids, and the
// device ingest path of the DataStream API is tested on machines without a GPU.
#include <cstring>
#include <stdexcept>

#include "ingest.h"
#include "mxs_kernels.h"

namespace mxs {
namespace cpu {

void line_starts(const uint8_t* buf, int64_t n, int64_t* idx, int64_t* total) {
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i)
    if (i == 0 || buf[i - 1] == (uint8_t)'\n') idx[k++] = i;
  *total = k;
}

static int32_t probe_insert(const DictState& d, uint64_t h) {
  uint32_t q = dict_home(h, d.mask);
  for (uint32_t i = 0; i <= d.mask; ++i) {
    if (d.tab_h[q] == h) return (int32_t)q;
    if (d.tab_h[q] == 0) {
      d.tab_h[q] = h;
      return (int32_t)q;
    }
    q = (q + 1) & d.mask;
  }
  return -1;
}

void ingest_parse(const char* text, int64_t text_len, const int64_t* starts, int64_t n,
                  const IngestSpec& sp, const IngestOut& o, const DictState& d) {
  if (sp.nfields < 1 || sp.nfields > kIngestMaxFields) throw std::invalid_argument("ingest: fields");
  for (int64_t li = 0; li < n; ++li) {
    const int64_t a = starts[li];
    int64_t b = li + 1 < n ? starts[li + 1] - 1 : text_len;
    if (b > text_len) b = text_len;
    if (b > a && text[b - 1] == '\n') --b;
    if (b > a && text[b - 1] == '\r') --b;
    int64_t ts = INT64_MIN;
    const uint8_t st = ingest_line(text, a, b, li, n, sp, o, &ts);
    o.status[li] = st;
    *o.nflag += st;
    if (!st && ts > *o.maxts) *o.maxts = ts;
    for (int s = 0; s < sp.nstr; ++s) {
      const int64_t p = li * sp.nstr + s;
      int32_t slot = -1;
      if (o.slen[p] >= 0) {
        slot = probe_insert(d, o.shash[p]);
        if (slot < 0) d.ctr[2] |= kDictErrFull;
        else if (d.tab_id[slot] < 0 && d.tab_first[slot] > p) d.tab_first[slot] = p;
      }
      o.sslot[p] = slot;
    }
  }
}

void dict_find_new(int64_t n, int32_t nstr, const IngestOut& o, const DictState& d,
                   int64_t* newpos) {
  const int64_t np = n * nstr;
  int64_t k = 0;
  for (int64_t p = 0; p < np; ++p) {
    const int32_t s = o.sslot[p];
    if (s >= 0 && d.tab_id[s] < 0 && d.tab_first[s] == p) newpos[k++] = p;
  }
  d.ctr[3] = k;
}

void dict_resolve(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                  const DictState& d) {
  const int64_t np = n * nstr;
  for (int64_t p = 0; p < np; ++p) {
    const int32_t s = o.sslot[p];
    int32_t id = -1;
    if (s >= 0) {
      id = d.tab_id[s];
      const bool same = id >= 0 && d.id_len[id] == o.slen[p] &&
                        std::memcmp(text + o.spos[p], d.arena + d.id_off[id], (size_t)o.slen[p]) == 0;
      if (!same) {
        d.ctr[2] |= kDictErrCollision;
        id = -1;
      }
    }
    const int64_t li = p / nstr, si = p - li * nstr;
    o.ids[si * n + li] = id;
  }
}

void dict_insert_ids(const uint8_t* buf, const int64_t* offs, const int32_t* lens, int64_t k,
                     int64_t id0, const DictState& d) {
  d.ctr[0] = id0 + k;
  for (int64_t i = 0; i < k; ++i) {
    const char* str = (const char*)buf + offs[i];
    const int32_t len = lens[i];
    const int32_t slot = probe_insert(d, text_hash64(str, len));
    const int64_t id = id0 + i;
    if (slot < 0 || id >= d.id_cap || d.ctr[1] + len > d.arena_cap) {
      d.ctr[2] |= slot < 0 ? kDictErrFull : kDictErrCapacity;
      continue;
    }
    const int64_t off = d.ctr[1];
    d.ctr[1] += len;
    std::memcpy(d.arena + off, str, (size_t)len);
    d.id_off[id] = off;
    d.id_len[id] = len;
    d.id_jh[id] = java_hash_utf8(str, len);
    d.tab_first[slot] = INT64_MAX;
    d.tab_id[slot] = (int32_t)id;
  }
}

void dict_assign_new(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                     const DictState& d, int64_t* newpos) {
  const int64_t np = n * nstr;
  dict_find_new(n, nstr, o, d, newpos);
  const int64_t k = d.ctr[3];
  const int64_t n_ids = d.ctr[0];
  for (int64_t j = 0; j < k; ++j) {
    const int64_t p = newpos[j];
    const int32_t s = o.sslot[p];
    const int64_t id = n_ids + j;
    const int32_t len = o.slen[p];
    if (id >= d.id_cap || d.ctr[1] + len > d.arena_cap) {
      d.ctr[2] |= kDictErrCapacity;
      continue;
    }
    const int64_t off = d.ctr[1];
    d.ctr[1] += len;
    std::memcpy(d.arena + off, text + o.spos[p], (size_t)len);
    d.id_off[id] = off;
    d.id_len[id] = len;
    d.id_jh[id] = o.sjh[p];
    d.tab_first[s] = INT64_MAX;
    d.tab_id[s] = (int32_t)id;
  }
  d.ctr[0] += k;
  (void)np;
  dict_resolve(text, n, nstr, o, d);
}

void dict_rehash(const uint64_t* old_h, const int32_t* old_id, int64_t old_cap, const DictState& d) {
  for (int64_t i = 0; i < old_cap; ++i) {
    if (old_h[i] == 0 || old_id[i] < 0) continue;
    const int32_t q = probe_insert(d, old_h[i]);
    if (q >= 0) d.tab_id[q] = old_id[i];
  }
}

namespace {
struct ColVarsCpu {
  const int64_t* cols;
  int64_t n, row;
  int32_t nf, dbl_mask;
  double get(int j) const {
    if (j >= nf) return 0.0;
    const int64_t v = cols[(int64_t)j * n + row];
    return ((dbl_mask >> j) & 1) ? as_f64((uint64_t)v) : (double)v;
  }
};
}  // namespace

void ingest_filter_compact(const int64_t* cols, int64_t n, int32_t nf, int32_t dbl_mask,
                           const ExprProg& prog, int64_t* idx, int64_t* total) {
  int64_t k = 0;
  LocalStack st;
  for (int64_t i = 0; i < n; ++i) {
    ColVarsCpu v{cols, n, i, nf, dbl_mask};
    if (expr_eval_t(prog, st, v) != 0.0) idx[k++] = i;
  }
  *total = k;
}

void ingest_gather(const int64_t* cols, int64_t n, int32_t nf, const int32_t* ids, int32_t nstr,
                   const int64_t* idx, const int64_t* total, int64_t* out_cols, int32_t* out_ids,
                   int64_t out_stride) {
  const int64_t m = *total < n ? *total : n;
  for (int64_t k = 0; k < m; ++k) {
    const int64_t r = idx[k];
    for (int f = 0; f < nf; ++f) out_cols[(int64_t)f * out_stride + k] = cols[(int64_t)f * n + r];
    for (int s = 0; s < nstr; ++s) out_ids[(int64_t)s * out_stride + k] = ids[(int64_t)s * n + r];
  }
}

}  // namespace cpu
}  // namespace mxs
