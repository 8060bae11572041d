// mxstream — device text ingest shared by the gfx950 kernels (csrc/ingest_hip.hip) and their C++
// twins (csrc/ingest_cpu.cpp): split a line, parse its numeric fields with Java semantics and
// describe its string fields for the device string dictionary (reference sites
// Main.java:21-24, ComputeCpuMax.java:20-23, BandwidthMonitor.java:28-30,
// BandwidthMonitorWithEventTime.java:33,39-43).
//
// A batch is parsed in five stream-ordered launches, no host round trip in between:
//   1. ingest_parse   : one thread per line -- numeric columns, and per string field its byte
//                       range, Java hashCode and 64-bit content hash; the hash is inserted into
//                       the dictionary's open-addressed HBM table (CAS on an empty slot) and the
//                       first position of every string not seen before is kept (atomic min);
//   2. new-string mask + the order-preserving compaction of filter_scan / filter_write: the
//      first occurrences of new strings, in (line, field) order;
//   3. dict_assign    : the k-th new string gets id n_ids + k -- the ids are exactly the host
//                       StringDict's (first appearance order over the stream), its bytes are
//                       appended to the arena;
//   4. dict_commit    : n_ids += number of new strings;
//   5. dict_resolve   : every string field gets its slot's id; its bytes are compared with the
//                       arena copy, so two strings with one 64-bit hash are reported (error bit
//                       2), never merged.
// Lines outside the kernel's exact fast paths (a double with more than 15 significant digits,
// NaN / hex / suffixed numbers, malformed fields) are flagged and re-parsed by the host runtime,
// which also produces Java's exception text.
#pragma once
#include <stdint.h>

#include "mxs_common.h"

namespace mxs {

constexpr int kIngestMaxFields = 8;
// Field kinds: csrc/runtime.cpp FieldKind.
constexpr int32_t IK_STR = 0, IK_DOUBLE = 1, IK_LONG = 2, IK_TS_INTSEC = 3, IK_TS_MS = 4,
                  IK_INT = 5, IK_RAW_LONG = 6, IK_ISO_SEC = 7;

struct IngestSpec {
  int32_t nfields;
  int32_t field[kIngestMaxFields];  // split index of output column f
  int32_t kind[kIngestMaxFields];   // IK_*
  int32_t sidx[kIngestMaxFields];   // string field number of column f (-1: numeric)
  int32_t nstr;                     // string columns
  int32_t ts_col;                   // column feeding the batch's max timestamp (-1: none)
  int64_t offset_s;                 // zone offset of ISO date-time fields
  int32_t sep;
};

// Per-batch outputs (n lines, S = nstr, string position p = line * S + s).
struct IngestOut {
  int64_t* cols;      // [nfields][n] numeric columns (f64 as bit patterns); string columns unused
  int32_t* ids;       // [S][n] dictionary ids (dict_resolve), -1 where the field is missing
  uint8_t* status;    // [n] 1: the host parser decides the line
  int64_t* spos;      // [n * S] byte offset of the string field in the batch
  int32_t* slen;      // [n * S] its length (-1: no such field)
  int32_t* sjh;       // [n * S] Java String.hashCode
  int32_t* sslot;     // [n * S] dictionary slot (-1: none)
  uint64_t* shash;    // [n * S] content hash (never 0)
  uint32_t* nflag;    // flagged lines (device counter)
  int64_t* maxts;     // max of column ts_col over the unflagged lines (device, atomic max)
  // [tiles] per-tile maxima reduced by one workgroup after the parse (nullptr: one atomic max
  // per workgroup -- same-address atomics from every workgroup serialise across the XCDs)
  int64_t* tile_max = nullptr;
};

// Device string dictionary: id <-> bytes, plus the Java hash of every id.
struct DictState {
  uint64_t* tab_h;     // [mask + 1] content hash, 0 = empty
  int32_t* tab_id;     // [mask + 1] id, -1 = claimed in this batch, not yet assigned
  int64_t* tab_first;  // [mask + 1] first string position of an unassigned slot (INT64_MAX)
  uint32_t mask;
  int64_t* id_off;     // [id_cap] arena offset of id
  int32_t* id_len;     // [id_cap]
  int32_t* id_jh;      // [id_cap] Java hashCode (key groups of dictionary-id keys)
  uint8_t* arena;
  int64_t arena_cap;
  int64_t id_cap;
  int64_t* ctr;        // [0] ids  [1] arena bytes used  [2] error bits  [3] new ids this batch
};
constexpr int64_t kDictErrFull = 1, kDictErrCollision = 2, kDictErrCapacity = 4;

MXS_HD uint64_t text_hash64(const char* p, int64_t len) {
  uint64_t h = 0xcbf29ce484222325ull ^ (uint64_t)len;
  for (int64_t k = 0; k < len; ++k) h = (h ^ (unsigned char)p[k]) * 0x100000001b3ull;
  h = mix64(h);
  return h ? h : 1ull;
}

MXS_HD uint32_t dict_home(uint64_t h, uint32_t mask) { return (uint32_t)(h >> 17) & mask; }

// Double.parseDouble for the exact Clinger fast path (<= 15 significant digits, |exp10| <= 22):
// m * 10^e is correctly rounded, i.e. bit-identical to strtod; anything else returns false.
MXS_HD bool fast_parse_double(const char* s, int64_t len, double* out) {
  while (len > 0 && (unsigned char)s[0] <= ' ') ++s, --len;  // Java trims chars <= ' '
  while (len > 0 && (unsigned char)s[len - 1] <= ' ') --len;
  if (len <= 0) return false;
  int64_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  uint64_t m = 0;
  int sig = 0, frac = 0;
  bool any = false;
  for (; i < len && s[i] >= '0' && s[i] <= '9'; ++i) {
    any = true;
    if (m == 0 && s[i] == '0') continue;
    if (++sig > 15) return false;
    m = m * 10 + (uint64_t)(s[i] - '0');
  }
  if (i < len && s[i] == '.') {
    ++i;
    for (; i < len && s[i] >= '0' && s[i] <= '9'; ++i) {
      any = true;
      ++frac;
      if (m == 0 && s[i] == '0') continue;
      if (++sig > 15) return false;
      m = m * 10 + (uint64_t)(s[i] - '0');
    }
  }
  if (!any) return false;
  int e = 0;
  if (i < len && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < len && (s[i] == '+' || s[i] == '-')) eneg = s[i++] == '-';
    int ne = 0;
    for (; i < len && s[i] >= '0' && s[i] <= '9'; ++i) {
      if (++ne > 4) return false;
      e = e * 10 + (s[i] - '0');
    }
    if (ne == 0) return false;
    if (eneg) e = -e;
  }
  if (i != len) return false;  // suffix (d/f), NaN, Infinity, hex, junk: the host decides
  e -= frac;
  if (e < -22 || e > 22) return false;
  double p10 = 1.0;
  for (int k = 0; k < (e < 0 ? -e : e); ++k) p10 *= 10.0;  // exact: 10^22 < 2^53 * 2^22
  double v = (double)m;  // exact: m < 10^15 < 2^53
  v = e >= 0 ? v * p10 : v / p10;
  *out = neg ? -v : v;
  return true;
}

MXS_HD const char* text_at(const char* t, int64_t i) { return t + i; }

// One line [a, b) of `text` (no '\n', trailing '\r' already dropped). Returns 1 when the host
// must decide the line. Numeric columns are written at row li; string fields are described at
// positions li * nstr + s (the dictionary probe follows in the caller). `text` is the batch in
// global memory, or its LDS tile (csrc/line_tile.h LdsText: same absolute positions).
template <class Text>
MXS_HD uint8_t ingest_line(Text text, int64_t a, int64_t b, int64_t li, int64_t n,
                           const IngestSpec& sp, const IngestOut& o, int64_t* ts_val) {
  // Field boundaries of the requested split indices (Java String.split: trailing empty fields
  // are dropped, "" splits to [""]).
  int64_t fs[kIngestMaxFields], fe[kIngestMaxFields];
#pragma unroll
  for (int f = 0; f < kIngestMaxFields; ++f) fs[f] = fe[f] = -1;
  int idx = 0;
  int64_t cur = a, last_nonempty = -1;
  const char sep = (char)sp.sep;
  for (int64_t pos = a; pos <= b; ++pos) {
    if (pos == b || text[pos] == sep) {
#pragma unroll
      for (int f = 0; f < kIngestMaxFields; ++f)
        if (f < sp.nfields && sp.field[f] == idx) {
          fs[f] = cur;
          fe[f] = pos;
        }
      if (pos > cur) last_nonempty = idx;
      ++idx;
      cur = pos + 1;
    }
  }
  const int64_t nfields_java = a == b ? 1 : last_nonempty + 1;
  uint8_t st = 0;
#pragma unroll
  for (int f = 0; f < kIngestMaxFields; ++f) {
    if (f >= sp.nfields) continue;
    const bool present = sp.field[f] < nfields_java && fs[f] >= 0;
    const int32_t kind = sp.kind[f];
    if (kind == IK_STR) {
      const int64_t p = li * sp.nstr + sp.sidx[f];
      if (!present) {
        o.slen[p] = -1;
        st = 1;  // ArrayIndexOutOfBounds: the host reports it
        continue;
      }
      const char* q = text_at(text, fs[f]);
      const int64_t len = fe[f] - fs[f];
      o.spos[p] = fs[f];
      o.slen[p] = (int32_t)len;
      o.sjh[p] = java_hash_utf8(q, len);
      o.shash[p] = text_hash64(q, len);
      continue;
    }
    if (!present) {
      st = 1;
      continue;
    }
    const char* q = text_at(text, fs[f]);
    const int64_t len = fe[f] - fs[f];
    int64_t* out = o.cols + (int64_t)f * n + li;
    int64_t v = 0;
    bool ok = true;
    switch (kind) {
      case IK_DOUBLE: {
        double d;
        ok = fast_parse_double(q, len, &d);
        v = (int64_t)f64_bits(d);
        break;
      }
      case IK_LONG:
      case IK_RAW_LONG:
        ok = parse_long_ascii(q, len, INT64_MIN, INT64_MAX, &v) == 0;
        break;
      case IK_INT:
        ok = parse_long_ascii(q, len, INT32_MIN, INT32_MAX, &v) == 0;
        break;
      case IK_TS_INTSEC:
      case IK_TS_MS:
      case IK_ISO_SEC: {
        int64_t es = 0, ms = 0;
        ok = iso_local_datetime(q, len, sp.offset_s, &es, &ms);
        v = kind == IK_TS_MS ? es * 1000 + ms
            : kind == IK_ISO_SEC ? (int64_t)(int32_t)(uint32_t)(uint64_t)es
                                 : (int64_t)(int32_t)(uint32_t)(uint64_t)es * 1000;  // (int) quirk
        break;
      }
      default: ok = false;
    }
    if (!ok) {
      st = 1;
      continue;
    }
    *out = v;
    if (f == sp.ts_col) *ts_val = v;
  }
  return st;
}

}  // namespace mxs
