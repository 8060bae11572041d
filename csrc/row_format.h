// mxstream — print() rows formatted where the columns live (SURVEY.md F-print).
//
// A keyed operator's columnar emit (the rolling max of ComputeCpuMax.java:26 prints one line per
// input record) used to be copied to the host column by column and formatted there by threads;
// at ~30 bytes a line the formatting itself bounds the job. The same Java text -- subtask prefix
// "N> ", Tuple.toString "(f0,f1,...)", String / Long.toString / Double.toString fields -- is
// produced here by one lane per row: a length pass, a scan, a write pass, then ONE copy of the
// finished bytes. The functions are shared by the gfx950 kernels (csrc/format_hip.hip) and the
// host twin (csrc/kernels_cpu.cpp), so tests/test_row_format.py checks them on the CPU against
// the host formatter (csrc/javafmt.h).
//
// Double.toString is exact here for values with at most 15 significant digits in plain notation
// (1e-3 <= |x| < 1e7; parsed metrics such as "91.5"): the shortest decimal c / 10^k with
// c < 10^15 that rounds to x is unique (decimals of <= 15 digits are farther apart than a
// double's rounding interval), rint(x * 10^k) finds it (the product's error is far below 1/2),
// and the correctly rounded division c / 10^k == x verifies it. Any other double -- 16-17
// digits, scientific notation -- flags the batch, and the caller formats that batch on the
// host instead.
#pragma once
#include <cstdint>

#include "mxs_common.h"

namespace mxs {

constexpr int kFmtMaxCols = 8;

struct FmtCol {
  int32_t kind;   // 0 = dictionary id (string), 1 = f64, 2 = integer
  int32_t width;  // bytes of an id / integer element: 4 or 8
  const void* p;
};

struct FmtArgs {
  int32_t ncols, as_tuple;
  FmtCol col[kFmtMaxCols];
  const uint8_t* arena;    // dictionary bytes; string id s is arena[id_off[s], + id_len[s])
  const int64_t* id_off;
  const int32_t* id_len;
  int64_t n_ids;
  const int32_t* sub;      // per-row subtask, or null: (sub0 + row) % par
  int64_t sub0;
  int32_t par;
  int32_t npfx;            // prefix k = pfx[pfx_off[k], pfx_off[k + 1]); npfx == 0: none
  const char* pfx;
  const int32_t* pfx_off;
};

MXS_HD int fmt_u64(uint64_t v, char* out) {  // decimal digits of v; out may be null
  char tmp[20];
  int n = 0;
  do {
    tmp[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  if (out)
    for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
  return n;
}

MXS_HD int fmt_long(int64_t v, char* out) {
  if (v < 0) {
    if (out) *out++ = '-';
    return 1 + fmt_u64(0ull - (uint64_t)v, out);
  }
  return fmt_u64((uint64_t)v, out);
}

MXS_HD int fmt_copy(const char* s, int n, char* out) {
  if (out)
    for (int i = 0; i < n; ++i) out[i] = s[i];
  return n;
}

// Java Double.toString of x, or -1 when x needs the host formatter (see the header comment).
MXS_HD int fmt_double(double x, char* out) {
  if (x != x) return fmt_copy("NaN", 3, out);
  const uint64_t bits = __builtin_bit_cast(uint64_t, x);
  const bool neg = bits >> 63;
  const double ax = neg ? -x : x;
  if (ax == 0.0) return neg ? fmt_copy("-0.0", 4, out) : fmt_copy("0.0", 3, out);
  if (ax > 1.7976931348623157e308) return neg ? fmt_copy("-Infinity", 9, out)
                                              : fmt_copy("Infinity", 8, out);
  if (!(ax >= 1e-3 && ax < 1e7)) return -1;
  double p = 1.0;
  for (int k = 0; k <= 18; ++k, p *= 10.0) {  // 10^k is exact for k <= 22
    const double y = ax * p;
    if (y >= 1e15) return -1;
    const double c = __builtin_rint(y);
    if (c / p != ax) continue;
    // c / 10^k: integer part, '.', k fraction digits (at least one: "x.0")
    const uint64_t ci = (uint64_t)c;
    uint64_t pk = 1;
    for (int j = 0; j < k; ++j) pk *= 10;
    const uint64_t ip = ci / pk, fp = ci % pk;
    int n = 0;
    if (neg) {
      if (out) out[n] = '-';
      ++n;
    }
    n += fmt_u64(ip, out ? out + n : nullptr);
    if (out) out[n] = '.';
    ++n;
    if (k == 0) {
      if (out) out[n] = '0';
      return n + 1;
    }
    for (int j = k - 1; j >= 0; --j) {  // zero-padded fraction digits, most significant first
      uint64_t d = fp;
      for (int q = 0; q < j; ++q) d /= 10;
      if (out) out[n] = (char)('0' + d % 10);
      ++n;
    }
    return n;
  }
  return -1;
}

// Row i as Java prints it, newline included; out may be null (length only). ok = false when a
// field needs the host formatter or a string id / subtask lies outside its table.
MXS_HD int fmt_row(const FmtArgs& a, int64_t i, char* out, bool& ok) {
  int n = 0;
  if (a.npfx) {
    int64_t s = a.sub ? (int64_t)a.sub[i] : (a.sub0 + i) % (a.par > 0 ? a.par : 1);
    if (s < 0 || s >= a.npfx) {
      ok = false;
      s = 0;
    }
    const int32_t o = a.pfx_off[s];
    n += fmt_copy(a.pfx + o, a.pfx_off[s + 1] - o, out);
  }
  if (a.as_tuple) {
    if (out) out[n] = '(';
    ++n;
  }
  for (int j = 0; j < a.ncols; ++j) {
    if (j) {
      if (out) out[n] = ',';
      ++n;
    }
    const FmtCol& c = a.col[j];
    char* w = out ? out + n : nullptr;
    if (c.kind == 0) {
      const int64_t id = c.width == 4 ? (int64_t)((const int32_t*)c.p)[i] : ((const int64_t*)c.p)[i];
      if (id < 0 || id >= a.n_ids) {
        ok = false;
        continue;
      }
      n += fmt_copy((const char*)a.arena + a.id_off[id], a.id_len[id], w);
    } else if (c.kind == 1) {
      const int d = fmt_double(((const double*)c.p)[i], w);
      if (d < 0) {
        ok = false;
        continue;
      }
      n += d;
    } else {
      const int64_t v = c.width == 4 ? (int64_t)((const int32_t*)c.p)[i] : ((const int64_t*)c.p)[i];
      n += fmt_long(v, w);
    }
  }
  if (a.as_tuple) {
    if (out) out[n] = ')';
    ++n;
  }
  if (out) out[n] = '\n';
  return n + 1;
}

}  // namespace mxs
