// mxstream — GPU text parsing: split delimited lines and parse their fields.
//
// Reference sites: Main.java:21-24 (split(" ") + Double.parseDouble), BandwidthMonitor.java:28-30
// (Long.parseLong), BandwidthMonitorWithEventTime.java:33,39-43 (ISO LocalDateTime at +08:00).
//
// One thread per line (lines are ~30-60 bytes; a wave covers 64 lines, loads are byte-granular
// but the whole batch is streamed once from HBM). Field semantics are Java's, shared with the host
// runtime through mxs_common.h (parse_long_ascii, iso_local_datetime); doubles take the exact
// Clinger fast path (<= 15 significant digits, |exp10| <= 22: m * 10^e is correctly rounded, so
// the result is bit-identical to strtod / Double.parseDouble). Any line the kernel cannot decide
// exactly -- a long mantissa, NaN/Infinity/hex/suffixed doubles, non-ASCII text in a key, a
// malformed field -- is flagged (status 1) and re-parsed by the C++ runtime on the host, which
// also produces Java's exception text for real errors.
//
// String fields become a 64-bit FNV-1a key plus the Java String.hashCode (ASCII == UTF-16 code
// units), which is what keyBy's key-group assignment needs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "line_tile.h"
#include "mxs_common.h"
#include "mxs_kernels.h"

namespace mxs {
namespace {

constexpr int kMaxFields = 8;
constexpr int FK_STR = 0, FK_DOUBLE = 1, FK_LONG = 2, FK_TS_INTSEC = 3, FK_TS_MS = 4, FK_INT = 5,
              FK_RAW_LONG = 6;

struct ParseSpec {
  int32_t nfields;
  int32_t field[kMaxFields];
  int32_t kind[kMaxFields];
  int64_t offset_s;
  char sep;
};

__device__ __forceinline__ bool fast_double(const char* s, int64_t len, double* out) {
  // Java trims chars <= ' ' around the number.
  while (len > 0 && (unsigned char)s[0] <= ' ') ++s, --len;
  while (len > 0 && (unsigned char)s[len - 1] <= ' ') --len;
  if (len <= 0) return false;
  int64_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  uint64_t m = 0;
  int nd = 0, sig = 0, frac = 0;
  bool any = false;
  for (; i < len && s[i] >= '0' && s[i] <= '9'; ++i) {
    any = true;
    if (m == 0 && s[i] == '0') continue;  // leading zeros are not significant
    if (++sig > 15) return false;
    m = m * 10 + (uint64_t)(s[i] - '0');
    ++nd;
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
  if (i != len) return false;  // suffix (d/f), NaN, Infinity, hex, junk: host decides
  // Trailing fraction zeros were counted as significant digits above only if after a nonzero;
  // the exponent accounts for every fraction digit.
  e -= frac;
  if (e < -22 || e > 22) return false;
  static constexpr double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                     1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                     1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  double v = (double)m;  // exact: m < 10^15 < 2^53
  v = e >= 0 ? v * p10[e] : v / p10[-e];
  *out = neg ? -v : v;
  return true;
}

__device__ __forceinline__ const char* ptext_at(const char* t, int64_t i) { return t + i; }
__device__ __forceinline__ const char* ptext_at(const LdsText& t, int64_t i) { return text_at(t, i); }

// One line li of the batch; `text` is the batch in global memory or its LDS tile (line_tile.h).
template <class Text>
__device__ __forceinline__ uint8_t parse_one_line(Text text, const int64_t* __restrict__ starts,
                                                  int64_t nlines, int64_t text_len,
                                                  const ParseSpec& spec, int64_t li,
                                                  int64_t* __restrict__ cols,
                                                  int32_t* __restrict__ jhash,
                                                  uint8_t* __restrict__ status) {
  const int64_t a = starts[li];
  int64_t b = li + 1 < nlines ? starts[li + 1] - 1 : text_len;  // exclusive end (drop '\n')
  if (b > a && text[b - 1] == '\r') --b;  // SocketTextStreamFunction strips a trailing '\r'
  // Field boundaries of the requested indices (Java String.split semantics: trailing empty
  // fields are dropped, so an index at or past them is out of bounds). Positions are kept per
  // requested field (compile-time slots, registers only).
  int64_t fs[kMaxFields], fe[kMaxFields];
#pragma unroll
  for (int f = 0; f < kMaxFields; ++f) fs[f] = fe[f] = -1;
  int idx = 0;
  int64_t cur = a, last_nonempty = -1;
  for (int64_t pos = a; pos <= b; ++pos) {
    if (pos == b || text[pos] == spec.sep) {
#pragma unroll
      for (int f = 0; f < kMaxFields; ++f)
        if (f < spec.nfields && spec.field[f] == idx) {
          fs[f] = cur;
          fe[f] = pos;
        }
      if (pos > cur) last_nonempty = idx;
      ++idx;
      cur = pos + 1;
    }
  }
  const int64_t nfields_java = a == b ? 1 : last_nonempty + 1;  // "".split(x) == [""]
  uint8_t st = 0;
#pragma unroll
  for (int f = 0; f < kMaxFields; ++f) {
    if (f >= spec.nfields || st != 0) continue;
    if (spec.field[f] >= nfields_java || fs[f] < 0) {
      st = 1;  // ArrayIndexOutOfBounds: the host reports it
      continue;
    }
    const char* p = ptext_at(text, fs[f]);
    const int64_t len = fe[f] - fs[f];
    int64_t* out = cols + (size_t)f * nlines + li;
    switch (spec.kind[f]) {
      case FK_STR: {
        uint64_t h = 0xcbf29ce484222325ull;
        int32_t jh = 0;
        for (int64_t k = 0; k < len; ++k) {
          const unsigned char c = (unsigned char)p[k];
          if (c >= 0x80) {
            st = 1;  // non-ASCII: UTF-16 hashing on the host
            break;
          }
          h = (h ^ c) * 0x100000001b3ull;
          jh = 31 * jh + (int32_t)c;
        }
        *out = (int64_t)(h == kEmptyKey || h == ~1ull ? h - 2 : h);  // keep -1/-2 reserved
        jhash[(size_t)f * nlines + li] = jh;
        break;
      }
      case FK_DOUBLE: {
        double d;
        if (!fast_double(p, len, &d)) st = 1;
        else *out = (int64_t)f64_bits(d);
        break;
      }
      case FK_LONG:
      case FK_RAW_LONG:
      case FK_INT: {
        int64_t v;
        const bool is_int = spec.kind[f] == FK_INT;
        if (parse_long_ascii(p, len, is_int ? INT32_MIN : INT64_MIN, is_int ? INT32_MAX : INT64_MAX,
                             &v) != 0)
          st = 1;
        else
          *out = v;
        break;
      }
      case FK_TS_INTSEC:
      case FK_TS_MS: {
        int64_t es, ms;
        if (!iso_local_datetime(p, len, spec.offset_s, &es, &ms)) {
          st = 1;
        } else if (spec.kind[f] == FK_TS_MS) {
          *out = es * 1000 + ms;
        } else {
          *out = (int64_t)(int32_t)(uint32_t)(uint64_t)es * 1000;  // (int) cast quirk
        }
        break;
      }
      default: st = 1;
    }
  }
  status[li] = st;
  return st;
}

// One workgroup per tile of 256 lines, staged in LDS (line_tile.h); `nlines_dev` (optional) is
// the device line count of line_starts: the grid is sized for a bound, tiles past the count exit.
__global__ __launch_bounds__(256) void parse_text_kernel(
    const char* __restrict__ text, const int64_t* __restrict__ starts, int64_t nlines_bound,
    const int64_t* __restrict__ nlines_dev, int64_t text_len, ParseSpec spec,
    int64_t* __restrict__ cols, int32_t* __restrict__ jhash, uint8_t* __restrict__ status,
    uint32_t* __restrict__ nflag) {
  __shared__ __attribute__((aligned(16))) char tile[kTileLdsBytes];
  int64_t nlines = nlines_dev ? *nlines_dev : nlines_bound;
  if (nlines > nlines_bound) nlines = nlines_bound;  // more lines than the outputs hold: redone
  const int64_t l0 = (int64_t)blockIdx.x * kTileLines;
  if (l0 >= nlines) return;  // uniform per workgroup: before any barrier
  const int64_t l1 = l0 + kTileLines < nlines ? l0 + kTileLines : nlines;
  const int64_t lo = starts[l0];
  const int64_t hi = l1 < nlines ? starts[l1] : text_len;
  const LdsText lt = stage_line_tile(text, lo, hi, tile, kTileLdsBytes);
  const int64_t li = l0 + threadIdx.x;
  uint8_t st = 0;
  if (li < l1) {
    st = lt.p != nullptr ? parse_one_line(lt, starts, nlines, text_len, spec, li, cols, jhash, status)
                         : parse_one_line(text, starts, nlines, text_len, spec, li, cols, jhash, status);
  }
  // flagged lines: one atomic per wave (the host patch reads the status column only then)
  const uint64_t m = __ballot(st != 0);
  if (nflag != nullptr && (threadIdx.x & 63) == 0 && m) atomicAdd(nflag, (uint32_t)__popcll(m));
}

}  // namespace

namespace gpu {

void parse_text(const char* text, int64_t text_len, const int64_t* starts, int64_t nlines,
                const int32_t* fields, const int32_t* kinds, int nfields, char sep,
                int64_t offset_s, int64_t* cols, int32_t* jhash, uint8_t* status,
                intptr_t stream, const int64_t* nlines_dev, uint32_t* nflag) {
  if (nlines <= 0) return;
  if (nfields <= 0 || nfields > kMaxFields) throw std::invalid_argument("parse_text: 1..8 fields");
  ParseSpec spec;
  spec.nfields = nfields;
  for (int f = 0; f < kMaxFields; ++f) {
    spec.field[f] = f < nfields ? fields[f] : 0;
    spec.kind[f] = f < nfields ? kinds[f] : 0;
    if (f < nfields && (spec.field[f] < 0 || spec.kind[f] < 0 || spec.kind[f] > 6))
      throw std::invalid_argument("parse_text: bad field spec");
  }
  spec.offset_s = offset_s;
  spec.sep = sep;
  const int64_t g = (nlines + kTileLines - 1) / kTileLines;
  if (g > INT32_MAX) throw std::invalid_argument("parse_text: batch too large");
  hipLaunchKernelGGL(parse_text_kernel, dim3((unsigned)g), dim3(kTileLines), 0,
                     (hipStream_t)stream, text, starts, nlines, nlines_dev, text_len, spec, cols,
                     jhash, status, nflag);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("parse_text: ") + hipGetErrorString(e));
}

}  // namespace gpu
}  // namespace mxs
