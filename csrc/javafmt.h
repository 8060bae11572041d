// mxstream — Java text formatting of print() sinks in bulk (the host twin of
// mxstream/utils/javafmt.py): Double.toString (shortest round-trip digits; plain notation for
// 1e-3 <= |x| < 1e7, d.dddE<exp> otherwise), Long.toString and Tuple.toString "(f0,f1,...)".
// A window firing of thousands of alerts is formatted here in one call instead of one Python
// str() chain per record (SURVEY.md F-print; golden outputs chapter3/README.md:295-296).
#pragma once
#include <charconv>
#include <cmath>
#include <cstdint>
#include <string>

namespace mxs {

inline void java_double_append(double x, std::string& out) {
  if (std::isnan(x)) {
    out += "NaN";
    return;
  }
  if (std::isinf(x)) {
    out += x > 0 ? "Infinity" : "-Infinity";
    return;
  }
  if (x == 0.0) {
    out += std::signbit(x) ? "-0.0" : "0.0";
    return;
  }
  if (x < 0) out.push_back('-');
  const double ax = std::fabs(x);
  // Shortest round-trip digits in scientific form: "d[.ddd]e[+-]XX".
  char b[48];
  const auto r = std::to_chars(b, b + sizeof(b), ax, std::chars_format::scientific);
  char digits[32];
  int nd = 0, e10 = 0;
  const char* p = b;
  for (; p < r.ptr && *p != 'e'; ++p)
    if (*p != '.') digits[nd++] = *p;
  if (p < r.ptr) std::from_chars(p + 1 + (p[1] == '+'), r.ptr, e10);
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  if (ax >= 1e-3 && ax < 1e7) {
    const int point = e10 + 1;  // digits before the decimal point
    if (point <= 0) {
      out += "0.";
      out.append((size_t)-point, '0');
      out.append(digits, (size_t)nd);
    } else if (point >= nd) {
      out.append(digits, (size_t)nd);
      out.append((size_t)(point - nd), '0');
      out += ".0";
    } else {
      out.append(digits, (size_t)point);
      out.push_back('.');
      out.append(digits + point, (size_t)(nd - point));
    }
    return;
  }
  out.push_back(digits[0]);
  out.push_back('.');
  if (nd > 1)
    out.append(digits + 1, (size_t)(nd - 1));
  else
    out.push_back('0');
  out.push_back('E');
  out += std::to_string(e10);
}

inline void java_long_append(int64_t v, std::string& out) {
  char b[24];
  const auto r = std::to_chars(b, b + sizeof(b), v);
  out.append(b, (size_t)(r.ptr - b));
}

}  // namespace mxs
