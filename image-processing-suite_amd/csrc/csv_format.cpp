// Host-side CSV rows for the per-plate measurement tables (cpx.csvout): the <Object>.csv files
// that Pycyto_pertime.py:46-49 reads are written by pandas DataFrame.to_csv in the reference's
// world, one row per object with ~160 float64 columns — about 10^8 numbers per 768 FOVs, a
// minute of pandas formatting against 2 s of GPU work.  This formats the same bytes natively:
// int64 columns in decimal, float64 columns as Python's repr (pandas' float64 text, na_rep ""
// for NaN), one call per row range so the host can format ranges on several threads (ctypes
// releases the GIL) and write them in order.
#include "../../include/cpx.h"

#include <cstdint>

#include <charconv>
#include <cmath>
#include <cstring>

namespace {

// Python repr of a finite or infinite double (CPython format_float_short, mode 'r' with
// Py_DTSF_ADD_DOT_0): the shortest round-trip digits; fixed notation when the decimal point
// position decpt = exponent + 1 satisfies -4 < decpt <= 16 (".0" appended to integral values),
// else d[.ddd]e±XX with at least two exponent digits.
inline char* put_repr(char* p, double v) {
  if (std::isnan(v)) return p;  // pandas na_rep
  if (std::isinf(v)) {
    if (v < 0) *p++ = '-';
    std::memcpy(p, "inf", 3);
    return p + 3;
  }
  char buf[48];
  const std::to_chars_result r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  const char* q = buf;
  if (*q == '-') {
    *p++ = '-';
    ++q;
  }
  char dg[24];
  int nd = 0;
  while (q < r.ptr && *q != 'e') {
    if (*q != '.') dg[nd++] = *q;
    ++q;
  }
  ++q;  // 'e'
  const bool eneg = *q == '-';
  ++q;  // sign (always written)
  int e = 0;
  while (q < r.ptr) e = e * 10 + (*q++ - '0');
  if (eneg) e = -e;
  const int decpt = e + 1;
  if (decpt <= -4 || decpt > 16) {
    *p++ = dg[0];
    if (nd > 1) {
      *p++ = '.';
      std::memcpy(p, dg + 1, nd - 1);
      p += nd - 1;
    }
    *p++ = 'e';
    *p++ = e < 0 ? '-' : '+';
    const int ae = e < 0 ? -e : e;
    if (ae >= 100) *p++ = (char)('0' + ae / 100);
    *p++ = (char)('0' + (ae / 10) % 10);
    *p++ = (char)('0' + ae % 10);
  } else if (decpt <= 0) {
    *p++ = '0';
    *p++ = '.';
    for (int i = 0; i < -decpt; ++i) *p++ = '0';
    std::memcpy(p, dg, nd);
    p += nd;
  } else if (decpt >= nd) {
    std::memcpy(p, dg, nd);
    p += nd;
    for (int i = nd; i < decpt; ++i) *p++ = '0';
    *p++ = '.';
    *p++ = '0';
  } else {
    std::memcpy(p, dg, decpt);
    p += decpt;
    *p++ = '.';
    std::memcpy(p, dg + decpt, nd - decpt);
    p += nd - decpt;
  }
  return p;
}

constexpr int64_t kMaxField = 32;  // "-1.7976931348623157e+308" is 24 bytes, an int64 20

}  // namespace

extern "C" int64_t cpx_csv_format(int64_t row0, int64_t row1, int n_cols, const void* const* cols,
                                  const int* types, const int64_t* strides, char* out, int64_t cap) {
  if (row1 < row0 || n_cols <= 0 || !cols || !types || !strides || !out) return -1;
  if ((row1 - row0) * (kMaxField + 1) * n_cols > cap) return -1;
  char* p = out;
  for (int64_t r = row0; r < row1; ++r) {
    for (int c = 0; c < n_cols; ++c) {
      if (c) *p++ = ',';
      if (types[c] == 0) {
        const int64_t v = static_cast<const int64_t*>(cols[c])[r * strides[c]];
        p = std::to_chars(p, p + kMaxField, v).ptr;
      } else {
        p = put_repr(p, static_cast<const double*>(cols[c])[r * strides[c]]);
      }
    }
    *p++ = '\n';
  }
  return (int64_t)(p - out);
}
