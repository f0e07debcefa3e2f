// Exact decimal -> binary64 conversion (Eisel-Lemire), shared by the device JSON loader and a host
// diagnostic.  The reference types a plain YAML / JSON number that is not an i64 with Rust's
// `str::parse::<f64>` (guard/src/rules/libyaml/loader.rs:86-99), which rounds correctly; this is the
// same algorithm as Rust's core::num::dec2flt fast path: the decimal significand w (<= 19 digits)
// times the 128-bit truncated 5^q (pow5_table.h) decides the correctly rounded result for every q
// in [-342, 308] (Mushtak & Lemire, "Fast number parsing without fallback").  Longer significands
// are truncated to 19 digits and decided when w and w + 1 round to the same double; otherwise (and
// for overflow to infinity) the caller refuses the document and the host loader parses it.
#pragma once
#include <stdint.h>

#include "pow5_table.h"

#ifndef GG_HD
#define GG_HD
#endif

namespace gg {

// the IEEE bits of the double nearest w * 10^q (ties to even); false: q beyond the table's range
// (the result is then 0 or infinity, which the caller handles by refusing)
template <typename Tab>
GG_HD inline bool eisel_lemire(uint64_t w, int64_t q, const Tab& tab, uint64_t& bits) {
  if (w == 0 || q < -342) { bits = 0; return true; }
  if (q > 308) { bits = 0x7FF0000000000000ull; return true; }
  const int lz = __builtin_clzll(w);
  w <<= lz;
  const uint32_t idx = 2u * (uint32_t)(q + 342);
  unsigned __int128 p = (unsigned __int128)w * tab[idx];
  uint64_t lo = (uint64_t)p, hi = (uint64_t)(p >> 64);
  const uint64_t mask = 0xFFFFFFFFFFFFFFFFull >> 55;   // 52 explicit bits + 3
  if ((hi & mask) == mask) {
    const unsigned __int128 p2 = (unsigned __int128)w * tab[idx + 1];
    const uint64_t h2 = (uint64_t)(p2 >> 64);
    lo += h2;
    if (h2 > lo) hi++;
  }
  const int upperbit = (int)(hi >> 63);
  const int shift = upperbit + 64 - 52 - 3;
  uint64_t mant = hi >> shift;
  int32_t pow2 = (int32_t)((((152170 + 65536) * q) >> 16) + 63) + upperbit - lz + 1023;
  if (pow2 <= 0) {   // subnormal (or zero)
    if (-pow2 + 1 >= 64) { bits = 0; return true; }
    mant >>= -pow2 + 1;
    mant += mant & 1;
    mant >>= 1;
    pow2 = mant < (1ull << 52) ? 0 : 1;
    bits = mant | ((uint64_t)pow2 << 52);
    return true;
  }
  // exactly halfway between two doubles: round to even (only possible for small |q|)
  if (lo <= 1 && q >= -4 && q <= 23 && (mant & 3) == 1) {
    if ((mant << shift) == hi) mant &= ~1ull;
  }
  mant += mant & 1;
  mant >>= 1;
  if (mant >= (2ull << 52)) { mant = 1ull << 52; pow2++; }
  mant &= ~(1ull << 52);
  if (pow2 >= 0x7FF) { pow2 = 0x7FF; mant = 0; }
  bits = mant | ((uint64_t)pow2 << 52);
  return true;
}

// A JSON number token [-]int[.frac][e[+-]exp] (at(k) = its byte k, L bytes) -> IEEE bits.  false:
// undecided (a truncated significand whose neighbours round apart), an infinite result, or an
// exponent beyond 10000 -- the caller refuses the document.
template <typename At, typename Tab>
GG_HD inline bool parse_json_f64(At&& at, uint64_t L, const Tab& tab, uint64_t& bits) {
  uint64_t k = 0;
  const bool neg = at(0) == '-';
  if (neg) k = 1;
  uint64_t w = 0;
  int32_t nd = 0, dropped = 0, exp10 = 0;
  bool frac = false, trunc = false;
  for (; k < L; k++) {
    const uint32_t c = at(k);
    if (c == '.') { frac = true; continue; }
    if (c == 'e' || c == 'E') break;
    const uint32_t d = c - '0';
    if (nd == 0 && d == 0) { if (frac) exp10--; continue; }   // leading zeros
    if (nd < 19) { w = w * 10u + d; nd++; if (frac) exp10--; }
    else { if (!frac) dropped++; if (d) trunc = true; }       // digits past the 19th
  }
  if (k < L) {
    k++;
    bool eneg = false;
    if (at(k) == '+' || at(k) == '-') { eneg = at(k) == '-'; k++; }
    int32_t e = 0;
    for (; k < L; k++) { e = e * 10 + (int32_t)(at(k) - '0'); if (e > 10000) return false; }
    exp10 += eneg ? -e : e;
  }
  const int64_t q = (int64_t)exp10 + dropped;
  uint64_t b = 0;
  if (w == 0) {
    b = 0;
  } else {
    if (!eisel_lemire(w, q, tab, b)) return false;
    if (trunc) {
      // non-zero digits past the 19th were cut off: decided when w + 1 rounds the same way
      uint64_t b2 = 0;
      if (!eisel_lemire(w + 1, q, tab, b2) || b2 != b) return false;
    }
    if ((b & 0x7FF0000000000000ull) == 0x7FF0000000000000ull) return false;   // overflow: the host decides
  }
  bits = b | (neg ? 0x8000000000000000ull : 0ull);
  return true;
}

}  // namespace gg
