// Host-side text formatting that must match the reference byte for byte:
//   * Rust `impl Display for f64` (shortest digits, never an exponent)
//   * Rust `impl Debug for f64`
//   * serde_json / ryu float output (ryu::Buffer::format_finite)
//   * serde_json string escaping, Rust `{:?}` string escaping
#pragma once
#if defined(__SSE2__)
#include <emmintrin.h>
#endif
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace gg {

struct ShortestDigits { bool neg; std::string d; int k; };  // |x| = d * 10^k

inline ShortestDigits shortest(double x) {
  ShortestDigits r;
  r.neg = std::signbit(x);
  double ax = std::fabs(x);
  if (ax == 0.0) { r.d = "0"; r.k = 0; return r; }
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof buf, ax, std::chars_format::scientific);
  std::string s(buf, res.ptr);
  size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  int exp = std::atoi(s.c_str() + e + 1);
  std::string digits;
  for (char c : mant) if (c != '.') digits.push_back(c);
  // mant = D.DDD -> value = DDDD * 10^(exp - (len-1))
  int k = exp - (int)(digits.size() - 1);
  while (digits.size() > 1 && digits.back() == '0') { digits.pop_back(); k++; }
  r.d = digits; r.k = k;
  return r;
}

inline std::string rust_display_f64(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "inf" : "-inf";
  ShortestDigits s = shortest(x);
  std::string out;
  if (s.d == "0") out = "0";
  else if (s.k >= 0) out = s.d + std::string(s.k, '0');
  else {
    int pos = (int)s.d.size() + s.k;
    if (pos > 0) out = s.d.substr(0, pos) + "." + s.d.substr(pos);
    else out = "0." + std::string(-pos, '0') + s.d;
  }
  return (s.neg ? "-" : "") + out;
}

inline std::string rust_debug_f64(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "inf" : "-inf";
  double ax = std::fabs(x);
  ShortestDigits s = shortest(x);
  std::string sign = s.neg ? "-" : "";
  if (ax == 0.0 || (ax >= 1e-4 && ax < 1e16)) {
    std::string t = rust_display_f64(ax);
    if (t.find('.') == std::string::npos) t += ".0";
    return sign + t;
  }
  int exp = (int)s.d.size() - 1 + s.k;
  std::string mant = s.d.substr(0, 1);
  if (s.d.size() > 1) mant += "." + s.d.substr(1);
  return sign + mant + "e" + std::to_string(exp);
}

inline std::string ryu_f64(double x) {
  ShortestDigits s = shortest(x);
  std::string sign = s.neg ? "-" : "";
  if (s.d == "0") return sign + "0.0";
  int length = (int)s.d.size();
  int kk = length + s.k;
  if (0 <= s.k && kk <= 16) return sign + s.d + std::string(s.k, '0') + ".0";
  if (0 < kk && kk <= 16) return sign + s.d.substr(0, kk) + "." + s.d.substr(kk);
  if (-5 < kk && kk <= 0) return sign + "0." + std::string(-kk, '0') + s.d;
  if (length == 1) return sign + s.d + "e" + std::to_string(kk - 1);
  return sign + s.d.substr(0, 1) + "." + s.d.substr(1) + "e" + std::to_string(kk - 1);
}

template <class Out>
inline void json_escape_into(Out& out, const char* p, size_t n) {
  // serde_json's escaping; plain runs are appended whole (found 16 bytes at a time)
  out.push_back('"');
  size_t run = 0;
  size_t i = 0;
#if defined(__SSE2__)
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), lim = _mm_set1_epi8(0x1F);
  while (i + 16 <= n) {
    const __m128i x = _mm_loadu_si128((const __m128i*)(p + i));
    const __m128i ctl = _mm_cmpeq_epi8(_mm_max_epu8(x, lim), lim);   // bytes <= 0x1F
    const __m128i m = _mm_or_si128(ctl, _mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)));
    if (_mm_movemask_epi8(m)) break;   // the byte loop below takes this chunk
    i += 16;
  }
#endif
  for (; i < n; i++) {
    const unsigned char c = (unsigned char)p[i];
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(p + run, i - run);
    run = i + 1;
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default: { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); out += b; }
    }
  }
  out.append(p + run, n - run);
  out.push_back('"');
}

inline std::string json_escape(const std::string& s) {
  std::string o; json_escape_into(o, s.data(), s.size()); return o;
}

// decode one UTF-8 scalar starting at p (assumes valid UTF-8)
inline uint32_t utf8_next(const unsigned char* p, size_t n, size_t& i) {
  unsigned char c = p[i];
  if (c < 0x80) { i += 1; return c; }
  if ((c >> 5) == 6 && i + 1 < n) { uint32_t v = ((c & 0x1F) << 6) | (p[i + 1] & 0x3F); i += 2; return v; }
  if ((c >> 4) == 14 && i + 2 < n) { uint32_t v = ((c & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F); i += 3; return v; }
  if (i + 3 < n) { uint32_t v = ((c & 0x07) << 18) | ((p[i + 1] & 0x3F) << 12) | ((p[i + 2] & 0x3F) << 6) | (p[i + 3] & 0x3F); i += 4; return v; }
  i += 1; return c;
}

inline void utf8_append(std::string& out, uint32_t cp) {
  if (cp < 0x80) out.push_back((char)cp);
  else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) { out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F))); }
  else { out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 0x3F))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F))); }
}

// Rust char::escape_debug-ish escaping used by `{:?}` on str (as used by derive(Debug))
inline std::string rust_debug_str(const char* p, size_t n) {
  std::string out = "\"";
  size_t i = 0;
  const unsigned char* u = (const unsigned char*)p;
  while (i < n) {
    size_t s = i;
    uint32_t cp = utf8_next(u, n, i);
    if (cp == '"') out += "\\\"";
    else if (cp == '\\') out += "\\\\";
    else if (cp == '\n') out += "\\n";
    else if (cp == '\r') out += "\\r";
    else if (cp == '\t') out += "\\t";
    else if (cp == 0) out += "\\0";
    else if (cp < 0x20 || cp == 0x7F || (cp >= 0x80 && cp < 0xA0)) { char b[16]; snprintf(b, sizeof b, "\\u{%x}", cp); out += b; }
    else out.append(p + s, i - s);
  }
  out += "\"";
  return out;
}
inline std::string rust_debug_str(const std::string& s) { return rust_debug_str(s.data(), s.size()); }

// char::is_whitespace (Unicode White_Space)
inline bool rust_is_whitespace(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
// str::trim: leading and trailing Unicode whitespace removed
inline std::string rust_trim(const std::string& s) {
  const unsigned char* p = (const unsigned char*)s.data();
  size_t i = 0, b = 0, e = 0;
  bool seen = false;
  while (i < s.size()) {
    const size_t at = i;
    const uint32_t c = utf8_next(p, s.size(), i);
    if (!rust_is_whitespace(c)) { if (!seen) { b = at; seen = true; } e = i; }
  }
  return seen ? s.substr(b, e - b) : std::string();
}

inline uint32_t fnv1a(const char* p, size_t n) {
  uint32_t h = 2166136261u;
  for (size_t i = 0; i < n; i++) { h ^= (unsigned char)p[i]; h *= 16777619u; }
  return h;
}

}  // namespace gg
