// GPU document loader: strict-JSON text -> columnar node arena (see json_gpu.h).
//
// One lane parses one document (documents are a few KB; a lane walks its text through a 16-byte
// window, so each load serves 16 bytes, and skips plain string runs a window at a time).  Passes:
//   1. count      validate the subset the host fast path accepts (doc_loader.cpp load_json_fast),
//                 count nodes, containers, string occurrences, and record the child count of every
//                 container, in pre-order (host: JsonFast::v1), as 16-bit counts at a document's
//                 half text offset (a container takes two bytes at least, so a document's counts
//                 never reach the next one's);
//   2. emit       the nodes in the host layout -- each container's children contiguous, blocks in
//                 DFS pre-order (host: JsonFast::v2) -- with marks, scalar typing, and every
//                 string inserted into a device hash table keyed by a 64-bit fingerprint of its
//                 decoded bytes; nodes carry table slots for now and each string occurrence's text
//                 offset;
//   3. own        every occupied slot copies its first occurrence's decoded bytes into the pool
//                 (16-byte aligned, zero padded: the evaluator compares in 16-byte chunks); the
//                 pool offset is the string id, as on the host;
//   4. fix+verify one wave per document over its nodes: slots -> ids, every occurrence's decoded
//                 bytes compared with its id's pool bytes, so a fingerprint collision cannot merge
//                 two strings silently, and every map key against its earlier siblings (duplicate
//                 keys); either refuses the document.
// A document outside the subset is refused on its own (per-document flag): the passes skip it, the
// host loader builds it (doc_loader.cpp, the libyaml path) and its nodes join the batch at the
// document's position, so results never depend on which loader ran.  Only batch-wide limits (string
// table or pool full, sizes) refuse the whole batch.
#include "json_gpu.h"

#include <hip/hip_runtime.h>

#define GG_HD __host__ __device__
#define GG_POW5_QUAL __constant__
#include "eisel_lemire.h"
#include "dev_cache.h"
#include "host_pinned.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <memory>
#include <mutex>
#include <thread>

#ifndef GG_JDIAG_NOINTERN
#define GG_JDIAG_NOINTERN 0   // diagnostic A/B builds only: skip the intern table
#endif

namespace gg {
namespace {

#define JCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); } while (0)

enum : uint32_t { M_COUNT = 0, M_EMIT = 2 };
enum : uint32_t {
  BAD_NONE = 0, BAD_SYNTAX = 1, BAD_DEPTH = 2, BAD_DUPKEY = 3, BAD_NUMBER = 4, BAD_TABLE = 5, BAD_POOL = 6,
  BAD_VERIFY = 7, BAD_SIZE = 8, BAD_WIDE = 9,
  BAD_NOTJSON = 10,   // count pass: not a JSON document (the YAML passes take it, yaml_gpu.inc)
  BAD_YAML = 11,      // outside the block-style YAML subset the YAML passes parse
  BAD_WIDEMAP = 12,   // a map with more keys than the verify pass's duplicate-key scan takes
};
static const uint32_t kMaxDepth = 64;
static const uint32_t kMaxPairwiseKeys = 256;

// the emit pass's output per node: the node and its marks in one 64-byte record, so a lane writes
// one line per node instead of seven scattered streams; the fix / verify pass splits the records
// into the arena's columns with coalesced stores
struct NodeRec {
  DNode n;
  uint32_t line, col, kline, kcol;
  uint32_t kpos, vpos;   // document offsets of the key's and the string value's opening quotes
  uint32_t pad0, pad1;
};
static_assert(sizeof(NodeRec) == 64, "one 64-byte record per node");

struct JArgs {
  const uint8_t* text;          // all documents, 16 zero bytes of padding at the end
  const uint64_t* off;          // [ndocs + 1]
  uint32_t ndocs;
  // pass 1 outputs (per document)
  uint32_t* n_nodes;
  uint32_t* n_cont;
  uint32_t* n_str;
  // pass 2 / 3 inputs
  const uint64_t* node_base;    // per document: first node
  uint16_t* counts;             // child counts: document d's container k at off[d] / 2 + k
  NodeRec* recs;                // emit -> fix / verify
  DNode* nodes;
  uint32_t* line;
  uint32_t* col;
  uint32_t* kline;
  uint32_t* kcol;
  // intern table
  unsigned long long* tkey;     // 0 = empty
  uint32_t* tlen;
  unsigned long long* towner;   // doc << 32 | offset of the opening quote in the document
  uint32_t* tid;
  uint64_t tmask;
  uint8_t* pool;
  unsigned long long* pool_cursor;
  uint64_t pool_cap;
  uint64_t fp_mask;             // fingerprint bits kept (~0; tests narrow it to force collisions)
  uint32_t* bad;                // batch-wide refusal (BAD_TABLE / BAD_POOL: grow and retry), 0 = none
  uint32_t* doc_bad;            // per document: its refusal reason (BAD_*), 0 = loaded on the device
  uint8_t* is_yaml;             // per document: parsed by the YAML passes
  uint32_t* bad_at;             // diagnostics (GG_LOAD_DIAG): the YAML passes' byte offset of a refusal
};

__device__ inline void refuse(const JArgs& A, uint32_t why) { atomicCAS(A.bad, 0u, why); }

struct Text {
  const uint8_t* s;
  uint64_t base, n;
  uint4 w;
  uint64_t wb;
  __device__ Text(const uint8_t* t, uint64_t b, uint64_t len) : s(t), base(b), n(len), wb(~0ull) {}
  // byte i of the document, 256 past its end
  __device__ __attribute__((always_inline)) uint32_t at(uint64_t i) {
    if (i >= n) return 256u;
    const uint64_t g = base + i, a = g & ~15ull;
    if (a != wb) { w = *(const uint4*)(s + a); wb = a; }
    const uint32_t k = (uint32_t)(g - a);
    const uint32_t word = k < 4 ? w.x : (k < 8 ? w.y : (k < 12 ? w.z : w.w));
    return (word >> ((k & 3u) * 8u)) & 0xFFu;
  }
  // bit 7 of each byte of x set where the byte ends a plain string run: '"', '\\', a control
  // byte (< 0x20), DEL or a non-ASCII byte (SWAR; only the lowest flagged byte is exact, which is
  // the one plain_run uses)
  __device__ static uint32_t special(uint32_t x) {
    const uint32_t q = x ^ 0x22222222u, b = x ^ 0x5C5C5C5Cu, d = x ^ 0x7F7F7F7Fu;
    const uint32_t zq = (q - 0x01010101u) & ~q, zb = (b - 0x01010101u) & ~b, zd = (d - 0x01010101u) & ~d;
    const uint32_t lt = (x - 0x20202020u) & ~x;
    return (zq | zb | zd | lt | x) & 0x80808080u;
  }
  // bytes k .. k+3 of the current window, little-endian (zeros past its end)
  __device__ uint32_t bytes4(uint32_t k) const {
    const uint32_t j = k >> 2;
    const uint32_t lo = j == 0 ? w.x : (j == 1 ? w.y : (j == 2 ? w.z : w.w));
    const uint32_t hi = j == 0 ? w.y : (j == 1 ? w.z : (j == 2 ? w.w : 0u));
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3u);
  }
  // the window offset of document byte i (after plain_run(i) loaded its window)
  __device__ uint32_t woff(uint64_t i) const { return (uint32_t)((base + i) & 15ull); }
  // YAML plain scalars (yaml_gpu.inc scan_plain): bit 7 set where the byte is not an ordinary plain-scalar
  // byte -- a space or control byte, ':', '#', DEL, a non-ASCII byte, and in flow context , [ ] { } (the
  // lowest flagged byte is exact; a borrow can only flag a later byte too, which shortens a run)
  __device__ static uint32_t eq_bytes(uint32_t x, uint32_t rep) { const uint32_t v = x ^ rep; return (v - 0x01010101u) & ~v; }
  template <bool FLOW>
  __device__ static uint32_t yplain_special(uint32_t x) {
    uint32_t m = eq_bytes(x, 0x3A3A3A3Au) | eq_bytes(x, 0x23232323u) | eq_bytes(x, 0x7F7F7F7Fu) | ((x - 0x21212121u) & ~x) | x;
    if (FLOW)
      m |= eq_bytes(x, 0x2C2C2C2Cu) | eq_bytes(x, 0x5B5B5B5Bu) | eq_bytes(x, 0x5D5D5D5Du) | eq_bytes(x, 0x7B7B7B7Bu) |
           eq_bytes(x, 0x7D7D7D7Du);
    return m & 0x80808080u;
  }
  // comments: bit 7 set where the byte is not printable ASCII (a control byte -- the tab and the line break
  // included --, DEL or a non-ASCII byte)
  __device__ static uint32_t not_printable(uint32_t x) {
    return (eq_bytes(x, 0x7F7F7F7Fu) | ((x - 0x20202020u) & ~x) | x) & 0x80808080u;
  }
  // bit 7 set where the byte is not a space (exact per byte: no borrows)
  __device__ static uint32_t not_space(uint32_t x) {
    const uint32_t v = x ^ 0x20202020u;
    return (((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
  }
  // the number of plain printable ASCII bytes from i to the first special byte, the end of i's
  // 16-byte block or the end of the document (0 when byte i is special)
  __device__ uint32_t plain_run(uint64_t i) { return run_of(i, [](uint32_t x) { return special(x); }); }
  // the same for the bytes SP flags (yplain_special, not_space)
  template <typename SP>
  __device__ __attribute__((always_inline)) uint32_t run_of(uint64_t i, SP&& sp) {
    if (i >= n) return 0;
    const uint64_t g = base + i, a = g & ~15ull;
    if (a != wb) { w = *(const uint4*)(s + a); wb = a; }
    const uint32_t k = (uint32_t)(g - a);
    uint64_t lo = (uint64_t)sp(w.x) | ((uint64_t)sp(w.y) << 32);
    uint64_t hi = (uint64_t)sp(w.z) | ((uint64_t)sp(w.w) << 32);
    if (k < 8) lo &= ~0ull << (8u * k);
    else { lo = 0; hi &= ~0ull << (8u * (k - 8u)); }
    const uint32_t first = lo ? (uint32_t)__builtin_ctzll(lo) >> 3 : (hi ? 8u + ((uint32_t)__builtin_ctzll(hi) >> 3) : 16u);
    const uint64_t left = n - i;
    const uint32_t r = first - k;
    return left < r ? (uint32_t)left : r;
  }
};

// The decoded bytes of a string as little-endian 4-byte words: on_word(word, bytes so far) for each
// full word; a plain run is taken from the text window 4 bytes at a time.  The caller handles the
// last partial word (`word`, len & 3 bytes).
struct WordStream {
  uint32_t word = 0, len = 0;
  template <typename F>
  __device__ void byte(uint32_t c, F&& on_word) {
    word |= c << ((len & 3u) * 8u);
    len++;
    if ((len & 3u) == 0) { on_word(word, len); word = 0; }
  }
  // r plain bytes at offset k of T's window (k + r <= 16)
  template <typename F>
  __device__ void run(const struct Text& T, uint32_t k, uint32_t r, F&& on_word);
};

__device__ inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Decodes the JSON string whose opening quote is at `q`; calls sink(byte) per decoded byte.
// Returns the index after the closing quote, or 0 when the string is outside the subset (bad
// escapes, surrogate \u escapes, control bytes, malformed UTF-8, and the raw characters libyaml's
// reader treats specially: C1 controls and U+FFFE / U+FFFF, which it rejects, and U+0085 / U+2028 /
// U+2029, which it reads as line breaks).  Raw UTF-8 passes through as it is, as libyaml keeps it;
// `cont` counts its continuation bytes, because libyaml's marks count characters, not bytes
// (a mark's column = bytes since the line start - continuation bytes since it).
// The sink takes decoded bytes one by one (sink.byte(c)) and plain runs whole (sink.run(T, k, r): r
// bytes at offset k of T's window).  BYTES: the sink reads the decoded bytes (false: only the end of
// the string matters, and plain runs are skipped a 16-byte block at a time)
template <bool BYTES = true, typename Sink>
__device__ uint64_t decode_string(Text& T, uint64_t q, Sink&& sink, uint32_t& cont) {
  uint64_t i = q + 1;
  for (;;) {
    const uint32_t r = T.plain_run(i);
    if (r) {
      if (BYTES) sink.run(T, T.woff(i), r);
      i += r;
      continue;
    }
    const uint32_t c = T.at(i);
    if (c == '"') return i + 1;
    if (c >= 0x80u && c < 0x100u) {
      // one UTF-8 sequence: lead byte, 1-3 continuation bytes, shortest form, a scalar value
      const uint32_t n = c >= 0xF0u ? 3u : (c >= 0xE0u ? 2u : (c >= 0xC2u ? 1u : 0u));
      if (!n || c > 0xF4u) return 0;
      uint32_t cp = c & (0x3Fu >> n);
      for (uint32_t k = 1; k <= n; k++) {
        const uint32_t b = T.at(i + k);
        if ((b & 0xC0u) != 0x80u) return 0;
        cp = (cp << 6) | (b & 0x3Fu);
      }
      if ((n == 2 && cp < 0x800u) || (n == 3 && (cp < 0x10000u || cp > 0x10FFFFu))) return 0;
      if (cp >= 0xD800u && cp <= 0xDFFFu) return 0;
      if (cp < 0xA0u || cp == 0x2028u || cp == 0x2029u || cp == 0xFFFEu || cp == 0xFFFFu) return 0;
      for (uint32_t k = 0; k <= n; k++) sink.byte(T.at(i + k));
      cont += n;
      i += n + 1;
      continue;
    }
    if (c < 0x20u || c > 0x7Eu) return 0;
    if (c != '\\') { sink.byte(c); i++; continue; }
    const uint32_t e = T.at(i + 1);
    uint32_t out;
    switch (e) {
      case '"': out = '"'; break;
      case '\\': out = '\\'; break;
      case '/': out = '/'; break;
      case 'b': out = '\b'; break;
      case 'f': out = '\f'; break;
      case 'n': out = '\n'; break;
      case 'r': out = '\r'; break;
      case 't': out = '\t'; break;
      case 'u': {
        uint32_t cp = 0;
        for (uint32_t k = 0; k < 4; k++) {
          const uint32_t h = T.at(i + 2 + k);
          cp <<= 4;
          if (h >= '0' && h <= '9') cp |= h - '0';
          else if (h >= 'a' && h <= 'f') cp |= h - 'a' + 10;
          else if (h >= 'A' && h <= 'F') cp |= h - 'A' + 10;
          else return 0;
        }
        if (cp >= 0xD800 && cp <= 0xDFFF) return 0;
        if (cp < 0x80) sink.byte(cp);
        else if (cp < 0x800) { sink.byte(0xC0u | (cp >> 6)); sink.byte(0x80u | (cp & 0x3Fu)); }
        else { sink.byte(0xE0u | (cp >> 12)); sink.byte(0x80u | ((cp >> 6) & 0x3Fu)); sink.byte(0x80u | (cp & 0x3Fu)); }
        i += 6;
        continue;
      }
      default: return 0;
    }
    sink.byte(out);
    i += 2;
  }
}

template <typename F>
__device__ void WordStream::run(const Text& T, uint32_t k, uint32_t r, F&& on_word) {
  while (r) {
    const uint32_t p = len & 3u;
    const uint32_t take = r < 4u - p ? r : 4u - p;
    uint32_t chunk = T.bytes4(k);
    if (take < 4u) chunk &= (1u << (8u * take)) - 1u;
    word |= chunk << (8u * p);
    len += take; k += take; r -= take;
    if ((len & 3u) == 0) { on_word(word, len); word = 0; }
  }
}

struct Fp { uint64_t h = 0xcbf29ce484222325ull; uint32_t len = 0; };

__device__ inline bool is_digit(uint32_t c) { return c >= '0' && c <= '9'; }

// length of the plain token at i (JSON number / true / false / null), 0 if not one
__device__ uint64_t plain_len(Text& T, uint64_t i) {
  const uint32_t c0 = T.at(i);
  if (c0 == 't' || c0 == 'f' || c0 == 'n') {
    const char* w = c0 == 't' ? "true" : (c0 == 'f' ? "false" : "null");
    uint64_t L = c0 == 'f' ? 5 : 4;
    for (uint64_t k = 0; k < L; k++) if (T.at(i + k) != (uint32_t)(uint8_t)w[k]) return 0;
    return L;
  }
  uint64_t j = i;
  if (T.at(j) == '-') j++;
  if (T.at(j) == '0') j++;
  else if (T.at(j) >= '1' && T.at(j) <= '9') { while (is_digit(T.at(j))) j++; }
  else return 0;
  if (T.at(j) == '.') { j++; const uint64_t d = j; while (is_digit(T.at(j))) j++; if (j == d) return 0; }
  if (T.at(j) == 'e' || T.at(j) == 'E') {
    j++;
    if (T.at(j) == '+' || T.at(j) == '-') j++;
    const uint64_t d = j;
    while (is_digit(T.at(j))) j++;
    if (j == d) return 0;
  }
  return j - i;
}

__device__ inline bool after_plain_ok(uint32_t c) { return c == 256u || c == ' ' || c == '\n' || c == ',' || c == ']' || c == '}'; }

// Scalar typing of a plain token (host JsonFast::v2: true / false / null, then Rust i64::from_str,
// then f64::from_str): i64 exactly; f64 correctly rounded by Eisel-Lemire (eisel_lemire.h); a
// significand it cannot decide or an infinite result refuses the document (the host loader parses it).
__device__ bool scalar(Text& T, uint64_t i, uint64_t L, DNode& d) {
  const uint32_t c0 = T.at(i);
  if (c0 == 't') { d.kind = K_BOOL; d.a = 1; return true; }
  if (c0 == 'f') { d.kind = K_BOOL; d.a = 0; return true; }
  if (c0 == 'n') { d.kind = K_NULL; return true; }
  bool neg = c0 == '-';
  uint64_t j = i + (neg ? 1 : 0);
  bool is_int = true;
  for (uint64_t k = j; k < i + L; k++) if (!is_digit(T.at(k))) { is_int = false; break; }
  if (is_int) {
    uint64_t v = 0;
    for (uint64_t k = j; k < i + L; k++) {
      const uint32_t dg = T.at(k) - '0';
      if (v > (0xFFFFFFFFFFFFFFFFull - dg) / 10ull) return false;   // beyond u64: refuse
      v = v * 10ull + dg;
    }
    if (!neg && v > 0x7FFFFFFFFFFFFFFFull) return false;
    if (neg && v > 0x8000000000000000ull) return false;
    const uint64_t u = neg ? (uint64_t)(-(int64_t)(v - 1) - 1) : v;
    d.kind = K_INT; d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32);
    return true;
  }
  uint64_t u = 0;
  if (!parse_json_f64([&](uint64_t k) { return T.at(i + k); }, L, kPow5_128, u)) return false;
  d.kind = K_FLOAT; d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32);
  return true;
}

// insert-or-find a string fingerprint; returns its slot, or ~0u when the table is full
__device__ uint32_t intern_slot(const JArgs& A, uint64_t key, uint32_t len, uint32_t doc, uint32_t q) {
  uint64_t idx = mix64(key) & A.tmask;
  for (uint32_t probe = 0; probe < 1024; probe++) {
    const unsigned long long k = A.tkey[idx];
    if (k == key) return (uint32_t)idx;
    if (k == 0) {
      const unsigned long long old = atomicCAS(&A.tkey[idx], 0ull, (unsigned long long)key);
      if (old == 0) {
        A.tlen[idx] = len;
        A.towner[idx] = ((unsigned long long)doc << 32) | q;
        return (uint32_t)idx;
      }
      if (old == key) return (uint32_t)idx;
    }
    idx = (idx + 1) & A.tmask;
  }
  return ~0u;
}

struct Frame {
  uint32_t first;   // EMIT / VERIFY: first child (document-relative)
  uint32_t j;       // elements done
  uint32_t slot;    // the container's own node (document-relative)
  uint32_t k;       // pre-order container index
  uint32_t map;     // 1 map, 0 list
};

template <uint32_t MODE>
__device__ void parse_doc(const JArgs& A, uint32_t d) {
  const uint64_t b0 = A.off[d], b1 = A.off[d + 1];
  Text T(A.text, b0, b1 - b0);
  uint64_t i = 0, ls = 0;
  uint32_t line = 0;
  uint32_t cont = 0;   // UTF-8 continuation bytes since the line start (marks count characters)
  auto ws = [&]() {
    for (;;) {
      const uint32_t c = T.at(i);
      if (c == ' ') i++;
      else if (c == '\n') { i++; line++; ls = i; cont = 0; }
      else break;
    }
  };
  auto column = [&]() { return (uint32_t)(i - ls) - cont; };
  // this document is outside the subset: the passes skip it and the host loads it
  auto bad = [&](uint32_t why) { if (!A.doc_bad[d]) A.doc_bad[d] = why; };   // the first reason
  if (MODE == M_COUNT) { A.n_nodes[d] = 0; A.n_cont[d] = 0; A.n_str[d] = 0; }
  else if (A.doc_bad[d] || A.is_yaml[d]) return;
  const uint64_t nb = (MODE >= M_EMIT) ? A.node_base[d] : 0;
  const uint64_t cb = b0 >> 1;
  uint32_t nn = 1, nc = 0, ns = 0, ci = 0, next = 1;
  // the open containers: the innermost one in registers (`top`), the ones around it in st[0, sp - 1)
  // (scratch), so an element's bookkeeping does not go through memory
  Frame st[kMaxDepth];
  Frame top{};
  uint32_t sp = 0;

  // a string occurrence at i (the opening quote): returns the index after it, 0 on refusal;
  // EMIT -> its intern table slot and decoded length
  auto string_at = [&](uint32_t* slot_out, uint32_t* len_out) -> uint64_t {
    Fp fp;
    uint64_t end;
    // fingerprint of the decoded bytes, 4 at a time (the device table's own key: nothing outside
    // this loader compares it)
    struct HashSink {
      WordStream ws;
      uint64_t h;
      __device__ void byte(uint32_t c) { ws.byte(c, [&](uint32_t w, uint32_t) { h = (h ^ w) * 0x100000001b3ull; }); }
      __device__ void run(const Text& T, uint32_t k, uint32_t r) {
        ws.run(T, k, r, [&](uint32_t w, uint32_t) { h = (h ^ w) * 0x100000001b3ull; });
      }
    } hs{WordStream(), fp.h};
    end = decode_string<MODE == M_EMIT>(T, i, hs, cont);
    if (!end) return 0;
    fp.h = (hs.h ^ hs.ws.word) * 0x100000001b3ull;
    fp.len = hs.ws.len;
    if (MODE == M_EMIT) {
      const uint64_t key64 = (mix64(fp.h ^ ((uint64_t)fp.len * 0x9E3779B97F4A7C15ull)) & A.fp_mask) | 1ull;
#if GG_JDIAG_NOINTERN
      const uint32_t s = (uint32_t)key64 & 1023u;
#else
      const uint32_t s = intern_slot(A, key64, fp.len, d, (uint32_t)i);
#endif
      if (s == ~0u) { refuse(A, BAD_TABLE); return 0; }
      *slot_out = s;
      *len_out = fp.len;
    }
    return end;
  };

  // EMIT: the element being emitted -- its key (table slot and length; NONE: no key), the key's
  // offset and mark, and the value's mark
  uint32_t ekey = NONE, elen = 0, ekpos = 0, ekl = 0, ekc = 0, eline = 0, ecol = 0;
  // EMIT: node `rel` and its marks, whole, in one record
  auto put = [&](uint32_t rel, DNode nd, uint32_t parent, uint32_t vpos) {
    nd.key_off = ekey; nd.key_len = elen; nd.key_hash = ekey == NONE ? 0u : ekey; nd.parent = parent;
    NodeRec r;
    r.n = nd; r.line = eline; r.col = ecol; r.kline = ekl; r.kcol = ekc; r.kpos = ekpos; r.vpos = vpos;
    r.pad0 = 0; r.pad1 = 0;
    A.recs[nb + rel] = r;
  };
  // one value at i for node `rel` whose parent is `parent`; containers push a frame
  auto value = [&](uint32_t rel, uint32_t parent) -> bool {
    const uint32_t c = T.at(i);
    if (c == '"') {
      uint32_t slot = 0, len = 0;
      const uint64_t e = string_at(&slot, &len);
      if (!e) return false;
      if (MODE == M_EMIT) {
        DNode nd; nd.kind = K_STRING; nd.count = len; nd.a = slot; nd.b = slot;
        put(rel, nd, parent, (uint32_t)i);
      }
      i = e;
      ns++;
      return true;
    }
    if (c == '{' || c == '[') {
      if (sp >= kMaxDepth) { bad(BAD_DEPTH); return false; }
      const uint32_t is_map = c == '{';
      const uint32_t k = ci++;
      nc++;
      uint32_t cnt = 0, first = 0;
      if (MODE >= M_EMIT) {
        cnt = A.counts[cb + k];
        first = next;
        next += cnt;
      }
      if (MODE == M_EMIT) {
        DNode nd; nd.kind = is_map ? K_MAP : K_LIST; nd.count = cnt; nd.a = first; nd.b = 0;
        put(rel, nd, parent, 0);
      }
      i++;
      ws();
      if (T.at(i) == (is_map ? (uint32_t)'}' : (uint32_t)']')) {
        i++;
        if (MODE == M_COUNT) A.counts[cb + k] = 0;
        return true;
      }
      if (sp) st[sp - 1] = top;
      top.first = first; top.j = 0; top.slot = rel; top.k = k; top.map = is_map;
      sp++;
      return true;
    }
    const uint64_t L = plain_len(T, i);
    if (!L || !after_plain_ok(T.at(i + L))) return false;
    if (MODE == M_EMIT) {
      DNode nd; nd.kind = K_NULL; nd.count = 0; nd.a = 0; nd.b = 0;
      if (!scalar(T, i, L, nd)) { bad(BAD_NUMBER); return false; }
      put(rel, nd, parent, 0);
    }
    i += L;
    return true;
  };

  ws();
  const uint32_t c0 = T.at(i);
  if (c0 != '{' && c0 != '[') { bad(BAD_NOTJSON); return; }
  if (MODE == M_EMIT) {
    const bool list = c0 == '[';
    eline = list ? 0 : line; ecol = list ? 0 : column();   // emit_root: lists keep (0,0)
  }
  if (!value(0, NONE)) { bad(BAD_SYNTAX); return; }
  while (sp) {
    Frame& F = top;
    const uint32_t close = F.map ? '}' : ']';
    // one element of F
    const uint32_t cs = F.first + F.j;
    if (F.map) {
      if (T.at(i) != '"') { bad(BAD_SYNTAX); return; }
      const uint64_t kstart = i;
      const uint32_t kl = line, kc = column();
      uint32_t slot = 0, len = 0;
      const uint64_t e = string_at(&slot, &len);
      if (!e) { bad(BAD_SYNTAX); return; }
      i = e;
      ns++;
      if (MODE == M_EMIT) {
        ekey = slot; elen = len;
        ekpos = (uint32_t)kstart; ekl = kl; ekc = kc;
        // duplicate keys are found by the fix / verify pass; maps past its scan bound are refused
        if (F.j >= kMaxPairwiseKeys) { bad(BAD_WIDEMAP); return; }
      }
      while (T.at(i) == ' ') i++;
      if (T.at(i) != ':' || line != kl || i - kstart > 1000) { bad(BAD_SYNTAX); return; }
      i++;
      ws();
    } else if (MODE == M_EMIT) {
      ekey = NONE; elen = 0;
      ekpos = 0; ekl = 0; ekc = 0;
    }
    if (MODE == M_EMIT) { eline = line; ecol = column(); }
    F.j++;
    nn++;
    const uint32_t depth_before = sp;
    if (!value(cs, F.slot)) { bad(BAD_SYNTAX); return; }
    if (sp > depth_before) continue;   // a nested container: its elements come first
    // after an element: ',' or the close of this container (and of every container it completes)
    for (;;) {
      Frame& G = top;
      const uint32_t gclose = G.map ? '}' : ']';
      ws();
      const uint32_t c = T.at(i);
      if (c == ',') { i++; ws(); break; }
      if (c != gclose) { bad(BAD_SYNTAX); return; }
      i++;
      // container complete
      if (MODE == M_COUNT) {
        if (G.j > 0xFFFFu) { bad(BAD_WIDE); return; }
        A.counts[cb + G.k] = (uint16_t)G.j;
      }
      sp--;
      if (!sp) break;
      top = st[sp - 1];
    }
    (void)close;
  }
  ws();
  if (i != T.n) { bad(BAD_SYNTAX); return; }
  if (MODE == M_COUNT) { A.n_nodes[d] = nn; A.n_cont[d] = nc; A.n_str[d] = ns; }
}

#include "yaml_gpu.inc"

// resident waves per SIMD the passes are compiled for (their VGPR budget: 512 / waves)
#ifndef GG_JSON_WPE_COUNT
#define GG_JSON_WPE_COUNT 8
#endif
#ifndef GG_JSON_WPE_EMIT
#define GG_JSON_WPE_EMIT 6
#endif
#ifndef GG_JSON_WPE_FIX
#define GG_JSON_WPE_FIX 8
#endif
template <uint32_t MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == M_EMIT ? GG_JSON_WPE_EMIT : GG_JSON_WPE_COUNT)))
json_pass_kernel(JArgs A) {
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < A.ndocs; d += gridDim.x * blockDim.x) {
    if (*A.bad) return;
    parse_doc<MODE>(A, d);
  }
}

// pass 4: every occupied slot copies its first occurrence's decoded bytes into the pool
__global__ void __launch_bounds__(256) json_own_kernel(JArgs A) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s <= A.tmask; s += (uint64_t)gridDim.x * blockDim.x) {
    if (A.tkey[s] == 0) continue;
    const uint32_t len = A.tlen[s];
    const uint64_t need = len ? (len + 15ull) & ~15ull : 16ull;   // as DocBatch::intern
    const unsigned long long at = atomicAdd(A.pool_cursor, (unsigned long long)need);
    if (at + need > A.pool_cap || at + need > 0xF0000000ull) { refuse(A, BAD_POOL); A.tid[s] = 0; continue; }
    A.tid[s] = (uint32_t)at;
    const uint32_t doc = (uint32_t)(A.towner[s] >> 32), q = (uint32_t)A.towner[s];
    Text T(A.text, A.off[doc], A.off[doc + 1] - A.off[doc]);
    uint64_t p = at;
    uint32_t cont = 0;
    struct CopySink {
      uint8_t* pool;
      uint64_t p;
      __device__ void byte(uint32_t c) { pool[p++] = (uint8_t)c; }
      __device__ void run(const Text& T, uint32_t k, uint32_t r) {
        for (uint32_t u = 0; u < r; u++) pool[p++] = (uint8_t)(T.bytes4(k + u) & 0xFFu);
      }
    } cs{A.pool, p};
    decode_at(T, q, len, cs, cont);
  }
}

// the decoded bytes of the string whose opening quote is at q equal pool string `id` of `want` bytes
// (compared 4 bytes at a time: a pool string is 16-byte aligned and zero padded, json_own_kernel)
__device__ bool same_string(const JArgs& A, Text& T, uint64_t q, uint32_t id, uint32_t want) {
  struct CmpSink {
    WordStream ws;
    const uint32_t* pw;
    uint32_t want;
    bool same;
    __device__ void check(uint32_t w, uint32_t len) { if (len > want || pw[(len >> 2) - 1] != w) same = false; }
    __device__ void byte(uint32_t c) { ws.byte(c, [&](uint32_t w, uint32_t len) { check(w, len); }); }
    __device__ void run(const Text& T, uint32_t k, uint32_t r) { ws.run(T, k, r, [&](uint32_t w, uint32_t len) { check(w, len); }); }
  } cs{WordStream(), (const uint32_t*)(A.pool + id), want, true};
  uint32_t cont = 0;
  const uint64_t end = decode_at(T, q, want, cs, cont);
  const uint32_t pos = cs.ws.len;
  if ((pos & 3u) && (pos > want || cs.pw[pos >> 2] != cs.ws.word)) cs.same = false;
  return end && cs.same && pos == want;
}

// passes 5 + 6, one wave per document over its nodes (consecutive nodes' strings are neighbours in
// the text): table slots -> string ids (pool offsets), and every string occurrence's decoded bytes
// compared with its id's pool bytes, so a fingerprint collision cannot merge two strings silently
// (the document is refused and loads on the host)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GG_JSON_WPE_FIX))) json_fix_verify_kernel(JArgs A) {
  if (*A.bad) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t waves = (gridDim.x * blockDim.x) >> 6;
  DNode dead;   // the nodes a refused document left: placeholders whose key fields stay consistent
  dead.kind = K_NULL; dead.count = 0; dead.a = 0; dead.b = 0; dead.key_off = NONE; dead.key_len = 0; dead.key_hash = 0;
  dead.parent = NONE;
  for (uint32_t d = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; d < A.ndocs; d += waves) {
    const uint64_t nb = A.node_base[d], nn = A.n_nodes[d];
    auto kill = [&]() {
      for (uint64_t r = lane; r < nn; r += 64) {
        A.nodes[nb + r] = dead; A.line[nb + r] = 0; A.col[nb + r] = 0; A.kline[nb + r] = 0; A.kcol[nb + r] = 0;
      }
    };
    if (A.doc_bad[d]) { kill(); continue; }   // refused by the emit pass part way (count-pass refusals have no nodes)
    Text T(A.text, A.off[d], A.off[d + 1] - A.off[d]);
    bool ok = true, dup = false;
    for (uint64_t r = lane; r < nn; r += 64) {
      const NodeRec rec = A.recs[nb + r];
      DNode x = rec.n;
      if (x.key_off != NONE) {
        // duplicate map keys (the host fast path refuses them too; IndexMap keeps the last value):
        // this key's slot against its earlier siblings' (siblings are contiguous; the lanes of one
        // map read the same sibling at the same step)
        for (uint32_t q = A.recs[nb + x.parent].n.a; q < (uint32_t)r; q++)
          if (A.recs[nb + q].n.key_hash == x.key_hash) { dup = true; break; }
      }
      bool w = false;
      if (x.kind == K_STRING) {
        x.a = A.tid[x.a]; x.b = x.a; w = true;
        if (!same_string(A, T, rec.vpos, x.a, x.count)) ok = false;
      }
      if (x.key_off != NONE) {
        x.key_off = A.tid[x.key_off]; x.key_hash = x.key_off; w = true;
        if (!same_string(A, T, rec.kpos, x.key_off, x.key_len)) ok = false;
      }
      (void)w;
      A.nodes[nb + r] = x;
      A.line[nb + r] = rec.line; A.col[nb + r] = rec.col; A.kline[nb + r] = rec.kline; A.kcol[nb + r] = rec.kcol;
    }
    // a bytes mismatch explains an apparent duplicate (two keys of one map sharing a fingerprint): the
    // collision is the reason then; a duplicate whose occurrences all match their pool bytes is real
    const bool any_dup = __ballot(dup) != 0, any_bad = __ballot(!ok) != 0;
    if (any_dup || any_bad) {
      kill();
      if (lane == 0) A.doc_bad[d] = any_bad ? BAD_VERIFY : BAD_DUPKEY;
    }
  }
}

// the loader's passes run on the null stream; a pass may still be queued when an error unwinds the
// loader, so every array goes back to the block cache behind a fence on that stream (dev_cache.h)
template <typename T>
struct DevArr {
  T* p = nullptr;
  size_t n = 0;
  ~DevArr() { dev_free_on(p, nullptr); }
  void alloc(size_t count) {
    dev_free_on(p, nullptr);
    p = nullptr;
    n = count;
    JCHK(dev_alloc(&p, std::max<size_t>(count, 1) * sizeof(T)));
  }
};

uint32_t grid_for(uint64_t items, uint32_t block) {
  return (uint32_t)std::min<uint64_t>((items + block - 1) / block, 65536ull);
}

// Host <-> device transfers of the loader's bulk arrays through two pinned bounce buffers: the
// DMA of one chunk overlaps the host threads' copy of the other (hipMemcpy from / to pageable
// memory stages through the runtime at a few GB/s, single threaded).
// one copy stream per device for every load's staging, created on first use and kept for the process
inline hipStream_t staging_stream(int dev) {
  static std::mutex mu;
  static hipStream_t st[64] = {};
  if (dev < 0 || dev >= 64) dev = 0;
  std::lock_guard<std::mutex> lk(mu);
  if (!st[dev]) JCHK(hipStreamCreateWithFlags(&st[dev], hipStreamNonBlocking));
  return st[dev];
}
struct Staging {
  static constexpr size_t kChunk = 64ull << 20;
  void* pin[2] = {nullptr, nullptr};
  hipStream_t s = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int threads = 1;
  Staging() {
    int dev = 0;
    JCHK(hipGetDevice(&dev));
    for (int i = 0; i < 2; i++)
      if (!(pin[i] = pinned_get(kChunk, dev))) throw std::runtime_error("pinned host staging: allocation failed");
    s = staging_stream(dev);
    JCHK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    JCHK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  }
  ~Staging() {
    if (s) hipStreamSynchronize(s);   // the stream stays (staging_stream): no create / destroy per load
    // back to the process-wide pinned cache: a streamed batch loads a chunk while another chunk's report runs,
    // and unpinning (hipHostUnregister) at the end of every load stalled it behind that report
    // (profiles/r06zi_stream_load_trace.log: 64-540 ms between the index and the loader's return)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    for (int i = 0; i < 2; i++) { pinned_put(pin[i], kChunk, dev); if (ev[i]) hipEventDestroy(ev[i]); }
  }
  // fn(t, nthreads) on `threads` host threads
  template <typename F>
  void par(F fn) {
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(fn, t, threads);
    fn(0, threads);
    for (auto& x : th) x.join();
  }
  void copy_par(void* dst, const void* src, size_t n) {
    par([&](int t, int nt) {
      size_t a = n * t / nt, b = n * (t + 1) / nt;
      if (b > a) memcpy((char*)dst + a, (const char*)src + a, b - a);
    });
  }
  void d2h(void* dst, const void* src, size_t bytes) {
    const size_t nch = (bytes + kChunk - 1) / kChunk;
    auto issue = [&](size_t i) {
      const size_t o = i * kChunk, n = std::min(kChunk, bytes - o);
      JCHK(hipMemcpyAsync(pin[i & 1], (const char*)src + o, n, hipMemcpyDeviceToHost, s));
      JCHK(hipEventRecord(ev[i & 1], s));
    };
    if (nch) issue(0);
    for (size_t i = 0; i < nch; i++) {
      JCHK(hipEventSynchronize(ev[i & 1]));
      if (i + 1 < nch) issue(i + 1);   // the other buffer: its chunk was copied out last iteration
      const size_t o = i * kChunk;
      copy_par((char*)dst + o, pin[i & 1], std::min(kChunk, bytes - o));
    }
  }
  // documents packed back to back into device memory `dst` (offsets off[]), 16 zero bytes after
  void h2d_docs(uint8_t* dst, const char* const* texts, const size_t* lens, const uint64_t* off, size_t n) {
    const uint64_t total = off[n] + 16;
    size_t doc = 0;
    for (size_t i = 0; i * kChunk < total; i++) {
      const uint64_t lo = i * kChunk, hi = std::min<uint64_t>(total, lo + kChunk);
      if (i >= 2) JCHK(hipEventSynchronize(ev[i & 1]));   // this buffer's previous DMA is done
      char* buf = (char*)pin[i & 1];
      while (doc < n && off[doc + 1] <= lo) doc++;
      const size_t d0 = doc;
      par([&](int t, int nt) {
        // bytes [lo, hi) of the packed stream, split by byte range over the threads
        const uint64_t a = lo + (hi - lo) * t / nt, b = lo + (hi - lo) * (t + 1) / nt;
        size_t d = d0;
        while (d < n && off[d + 1] <= a) d++;
        for (uint64_t p = a; p < b;) {
          if (d >= n) { memset(buf + (p - lo), 0, b - p); break; }
          const uint64_t e = std::min<uint64_t>(b, off[d + 1]);
          memcpy(buf + (p - lo), texts[d] + (p - off[d]), e - p);
          p = e;
          d++;
        }
      });
      JCHK(hipMemcpyAsync(dst + lo, buf, hi - lo, hipMemcpyHostToDevice, s));
      JCHK(hipEventRecord(ev[i & 1], s));
    }
    JCHK(hipStreamSynchronize(s));
  }
};

}  // namespace

// root.Resources of every document of a device-resident arena (the scan session_upload runs over host
// nodes otherwise): rmap[d] = document-relative node of the entry (NONE: none, or not a map), cnt[d] =
// its entry count.  The first entry keyed `rkey` decides, as on the host.
__global__ void __launch_bounds__(256) root_resources_kernel(const DNode* nodes, const uint64_t* base, const uint32_t* roots,
                                                             uint32_t nd, uint32_t rkey, uint32_t* rmap, uint32_t* cnt) {
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < nd; d += gridDim.x * blockDim.x) {
    const DNode* N = nodes + base[d];
    const DNode root = N[roots[d]];
    uint32_t r = NONE, c = 0;
    if (root.kind == K_MAP) {
      for (uint32_t k = 0; k < root.count; k++) {
        const DNode e = N[root.a + k];
        if (e.key_hash != rkey) continue;
        if (e.kind == K_MAP) { r = root.a + k; c = e.count; }
        break;
      }
    }
    rmap[d] = r;
    cnt[d] = c;
  }
}

bool gpu_load_json(DocBatch& out, const char* const* texts, const size_t* lens, const std::vector<std::string>& names,
                   size_t n, GpuLoadStats& st, std::string& why, std::vector<uint32_t>* refused,
                   void** keep_nodes, ResidentArena* resident) {
  if (resident) *resident = ResidentArena{};
  if (!keep_nodes) resident = nullptr;   // the columns stay only beside the nodes
  static const char* kWhy[] = {"", "outside the strict-JSON subset", "nesting deeper than 64", "duplicate map keys",
                               "a number the host types (beyond 64 bits, or an infinite / undecided float)", "string table full", "string pool full",
                               "string fingerprint collision", "batch too large", "a container with more than 65535 elements",
                               "not a JSON document (YAML device parser off)", "outside the block-style YAML subset",
                               "a map with more than 256 keys"};
  if (!out.nodes.empty() || !out.roots.empty()) { why = "the device loader fills an empty batch"; return false; }
  if (n == 0) return true;
  if (n > 0xFFFFFFF0ull) { why = kWhy[BAD_SIZE]; return false; }
  // documents back to back, 16 zero bytes of padding for the 16-byte window
  std::vector<uint64_t> off(n + 1, 0);
  for (size_t k = 0; k < n; k++) {
    if (lens[k] > 0xFFFFFFF0ull) { why = kWhy[BAD_SIZE]; return false; }
    off[k + 1] = off[k] + lens[k];
  }
  const uint64_t total = off[n];
  st.text_bytes = total;
  // one Staging per device, kept between loads (hipHostFree waits for the device to go idle, as hipFree
  // does); a concurrent load on the same device builds its own
  static std::mutex stg_mu[64];
  static Staging* stg_cache[64];
  int cur_dev = 0;
  if (hipGetDevice(&cur_dev) != hipSuccess) cur_dev = 0;
  cur_dev &= 63;
  std::unique_lock<std::mutex> stg_lk(stg_mu[cur_dev], std::try_to_lock);
  std::unique_ptr<Staging> stg_own;
  if (stg_lk.owns_lock() && !stg_cache[cur_dev]) stg_cache[cur_dev] = new Staging;
  if (!stg_lk.owns_lock()) stg_own.reset(new Staging);
  Staging& stg = stg_lk.owns_lock() ? *stg_cache[cur_dev] : *stg_own;
  // GG_LOAD_TRACE=1: wall-clock phase marks on stderr
  const bool trace = getenv("GG_LOAD_TRACE") != nullptr;
  const auto tw = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (trace) fprintf(stderr, "[load] %-22s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count());
  };

  hipEvent_t e0, e1;
  JCHK(hipEventCreate(&e0));
  JCHK(hipEventCreate(&e1));
  auto t0 = std::chrono::steady_clock::now();
  DevArr<uint8_t> d_text; d_text.alloc(total + 16);
  DevArr<uint64_t> d_off; d_off.alloc(n + 1);
  stg.h2d_docs(d_text.p, texts, lens, off.data(), n);
  JCHK(hipMemcpy(d_off.p, off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
  st.h2d_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  mark("h2d");

  DevArr<uint32_t> d_nn, d_nc, d_ns, d_bad, d_doc_bad, d_doc_bad0;
  DevArr<uint8_t> d_yaml;
  d_nn.alloc(n); d_nc.alloc(n); d_ns.alloc(n); d_bad.alloc(1); d_doc_bad.alloc(n); d_doc_bad0.alloc(n); d_yaml.alloc(n);
  JCHK(hipMemset(d_bad.p, 0, 4));
  JCHK(hipMemset(d_doc_bad.p, 0, n * 4));
  JCHK(hipMemset(d_yaml.p, 0, n));
  DevArr<uint32_t> d_bad_at;
  const bool diag = getenv("GG_LOAD_DIAG") != nullptr;
  if (diag) { d_bad_at.alloc(n); JCHK(hipMemset(d_bad_at.p, 0xFF, n * 4)); }
  // block-style YAML documents parse on the device too (yaml_gpu.inc) unless GG_YAML_DEVICE=0
  const bool yaml_on = !getenv("GG_YAML_DEVICE") || atoi(getenv("GG_YAML_DEVICE")) != 0;
  JArgs A{};
  A.text = d_text.p; A.off = d_off.p; A.ndocs = (uint32_t)n;
  A.fp_mask = ~0ull;
  if (const char* e = getenv("GG_JSON_FP_MASK")) {
    // tests only: narrowed fingerprints collide, and every colliding document falls back to the host
    A.fp_mask = strtoull(e, nullptr, 0);
    static bool warned = false;
    if (!warned) { warned = true; fprintf(stderr, "cfn-guard-mi355x: GG_JSON_FP_MASK=%s narrows the device loader's string fingerprints (test setting)\n", e); }
  }
  A.n_nodes = d_nn.p; A.n_cont = d_nc.p; A.n_str = d_ns.p; A.bad = d_bad.p; A.doc_bad = d_doc_bad.p; A.is_yaml = d_yaml.p; A.bad_at = diag ? d_bad_at.p : nullptr;
  DevArr<uint16_t> d_counts; d_counts.alloc(total / 2 + 1);
  A.counts = d_counts.p;
  const uint32_t dgrid = grid_for(n, 256);
  float ms_total = 0, ms = 0;
  auto bad_now = [&]() {
    uint32_t b = 0;
    JCHK(hipMemcpy(&b, d_bad.p, 4, hipMemcpyDeviceToHost));
    if (b) why = b < 13 ? kWhy[b] : "refused";
    return b != 0;
  };

  // 1. count
  JCHK(hipEventRecord(e0));
  hipLaunchKernelGGL(json_pass_kernel<M_COUNT>, dim3(dgrid), dim3(256), 0, 0, A);
  JCHK(hipGetLastError());
  if (yaml_on) {
    hipLaunchKernelGGL(yaml_pass_kernel<M_COUNT>, dim3(dgrid), dim3(256), 0, 0, A);
    JCHK(hipGetLastError());
  }
  JCHK(hipEventRecord(e1));
  JCHK(hipEventSynchronize(e1));
  JCHK(hipEventElapsedTime(&ms, e0, e1)); ms_total += ms;
  mark("count pass");
  if (bad_now()) return false;
  // the count pass's per-document refusals; a table / pool retry starts again from them
  JCHK(hipMemcpy(d_doc_bad0.p, d_doc_bad.p, n * 4, hipMemcpyDeviceToDevice));
  std::vector<uint32_t> nn(n), nc(n), ns(n);
  JCHK(hipMemcpy(nn.data(), d_nn.p, n * 4, hipMemcpyDeviceToHost));
  JCHK(hipMemcpy(nc.data(), d_nc.p, n * 4, hipMemcpyDeviceToHost));
  JCHK(hipMemcpy(ns.data(), d_ns.p, n * 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> nbase(n);
  uint64_t N = 0, S = 0;
  for (size_t k = 0; k < n; k++) {
    if (nn[k] > kMaxDocNodes) { why = kWhy[BAD_SIZE]; return false; }
    nbase[k] = N;
    N += nn[k]; S += ns[k];
  }
  // the host columns are sized (page faults, seconds at 1M documents) while the device passes run; one
  // thread per column.  A device-resident arena sizes them only if a document is refused (the host
  // loader's documents are merged into host columns).
  auto size_columns = [&out, N]() {
    std::thread a([&]() { out.nodes.resize(N); });
    std::thread b([&]() { out.line.resize(N); out.col.resize(N); });
    out.kline.resize(N); out.kcol.resize(N);
    a.join(); b.join();
  };
  std::thread resizer;
  if (!resident) resizer = std::thread(size_columns);
  struct Joiner { std::thread& t; ~Joiner() { if (t.joinable()) t.join(); } } join_resizer{resizer};
  mark("count D2H + scan");
  DevArr<uint64_t> d_nbase;
  d_nbase.alloc(n);
  JCHK(hipMemcpy(d_nbase.p, nbase.data(), n * 8, hipMemcpyHostToDevice));
  DevArr<DNode> d_nodes; d_nodes.alloc(N);
  DevArr<uint32_t> d_line, d_col, d_kline, d_kcol;
  d_line.alloc(N); d_col.alloc(N); d_kline.alloc(N); d_kcol.alloc(N);
  // Intern table: 2 slots per string occurrence, between 2^16 and 2^23 slots to start with (at
  // most 64 MB of keys, so the probes hit the L2 / Infinity Cache instead of HBM: templates repeat
  // their keys and values, distinct strings are a few per cent of the occurrences).  A full table
  // doubles and the table passes run again, up to 2 slots per occurrence or 2^28 slots.
  uint32_t start_log = 23;
  if (const char* e = getenv("GG_JSON_TABLE_LOG")) start_log = (uint32_t)std::max(16, std::min(28, atoi(e)));   // tests
  uint64_t tslots = 1ull << 16;
  while (tslots < 2 * S && tslots < (1ull << start_log)) tslots <<= 1;
  DevArr<unsigned long long> d_tkey, d_towner, d_pool_cursor;
  DevArr<uint32_t> d_tlen, d_tid;
  d_pool_cursor.alloc(1);
  // pool: a quarter of the text to start with (templates repeat their strings); doubles when full,
  // up to the bound every distinct string fits in (its bytes + 16 of alignment padding)
  const uint64_t pool_max = std::min<uint64_t>(total + 16 * S + 16, 0xF0000000ull);
  uint64_t pool_cap = std::min<uint64_t>(std::max<uint64_t>(total / 4, 1ull << 20), pool_max);
  DevArr<uint8_t> d_pool;
  A.node_base = d_nbase.p; A.nodes = d_nodes.p;
  DevArr<NodeRec> d_recs;
  d_recs.alloc(N);
  A.recs = d_recs.p;
  A.line = d_line.p; A.col = d_col.p; A.kline = d_kline.p; A.kcol = d_kcol.p;
  mark("device allocs");
  for (;;) {
    if (d_pool.n != pool_cap + 16) d_pool.alloc(pool_cap + 16);
    A.pool = d_pool.p; A.pool_cursor = d_pool_cursor.p; A.pool_cap = pool_cap;
    d_tkey.alloc(tslots); d_towner.alloc(tslots); d_tlen.alloc(tslots); d_tid.alloc(tslots);
    JCHK(hipMemset(d_tkey.p, 0, tslots * 8));
    JCHK(hipMemset(d_pool_cursor.p, 0, 8));
    JCHK(hipMemset(d_pool.p, 0, pool_cap + 16));
    JCHK(hipMemcpy(d_doc_bad.p, d_doc_bad0.p, n * 4, hipMemcpyDeviceToDevice));
    A.tkey = d_tkey.p; A.tlen = d_tlen.p; A.towner = d_towner.p; A.tid = d_tid.p; A.tmask = tslots - 1;

    // 2. emit, 3. own, 4. fix + verify
    JCHK(hipEventRecord(e0));
    hipLaunchKernelGGL(json_pass_kernel<M_EMIT>, dim3(dgrid), dim3(256), 0, 0, A);
    if (yaml_on) hipLaunchKernelGGL(yaml_pass_kernel<M_EMIT>, dim3(dgrid), dim3(256), 0, 0, A);
#if !GG_JDIAG_NOINTERN
    hipLaunchKernelGGL(json_own_kernel, dim3(grid_for(tslots, 256)), dim3(256), 0, 0, A);
    hipLaunchKernelGGL(json_fix_verify_kernel, dim3(grid_for(n * 64ull, 256)), dim3(256), 0, 0, A);
#else
    { const uint32_t diag = BAD_SIZE; JCHK(hipMemcpy(d_bad.p, &diag, 4, hipMemcpyHostToDevice)); }
#endif
    JCHK(hipGetLastError());
    JCHK(hipEventRecord(e1));
    JCHK(hipEventSynchronize(e1));
    JCHK(hipEventElapsedTime(&ms, e0, e1)); ms_total += ms;
    uint32_t b = 0;
    JCHK(hipMemcpy(&b, d_bad.p, 4, hipMemcpyDeviceToHost));
    if (b == BAD_TABLE && tslots < 2 * S && tslots < (1ull << 28)) {
      tslots <<= 1;
      JCHK(hipMemset(d_bad.p, 0, 4));
      st.table_retries++;
      continue;
    }
    if (b == BAD_POOL && pool_cap < pool_max) {
      pool_cap = std::min<uint64_t>(pool_cap * 2, pool_max);
      JCHK(hipMemset(d_bad.p, 0, 4));
      st.table_retries++;
      continue;
    }
    break;
  }
  st.kernel_ms = ms_total;
  mark("emit/own/fix passes");
  JCHK(hipEventDestroy(e0));
  JCHK(hipEventDestroy(e1));
  if (bad_now()) {
    if (resizer.joinable()) resizer.join();
    out.clear();   // refused: the batch stays empty
    return false;
  }
  std::vector<uint32_t> doc_bad(n);
  JCHK(hipMemcpy(doc_bad.data(), d_doc_bad.p, n * 4, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < n; k++) {
    if (!doc_bad[k]) continue;
    if (!refused) {   // strict: one refused document refuses the batch
      why = doc_bad[k] < 13 ? kWhy[doc_bad[k]] : "refused";
      if (diag) {
        uint32_t at = 0;
        JCHK(hipMemcpy(&at, d_bad_at.p + k, 4, hipMemcpyDeviceToHost));
        why += " (document " + std::to_string(k);
        if (at != 0xFFFFFFFFu && at <= lens[k]) {
          const size_t a = at > 40 ? at - 40 : 0;
          why += ", byte " + std::to_string(at) + ": ..." + std::string(texts[k] + a, std::min<size_t>(lens[k] - a, 80)) + "...";
        }
        why += ")";
      }
      if (resizer.joinable()) resizer.join();
      out.clear();
      return false;
    }
    refused->push_back((uint32_t)k);
  }
  st.refused_docs = refused ? refused->size() : 0;
  mark("doc_bad");

  // results to the host batch (the host keeps the reporter's columns and the intern index)
  t0 = std::chrono::steady_clock::now();
  unsigned long long pool_used = 0;
  JCHK(hipMemcpy(&pool_used, d_pool_cursor.p, 8, hipMemcpyDeviceToHost));
  mark("pre-join");
  if (resident && refused && !refused->empty()) resident = nullptr;   // host documents join: host columns
  if (resident) {
    resident->line = d_line.p; resident->col = d_col.p; resident->kline = d_kline.p; resident->kcol = d_kcol.p;
    resident->nodes = N;
    d_line.p = d_col.p = d_kline.p = d_kcol.p = nullptr;
  } else {
    if (resizer.joinable()) resizer.join(); else size_columns();
    mark("columns sized");
    stg.d2h(out.nodes.data(), d_nodes.p, N * sizeof(DNode));
    stg.d2h(out.line.data(), d_line.p, N * 4);
    stg.d2h(out.col.data(), d_col.p, N * 4);
    stg.d2h(out.kline.data(), d_kline.p, N * 4);
    stg.d2h(out.kcol.data(), d_kcol.p, N * 4);
  }
  out.bytes.resize(pool_used);
  if (pool_used) stg.d2h(&out.bytes[0], d_pool.p, pool_used);
  mark("arena D2H");
  std::vector<unsigned long long> tkey(tslots);
  std::vector<uint32_t> tlen(tslots), tid(tslots);
  JCHK(hipMemcpy(tkey.data(), d_tkey.p, tslots * 8, hipMemcpyDeviceToHost));
  JCHK(hipMemcpy(tlen.data(), d_tlen.p, tslots * 4, hipMemcpyDeviceToHost));
  JCHK(hipMemcpy(tid.data(), d_tid.p, tslots * 4, hipMemcpyDeviceToHost));
  st.d2h_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  mark("table D2H");
  uint64_t distinct = 0;
  {
    std::vector<uint32_t> aoff, alen;
    aoff.reserve(tslots / 2); alen.reserve(tslots / 2);
    for (uint64_t s = 0; s < tslots; s++) if (tkey[s]) { aoff.push_back(tid[s]); alen.push_back(tlen[s]); }
    distinct = aoff.size();
    mark("table scan");
    out.adopt_bulk(aoff.data(), alen.data(), aoff.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    mark("index built");
  }
  out.roots.assign(n, 0);
  out.base.assign(nbase.begin(), nbase.end());
  out.names.assign(names.begin(), names.begin() + n);
  st.nodes = N; st.distinct_strings = distinct; st.pool_bytes = pool_used;
  mark("adopt + names");
  if (keep_nodes) { *keep_nodes = d_nodes.p; d_nodes.p = nullptr; }
  return true;
}

}  // namespace gg
