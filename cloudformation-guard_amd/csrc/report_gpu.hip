// The structured JSON report rendered on the MI355X (see report_gpu.h).  Device restatement of
// reporter.cpp's streamed JSON writer: JW (serde_json PrettyFormatter), write_value / write_pav /
// write_unresolved, StreamWalker::items and write_file_report, R's Display / message helpers.
// Reference: guard/src/rules/eval_context.rs:1965-2435 (report_all_failed_clauses_for_rules,
// simplified_json_from_root), reporters/validate/structured.rs:99-133, rules/display.rs:33-107,
// path_value.rs:864-880 (PathAwareValue serde), rules/mod.rs:165-177 (UnResolved serde).
#include <hip/hip_runtime.h>

#include "report_gpu.h"

namespace gg {
namespace rg {

#define RD __device__ __attribute__((always_inline)) inline

static const uint32_t SYN_BIT = 0x40000000u;
static const uint32_t KEY_BIT = 0x20000000u;
static const uint32_t kMaxDepth = 48;   // JSON nesting a document may reach on the device (else the host writes it)

// fallback reasons (W.fb): why the host writer takes a document
enum : uint32_t { FB_NONE = 0, FB_FLOAT = 1, FB_DEBUG = 2, FB_REF = 3, FB_KIND = 4, FB_DEPTH = 5 };

// ---------------------------------------------------------------------------------- writer ---
// p == null: the size pass (only counts).  JW state: `depth` open containers, bit i of `first`: container
// i has no item yet; container i is indented base + i.  Text inside a JSON string goes through the
// dot-bracket filter (REC_IN's message) and serde's escaping.
struct W {
  char* p;          // the document's text, or null: the size pass (count only)
  uint64_t n;       // bytes produced
  uint32_t fb;
  uint32_t depth, base;
  uint64_t first;
  bool esc, dotf, held;
};

// (every writer function is inlined into the kernels: a W passed to a real call would live in scratch and
// every byte would become scratch traffic; the byte-level functions stay trivial so the inlined kernels
// compile in reasonable time)
#define RN RD
RD void raw(W& w, char c) {
  if (w.p) w.p[w.n] = c;
  w.n++;
}
RD void raws(W& w, const char* s) { for (; *s; s++) raw(w, *s); }
RD void spaces(W& w, uint32_t k) {
  if (w.p) for (uint32_t i = 0; i < k; i++) w.p[w.n + i] = ' ';
  w.n += k;
}
// serde_json's string escaping of one byte
RD void esc1(W& w, unsigned char c) {
  if (c >= 0x20 && c != '"' && c != '\\') { raw(w, (char)c); return; }
  raw(w, '\\');
  switch (c) {
    case '"': raw(w, '"'); return;
    case '\\': raw(w, '\\'); return;
    case '\n': raw(w, 'n'); return;
    case '\r': raw(w, 'r'); return;
    case '\t': raw(w, 't'); return;
    case 0x08: raw(w, 'b'); return;
    case 0x0C: raw(w, 'f'); return;
    default: {
      const char* hx = "0123456789abcdef";
      raw(w, 'u'); raw(w, '0'); raw(w, '0'); raw(w, hx[c >> 4]); raw(w, hx[c & 15]);
    }
  }
}
// 8 bytes none of which serde escapes (< 0x20, '"', '\\'); bytes >= 0x80 (UTF-8) pass
RD bool plain8(uint64_t x) {
  const uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
  const uint64_t lt = (x - ones * 0x20u) & ~x & highs;
  const uint64_t q = x ^ (ones * (uint64_t)'"'), b = x ^ (ones * (uint64_t)'\\');
  return !(lt | ((q - ones) & ~q & highs) | ((b - ones) & ~b & highs));
}
// n bytes at s, escaped or not; a 16-byte aligned source (the interned string pool: strings start
// 16-byte aligned and are zero-padded) is read 16 bytes at a time
RD void bulk(W& w, const char* s, uint32_t n, bool escape) {
  uint32_t i = 0;
  if ((((uintptr_t)s) & 15u) == 0) {
    for (; i < n; i += 16) {
      const uint4 q = *(const uint4*)(s + i);
      const uint64_t lo = (uint64_t)q.x | ((uint64_t)q.y << 32), hi = (uint64_t)q.z | ((uint64_t)q.w << 32);
      const uint32_t m = n - i < 16 ? n - i : 16;
      const bool plain = !escape || (plain8(lo) && plain8(hi));
#pragma unroll 1
      for (uint32_t k = 0; k < m; k++) {
        const char c = (char)((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8))) & 0xFF);
        if (plain) raw(w, c); else esc1(w, (unsigned char)c);
      }
    }
    return;
  }
#pragma unroll 1
  for (; i < n; i++) { if (escape) esc1(w, (unsigned char)s[i]); else raw(w, s[i]); }
}
RD void emit(W& w, char c) { if (w.esc) esc1(w, (unsigned char)c); else raw(w, c); }
// a text character: through the dot filter ('.' dropped before '['), then the escaping
RD void tput(W& w, char c) {
  if (w.dotf) {
    if (w.held) { w.held = false; if (c != '[') emit(w, '.'); }
    if (c == '.') { w.held = true; return; }
  }
  emit(w, c);
}
RN void tlit(W& w, const char* s) { for (; *s; s++) tput(w, *s); }
RD void tstr(W& w, const char* s, uint32_t n) {
  if (!w.dotf) { bulk(w, s, n, w.esc); return; }
  for (uint32_t i = 0; i < n; i++) tput(w, s[i]);
}
RN void tu64(W& w, uint64_t v) {
  char b[24];
  int k = 0;
  do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (k) tput(w, b[--k]);
}
RD void ti64(W& w, int64_t v) {
  if (v < 0) { tput(w, '-'); tu64(w, (uint64_t)0 - (uint64_t)v); } else tu64(w, (uint64_t)v);
}
RD void sbeg(W& w) { raw(w, '"'); w.esc = true; }
RD void send(W& w) {
  if (w.held) { w.held = false; emit(w, '.'); }
  w.dotf = false;
  w.esc = false;
  raw(w, '"');
}
RD void jstr(W& w, const char* s, uint32_t n) { raw(w, '"'); bulk(w, s, n, true); raw(w, '"'); }
RN void jlit(W& w, const char* s) { raw(w, '"'); for (; *s; s++) esc1(w, (unsigned char)*s); raw(w, '"'); }

// JW (reporter.cpp): open / close / item / key
RD void open(W& w, char c) {
  raw(w, c);
  if (w.depth >= 63) { w.fb = FB_DEPTH; return; }
  w.first |= 1ull << w.depth;
  w.depth++;
}
RD void close(W& w, char c) {
  if (w.depth == 0) { w.fb = FB_DEPTH; return; }
  w.depth--;
  if (!((w.first >> w.depth) & 1ull)) { raw(w, '\n'); spaces(w, 2 * (w.base + w.depth)); }
  raw(w, c);
}
RD void item(W& w) {
  if (w.depth == 0) { w.fb = FB_DEPTH; return; }
  const uint32_t L = w.depth - 1;
  if ((w.first >> L) & 1ull) { raw(w, '\n'); w.first &= ~(1ull << L); }
  else { raw(w, ','); raw(w, '\n'); }
  spaces(w, 2 * (w.base + L + 1));
}
RD void key(W& w, const char* k) { item(w); raw(w, '"'); raws(w, k); raw(w, '"'); raw(w, ':'); raw(w, ' '); }
RD void jnull(W& w) { raws(w, "null"); }
__device__ const char* const kCmp[] = {"Eq", "In", "Gt", "Lt", "Le", "Ge", "Exists", "Empty", "IsString", "IsList", "IsMap",
                                      "IsBool", "IsInt", "IsFloat", "IsNull"};
RN void cmp(W& w, uint32_t op, bool neg) {
  open(w, '[');
  item(w); raw(w, '"'); raws(w, op < 15 ? kCmp[op] : "Eq"); raw(w, '"');
  item(w); raws(w, neg ? "true" : "false");
  close(w, ']');
}

// ---------------------------------------------------------------------------------- values ---
struct Ctx {
  const RenderArgs* A;
  const RProg* P;
  uint64_t dbase;   // global index of the document's first node
};
struct NV { uint32_t kind, count, a, b, key_off, key_len, parent; };

// node `ref` (document-relative, or LIT_BIT | literal index); false for refs the device writer leaves to
// the host (a map key or a count() value as a value)
RD bool nv(const Ctx& c, uint32_t ref, NV& n) {
  if (ref == NONE || (ref & (SYN_BIT | KEY_BIT))) return false;
  if (ref & LIT_BIT) {
    if ((ref & ~LIT_BIT) >= c.P->n_lit) return false;
    const DNode d = c.P->lit[ref & ~LIT_BIT];
    n.kind = d.kind; n.count = d.count; n.a = d.a; n.b = d.b; n.key_off = d.key_off; n.key_len = d.key_len; n.parent = d.parent;
    return true;
  }
  const uint64_t g = c.dbase + ref;
  if (g >= c.A->n_nodes) return false;
  const DNodeP p = c.A->nodes[g];
  n.kind = p.kc & 15u; n.count = p.kc >> 4; n.a = p.a; n.b = p.b; n.key_off = p.key_hash; n.key_len = c.A->klen[g];
  n.parent = c.A->parent[g];
  return true;
}
RD const char* bytes_of(const Ctx& c, uint32_t ref) { return (ref & LIT_BIT) ? c.P->lit_bytes : c.A->pool; }
RD uint32_t child(uint32_t ref, const NV& n, uint32_t j) { return (ref & LIT_BIT) | (n.a + j); }
RD int64_t ival(const NV& n) { return (int64_t)(((uint64_t)n.b << 32) | n.a); }
RD uint32_t line_of(const Ctx& c, uint32_t ref) { return (ref & LIT_BIT) ? c.P->lit_line[ref & ~LIT_BIT] : c.A->line[c.dbase + ref]; }
RD uint32_t col_of(const Ctx& c, uint32_t ref) { return (ref & LIT_BIT) ? c.P->lit_col[ref & ~LIT_BIT] : c.A->col[c.dbase + ref]; }

RD const char* type_info(uint32_t k) {
  switch (k) {
    case K_NULL: return "null";
    case K_STRING: return "String";
    case K_REGEX: return "Regex";
    case K_BOOL: return "bool";
    case K_INT: return "int";
    case K_FLOAT: return "float";
    case K_CHAR: return "char";
    case K_LIST: return "array";
    case K_MAP: return "map";
    case K_RANGE_INT: return "range(int, int)";
    case K_RANGE_FLOAT: return "range(float, float)";
    default: return "range(char, char)";
  }
}

// JSON pointer of `ref` (DocBatch::path): the ancestors' keys / indices, root first
RN void path(W& w, const Ctx& c, uint32_t ref) {
  uint32_t chain[64];
  uint32_t n = 0;
  NV v;
  if (!nv(c, ref, v)) { w.fb = FB_REF; return; }
  uint32_t cur = ref;
  while (v.parent != NONE) {
    if (n == 64) { w.fb = FB_DEPTH; return; }
    chain[n++] = cur;
    cur = (ref & LIT_BIT) | v.parent;
    if (!nv(c, cur, v)) { w.fb = FB_REF; return; }
  }
  for (uint32_t i = n; i-- > 0;) {
    NV x, p;
    nv(c, chain[i], x);
    nv(c, (ref & LIT_BIT) | x.parent, p);
    tput(w, '/');
    if (p.kind == K_MAP) tstr(w, bytes_of(c, chain[i]) + x.key_off, x.key_len);
    else tu64(w, (chain[i] & ~LIT_BIT) - p.a);
  }
}
RD void loc(W& w, uint32_t l, uint32_t col) { tlit(w, "[L:"); tu64(w, l); tlit(w, ",C:"); tu64(w, col); tput(w, ']'); }
RN void path_display(W& w, const Ctx& c, uint32_t ref) {
  path(w, c, ref);
  if (!w.fb) loc(w, line_of(c, ref), col_of(c, ref));
}

// serde of a value (R::value_json / write_value): pretty JSON through the JW state
RN void write_value(W& w, const Ctx& c, uint32_t ref) {
  uint32_t sref[kMaxDepth], sj[kMaxDepth];
  uint32_t sp = 0;
  uint32_t cur = ref;
  for (;;) {
    // write `cur`; containers are entered
    NV n;
    if (!nv(c, cur, n)) { w.fb = FB_REF; return; }
    bool entered = false;
    switch (n.kind) {
      case K_NULL: jnull(w); break;
      case K_STRING: jstr(w, bytes_of(c, cur) + n.a, n.count); break;
      case K_REGEX: raw(w, '"'); esc1(w, '/'); for (uint32_t i = 0; i < n.count; i++) esc1(w, (unsigned char)bytes_of(c, cur)[n.a + i]); esc1(w, '/'); raw(w, '"'); break;
      case K_BOOL: raws(w, n.a ? "true" : "false"); break;
      case K_INT: { const bool e = w.esc; w.esc = false; ti64(w, ival(n)); w.esc = e; break; }
      case K_LIST:
      case K_MAP:
        if (sp == kMaxDepth) { w.fb = FB_DEPTH; return; }
        open(w, n.kind == K_LIST ? '[' : '{');
        sref[sp] = cur; sj[sp] = 0; sp++;
        entered = true;
        break;
      case K_FLOAT: w.fb = FB_FLOAT; return;
      default: w.fb = FB_KIND; return;
    }
    (void)entered;
    if (w.fb) return;
    // next: the first unvisited child of the innermost open container, closing finished ones
    for (;;) {
      if (sp == 0) return;
      NV m;
      nv(c, sref[sp - 1], m);
      if (sj[sp - 1] < m.count) {
        const uint32_t ch = child(sref[sp - 1], m, sj[sp - 1]++);
        item(w);
        if (m.kind == K_MAP) {
          NV k;
          nv(c, ch, k);
          jstr(w, bytes_of(c, ch) + k.key_off, k.key_len);
          raw(w, ':'); raw(w, ' ');
        }
        cur = ch;
        break;
      }
      close(w, m.kind == K_LIST ? ']' : '}');
      sp--;
    }
  }
}

// ValueOnlyDisplay (display.rs:33-107) into the current text
RN void value_only(W& w, const Ctx& c, uint32_t ref) {
  uint32_t sref[kMaxDepth], sj[kMaxDepth];
  uint32_t sp = 0;
  uint32_t cur = ref;
  for (;;) {
    NV n;
    if (!nv(c, cur, n)) { w.fb = FB_REF; return; }
    switch (n.kind) {
      case K_NULL: tlit(w, "\"NULL\""); break;
      case K_STRING: tput(w, '"'); tstr(w, bytes_of(c, cur) + n.a, n.count); tput(w, '"'); break;
      case K_REGEX: tlit(w, "\"/"); tstr(w, bytes_of(c, cur) + n.a, n.count); tlit(w, "/\""); break;
      case K_BOOL: tlit(w, n.a ? "true" : "false"); break;
      case K_INT: ti64(w, ival(n)); break;
      case K_LIST:
      case K_MAP:
        if (sp == kMaxDepth) { w.fb = FB_DEPTH; return; }
        tput(w, n.kind == K_LIST ? '[' : '{');
        sref[sp] = cur; sj[sp] = 0; sp++;
        break;
      case K_FLOAT: w.fb = FB_FLOAT; return;
      default: w.fb = FB_KIND; return;
    }
    if (w.fb) return;
    for (;;) {
      if (sp == 0) return;
      NV m;
      nv(c, sref[sp - 1], m);
      if (sj[sp - 1] < m.count) {
        const uint32_t j = sj[sp - 1]++;
        const uint32_t ch = child(sref[sp - 1], m, j);
        if (j) tput(w, ',');
        if (m.kind == K_MAP) {
          NV k;
          nv(c, ch, k);
          tput(w, '"'); tstr(w, bytes_of(c, ch) + k.key_off, k.key_len); tlit(w, "\":");
        }
        cur = ch;
        break;
      }
      tput(w, m.kind == K_LIST ? ']' : '}');
      sp--;
    }
  }
}

// ------------------------------------------------------------------------- query results ---
RD uint32_t qkind(const QR& q) { return q.meta & 3u; }
RD int64_t synth_val(const QR& q) { return (int64_t)(((uint64_t)q.aux << 32) | q.uref); }
RD void q_path(W& w, const Ctx& c, const QR& q) {
  if (qkind(q) == QR_SYNTH_INT && q.node == NONE) return;
  path(w, c, q.node);
}
RD void q_path_display(W& w, const Ctx& c, const QR& q) {
  if (qkind(q) == QR_SYNTH_INT && q.node == NONE) { tlit(w, "[L:0,C:0]"); return; }
  path_display(w, c, q.node);
}
RN void pav_display(W& w, const Ctx& c, const QR& q) {
  tlit(w, "Path="); q_path_display(w, c, q);
  tlit(w, " Value=");
  if (qkind(q) == QR_SYNTH_INT) ti64(w, synth_val(q)); else value_only(w, c, q.node);
}
RN void unresolved_display(W& w, const Ctx& c, const QR& q) {
  tlit(w, "Path="); path_display(w, c, q.node);
  tlit(w, " Value="); value_only(w, c, q.node);
}
RN void remaining(W& w, const Ctx& c, const QR& q) {
  const uint32_t qid = q.uref >> 12, step = q.uref & 0xFFFu;
  if (qid >= c.P->n_queries) { w.fb = FB_REF; return; }
  const uint32_t f = c.P->rem_first[qid], last = c.P->rem_first[qid + 1] - 1;   // entries: steps 0 .. nparts
  const RStr r = c.P->rem[f + step < last ? f + step : last];
  tstr(w, c.P->text + r.off, r.len);
}
// the unresolved reasons the device writer covers (R::reason); Debug-formatted ones go to the host
RN void reason(W& w, const Ctx& c, const QR& q) {
  const uint32_t code = (q.meta >> 8) & 0xFFu;
  const uint32_t qid = q.uref >> 12, step = q.uref & 0xFFFu;
  const uint32_t cur = q.node;
  NV n;
  if (code != R_NONE && !nv(c, cur, n)) { w.fb = FB_REF; return; }
  if (qid >= c.P->n_queries) { w.fb = FB_REF; return; }
  const uint32_t f = c.P->rem_first[qid], np = c.P->rem_first[qid + 1] - f - 1;
  switch (code) {
    case R_NO_MORE_ENTRIES:
      tlit(w, "No more entries for value at path = "); path_display(w, c, cur);
      tlit(w, " on type = "); tlit(w, type_info(n.kind)); tput(w, ' ');
      return;
    case R_KEY_INDEX_NOT_ARRAY:
      tlit(w, "Attempting to retrieve from index "); ti64(w, (int32_t)q.aux);
      tlit(w, " but type is not an array at path "); path_display(w, c, cur);
      return;
    case R_LOCATE_KEY:
    case R_LOCATE_KEY_LIST: {
      NV k;
      if (!nv(c, q.aux, k)) { w.fb = FB_REF; return; }
      tlit(w, "Could not locate key = "); tstr(w, bytes_of(c, q.aux) + k.a, k.count);
      tlit(w, " inside struct at path = "); path_display(w, c, code == R_LOCATE_KEY ? cur : q.aux);
      return;
    }
    case R_KEY_NOT_FOUND: {
      if (step >= np) { w.fb = FB_DEBUG; return; }
      const RStr k = c.P->pkey[f + step];
      tlit(w, "Could not find key "); tstr(w, c.P->text + k.off, k.len);
      tlit(w, " inside struct at path "); path_display(w, c, cur);
      return;
    }
    case R_INDEX_NOT_ARRAY:
      if (step >= np) { w.fb = FB_DEBUG; return; }
      tlit(w, "Attempting to retrieve from index "); ti64(w, c.P->pidx[f + step]);
      tlit(w, " but type is not an array at path "); path_display(w, c, cur);
      tlit(w, ", type "); tlit(w, type_info(n.kind));
      return;
    case R_FILTER_NOT_STRUCT:
      tlit(w, "Filter on value type that was not a struct or array "); tlit(w, type_info(n.kind)); tput(w, ' ');
      path_display(w, c, cur);
      return;
    case R_MAPFILTER_NOT_STRUCT:
      tlit(w, "Map Filter for keys was not a struct "); tlit(w, type_info(n.kind)); tput(w, ' ');
      path_display(w, c, cur);
      return;
    case R_NONE:
      return;
    default:   // R_INDEX_OOB / R_NOT_STRUCT (Debug of values), R_VAR_* (side records): the host writer
      w.fb = FB_DEBUG;
      return;
  }
}

RN void write_pav(W& w, const Ctx& c, const QR& q) {
  open(w, '{');
  key(w, "path"); sbeg(w); q_path(w, c, q); send(w);
  key(w, "value");
  if (qkind(q) == QR_SYNTH_INT) ti64(w, synth_val(q)); else write_value(w, c, q.node);
  close(w, '}');
}
RN void write_unresolved(W& w, const Ctx& c, const QR& q) {
  open(w, '{');
  key(w, "traversed_to");
  open(w, '{');
  key(w, "path"); sbeg(w); path(w, c, q.node); send(w);
  key(w, "value"); write_value(w, c, q.node);
  close(w, '}');
  key(w, "remaining_query"); sbeg(w); remaining(w, c, q); send(w);
  key(w, "reason"); sbeg(w); reason(w, c, q); send(w);
  close(w, '}');
}
// table entries by index, bounds-checked (an index past the table sends the document to the host writer)
RD uint32_t tab_n(const Ctx& c, const RStr* tab) {
  return tab == c.P->ctx ? c.P->n_ctx : tab == c.P->msgs ? c.P->n_msgs : c.P->n_rule_names;
}
RD void str_tab(W& w, const Ctx& c, const RStr* tab, uint32_t i) {
  if (i >= tab_n(c, tab)) { w.fb = FB_REF; return; }
  const RStr r = tab[i]; jstr(w, c.P->text + r.off, r.len);
}
RD void tstr_tab(W& w, const Ctx& c, const RStr* tab, uint32_t i) {
  if (i >= tab_n(c, tab)) { w.fb = FB_REF; return; }
  const RStr r = tab[i]; tstr(w, c.P->text + r.off, r.len);
}
RD bool clause_ok(W& w, const Ctx& c, uint32_t cid) { if (cid < c.P->n_clauses) return true; w.fb = FB_REF; return false; }

RD const char* unary_msg(uint32_t op, bool neg) {
  switch (op) {
    case OP_EXISTS: return neg ? "existed" : "did not exist";
    case OP_EMPTY: return neg ? "was empty" : "was not empty";
    case OP_IS_LIST: return neg ? "was a list " : "was not list";
    case OP_IS_MAP: return neg ? "was a struct" : "was not struct";
    case OP_IS_STRING: return neg ? "was a string " : "was not string";
    case OP_IS_INT: return neg ? "was int" : "was not int";
    case OP_IS_BOOL: return neg ? "was bool" : "was not bool";
    case OP_IS_NULL: return neg ? "was null" : "was not null";
    default: return neg ? "was float" : "was not float";
  }
}
RD const char* op_msg(uint32_t op, bool neg) {
  switch (op) {
    case OP_EQ: return neg ? "equal to" : "not equal to";
    case OP_LE: return neg ? "less than equal to" : "not less than equal to";
    case OP_LT: return neg ? "less than" : "not less than";
    case OP_GE: return neg ? "greater than equal to" : "not greater than equal";
    case OP_GT: return neg ? "greater than" : "not greater than";
    default: return neg ? "in" : "not in";
  }
}
// custom message of a clause: the text, or "" (R::custom)
RD void custom_text(W& w, const Ctx& c, const PClause& pc) { if (pc.e != NONE) tstr_tab(w, c, c.P->msgs, pc.e); }

// NotComparable reason of a REC_CMP (R::nc_reason)
RN void nc_reason(W& w, const Ctx& c, const Rec& rc) {
  if (rc.x == NC_TYPES) {
    tlit(w, "PathAwareValues are not comparable "); tlit(w, type_info(rc.y >> 8)); tlit(w, ", "); tlit(w, type_info(rc.y & 0xFFu));
  } else if (rc.x == NC_FLOAT) {
    tlit(w, "Float values are not comparable");
  } else {
    tlit(w, rc.x == NC_STRING_IN ? "Type not comparable, " : "Can not compare type ");
    pav_display(w, c, rc.from); tlit(w, ", "); pav_display(w, c, rc.to);
  }
}

// ------------------------------------------------------------------------------- records ---
// one tile's ClauseReports (StreamWalker::items over its records), into the open not_compliant array
// A tile's records as the evaluation left them: contiguous (stride 1), or in place in its lane's direct
// record chunk (TileOut.pad1 = stride s > 1: record k at rec_off + s k, eval_kernel.hip) -- read where they are,
// so no compaction pass runs between the evaluation and the report
struct RecSeq {
  const Rec* p;
  uint32_t stride;
  __device__ const Rec& operator[](uint32_t i) const { return p[(size_t)i * stride]; }
};
RN void tile_items(W& w, const Ctx& c, const RecSeq recs, uint32_t nrec) {
  uint32_t closes[kMaxDepth];
  uint32_t sp = 0;
  uint32_t i = 0;
  while (i < nrec && !w.fb) {
    const Rec rc = recs[i];
    if (sp && rc.kind == closes[sp - 1]) {
      // the container's checks end: end_arr, end_obj, end_obj
      i++;
      close(w, ']'); close(w, '}'); close(w, '}');
      sp--;
      continue;
    }
    i++;
    switch (rc.kind) {
      case REC_RULE_OPEN: {
        if (sp == kMaxDepth) { w.fb = FB_DEPTH; return; }
        item(w); open(w, '{'); key(w, "Rule"); open(w, '{');
        key(w, "name"); str_tab(w, c, c.P->rule_names, rc.clause);
        key(w, "metadata"); open(w, '{'); close(w, '}');
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); if (rc.x == NONE) jnull(w); else str_tab(w, c, c.P->msgs, rc.x);
        key(w, "error_message"); jnull(w);
        close(w, '}');
        key(w, "checks"); open(w, '[');
        closes[sp++] = REC_RULE_CLOSE;
        break;
      }
      case REC_DISJ_OPEN:
        if (sp == kMaxDepth) { w.fb = FB_DEPTH; return; }
        item(w); open(w, '{'); key(w, "Disjunctions"); open(w, '{');
        key(w, "checks"); open(w, '[');
        closes[sp++] = REC_DISJ_CLOSE;
        break;
      case REC_BLOCK_EMPTY: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        item(w); open(w, '{'); key(w, "Block"); open(w, '{');
        key(w, "context"); str_tab(w, c, c.P->ctx, pc.d);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); jnull(w);
        key(w, "error_message"); jlit(w, "query for block clause did not retrieve any value");
        close(w, '}');
        key(w, "unresolved"); jnull(w);
        close(w, '}'); close(w, '}');
        break;
      }
      case REC_MISSING_BLOCK_VALUE: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        item(w); open(w, '{'); key(w, "Block"); open(w, '{');
        key(w, "context"); str_tab(w, c, c.P->ctx, pc.f);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); jlit(w, "");
        key(w, "error_message"); sbeg(w);
        tlit(w, "Check was not compliant as property ["); remaining(w, c, rc.from);
        tlit(w, "] is missing. Value traversed to ["); unresolved_display(w, c, rc.from); tput(w, ']');
        send(w);
        close(w, '}');
        key(w, "unresolved"); write_unresolved(w, c, rc.from);
        close(w, '}'); close(w, '}');
        break;
      }
      case REC_UNARY: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        const uint32_t op = pc.flags & 15u;
        const bool neg = (pc.flags >> 4) & 1u;
        const bool unres = qkind(rc.from) == QR_UNRESOLVED;
        item(w); open(w, '{'); key(w, "Clause"); open(w, '{'); key(w, "Unary"); open(w, '{');
        key(w, "check"); open(w, '{'); key(w, unres ? "UnResolved" : "Resolved"); open(w, '{');
        key(w, "value"); if (unres) write_unresolved(w, c, rc.from); else write_pav(w, c, rc.from);
        key(w, "comparison"); cmp(w, op, neg);
        close(w, '}'); close(w, '}');
        key(w, "context"); str_tab(w, c, c.P->ctx, pc.d);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); sbeg(w); custom_text(w, c, pc); send(w);
        key(w, "error_message"); sbeg(w);
        if (unres) {
          tlit(w, "Check was not compliant as property ["); remaining(w, c, rc.from);
          tlit(w, "] is missing. Value traversed to ["); unresolved_display(w, c, rc.from); tlit(w, "].");
        } else {
          tlit(w, "Check was not compliant as property ["); q_path_display(w, c, rc.from); tlit(w, "] ");
          tlit(w, unary_msg(op, neg)); tput(w, '.');
        }
        send(w);
        close(w, '}');
        close(w, '}'); close(w, '}'); close(w, '}');
        break;
      }
      case REC_NOVALUE_EMPTY: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        item(w); open(w, '{'); key(w, "Clause"); open(w, '{'); key(w, "Unary"); open(w, '{');
        key(w, "check"); open(w, '{'); key(w, "UnResolvedContext"); str_tab(w, c, c.P->ctx, pc.d); close(w, '}');
        key(w, "context"); str_tab(w, c, c.P->ctx, pc.d);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); sbeg(w);
        if (pc.e != NONE && pc.e < c.P->n_msgs) {   // newlines become ';'
          const RStr r = c.P->msgs[pc.e];
          for (uint32_t k = 0; k < r.len; k++) { const char ch = c.P->text[r.off + k]; tput(w, ch == '\n' ? ';' : ch); }
        }
        send(w);
        key(w, "error_message"); sbeg(w);
        tlit(w, "Check was not compliant as variable in context ["); tstr_tab(w, c, c.P->ctx, pc.d); tlit(w, "] was not empty");
        send(w);
        close(w, '}');
        close(w, '}'); close(w, '}'); close(w, '}');
        break;
      }
      case REC_DEPENDENT_RULE: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        item(w); open(w, '{'); key(w, "Clause"); open(w, '{'); key(w, "Unary"); open(w, '{');
        key(w, "check"); open(w, '{'); key(w, "UnResolvedContext"); str_tab(w, c, c.P->ctx, pc.f); close(w, '}');
        key(w, "context"); str_tab(w, c, c.P->ctx, pc.d);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); sbeg(w); custom_text(w, c, pc); send(w);
        key(w, "error_message"); sbeg(w);
        tlit(w, "Check was not compliant as dependent rule ["); tstr_tab(w, c, c.P->ctx, pc.f);
        tlit(w, "] did not PASS. Context ["); tstr_tab(w, c, c.P->ctx, pc.d); tput(w, ']');
        send(w);
        close(w, '}');
        close(w, '}'); close(w, '}'); close(w, '}');
        break;
      }
      case REC_CMP: {
        const bool mk = rc.clause == NONE;
        if (!mk && !clause_ok(w, c, rc.clause)) return;
        const PClause pc = mk ? PClause{} : c.P->clauses[rc.clause];
        const uint32_t op = mk ? (rc.y & 15u) : (pc.flags & 15u);
        const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pc.flags >> 4) & 1u);
        const bool from_unres = qkind(rc.from) == QR_UNRESOLVED;
        if (!from_unres && rc.to.meta == 0xFFFFFFFFu) break;   // `to` absent: nothing reported (eval_context.rs:2283)
        const bool to_unres = !from_unres && qkind(rc.to) == QR_UNRESOLVED;
        item(w); open(w, '{'); key(w, "Clause"); open(w, '{'); key(w, "Binary"); open(w, '{');
        key(w, "context"); if (mk) jlit(w, ""); else str_tab(w, c, c.P->ctx, pc.d);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); sbeg(w); if (!mk) custom_text(w, c, pc); send(w);
        key(w, "error_message"); sbeg(w);
        if (from_unres || to_unres) {
          const QR& u = from_unres ? rc.from : rc.to;
          tlit(w, "Check was not compliant as property ["); remaining(w, c, u);
          tlit(w, from_unres ? "] to compare from is missing. Value traversed to [" : "] to compare to is missing. Value traversed to [");
          unresolved_display(w, c, u); tlit(w, "].");
        } else {
          tlit(w, "Check was not compliant as property value ["); pav_display(w, c, rc.from); tlit(w, "] ");
          tlit(w, op_msg(op, neg)); tlit(w, " value ["); pav_display(w, c, rc.to); tlit(w, "].");
        }
        if (rc.x) { tlit(w, " Error = ["); nc_reason(w, c, rc); tput(w, ']'); }
        send(w);
        close(w, '}');
        key(w, "check"); open(w, '{');
        if (from_unres || to_unres) {
          key(w, "UnResolved"); open(w, '{');
          key(w, "value"); write_unresolved(w, c, from_unres ? rc.from : rc.to);
          key(w, "comparison"); cmp(w, op, neg);
          close(w, '}');
        } else {
          key(w, "Resolved"); open(w, '{');
          key(w, "from"); write_pav(w, c, rc.from);
          key(w, "to"); write_pav(w, c, rc.to);
          key(w, "comparison"); cmp(w, op, neg);
          close(w, '}');
        }
        close(w, '}');
        close(w, '}'); close(w, '}'); close(w, '}');
        break;
      }
      case REC_IN: {
        const bool mk = rc.clause == NONE;
        if (!mk && !clause_ok(w, c, rc.clause)) return;
        const PClause pc = mk ? PClause{} : c.P->clauses[rc.clause];
        const uint32_t op = mk ? (rc.y & 15u) : (pc.flags & 15u);
        const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pc.flags >> 4) & 1u);
        // the `to` values: the REC_LIST records that follow, two per record
        const uint32_t nto = rc.x;
        const uint32_t l0 = i;
        uint32_t have = 0;
        while (have < nto && i < nrec && recs[i].kind == REC_LIST) { have += (have + 1 < nto) ? 2u : 1u; i++; }
        auto to_at = [&](uint32_t k) -> QR { const Rec& lr = recs[l0 + k / 2]; return (k & 1u) ? lr.to : lr.from; };
        item(w); open(w, '{'); key(w, "Clause"); open(w, '{'); key(w, "Binary"); open(w, '{');
        key(w, "context"); if (mk) jlit(w, ""); else str_tab(w, c, c.P->ctx, pc.d);
        key(w, "messages"); open(w, '{');
        key(w, "custom_message"); if (mk || pc.e == NONE) jnull(w); else str_tab(w, c, c.P->msgs, pc.e);
        key(w, "error_message"); sbeg(w);
        tlit(w, "Check was not compliant as property ["); q_path_display(w, c, rc.from); tlit(w, "] was not present in [");
        w.dotf = true;   // the items joined by '.', then every '.' before a '[' dropped (reporter.cpp "fixed")
        for (uint32_t k = 0; k < have; k++) {
          const QR t = to_at(k);
          if (k) tput(w, '.');
          if (qkind(t) == QR_UNRESOLVED) { tlit(w, "(unresolved, "); unresolved_display(w, c, t); }
          else { tlit(w, "(resolved, "); pav_display(w, c, t); }
          tput(w, ')');
        }
        if (w.held) { w.held = false; emit(w, '.'); }
        w.dotf = false;
        tput(w, ']');
        send(w);
        close(w, '}');
        key(w, "check"); open(w, '{'); key(w, "InResolved"); open(w, '{');
        key(w, "from"); write_pav(w, c, rc.from);
        key(w, "to"); open(w, '[');
        for (uint32_t k = 0; k < have; k++) {
          const QR t = to_at(k);
          if (qkind(t) != QR_UNRESOLVED) { item(w); write_pav(w, c, t); }
        }
        close(w, ']');
        key(w, "comparison"); cmp(w, op, neg);
        close(w, '}'); close(w, '}');
        close(w, '}'); close(w, '}'); close(w, '}');
        break;
      }
      default:
        break;
    }
  }
  // records end inside containers: the walker's recursion unwinds
  while (sp && !w.fb) { close(w, ']'); close(w, '}'); close(w, '}'); sp--; }
}

// ------------------------------------------------------------------------------- SARIF ---
// SarifResults::from (sarif.rs:127-160) for one tile: every message of every ClauseReport
// (ClauseReport::get_message, eval_context.rs:1808-1826 -- a Rule's and a Disjunction's checks flattened,
// a Block's and a Clause's own Messages) becomes a SarifResult in record order: ruleId from the enclosing
// top-level Rule's name (extract_rule_id: the part before the first '.', upper-cased), level "error",
// message.text = error_message + " " + custom_message (None as ""), one location in the data file at
// Messages.location (a Binary clause's compared value; (0, 0) elsewhere), clamped to 1.  Each result is
// preceded by ",\n" and the results array's indent; the host drops the report's first comma.
RD void sarif_rule_id(W& w, const Ctx& c, uint32_t rule) {
  if (rule == NONE) { raw(w, '"'); raw(w, '"'); return; }
  if (rule >= c.P->n_rule_names) { w.fb = FB_REF; return; }
  const RStr r = c.P->rule_names[rule];
  raw(w, '"');
  for (uint32_t k = 0; k < r.len; k++) {
    const char ch = c.P->text[r.off + k];
    if (ch == '.') break;
    esc1(w, (unsigned char)(ch >= 'a' && ch <= 'z' ? ch - 32 : ch));
  }
  raw(w, '"');
}
// Messages.location of a compared value (the host's q_loc): (0, 0) without a node
RD void sarif_loc(W& w, const Ctx& c, const QR& q, uint32_t& line, uint32_t& col) {
  line = 0; col = 0;
  if (q.node == NONE) return;
  if (q.node & (SYN_BIT | KEY_BIT)) { w.fb = FB_REF; return; }
  if (!(q.node & LIT_BIT) && c.dbase + q.node >= c.A->n_nodes) { w.fb = FB_REF; return; }
  line = line_of(c, q.node); col = col_of(c, q.node);
}
// opens one result: ",\n", its indent, `{`, ruleId, level, message { text: "  -- the caller writes the text
RD void sarif_open(W& w, const Ctx& c, uint32_t rule) {
  raw(w, ','); raw(w, '\n'); spaces(w, 8);
  w.depth = 0; w.base = 4; w.first = 0; w.esc = false; w.dotf = false; w.held = false;
  open(w, '{');
  key(w, "ruleId"); sarif_rule_id(w, c, rule);
  key(w, "level"); jlit(w, "error");
  key(w, "message"); open(w, '{');
  key(w, "text"); sbeg(w);
}
// ... closes the text and writes the location
RD void sarif_close(W& w, const char* uri, uint32_t urin, uint32_t line, uint32_t col) {
  send(w);
  close(w, '}');
  key(w, "locations"); open(w, '[');
  item(w); open(w, '{');
  key(w, "physicalLocation"); open(w, '{');
  key(w, "artifactLocation"); open(w, '{'); key(w, "uri"); jstr(w, uri, urin); close(w, '}');
  key(w, "region"); open(w, '{');
  key(w, "startLine"); tu64(w, line > 1 ? line : 1);
  key(w, "startColumn"); tu64(w, col > 1 ? col : 1);
  close(w, '}');
  close(w, '}');
  close(w, '}');
  close(w, ']');
  close(w, '}');
}
RN void tile_sarif(W& w, const Ctx& c, const RecSeq recs, uint32_t nrec, const char* uri, uint32_t urin) {
  uint32_t closes[kMaxDepth];
  uint32_t sp = 0;
  uint32_t rule = NONE;   // the enclosing top-level Rule (its name index), NONE outside one
  uint32_t i = 0;
  while (i < nrec && !w.fb) {
    const Rec rc = recs[i];
    if (sp && rc.kind == closes[sp - 1]) {
      i++;
      if (--sp == 0) rule = NONE;
      continue;
    }
    i++;
    switch (rc.kind) {
      case REC_RULE_OPEN:
        if (sp == kMaxDepth) { w.fb = FB_DEPTH; return; }
        if (sp == 0) rule = rc.clause;
        closes[sp++] = REC_RULE_CLOSE;
        break;
      case REC_DISJ_OPEN:
        if (sp == kMaxDepth) { w.fb = FB_DEPTH; return; }
        closes[sp++] = REC_DISJ_CLOSE;
        break;
      case REC_BLOCK_EMPTY:
        if (!clause_ok(w, c, rc.clause)) return;
        sarif_open(w, c, rule);
        tlit(w, "query for block clause did not retrieve any value ");
        sarif_close(w, uri, urin, 0, 0);
        break;
      case REC_MISSING_BLOCK_VALUE:
        if (!clause_ok(w, c, rc.clause)) return;
        sarif_open(w, c, rule);
        tlit(w, "Check was not compliant as property ["); remaining(w, c, rc.from);
        tlit(w, "] is missing. Value traversed to ["); unresolved_display(w, c, rc.from); tput(w, ']');
        tput(w, ' ');
        sarif_close(w, uri, urin, 0, 0);
        break;
      case REC_UNARY: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        const uint32_t op = pc.flags & 15u;
        const bool neg = (pc.flags >> 4) & 1u;
        // eval_context.rs:2231-2234: an unresolved value's location, Location::default() otherwise
        uint32_t line = 0, col = 0;
        if (qkind(rc.from) == QR_UNRESOLVED) sarif_loc(w, c, rc.from, line, col);
        sarif_open(w, c, rule);
        if (qkind(rc.from) == QR_UNRESOLVED) {
          tlit(w, "Check was not compliant as property ["); remaining(w, c, rc.from);
          tlit(w, "] is missing. Value traversed to ["); unresolved_display(w, c, rc.from); tlit(w, "].");
        } else {
          tlit(w, "Check was not compliant as property ["); q_path_display(w, c, rc.from); tlit(w, "] ");
          tlit(w, unary_msg(op, neg)); tput(w, '.');
        }
        tput(w, ' '); custom_text(w, c, pc);
        sarif_close(w, uri, urin, line, col);
        break;
      }
      case REC_NOVALUE_EMPTY: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        sarif_open(w, c, rule);
        tlit(w, "Check was not compliant as variable in context ["); tstr_tab(w, c, c.P->ctx, pc.d); tlit(w, "] was not empty");
        tput(w, ' ');
        if (pc.e != NONE && pc.e < c.P->n_msgs) {   // newlines become ';'
          const RStr r = c.P->msgs[pc.e];
          for (uint32_t k = 0; k < r.len; k++) { const char ch = c.P->text[r.off + k]; tput(w, ch == '\n' ? ';' : ch); }
        }
        sarif_close(w, uri, urin, 0, 0);
        break;
      }
      case REC_DEPENDENT_RULE: {
        if (!clause_ok(w, c, rc.clause)) return;
        const PClause pc = c.P->clauses[rc.clause];
        sarif_open(w, c, rule);
        tlit(w, "Check was not compliant as dependent rule ["); tstr_tab(w, c, c.P->ctx, pc.f);
        tlit(w, "] did not PASS. Context ["); tstr_tab(w, c, c.P->ctx, pc.d); tput(w, ']');
        tput(w, ' '); custom_text(w, c, pc);
        sarif_close(w, uri, urin, 0, 0);
        break;
      }
      case REC_CMP: {
        const bool mk = rc.clause == NONE;
        if (!mk && !clause_ok(w, c, rc.clause)) return;
        const PClause pc = mk ? PClause{} : c.P->clauses[rc.clause];
        const uint32_t op = mk ? (rc.y & 15u) : (pc.flags & 15u);
        const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pc.flags >> 4) & 1u);
        const bool from_unres = qkind(rc.from) == QR_UNRESOLVED;
        if (!from_unres && rc.to.meta == 0xFFFFFFFFu) break;   // `to` absent: nothing reported (eval_context.rs:2283)
        const bool to_unres = !from_unres && qkind(rc.to) == QR_UNRESOLVED;
        uint32_t line, col;
        sarif_loc(w, c, from_unres ? rc.from : rc.to, line, col);
        sarif_open(w, c, rule);
        if (from_unres || to_unres) {
          const QR& u = from_unres ? rc.from : rc.to;
          tlit(w, "Check was not compliant as property ["); remaining(w, c, u);
          tlit(w, from_unres ? "] to compare from is missing. Value traversed to [" : "] to compare to is missing. Value traversed to [");
          unresolved_display(w, c, u); tlit(w, "].");
        } else {
          tlit(w, "Check was not compliant as property value ["); pav_display(w, c, rc.from); tlit(w, "] ");
          tlit(w, op_msg(op, neg)); tlit(w, " value ["); pav_display(w, c, rc.to); tlit(w, "].");
        }
        if (rc.x) { tlit(w, " Error = ["); nc_reason(w, c, rc); tput(w, ']'); }
        tput(w, ' '); if (!mk) custom_text(w, c, pc);
        sarif_close(w, uri, urin, line, col);
        break;
      }
      case REC_IN: {
        const bool mk = rc.clause == NONE;
        if (!mk && !clause_ok(w, c, rc.clause)) return;
        const PClause pc = mk ? PClause{} : c.P->clauses[rc.clause];
        const uint32_t nto = rc.x;
        const uint32_t l0 = i;
        uint32_t have = 0;
        while (have < nto && i < nrec && recs[i].kind == REC_LIST) { have += (have + 1 < nto) ? 2u : 1u; i++; }
        auto to_at = [&](uint32_t k) -> QR { const Rec& lr = recs[l0 + k / 2]; return (k & 1u) ? lr.to : lr.from; };
        uint32_t line, col;
        sarif_loc(w, c, rc.from, line, col);
        sarif_open(w, c, rule);
        tlit(w, "Check was not compliant as property ["); q_path_display(w, c, rc.from); tlit(w, "] was not present in [");
        w.dotf = true;   // the items joined by '.', then every '.' before a '[' dropped (reporter.cpp "fixed")
        for (uint32_t k = 0; k < have; k++) {
          const QR t = to_at(k);
          if (k) tput(w, '.');
          if (qkind(t) == QR_UNRESOLVED) { tlit(w, "(unresolved, "); unresolved_display(w, c, t); }
          else { tlit(w, "(resolved, "); pav_display(w, c, t); }
          tput(w, ')');
        }
        if (w.held) { w.held = false; emit(w, '.'); }
        w.dotf = false;
        tput(w, ']');
        tput(w, ' ');
        if (!mk && pc.e != NONE) tstr_tab(w, c, c.P->msgs, pc.e);
        sarif_close(w, uri, urin, line, col);
        break;
      }
      default:
        break;
    }
  }
}

// one document's SarifResults: only a FAILed FileReport contributes (SarifRun::from, sarif.rs:29-51);
// the artifact URI is the document name without one leading '/' (sanitize_path)
RN void file_sarif(W& w, const RenderArgs& A, uint32_t doc) {
  const uint32_t k = doc - A.doc0;
  const uint32_t nf = A.nfiles;
  uint32_t status = ST_SKIP;
  for (uint32_t f = 0; f < nf; f++) {
    const uint32_t st = A.tiles[(size_t)doc * nf + f].status;
    if (status == ST_FAIL) continue;
    if (status == ST_PASS) status = st == ST_FAIL ? ST_FAIL : ST_PASS;
    else status = st;
  }
  if (status != ST_FAIL) return;
  const char* uri = A.names + A.name_off[k];
  uint32_t urin = (uint32_t)(A.name_off[k + 1] - A.name_off[k]);
  if (urin && uri[0] == '/') { uri++; urin--; }
  for (uint32_t f = 0; f < nf && !w.fb; f++) {
    const size_t t = (size_t)doc * nf + f;
    const TileOut to = A.tiles[t];
    Ctx c{&A, &A.progs[f], A.base[doc]};
    tile_sarif(w, c, RecSeq{A.recs + to.rec_off, to.pad1 > 1u ? to.pad1 : 1u}, to.rec_n, uri, urin);
  }
}

// one document's FileReport (write_file_report), preceded by ",\n" after the report's first document and
// the array's two-space indent
RN void file_report(W& w, const RenderArgs& A, uint32_t doc) {
  const uint32_t k = doc - A.doc0;
  if (doc != A.report_first) { raw(w, ','); raw(w, '\n'); }
  spaces(w, 2);
  w.depth = 0; w.base = 1; w.first = 0; w.esc = false; w.dotf = false; w.held = false;
  const uint32_t nf = A.nfiles;
  uint32_t status = ST_SKIP;
  for (uint32_t f = 0; f < nf; f++) {
    const uint32_t st = A.tiles[(size_t)doc * nf + f].status;
    // Status::and (rules/mod.rs:122-133)
    if (status == ST_FAIL) continue;
    if (status == ST_PASS) status = st == ST_FAIL ? ST_FAIL : ST_PASS;
    else status = st;
  }
  open(w, '{');
  key(w, "name"); jstr(w, A.names + A.name_off[k], (uint32_t)(A.name_off[k + 1] - A.name_off[k]));
  key(w, "metadata"); open(w, '{'); close(w, '}');
  key(w, "status"); jlit(w, status == ST_PASS ? "PASS" : status == ST_FAIL ? "FAIL" : "SKIP");
  key(w, "not_compliant"); open(w, '[');
  for (uint32_t f = 0; f < nf && !w.fb; f++) {
    const size_t t = (size_t)doc * nf + f;
    const TileOut to = A.tiles[t];
    Ctx c{&A, &A.progs[f], A.base[doc]};
    tile_items(w, c, RecSeq{A.recs + to.rec_off, to.pad1 > 1u ? to.pad1 : 1u}, to.rec_n);
  }
  close(w, ']');
  // the distinct top-level rule names that SKIPped / PASSed in any file, sorted (std::set)
  for (uint32_t pass = 0; pass < 2; pass++) {
    key(w, pass ? "compliant" : "not_applicable"); open(w, '[');
    const uint8_t want = pass ? (uint8_t)ST_PASS : (uint8_t)ST_SKIP;
    for (uint32_t r = 0; r < A.n_sname; r++) {
      bool hit = false;
      for (uint32_t e = 0; e < A.sname_n[r] && !hit; e++) {
        const uint32_t fk = A.sname_fk[A.sname_first[r] + e];
        hit = A.rule_status[((size_t)doc * nf + (fk >> 16)) * A.max_top + (fk & 0xFFFFu)] == want;
      }
      if (hit) { item(w); const RStr s = A.sname[r]; jstr(w, A.sname_text + s.off, s.len); }
    }
    close(w, ']');
  }
  close(w, '}');
}

}  // namespace rg

// One kernel for both passes (one instantiation of the inlined writer: it is large).  Size pass (write 0):
// the bytes of each document of the block, or kHostDoc | reason for the host writer.  Write pass (write 1):
// each device document at offsets[k] of the block's contiguous text.  Capped at 128 VGPRs (4 waves per
// SIMD): the lanes wait on scattered arena loads, so resident waves matter more than registers.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) report_kernel(RenderArgs A, uint32_t write) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < A.ndocs; k += gridDim.x * blockDim.x) {
    rg::W w{};
    if (write) {
      if (A.sizes[k] & kHostDoc) continue;
      w.p = A.out + A.offsets[k];
    }
    rg::file_report(w, A, A.doc0 + k);
    if (!write) A.sizes[k] = w.fb ? (kHostDoc | w.fb) : w.n;
  }
}

// The SARIF report's results (rg::file_sarif), one lane per document, in the same two passes; a kernel of
// its own so the JSON writer's instantiation is unchanged.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) report_sarif_kernel(RenderArgs A, uint32_t write) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < A.ndocs; k += gridDim.x * blockDim.x) {
    rg::W w{};
    if (write) {
      if (A.sizes[k] & kHostDoc) continue;
      w.p = A.out + A.offsets[k];
    }
    rg::file_sarif(w, A, A.doc0 + k);
    if (!write) A.sizes[k] = w.fb ? (kHostDoc | w.fb) : w.n;
  }
}

}  // namespace gg
