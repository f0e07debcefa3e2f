// MI355X batch evaluator kernel: one wavefront per (document, rules-file) tile.
//
// The wave interprets the compiled rules program (program.h) over the document arena
// (doc_loader.h).  Control flow is wave-uniform: every lane executes the same interpreter
// steps on identical scalar state (redundant but divergence-free, and every lane only reads
// what it wrote, so no intra-wave fences are needed); map key lookups are wave-cooperative
// (64 children compared per step, first hit via __ballot).  Failure records are staged in the
// wave's scratch heap and published to the global record arena with one atomic per tile.
//
// Function-for-function restatement of the reference evaluation path:
//   eval_rules_file / eval_rule / eval_conjunction_clauses   guard/src/rules/eval.rs:1837-2065
//   eval_type_block_clause / eval_guard_block_clause          eval.rs:1303-1426, 1649-1822
//   eval_when_condition_block / eval_guard_named_clause       eval.rs:1227-1289, 1428-1502
//   eval_guard_access_clause / unary_operation / binary_op    eval.rs:174-405, 765-974, 1077-1225
//   operators (Eq / In / Common / not reverse-diffs)          guard/src/rules/eval/operators.rs
//   query_retrieval_with_converter                            guard/src/rules/eval_context.rs:337-924
//   scopes (Root/Block/Value/ResolvedParameter)               eval_context.rs:1062-1606, eval.rs:1504-1572
//   compare_eq / compare_values / PartialEq                   guard/src/rules/path_value.rs:245-291, 1047-1192
#include <hip/hip_runtime.h>

#include "eval_device.h"

namespace gg {

#define DEV __device__ __attribute__((always_inline)) inline
#define DEVN __device__ __attribute__((noinline))

static const uint32_t SYN_BIT = 0x40000000u;
static const uint32_t KEY_BIT = 0x20000000u;
static const uint32_t FRAMES_BYTES = 16384;
static const uint32_t RECS_BYTES = 65536;
static const uint32_t MAX_DEPTH = 48;

enum FrameKind : uint32_t { F_ROOT = 0, F_BLOCK = 1, F_VALUE = 2, F_PARAM = 3 };

struct Frame {
  uint32_t kind, parent, root, block;
  uint32_t cache;   // persist offset of per-let cache (16 B each: state, off, n, pad)
  uint32_t call;    // F_PARAM: param clause id
  uint32_t params;  // F_PARAM: persist offset of per-param views (8 B each: off, n)
  uint32_t prule;   // F_PARAM: param rule id
};

struct View { uint32_t off, n; };

struct Ctx {
  const DevProg* P;
  const DNode* dn;
  const char* db;
  uint8_t* heap;
  uint32_t cap;
  uint32_t tmp;          // grows up from tmp_base
  uint32_t pers;         // grows down from cap
  uint32_t nframes;
  uint32_t nrec;
  uint32_t err, err_a, err_b;
  uint32_t suppress;
  uint32_t rec_created;
  uint32_t memo;         // persist offset: u32 per name slot (3 = unknown)
  uint32_t depth;
  uint32_t nsyn;         // synthetic ints (count()) in this tile
  uint32_t syn_off;      // persist offset of synthetic table (16 B each: src, lo, hi, pad)
};

#define CHK(c) do { if ((c).err) return; } while (0)
#define CHKV(c, v) do { if ((c).err) return (v); } while (0)

DEV void fail(Ctx& c, uint32_t e, uint32_t a = 0, uint32_t b = 0) {
  if (!c.err) { c.err = e; c.err_a = a; c.err_b = b; }
}

// ------------------------------------------------------------------ memory ---
DEV uint32_t alloc_tmp(Ctx& c, uint32_t bytes) {
  bytes = (bytes + 15u) & ~15u;
  uint32_t o = c.tmp;
  if (c.tmp + bytes > c.pers) { fail(c, E_HEAP); return FRAMES_BYTES + RECS_BYTES; }
  c.tmp += bytes;
  return o;
}
DEV uint32_t alloc_pers(Ctx& c, uint32_t bytes) {
  bytes = (bytes + 15u) & ~15u;
  if (c.pers < c.tmp + bytes) { fail(c, E_HEAP); return FRAMES_BYTES + RECS_BYTES; }
  c.pers -= bytes;
  return c.pers;
}
DEV QR* qra(Ctx& c, uint32_t off) { return (QR*)(c.heap + off); }
DEV uint32_t* u32a(Ctx& c, uint32_t off) { return (uint32_t*)(c.heap + off); }
DEV Frame* fr(Ctx& c, uint32_t idx) { return (Frame*)(c.heap) + idx; }

DEV void qr_push(Ctx& c, QR q) {
  uint32_t o = alloc_tmp(c, 16);
  CHK(c);
  *qra(c, o) = q;
}
DEV QR mk_qr(uint32_t node, uint32_t kind) { QR q; q.node = node; q.meta = kind; q.uref = 0; q.aux = 0; return q; }
DEV QR mk_unres(uint32_t node, uint32_t reason, uint32_t qid, uint32_t step, uint32_t aux) {
  QR q; q.node = node; q.meta = QR_UNRESOLVED | (reason << 8); q.uref = (qid << 12) | step; q.aux = aux; return q;
}
DEV uint32_t qkind(const QR& q) { return q.meta & 3u; }

// ------------------------------------------------------------------- nodes ---
DEV DNode node(const Ctx& c, uint32_t ref) {
  if (ref & SYN_BIT) {
    const uint32_t* s = (const uint32_t*)(c.heap + c.syn_off) + 4 * (ref & 0xFFFFu);
    DNode d; d.kind = K_INT; d.count = 0; d.a = s[1]; d.b = s[2]; d.key_off = NONE; d.key_len = 0; d.key_hash = 0; d.parent = NONE;
    return d;
  }
  if (ref & KEY_BIT) {
    // the key of a map entry as a String value (MapValue.keys, path_value.rs:459-466)
    uint32_t e = ref & ~KEY_BIT;
    DNode en = (e & LIT_BIT) ? c.P->lit_nodes[e & ~LIT_BIT] : c.dn[e];
    DNode d; d.kind = K_STRING; d.count = en.key_len; d.a = en.key_off; d.b = en.key_hash;
    d.key_off = NONE; d.key_len = 0; d.key_hash = 0; d.parent = NONE;
    return d;
  }
  if (ref & LIT_BIT) return c.P->lit_nodes[ref & ~LIT_BIT];
  return c.dn[ref];
}
DEV const char* bytes_of(const Ctx& c, uint32_t ref) { return (ref & LIT_BIT) ? c.P->bytes : c.db; }
DEV uint32_t child(uint32_t ref, const DNode& n, uint32_t j) { return (ref & LIT_BIT) | (n.a + j); }
DEV int64_t ival(const DNode& n) { return (int64_t)(((uint64_t)n.b << 32) | n.a); }
DEV double fval(const DNode& n) { return __longlong_as_double((long long)(((uint64_t)n.b << 32) | n.a)); }
DEV bool is_scalar_k(uint32_t k) { return k != K_LIST && k != K_MAP; }

DEV bool bytes_eq(const char* a, const char* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) if (a[i] != b[i]) return false;
  return true;
}

// wave-cooperative: child of map `ref` whose key == (kp, klen, khash); NONE if absent
DEVN uint32_t map_get(const Ctx& c, uint32_t ref, const char* kp, uint32_t klen, uint32_t khash) {
  DNode m = node(c, ref);
  const char* base = bytes_of(c, ref);
  const uint32_t lane = __lane_id();
  for (uint32_t start = 0; start < m.count; start += 64) {
    uint32_t i = start + lane;
    bool hit = false;
    if (i < m.count) {
      DNode ch = node(c, child(ref, m, i));
      hit = ch.key_hash == khash && ch.key_len == klen && bytes_eq(base + ch.key_off, kp, klen);
    }
    unsigned long long mask = __ballot(hit);
    if (mask) return child(ref, m, start + (uint32_t)__ffsll((long long)mask) - 1u);
  }
  return NONE;
}

DEV uint32_t map_get_pstr(const Ctx& c, uint32_t ref, uint32_t sid) {
  PStr s = c.P->strs[sid];
  return map_get(c, ref, c.P->bytes + s.off, s.len, s.hash);
}

// ---------------------------------------------------------------- records ---
// a count() result referenced by a record travels as QR_SYNTH_INT (source node + value)
DEV QR publishable(const Ctx& c, QR q) {
  if (q.meta != 0xFFFFFFFFu && (q.node & SYN_BIT) && q.node != NONE) {
    const uint32_t* s = (const uint32_t*)(c.heap + c.syn_off) + 4 * (q.node & 0xFFFFu);
    QR o; o.node = s[0]; o.meta = QR_SYNTH_INT; o.uref = s[1]; o.aux = s[2];
    return o;
  }
  return q;
}
DEV void rec_push(Ctx& c, const Rec& r) {
  if (c.suppress) return;
  if ((c.nrec + 1) * sizeof(Rec) > RECS_BYTES) { fail(c, E_RECORDS); return; }
  Rec* dst = (Rec*)(c.heap + FRAMES_BYTES) + c.nrec;
  Rec w = r;
  w.from = publishable(c, r.from);
  w.to = publishable(c, r.to);
  *dst = w;
  c.nrec++;
}
DEV Rec mk_rec(uint32_t kind, uint32_t clause) {
  Rec r; r.kind = kind; r.clause = clause; r.x = 0; r.y = 0;
  r.from = mk_qr(NONE, 0); r.to = mk_qr(NONE, 0); r.to.meta = 0xFFFFFFFFu;
  return r;
}

// ---------------------------------------------------------------- frames ---
DEV uint32_t push_frame(Ctx& c, uint32_t kind, uint32_t parent, uint32_t root, uint32_t block) {
  if ((c.nframes + 1) * sizeof(Frame) > FRAMES_BYTES) { fail(c, E_DEPTH); return 0; }
  uint32_t idx = c.nframes++;
  Frame* f = fr(c, idx);
  f->kind = kind; f->parent = parent; f->root = root; f->block = block;
  f->cache = NONE; f->call = NONE; f->params = NONE; f->prule = NONE;
  if ((kind == F_ROOT || kind == F_BLOCK) && block != NONE) {
    uint32_t nl = c.P->blocks[block].nlets;
    if (nl) {
      uint32_t o = alloc_pers(c, nl * 16);
      if (c.err) return idx;
      for (uint32_t i = 0; i < nl; i++) u32a(c, o)[i * 4] = 0;
      f->cache = o;
    }
  }
  return idx;
}
DEV void pop_frame(Ctx& c) { c.nframes--; }

DEV uint32_t frame_root(Ctx& c, uint32_t f) {
  while (fr(c, f)->kind == F_PARAM) f = fr(c, f)->parent;
  return fr(c, f)->root;
}

// forward decls
DEVN void query_retrieval(Ctx& c, uint32_t qi, uint32_t qid, uint32_t cur, uint32_t resolver, uint32_t conv);
DEVN View scope_query(Ctx& c, uint32_t frame, uint32_t qid);
DEVN View resolve_variable(Ctx& c, uint32_t frame, uint32_t var);
DEVN uint32_t eval_conj(Ctx& c, uint32_t conj, uint32_t frame);
DEVN uint32_t eval_rule(Ctx& c, uint32_t rule, uint32_t frame, uint32_t custom_msg);
DEVN View resolve_function(Ctx& c, uint32_t fid, uint32_t frame);

// ---------------------------------------------------------- comparisons ---
// compare_values (path_value.rs:1047-1068): 0 ok (ord in *ord), 1 NotComparable(types), 2 NotComparable(float)
struct Cmp { int32_t status; int32_t ord; uint32_t ka, kb; };

DEV int32_t bytes_cmp(const char* a, uint32_t na, const char* b, uint32_t nb) {
  uint32_t n = na < nb ? na : nb;
  for (uint32_t i = 0; i < n; i++) {
    unsigned char x = (unsigned char)a[i], y = (unsigned char)b[i];
    if (x != y) return x < y ? -1 : 1;
  }
  return na == nb ? 0 : (na < nb ? -1 : 1);
}

DEV Cmp compare_values(const Ctx& c, uint32_t ra, const DNode& a, uint32_t rb, const DNode& b) {
  Cmp r; r.status = 0; r.ord = 0; r.ka = a.kind; r.kb = b.kind;
  if (a.kind == K_NULL && b.kind == K_NULL) return r;
  if (a.kind == K_INT && b.kind == K_INT) { int64_t x = ival(a), y = ival(b); r.ord = x < y ? -1 : (x > y ? 1 : 0); return r; }
  if (a.kind == K_STRING && b.kind == K_STRING) { r.ord = bytes_cmp(bytes_of(c, ra) + a.a, a.count, bytes_of(c, rb) + b.a, b.count); return r; }
  if (a.kind == K_FLOAT && b.kind == K_FLOAT) {
    double x = fval(a), y = fval(b);
    if (x != x || y != y) { r.status = 2; return r; }
    r.ord = x < y ? -1 : (x > y ? 1 : 0); return r;
  }
  if (a.kind == K_CHAR && b.kind == K_CHAR) { r.ord = a.a < b.a ? -1 : (a.a > b.a ? 1 : 0); return r; }
  r.status = 1;
  return r;
}

// regex is_match over a UTF-8 haystack; -1 = unsupported (error raised by caller)
DEV int regex_match(const Ctx& c, uint32_t rid, const char* s, uint32_t n) {
  PRegex rx = c.P->regex[rid];
  if (rx.flags & 1u) return -1;
  if (rx.flags & 2u) for (uint32_t i = 0; i < n; i++) if ((unsigned char)s[i] >= 0x80) return -1;
  const uint16_t* T = c.P->dfa + rx.table;
  const uint16_t* A = T + (size_t)rx.nstates * 256;
  bool end_anchored = (rx.flags & 4u) != 0;
  uint32_t st = rx.start;
  if (!end_anchored && A[st]) return 1;
  for (uint32_t i = 0; i < n; i++) {
    st = T[(size_t)st * 256 + (unsigned char)s[i]];
    if (st == 0) return 0;
    if (!end_anchored && A[st]) return 1;
  }
  return A[st] ? 1 : 0;
}

DEV bool within(const DRange& r, uint32_t kind, const DNode& v) {
  if (kind == K_RANGE_INT) {
    int64_t x = ival(v), lo = (int64_t)r.lo, hi = (int64_t)r.hi;
    bool l = (r.incl & 1) ? lo <= x : lo < x;
    bool u = (r.incl & 2) ? hi >= x : hi > x;
    return l && u;
  }
  if (kind == K_RANGE_FLOAT) {
    double x = fval(v), lo = __longlong_as_double((long long)r.lo), hi = __longlong_as_double((long long)r.hi);
    bool l = (r.incl & 1) ? lo <= x : lo < x;
    bool u = (r.incl & 2) ? hi >= x : hi > x;
    return l && u;
  }
  uint32_t x = v.a, lo = (uint32_t)r.lo, hi = (uint32_t)r.hi;
  bool l = (r.incl & 1) ? lo <= x : lo < x;
  bool u = (r.incl & 2) ? hi >= x : hi > x;
  return l && u;
}

// compare_eq (path_value.rs:1070-1152).  Returns Cmp with status 0 and ord 0 (equal) / 1 (not equal),
// status 1/2 for NotComparable, status 3 for an unsupported regex (raises E_REGEX_UNSUPPORTED).
DEVN Cmp compare_eq(Ctx& c, uint32_t ra, uint32_t rb, uint32_t depth) {
  DNode a = node(c, ra), b = node(c, rb);
  Cmp r; r.status = 0; r.ord = 1; r.ka = a.kind; r.kb = b.kind;
  if (depth > 64) { fail(c, E_DEPTH); return r; }
  if ((a.kind == K_STRING && b.kind == K_REGEX) || (a.kind == K_REGEX && b.kind == K_STRING)) {
    uint32_t rs = a.kind == K_STRING ? ra : rb, rr = a.kind == K_STRING ? rb : ra;
    DNode s = a.kind == K_STRING ? a : b, x = a.kind == K_STRING ? b : a;
    int m = regex_match(c, x.b, bytes_of(c, rs) + s.a, s.count);
    (void)rr;
    if (m < 0) { fail(c, E_REGEX_UNSUPPORTED, x.b); r.status = 3; return r; }
    r.ord = m ? 0 : 1; return r;
  }
  if (a.kind == K_STRING && b.kind == K_STRING) {
    r.ord = (a.count == b.count && a.b == b.b && bytes_eq(bytes_of(c, ra) + a.a, bytes_of(c, rb) + b.a, a.count)) ? 0 : 1;
    return r;
  }
  if (a.kind == K_MAP && b.kind == K_MAP) {
    if (a.count != b.count) return r;
    for (uint32_t i = 0; i < a.count; i++) {
      uint32_t ca = child(ra, a, i);
      DNode cn = node(c, ca);
      uint32_t cb = map_get(c, rb, bytes_of(c, ra) + cn.key_off, cn.key_len, cn.key_hash);
      if (cb == NONE) return r;
      Cmp x = compare_eq(c, ca, cb, depth + 1);
      if (x.status || x.ord) return x;
    }
    r.ord = 0; return r;
  }
  if (a.kind == K_LIST && b.kind == K_LIST) {
    if (a.count != b.count) return r;
    for (uint32_t i = 0; i < a.count; i++) {
      Cmp x = compare_eq(c, child(ra, a, i), child(rb, b, i), depth + 1);
      if (x.status || x.ord) return x;
    }
    r.ord = 0; return r;
  }
  if (a.kind == K_BOOL && b.kind == K_BOOL) { r.ord = a.a == b.a ? 0 : 1; return r; }
  if (a.kind == K_REGEX && b.kind == K_REGEX) {
    r.ord = (a.count == b.count && bytes_eq(bytes_of(c, ra) + a.a, bytes_of(c, rb) + b.a, a.count)) ? 0 : 1;
    return r;
  }
  if ((a.kind == K_INT && b.kind == K_RANGE_INT) || (a.kind == K_FLOAT && b.kind == K_RANGE_FLOAT) ||
      (a.kind == K_CHAR && b.kind == K_RANGE_CHAR)) {
    r.ord = within(c.P->lit_ranges[b.a], b.kind, a) ? 0 : 1; return r;
  }
  Cmp v = compare_values(c, ra, a, rb, b);
  if (v.status) return v;
  r.ord = v.ord == 0 ? 0 : 1;
  return r;
}

// PartialEq for PathAwareValue (path_value.rs:245-291): errors => false
DEVN bool pv_eq(Ctx& c, uint32_t ra, uint32_t rb, uint32_t depth) {
  DNode a = node(c, ra), b = node(c, rb);
  if (depth > 64) { fail(c, E_DEPTH); return false; }
  if (a.kind == K_MAP && b.kind == K_MAP) {
    if (a.count != b.count) return false;
    for (uint32_t i = 0; i < a.count; i++) {
      uint32_t ca = child(ra, a, i);
      DNode cn = node(c, ca);
      uint32_t cb = map_get(c, rb, bytes_of(c, ra) + cn.key_off, cn.key_len, cn.key_hash);
      if (cb == NONE || !pv_eq(c, ca, cb, depth + 1)) return false;
    }
    return true;
  }
  if (a.kind == K_LIST && b.kind == K_LIST) {
    if (a.count != b.count) return false;
    for (uint32_t i = 0; i < a.count; i++) if (!pv_eq(c, child(ra, a, i), child(rb, b, i), depth + 1)) return false;
    return true;
  }
  if (a.kind == K_BOOL && b.kind == K_BOOL) return a.a == b.a;
  if ((a.kind == K_STRING && b.kind == K_REGEX) || (a.kind == K_REGEX && b.kind == K_STRING)) {
    uint32_t rs = a.kind == K_STRING ? ra : rb;
    DNode s = a.kind == K_STRING ? a : b, x = a.kind == K_STRING ? b : a;
    int m = regex_match(c, x.b, bytes_of(c, rs) + s.a, s.count);
    if (m < 0) { fail(c, E_REGEX_UNSUPPORTED, x.b); return false; }
    return m == 1;
  }
  if (a.kind == K_REGEX && b.kind == K_REGEX)
    return a.count == b.count && bytes_eq(bytes_of(c, ra) + a.a, bytes_of(c, rb) + b.a, a.count);
  if ((a.kind == K_INT && b.kind == K_RANGE_INT) || (a.kind == K_FLOAT && b.kind == K_RANGE_FLOAT) ||
      (a.kind == K_CHAR && b.kind == K_RANGE_CHAR))
    return within(c.P->lit_ranges[b.a], b.kind, a);
  Cmp v = compare_values(c, ra, a, rb, b);
  return v.status == 0 && v.ord == 0;
}

// ---------------------------------------------------------- query engine ---
DEV uint32_t qpart_index(const Ctx& c, uint32_t qid, uint32_t qi) { return c.P->queries[qid].first + qi; }

DEV Rec mk_rec(uint32_t kind, uint32_t clause);
DEV void rec_push(Ctx& c, const Rec& r);

// in_cmp(not_in) (eval.rs:540-566): 1 true, 0 false, -1 NotComparable
DEVN int in_cmp(Ctx& c, uint32_t l, uint32_t r, bool not_in) {
  DNode a = node(c, l), b = node(c, r);
  if (a.kind == K_STRING && b.kind == K_STRING) {
    const char* hay = bytes_of(c, r) + b.a;
    const char* nd = bytes_of(c, l) + a.a;
    bool found = a.count == 0;
    for (uint32_t i = 0; !found && i + a.count <= b.count; i++) found = bytes_eq(hay + i, nd, a.count);
    return (found != not_in) ? 1 : 0;
  }
  if (b.kind == K_LIST) {
    bool found = false;
    for (uint32_t i = 0; i < b.count; i++) {
      Cmp x = compare_eq(c, l, child(r, b, i), 0);
      if (x.status) return -1;
      if (x.ord == 0) found = true;
    }
    return (found != not_in) ? 1 : 0;
  }
  Cmp x = compare_eq(c, l, r, 0);
  if (x.status) return -1;
  return ((x.ord == 0) != not_in) ? 1 : 0;
}

// MapKeyFilter step (eval_context.rs:830-922): real_binary_operation over the map's keys with
// context "" (records leak into the enclosing clause, exactly as in the reference)
DEVN void map_key_filter(Ctx& c, uint32_t qi, uint32_t qid, uint32_t cur, const DNode& cn, uint32_t resolver,
                         uint32_t conv, const PPart& part) {
  const uint32_t m0 = c.tmp;
  View rhs;
  if (part.a == RHS_LITERAL) {
    rhs.off = alloc_tmp(c, 16); rhs.n = 1;
    if (c.err) return;
    *qra(c, rhs.off) = mk_qr(part.b, QR_LITERAL);
  } else if (part.a == RHS_QUERY) {
    uint32_t start = c.tmp;
    query_retrieval(c, 0, part.b, cur, resolver, conv);
    rhs.off = start; rhs.n = (c.tmp - start) / 16;
  } else {
    rhs = resolve_function(c, part.b, resolver);
  }
  if (c.err) return;
  uint32_t op = part.c & 15u;
  bool neg = (part.c >> 4) & 1u;
  if (op == OP_EQ && rhs.n > 1) op = OP_IN;
  uint32_t yop = op | (neg ? 16u : 0u) | 0x100u;
  uint32_t sel_off = alloc_tmp(c, (cn.count ? cn.count : 1) * 4);
  uint32_t items_off = alloc_tmp(c, (rhs.n ? rhs.n : 1) * 16);
  if (c.err) return;
  uint32_t nsel = 0;
  for (uint32_t j = 0; j < cn.count && !c.err; j++) {
    uint32_t entry = child(cur, cn, j);
    uint32_t kref = KEY_BIT | entry;
    if (op == OP_IN) {
      bool found = false;
      for (uint32_t i = 0; i < rhs.n && !c.err; i++) {
        QR r = *qra(c, rhs.off + i * 16);
        if (qkind(r) == QR_UNRESOLVED) { *qra(c, items_off + i * 16) = r; continue; }
        uint32_t rr = r.node;
        int res = in_cmp(c, kref, rr, neg);
        if (res < 0 && qkind(r) == QR_LITERAL) {
          DNode rn = node(c, rr);
          if (rn.kind == K_LIST && rn.count == 1) { rr = child(rr, rn, 0); res = in_cmp(c, kref, rr, neg); }
        }
        *qra(c, items_off + i * 16) = mk_qr(rr, QR_RESOLVED);
        if (res == 1) found = true;
      }
      if (c.err) break;
      c.rec_created++;
      if (found) { u32a(c, sel_off)[nsel++] = entry; continue; }
      if (!c.suppress) {
        Rec rc = mk_rec(REC_IN, NONE);
        rc.from = mk_qr(kref, QR_RESOLVED); rc.x = rhs.n; rc.y = yop;
        rec_push(c, rc);
        for (uint32_t i = 0; i < rhs.n; i += 2) {
          Rec l = mk_rec(REC_LIST, NONE);
          l.from = *qra(c, items_off + i * 16);
          if (i + 1 < rhs.n) l.to = *qra(c, items_off + (i + 1) * 16);
          rec_push(c, l);
        }
      }
    } else {
      for (uint32_t i = 0; i < rhs.n && !c.err; i++) {
        QR r = *qra(c, rhs.off + i * 16);
        c.rec_created++;
        Rec rc = mk_rec(REC_CMP, NONE);
        rc.from = mk_qr(kref, QR_RESOLVED); rc.y = yop;
        if (qkind(r) == QR_UNRESOLVED) { rc.to = r; rec_push(c, rc); continue; }
        uint32_t rr = r.node;
        Cmp x = compare_eq(c, kref, rr, 0);
        if (x.status && qkind(r) == QR_LITERAL) {
          DNode rn = node(c, rr);
          if (rn.kind == K_LIST && rn.count == 1) { rr = child(rr, rn, 0); x = compare_eq(c, kref, rr, 0); }
        }
        if (c.err) break;
        bool ok = x.status == 0 && ((x.ord == 0) != neg);
        if (ok) { u32a(c, sel_off)[nsel++] = entry; continue; }
        rc.to = mk_qr(rr, QR_RESOLVED);
        rec_push(c, rc);
      }
    }
  }
  uint32_t res0 = c.tmp;
  for (uint32_t k = 0; k < nsel && !c.err; k++) query_retrieval(c, qi + 1, qid, u32a(c, sel_off)[k], resolver, conv);
  if (c.err) return;
  // results must stay contiguous for the caller: slide them over the temporaries
  // (every lane copies everything in the same order, so each lane only reads its own writes)
  uint32_t n = (c.tmp - res0) / 4;
  uint32_t* dst = u32a(c, m0);
  const uint32_t* src = u32a(c, res0);
  for (uint32_t i = 0; i < n; i++) dst[i] = src[i];
  c.tmp = m0 + n * 4;
}

DEVN void query_retrieval(Ctx& c, uint32_t qi, uint32_t qid, uint32_t cur, uint32_t resolver, uint32_t conv) {
  CHK(c);
  if (++c.depth > MAX_DEPTH * 4) { fail(c, E_DEPTH); c.depth--; return; }
  const PQuery Q = c.P->queries[qid];
  if (qi >= Q.n) { qr_push(c, mk_qr(cur, QR_RESOLVED)); c.depth--; return; }
  const PPart part = c.P->parts[Q.first + qi];

  if (qi == 0 && part.kind == P_VAR_HEAD) {
    View v = resolve_variable(c, resolver, part.a);
    if (c.err) { c.depth--; return; }
    for (uint32_t i = 0; i < v.n; i++) {
      QR e = *qra(c, v.off + i * 16);
      if (qkind(e) == QR_UNRESOLVED) { qr_push(c, e); continue; }
      uint32_t index = qi + 1;
      if (qi + 1 < Q.n && c.P->parts[Q.first + qi + 1].kind == P_ALL_INDICES) index = qi + 2;
      if (index < Q.n) {
        if (e.node & SYN_BIT) { fail(c, E_UNSUPPORTED, 3); break; }
        uint32_t f = push_frame(c, F_VALUE, resolver, e.node, NONE);
        if (c.err) break;
        query_retrieval(c, index, qid, e.node, f, conv);
        pop_frame(c);
      } else {
        qr_push(c, e);
      }
      if (c.err) break;
    }
    c.depth--;
    return;
  }

  DNode cn = node(c, cur);
  switch (part.kind) {
    case P_THIS:
      query_retrieval(c, qi + 1, qid, cur, resolver, conv);
      break;
    case P_KEY_INDEX: {
      int32_t idx = (int32_t)part.a;
      if (cn.kind == K_LIST) {
        uint32_t check = (uint32_t)(idx >= 0 ? idx : -idx);
        if (check < cn.count) query_retrieval(c, qi + 1, qid, child(cur, cn, check), resolver, conv);
        else qr_push(c, mk_unres(cur, R_INDEX_OOB, qid, 0, (uint32_t)idx));
      } else {
        qr_push(c, mk_unres(cur, R_KEY_INDEX_NOT_ARRAY, qid, 0, (uint32_t)idx));
      }
      break;
    }
    case P_KEY: {
      if (cn.kind != K_MAP) { qr_push(c, mk_unres(cur, R_NOT_STRUCT, qid, qi, 0)); break; }
      uint32_t hit = map_get_pstr(c, cur, part.a);
      if (hit != NONE) { query_retrieval(c, qi + 1, qid, hit, resolver, conv); break; }
      if (conv) {
        uint32_t alt = c.P->alts[part.b + conv - 1];
        hit = map_get_pstr(c, cur, alt);
        if (hit != NONE) { query_retrieval(c, qi + 1, qid, hit, resolver, conv); break; }
      } else {
        for (uint32_t k = 0; k < 7; k++) {
          hit = map_get_pstr(c, cur, c.P->alts[part.b + k]);
          if (hit != NONE) { query_retrieval(c, qi + 1, qid, hit, resolver, k + 1); break; }
        }
        if (hit != NONE) break;
      }
      qr_push(c, mk_unres(cur, R_KEY_NOT_FOUND, qid, qi, 0));
      break;
    }
    case P_KEY_VAR: {
      if (cn.kind != K_MAP) { qr_push(c, mk_unres(cur, R_NOT_STRUCT, qid, qi, 0)); break; }
      View keys = resolve_variable(c, resolver, part.a);
      if (c.err) break;
      uint32_t first = 0, last = keys.n;
      if (qi + 1 < Q.n) {
        PPart nx = c.P->parts[Q.first + qi + 1];
        if (nx.kind == P_ALL_INDICES || nx.kind == P_KEY || nx.kind == P_KEY_INDEX || nx.kind == P_KEY_VAR) {
        } else if (nx.kind == P_INDEX) {
          int32_t ix = (int32_t)nx.a;
          uint32_t check = (uint32_t)(ix >= 0 ? ix : -ix);
          if (check < keys.n) { first = check; last = check + 1; }
          else { fail(c, E_UNSUPPORTED, 4); break; }  // R4 (needs Debug of the key list)
        } else {
          fail(c, E_INTERP_QUERY, qid, qi); break;
        }
      }
      for (uint32_t i = first; i < last && !c.err; i++) {
        QR k = *qra(c, keys.off + i * 16);
        if (qkind(k) == QR_UNRESOLVED) { fail(c, E_UNSUPPORTED, 5); break; }  // R5
        DNode kn = node(c, k.node);
        if (kn.kind == K_STRING) {
          uint32_t hit = map_get(c, cur, bytes_of(c, k.node) + kn.a, kn.count, kn.b);
          if (hit != NONE) query_retrieval(c, qi + 1, qid, hit, resolver, conv);
          else qr_push(c, mk_unres(cur, R_LOCATE_KEY, qid, qi, k.node));
        } else if (kn.kind == K_LIST) {
          for (uint32_t j = 0; j < kn.count && !c.err; j++) {
            uint32_t inner = child(k.node, kn, j);
            DNode in = node(c, inner);
            if (in.kind != K_STRING) { fail(c, E_INTERP_NON_STRING, k.node); break; }
            uint32_t hit = map_get(c, cur, bytes_of(c, inner) + in.a, in.count, in.b);
            if (hit != NONE) query_retrieval(c, qi + 1, qid, hit, resolver, conv);
            else qr_push(c, mk_unres(cur, R_LOCATE_KEY_LIST, qid, qi, inner));
          }
        } else {
          fail(c, E_INTERP_NON_STRING, k.node);
        }
      }
      break;
    }
    case P_INDEX: {
      int32_t idx = (int32_t)part.a;
      if (cn.kind == K_LIST) {
        uint32_t check = (uint32_t)(idx >= 0 ? idx : -idx);
        if (check < cn.count) query_retrieval(c, qi + 1, qid, child(cur, cn, check), resolver, conv);
        else qr_push(c, mk_unres(cur, R_INDEX_OOB, qid, 0, (uint32_t)idx));
      } else {
        qr_push(c, mk_unres(cur, R_INDEX_NOT_ARRAY, qid, qi, (uint32_t)idx));
      }
      break;
    }
    case P_ALL_INDICES:
    case P_ALL_VALUES: {
      bool named = part.a != NONE;
      if (cn.kind == K_LIST) {
        if (cn.count == 0) { qr_push(c, mk_unres(cur, R_NO_MORE_ENTRIES, qid, qi, 0)); break; }
        for (uint32_t j = 0; j < cn.count && !c.err; j++) query_retrieval(c, qi + 1, qid, child(cur, cn, j), resolver, conv);
      } else if (cn.kind == K_MAP) {
        if (part.kind == P_ALL_INDICES && !named) { query_retrieval(c, qi + 1, qid, cur, resolver, conv); break; }
        if (named) { fail(c, E_UNSUPPORTED, 1); break; }   // variable captures
        if (cn.count == 0) { qr_push(c, mk_unres(cur, R_NO_MORE_ENTRIES, qid, qi, 0)); break; }
        for (uint32_t j = 0; j < cn.count && !c.err; j++) {
          uint32_t v = child(cur, cn, j);
          uint32_t f = push_frame(c, F_VALUE, resolver, v, NONE);
          if (c.err) break;
          query_retrieval(c, qi + 1, qid, v, f, conv);
          pop_frame(c);
        }
      } else {
        query_retrieval(c, qi + 1, qid, cur, resolver, conv);
      }
      break;
    }
    case P_FILTER: {
      if (part.b != NONE) { fail(c, E_UNSUPPORTED, 1); break; }   // named filter capture
      uint32_t conj = part.a;
      if (cn.kind == K_MAP) {
        uint32_t prev = qi > 0 ? c.P->parts[Q.first + qi - 1].kind : P_THIS;
        if (prev == P_ALL_VALUES || prev == P_ALL_INDICES) {
          // check_and_delegate(...)(resolver)  eval_context.rs:268-313
          c.rec_created++;
          uint32_t mark = c.tmp;
          c.suppress++;
          uint32_t st = eval_conj(c, conj, resolver);
          c.suppress--;
          c.tmp = mark;
          if (c.err) break;
          if (st == ST_PASS) query_retrieval(c, qi + 1, qid, cur, resolver, conv);
        } else if (prev == P_KEY || prev == P_KEY_VAR || prev == P_KEY_INDEX) {
          // accumulate_map(check_and_delegate(..)) over the map's values
          for (uint32_t j = 0; j < cn.count && !c.err; j++) {
            uint32_t v = child(cur, cn, j);
            uint32_t f = push_frame(c, F_VALUE, resolver, v, NONE);
            if (c.err) break;
            c.rec_created++;
            uint32_t mark = c.tmp;
            c.suppress++;
            uint32_t st = eval_conj(c, conj, f);
            c.suppress--;
            c.tmp = mark;
            if (!c.err && st == ST_PASS) query_retrieval(c, qi + 1, qid, v, f, conv);
            pop_frame(c);
          }
        } else {
          fail(c, E_UNSUPPORTED, 2);
        }
      } else if (cn.kind == K_LIST) {
        for (uint32_t j = 0; j < cn.count && !c.err; j++) {
          uint32_t v = child(cur, cn, j);
          c.rec_created++;
          uint32_t f = push_frame(c, F_VALUE, resolver, v, NONE);
          if (c.err) break;
          uint32_t mark = c.tmp;
          c.suppress++;
          uint32_t st = eval_conj(c, conj, f);
          c.suppress--;
          c.tmp = mark;
          pop_frame(c);
          if (!c.err && st == ST_PASS) query_retrieval(c, qi + 1, qid, v, resolver, conv);
        }
      } else {
        uint32_t prev = qi > 0 ? c.P->parts[Q.first + qi - 1].kind : P_THIS;
        if (prev == P_ALL_INDICES) {
          uint32_t f = push_frame(c, F_VALUE, resolver, cur, NONE);
          if (c.err) break;
          uint32_t mark = c.tmp;
          c.suppress++;
          uint32_t st = eval_conj(c, conj, f);
          c.suppress--;
          c.tmp = mark;
          pop_frame(c);
          if (!c.err && st == ST_PASS) query_retrieval(c, qi + 1, qid, cur, resolver, conv);
        } else {
          qr_push(c, mk_unres(cur, R_FILTER_NOT_STRUCT, qid, qi, 0));
        }
      }
      break;
    }
    case P_MAP_KEY_FILTER:
      if (cn.kind != K_MAP) { qr_push(c, mk_unres(cur, R_MAPFILTER_NOT_STRUCT, qid, qi, 0)); break; }
      map_key_filter(c, qi, qid, cur, cn, resolver, conv, part);
      break;
    default:
      fail(c, E_UNSUPPORTED, 6);
      break;
  }
  c.depth--;
}

// EvalContext::query for a frame
DEVN View scope_query(Ctx& c, uint32_t frame, uint32_t qid) {
  View v; v.off = c.tmp; v.n = 0;
  uint32_t f = frame;
  while (fr(c, f)->kind == F_PARAM) f = fr(c, f)->parent;
  Frame F = *fr(c, f);
  uint32_t start = c.tmp;
  if (F.kind == F_VALUE) query_retrieval(c, 0, qid, F.root, F.parent, 0);
  else query_retrieval(c, 0, qid, F.root, f, 0);
  v.off = start;
  v.n = (c.tmp - start) / 16;
  return v;
}

// copies a tmp view into the persist region
DEV View persist_view(Ctx& c, View v) {
  View p; p.n = v.n; p.off = alloc_pers(c, v.n ? v.n * 16 : 16);
  if (c.err) return p;
  for (uint32_t i = 0; i < v.n; i++) *qra(c, p.off + i * 16) = *qra(c, v.off + i * 16);
  return p;
}

// scope variable resolution (RootScope/BlockScope/ValueScope/ResolvedParameterContext)
DEVN View resolve_variable(Ctx& c, uint32_t frame, uint32_t var) {
  View none; none.off = 0; none.n = 0;
  uint32_t f = frame;
  for (uint32_t guard = 0; guard < 4096; guard++) {
    Frame F = *fr(c, f);
    if (F.kind == F_VALUE) { f = F.parent; continue; }
    if (F.kind == F_PARAM) {
      PParamRule pr = c.P->params[F.prule];
      for (uint32_t i = 0; i < pr.nparams; i++) {
        if (c.P->param_vars[pr.first_param + i] == var) {
          View v; v.off = u32a(c, F.params)[i * 2]; v.n = u32a(c, F.params)[i * 2 + 1];
          return v;
        }
      }
      f = F.parent; continue;
    }
    // ROOT / BLOCK: literal (last) > cached > function (last) > query (last)  (extract_variables)
    PBlock B = c.P->blocks[F.block];
    uint32_t lit_i = NONE, fn_i = NONE, q_i = NONE;
    for (uint32_t i = 0; i < B.nlets; i++) {
      PLet L = c.P->lets[B.first_let + i];
      if (L.var != var) continue;
      if (L.kind == L_LITERAL) lit_i = i; else if (L.kind == L_FUNC) fn_i = i; else q_i = i;
    }
    if (lit_i != NONE) {
      uint32_t* slot = u32a(c, F.cache + lit_i * 16);
      if (slot[0] == 0) {
        uint32_t o = alloc_pers(c, 16);
        if (c.err) return none;
        *qra(c, o) = mk_qr(c.P->lets[B.first_let + lit_i].id, QR_LITERAL);
        slot = u32a(c, F.cache + lit_i * 16);
        slot[0] = 1; slot[1] = o; slot[2] = 1;
      }
      View v; v.off = slot[1]; v.n = slot[2]; return v;
    }
    uint32_t use = fn_i != NONE ? fn_i : q_i;
    if (use == NONE) {
      if (F.kind == F_ROOT) { fail(c, E_VAR_MISSING, var); return none; }
      f = F.parent; continue;
    }
    uint32_t* slot = u32a(c, F.cache + use * 16);
    if (slot[0] == 1) { View v; v.off = slot[1]; v.n = slot[2]; return v; }
    PLet L = c.P->lets[B.first_let + use];
    uint32_t mark = c.tmp;
    View r;
    if (L.kind == L_FUNC) {
      r = resolve_function(c, L.id, f);
    } else {
      r = scope_query(c, f, L.id);
      if (!c.err && !c.P->queries[L.id].match_all) {
        // `some` lets keep only Resolved results (eval_context.rs:1148-1158)
        uint32_t k = 0;
        for (uint32_t i = 0; i < r.n; i++) {
          QR q = *qra(c, r.off + i * 16);
          if (qkind(q) == QR_RESOLVED) *qra(c, r.off + (k++) * 16) = q;
        }
        r.n = k;
      }
    }
    if (c.err) return none;
    View p = persist_view(c, r);
    c.tmp = mark;
    if (c.err) return none;
    slot = u32a(c, F.cache + use * 16);
    slot[0] = 1; slot[1] = p.off; slot[2] = p.n;
    return p;
  }
  fail(c, E_DEPTH);
  return none;
}

// count() (functions/collections.rs:6-23); other functions are outside the MI355X path
DEVN View resolve_function(Ctx& c, uint32_t fid, uint32_t frame) {
  PFunc F = c.P->funcs[fid];
  View out; out.off = c.tmp; out.n = 0;
  if (F.fname != F_COUNT || F.nargs != 1) { fail(c, E_UNSUPPORTED, 7); return out; }
  PLet A = c.P->lets[F.first_arg];
  View arg;
  if (A.kind == L_LITERAL) {
    arg.off = alloc_tmp(c, 16); arg.n = 1;
    if (c.err) return out;
    *qra(c, arg.off) = mk_qr(A.id, QR_LITERAL);
  } else if (A.kind == L_QUERY) {
    arg = scope_query(c, frame, A.id);
  } else {
    arg = resolve_function(c, A.id, frame);
  }
  if (c.err) return out;
  uint32_t cnt = 0;
  for (uint32_t i = 0; i < arg.n; i++) if (qkind(*qra(c, arg.off + i * 16)) != QR_UNRESOLVED) cnt++;
  uint32_t src = NONE;
  if (arg.n) src = qra(c, arg.off)->node;
  if (c.nsyn >= 256) { fail(c, E_HEAP); return out; }
  uint32_t* s = u32a(c, c.syn_off) + 4 * c.nsyn;
  s[0] = src; s[1] = cnt; s[2] = 0; s[3] = 0;
  uint32_t ref = SYN_BIT | c.nsyn++;
  out.off = alloc_tmp(c, 16); out.n = 1;
  if (c.err) return out;
  QR q = mk_qr(ref, QR_RESOLVED);
  *qra(c, out.off) = q;
  return out;
}

// ----------------------------------------------------------------- unary ---
DEV uint32_t cl_op(const PClause& pc) { return pc.flags & 15u; }
DEV bool cl_not(const PClause& pc) { return (pc.flags >> 4) & 1u; }
DEV bool cl_neg(const PClause& pc) { return (pc.flags >> 5) & 1u; }
DEV uint32_t cl_rhs(const PClause& pc) { return (pc.flags >> 8) & 15u; }
DEV bool cl_empty_expr(const PClause& pc) { return (pc.flags >> 12) & 1u; }

DEV void rec_unary(Ctx& c, uint32_t clause, QR from) {
  Rec r = mk_rec(REC_UNARY, clause); r.from = from; rec_push(c, r);
}

// returns: 0 = empty/skip, fills pass/fail counts
struct Agg { uint32_t pass, fail; bool empty; uint32_t empty_status; };

DEVN Agg unary_operation(Ctx& c, uint32_t clause, const PClause& pc, uint32_t frame) {
  Agg g; g.pass = 0; g.fail = 0; g.empty = false; g.empty_status = ST_SKIP;
  View lhs = scope_query(c, frame, pc.a);
  if (c.err) return g;
  uint32_t op = cl_op(pc);
  bool neg = cl_not(pc), inverse = cl_neg(pc);
  if (cl_empty_expr(pc) && op == OP_EMPTY) {
    if (lhs.n) {
      for (uint32_t i = 0; i < lhs.n; i++) {
        QR e = *qra(c, lhs.off + i * 16);
        bool pass;
        QR res = e;
        if (qkind(e) != QR_UNRESOLVED) {
          DNode n = node(c, e.node);
          bool isnull = n.kind == K_NULL;
          pass = neg ? !isnull : isnull;
          res = mk_qr(e.node, QR_RESOLVED);
        } else {
          pass = !neg;
        }
        if (inverse) pass = !pass;
        if (pass) g.pass++; else { g.fail++; rec_unary(c, clause, res); }
      }
      return g;
    }
    bool result = !neg;
    if (inverse) result = !result;
    g.empty = true;
    if (result) g.empty_status = ST_PASS;
    else { g.empty_status = ST_FAIL; rec_push(c, mk_rec(REC_NOVALUE_EMPTY, clause)); }
    return g;
  }
  if (lhs.n == 0) { g.empty = true; g.empty_status = ST_SKIP; return g; }
  for (uint32_t i = 0; i < lhs.n; i++) {
    QR e = *qra(c, lhs.off + i * 16);
    bool r;
    if (qkind(e) == QR_UNRESOLVED) {
      r = op == OP_EMPTY;   // !EXISTS == EMPTY; IS_* false
    } else {
      DNode n = node(c, e.node);
      switch (op) {
        case OP_EXISTS: r = true; break;
        case OP_EMPTY:
          if (n.kind == K_LIST || n.kind == K_MAP || n.kind == K_STRING) r = n.count == 0;
          else if (n.kind == K_BOOL) r = false;
          else { fail(c, E_EMPTY_INCOMPATIBLE, e.node, n.kind); return g; }
          break;
        case OP_IS_STRING: r = n.kind == K_STRING; break;
        case OP_IS_LIST: r = n.kind == K_LIST; break;
        case OP_IS_MAP: r = n.kind == K_MAP; break;
        case OP_IS_BOOL: r = n.kind == K_BOOL; break;
        case OP_IS_INT: r = n.kind == K_INT; break;
        case OP_IS_FLOAT: r = n.kind == K_FLOAT; break;
        default: r = n.kind == K_NULL; break;
      }
    }
    if (neg) r = !r;
    if (inverse) r = !r;
    if (r) g.pass++; else { g.fail++; rec_unary(c, clause, e); }
  }
  return g;
}

// ---------------------------------------------------------------- binary ---
// ValueEvalResult (operators.rs:62-96) staged on the tmp stack
enum VerKind : uint32_t { V_LHS_UNRES = 0, V_RHS_UNRES = 1, V_NOTCMP = 2, V_SUCCESS = 3, V_FAIL = 4 };
enum CmpKind : uint32_t { CK_VALUE = 0, CK_VALUEIN = 1, CK_LISTIN = 2, CK_QUERYIN = 3 };

struct Ver {
  uint32_t kind, ck;
  uint32_t a, b;         // lhs / rhs node refs (or list nodes)
  QR u;                  // unresolved (LHS/RHS_UNRES)
  uint32_t diff_off, diff_n, l_off, l_n, r_off, r_n, nc, nct;
};

DEV Ver* vera(Ctx& c, uint32_t off) { return (Ver*)(c.heap + off); }

DEV void ver_push(Ctx& c, const Ver& v) {
  uint32_t o = alloc_tmp(c, sizeof(Ver));
  CHK(c);
  *vera(c, o) = v;
}
DEV Ver mk_ver(uint32_t kind, uint32_t ck, uint32_t a, uint32_t b) {
  Ver v; v.kind = kind; v.ck = ck; v.a = a; v.b = b; v.u = mk_qr(NONE, 0);
  v.diff_off = 0; v.diff_n = 0; v.l_off = 0; v.l_n = 0; v.r_off = 0; v.r_n = 0; v.nc = 0; v.nct = 0;
  return v;
}

// node-ref arrays on the tmp stack
struct Arr { uint32_t off, n; };
DEV Arr arr_new(Ctx& c, uint32_t cap) { Arr a; a.off = alloc_tmp(c, (cap ? cap : 1) * 4); a.n = 0; return a; }
DEV void arr_put(Ctx& c, Arr& a, uint32_t v) { u32a(c, a.off)[a.n++] = v; }
DEV uint32_t arr_at(Ctx& c, const Arr& a, uint32_t i) { return u32a(c, a.off)[i]; }

DEV bool arr_contains(Ctx& c, const Arr& a, uint32_t ref) {
  for (uint32_t i = 0; i < a.n; i++) if (pv_eq(c, arr_at(c, a, i), ref, 0)) return true;
  return false;
}
DEV bool list_contains(Ctx& c, uint32_t list_ref, uint32_t ref) {
  DNode l = node(c, list_ref);
  for (uint32_t i = 0; i < l.count; i++) if (pv_eq(c, child(list_ref, l, i), ref, 0)) return true;
  return false;
}

// match_value with compare_eq / Common comparator
DEV Ver match_value(Ctx& c, uint32_t l, uint32_t r, uint32_t op) {
  Cmp x;
  if (op == OP_EQ) x = compare_eq(c, l, r, 0);
  else { DNode a = node(c, l), b = node(c, r); x = compare_values(c, l, a, r, b); }
  if (x.status == 3) return mk_ver(V_FAIL, CK_VALUE, l, r);  // error already raised
  if (x.status) { Ver v = mk_ver(V_NOTCMP, CK_VALUE, l, r); v.nc = x.status == 1 ? NC_TYPES : NC_FLOAT; v.nct = (x.ka << 8) | x.kb; return v; }
  bool ok;
  if (op == OP_EQ) ok = x.ord == 0;
  else if (op == OP_LT) ok = x.ord < 0;
  else if (op == OP_LE) ok = x.ord <= 0;
  else if (op == OP_GT) ok = x.ord > 0;
  else ok = x.ord >= 0;
  return mk_ver(ok ? V_SUCCESS : V_FAIL, CK_VALUE, l, r);
}

DEV Ver string_in(Ctx& c, uint32_t l, uint32_t r) {
  DNode a = node(c, l), b = node(c, r);
  if (a.kind == K_STRING && b.kind == K_STRING) {
    const char* hay = bytes_of(c, r) + b.a;
    const char* nd = bytes_of(c, l) + a.a;
    bool found = a.count == 0;
    for (uint32_t i = 0; !found && i + a.count <= b.count; i++) found = bytes_eq(hay + i, nd, a.count);
    return mk_ver(found ? V_SUCCESS : V_FAIL, CK_VALUE, l, r);
  }
  Ver v = mk_ver(V_NOTCMP, CK_VALUE, l, r); v.nc = NC_STRING_IN; return v;
}

DEV Ver contained_in(Ctx& c, uint32_t l, uint32_t r) {
  DNode a = node(c, l), b = node(c, r);
  if (a.kind == K_LIST) {
    if (b.kind == K_LIST) {
      if (b.count && node(c, child(r, b, 0)).kind == K_LIST) {
        bool in = list_contains(c, r, l);
        Ver v = mk_ver(in ? V_SUCCESS : V_FAIL, CK_LISTIN, l, r);
        if (!in) { Arr d = arr_new(c, 1); if (!c.err) arr_put(c, d, l); v.diff_off = d.off; v.diff_n = d.n; }
        return v;
      }
      Arr d = arr_new(c, a.count);
      if (c.err) return mk_ver(V_FAIL, CK_LISTIN, l, r);
      for (uint32_t i = 0; i < a.count; i++) {
        uint32_t e = child(l, a, i);
        if (!list_contains(c, r, e)) arr_put(c, d, e);
      }
      Ver v = mk_ver(d.n == 0 ? V_SUCCESS : V_FAIL, CK_LISTIN, l, r);
      v.diff_off = d.off; v.diff_n = d.n;
      return v;
    }
    Ver v = mk_ver(V_NOTCMP, CK_VALUE, l, r); v.nc = NC_CONTAINED_IN; return v;
  }
  if (b.kind == K_LIST) return mk_ver(list_contains(c, r, l) ? V_SUCCESS : V_FAIL, CK_VALUEIN, l, r);
  return match_value(c, l, r, OP_EQ);
}

DEV bool is_literal_view(Ctx& c, View v, uint32_t& node_out) {
  if (v.n == 1) { QR q = *qra(c, v.off); if (qkind(q) == QR_LITERAL) { node_out = q.node; return true; } }
  return false;
}

// resolved/literal selection (operators.rs:116-130); unresolved go through on_unres
DEV Arr selected(Ctx& c, View v) {
  Arr a = arr_new(c, v.n);
  if (c.err) return a;
  for (uint32_t i = 0; i < v.n; i++) { QR q = *qra(c, v.off + i * 16); if (qkind(q) != QR_UNRESOLVED) arr_put(c, a, q.node); }
  return a;
}
DEV Arr flattened(Ctx& c, View v) {
  uint32_t cap = 0;
  for (uint32_t i = 0; i < v.n; i++) {
    QR q = *qra(c, v.off + i * 16);
    if (qkind(q) == QR_UNRESOLVED) continue;
    DNode n = node(c, q.node);
    cap += n.kind == K_LIST ? n.count : 1;
  }
  Arr a = arr_new(c, cap);
  if (c.err) return a;
  for (uint32_t i = 0; i < v.n; i++) {
    QR q = *qra(c, v.off + i * 16);
    if (qkind(q) == QR_UNRESOLVED) continue;
    DNode n = node(c, q.node);
    if (n.kind == K_LIST) for (uint32_t j = 0; j < n.count; j++) arr_put(c, a, child(q.node, n, j));
    else arr_put(c, a, q.node);
  }
  return a;
}
DEV void push_lhs_unres(Ctx& c, View v) {
  for (uint32_t i = 0; i < v.n; i++) {
    QR q = *qra(c, v.off + i * 16);
    if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_LHS_UNRES, 0, NONE, NONE); e.u = q; ver_push(c, e); }
  }
}
DEV void push_rhs_unres(Ctx& c, View rhs, const Arr& lhs_sel) {
  for (uint32_t i = 0; i < rhs.n; i++) {
    QR q = *qra(c, rhs.off + i * 16);
    if (qkind(q) != QR_UNRESOLVED) continue;
    for (uint32_t j = 0; j < lhs_sel.n; j++) { Ver e = mk_ver(V_RHS_UNRES, 0, arr_at(c, lhs_sel, j), NONE); e.u = q; ver_push(c, e); }
  }
}
DEV void push_rhs_unres_single(Ctx& c, View rhs, uint32_t l) {
  for (uint32_t i = 0; i < rhs.n; i++) {
    QR q = *qra(c, rhs.off + i * 16);
    if (qkind(q) != QR_UNRESOLVED) continue;
    Ver e = mk_ver(V_RHS_UNRES, 0, l, NONE); e.u = q; ver_push(c, e);
  }
}

// QueryIn over selected lhs/rhs with a diff built by `contained_in` (InOperation) or PartialEq (Eq)
DEV void push_queryin(Ctx& c, Arr diff, Arr ls, Arr rs) {
  Ver v = mk_ver(diff.n == 0 ? V_SUCCESS : V_FAIL, CK_QUERYIN, NONE, NONE);
  v.diff_off = diff.off; v.diff_n = diff.n; v.l_off = ls.off; v.l_n = ls.n; v.r_off = rs.off; v.r_n = rs.n;
  ver_push(c, v);
}

// operators.rs: EqOperation / InOperation / CommonOperator then (op, not) reverse diffs.
// Returns number of Ver entries written starting at *start; returns false for Skip.
DEVN bool compare_op(Ctx& c, uint32_t op, bool neg, View lhs, View rhs, uint32_t& start, uint32_t& count) {
  if (lhs.n == 0 || rhs.n == 0) return false;
  uint32_t aux_mark = c.tmp;
  // all auxiliary arrays are allocated before the Ver list so the list stays contiguous:
  // collect Vers into a separate region by first computing into the tmp stack, then compacting.
  uint32_t vstart = c.tmp;
  uint32_t lnode, rnode;
  bool ll = is_literal_view(c, lhs, lnode), rl = is_literal_view(c, rhs, rnode);
  // Ver entries and arrays interleave on the tmp stack; we record Ver offsets in an index array.
  // (simple approach: push Vers into a linked list via a side index)
  const uint32_t MAXV = 4096;
  uint32_t idx_off = alloc_tmp(c, MAXV * 4);
  if (c.err) return false;
  uint32_t nv = 0;
  auto add = [&](const Ver& v) {
    if (nv >= MAXV) { fail(c, E_HEAP); return; }
    uint32_t o = alloc_tmp(c, sizeof(Ver));
    if (c.err) return;
    *vera(c, o) = v;
    u32a(c, idx_off)[nv++] = o;
  };
  if (op == OP_EQ) {
    if (ll && rl) add(match_value(c, lnode, rnode, OP_EQ));
    else if (ll) {
      for (uint32_t i = 0; i < rhs.n; i++) { QR q = *qra(c, rhs.off + i * 16); if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_RHS_UNRES, 0, lnode, NONE); e.u = q; add(e); } }
      DNode ln = node(c, lnode);
      for (uint32_t i = 0; i < rhs.n && !c.err; i++) {
        QR q = *qra(c, rhs.off + i * 16);
        if (qkind(q) == QR_UNRESOLVED) continue;
        if (ln.kind == K_LIST) add(match_value(c, lnode, q.node, OP_EQ));
        else {
          DNode rn = node(c, q.node);
          if (rn.kind == K_LIST) for (uint32_t j = 0; j < rn.count && !c.err; j++) add(match_value(c, lnode, child(q.node, rn, j), OP_EQ));
          else add(match_value(c, lnode, q.node, OP_EQ));
        }
      }
    } else if (rl) {
      for (uint32_t i = 0; i < lhs.n; i++) { QR q = *qra(c, lhs.off + i * 16); if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_LHS_UNRES, 0, NONE, NONE); e.u = q; add(e); } }
      DNode rn = node(c, rnode);
      for (uint32_t i = 0; i < lhs.n && !c.err; i++) {
        QR q = *qra(c, lhs.off + i * 16);
        if (qkind(q) == QR_UNRESOLVED) continue;
        DNode en = node(c, q.node);
        if (rn.kind == K_LIST) {
          if (is_scalar_k(en.kind) && rn.count == 1) add(match_value(c, q.node, child(rnode, rn, 0), OP_EQ));
          else add(match_value(c, q.node, rnode, OP_EQ));
        } else {
          if (en.kind == K_LIST) for (uint32_t j = 0; j < en.count && !c.err; j++) add(match_value(c, child(q.node, en, j), rnode, OP_EQ));
          else add(match_value(c, q.node, rnode, OP_EQ));
        }
      }
    } else {
      for (uint32_t i = 0; i < lhs.n; i++) { QR q = *qra(c, lhs.off + i * 16); if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_LHS_UNRES, 0, NONE, NONE); e.u = q; add(e); } }
      Arr ls = selected(c, lhs);
      Arr rs = selected(c, rhs);
      if (c.err) return false;
      for (uint32_t i = 0; i < rhs.n; i++) {
        QR q = *qra(c, rhs.off + i * 16);
        if (qkind(q) != QR_UNRESOLVED) continue;
        for (uint32_t j = 0; j < ls.n; j++) { Ver e = mk_ver(V_RHS_UNRES, 0, arr_at(c, ls, j), NONE); e.u = q; add(e); }
      }
      Arr diff;
      if (ls.n > rs.n) { diff = arr_new(c, ls.n); for (uint32_t i = 0; i < ls.n && !c.err; i++) { uint32_t e = arr_at(c, ls, i); if (!arr_contains(c, rs, e)) arr_put(c, diff, e); } }
      else { diff = arr_new(c, rs.n); for (uint32_t i = 0; i < rs.n && !c.err; i++) { uint32_t e = arr_at(c, rs, i); if (!arr_contains(c, ls, e)) arr_put(c, diff, e); } }
      Ver v = mk_ver(diff.n == 0 ? V_SUCCESS : V_FAIL, CK_QUERYIN, NONE, NONE);
      v.diff_off = diff.off; v.diff_n = diff.n; v.l_off = ls.off; v.l_n = ls.n; v.r_off = rs.off; v.r_n = rs.n;
      add(v);
    }
  } else if (op == OP_IN) {
    if (ll && rl) {
      Ver v = string_in(c, lnode, rnode);
      if (v.kind != V_SUCCESS) v = contained_in(c, lnode, rnode);
      add(v);
    } else if (ll) {
      for (uint32_t i = 0; i < rhs.n; i++) { QR q = *qra(c, rhs.off + i * 16); if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_RHS_UNRES, 0, lnode, NONE); e.u = q; add(e); } }
      Arr rs = selected(c, rhs);
      if (c.err) return false;
      bool any_list = false;
      for (uint32_t i = 0; i < rs.n; i++) if (node(c, arr_at(c, rs, i)).kind == K_LIST) any_list = true;
      DNode ln = node(c, lnode);
      if (any_list) { for (uint32_t i = 0; i < rs.n && !c.err; i++) add(contained_in(c, lnode, arr_at(c, rs, i))); }
      else if (ln.kind == K_LIST) {
        Arr diff = arr_new(c, ln.count);
        for (uint32_t i = 0; i < ln.count && !c.err; i++) { uint32_t e = child(lnode, ln, i); if (!arr_contains(c, rs, e)) arr_put(c, diff, e); }
        Arr ls = arr_new(c, 1); if (!c.err) arr_put(c, ls, lnode);
        Ver v = mk_ver(diff.n == 0 ? V_SUCCESS : V_FAIL, CK_QUERYIN, NONE, NONE);
        v.diff_off = diff.off; v.diff_n = diff.n; v.l_off = ls.off; v.l_n = ls.n; v.r_off = rs.off; v.r_n = rs.n;
        add(v);
      } else {
        for (uint32_t i = 0; i < rs.n && !c.err; i++) add(contained_in(c, lnode, arr_at(c, rs, i)));
      }
    } else if (rl) {
      DNode rn = node(c, rnode);
      for (uint32_t i = 0; i < lhs.n && !c.err; i++) {
        QR q = *qra(c, lhs.off + i * 16);
        if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_LHS_UNRES, 0, NONE, NONE); e.u = q; add(e); continue; }
      }
      for (uint32_t i = 0; i < lhs.n && !c.err; i++) {
        QR q = *qra(c, lhs.off + i * 16);
        if (qkind(q) == QR_UNRESOLVED) continue;
        DNode en = node(c, q.node);
        if (rn.kind == K_STRING) {
          if (en.kind == K_LIST) for (uint32_t j = 0; j < en.count && !c.err; j++) add(string_in(c, child(q.node, en, j), rnode));
          else add(string_in(c, q.node, rnode));
        } else add(contained_in(c, q.node, rnode));
      }
    } else {
      for (uint32_t i = 0; i < lhs.n; i++) { QR q = *qra(c, lhs.off + i * 16); if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_LHS_UNRES, 0, NONE, NONE); e.u = q; add(e); } }
      Arr ls = selected(c, lhs);
      Arr rs = selected(c, rhs);
      if (c.err) return false;
      for (uint32_t i = 0; i < rhs.n; i++) {
        QR q = *qra(c, rhs.off + i * 16);
        if (qkind(q) != QR_UNRESOLVED) continue;
        for (uint32_t j = 0; j < ls.n; j++) { Ver e = mk_ver(V_RHS_UNRES, 0, arr_at(c, ls, j), NONE); e.u = q; add(e); }
      }
      Arr diff = arr_new(c, ls.n);
      for (uint32_t i = 0; i < ls.n && !c.err; i++) {
        uint32_t el = arr_at(c, ls, i);
        bool found = false;
        for (uint32_t j = 0; j < rs.n && !c.err && !found; j++) {
          uint32_t mark = c.tmp;
          found = contained_in(c, el, arr_at(c, rs, j)).kind == V_SUCCESS;
          c.tmp = mark;
        }
        if (!found) arr_put(c, diff, el);
      }
      Ver v = mk_ver(diff.n == 0 ? V_SUCCESS : V_FAIL, CK_QUERYIN, NONE, NONE);
      v.diff_off = diff.off; v.diff_n = diff.n; v.l_off = ls.off; v.l_n = ls.n; v.r_off = rs.off; v.r_n = rs.n;
      add(v);
    }
  } else {
    // CommonOperator (Lt/Gt/Le/Ge): flattened cross product
    for (uint32_t i = 0; i < lhs.n; i++) { QR q = *qra(c, lhs.off + i * 16); if (qkind(q) == QR_UNRESOLVED) { Ver e = mk_ver(V_LHS_UNRES, 0, NONE, NONE); e.u = q; add(e); } }
    Arr lf = flattened(c, lhs);
    if (c.err) return false;
    for (uint32_t i = 0; i < rhs.n; i++) {
      QR q = *qra(c, rhs.off + i * 16);
      if (qkind(q) != QR_UNRESOLVED) continue;
      for (uint32_t j = 0; j < lf.n; j++) { Ver e = mk_ver(V_RHS_UNRES, 0, arr_at(c, lf, j), NONE); e.u = q; add(e); }
    }
    Arr rf = flattened(c, rhs);
    if (c.err) return false;
    for (uint32_t i = 0; i < lf.n && !c.err; i++)
      for (uint32_t j = 0; j < rf.n && !c.err; j++) add(match_value(c, arr_at(c, lf, i), arr_at(c, rf, j), op));
  }
  if (c.err) return false;
  (void)aux_mark; (void)vstart;
  if (neg) {
    for (uint32_t k = 0; k < nv && !c.err; k++) {
      Ver* v = vera(c, u32a(c, idx_off)[k]);
      if (v->kind == V_FAIL) {
        if (v->ck == CK_QUERYIN) {
          bool use_r = rhs.n >= lhs.n && op == OP_EQ;
          Arr other; other.off = use_r ? v->r_off : v->l_off; other.n = use_r ? v->r_n : v->l_n;
          Arr d; d.off = v->diff_off; d.n = v->diff_n;
          Arr rd = arr_new(c, other.n);
          for (uint32_t i = 0; i < other.n && !c.err; i++) { uint32_t e = arr_at(c, other, i); if (!arr_contains(c, d, e)) arr_put(c, rd, e); }
          v = vera(c, u32a(c, idx_off)[k]);
          v->kind = rd.n == 0 ? V_SUCCESS : V_FAIL; v->diff_off = rd.off; v->diff_n = rd.n;
        } else if (v->ck == CK_LISTIN) {
          DNode ln = node(c, v->a);
          Arr d; d.off = v->diff_off; d.n = v->diff_n;
          Arr rd = arr_new(c, ln.count);
          for (uint32_t i = 0; i < ln.count && !c.err; i++) { uint32_t e = child(v->a, ln, i); if (!arr_contains(c, d, e)) arr_put(c, rd, e); }
          v = vera(c, u32a(c, idx_off)[k]);
          v->kind = rd.n == 0 ? V_SUCCESS : V_FAIL; v->diff_off = rd.off; v->diff_n = rd.n;
        } else {
          v->kind = V_SUCCESS;
        }
      } else if (v->kind == V_SUCCESS) {
        if (v->ck == CK_QUERYIN) { v->kind = V_FAIL; v->diff_off = v->l_off; v->diff_n = v->l_n; }
        else if (v->ck == CK_LISTIN) {
          DNode ln = node(c, v->a);
          Arr rd = arr_new(c, ln.count);
          for (uint32_t i = 0; i < ln.count && !c.err; i++) arr_put(c, rd, child(v->a, ln, i));
          v = vera(c, u32a(c, idx_off)[k]);
          v->kind = V_FAIL; v->diff_off = rd.off; v->diff_n = rd.n;
        } else v->kind = V_FAIL;
      }
    }
  }
  start = idx_off;
  count = nv;
  return !c.err;
}

DEV void rec_cmp(Ctx& c, uint32_t clause, QR from, QR to, bool has_to, uint32_t nc, uint32_t nct) {
  Rec r = mk_rec(REC_CMP, clause);
  r.from = from;
  if (has_to) r.to = to;
  r.x = nc; r.y = nct;
  rec_push(c, r);
}
DEV void rec_in(Ctx& c, uint32_t clause, uint32_t from, uint32_t to_off, uint32_t to_n, bool to_is_single, uint32_t single) {
  if (c.suppress) return;
  Rec r = mk_rec(REC_IN, clause);
  r.from = mk_qr(from, QR_RESOLVED);
  r.x = to_is_single ? 1 : to_n;
  rec_push(c, r);
  uint32_t n = to_is_single ? 1 : to_n;
  for (uint32_t i = 0; i < n; i += 2) {
    Rec l = mk_rec(REC_LIST, clause);
    l.from = mk_qr(to_is_single ? single : u32a(c, to_off)[i], QR_RESOLVED);
    if (i + 1 < n) l.to = mk_qr(u32a(c, to_off)[i + 1], QR_RESOLVED);
    rec_push(c, l);
  }
}

DEVN Agg binary_operation(Ctx& c, uint32_t clause, const PClause& pc, View rhs, uint32_t frame) {
  Agg g; g.pass = 0; g.fail = 0; g.empty = false; g.empty_status = ST_SKIP;
  View lhs = scope_query(c, frame, pc.a);
  if (c.err) return g;
  uint32_t start = 0, nv = 0;
  if (!compare_op(c, cl_op(pc), cl_not(pc), lhs, rhs, start, nv)) {
    if (!c.err) { g.empty = true; g.empty_status = ST_SKIP; }
    return g;
  }
  for (uint32_t k = 0; k < nv && !c.err; k++) {
    Ver v = *vera(c, u32a(c, start)[k]);
    switch (v.kind) {
      case V_LHS_UNRES: rec_cmp(c, clause, v.u, v.u, false, 0, 0); g.fail++; break;
      case V_RHS_UNRES: rec_cmp(c, clause, mk_qr(v.a, QR_RESOLVED), v.u, true, 0, 0); g.fail++; break;
      case V_NOTCMP: rec_cmp(c, clause, mk_qr(v.a, QR_RESOLVED), mk_qr(v.b, QR_RESOLVED), true, v.nc, v.nct); g.fail++; break;
      case V_SUCCESS:
        if (v.ck == CK_QUERYIN) g.pass += v.l_n; else g.pass++;
        break;
      default:
        if (v.ck == CK_VALUE) { rec_cmp(c, clause, mk_qr(v.a, QR_RESOLVED), mk_qr(v.b, QR_RESOLVED), true, 0, 0); g.fail++; }
        else if (v.ck == CK_VALUEIN) { rec_in(c, clause, v.a, 0, 0, true, v.b); g.fail++; }
        else if (v.ck == CK_LISTIN) { rec_in(c, clause, v.a, 0, 0, true, v.b); g.fail++; }
        else {
          for (uint32_t i = 0; i < v.diff_n && !c.err; i++) { rec_in(c, clause, u32a(c, v.diff_off)[i], v.r_off, v.r_n, false, 0); g.fail++; }
        }
        break;
    }
  }
  return g;
}

// ----------------------------------------------------------------- clauses ---
DEVN uint32_t eval_clause(Ctx& c, uint32_t cid, uint32_t frame);

// container that is "flattened" into its parent when FAIL and dropped otherwise
DEV void flat_close(Ctx& c, uint32_t mark, uint32_t status) { if (status != ST_FAIL && !c.suppress) c.nrec = mark; }

DEVN uint32_t eval_access(Ctx& c, uint32_t cid, const PClause& pc, uint32_t frame) {
  uint32_t mark = c.nrec;
  uint32_t tmark = c.tmp;
  bool all = c.P->queries[pc.a].match_all != 0;
  Agg g;
  uint32_t op = cl_op(pc);
  if (op >= OP_EXISTS) {
    g = unary_operation(c, cid, pc, frame);
  } else {
    uint32_t rk = cl_rhs(pc);
    View rhs;
    if (rk == RHS_LITERAL) {
      rhs.off = alloc_tmp(c, 16); rhs.n = 1;
      if (c.err) return ST_FAIL;
      *qra(c, rhs.off) = mk_qr(pc.b, QR_LITERAL);
    } else if (rk == RHS_QUERY) {
      rhs = scope_query(c, frame, pc.b);
    } else if (rk == RHS_FUNC) {
      rhs = resolve_function(c, pc.b, frame);
    } else {
      fail(c, E_NO_RHS, cid);
      return ST_FAIL;
    }
    if (c.err) return ST_FAIL;
    g = binary_operation(c, cid, pc, rhs, frame);
  }
  c.tmp = tmark;
  if (c.err) return ST_FAIL;
  uint32_t st;
  if (g.empty) st = g.empty_status;
  else if (all) st = g.fail ? ST_FAIL : ST_PASS;
  else st = g.pass ? ST_PASS : ST_FAIL;
  flat_close(c, mark, st);   // GuardClauseBlockCheck
  return st;
}

DEVN uint32_t rule_status(Ctx& c, uint32_t slot) {
  uint32_t* memo = u32a(c, c.memo);
  if (memo[slot] != 3u) return memo[slot];
  PRange2 nr = c.P->name_rules[slot];
  uint32_t st = ST_SKIP;
  c.suppress++;
  for (uint32_t i = 0; i < nr.n && !c.err; i++) {
    uint32_t s = eval_rule(c, c.P->name_rule_ids[nr.first + i], 0, NONE);
    if (s != ST_SKIP) { st = s; break; }
  }
  c.suppress--;
  if (c.err) return ST_FAIL;
  u32a(c, c.memo)[slot] = st;
  return st;
}

DEVN uint32_t eval_named(Ctx& c, uint32_t cid, const PClause& pc) {
  if (pc.a == NONE) { fail(c, E_RULE_MISSING, cid); return ST_FAIL; }
  uint32_t st = rule_status(c, pc.a);
  if (c.err) return ST_FAIL;
  bool neg = pc.flags & 1u;
  uint32_t out = st == ST_PASS ? (neg ? ST_FAIL : ST_PASS) : (neg ? ST_PASS : ST_FAIL);
  if (out == ST_FAIL) rec_push(c, mk_rec(REC_DEPENDENT_RULE, cid));
  return out;
}

// eval_general_block_clause: BlockScope(block, resolver.root(), resolver)
DEVN uint32_t eval_block(Ctx& c, uint32_t block, uint32_t frame) {
  uint32_t root = frame_root(c, frame);
  uint32_t f = push_frame(c, F_BLOCK, frame, root, block);
  if (c.err) return ST_FAIL;
  uint32_t st = eval_conj(c, c.P->blocks[block].conj, f);
  pop_frame(c);
  return st;
}

DEVN uint32_t eval_block_clause(Ctx& c, uint32_t cid, const PClause& pc, uint32_t frame) {
  uint32_t mark = c.nrec;
  uint32_t created0 = c.rec_created;
  uint32_t tmark = c.tmp;
  bool match_all = c.P->queries[pc.a].match_all != 0;
  View vals = scope_query(c, frame, pc.a);
  if (c.err) return ST_FAIL;
  if (vals.n == 0) {
    uint32_t st = (pc.flags & 1u) ? ST_FAIL : ST_SKIP;
    if (st == ST_FAIL && c.rec_created == created0) rec_push(c, mk_rec(REC_BLOCK_EMPTY, cid));
    c.tmp = tmark;
    if (st != ST_FAIL && !c.suppress) c.nrec = mark;
    return st;
  }
  uint32_t fails = 0, passes = 0;
  for (uint32_t i = 0; i < vals.n && !c.err; i++) {
    QR e = *qra(c, vals.off + i * 16);
    if (qkind(e) == QR_UNRESOLVED) {
      fails++;
      c.rec_created++;
      Rec r = mk_rec(REC_MISSING_BLOCK_VALUE, cid); r.from = e; rec_push(c, r);
      continue;
    }
    if (e.node & SYN_BIT) { fail(c, E_UNSUPPORTED, 3); break; }
    uint32_t f = push_frame(c, F_VALUE, frame, e.node, NONE);
    if (c.err) break;
    uint32_t st = eval_block(c, pc.b, f);
    pop_frame(c);
    if (st == ST_PASS) passes++; else if (st == ST_FAIL) fails++;
  }
  c.tmp = tmark;
  if (c.err) return ST_FAIL;
  uint32_t st;
  if (match_all) st = fails ? ST_FAIL : (passes ? ST_PASS : ST_SKIP);
  else st = passes ? ST_PASS : (fails ? ST_FAIL : ST_SKIP);
  flat_close(c, mark, st);
  return st;
}

DEVN uint32_t eval_when_block(Ctx& c, const PClause& pc, uint32_t frame) {
  uint32_t mark = c.nrec;
  c.suppress++;
  uint32_t cond = eval_conj(c, pc.a, frame);
  c.suppress--;
  if (c.err) return ST_FAIL;
  if (cond != ST_PASS) { if (!c.suppress) c.nrec = mark; return ST_SKIP; }
  uint32_t st = eval_block(c, pc.b, frame);
  if (c.err) return ST_FAIL;
  flat_close(c, mark, st);   // WhenCheck
  return st;
}

DEVN uint32_t eval_type_block(Ctx& c, uint32_t cid, const PClause& pc, uint32_t frame) {
  uint32_t mark = c.nrec;
  if (pc.c != NONE) {
    c.suppress++;
    uint32_t cond = eval_conj(c, pc.c, frame);
    c.suppress--;
    if (c.err) return ST_FAIL;
    if (cond != ST_PASS) return ST_SKIP;
  }
  uint32_t tmark = c.tmp;
  View vals = scope_query(c, frame, pc.a);
  if (c.err) return ST_FAIL;
  if (vals.n == 0) { c.tmp = tmark; return ST_SKIP; }
  uint32_t fails = 0, passes = 0;
  for (uint32_t i = 0; i < vals.n && !c.err; i++) {
    QR e = *qra(c, vals.off + i * 16);
    if (qkind(e) == QR_UNRESOLVED) { fail(c, E_TYPEBLOCK_UNRESOLVED, cid); break; }
    uint32_t vmark = c.nrec;
    uint32_t f = push_frame(c, F_VALUE, frame, e.node, NONE);
    if (c.err) break;
    uint32_t st = eval_block(c, pc.b, f);
    pop_frame(c);
    if (st == ST_PASS) passes++; else if (st == ST_FAIL) fails++;
    flat_close(c, vmark, st);   // TypeBlock(status) per value
  }
  c.tmp = tmark;
  if (c.err) return ST_FAIL;
  uint32_t st = fails ? ST_FAIL : (passes ? ST_PASS : ST_SKIP);
  flat_close(c, mark, st);       // TypeCheck
  return st;
}

DEVN uint32_t eval_param_call(Ctx& c, uint32_t cid, const PClause& pc, uint32_t frame) {
  if (pc.a == NONE) { fail(c, E_PARAM_MISSING, cid); return ST_FAIL; }
  PParamRule pr = c.P->params[pc.a];
  if (pr.nparams != pc.c) { fail(c, E_PARAM_ARITY, cid, pr.nparams); return ST_FAIL; }
  uint32_t po = alloc_pers(c, (pr.nparams ? pr.nparams : 1) * 8);
  if (c.err) return ST_FAIL;
  for (uint32_t i = 0; i < pc.c && !c.err; i++) {
    PLet a = c.P->lets[pc.b + i];
    View v;
    uint32_t tmark = c.tmp;
    if (a.kind == L_LITERAL) {
      v.off = alloc_tmp(c, 16); v.n = 1;
      if (c.err) break;
      *qra(c, v.off) = mk_qr(a.id, QR_RESOLVED);
    } else if (a.kind == L_QUERY) {
      v = scope_query(c, frame, a.id);
    } else {
      v = resolve_function(c, a.id, frame);
    }
    if (c.err) break;
    View p = persist_view(c, v);
    c.tmp = tmark;
    u32a(c, po)[i * 2] = p.off;
    u32a(c, po)[i * 2 + 1] = p.n;
  }
  if (c.err) return ST_FAIL;
  uint32_t f = push_frame(c, F_PARAM, frame, NONE, NONE);
  if (c.err) return ST_FAIL;
  fr(c, f)->call = cid; fr(c, f)->params = po; fr(c, f)->prule = pc.a;
  uint32_t st = eval_rule(c, pr.rule, f, pc.e);
  pop_frame(c);
  return st;
}

DEVN uint32_t eval_clause(Ctx& c, uint32_t cid, uint32_t frame) {
  if (++c.depth > MAX_DEPTH) { fail(c, E_DEPTH); c.depth--; return ST_FAIL; }
  const PClause pc = c.P->clauses[cid];
  uint32_t st;
  switch (pc.kind) {
    case C_ACCESS: st = eval_access(c, cid, pc, frame); break;
    case C_NAMED: st = eval_named(c, cid, pc); break;
    case C_BLOCK: st = eval_block_clause(c, cid, pc, frame); break;
    case C_WHEN: st = eval_when_block(c, pc, frame); break;
    case C_TYPEBLOCK: st = eval_type_block(c, cid, pc, frame); break;
    case C_PARAM: st = eval_param_call(c, cid, pc, frame); break;
    default: fail(c, E_UNSUPPORTED, 8); st = ST_FAIL; break;
  }
  c.depth--;
  return st;
}

// eval_conjunction_clauses (eval.rs:1970-2065)
DEVN uint32_t eval_conj(Ctx& c, uint32_t conj, uint32_t frame) {
  PRange2 cj = c.P->conjs[conj];
  uint32_t num_pass = 0, num_fail = 0;
  for (uint32_t i = 0; i < cj.n && !c.err; i++) {
    PRange2 d = c.P->disjs[c.P->disj_refs[cj.first + i]];
    bool multi = d.n > 1;
    uint32_t mark = c.nrec;
    if (multi) rec_push(c, mk_rec(REC_DISJ_OPEN, 0));
    uint32_t dfails = 0;
    bool passed = false;
    for (uint32_t j = 0; j < d.n && !c.err; j++) {
      uint32_t st = eval_clause(c, c.P->clause_refs[d.first + j], frame);
      if (c.err) break;
      if (st == ST_PASS) { num_pass++; passed = true; break; }
      if (st == ST_FAIL) dfails++;
    }
    if (c.err) break;
    if (passed) { if (multi && !c.suppress) c.nrec = mark; continue; }
    if (dfails) num_fail++;
    if (multi) {
      if (dfails) rec_push(c, mk_rec(REC_DISJ_CLOSE, 0));
      else if (!c.suppress) c.nrec = mark;
    }
  }
  if (c.err) return ST_FAIL;
  if (num_fail) return ST_FAIL;
  if (num_pass) return ST_PASS;
  return ST_SKIP;
}

// eval_rule (eval.rs:1837-1906).  frame: 0 = root frame
DEVN uint32_t eval_rule(Ctx& c, uint32_t rid, uint32_t frame, uint32_t custom_msg) {
  PRule R = c.P->rules[rid];
  uint32_t mark = c.nrec;
  Rec open = mk_rec(REC_RULE_OPEN, rid); open.x = custom_msg;
  rec_push(c, open);
  if (R.cond != NONE) {
    c.suppress++;
    uint32_t cond = eval_conj(c, R.cond, frame);
    c.suppress--;
    if (c.err) return ST_FAIL;
    if (cond != ST_PASS) { if (!c.suppress) c.nrec = mark; return ST_SKIP; }
  }
  uint32_t st = eval_block(c, R.block, frame);
  if (c.err) return ST_FAIL;
  if (st == ST_FAIL) rec_push(c, mk_rec(REC_RULE_CLOSE, rid));
  else if (!c.suppress) c.nrec = mark;
  return st;
}

// ------------------------------------------------------------------ kernel ---
__global__ void __launch_bounds__(64) guard_eval_kernel(LaunchArgs A) {
  const uint32_t lane = __lane_id();
  uint8_t* heap = A.heaps + (size_t)blockIdx.x * A.heap_bytes;
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(A.tile_cursor, 1u);
    t = __shfl(t, 0);
    if (t >= A.ntiles) break;
    uint32_t tile = A.tile_base + t;
    uint32_t doc = tile / A.nfiles, file = tile % A.nfiles;
    const DevProg* P = &A.progs[file];
    Ctx c;
    c.P = P; c.dn = A.docs.nodes; c.db = A.docs.bytes; c.heap = heap; c.cap = A.heap_bytes;
    c.tmp = FRAMES_BYTES + RECS_BYTES; c.pers = A.heap_bytes; c.nframes = 0; c.nrec = 0;
    c.err = 0; c.err_a = 0; c.err_b = 0; c.suppress = 0; c.rec_created = 0; c.depth = 0; c.nsyn = 0;
    c.syn_off = alloc_pers(c, 256 * 16);
    c.memo = alloc_pers(c, (P->n_slots ? P->n_slots : 1) * 4);
    if (!c.err) for (uint32_t i = 0; i < P->n_slots; i++) u32a(c, c.memo)[i] = 3u;
    uint32_t root = A.docs.roots[doc];
    uint32_t rf = push_frame(c, F_ROOT, NONE, root, P->root_block);
    (void)rf;
    uint32_t fails = 0, passes = 0;
    uint8_t* rs = A.rule_status + (size_t)tile * A.max_top;
    for (uint32_t r = 0; r < P->n_top && !c.err; r++) {
      uint32_t st = eval_rule(c, P->top_first + r, 0, NONE);
      if (c.err) break;
      if (lane == 0) rs[r] = (uint8_t)st;
      if (st == ST_PASS) passes++; else if (st == ST_FAIL) fails++;
    }
    uint32_t status = fails ? ST_FAIL : (passes ? ST_PASS : ST_SKIP);
    // publish records
    uint32_t off = 0;
    uint32_t n = c.err ? 0 : c.nrec;
    if (lane == 0 && n) off = atomicAdd(A.rec_cursor, n);
    off = __shfl(off, 0);
    if (n && off + n > A.rec_cap) { c.err = E_RECORDS; n = 0; }
    const Rec* src = (const Rec*)(heap + FRAMES_BYTES);
    for (uint32_t i = lane; i < n; i += 64) A.recs[off + i] = src[i];
    if (lane == 0) {
      TileOut o;
      o.status = status; o.err = c.err; o.err_a = c.err_a; o.err_b = c.err_b;
      o.rec_off = off; o.rec_n = n; o.pad0 = 0; o.pad1 = 0;
      A.tiles[tile] = o;
    }
  }
}

}  // namespace gg

namespace gg {

// Per-(rules file, top rule) PASS/FAIL/SKIP tallies over every tile of one evaluation, plus a
// per-file line (index max_top) holding file statuses and errored tiles (status slot 3).
// counts[((file * (max_top + 1) + rule) * 4) + status]; the same buffer is what the multi-GPU
// path all-reduces over RCCL.  LDS-privatised so global atomics are per block.
__global__ void __launch_bounds__(256) rule_count_kernel(const TileOut* tiles, const uint8_t* rule_status,
                                                          const DevProg* progs, uint32_t nfiles, uint32_t ntiles,
                                                          uint32_t max_top, unsigned long long* counts) {
  extern __shared__ uint32_t lds_counts[];
  const uint32_t ncount = nfiles * (max_top + 1) * 4;
  for (uint32_t i = threadIdx.x; i < ncount; i += blockDim.x) lds_counts[i] = 0;
  __syncthreads();
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x) {
    uint32_t file = t % nfiles;
    TileOut o = tiles[t];
    uint32_t base = file * (max_top + 1) * 4;
    if (o.err) { atomicAdd(&lds_counts[base + max_top * 4 + 3], 1u); continue; }
    atomicAdd(&lds_counts[base + max_top * 4 + o.status], 1u);
    uint32_t ntop = progs[file].n_top;
    const uint8_t* rs = rule_status + (size_t)t * max_top;
    for (uint32_t r = 0; r < ntop; r++) atomicAdd(&lds_counts[base + r * 4 + rs[r]], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ncount; i += blockDim.x)
    if (lds_counts[i]) atomicAdd(&counts[i], (unsigned long long)lds_counts[i]);
}

}  // namespace gg
