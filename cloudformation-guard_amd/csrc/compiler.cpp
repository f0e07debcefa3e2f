// Rules AST -> flat device program (see program.h).
#include <cstring>
#include <functional>
#include <map>

#include "host_format.h"
#include "program.h"

namespace gg {

namespace {

const char* OPS[] = {"Eq", "In", "Gt", "Lt", "Le", "Ge", "Exists", "Empty", "IsString", "IsList", "IsMap", "IsBool",
                     "IsInt", "IsFloat", "IsNull"};

uint32_t op_id(const std::string& op) {
  for (uint32_t i = 0; i < 15; i++) if (op == OPS[i]) return i;
  return 0;
}

bool parse_i32(const std::string& s, int32_t& v) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
  if (i >= s.size()) return false;
  int64_t x = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    x = x * 10 + (s[i] - '0');
    if (x > (int64_t)1 << 32) return false;
  }
  if (neg) x = -x;
  if (x < INT32_MIN || x > INT32_MAX) return false;
  v = (int32_t)x;
  return true;
}

struct Compiler {
  Program& P;
  std::vector<PPart> parts;
  std::vector<PQuery> queries;
  std::vector<PClause> clauses;
  std::vector<PRange2> conjs, disjs;
  std::vector<uint32_t> disj_refs, clause_refs;
  std::vector<PBlock> blocks;
  std::vector<PLet> lets;
  std::vector<PRule> rules;
  std::vector<PRange2> name_rules;
  std::vector<uint32_t> name_rule_ids;
  std::vector<PFunc> funcs;
  std::vector<PParamRule> params;
  std::vector<uint32_t> param_vars;
  std::vector<uint32_t> alts;
  std::vector<PRegex> regexes;
  std::vector<uint16_t> dfa;
  std::map<std::string, uint32_t> var_ids, slot_ids, str_ids, regex_ids, param_ids;
  std::string err;

  explicit Compiler(Program& p) : P(p) {}

  uint32_t ctx(const std::string& s) { P.ctx.push_back(s); return (uint32_t)P.ctx.size() - 1; }
  uint32_t msg(bool has, const std::string& s) { if (!has) return NONE; P.msgs.push_back(s); return (uint32_t)P.msgs.size() - 1; }

  uint32_t var(const std::string& name) {
    auto it = var_ids.find(name);
    if (it != var_ids.end()) return it->second;
    uint32_t id = (uint32_t)P.var_names.size();
    P.var_names.push_back(name);
    var_ids[name] = id;
    return id;
  }

  uint32_t pstr(const std::string& s) {
    auto it = str_ids.find(s);
    if (it != str_ids.end()) return it->second;
    PStr ps;
    ps.off = lit_str(s); ps.len = (uint32_t)s.size(); ps.hash = fnv1a(s.data(), s.size()); ps.pad = 0;
    P.strs.push_back(ps);
    uint32_t id = (uint32_t)P.strs.size() - 1;
    str_ids[s] = id;
    return id;
  }

  uint32_t regex(const std::string& src) {
    auto it = regex_ids.find(src);
    if (it != regex_ids.end()) return it->second;
    CompiledRegex cr = compile_regex(src);
    if (!cr.valid) { err = "Could not parse regular expression: " + src + " (" + cr.why + ")"; }
    PRegex pr{};
    pr.nstates = cr.nstates;
    pr.start = cr.start;
    pr.ncls = cr.ncls;
    pr.flags = (cr.unsupported ? 1u : 0u) | (cr.nfa ? 2u : 0u) | ((uint32_t)cr.bounds.size() << 8);
    if (cr.nfa) {   // the NFA simulation's u32 tables (regex_dfa.h kNfa*), 4-B aligned in the u16 section
      while (dfa.size() & 1) dfa.push_back(0);
      pr.table = (uint32_t)dfa.size();
      for (uint32_t w : cr.nfa_tab) { dfa.push_back((uint16_t)(w & 0xFFFFu)); dfa.push_back((uint16_t)(w >> 16)); }
      regexes.push_back(pr);
      P.regex.push_back(cr);
      P.regex_src.push_back(src);
      const uint32_t id = (uint32_t)regexes.size() - 1;
      regex_ids[src] = id;
      return id;
    }
    pr.table = (uint32_t)dfa.size();
    for (uint16_t t : cr.table) dfa.push_back(t);
    pr.accept = (uint32_t)dfa.size();
    for (uint8_t a : cr.accept) dfa.push_back(a);
    while (dfa.size() & 1) dfa.push_back(0);
    pr.ascii = (uint32_t)dfa.size();
    for (int k = 0; k < 128; k += 2) dfa.push_back((uint16_t)(cr.ascii[k] | (cr.ascii[k + 1] << 8)));
    pr.bounds = (uint32_t)dfa.size();
    for (auto& b : cr.bounds) {
      const uint32_t w = (b.first << 8) | b.second;
      dfa.push_back((uint16_t)(w & 0xFFFFu));
      dfa.push_back((uint16_t)(w >> 16));
    }
    regexes.push_back(pr);
    P.regex.push_back(cr);
    P.regex_src.push_back(src);
    uint32_t id = (uint32_t)regexes.size() - 1;
    regex_ids[src] = id;
    return id;
  }

  // ---- literal arena ---------------------------------------------------------
  // literal pool strings: 16-byte aligned, zero-padded to 16 bytes (the device compares in chunks)
  uint32_t lit_str(const std::string& v) {
    std::string& B = P.lit.bytes;
    B.append((16 - (B.size() & 15)) & 15, '\0');
    uint32_t off = (uint32_t)B.size();
    B += v;
    B.append((16 - (v.size() & 15)) & 15, '\0');
    return off;
  }
  void lit_fill(const LitValue& v, uint32_t slot, uint32_t parent) {
    DocBatch& L = P.lit;
    DNode& d = L.nodes[slot];
    d.parent = parent; d.count = 0; d.a = 0; d.b = 0;
    L.line[slot] = 0; L.col[slot] = 0;
    switch (v.k) {
      case LitValue::Null: d.kind = K_NULL; break;
      case LitValue::String: {
        d.kind = K_STRING; d.count = (uint32_t)v.s.size(); d.b = fnv1a(v.s.data(), v.s.size());
        d.a = lit_str(v.s); break;
      }
      case LitValue::Regex: {
        uint32_t rid = regex(v.s);
        DNode& dd = L.nodes[slot];
        uint32_t off = lit_str(v.s);
        DNode& dr = L.nodes[slot];
        dr.kind = K_REGEX; dr.a = off; dr.count = (uint32_t)v.s.size(); dr.b = rid;
        break;
      }
      case LitValue::Bool: d.kind = K_BOOL; d.a = v.b ? 1 : 0; break;
      case LitValue::Int: { d.kind = K_INT; uint64_t u = (uint64_t)v.i; d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32); break; }
      case LitValue::Float: { d.kind = K_FLOAT; uint64_t u; memcpy(&u, &v.f, 8); d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32); break; }
      case LitValue::Char: d.kind = K_CHAR; d.a = v.ch; break;
      case LitValue::RangeInt: case LitValue::RangeFloat: case LitValue::RangeChar: {
        DRange r{};
        r.incl = v.incl;
        if (v.k == LitValue::RangeInt) { r.kind = K_RANGE_INT; r.lo = (uint64_t)v.ilo; r.hi = (uint64_t)v.ihi; }
        else if (v.k == LitValue::RangeFloat) { r.kind = K_RANGE_FLOAT; memcpy(&r.lo, &v.flo, 8); memcpy(&r.hi, &v.fhi, 8); }
        else { r.kind = K_RANGE_CHAR; r.lo = v.clo; r.hi = v.chi; }
        d.kind = r.kind; d.a = (uint32_t)P.ranges.size();
        P.ranges.push_back(r);
        break;
      }
      case LitValue::List: {
        d.kind = K_LIST;
        uint32_t n = (uint32_t)v.items.size();
        uint32_t first = lit_grow(n);
        L.nodes[slot].a = first; L.nodes[slot].count = n;
        for (uint32_t j = 0; j < n; j++) {
          L.nodes[first + j].key_off = NONE; L.nodes[first + j].key_len = 0; L.nodes[first + j].key_hash = 0;
          lit_fill(v.items[j], first + j, slot);
        }
        break;
      }
      case LitValue::Map: {
        d.kind = K_MAP;
        uint32_t n = (uint32_t)v.kv.size();
        uint32_t first = lit_grow(n);
        L.nodes[slot].a = first; L.nodes[slot].count = n;
        for (uint32_t j = 0; j < n; j++) {
          const std::string& k = v.kv[j].first;
          uint32_t koff = lit_str(k);
          DNode& c = L.nodes[first + j];
          c.key_off = koff; c.key_len = (uint32_t)k.size(); c.key_hash = fnv1a(k.data(), k.size());
          lit_fill(v.kv[j].second, first + j, slot);
        }
        break;
      }
    }
  }
  uint32_t lit_grow(uint32_t n) {
    DocBatch& L = P.lit;
    uint32_t first = (uint32_t)L.nodes.size();
    L.grow_zeroed(L.nodes.size() + n);
    return first;
  }
  uint32_t literal(const LitValue& v) {
    uint32_t slot = lit_grow(1);
    P.lit.nodes[slot].key_off = NONE; P.lit.nodes[slot].key_len = 0; P.lit.nodes[slot].key_hash = 0;
    lit_fill(v, slot, NONE);
    P.lit.roots.push_back(slot);
    P.lit.names.push_back("");
    return slot | LIT_BIT;
  }

  // ---- queries -----------------------------------------------------------------
  // A filter whose conjunctions are the single clause `<key> == '<string literal>'` (the
  // desugared type block `Resources.*[ Type == 'AWS::S3::Bucket' ]` and most `let x =
  // Resources.*[ Type == ... ]`) is marked so the device can test a value with one map lookup
  // and one string compare (PPart.c = clause id + 1); values the shortcut cannot decide exactly
  // (lists, missing keys that need case conversion, non-map values) take the generic path.
  //
  // A filter whose FIRST conjunction is that clause and whose other conjunctions can never raise
  // an error (error_free_clause) is marked as well, with bit 31 set: when the shortcut says the
  // first clause FAILs, the conjunction is FAIL whatever the rest yields -- the reference still
  // evaluates the rest (conjunctions do not short-circuit, eval.rs:1970-2065), but inside a filter
  // its records are discarded and it cannot raise, so skipping it changes nothing observable.
  bool lit_has_regex(uint32_t ref) const {
    const DNode& n = P.lit.nodes[ref & ~LIT_BIT];
    if (n.kind == K_REGEX) return true;
    if (n.kind == K_LIST || n.kind == K_MAP)
      for (uint32_t j = 0; j < n.count; j++) if (lit_has_regex(n.a + j)) return true;
    return false;
  }
  // A literal whose regexes (if any) all compile to DFAs: comparing against it cannot raise.
  bool lit_dfa_only(uint32_t ref) const {
    const DNode& n = P.lit.nodes[ref & ~LIT_BIT];
    if (n.kind == K_REGEX) return n.b < P.regex.size() && !P.regex[n.b].unsupported;
    if (n.kind == K_LIST || n.kind == K_MAP)
      for (uint32_t j = 0; j < n.count; j++) if (!lit_dfa_only(n.a + j)) return false;
    return true;
  }
  // `%v` whose resolution cannot raise:
  //  * in block `blk` (a let query's own block): v is one of blk's lets -- the lazy evaluation of a
  //    block let runs in that block's scope (BlockScope::resolve_variable, eval_context.rs:1564-1590),
  //    and filters and value scopes in between define no variables -- and that let cannot raise;
  //  * otherwise: v is defined by root-block lets only (no block let or rule parameter anywhere shares
  //    the name, so every scope chain reaches the root's), every one a literal or a query that cannot
  //    raise.  A capture-only name does not qualify (MissingVariable when nothing was captured).
  bool let_error_free(const PLet& l, uint32_t blk, int depth) const {
    if (l.kind == L_FUNC) return false;
    if (l.kind == L_LITERAL) return lit_dfa_only(l.id);
    return error_free_query(l.id, depth, blk);
  }
  bool safe_var(uint32_t var, uint32_t blk, int depth) const {
    if (blk != NONE) {
      bool found = false;
      for (uint32_t i = 0; i < blocks[blk].nlets; i++) {
        const PLet& l = lets[blocks[blk].first_let + i];
        if (l.var != var) continue;
        if (!let_error_free(l, blk, depth)) return false;
        found = true;
      }
      if (found) return true;
    }
    bool defined = false;
    for (size_t b = 0; b < blocks.size(); b++)
      for (uint32_t i = 0; i < blocks[b].nlets; i++) {
        const PLet& l = lets[blocks[b].first_let + i];
        if (l.var != var) continue;
        if (b != P.hdr.root_block) return false;
        if (!let_error_free(l, P.hdr.root_block, depth)) return false;
        defined = true;
      }
    for (uint32_t v : param_vars) if (v == var) return false;
    return defined;
  }
  // a query of navigation steps, variable heads (safe_var) and filters that cannot raise (no `%var`
  // key interpolation, no named capture -- captures change the root scope); `blk`: the block whose
  // scope evaluates it (a let query), or NONE
  bool error_free_query(uint32_t qid, int depth, uint32_t blk = NONE) const {
    if (depth > 16) return false;
    const PQuery& q = queries[qid];
    for (uint32_t i = 0; i < q.n; i++) {
      const PPart& pp = parts[q.first + i];
      bool ok = pp.kind == P_THIS || pp.kind == P_KEY || pp.kind == P_KEY_INDEX || pp.kind == P_INDEX ||
                ((pp.kind == P_ALL_VALUES || pp.kind == P_ALL_INDICES) && pp.a == NONE);
      if (!ok && i == 0 && pp.kind == P_VAR_HEAD) ok = safe_var(pp.a, blk, depth + 1);
      if (!ok && pp.kind == P_FILTER && pp.b == NONE) ok = error_free_conj(pp.a, depth + 1, blk);
      if (!ok) return false;
    }
    return true;
  }
  bool error_free_conj(uint32_t cj, int depth, uint32_t blk = NONE) const {
    if (depth > 16) return false;
    const PRange2 C = conjs[cj];
    for (uint32_t i = 0; i < C.n; i++) {
      const PRange2 Di = disjs[disj_refs[C.first + i]];
      for (uint32_t j = 0; j < Di.n; j++) if (!error_free_clause(clause_refs[Di.first + j], depth, blk)) return false;
    }
    return true;
  }
  // access clause with no EMPTY (raises on scalars), whose operands are literals with DFA-compilable
  // regexes or queries that cannot raise: its evaluation can only produce statuses and records
  bool error_free_clause(uint32_t cid, int depth = 0, uint32_t blk = NONE) const {
    const PClause& pc = clauses[cid];
    if (pc.kind != C_ACCESS) return false;
    uint32_t op = pc.flags & 15u, rk = (pc.flags >> 8) & 15u;
    if (op == OP_EMPTY) return false;
    if (op < OP_EXISTS) {
      if (rk == RHS_LITERAL) { if (!(pc.b & LIT_BIT) || !lit_dfa_only(pc.b)) return false; }
      else if (rk == RHS_QUERY) { if (!error_free_query(pc.b, depth + 1, blk)) return false; }
      else return false;
    }
    return error_free_query(pc.a, depth + 1, blk);
  }
  uint32_t fast_filter_clause(uint32_t cj, uint32_t blk = NONE) {
    const PRange2 C = conjs[cj];
    if (C.n < 1) return 0;
    const PRange2 D = disjs[disj_refs[C.first]];
    if (D.n != 1) return 0;
    uint32_t cid = clause_refs[D.first];
    const PClause& pc = clauses[cid];
    if (pc.kind != C_ACCESS) return 0;
    uint32_t op = pc.flags & 15u, nt = (pc.flags >> 4) & 1u, neg = (pc.flags >> 5) & 1u, rk = (pc.flags >> 8) & 15u;
    if (op != OP_EQ || nt || neg || rk != RHS_LITERAL) return 0;
    const PQuery& q = queries[pc.a];
    if (q.n != 1 || parts[q.first].kind != P_KEY) return 0;
    if (!(pc.b & LIT_BIT)) return 0;
    // `<key> == '<string>'`, or `<key> == /<regex>/` with a DFA-compilable regex (the device runs the
    // DFA over the value instead of the generic filter path; an unsupported regex must raise when it
    // is reached, so it stays on the generic path)
    const DNode& lit = P.lit.nodes[pc.b & ~LIT_BIT];
    if (lit.kind != K_STRING && !(lit.kind == K_REGEX && lit.b < P.regex.size() && !P.regex[lit.b].unsupported)) return 0;
    if (C.n == 1) return cid + 1;
    for (uint32_t i = 1; i < C.n; i++) {
      const PRange2 Di = disjs[disj_refs[C.first + i]];
      for (uint32_t j = 0; j < Di.n; j++) if (!error_free_clause(clause_refs[Di.first + j], 0, blk)) return 0;
    }
    return (cid + 1) | 0x80000000u;
  }

  // A filter conjunction that reads only the value it tests: access clauses over navigation steps (keys,
  // indices, unnamed `*` / `[*]`, nested filters of the same kind) against literals or such queries -- no
  // `%var` (lets are evaluated lazily and cached), rule references, functions, captures or map-key filters.
  // Its evaluation for one value has no effect beyond its status (records are suppressed inside filters) and
  // a possible error, so the lanes of a document's group may test a list's values at once (PPart.c bit 30,
  // eval_recursive.inc coop_chunk).
  bool coop_query(uint32_t qid, int depth) const {
    if (depth > 16) return false;
    const PQuery& q = queries[qid];
    for (uint32_t i = 0; i < q.n; i++) {
      const PPart& pp = parts[q.first + i];
      const bool nav = pp.kind == P_THIS || pp.kind == P_KEY || pp.kind == P_KEY_INDEX || pp.kind == P_INDEX ||
                       ((pp.kind == P_ALL_VALUES || pp.kind == P_ALL_INDICES) && pp.a == NONE);
      if (nav) continue;
      if (pp.kind == P_FILTER && pp.b == NONE && coop_conj(pp.a, depth + 1)) continue;
      return false;
    }
    return true;
  }
  bool coop_conj(uint32_t cj, int depth) const {
    if (depth > 16) return false;
    const PRange2 C = conjs[cj];
    for (uint32_t i = 0; i < C.n; i++) {
      const PRange2 Di = disjs[disj_refs[C.first + i]];
      for (uint32_t j = 0; j < Di.n; j++) {
        const PClause& pc = clauses[clause_refs[Di.first + j]];
        if (pc.kind != C_ACCESS) return false;
        const uint32_t op = pc.flags & 15u, rk = (pc.flags >> 8) & 15u;
        if (op < OP_EXISTS) {
          if (rk == RHS_QUERY) { if (!coop_query(pc.b, depth + 1)) return false; }
          else if (rk != RHS_LITERAL) return false;
        }
        if (!coop_query(pc.a, depth + 1)) return false;
      }
    }
    return true;
  }

  // A filter conjunction the device tests for one value without the evaluator (PPart.c bit 29, eval_core.inc
  // quick_conj): every clause an access clause that cannot raise (error_free_clause), over a path of plain keys
  // optionally ending in an unnamed `[*]` / `*`, compared with one literal or checked by a unary operator.
  // Records are suppressed inside filters, so its status is all the test needs.
  bool quick_conj(uint32_t cj) const {
    const PRange2 C = conjs[cj];
    if (C.n < 1) return false;
    for (uint32_t i = 0; i < C.n; i++) {
      const PRange2 Di = disjs[disj_refs[C.first + i]];
      for (uint32_t j = 0; j < Di.n; j++) {
        const uint32_t cid = clause_refs[Di.first + j];
        const PClause& pc = clauses[cid];
        if (pc.kind != C_ACCESS || !error_free_clause(cid)) return false;
        const uint32_t op = pc.flags & 15u, rk = (pc.flags >> 8) & 15u;
        if (op < OP_EXISTS && rk != RHS_LITERAL) return false;
        const PQuery& q = queries[pc.a];
        if (q.n < 1) return false;
        for (uint32_t k = 0; k < q.n; k++) {
          const PPart& pp = parts[q.first + k];
          if (pp.kind == P_THIS || pp.kind == P_KEY) continue;
          if ((pp.kind == P_ALL_VALUES || pp.kind == P_ALL_INDICES) && pp.a == NONE && k + 1 == q.n) continue;
          return false;
        }
      }
    }
    return true;
  }

  uint32_t query(const AccessQuery& q) {
    uint32_t qid = (uint32_t)queries.size();
    queries.push_back(PQuery{0, 0, q.match_all ? 1u : 0u, 0});
    P.queries.push_back(q.parts);
    std::vector<PPart> local;
    for (size_t i = 0; i < q.parts.size(); i++) {
      const QueryPart& qp = q.parts[i];
      PPart pp{0, 0, 0, 0};
      switch (qp.k) {
        case QueryPart::This: pp.kind = P_THIS; break;
        case QueryPart::Key: {
          if (!qp.key.empty() && qp.key[0] == '%') {
            pp.kind = i == 0 ? P_VAR_HEAD : P_KEY_VAR;
            pp.a = var(qp.key.substr(1));
            break;
          }
          int32_t iv;
          if (parse_i32(qp.key, iv)) { pp.kind = P_KEY_INDEX; pp.a = (uint32_t)iv; break; }
          pp.kind = P_KEY;
          pp.a = pstr(qp.key);
          std::string alt[7];
          key_alternates(qp.key, alt);
          pp.b = (uint32_t)alts.size();
          for (int k = 0; k < 7; k++) alts.push_back(pstr(alt[k]));
          break;
        }
        case QueryPart::Index: pp.kind = P_INDEX; pp.a = (uint32_t)qp.index; break;
        case QueryPart::AllValues: pp.kind = P_ALL_VALUES; pp.a = qp.has_name ? var(qp.key) : NONE; break;
        case QueryPart::AllIndices: pp.kind = P_ALL_INDICES; pp.a = qp.has_name ? var(qp.key) : NONE; break;
        case QueryPart::Filter:
          pp.kind = P_FILTER; pp.a = conj(*qp.filter); pp.b = qp.has_name ? var(qp.key) : NONE;
          pp.c = 0;   // fast_filter_clause, once the whole file is compiled (assemble: lets seen)
          break;
        case QueryPart::MapKeyFilter: {
          // MapKeyFilterClause (exprs.rs:183-187): rhs literal | query (rooted at the map) | function
          pp.kind = P_MAP_KEY_FILTER;
          const LetValue& w = *qp.mk_with;
          if (w.k == LetValue::Value) { pp.a = RHS_LITERAL; pp.b = literal(w.value); }
          else if (w.k == LetValue::Access) { pp.a = RHS_QUERY; pp.b = query(w.access); }
          else { pp.a = RHS_FUNC; pp.b = func(*w.func); }
          pp.c = op_id(qp.mk_op) | (qp.mk_not ? 1u << 4 : 0) | (qp.has_name ? 1u << 8 : 0);
          break;
        }
      }
      local.push_back(pp);
    }
    // PPart.b of a `%var` head or a `*` / `[*]` step: 1 when a later step reads the scope a value
    // frame would give each fanned-out value (a filter, a map-key filter or a `%var` key); the walker
    // pushes value frames only then (eval_core.inc walk_run)
    for (size_t i = 0; i < local.size(); i++) {
      PPart& pp = local[i];
      if (pp.kind != P_VAR_HEAD && pp.kind != P_ALL_VALUES && pp.kind != P_ALL_INDICES) continue;
      pp.b = 0;
      for (size_t j = i + 1; j < local.size(); j++)
        if (local[j].kind == P_FILTER || local[j].kind == P_MAP_KEY_FILTER || local[j].kind == P_KEY_VAR) pp.b = 1;
    }
    queries[qid].first = (uint32_t)parts.size();
    queries[qid].n = (uint32_t)local.size();
    for (auto& pp : local) parts.push_back(pp);
    return qid;
  }

  uint32_t func(const FuncExpr& f) {
    PFunc pf{};
    pf.fname = f.name == "count" ? F_COUNT : F_OTHER;
    std::vector<PLet> args;
    for (auto& a : f.params) args.push_back(let_value(NONE, a));
    pf.first_arg = (uint32_t)lets.size();
    pf.nargs = (uint32_t)args.size();
    for (auto& a : args) lets.push_back(a);
    funcs.push_back(pf);
    if (pf.fname == F_OTHER) P.unsupported.push_back("function " + f.name + "() is outside the MI355X path");
    return (uint32_t)funcs.size() - 1;
  }

  PLet let_value(uint32_t var_id, const LetValue& lv) {
    PLet l{var_id, 0, 0, 0};
    if (lv.k == LetValue::Value) { l.kind = L_LITERAL; l.id = literal(lv.value); }
    else if (lv.k == LetValue::Access) { l.kind = L_QUERY; l.id = query(lv.access); }
    else { l.kind = L_FUNC; l.id = func(*lv.func); }
    return l;
  }

  uint32_t block(const Block& b, bool rule_level) {
    std::vector<PLet> ls;
    for (auto& a : b.assignments) ls.push_back(let_value(var(a.var), a.value));
    uint32_t c = conj(b.conjunctions);
    PBlock pb{(uint32_t)lets.size(), (uint32_t)ls.size(), c, rule_level ? 1u : 0u};
    for (auto& l : ls) lets.push_back(l);
    blocks.push_back(pb);
    return (uint32_t)blocks.size() - 1;
  }

  uint32_t conj(const Conj& cj) {
    std::vector<uint32_t> dids;
    for (auto& d : cj) {
      std::vector<uint32_t> cids;
      for (auto& c : d) cids.push_back(clause(*c));
      disjs.push_back(PRange2{(uint32_t)clause_refs.size(), (uint32_t)cids.size()});
      for (auto x : cids) clause_refs.push_back(x);
      dids.push_back((uint32_t)disjs.size() - 1);
    }
    conjs.push_back(PRange2{(uint32_t)disj_refs.size(), (uint32_t)dids.size()});
    for (auto x : dids) disj_refs.push_back(x);
    return (uint32_t)conjs.size() - 1;
  }

  uint32_t slot_of(const std::string& name) {
    auto it = slot_ids.find(name);
    return it == slot_ids.end() ? NONE : it->second;
  }

  uint32_t clause(const Clause& c) {
    PClause pc{};
    pc.d = NONE; pc.e = NONE; pc.f = NONE; pc.c = NONE;
    switch (c.k) {
      case Clause::Access: {
        pc.kind = C_ACCESS;
        pc.a = query(c.query);
        uint32_t op = op_id(c.op);
        uint32_t rk = RHS_NONE;
        if (c.has_rhs) {
          if (c.rhs.k == LetValue::Value) { rk = RHS_LITERAL; pc.b = literal(c.rhs.value); }
          else if (c.rhs.k == LetValue::Access) { rk = RHS_QUERY; pc.b = query(c.rhs.access); }
          else { rk = RHS_FUNC; pc.b = func(*c.rhs.func); }
        }
        bool empty_on_expr = false;
        if (!c.query.parts.empty()) {
          const QueryPart& last = c.query.parts.back();
          empty_on_expr = last.k == QueryPart::Filter || last.k == QueryPart::MapKeyFilter ||
                          (last.k == QueryPart::Key && !last.key.empty() && last.key[0] == '%' && c.query.parts.size() == 1);
        }
        pc.flags = op | (c.op_not ? 1u << 4 : 0) | (c.negation ? 1u << 5 : 0) | (rk << 8) | (empty_on_expr ? 1u << 12 : 0);
        pc.d = ctx(gac_display(c));
        pc.e = msg(c.has_msg, c.msg);
        break;
      }
      case Clause::NamedRule: {
        pc.kind = C_NAMED;
        pc.a = slot_of(c.rule);
        pc.flags = c.negation ? 1 : 0;
        pc.d = ctx("Rule(" + c.rule + "@" + file_location_display(c.loc) + ")");
        pc.e = msg(c.has_msg, c.msg);
        pc.f = ctx(c.rule);
        break;
      }
      case Clause::ParamRule: {
        pc.kind = C_PARAM;
        auto it = param_ids.find(c.rule);
        pc.a = it == param_ids.end() ? NONE : it->second;
        std::vector<PLet> args;
        for (auto& a : c.params) args.push_back(let_value(NONE, a));
        pc.b = (uint32_t)lets.size();
        pc.c = (uint32_t)args.size();
        for (auto& a : args) lets.push_back(a);
        pc.flags = c.negation ? 1 : 0;
        pc.d = ctx("Rule(" + c.rule + "@" + file_location_display(c.loc) + ")");
        pc.e = msg(c.has_msg, c.msg);
        pc.f = ctx(c.rule);
        break;
      }
      case Clause::BlockClause: {
        pc.kind = C_BLOCK;
        pc.a = query(c.query);
        pc.b = block(c.block, false);
        pc.flags = c.not_empty ? 1 : 0;
        pc.d = ctx("BlockGuardClause#" + file_location_display(c.loc));
        pc.f = ctx("GuardBlockAccessClause#" + file_location_display(c.loc));
        break;
      }
      case Clause::WhenBlock: {
        pc.kind = C_WHEN;
        pc.a = conj(c.conditions);
        pc.b = block(c.block, c.rule_level);
        pc.flags = c.rule_level ? 1 : 0;
        break;
      }
      case Clause::TypeBlockK: {
        pc.kind = C_TYPEBLOCK;
        pc.c = c.tb->has_conditions ? conj(c.tb->conditions) : NONE;
        pc.a = query(c.tb->query);
        pc.b = block(c.tb->block, false);
        pc.d = ctx("TypeBlock#" + c.tb->type_name);
        pc.f = ctx(c.tb->type_name);
        break;
      }
    }
    clauses.push_back(pc);
    return (uint32_t)clauses.size() - 1;
  }

  void run(const RulesFile& rf) {
    // name slots (rule_status lookup, eval_context.rs:926-978) -- built before clauses reference them
    for (auto& r : rf.rules) if (!slot_ids.count(r.name)) { slot_ids[r.name] = (uint32_t)P.slot_names.size(); P.slot_names.push_back(r.name); }
    for (auto& pr : rf.param_rules) {
      // HashMap::insert -- the last definition with a name wins
      uint32_t id;
      auto it = param_ids.find(pr.rule.name);
      if (it == param_ids.end()) { id = (uint32_t)P.param_rule_names.size(); param_ids[pr.rule.name] = id; P.param_rule_names.push_back(pr.rule.name); params.push_back({}); P.param_rule_nparams.push_back(0); }
      else id = it->second;
      (void)id;
    }
    // root lets
    {
      Block root;
      root.assignments = rf.assignments;
      P.hdr.root_block = block(root, true);
    }
    // parameterized rules (compiled as rules not in the top-level list)
    std::vector<uint32_t> param_rule_ids(params.size(), NONE);
    for (auto& pr : rf.param_rules) {
      uint32_t id = param_ids[pr.rule.name];
      PRule r{NONE, NONE, 0, 0};
      r.block = block(pr.rule.block, true);
      uint32_t rid = (uint32_t)rules.size();
      rules.push_back(r);
      P.rule_names.push_back(pr.rule.name);
      PParamRule ppr{rid, (uint32_t)param_vars.size(), (uint32_t)pr.params.size(), 0};
      for (auto& nm : pr.params) param_vars.push_back(var(nm));
      params[id] = ppr;
      P.param_rule_nparams[id] = (uint32_t)pr.params.size();
    }
    uint32_t first_top = (uint32_t)rules.size();
    std::vector<std::vector<uint32_t>> by_slot(P.slot_names.size());
    for (auto& r : rf.rules) {
      PRule pr{slot_ids[r.name], NONE, 0, 0};
      pr.cond = r.has_conditions ? conj(r.conditions) : NONE;
      pr.block = block(r.block, true);
      by_slot[pr.name_slot].push_back((uint32_t)rules.size());
      rules.push_back(pr);
      P.rule_names.push_back(r.name);
    }
    for (auto& v : by_slot) {
      name_rules.push_back(PRange2{(uint32_t)name_rule_ids.size(), (uint32_t)v.size()});
      for (auto x : v) name_rule_ids.push_back(x);
    }
    P.n_rules = (uint32_t)rf.rules.size();
    P.hdr.magic = 0x47554152;  // "GUAR"
    P.hdr.n_vars = (uint32_t)P.var_names.size();
    P.hdr.n_name_slots = (uint32_t)P.slot_names.size();
    uint32_t max_lets = 0;
    for (auto& b : blocks) max_lets = std::max(max_lets, b.nlets);
    P.hdr.max_lets = max_lets;
    // top-level rules are rules[first_top ..]; record via n_rules (first_top stored in pad of header? keep simple)
    P.hdr.n_rules = (uint32_t)rules.size();
    top_first = first_top;
  }
  uint32_t top_first = 0;

  template <class T, class A>
  void put(std::vector<uint32_t>& blob, uint32_t& off, uint32_t& n, const std::vector<T, A>& v) {
    while (blob.size() & 3) blob.push_back(0);   // 16-byte aligned sections
    off = (uint32_t)blob.size();
    n = (uint32_t)v.size();
    size_t words = (v.size() * sizeof(T) + 3) / 4;
    size_t at = blob.size();
    blob.resize(at + words);
    if (!v.empty()) memcpy(blob.data() + at, v.data(), v.size() * sizeof(T));
  }

  // `%var` heads whose variable can only come from the root scope's resolved variables (a root
  // query / function let or a key capture): no block let or rule parameter anywhere in the file
  // has the name, and no root literal let shadows it.  The walker reads those straight from the
  // root table (PPart.c = 1) instead of asking the scope chain.
  void mark_root_vars() {
    std::vector<uint8_t> scoped(P.var_names.size(), 0);
    const PBlock& rb = blocks[P.hdr.root_block];
    for (size_t b = 0; b < blocks.size(); b++) {
      for (uint32_t i = 0; i < blocks[b].nlets; i++) {
        const PLet& l = lets[blocks[b].first_let + i];
        if (b != P.hdr.root_block || l.kind == L_LITERAL) scoped[l.var] = 1;
      }
    }
    (void)rb;
    for (uint32_t v : param_vars) scoped[v] = 1;
    for (auto& pp : parts)
      if (pp.kind == P_VAR_HEAD) pp.c = scoped[pp.a] ? 0u : 1u;
  }

  void assemble() {
    // a let's query is evaluated in its block's scope: its filters may lean on that block's lets
    std::vector<uint32_t> query_block(queries.size(), NONE);
    for (size_t b = 0; b < blocks.size(); b++)
      for (uint32_t i = 0; i < blocks[b].nlets; i++) {
        const PLet& l = lets[blocks[b].first_let + i];
        if (l.kind == L_QUERY && l.id < queries.size()) query_block[l.id] = (uint32_t)b;
      }
    for (size_t q = 0; q < queries.size(); q++)
      for (uint32_t i = 0; i < queries[q].n; i++) {
        PPart& pp = parts[queries[q].first + i];
        if (pp.kind == P_FILTER) {
          pp.c = fast_filter_clause(pp.a, query_block[q]);
          if (pp.b == NONE && coop_conj(pp.a, 0)) pp.c |= 1u << 30;   // eval_core.inc COOP_FILTER
          if (pp.b == NONE && quick_conj(pp.a)) pp.c |= 1u << 29;     // eval_core.inc QUICK_FILTER
        }
      }
    // PQuery.pad = 1: a walk of the query does nothing but produce results -- no named `*` / `[*]` / filter
    // (captures into the root scope), no `%var` key, no map-key filter (its records join the clause's) -- so
    // the lanes of a document's group may split its first fan-out (eval_recursive.inc split_merge)
    for (size_t q = 0; q < queries.size(); q++) {
      bool ok = true;
      for (uint32_t i = 0; i < queries[q].n && ok; i++) {
        const PPart& pp = parts[queries[q].first + i];
        if ((pp.kind == P_ALL_VALUES || pp.kind == P_ALL_INDICES) && pp.a != NONE) ok = false;
        if (pp.kind == P_FILTER && pp.b != NONE) ok = false;
        if (pp.kind == P_KEY_VAR || pp.kind == P_MAP_KEY_FILTER) ok = false;
      }
      queries[q].pad = ok ? 1u : 0u;
    }
    // PClause.c = 1 on a block clause whose block (no lets of its own) is such a conjunction: the evaluation of
    // the block for one value reads only that value and produces only its records and status, so the lanes of a
    // document's group may evaluate the values at once and merge their records in value order
    // (eval_recursive.inc split_block)
    for (auto& pc : clauses)
      if (pc.kind == C_BLOCK && blocks[pc.b].nlets == 0 && coop_conj(blocks[pc.b].conj, 0)) pc.c = 1;
    mark_root_vars();
    std::vector<uint32_t> blob(sizeof(ProgHeader) / 4 + 2, 0);
    ProgHeader& h = P.hdr;
    put(blob, h.off_strs, h.n_strs, P.strs);
    put(blob, h.off_parts, h.n_parts, parts);
    put(blob, h.off_queries, h.n_queries, queries);
    put(blob, h.off_clauses, h.n_clauses, clauses);
    put(blob, h.off_conjs, h.n_conjs, conjs);
    put(blob, h.off_disjs, h.n_disjs, disjs);
    put(blob, h.off_clause_refs, h.n_clause_refs, clause_refs);
    put(blob, h.off_disj_refs, h.n_disj_refs, disj_refs);
    put(blob, h.off_blocks, h.n_blocks, blocks);
    put(blob, h.off_lets, h.n_lets, lets);
    put(blob, h.off_rules, h.n_rules, rules);
    put(blob, h.off_name_rules, h.n_name_rules, name_rules);
    put(blob, h.off_name_rule_ids, h.n_name_rule_ids, name_rule_ids);
    put(blob, h.off_funcs, h.n_funcs, funcs);
    put(blob, h.off_params, h.n_params, params);
    put(blob, h.off_param_vars, h.n_param_vars, param_vars);
    put(blob, h.off_alts, h.n_alts, alts);
    put(blob, h.off_regex, h.n_regex, regexes);
    put(blob, h.off_lit_nodes, h.n_lit_nodes, P.lit.nodes);
    put(blob, h.off_lit_ranges, h.n_lit_ranges, P.ranges);
    std::vector<char> bytes(P.lit.bytes.begin(), P.lit.bytes.end());
    put(blob, h.off_bytes, h.n_bytes, bytes);
    // regex DFA tables last: the kernels stage everything before them in LDS (eval_kernel.hip)
    put(blob, h.off_dfa, h.n_dfa, dfa);
    h.nwords = (uint32_t)blob.size();
    memcpy(blob.data(), &h, sizeof(ProgHeader));
    blob[sizeof(ProgHeader) / 4] = top_first;
    blob[sizeof(ProgHeader) / 4 + 1] = P.n_rules;
    P.blob = blob;
    P.clauses = clauses;
    P.pqueries = queries;
    P.parts = parts;
  }
};

}  // namespace

bool compile_program(const RulesFile& rf, const std::string& file_name, Program& out, std::string& err) {
  out = Program();
  out.file_name = file_name;
  Compiler c(out);
  c.run(rf);
  if (!c.err.empty()) { err = c.err; return false; }
  c.assemble();
  return true;
}

}  // namespace gg
