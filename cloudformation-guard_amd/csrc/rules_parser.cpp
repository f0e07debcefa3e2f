// Guard DSL parser -- a PEG over the same grammar as the reference's nom 7 combinators
// (guard/src/rules/parser.rs; each method names the combinator it restates).
// `Err` = nom::Err::Error (recoverable), `Fail` = nom::Err::Failure (cut).  Both carry nom 7's
// ParserError payload -- the input position the failing combinator saw and its context string --
// propagated the way nom 7.1.3 propagates them (alt: the last alternative's error; many1 /
// separated_list: the element's error; fold_many1: a fresh error at its own input; context(): its
// input position and "ctx/inner"; cut: Error -> Failure), so a rules file that does not parse
// reports the reference's "Error parsing file F at line L at column C, when handling CTX, fragment
// REST" (parser.rs:48-101).
#include <cstring>
#include <map>
#include <stdexcept>

#include "host_format.h"
#include "regex_dfa.h"
#include "rules_ast.h"

namespace gg {

namespace {

struct Err { size_t pos; std::string ctx; };
struct Fail { size_t pos; std::string ctx; };
[[noreturn]] void E(size_t p, const std::string& c = std::string()) { throw Err{p, c}; }
[[noreturn]] void F(size_t p, const std::string& c = std::string()) { throw Fail{p, c}; }
// nom's ContextError::add_context (parser.rs:48-62): the context's own input, "ctx" or "ctx/inner"
std::string add_ctx(const char* ctx, const std::string& inner) { return inner.empty() ? ctx : std::string(ctx) + "/" + inner; }
const char* const CTX_CMP = "expecting comparison binary operators like >, <= or unary operators KEYS, EXISTS, EMPTY or NOT";
const char* const CTX_RHS = "expecting either a property access \"engine.core\" or value like \"string\" or [\"this\", \"that\"]";

const std::vector<std::string> UNARY = {"Exists", "Empty", "IsString", "IsList", "IsMap", "IsBool", "IsInt", "IsFloat", "IsNull"};

bool is_unary(const std::string& op) {
  for (auto& u : UNARY) if (u == op) return true;
  return false;
}

const char* FUNCS[][2] = {{"count", "1"}, {"join", "2"}, {"json_parse", "1"}, {"now", "0"}, {"parse_boolean", "1"},
                          {"parse_char", "1"}, {"parse_epoch", "1"}, {"parse_float", "1"}, {"parse_int", "1"},
                          {"parse_string", "1"}, {"regex_replace", "3"}, {"substring", "3"}, {"to_lower", "1"},
                          {"to_upper", "1"}, {"url_decode", "1"}};

inline bool is_ascii_alpha(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
inline bool is_alnum_u(unsigned char c) { return isalnum(c) || c >= 0x80; }

struct P {
  const std::string& s;
  size_t n;
  std::string file;
  explicit P(const std::string& s_, const std::string& f) : s(s_), n(s_.size()), file(f) {}

  FileLoc loc(size_t p) const {
    FileLoc l;
    l.file = file;
    uint32_t line = 1;
    size_t start = 0;
    for (size_t i = 0; i < p; i++) if (s[i] == '\n') { line++; start = i + 1; }
    uint32_t col = 1;
    for (size_t i = start; i < p; i++) if (((unsigned char)s[i] & 0xC0) != 0x80) col++;
    l.line = line; l.column = col;
    return l;
  }

  mutable std::map<std::string, bool> rx_ok;   // fancy-regex validity per pattern (parses backtrack)
  bool regex_ok(const std::string& rx) const {
    auto it = rx_ok.find(rx);
    if (it != rx_ok.end()) return it->second;
    const bool ok = compile_regex(rx).valid;
    rx_ok[rx] = ok;
    return ok;
  }
  // nom_locate position of offset p: 1-based line, 1-based column counted in UTF-8 characters
  std::string error_text(size_t p, const std::string& ctx) const {
    FileLoc l = loc(p);
    return "Error parsing file " + file + " at line " + std::to_string(l.line) + " at column " + std::to_string(l.column) +
           ", when handling " + ctx + ", fragment " + s.substr(p);
  }

  bool starts(size_t p, const char* t) const { size_t m = strlen(t); return p + m <= n && s.compare(p, m, t) == 0; }
  size_t tag(size_t p, const char* t) const { if (starts(p, t)) return p + strlen(t); E(p); }
  size_t ch(size_t p, char c) const { if (p < n && s[p] == c) return p + 1; E(p); }
  static bool ms(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
  size_t multispace0(size_t p) const { while (p < n && ms(s[p])) p++; return p; }
  size_t space0(size_t p) const { while (p < n && (s[p] == ' ' || s[p] == '\t')) p++; return p; }
  size_t space1(size_t p) const { size_t q = space0(p); if (q == p) E(p); return q; }
  size_t digit1(size_t p) const { size_t q = p; while (q < n && s[q] >= '0' && s[q] <= '9') q++; if (q == p) E(p); return q; }
  size_t comment2(size_t p) const { p = ch(p, '#'); while (p < n && s[p] != '\n') p++; return multispace0(p); }
  size_t ws_or_comment(size_t p) const { size_t q = multispace0(p); if (q > p) return q; return comment2(p); }
  size_t ws0(size_t p) const {
    for (;;) { size_t q; try { q = ws_or_comment(p); } catch (Err&) { return p; } if (q == p) return p; p = q; }
  }
  size_t ws1(size_t p) const { return ws0(ws_or_comment(p)); }
  size_t white_space(size_t p, char c) const { return ch(ws0(p), c); }

  // ---- values -----------------------------------------------------------------
  size_t parse_int_value(size_t p, LitValue& v) const {
    try {
      size_t q = digit1(p);
      std::string d = s.substr(p, q - p);
      if (d.size() > 19 || (d.size() == 19 && d > "9223372036854775807")) E(p);
      v = LitValue(); v.k = LitValue::Int; v.i = std::stoll(d); return q;
    } catch (Err&) {}
    size_t q = tag(p, "-");
    size_t r = digit1(q);
    std::string d = s.substr(q, r - q);
    if (d.size() > 19 || (d.size() == 19 && d > "9223372036854775807")) E(p);
    v = LitValue(); v.k = LitValue::Int; v.i = -std::stoll(d); return r;
  }

  size_t parse_string_inner(size_t p, char q, std::string& out) const {
    p = ch(p, q);
    size_t span = p;
    out.clear();
    for (;;) {
      size_t e = span;
      while (e < n && s[e] != q) e++;
      std::string frag = s.substr(span, e - span);
      if (!frag.empty() && frag.back() == '\\') {
        out += frag.substr(0, frag.size() - 1);
        out.push_back(q);
        if (e >= n) E(p, "Could not parse string");
        span = e + 1;
        continue;
      }
      out += frag;
      if (e >= n) F(e);   // cut(char(q))
      return e + 1;
    }
  }
  size_t parse_string(size_t p, std::string& out) const {
    try { return parse_string_inner(p, '\'', out); } catch (Err&) {}
    return parse_string_inner(p, '"', out);
  }
  size_t parse_bool(size_t p, LitValue& v) const {
    const char* t[] = {"true", "True", "false", "False"};
    for (int i = 0; i < 4; i++) if (starts(p, t[i])) { v = LitValue(); v.k = LitValue::Bool; v.b = i < 2; return p + strlen(t[i]); }
    E(p);
  }
  size_t recognize_float(size_t p) const {
    size_t q = p;
    if (q < n && (s[q] == '+' || s[q] == '-')) q++;
    if (q < n && isdigit((unsigned char)s[q])) {
      q = digit1(q);
      if (q < n && s[q] == '.') { q++; while (q < n && isdigit((unsigned char)s[q])) q++; }
    } else if (q + 1 < n && s[q] == '.' && isdigit((unsigned char)s[q + 1])) {
      q = digit1(q + 1);
    } else E(p);
    if (q < n && (s[q] == 'e' || s[q] == 'E')) {
      size_t r = q + 1;
      if (r < n && (s[r] == '+' || s[r] == '-')) r++;
      try { r = digit1(r); } catch (Err& e) { F(e.pos, e.ctx); }   // nom recognize_float: cut(digit1)
      q = r;
    }
    return q;
  }
  size_t parse_float(size_t p, LitValue& v) const {
    size_t whole = digit1(p), q = whole;
    bool frac = false, expo = false;
    if (q < n && s[q] == '.') { try { q = digit1(q + 1); frac = true; } catch (Err&) { q = whole; } }
    if (q + 1 < n && (s[q] == 'e' || s[q] == 'E') && (s[q + 1] == '+' || s[q + 1] == '-')) {
      try { digit1(q + 2); expo = true; } catch (Err&) {}
    }
    if (frac || expo) {
      size_t r = recognize_float(p);
      v = LitValue(); v.k = LitValue::Float; v.f = strtod(s.substr(p, r - p).c_str(), nullptr);
      return r;
    }
    E(p, "Could not parse floating number");
  }
  size_t parse_regex(size_t p, LitValue& v) const {
    p = ch(p, '/');
    std::string rx;
    size_t span = p;
    for (;;) {
      size_t e = span;
      while (e < n && s[e] != '/') e++;
      if (e == span) E(span);   // is_not("/")
      std::string frag = s.substr(span, e - span);
      if (frag.back() == '\\') {
        rx += frag.substr(0, frag.size() - 1);
        rx.push_back('/');
        if (e >= n) E(p, "Could not parse regular expression");
        span = e + 1;
        continue;
      }
      rx += frag;
      // Regex::try_from (parser.rs:273-280): a pattern fancy-regex rejects fails the parse here.
      // The reference's context then quotes fancy-regex's error text; that text is not restated
      // (the alternatives around a regex literal always report a later alternative's error).
      if (!regex_ok(rx)) E(p, "Could not parse regular expression");
      size_t q = ch(e, '/');
      v = LitValue(); v.k = LitValue::Regex; v.s = rx;
      return q;
    }
  }
  size_t parse_char(size_t p, LitValue& v) const {
    if (p >= n) E(p);
    size_t i = p;
    uint32_t cp = utf8_next((const unsigned char*)s.data(), n, i);
    v = LitValue(); v.k = LitValue::Char; v.ch = cp;
    return i;
  }
  size_t range_value(size_t p, LitValue& v) const {
    p = space0(p);
    size_t q;
    try { q = parse_float(p, v); return space0(q); } catch (Err&) {}
    try { q = parse_int_value(p, v); return space0(q); } catch (Err&) {}
    q = parse_char(p, v);
    return space0(q);
  }
  size_t parse_range(size_t p, LitValue& v) const {
    p = ch(p, 'r');
    if (!(p < n && (s[p] == '(' || s[p] == '['))) E(p);
    char open = s[p++];
    LitValue a, b;
    p = range_value(p, a);
    p = ch(p, ',');
    p = range_value(p, b);
    if (!(p < n && (s[p] == ')' || s[p] == ']'))) E(p);
    char close = s[p++];
    uint8_t incl = (open == '[' ? 1 : 0) | (close == ']' ? 2 : 0);
    v = LitValue(); v.incl = incl;
    if (a.k == LitValue::Int && b.k == LitValue::Int) { v.k = LitValue::RangeInt; v.ilo = a.i; v.ihi = b.i; }
    else if (a.k == LitValue::Float && b.k == LitValue::Float) { v.k = LitValue::RangeFloat; v.flo = a.f; v.fhi = b.f; }
    else if (a.k == LitValue::Char && b.k == LitValue::Char) { v.k = LitValue::RangeChar; v.clo = a.ch; v.chi = b.ch; }
    else F(p, "Could not parse range");
    return p;
  }
  size_t parse_scalar_value(size_t p, LitValue& v) const {
    try { std::string str; size_t q = parse_string(p, str); v = LitValue(); v.k = LitValue::String; v.s = str; return q; } catch (Err&) {}
    try { return parse_float(p, v); } catch (Err&) {}
    try { return parse_int_value(p, v); } catch (Err&) {}
    try { return parse_bool(p, v); } catch (Err&) {}
    return parse_regex(p, v);
  }
  size_t parse_list(size_t p, LitValue& v) const {
    p = white_space(p, '[');
    LitValue out; out.k = LitValue::List;
    try {
      LitValue e; p = parse_value(p, e); out.items.push_back(e);
      for (;;) {
        size_t q;
        try { q = white_space(p, ','); } catch (Err&) { break; }
        LitValue e2;
        try { q = parse_value(q, e2); } catch (Err&) { break; }
        out.items.push_back(e2); p = q;
      }
    } catch (Err&) {}
    p = white_space(p, ']');
    v = out;
    return p;
  }
  size_t key_part(size_t p, std::string& k) const {
    size_t q = p;
    while (q < n && (is_alnum_u((unsigned char)s[q]) || s[q] == '-' || s[q] == '_')) q++;
    if (q > p) { k = s.substr(p, q - p); return q; }
    return parse_string(p, k);
  }
  size_t key_value(size_t p, std::string& k, LitValue& v) const {
    p = ws0(p);
    p = key_part(p, k);
    p = white_space(p, ':');
    return parse_value(p, v);
  }
  size_t parse_map(size_t p, LitValue& v) const {
    p = ch(p, '{');
    LitValue out; out.k = LitValue::Map;
    auto put = [&](const std::string& k, const LitValue& val) {
      for (auto& kv : out.kv) if (kv.first == k) { kv.second = val; return; }
      out.kv.push_back({k, val});
    };
    try {
      std::string k; LitValue e; p = key_value(p, k, e); put(k, e);
      for (;;) {
        size_t q;
        try { q = white_space(p, ','); } catch (Err&) { break; }
        std::string k2; LitValue e2;
        try { q = key_value(q, k2, e2); } catch (Err&) { break; }
        put(k2, e2); p = q;
      }
    } catch (Err&) {}
    p = white_space(p, '}');
    v = out;
    return p;
  }
  size_t parse_null(size_t p, LitValue& v) const {
    if (starts(p, "null") || starts(p, "NULL")) { v = LitValue(); v.k = LitValue::Null; return p + 4; }
    E(p);
  }
  size_t parse_value(size_t p, LitValue& v) const {
    p = ws0(p);
    try { return parse_null(p, v); } catch (Err&) {}
    try { return parse_scalar_value(p, v); } catch (Err&) {}
    try { return parse_range(p, v); } catch (Err&) {}
    try { return parse_list(p, v); } catch (Err&) {}
    return parse_map(p, v);
  }

  // ---- expressions --------------------------------------------------------------
  size_t var_name(size_t p, std::string& out) const {
    size_t q = p;
    while (q < n && is_ascii_alpha((unsigned char)s[q])) q++;
    if (q == p) E(p);
    while (q < n && (is_alnum_u((unsigned char)s[q]) || s[q] == '_')) q++;
    out = s.substr(p, q - p);
    return q;
  }
  size_t var_name_access_inclusive(size_t p, std::string& out) const {
    p = ch(p, '%');
    std::string nm;
    size_t q = var_name(p, nm);
    out = "%" + nm;
    return q;
  }
  size_t in_keyword(size_t p) const {
    if (starts(p, "in") || starts(p, "IN")) return p + 2;
    E(p);
  }
  size_t not_(size_t p) const {
    for (const char* t : {"not", "NOT"}) {
      if (starts(p, t)) { try { return space1(p + 3); } catch (Err&) {} }
    }
    return ch(p, '!');
  }
  size_t eq(size_t p, std::string& op, bool& neg) const {
    if (starts(p, "==")) { op = "Eq"; neg = false; return p + 2; }
    if (starts(p, "!=")) { op = "Eq"; neg = true; return p + 2; }
    E(p);
  }
  size_t other_operations(size_t p, std::string& op, bool& neg) const {
    neg = false;
    try { p = not_(p); neg = true; } catch (Err&) {}
    try { size_t q = in_keyword(p); op = "In"; return q; } catch (Err&) {}
    static const char* words[][2] = {{"EXISTS", "Exists"}, {"exists", "Exists"}, {"EMPTY", "Empty"}, {"empty", "Empty"},
                                     {"IS_STRING", "IsString"}, {"is_string", "IsString"}, {"IS_LIST", "IsList"},
                                     {"is_list", "IsList"}, {"IS_STRUCT", "IsMap"}, {"is_struct", "IsMap"},
                                     {"IS_BOOL", "IsBool"}, {"is_bool", "IsBool"}, {"IS_INT", "IsInt"}, {"is_int", "IsInt"},
                                     {"IS_NULL", "IsNull"}, {"is_null", "IsNull"}, {"IS_FLOAT", "IsFloat"},
                                     {"is_float", "IsFloat"}};
    for (auto& w : words) if (starts(p, w[0])) { op = w[1]; return p + strlen(w[0]); }
    E(p);
  }
  size_t value_cmp(size_t p, std::string& op, bool& neg) const {
    if (starts(p, "<<")) E(p, "Custom message tag detected");
    try { return eq(p, op, neg); } catch (Err&) {}
    static const char* cmps[][2] = {{">=", "Ge"}, {"<=", "Le"}, {">", "Gt"}, {"<", "Lt"}};
    for (auto& c : cmps) if (starts(p, c[0])) { op = c[1]; neg = false; return p + strlen(c[0]); }
    return other_operations(p, op, neg);
  }
  size_t custom_message(size_t p, std::string& msg) const {
    p = tag(p, "<<");
    size_t j = s.find(">>", p);
    if (j == std::string::npos) F(p, "Unable to find a closing >> tag for message");
    msg = s.substr(p, j - p);
    return j + 2;
  }
  size_t variable_capture(size_t p, std::string& var) const {
    p = ws0(p);
    p = var_name(p, var);
    p = space0(p);
    return ch(p, '|');
  }
  size_t open_array(size_t p) const { return white_space(p, '['); }
  size_t close_array(size_t p) const { return white_space(p, ']'); }

  size_t predicate_filter_clauses(size_t p, QueryPart& part) const {
    p = open_array(p);
    std::string var; bool has = false;
    try { p = variable_capture(p, var); has = true; } catch (Err&) {}
    auto conj = std::make_shared<Conj>();
    p = cnf_clauses(p, *conj, 0);
    try { p = close_array(p); } catch (Err& e) { F(e.pos, e.ctx); }
    part = QueryPart(); part.k = QueryPart::Filter; part.filter = conj; part.has_name = has; part.key = var;
    return p;
  }
  size_t dotted_property(size_t p, QueryPart& part) const {
    p = ws0(p);
    p = ch(p, '.');
    try { LitValue v; size_t q = parse_int_value(p, v); part = QueryPart(); part.k = QueryPart::Index; part.index = (int32_t)v.i; return q; } catch (Err&) {}
    try { std::string nm; size_t q = property_name(p, nm); part = QueryPart(); part.k = QueryPart::Key; part.key = nm; return q; } catch (Err&) {}
    try { std::string nm; size_t q = var_name_access_inclusive(p, nm); part = QueryPart(); part.k = QueryPart::Key; part.key = nm; return q; } catch (Err&) {}
    size_t q = ch(p, '*');
    part = QueryPart(); part.k = QueryPart::AllValues;
    return q;
  }
  size_t all_indices(size_t p, QueryPart& part) const {
    p = open_array(p);
    size_t q = ws0(p);
    part = QueryPart(); part.k = QueryPart::AllIndices;
    if (q < n && s[q] == '*') p = q + 1;
    else { std::string nm; p = var_name(p, nm); part.has_name = true; part.key = nm; }
    return close_array(p);
  }
  size_t array_index(size_t p, QueryPart& part) const {
    p = open_array(p);
    LitValue v; p = parse_int_value(p, v);
    try { p = close_array(p); } catch (Err& e) { F(e.pos, e.ctx); }
    part = QueryPart(); part.k = QueryPart::Index; part.index = (int32_t)v.i;
    return p;
  }
  size_t map_key_lookup(size_t p, QueryPart& part) const {
    p = open_array(p);
    size_t q;
    try {
      std::string str; q = parse_string(p, str);
      part = QueryPart(); part.k = QueryPart::Key; part.key = str;
    } catch (Err&) {
      q = ws0(p); std::string nm; q = var_name(q, nm); q = ws0(q);
      part = QueryPart(); part.k = QueryPart::AllValues; part.has_name = true; part.key = nm;
    }
    return close_array(q);
  }
  size_t map_keys_match(size_t p, QueryPart& part) const {
    p = open_array(p);
    std::string var; bool has = false;
    try { p = variable_capture(p, var); has = true; } catch (Err&) {}
    p = ws0(p);
    if (starts(p, "KEYS") || starts(p, "keys")) p += 4; else E(p);
    std::string op; bool neg = false;
    try {
      size_t q = ws0(p);
      try { p = eq(q, op, neg); }
      catch (Err&) {
        try { p = in_keyword(q); op = "In"; neg = false; }
        catch (Err&) { q = not_(q); p = in_keyword(q); op = "In"; neg = true; }
      }
    } catch (Err& e) { F(e.pos, e.ctx); }
    auto with = std::make_shared<LetValue>();
    try {
      size_t q = ws0(p);
      try { LitValue v; p = parse_value(q, v); with->k = LetValue::Value; with->value = v; }
      catch (Err&) { q = ws0(q); p = access(q, with->access); with->k = LetValue::Access; }
    } catch (Err& e) { F(e.pos, e.ctx); }
    p = close_array(p);
    part = QueryPart(); part.k = QueryPart::MapKeyFilter; part.has_name = has; part.key = var;
    part.mk_op = op; part.mk_not = neg; part.mk_with = with;
    return p;
  }
  size_t predicate_or_index(size_t p, QueryPart& part) const {
    try { return all_indices(p, part); } catch (Err&) {}
    try { return array_index(p, part); } catch (Err&) {}
    try { return map_key_lookup(p, part); } catch (Err&) {}
    try { return map_keys_match(p, part); } catch (Err&) {}
    return predicate_filter_clauses(p, part);
  }
  size_t one_dotted(size_t p, QueryPart& part) const {
    try { return dotted_property(p, part); } catch (Err&) {}
    return predicate_or_index(p, part);
  }
  size_t dotted_access(size_t p, std::vector<QueryPart>& out) const {
    QueryPart part;
    try { p = one_dotted(p, part); } catch (Err&) { E(p); }   // fold_many1: from_error_kind(input, Many1)
    out.push_back(part);
    for (;;) {
      QueryPart q2; size_t q;
      try { q = one_dotted(p, q2); } catch (Err&) { return p; }
      out.push_back(q2); p = q;
    }
  }
  size_t property_name(size_t p, std::string& out) const {
    try { return var_name(p, out); } catch (Err&) {}
    return parse_string(p, out);
  }
  size_t some_keyword(size_t p) const {
    p = ws0(p);
    if (starts(p, "SOME") || starts(p, "some")) return ws1(p + 4);
    E(p);
  }
  size_t this_keyword(size_t p) const {
    p = ws0(p);
    if (starts(p, "this") || starts(p, "THIS")) return p + 4;
    E(p);
  }
  size_t access(size_t p, AccessQuery& q) const {
    bool some = false;
    try { p = some_keyword(p); some = true; } catch (Err&) {}
    QueryPart first;
    try { p = this_keyword(p); first.k = QueryPart::This; }
    catch (Err&) {
      std::string nm;
      try { p = var_name_access_inclusive(p, nm); } catch (Err&) { p = property_name(p, nm); }
      first.k = QueryPart::Key; first.key = nm;
    }
    std::vector<QueryPart> parts;
    bool has_rest = false;
    try { p = dotted_access(p, parts); has_rest = true; } catch (Err&) {}
    q.parts.clear();
    q.parts.push_back(first);
    if (has_rest) {
      for (auto& x : parts) q.parts.push_back(x);
      if (first.k == QueryPart::Key && !first.key.empty() && first.key[0] == '%') {
        if (!(q.parts.size() > 1 && q.parts[1].k == QueryPart::AllIndices)) {
          QueryPart ai; ai.k = QueryPart::AllIndices;
          q.parts.insert(q.parts.begin() + 1, ai);
        }
      }
    }
    q.match_all = !some;
    return p;
  }

  size_t function_expr(size_t p, FuncExpr& f) const {
    f.loc = loc(p);
    std::vector<LetValue> params;
    std::string name;
    p = call_expr(p, name, params);
    int arity = -1;
    for (auto& fn : FUNCS) if (name == fn[0]) arity = atoi(fn[1]);
    // parser.rs:1082-1100 (errors at the input after the call; FunctionName Display = its name)
    if (arity < 0) E(p, "Parser Error when parsing `No function with the name '" + name + "' exists.`");
    if ((int)params.size() != arity)
      E(p, "function: " + name + " requires: " + std::to_string(arity) + " parameters to be passed, but received: " +
               std::to_string(params.size()));
    f.name = name; f.params = params;
    return p;
  }
  size_t let_value(size_t p, LetValue& lv) const {
    p = ws0(p);
    try { LitValue v; size_t q = parse_value(p, v); lv = LetValue(); lv.k = LetValue::Value; lv.value = v; return q; } catch (Err&) {}
    try {
      auto f = std::make_shared<FuncExpr>(); size_t q = function_expr(p, *f);
      lv = LetValue(); lv.k = LetValue::Func; lv.func = f; return q;
    } catch (Err&) {}
    lv = LetValue(); lv.k = LetValue::Access;
    return access(p, lv.access);
  }
  size_t call_expr(size_t p, std::string& name, std::vector<LetValue>& params) const {
    p = var_name(p, name);
    p = ch(p, '(');
    params.clear();
    auto elem = [&](size_t q, LetValue& lv) { q = multispace0(q); q = let_value(q, lv); return multispace0(q); };
    try {
      LetValue lv; p = elem(p, lv); params.push_back(lv);
      for (;;) {
        size_t q;
        try { q = ch(p, ','); } catch (Err&) { break; }
        LetValue lv2;
        try { q = elem(q, lv2); } catch (Err&) { break; }
        params.push_back(lv2); p = q;
      }
    } catch (Err&) {}
    return ch(p, ')');
  }

  size_t clause_with_map(size_t p, Clause& c) const {
    c = Clause(); c.k = Clause::Access; c.loc = loc(p);
    p = ws0(p);
    try { p = not_(p); c.negation = true; } catch (Err&) {}
    p = access(p, c.query);
    p = ws0(p);
    try { p = value_cmp(p, c.op, c.op_not); }
    catch (Err& e) { E(p, add_ctx(CTX_CMP, e.ctx)); }   // context(.., value_cmp), parser.rs:974
    if (is_unary(c.op)) {
      size_t q = ws0(p);
      try { p = custom_message(q, c.msg); c.has_msg = true; } catch (Err&) { p = q; }
      return p;
    }
    // context(.., cut(alt((value msg?, function msg?, access msg?)))), parser.rs:1000-1023
    const size_t at = p;
    try {
      auto msg = [&](size_t r) {
        size_t q = ws0(r);
        try { r = custom_message(q, c.msg); c.has_msg = true; } catch (Err&) { r = q; }
        return r;
      };
      bool done = false;
      try {
        LitValue v; size_t q = parse_value(p, v);
        c.rhs = LetValue(); c.rhs.k = LetValue::Value; c.rhs.value = v; p = msg(q); done = true;
      } catch (Err&) {}
      if (!done) {
        try {
          size_t q = ws0(p); auto f = std::make_shared<FuncExpr>(); q = function_expr(q, *f);
          c.rhs = LetValue(); c.rhs.k = LetValue::Func; c.rhs.func = f; p = msg(q); done = true;
        } catch (Err&) {}
      }
      if (!done) {
        size_t q = ws0(p); c.rhs = LetValue(); c.rhs.k = LetValue::Access; q = access(q, c.rhs.access); p = msg(q);
      }
    } catch (Err& e) { F(at, add_ctx(CTX_RHS, e.ctx)); }
    catch (Fail& e) { F(at, add_ctx(CTX_RHS, e.ctx)); }
    c.has_rhs = true;
    return p;
  }
  size_t block_clause(size_t p, Clause& c) const {
    c = Clause(); c.k = Clause::BlockClause; c.loc = loc(p);
    p = access(p, c.query);
    try {
      size_t q = ws0(p); q = not_(q);
      if (starts(q, "EMPTY") || starts(q, "empty")) { p = q + 5; c.not_empty = true; }
    } catch (Err&) {}
    return block(p, c.block, 0);
  }
  size_t parameterized_rule_call_clause(size_t p, Clause& c) const {
    c = Clause(); c.k = Clause::ParamRule; c.loc = loc(p);
    try { p = not_(p); c.negation = true; } catch (Err&) {}
    p = call_expr(p, c.rule, c.params);
    try { size_t q = ws0(p); p = custom_message(q, c.msg); c.has_msg = true; } catch (Err&) {}
    return p;
  }
  // clause  (parser.rs:1202-1219)
  size_t clause(size_t p, Clause& c) const {
    try { return when_block(p, c, /*rule_level_block=*/false); } catch (Err&) {}
    try { return block_clause(p, c); } catch (Err&) {}
    try { return parameterized_rule_call_clause(p, c); } catch (Err&) {}
    return clause_with_map(p, c);
  }
  size_t newline(size_t p) const { if (starts(p, "\n")) return p + 1; if (starts(p, "\r\n")) return p + 2; E(p); }
  size_t rule_clause(size_t p, Clause& c) const {
    c = Clause(); c.k = Clause::NamedRule; c.loc = loc(p);
    try { p = not_(p); c.negation = true; } catch (Err&) {}
    p = var_name(p, c.rule);
    bool ret = p >= n;
    if (!ret) {
      try { newline(space0(p)); ret = true; } catch (Err&) {}
      if (!ret) try { comment2(space0(p)); ret = true; } catch (Err&) {}
      if (!ret) try { ch(space0(p), '{'); ret = true; } catch (Err&) {}
      if (!ret) try { or_join(p); ret = true; } catch (Err&) {}
    }
    if (ret) return p;
    try { p = custom_message(space0(p), c.msg); c.has_msg = true; } catch (Err& e) { F(e.pos, e.ctx); }
    return p;
  }
  // parser kinds for cnf: 0 = clause, 1 = single_clauses element, 2 = clause | rule_clause, 3 = type_block
  size_t elem(size_t p, int kind, Clause& c) const {
    switch (kind) {
      case 0: return clause(p, c);
      case 1:
        try { return clause_with_map(p, c); } catch (Err&) {}
        try { return parameterized_rule_call_clause(p, c); } catch (Err&) {}
        return rule_clause(p, c);
      case 2:
        try { return clause(p, c); } catch (Err&) {}
        return rule_clause(p, c);
      default: {
        c = Clause(); c.k = Clause::TypeBlockK; c.rule_level = true;
        c.tb = std::make_shared<TypeBlock>();
        return type_block(p, *c.tb);
      }
    }
  }
  size_t disjunction_clauses(size_t p, Disj& out, int kind) const {
    out.clear();
    auto one = [&](size_t q, Disj& d) { auto c = std::make_shared<Clause>(); q = elem(ws0(q), kind, *c); d.push_back(c); return q; };
    p = one(p, out);
    for (;;) {
      size_t q;
      try { q = or_join(p); } catch (Err&) { return p; }
      Disj tmp;
      try { q = one(q, tmp); } catch (Err&) { return p; }
      out.push_back(tmp[0]); p = q;
    }
  }
  size_t cnf_clauses(size_t p, Conj& out, int kind) const {
    out.clear();
    const size_t p0 = p;
    for (;;) {
      Disj d; size_t q;
      try { q = disjunction_clauses(p, d, kind); }
      catch (Err&) {
        if (out.empty()) {   // parser.rs:1300-1312: a Failure at the conjunction's own input
          FileLoc l = loc(p0);
          F(p0, "There were no clauses present " + file + "#" + std::to_string(l.line) + "@" + std::to_string(l.column));
        }
        return p;
      }
      out.push_back(d); p = q;
    }
  }
  size_t let_assignment_expr(size_t p, std::string& name) const {
    p = tag(p, "let");
    p = ws1(p);
    p = var_name(p, name);
    size_t q = ws0(p);
    if (starts(q, "=")) return q + 1;
    if (starts(q, ":=")) return q + 2;
    F(q);   // cut(preceded(ws, alt((tag("="), tag(":=")))))
  }
  size_t assignment(size_t p, LetExpr& le) const {
    p = let_assignment_expr(p, le.var);
    try { LitValue v; size_t q = parse_value(p, v); le.value = LetValue(); le.value.k = LetValue::Value; le.value.value = v; return q; } catch (Err&) {}
    try {
      size_t q = ws0(p); auto f = std::make_shared<FuncExpr>(); q = function_expr(q, *f);
      le.value = LetValue(); le.value.k = LetValue::Func; le.value.func = f; return q;
    } catch (Err&) {} catch (Fail&) {}
    try {
      size_t q = ws0(p); le.value = LetValue(); le.value.k = LetValue::Access; return access(q, le.value.access);
    } catch (Err& e) { F(e.pos, e.ctx); }
  }
  size_t when_conditions(size_t p, Conj& conds) const {
    p = ws0(p);
    if (starts(p, "when") || starts(p, "WHEN")) p += 4; else E(p);
    try { p = ws1(p); return cnf_clauses(p, conds, 1); } catch (Err& e) { F(e.pos, e.ctx); }
  }
  // block(clause_parser) with items: assignment | disjunction_clauses(kind)
  size_t block(size_t p, Block& b, int kind) const {
    p = white_space(p, '{');
    b = Block();
    auto item = [&](size_t q) -> size_t {
      try { size_t r = ws0(q); LetExpr le; r = assignment(r, le); b.assignments.push_back(le); return r; } catch (Err&) {}
      Disj d; size_t r = disjunction_clauses(q, d, kind); b.conjunctions.push_back(d); return r;
    };
    try { p = item(p); } catch (Err&) { E(p); }   // fold_many1
    for (;;) { size_t q; try { q = item(p); } catch (Err&) { break; } p = q; }
    try { return white_space(p, '}'); } catch (Err& e) { F(e.pos, e.ctx); }
  }
  size_t rule_block_items(size_t p, Block& b) const {
    // block(rule_block_clause)
    p = white_space(p, '{');
    b = Block();
    auto item = [&](size_t q) -> size_t {
      try { size_t r = ws0(q); LetExpr le; r = assignment(r, le); b.assignments.push_back(le); return r; } catch (Err&) {}
      Disj d;
      size_t r = rule_disjunction(q, d);
      b.conjunctions.push_back(d);
      return r;
    };
    try { p = item(p); } catch (Err&) { E(p); }   // fold_many1
    for (;;) { size_t q; try { q = item(p); } catch (Err&) { break; } p = q; }
    try { return white_space(p, '}'); } catch (Err& e) { F(e.pos, e.ctx); }
  }
  size_t rule_disjunction(size_t p, Disj& out) const {
    out.clear();
    auto one = [&](size_t q, Disj& d) { auto c = std::make_shared<Clause>(); q = rule_block_clause(ws0(q), *c); d.push_back(c); return q; };
    p = one(p, out);
    for (;;) {
      size_t q;
      try { q = or_join(p); } catch (Err&) { return p; }
      Disj tmp;
      try { q = one(q, tmp); } catch (Err&) { return p; }
      out.push_back(tmp[0]); p = q;
    }
  }
  size_t type_name(size_t p, std::string& out) const {
    try {
      std::string a, b, c;
      size_t q = var_name(p, a); q = tag(q, "::"); q = var_name(q, b); q = tag(q, "::"); q = var_name(q, c);
      if (starts(q, "::MODULE")) q += 8;
      out = a + "::" + b + "::" + c;
      return q;
    } catch (Err&) {}
    std::string a, b;
    size_t q = var_name(p, a); q = tag(q, "::"); q = var_name(q, b);
    out = a + "::" + b;
    return q;
  }
  size_t type_block(size_t p, TypeBlock& tb) const {
    FileLoc l = loc(p);
    p = type_name(p, tb.type_name);
    try { p = ws1(p); } catch (Err& e) { F(e.pos, e.ctx); }
    tb.has_conditions = false;
    try { p = when_conditions(p, tb.conditions); tb.has_conditions = true; } catch (Err&) {}
    if (tb.has_conditions) {
      try { p = block(p, tb.block, 0); } catch (Err& e) { F(e.pos, e.ctx); }
    } else {
      try { p = block(p, tb.block, 0); }
      catch (Err&) {
        try {
          size_t q = ws0(p);
          auto c = std::make_shared<Clause>();
          p = clause(q, *c);
          tb.block = Block();
          tb.block.conjunctions.push_back(Disj{c});
        } catch (Err& e) { F(e.pos, e.ctx); }
      }
    }
    // desugaring: Resources.*[ Type == "<type>" ]   (parser.rs:1631-1655)
    auto tc = std::make_shared<Clause>();
    tc->k = Clause::Access; tc->loc = l;
    QueryPart tk; tk.k = QueryPart::Key; tk.key = "Type";
    tc->query.parts = {tk}; tc->query.match_all = true;
    tc->op = "Eq"; tc->op_not = false; tc->has_rhs = true;
    tc->rhs.k = LetValue::Value; tc->rhs.value.k = LitValue::String; tc->rhs.value.s = tb.type_name;
    auto conj = std::make_shared<Conj>();
    conj->push_back(Disj{tc});
    QueryPart r; r.k = QueryPart::Key; r.key = "Resources";
    QueryPart av; av.k = QueryPart::AllValues;
    QueryPart f; f.k = QueryPart::Filter; f.filter = conj;
    tb.query.parts = {r, av, f};
    tb.query.match_all = true;
    return p;
  }
  size_t when_block(size_t p, Clause& c, bool rule_level_items) const {
    p = ws0(p);
    Conj conds;
    p = when_conditions(p, conds);
    c = Clause(); c.k = Clause::WhenBlock; c.conditions = conds;
    return block(p, c.block, rule_level_items ? 2 : 0);
  }
  size_t rule_block_clause(size_t p, Clause& c) const {
    try {
      size_t q = ws0(p);
      auto tb = std::make_shared<TypeBlock>();
      q = type_block(q, *tb);
      c = Clause(); c.k = Clause::TypeBlockK; c.tb = tb; c.rule_level = true;
      return q;
    } catch (Err&) {}
    try {
      size_t q = ws0(p);
      Conj conds;
      q = when_conditions(q, conds);
      Block b;
      q = block(q, b, 2);
      c = Clause(); c.k = Clause::WhenBlock; c.rule_level = true; c.conditions = conds; c.block = b;
      return q;
    } catch (Err&) {}
    size_t q = ws0(p);
    try { return clause(q, c); } catch (Err&) {}
    return rule_clause(q, c);
  }
  size_t rule_block(size_t p, Rule& r) const {
    p = ws0(p);
    p = tag(p, "rule");
    p = ws1(p);
    try { p = var_name(p, r.name); } catch (Err& e) { F(e.pos, e.ctx); }
    r.has_conditions = false;
    try { p = when_conditions(p, r.conditions); r.has_conditions = true; } catch (Err&) {}
    try { return rule_block_items(p, r.block); } catch (Err& e) { F(e.pos, e.ctx); }
  }
  size_t parameter_names(size_t p, std::vector<std::string>& names) const {
    p = ch(p, '(');
    auto elem2 = [&](size_t q, std::string& nm) -> size_t {
      try { q = multispace0(q); q = var_name(q, nm); return multispace0(q); } catch (Err& e) { F(e.pos, e.ctx); }
    };
    std::string nm; p = elem2(p, nm);
    names.clear(); names.push_back(nm);
    for (;;) {
      size_t q;
      try { q = ch(p, ','); } catch (Err&) { break; }
      std::string nm2;
      q = elem2(q, nm2);
      bool dup = false;
      for (auto& x : names) if (x == nm2) dup = true;
      if (!dup) names.push_back(nm2);
      p = q;
    }
    try { return ch(p, ')'); } catch (Err& e) { F(e.pos, e.ctx); }
  }
  size_t parameterized_rule_block(size_t p, ParamRule& pr) const {
    p = ws0(p);
    p = tag(p, "rule");
    p = ws1(p);
    try { p = var_name(p, pr.rule.name); } catch (Err& e) { F(e.pos, e.ctx); }
    p = parameter_names(p, pr.params);
    pr.rule.has_conditions = false;
    try { return rule_block_items(p, pr.rule.block); } catch (Err& e) { F(e.pos, e.ctx); }
  }
  size_t or_join(size_t p) const {
    p = ws0(p);
    if (starts(p, "|OR|")) p += 4;
    else if (starts(p, "or") || starts(p, "OR")) p += 2;
    else E(p);
    return ws1(p);
  }

  bool rules_file(RulesFile& rf, bool& empty) const {
    size_t p = ws0(0);
    empty = false;
    if (p >= n) { empty = true; return true; }
    Conj defaults;
    bool any = false;
    const size_t p0 = p;
    for (;;) {
      size_t q = ws0(p);
      bool matched = false;
      try { LetExpr le; size_t r = assignment(q, le); rf.assignments.push_back(le); p = ws0(r); matched = true; } catch (Err&) {}
      if (!matched) try { ParamRule pr; size_t r = parameterized_rule_block(q, pr); rf.param_rules.push_back(pr); p = ws0(r); matched = true; } catch (Err&) {}
      if (!matched) try { Rule r0; size_t r = rule_block(q, r0); rf.rules.push_back(r0); p = ws0(r); matched = true; } catch (Err&) {}
      if (!matched) try { Disj d; size_t r = disjunction_clauses(q, d, 3); defaults.push_back(d); p = ws0(r); matched = true; } catch (Err&) {}
      if (!matched) try {
        auto c = std::make_shared<Clause>(); size_t r = when_block(q, *c, true); c->rule_level = true;
        defaults.push_back(Disj{c}); p = ws0(r); matched = true;
      } catch (Err&) {}
      if (!matched) try { Disj d; size_t r = disjunction_clauses(q, d, 0); defaults.push_back(d); p = ws0(r); matched = true; } catch (Err&) {}
      if (!matched) { if (!any) E(p0); break; }   // fold_many1: from_error_kind(input, Many1)
      any = true;
      if (p >= n) break;
    }
    if (p != n) E(p);   // all_consuming: Eof at the first unparsed item
    if (!defaults.empty()) {
      Rule d;
      std::string trimmed = file;
      bool blank = true;
      for (char c : trimmed) if (!isspace((unsigned char)c)) blank = false;
      d.name = blank ? "default" : file + "/default";
      d.block.conjunctions = defaults;
      rf.rules.insert(rf.rules.begin(), d);
    }
    return true;
  }
};

}  // namespace

bool parse_rules_file(const std::string& text, const std::string& file_name, RulesFile& out, bool& empty, std::string& msg) {
  P p(text, file_name);
  // nom::Err<ParserError> -> Error::ParseError("Parsing Error {ParserError}") (errors.rs:107-115)
  try {
    return p.rules_file(out, empty);
  } catch (Err& e) {
    msg = "Parsing Error " + p.error_text(e.pos, e.ctx);
  } catch (Fail& e) {
    msg = "Parsing Error " + p.error_text(e.pos, e.ctx);
  }
  return false;
}

// ------------------------------------------------------------------ display ---
static std::string part_display(const QueryPart& q) {
  switch (q.k) {
    case QueryPart::Key: return q.key;
    case QueryPart::AllIndices: return "[*]";
    case QueryPart::AllValues: return "*";
    case QueryPart::Index: return std::to_string(q.index);
    case QueryPart::Filter: return (q.has_name ? q.key : std::string()) + " (filter-clauses)";
    case QueryPart::MapKeyFilter: return (q.has_name ? q.key : std::string()) + " (map-key-filter-clauses)";
    default: return "_";
  }
}

std::string slice_display(const std::vector<QueryPart>& parts, size_t from) {
  std::string q;
  bool first = true;
  for (size_t i = from; i < parts.size(); i++) {
    if (!first) q += "." + part_display(parts[i]);
    else q = part_display(parts[i]);
    first = false;
  }
  std::string out;
  for (size_t i = 0; i < q.size(); i++) {
    if (q[i] == '.' && i + 1 < q.size() && q[i + 1] == '[') continue;
    out.push_back(q[i]);
  }
  return out;
}

std::string value_only_display(const LitValue& v) {
  switch (v.k) {
    case LitValue::Null: return "\"NULL\"";
    case LitValue::String: return "\"" + v.s + "\"";
    case LitValue::Regex: return "\"/" + v.s + "/\"";
    case LitValue::Bool: return v.b ? "true" : "false";
    case LitValue::Int: return std::to_string(v.i);
    case LitValue::Float: return rust_display_f64(v.f);
    case LitValue::Char: { std::string s = "'"; utf8_append(s, v.ch); return s + "'"; }
    case LitValue::List: {
      std::string s = "[";
      for (size_t i = 0; i < v.items.size(); i++) { if (i) s += ","; s += value_only_display(v.items[i]); }
      return s + "]";
    }
    case LitValue::Map: {
      std::string s = "{";
      for (size_t i = 0; i < v.kv.size(); i++) { if (i) s += ","; s += "\"" + v.kv[i].first + "\":" + value_only_display(v.kv[i].second); }
      return s + "}";
    }
    default: {
      std::string lo, hi;
      if (v.k == LitValue::RangeInt) { lo = std::to_string(v.ilo); hi = std::to_string(v.ihi); }
      else if (v.k == LitValue::RangeFloat) { lo = rust_display_f64(v.flo); hi = rust_display_f64(v.fhi); }
      else { utf8_append(lo, v.clo); utf8_append(hi, v.chi); }
      return std::string(v.incl & 1 ? "[" : "(") + lo + "," + hi + (v.incl & 2 ? "]" : ")");
    }
  }
}

static std::string let_value_display(const LetValue& lv) {
  if (lv.k == LetValue::Access) return slice_display(lv.access.parts);
  if (lv.k == LetValue::Value) return value_only_display(lv.value);
  std::string s = lv.func->name + "(";
  for (size_t i = 0; i < lv.func->params.size(); i++) { if (i) s += ", "; s += let_value_display(lv.func->params[i]); }
  return s + ")";
}

static const char* cmp_display(const std::string& op) {
  static const char* m[][2] = {{"Eq", "EQUALS"}, {"In", "IN"}, {"Gt", "GREATER THAN"}, {"Lt", "LESS THAN"},
                               {"Ge", "GREATER THAN EQUALS"}, {"Le", "LESS THAN EQUALS"}, {"Exists", "EXISTS"},
                               {"Empty", "EMPTY"}, {"IsString", "IS STRING"}, {"IsBool", "IS BOOL"}, {"IsInt", "IS INT"},
                               {"IsList", "IS LIST"}, {"IsMap", "IS MAP"}, {"IsNull", "IS NULL"}, {"IsFloat", "IS FLOAT"}};
  for (auto& e : m) if (op == e[0]) return e[1];
  return "";
}

std::string gac_display(const Clause& c) {
  std::string cmp = std::string(c.op_not ? "not " : "") + cmp_display(c.op) + " ";
  std::string ac = slice_display(c.query.parts) + " " + cmp + " " + (c.has_rhs ? let_value_display(c.rhs) : std::string());
  return std::string(c.negation ? "not" : "") + " " + ac;
}

std::string file_location_display(const FileLoc& l) {
  return "Location[file:" + l.file + ", line:" + std::to_string(l.line) + ", column:" + std::to_string(l.column) + "]";
}

}  // namespace gg
