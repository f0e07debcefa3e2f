// Device records -> structured JSON (see reporter.h).
#include "reporter.h"

#include <functional>
#include <memory>
#include <thread>

#include <yaml.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>
#include <stdexcept>

#include "host_format.h"

namespace gg {

namespace {

const char* const CMP_NAMES[] = {"Eq", "In", "Gt", "Lt", "Le", "Ge", "Exists", "Empty", "IsString", "IsList", "IsMap",
                                 "IsBool", "IsInt", "IsFloat", "IsNull"};

struct J {
  // Cmp: the `comparison` pair [CmpOperator, not] (op in `op`, not in `b`), kept unboxed because
  // every clause record carries one
  enum T { Null, Bool, Raw, Str, Arr, Obj, Cmp } t = Null;
  uint32_t op = 0;
  std::string s;
  bool b = false;
  std::vector<J> a;
  std::vector<std::pair<std::string, J>> o;
  int64_t loc_line = -1, loc_col = -1;   // Messages.location (skip_serializing; read by the SARIF writer)
  // a serialized PathAwareValue / UnResolved keeps the value it came from (the console reporters read
  // its location and ValueOnlyDisplay)
  QR q{};
  bool hasq = false;
  static J null() { return J(); }
  static J str(const std::string& v) { J j; j.t = Str; j.s = v; return j; }
  static J raw(const std::string& v) { J j; j.t = Raw; j.s = v; return j; }
  static J boolean(bool v) { J j; j.t = Bool; j.b = v; return j; }
  static J arr() { J j; j.t = Arr; return j; }
  static J obj() { J j; j.t = Obj; return j; }
  static J cmp(uint32_t op, bool neg) { J j; j.t = Cmp; j.op = op; j.b = neg; return j; }
  J& add(const std::string& k, J v) { o.push_back({k, std::move(v)}); return *this; }
  J& push(J v) { a.push_back(std::move(v)); return *this; }
};

void pretty(const J& j, int indent, std::string& out) {
  switch (j.t) {
    case J::Null: out += "null"; return;
    case J::Bool: out += j.b ? "true" : "false"; return;
    case J::Raw: out += j.s; return;
    case J::Str: json_escape_into(out, j.s.data(), j.s.size()); return;
    case J::Cmp:
      out += "[\n";
      out.append((indent + 1) * 2, ' ');
      out += '"'; out += CMP_NAMES[j.op]; out += "\",\n";
      out.append((indent + 1) * 2, ' ');
      out += j.b ? "true\n" : "false\n";
      out.append(indent * 2, ' ');
      out += "]";
      return;
    case J::Arr: {
      if (j.a.empty()) { out += "[]"; return; }
      out += "[\n";
      for (size_t i = 0; i < j.a.size(); i++) {
        out.append((indent + 1) * 2, ' ');
        pretty(j.a[i], indent + 1, out);
        if (i + 1 < j.a.size()) out += ",";
        out += "\n";
      }
      out.append(indent * 2, ' ');
      out += "]";
      return;
    }
    case J::Obj: {
      if (j.o.empty()) { out += "{}"; return; }
      out += "{\n";
      for (size_t i = 0; i < j.o.size(); i++) {
        out.append((indent + 1) * 2, ' ');
        json_escape_into(out, j.o[i].first.data(), j.o[i].first.size());
        out += ": ";
        pretty(j.o[i].second, indent + 1, out);
        if (i + 1 < j.o.size()) out += ",";
        out += "\n";
      }
      out.append(indent * 2, ' ');
      out += "}";
      return;
    }
  }
}

const char* type_info(uint32_t k) {
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

struct Fatal { std::string kind, msg; };

struct R {
  const DocBatch& docs;
  const Program& prog;
  bool serde;
  uint64_t dbase;   // global index of the reported document's first node (refs are relative)
  const RecSpan* aux = nullptr;   // the tile's side records (join-key lists, R4 / R5)

  static const uint32_t KEY_BIT = 0x20000000u;   // "the key of map entry X" (MapValue.keys)
  // an unresolved result whose traversed_to is a count() value: SYN_BIT | the side record holding it
  // (eval_core.inc publishable) -- an Int at the path and location of the count's first argument
  static const uint32_t SYN_BIT = 0x40000000u;
  bool is_syn(uint32_t ref) const { return ref != NONE && (ref & SYN_BIT) != 0; }
  const QR& syn_of(uint32_t ref) const { return aux_at(ref & ~SYN_BIT).from; }
  const DocBatch& B(uint32_t ref) const { return (ref & LIT_BIT) ? prog.lit : docs; }
  uint32_t I(uint32_t ref) const { return ref & ~(LIT_BIT | KEY_BIT); }
  uint64_t base_of(uint32_t ref) const { return (ref & LIT_BIT) ? 0 : dbase; }
  uint64_t G(uint32_t ref) const { return base_of(ref) + I(ref); }
  bool is_key(uint32_t ref) const { return (ref & KEY_BIT) != 0; }
  // key refs read as a String node whose bytes are the entry's key
  DNode key_node(uint32_t ref) const {
    const DNode& e = B(ref).nodes[G(ref)];
    DNode d; d.kind = K_STRING; d.count = e.key_len; d.a = e.key_off; d.b = e.key_hash;
    d.key_off = NONE; d.key_len = 0; d.key_hash = 0; d.parent = NONE;
    return d;
  }
  DNode N(uint32_t ref) const {
    if (is_syn(ref)) {
      const QR& q = syn_of(ref);
      DNode d{}; d.kind = K_INT; d.a = q.uref; d.b = q.aux; d.key_off = NONE; d.parent = NONE;
      return d;
    }
    return is_key(ref) ? key_node(ref) : B(ref).nodes[G(ref)];
  }
  std::string str(uint32_t ref) const { DNode n = N(ref); return B(ref).bytes.substr(n.a, n.count); }
  std::string key(uint32_t ref) const { DNode n = N(ref); return B(ref).bytes.substr(n.key_off, n.key_len); }
  uint32_t child(uint32_t ref, uint32_t j) const { return (ref & LIT_BIT) | (N(ref).a + j); }
  // key PV paths: libyaml loader -> the map's path at the key mark (path_value.rs:467-470);
  // serde loader / rule literals -> map path + "/key" at the map's (0,0) location (:391-395)
  bool key_serde(uint32_t ref) const { return (ref & LIT_BIT) || docs.serde; }
  // a key PathAwareValue::merge pushed (input parameters): map path + "/key" at kline's location
  bool key_ext(uint32_t ref) const { return !(ref & LIT_BIT) && (B(ref).kline[G(ref)] & kKeyPathExt) != 0; }
  uint32_t parent_of(uint32_t ref) const { return B(ref).nodes[G(ref)].parent; }
  std::string path(uint32_t ref) const {
    if (is_syn(ref)) { const uint32_t src = syn_of(ref).node; return src == NONE ? std::string() : path(src); }
    if (!is_key(ref)) return B(ref).path(base_of(ref), I(ref));
    std::string mp = B(ref).path(base_of(ref), parent_of(ref));
    if (key_serde(ref) || key_ext(ref)) { const DNode& e = B(ref).nodes[G(ref)]; return mp + "/" + B(ref).bytes.substr(e.key_off, e.key_len); }
    return mp;
  }
  uint32_t line(uint32_t ref) const {
    if (is_syn(ref)) { const uint32_t src = syn_of(ref).node; return src == NONE ? 0 : line(src); }
    if (!is_key(ref)) return B(ref).line[G(ref)];
    return key_serde(ref) ? 0 : B(ref).kline[G(ref)] & ~kKeyPathExt;
  }
  uint32_t col(uint32_t ref) const {
    if (is_syn(ref)) { const uint32_t src = syn_of(ref).node; return src == NONE ? 0 : col(src); }
    if (!is_key(ref)) return B(ref).col[G(ref)];
    return key_serde(ref) ? 0 : B(ref).kcol[G(ref)];
  }
  std::string loc(uint32_t l, uint32_t c) const { return "[L:" + std::to_string(l) + ",C:" + std::to_string(c) + "]"; }
  std::string path_display(uint32_t ref) const { return path(ref) + loc(line(ref), col(ref)); }
  int64_t ival(const DNode& n) const { return (int64_t)(((uint64_t)n.b << 32) | n.a); }
  double fval(const DNode& n) const { uint64_t u = ((uint64_t)n.b << 32) | n.a; double d; memcpy(&d, &u, 8); return d; }

  std::string range_str(const DNode& n) const {
    const DRange& r = prog.ranges[n.a];
    std::string lo, hi;
    if (n.kind == K_RANGE_INT) { lo = std::to_string((int64_t)r.lo); hi = std::to_string((int64_t)r.hi); }
    else if (n.kind == K_RANGE_FLOAT) { double a, b; memcpy(&a, &r.lo, 8); memcpy(&b, &r.hi, 8); lo = rust_display_f64(a); hi = rust_display_f64(b); }
    else { utf8_append(lo, (uint32_t)r.lo); utf8_append(hi, (uint32_t)r.hi); }
    return std::string(r.incl & 1 ? "[" : "(") + lo + "," + hi + (r.incl & 2 ? "]" : ")");
  }

  J value_json(uint32_t ref) const {
    const DNode& n = N(ref);
    switch (n.kind) {
      case K_NULL: return J::null();
      case K_STRING: return J::str(str(ref));
      case K_REGEX: return J::str("/" + str(ref) + "/");
      case K_BOOL: return J::boolean(n.a != 0);
      case K_INT: return J::raw(std::to_string(ival(n)));
      case K_FLOAT: {
        double d = fval(n);
        if (std::isnan(d) || std::isinf(d))
          throw Fatal{"IncompatibleError", "Could not convert float " + rust_display_f64(d) + " to serde::Value::Number"};
        return J::raw(ryu_f64(d));
      }
      case K_CHAR: { std::string s; utf8_append(s, n.a); return J::str(s); }
      case K_LIST: { J a = J::arr(); for (uint32_t j = 0; j < n.count; j++) a.push(value_json(child(ref, j))); return a; }
      case K_MAP: { J o = J::obj(); for (uint32_t j = 0; j < n.count; j++) { uint32_t c = child(ref, j); o.add(key(c), value_json(c)); } return o; }
      default: return J::str(range_str(n));
    }
  }

  // ValueOnlyDisplay (display.rs:33-107), appended to `s`
  void value_only_into(std::string& s, uint32_t ref) const {
    const DNode& n = N(ref);
    switch (n.kind) {
      case K_NULL: s += "\"NULL\""; return;
      case K_STRING: { const DocBatch& b = B(ref); s += '"'; s.append(b.bytes.data() + n.a, n.count); s += '"'; return; }
      case K_REGEX: { const DocBatch& b = B(ref); s += "\"/"; s.append(b.bytes.data() + n.a, n.count); s += "/\""; return; }
      case K_BOOL: s += n.a ? "true" : "false"; return;
      case K_INT: s += std::to_string(ival(n)); return;
      case K_FLOAT: s += rust_display_f64(fval(n)); return;
      case K_CHAR: s += '\''; utf8_append(s, n.a); s += '\''; return;
      case K_LIST:
        s += '[';
        for (uint32_t j = 0; j < n.count; j++) { if (j) s += ','; value_only_into(s, child(ref, j)); }
        s += ']';
        return;
      case K_MAP:
        s += '{';
        for (uint32_t j = 0; j < n.count; j++) {
          if (j) s += ',';
          const uint32_t c = child(ref, j);
          const DNode& cn = N(c);
          s += '"'; s.append(B(c).bytes.data() + cn.key_off, cn.key_len); s += "\":";
          value_only_into(s, c);
        }
        s += '}';
        return;
      default: s += range_str(n); return;
    }
  }
  std::string value_only(uint32_t ref) const { std::string s; value_only_into(s, ref); return s; }

  std::string dbg_path(const std::string& p, uint32_t l, uint32_t c) const {
    return "Path(" + rust_debug_str(p) + ", Location { line: " + std::to_string(l) + ", col: " + std::to_string(c) + " })";
  }

  std::string debug(uint32_t ref) const {
    const DNode& n = N(ref);
    std::string p = dbg_path(path(ref), line(ref), col(ref));
    switch (n.kind) {
      case K_NULL: return "Null(" + p + ")";
      case K_STRING: return "String((" + p + ", " + rust_debug_str(str(ref)) + "))";
      case K_REGEX: return "Regex((" + p + ", " + rust_debug_str(str(ref)) + "))";
      case K_BOOL: return std::string("Bool((") + p + ", " + (n.a ? "true" : "false") + "))";
      case K_INT: return "Int((" + p + ", " + std::to_string(ival(n)) + "))";
      case K_FLOAT: return "Float((" + p + ", " + rust_debug_f64(fval(n)) + "))";
      case K_CHAR: { std::string s; utf8_append(s, n.a); return "Char((" + p + ", '" + s + "'))"; }
      case K_LIST: {
        std::string s = "List((" + p + ", [";
        for (uint32_t j = 0; j < n.count; j++) { if (j) s += ", "; s += debug(child(ref, j)); }
        return s + "]))";
      }
      case K_MAP: {
        std::string keys, vals;
        std::string mp = path(ref);
        const bool lit = (ref & LIT_BIT) != 0;
        // MapValue.keys: the entries' keys, or the key block of a map with a repeated key (every
        // occurrence; doc_loader.cpp Emitter)
        const uint32_t kb = lit ? 0u : n.b;
        const uint32_t nkeys = kb ? B(ref).nodes[base_of(ref) + kb].count : n.count;
        for (uint32_t j = 0; j < nkeys; j++) {
          const uint32_t c = kb ? kb + j : child(ref, j);
          std::string k = key(c);
          if (j) keys += ", ";
          // libyaml mode -> parent path at the key mark; serde mode -> path/key at L0,C0
          if (serde || lit) keys += "String((" + dbg_path(mp + "/" + k, 0, 0) + ", " + rust_debug_str(k) + "))";
          else {
            const uint32_t kl = B(c).kline[G(c)];
            keys += "String((" + dbg_path((kl & kKeyPathExt) ? mp + "/" + k : mp, kl & ~kKeyPathExt, B(c).kcol[G(c)]) + ", " +
                    rust_debug_str(k) + "))";
          }
        }
        for (uint32_t j = 0; j < n.count; j++) {
          uint32_t c = child(ref, j);
          if (j) vals += ", ";
          vals += rust_debug_str(key(c)) + ": " + debug(c);
        }
        return "Map((" + p + ", MapValue { keys: [" + keys + "], values: {" + vals + "} }))";
      }
      default: {
        const DRange& r = prog.ranges[n.a];
        std::string lo, hi;
        const char* nm = n.kind == K_RANGE_INT ? "RangeInt" : n.kind == K_RANGE_FLOAT ? "RangeFloat" : "RangeChar";
        if (n.kind == K_RANGE_INT) { lo = std::to_string((int64_t)r.lo); hi = std::to_string((int64_t)r.hi); }
        else if (n.kind == K_RANGE_FLOAT) { double a, b; memcpy(&a, &r.lo, 8); memcpy(&b, &r.hi, 8); lo = rust_debug_f64(a); hi = rust_debug_f64(b); }
        else { std::string a, b; utf8_append(a, (uint32_t)r.lo); utf8_append(b, (uint32_t)r.hi); lo = "'" + a + "'"; hi = "'" + b + "'"; }
        return std::string(nm) + "((" + p + ", RangeType { upper: " + hi + ", lower: " + lo + ", inclusive: " + std::to_string(r.incl) + " }))";
      }
    }
  }

  // QR helpers ------------------------------------------------------------
  bool is_synth(const QR& q) const { return (q.meta & 3u) == QR_SYNTH_INT; }
  std::string q_path(const QR& q) const { return is_synth(q) ? (q.node == NONE ? "" : path(q.node)) : path(q.node); }
  std::string q_path_display(const QR& q) const {
    if (is_synth(q)) return q.node == NONE ? "[L:0,C:0]" : path_display(q.node);
    return path_display(q.node);
  }
  int64_t synth_val(const QR& q) const { return (int64_t)(((uint64_t)q.aux << 32) | q.uref); }
  J pav_json(const QR& q) const {
    J o = J::obj();
    o.q = q; o.hasq = true;
    o.add("path", J::str(q_path(q)));
    o.add("value", is_synth(q) ? J::raw(std::to_string(synth_val(q))) : value_json(q.node));
    return o;
  }
  std::string pav_display(const QR& q) const {
    if (is_synth(q)) return "Path=" + q_path_display(q) + " Value=" + std::to_string(synth_val(q));
    return "Path=" + path_display(q.node) + " Value=" + value_only(q.node);
  }

  std::string reason(const QR& q) const {
    uint32_t code = (q.meta >> 8) & 0xFF;
    uint32_t qid = q.uref >> 12;
    uint32_t step = q.uref & 0xFFF;
    uint32_t cur = q.node;
    const auto& parts = prog.queries[qid];
    const DNode& n = N(cur);
    switch (code) {
      case R_INDEX_OOB: {
        std::string els;
        for (uint32_t j = 0; j < n.count; j++) { if (j) els += ", "; els += debug(child(cur, j)); }
        return "Array Index out of bounds for path = " + path_display(cur) + " on index = " + std::to_string((int32_t)q.aux) +
               " inside Array = [" + els + "], remaining query = " + slice_display(parts, 0);
      }
      case R_NO_MORE_ENTRIES:
        return "No more entries for value at path = " + path_display(cur) + " on type = " + type_info(n.kind) + " ";
      case R_KEY_INDEX_NOT_ARRAY:
        return "Attempting to retrieve from index " + std::to_string((int32_t)q.aux) + " but type is not an array at path " + path_display(cur);
      case R_LOCATE_KEY:
        return "Could not locate key = " + str(q.aux) + " inside struct at path = " + path_display(cur);
      case R_LOCATE_KEY_LIST:
        return "Could not locate key = " + str(q.aux) + " inside struct at path = " + path_display(q.aux);
      case R_KEY_NOT_FOUND:
        return "Could not find key " + parts[step].key + " inside struct at path " + path_display(cur);
      case R_NOT_STRUCT:
        return "Attempting to retrieve from key " + parts[step].key + " but type is not an struct type at path " +
               path_display(cur) + ", Type = " + type_info(n.kind) + ", Value = " + debug(cur);
      case R_INDEX_NOT_ARRAY:
        return "Attempting to retrieve from index " + std::to_string(parts[step].index) + " but type is not an array at path " +
               path_display(cur) + ", type " + type_info(n.kind);
      case R_FILTER_NOT_STRUCT:
        return std::string("Filter on value type that was not a struct or array ") + type_info(n.kind) + " " + path_display(cur);
      case R_MAPFILTER_NOT_STRUCT:   // eval_context.rs:913-919
        return std::string("Map Filter for keys was not a struct ") + type_info(n.kind) + " " + path_display(cur);
      case R_VAR_INDEX_OOB: {
        // eval_context.rs:432-435: aux[q.aux] = {clause: var, x: #keys, y: index}, then the keys in pairs
        const Rec& h = aux_at(q.aux);
        std::string keys;
        for (uint32_t k = 0; k < h.x; k++) {
          const Rec& pr = aux_at(q.aux + 1 + k / 2);
          if (k) keys += ", ";
          keys += qr_debug(k & 1 ? pr.to : pr.from);
        }
        return "Index " + std::to_string(h.y) + " on the set of values returned for variable " + prog.var_names[h.clause] +
               " on the join, is out of bounds. Length " + std::to_string(h.x) + ", Values = [" + keys + "]";
      }
      case R_VAR_KEYS_UNRESOLVED: {
        // eval_context.rs:452-457: aux[q.aux] = {clause: var, from: the unresolved key}
        const Rec& h = aux_at(q.aux);
        return "Keys returned for variable " + prog.var_names[h.clause] + " could not completely resolve. Path traversed until " +
               path_display(h.from.node) + reason(h.from);
      }
      default:
        return "";
    }
  }
  const Rec& aux_at(uint32_t i) const {
    if (!aux || i >= aux->size()) throw Fatal{"Unsupported", "MI355X path: side record out of range"};
    return (*aux)[i];
  }
  // Debug of a QueryResult (rules/mod.rs:172-177, derived)
  std::string qr_debug(const QR& q) const {
    const uint32_t k = q.meta & 3u;
    if (k == QR_SYNTH_INT) {
      std::string p = q.node == NONE ? dbg_path("", 0, 0) : dbg_path(path(q.node), line(q.node), col(q.node));
      return "Resolved(Int((" + p + ", " + std::to_string(synth_val(q)) + ")))";
    }
    if (k == QR_LITERAL) return "Literal(" + debug(q.node) + ")";
    if (k == QR_RESOLVED) return "Resolved(" + debug(q.node) + ")";
    const std::string why = reason(q);
    return "UnResolved(UnResolved { traversed_to: " + debug(q.node) + ", remaining_query: " + rust_debug_str(remaining(q)) +
           ", reason: " + (why.empty() ? std::string("None") : "Some(" + rust_debug_str(why) + ")") + " })";
  }
  std::string remaining(const QR& q) const { return prog.query_remaining(q.uref >> 12, q.uref & 0xFFF); }
  // self_path().1.line and ValueOnlyDisplay of the value a QR carries (an unresolved one's traversed_to)
  uint32_t q_line(const QR& q) const { return q.node == NONE ? 0 : line(q.node); }
  std::string q_value_only(const QR& q) const { return is_synth(q) ? std::to_string(synth_val(q)) : value_only(q.node); }

  J unresolved_json(const QR& q) const {
    J o = J::obj();
    o.q = q; o.hasq = true;
    J t = J::obj();
    t.add("path", J::str(path(q.node)));
    t.add("value", value_json(q.node));
    o.add("traversed_to", t);
    o.add("remaining_query", J::str(remaining(q)));
    o.add("reason", J::str(reason(q)));
    return o;
  }
  std::string unresolved_display(const QR& q) const { return "Path=" + path_display(q.node) + " Value=" + value_only(q.node); }

  static J messages(const J& custom, const J& error) {
    J m = J::obj(); m.add("custom_message", custom); m.add("error_message", error); return m;
  }
  static J messages(const J& custom, const J& error, std::pair<int64_t, int64_t> loc) {
    J m = messages(custom, error); m.loc_line = loc.first; m.loc_col = loc.second; return m;
  }
  // self_path().1 of the value a QR carries (resolved value, or an unresolved one's traversed_to)
  std::pair<int64_t, int64_t> q_loc(const QR& q) const {
    if (q.node == NONE) return {0, 0};
    return {(int64_t)line(q.node), (int64_t)col(q.node)};
  }
  J comparison(uint32_t op, bool neg) const { return J::cmp(op, neg); }
  std::string custom(const PClause& pc) const { return pc.e == NONE ? "" : prog.msgs[pc.e]; }
  // NotComparable reason of a REC_CMP (rc.x != NC_NONE; operators.rs / path_value.rs compare_*)
  std::string nc_reason(const Rec& rc) const {
    if (rc.x == NC_TYPES) return std::string("PathAwareValues are not comparable ") + type_info(rc.y >> 8) + ", " + type_info(rc.y & 0xFF);
    if (rc.x == NC_FLOAT) return "Float values are not comparable";
    if (rc.x == NC_STRING_IN) return "Type not comparable, " + pav_display(rc.from) + ", " + pav_display(rc.to);
    return "Can not compare type " + pav_display(rc.from) + ", " + pav_display(rc.to);
  }
  // serde of a QueryResult (rules/mod.rs:172-177): externally tagged {"Resolved" | "Literal": PathAwareValue}
  // or {"UnResolved": {traversed_to, remaining_query, reason}}
  J qr_json(const QR& q, bool keep_literal) const {
    const uint32_t k = q.meta & 3u;
    J o = J::obj();
    if (k == QR_UNRESOLVED) o.add("UnResolved", unresolved_json(q));
    else o.add(keep_literal && k == QR_LITERAL ? "Literal" : "Resolved", pav_json(q));
    return o;
  }
  J custom_opt(const PClause& pc) const { return pc.e == NONE ? J::null() : J::str(prog.msgs[pc.e]); }
};

const char* unary_msg(uint32_t op, bool neg) {
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

const char* op_msg(uint32_t op, bool neg) {
  switch (op) {
    case OP_EQ: return neg ? "equal to" : "not equal to";
    case OP_LE: return neg ? "less than equal to" : "not less than equal to";
    case OP_LT: return neg ? "less than" : "not less than";
    case OP_GE: return neg ? "greater than equal to" : "not greater than equal";
    case OP_GT: return neg ? "greater than" : "not greater than";
    default: return neg ? "in" : "not in";
  }
}

struct Walker {
  const R& r;
  const RecSpan& recs;
  size_t i = 0;

  J clause_wrap(const char* kind, J inner) {
    J o = J::obj(); o.add(kind, std::move(inner)); return o;
  }

  // parse records until a closing record (or end); returns list of ClauseReport JSON
  J items(uint32_t close_kind) {
    J list = J::arr();
    while (i < recs.size()) {
      const Rec& rc = recs[i];
      if (rc.kind == close_kind) { i++; return list; }
      i++;
      switch (rc.kind) {
        case REC_RULE_OPEN: {
          J checks = items(REC_RULE_CLOSE);
          J rule = J::obj();
          rule.add("name", J::str(r.prog.rule_names[rc.clause]));
          rule.add("metadata", J::obj());
          rule.add("messages", R::messages(rc.x == NONE ? J::null() : J::str(r.prog.msgs[rc.x]), J::null()));
          rule.add("checks", std::move(checks));
          list.push(clause_wrap("Rule", std::move(rule)));
          break;
        }
        case REC_DISJ_OPEN: {
          J checks = items(REC_DISJ_CLOSE);
          J d = J::obj(); d.add("checks", std::move(checks));
          list.push(clause_wrap("Disjunctions", std::move(d)));
          break;
        }
        case REC_BLOCK_EMPTY: {
          const PClause& pc = r.prog.clauses[rc.clause];
          J b = J::obj();
          b.add("context", J::str(r.prog.ctx[pc.d]));
          b.add("messages", R::messages(J::null(), J::str("query for block clause did not retrieve any value")));
          b.add("unresolved", J::null());
          list.push(clause_wrap("Block", std::move(b)));
          break;
        }
        case REC_MISSING_BLOCK_VALUE: {
          const PClause& pc = r.prog.clauses[rc.clause];
          std::string err = "Check was not compliant as property [" + r.remaining(rc.from) + "] is missing. Value traversed to [" +
                            r.unresolved_display(rc.from) + "]";
          J b = J::obj();
          b.add("context", J::str(r.prog.ctx[pc.f]));
          b.add("messages", R::messages(J::str(""), J::str(err)));
          b.add("unresolved", r.unresolved_json(rc.from));
          list.push(clause_wrap("Block", std::move(b)));
          break;
        }
        case REC_UNARY: {
          const PClause& pc = r.prog.clauses[rc.clause];
          uint32_t op = pc.flags & 15u;
          bool neg = (pc.flags >> 4) & 1u;
          std::string ctx = r.prog.ctx[pc.d];
          J check = J::obj();
          std::string msg;
          if ((rc.from.meta & 3u) == QR_UNRESOLVED) {
            msg = "Check was not compliant as property [" + r.remaining(rc.from) + "] is missing. Value traversed to [" +
                  r.unresolved_display(rc.from) + "].";
            J u = J::obj(); u.add("value", r.unresolved_json(rc.from)); u.add("comparison", r.comparison(op, neg));
            check.add("UnResolved", std::move(u));
          } else {
            msg = "Check was not compliant as property [" + r.q_path_display(rc.from) + "] " + unary_msg(op, neg) + ".";
            J u = J::obj(); u.add("value", r.pav_json(rc.from)); u.add("comparison", r.comparison(op, neg));
            check.add("Resolved", std::move(u));
          }
          J un = J::obj();
          un.add("check", std::move(check));
          un.add("context", J::str(ctx));
          // eval_context.rs:2231-2234: the unresolved value's location, Location::default() otherwise
          un.add("messages", R::messages(J::str(r.custom(pc)), J::str(msg),
                                         (rc.from.meta & 3u) == QR_UNRESOLVED ? r.q_loc(rc.from) : std::make_pair<int64_t, int64_t>(0, 0)));
          list.push(clause_wrap("Clause", clause_wrap("Unary", std::move(un))));
          break;
        }
        case REC_NOVALUE_EMPTY: {
          const PClause& pc = r.prog.clauses[rc.clause];
          std::string ctx = r.prog.ctx[pc.d];
          std::string cm = r.custom(pc);
          for (auto& ch : cm) if (ch == '\n') ch = ';';
          J check = J::obj(); check.add("UnResolvedContext", J::str(ctx));
          J un = J::obj();
          un.add("check", std::move(check));
          un.add("context", J::str(ctx));
          un.add("messages", R::messages(J::str(cm), J::str("Check was not compliant as variable in context [" + ctx + "] was not empty")));
          list.push(clause_wrap("Clause", clause_wrap("Unary", std::move(un))));
          break;
        }
        case REC_DEPENDENT_RULE: {
          const PClause& pc = r.prog.clauses[rc.clause];
          std::string ctx = r.prog.ctx[pc.d];
          std::string rule = r.prog.ctx[pc.f];
          J check = J::obj(); check.add("UnResolvedContext", J::str(rule));
          J un = J::obj();
          un.add("messages", R::messages(J::str(r.custom(pc)),
                                         J::str("Check was not compliant as dependent rule [" + rule + "] did not PASS. Context [" + ctx + "]")));
          un.add("context", J::str(ctx));
          un.add("check", std::move(check));
          // field order: UnaryReport = check, context, messages
          J ordered = J::obj();
          ordered.add("check", un.o[2].second);
          ordered.add("context", un.o[1].second);
          ordered.add("messages", un.o[0].second);
          list.push(clause_wrap("Clause", clause_wrap("Unary", std::move(ordered))));
          break;
        }
        case REC_CMP: {
          // clause == NONE: a map-key-filter comparison (real_binary_operation, eval.rs:976-1075):
          // context "", no custom message, comparison carried in rc.y
          bool mk = rc.clause == NONE;
          const PClause* pcp = mk ? nullptr : &r.prog.clauses[rc.clause];
          uint32_t op = mk ? (rc.y & 15u) : (pcp->flags & 15u);
          bool neg = mk ? ((rc.y >> 4) & 1u) : ((pcp->flags >> 4) & 1u);
          std::string ctx = mk ? std::string() : r.prog.ctx[pcp->d];
          std::string cust = mk ? std::string() : r.custom(*pcp);
          std::string errm;
          if (rc.x) errm = " Error = [" + r.nc_reason(rc) + "]";
          J bin = J::obj();
          bin.add("context", J::str(ctx));
          if ((rc.from.meta & 3u) == QR_UNRESOLVED) {
            std::string msg = "Check was not compliant as property [" + r.remaining(rc.from) +
                              "] to compare from is missing. Value traversed to [" + r.unresolved_display(rc.from) + "]." + errm;
            bin.add("messages", R::messages(J::str(cust), J::str(msg), r.q_loc(rc.from)));
            J u = J::obj(); u.add("value", r.unresolved_json(rc.from)); u.add("comparison", r.comparison(op, neg));
            J check = J::obj(); check.add("UnResolved", std::move(u));
            bin.add("check", std::move(check));
          } else {
            if (rc.to.meta == 0xFFFFFFFFu) break;   // `to` absent: nothing reported (eval_context.rs:2283)
            if ((rc.to.meta & 3u) == QR_UNRESOLVED) {
              std::string msg = "Check was not compliant as property [" + r.remaining(rc.to) +
                                "] to compare to is missing. Value traversed to [" + r.unresolved_display(rc.to) + "]." + errm;
              bin.add("messages", R::messages(J::str(cust), J::str(msg), r.q_loc(rc.to)));
              J u = J::obj(); u.add("value", r.unresolved_json(rc.to)); u.add("comparison", r.comparison(op, neg));
              J check = J::obj(); check.add("UnResolved", std::move(u));
              bin.add("check", std::move(check));
            } else {
              std::string msg = "Check was not compliant as property value [" + r.pav_display(rc.from) + "] " + op_msg(op, neg) +
                                " value [" + r.pav_display(rc.to) + "]." + errm;
              bin.add("messages", R::messages(J::str(cust), J::str(msg), r.q_loc(rc.to)));
              J rr = J::obj(); rr.add("from", r.pav_json(rc.from)); rr.add("to", r.pav_json(rc.to)); rr.add("comparison", r.comparison(op, neg));
              J check = J::obj(); check.add("Resolved", std::move(rr));
              bin.add("check", std::move(check));
            }
          }
          list.push(clause_wrap("Clause", clause_wrap("Binary", std::move(bin))));
          break;
        }
        case REC_IN: {
          bool mk = rc.clause == NONE;
          const PClause* pcp = mk ? nullptr : &r.prog.clauses[rc.clause];
          uint32_t op = mk ? (rc.y & 15u) : (pcp->flags & 15u);
          bool neg = mk ? ((rc.y >> 4) & 1u) : ((pcp->flags >> 4) & 1u);
          std::vector<QR> to;
          uint32_t n = rc.x;
          while (to.size() < n && i < recs.size() && recs[i].kind == REC_LIST) {
            to.push_back(recs[i].from);
            if (to.size() < n) to.push_back(recs[i].to);
            i++;
          }
          std::string sd;
          for (size_t k = 0; k < to.size(); k++) {
            std::string item = (to[k].meta & 3u) == QR_UNRESOLVED ? "(unresolved, " + r.unresolved_display(to[k]) + ")"
                                                                  : "(resolved, " + r.pav_display(to[k]) + ")";
            sd = k ? sd + "." + item : item;
          }
          std::string fixed;
          for (size_t k = 0; k < sd.size(); k++) { if (sd[k] == '.' && k + 1 < sd.size() && sd[k + 1] == '[') continue; fixed.push_back(sd[k]); }
          std::string err = "Check was not compliant as property [" + r.q_path_display(rc.from) + "] was not present in [" + fixed + "]";
          J bin = J::obj();
          bin.add("context", J::str(mk ? std::string() : r.prog.ctx[pcp->d]));
          bin.add("messages", R::messages(mk ? J::null() : r.custom_opt(*pcp), J::str(err), r.q_loc(rc.from)));
          J inr = J::obj();
          inr.add("from", r.pav_json(rc.from));
          J arr = J::arr();
          for (auto& t : to) if ((t.meta & 3u) != QR_UNRESOLVED) arr.push(r.pav_json(t));
          inr.add("to", std::move(arr));
          inr.add("comparison", r.comparison(op, neg));
          J check = J::obj(); check.add("InResolved", std::move(inr));
          bin.add("check", std::move(check));
          list.push(clause_wrap("Clause", clause_wrap("Binary", std::move(bin))));
          break;
        }
        default:
          break;
      }
    }
    return list;
  }
};

// ---- streaming JSON ------------------------------------------------------------------------------
// The FileReport JSON written straight into the output, byte-identical to building the J tree and
// pretty() printing it (serde_json's PrettyFormatter: 2-space indent, "[]" / "{}" when empty), without
// the tree: no per-value allocations, one pass.  Used for the JSON format (validate batches and the
// FFI's non-verbose run_checks); YAML / SARIF / JUnit still read the tree.
struct JW {
  TextBuf& out;
  struct Level { int indent; bool first; };
  std::vector<Level> st;
  int base;
  JW(TextBuf& o, int indent) : out(o), base(indent) {}
  int cur() const { return st.empty() ? base : st.back().indent + 1; }
  void open(char c) { out += c; st.push_back(Level{cur(), true}); }
  void close(char c) {
    const Level L = st.back();
    st.pop_back();
    if (!L.first) { out += '\n'; out.append(L.indent * 2, ' '); }
    out += c;
  }
  void item() {   // element / member prefix inside the innermost container
    Level& L = st.back();
    if (L.first) out.push_back('\n'); else out.append(",\n", 2);
    L.first = false;
    out.append((L.indent + 1) * 2, ' ');
  }
  void key(const char* k) { item(); out += '"'; out += k; out += "\": "; }
  void key(const std::string& k) { item(); json_escape_into(out, k.data(), k.size()); out += ": "; }
  void str(const std::string& v) { json_escape_into(out, v.data(), v.size()); }
  void str(const char* v) { json_escape_into(out, v, strlen(v)); }
  void raw(const std::string& v) { out += v; }
  void null() { out += "null"; }
  void boolean(bool b) { out += b ? "true" : "false"; }
  void obj() { open('{'); }
  void end_obj() { close('}'); }
  void arr() { open('['); }
  void end_arr() { close(']'); }
  void cmp(uint32_t op, bool neg) {
    arr();
    item(); out += '"'; out += CMP_NAMES[op]; out += '"';
    item(); boolean(neg);
    end_arr();
  }
};

// R::value_json / pav_json / unresolved_json, streamed
void write_value(const R& r, JW& w, uint32_t ref) {
  const DNode& n = r.N(ref);
  switch (n.kind) {
    case K_NULL: w.null(); return;
    case K_STRING: { const DocBatch& B = r.B(ref); json_escape_into(w.out, B.bytes.data() + n.a, n.count); return; }
    case K_REGEX: w.str("/" + r.str(ref) + "/"); return;
    case K_BOOL: w.boolean(n.a != 0); return;
    case K_INT: w.raw(std::to_string(r.ival(n))); return;
    case K_FLOAT: {
      double d = r.fval(n);
      if (std::isnan(d) || std::isinf(d))
        throw Fatal{"IncompatibleError", "Could not convert float " + rust_display_f64(d) + " to serde::Value::Number"};
      w.raw(ryu_f64(d));
      return;
    }
    case K_CHAR: { std::string s; utf8_append(s, n.a); w.str(s); return; }
    case K_LIST:
      w.arr();
      for (uint32_t j = 0; j < n.count; j++) { w.item(); write_value(r, w, r.child(ref, j)); }
      w.end_arr();
      return;
    case K_MAP:
      w.obj();
      for (uint32_t j = 0; j < n.count; j++) {
        const uint32_t c = r.child(ref, j);
        const DNode& cn = r.N(c);
        const DocBatch& B = r.B(c);
        w.item(); json_escape_into(w.out, B.bytes.data() + cn.key_off, cn.key_len); w.out += ": ";
        write_value(r, w, c);
      }
      w.end_obj();
      return;
    default: w.str(r.range_str(n)); return;
  }
}
void write_pav(const R& r, JW& w, const QR& q) {
  w.obj();
  w.key("path"); w.str(r.q_path(q));
  w.key("value");
  if (r.is_synth(q)) w.raw(std::to_string(r.synth_val(q)));
  else write_value(r, w, q.node);
  w.end_obj();
}
void write_unresolved(const R& r, JW& w, const QR& q) {
  w.obj();
  w.key("traversed_to");
  w.obj();
  w.key("path"); w.str(r.path(q.node));
  w.key("value"); write_value(r, w, q.node);
  w.end_obj();
  w.key("remaining_query"); w.str(r.remaining(q));
  w.key("reason"); w.str(r.reason(q));
  w.end_obj();
}
void write_messages(JW& w, const std::string* custom, const std::string* error) {
  w.obj();
  w.key("custom_message"); if (custom) w.str(*custom); else w.null();
  w.key("error_message"); if (error) w.str(*error); else w.null();
  w.end_obj();
}

// Walker::items, streamed: writes the ClauseReports of records [i, close) into the open array
struct StreamWalker {
  const R& r;
  const RecSpan& recs;
  JW& w;
  size_t i = 0;

  void items(uint32_t close_kind) {
    while (i < recs.size()) {
      const Rec& rc = recs[i];
      if (rc.kind == close_kind) { i++; return; }
      i++;
      switch (rc.kind) {
        case REC_RULE_OPEN: {
          w.item(); w.obj(); w.key("Rule"); w.obj();
          w.key("name"); w.str(r.prog.rule_names[rc.clause]);
          w.key("metadata"); w.obj(); w.end_obj();
          w.key("messages"); write_messages(w, rc.x == NONE ? nullptr : &r.prog.msgs[rc.x], nullptr);
          w.key("checks"); w.arr();
          items(REC_RULE_CLOSE);
          w.end_arr();
          w.end_obj(); w.end_obj();
          break;
        }
        case REC_DISJ_OPEN: {
          w.item(); w.obj(); w.key("Disjunctions"); w.obj();
          w.key("checks"); w.arr();
          items(REC_DISJ_CLOSE);
          w.end_arr();
          w.end_obj(); w.end_obj();
          break;
        }
        case REC_BLOCK_EMPTY: {
          const PClause& pc = r.prog.clauses[rc.clause];
          static const std::string msg = "query for block clause did not retrieve any value";
          w.item(); w.obj(); w.key("Block"); w.obj();
          w.key("context"); w.str(r.prog.ctx[pc.d]);
          w.key("messages"); write_messages(w, nullptr, &msg);
          w.key("unresolved"); w.null();
          w.end_obj(); w.end_obj();
          break;
        }
        case REC_MISSING_BLOCK_VALUE: {
          const PClause& pc = r.prog.clauses[rc.clause];
          const std::string err = "Check was not compliant as property [" + r.remaining(rc.from) + "] is missing. Value traversed to [" +
                                  r.unresolved_display(rc.from) + "]";
          static const std::string empty;
          w.item(); w.obj(); w.key("Block"); w.obj();
          w.key("context"); w.str(r.prog.ctx[pc.f]);
          w.key("messages"); write_messages(w, &empty, &err);
          w.key("unresolved"); write_unresolved(r, w, rc.from);
          w.end_obj(); w.end_obj();
          break;
        }
        case REC_UNARY: {
          const PClause& pc = r.prog.clauses[rc.clause];
          const uint32_t op = pc.flags & 15u;
          const bool neg = (pc.flags >> 4) & 1u;
          const bool unres = (rc.from.meta & 3u) == QR_UNRESOLVED;
          const std::string msg = unres ? "Check was not compliant as property [" + r.remaining(rc.from) + "] is missing. Value traversed to [" +
                                              r.unresolved_display(rc.from) + "]."
                                        : "Check was not compliant as property [" + r.q_path_display(rc.from) + "] " + unary_msg(op, neg) + ".";
          const std::string cm = r.custom(pc);
          w.item(); w.obj(); w.key("Clause"); w.obj(); w.key("Unary"); w.obj();
          w.key("check"); w.obj(); w.key(unres ? "UnResolved" : "Resolved"); w.obj();
          w.key("value"); if (unres) write_unresolved(r, w, rc.from); else write_pav(r, w, rc.from);
          w.key("comparison"); w.cmp(op, neg);
          w.end_obj(); w.end_obj();
          w.key("context"); w.str(r.prog.ctx[pc.d]);
          w.key("messages"); write_messages(w, &cm, &msg);
          w.end_obj(); w.end_obj(); w.end_obj();
          break;
        }
        case REC_NOVALUE_EMPTY: {
          const PClause& pc = r.prog.clauses[rc.clause];
          const std::string& ctx = r.prog.ctx[pc.d];
          std::string cm = r.custom(pc);
          for (auto& ch : cm) if (ch == '\n') ch = ';';
          const std::string msg = "Check was not compliant as variable in context [" + ctx + "] was not empty";
          w.item(); w.obj(); w.key("Clause"); w.obj(); w.key("Unary"); w.obj();
          w.key("check"); w.obj(); w.key("UnResolvedContext"); w.str(ctx); w.end_obj();
          w.key("context"); w.str(ctx);
          w.key("messages"); write_messages(w, &cm, &msg);
          w.end_obj(); w.end_obj(); w.end_obj();
          break;
        }
        case REC_DEPENDENT_RULE: {
          const PClause& pc = r.prog.clauses[rc.clause];
          const std::string& ctx = r.prog.ctx[pc.d];
          const std::string& rule = r.prog.ctx[pc.f];
          const std::string cm = r.custom(pc);
          const std::string msg = "Check was not compliant as dependent rule [" + rule + "] did not PASS. Context [" + ctx + "]";
          w.item(); w.obj(); w.key("Clause"); w.obj(); w.key("Unary"); w.obj();
          w.key("check"); w.obj(); w.key("UnResolvedContext"); w.str(rule); w.end_obj();
          w.key("context"); w.str(ctx);
          w.key("messages"); write_messages(w, &cm, &msg);
          w.end_obj(); w.end_obj(); w.end_obj();
          break;
        }
        case REC_CMP: {
          const bool mk = rc.clause == NONE;
          const PClause* pcp = mk ? nullptr : &r.prog.clauses[rc.clause];
          const uint32_t op = mk ? (rc.y & 15u) : (pcp->flags & 15u);
          const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pcp->flags >> 4) & 1u);
          const bool from_unres = (rc.from.meta & 3u) == QR_UNRESOLVED;
          if (!from_unres && rc.to.meta == 0xFFFFFFFFu) break;   // `to` absent: nothing reported (eval_context.rs:2283)
          const std::string cust = mk ? std::string() : r.custom(*pcp);
          const std::string errm = rc.x ? " Error = [" + r.nc_reason(rc) + "]" : std::string();
          w.item(); w.obj(); w.key("Clause"); w.obj(); w.key("Binary"); w.obj();
          w.key("context"); w.str(mk ? std::string() : r.prog.ctx[pcp->d]);
          if (from_unres) {
            const std::string msg = "Check was not compliant as property [" + r.remaining(rc.from) +
                                    "] to compare from is missing. Value traversed to [" + r.unresolved_display(rc.from) + "]." + errm;
            w.key("messages"); write_messages(w, &cust, &msg);
            w.key("check"); w.obj(); w.key("UnResolved"); w.obj();
            w.key("value"); write_unresolved(r, w, rc.from);
            w.key("comparison"); w.cmp(op, neg);
            w.end_obj(); w.end_obj();
          } else if ((rc.to.meta & 3u) == QR_UNRESOLVED) {
            const std::string msg = "Check was not compliant as property [" + r.remaining(rc.to) +
                                    "] to compare to is missing. Value traversed to [" + r.unresolved_display(rc.to) + "]." + errm;
            w.key("messages"); write_messages(w, &cust, &msg);
            w.key("check"); w.obj(); w.key("UnResolved"); w.obj();
            w.key("value"); write_unresolved(r, w, rc.to);
            w.key("comparison"); w.cmp(op, neg);
            w.end_obj(); w.end_obj();
          } else {
            const std::string msg = "Check was not compliant as property value [" + r.pav_display(rc.from) + "] " + op_msg(op, neg) +
                                    " value [" + r.pav_display(rc.to) + "]." + errm;
            w.key("messages"); write_messages(w, &cust, &msg);
            w.key("check"); w.obj(); w.key("Resolved"); w.obj();
            w.key("from"); write_pav(r, w, rc.from);
            w.key("to"); write_pav(r, w, rc.to);
            w.key("comparison"); w.cmp(op, neg);
            w.end_obj(); w.end_obj();
          }
          w.end_obj(); w.end_obj(); w.end_obj();
          break;
        }
        case REC_IN: {
          const bool mk = rc.clause == NONE;
          const PClause* pcp = mk ? nullptr : &r.prog.clauses[rc.clause];
          const uint32_t op = mk ? (rc.y & 15u) : (pcp->flags & 15u);
          const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pcp->flags >> 4) & 1u);
          std::vector<QR> to;
          const uint32_t n = rc.x;
          while (to.size() < n && i < recs.size() && recs[i].kind == REC_LIST) {
            to.push_back(recs[i].from);
            if (to.size() < n) to.push_back(recs[i].to);
            i++;
          }
          std::string sd;
          for (size_t k = 0; k < to.size(); k++) {
            std::string item = (to[k].meta & 3u) == QR_UNRESOLVED ? "(unresolved, " + r.unresolved_display(to[k]) + ")"
                                                                  : "(resolved, " + r.pav_display(to[k]) + ")";
            sd = k ? sd + "." + item : item;
          }
          std::string fixed;
          for (size_t k = 0; k < sd.size(); k++) { if (sd[k] == '.' && k + 1 < sd.size() && sd[k + 1] == '[') continue; fixed.push_back(sd[k]); }
          const std::string err = "Check was not compliant as property [" + r.q_path_display(rc.from) + "] was not present in [" + fixed + "]";
          const std::string* cm = (mk || pcp->e == NONE) ? nullptr : &r.prog.msgs[pcp->e];
          w.item(); w.obj(); w.key("Clause"); w.obj(); w.key("Binary"); w.obj();
          w.key("context"); w.str(mk ? std::string() : r.prog.ctx[pcp->d]);
          w.key("messages"); write_messages(w, cm, &err);
          w.key("check"); w.obj(); w.key("InResolved"); w.obj();
          w.key("from"); write_pav(r, w, rc.from);
          w.key("to"); w.arr();
          for (auto& t : to) if ((t.meta & 3u) != QR_UNRESOLVED) { w.item(); write_pav(r, w, t); }
          w.end_arr();
          w.key("comparison"); w.cmp(op, neg);
          w.end_obj(); w.end_obj();
          w.end_obj(); w.end_obj(); w.end_obj();
          break;
        }
        default:
          break;
      }
    }
  }
};

std::string status_str(uint32_t s) { return s == ST_PASS ? "PASS" : s == ST_FAIL ? "FAIL" : "SKIP"; }
uint32_t status_and(uint32_t a, uint32_t b) {
  if (a == ST_FAIL) return ST_FAIL;
  if (a == ST_PASS) return b == ST_FAIL ? ST_FAIL : ST_PASS;
  return b;
}

}  // namespace

std::string error_display(const std::string& kind, const std::string& msg) {
  if (kind == "ParseError") return "Parser Error when parsing `" + msg + "`";
  if (kind == "MissingValue") return "There was no variable or value object to resolve. Error = `" + msg + "`";
  if (kind == "IncompatibleError") return "Types or variable assignments are incompatible `" + msg + "`";
  if (kind == "NotComparable") return "Comparing incoming context with literals or dynamic results wasn't possible `" + msg + "`";
  if (kind == "YamlError") return "Error parsing incoming YAML context " + msg;
  if (kind == "JsonError") return "Error parsing incoming JSON context " + msg;
  // the rest of errors.rs:11-54's Display strings
  if (kind == "MultipleValues") return "Conflicting rule or variable assignments inside the same scope `" + msg + "`";
  if (kind == "MissingVariable") return "Variable assignment could not be resolved in rule file or incoming context `" + msg + "`";
  if (kind == "MissingProperty") return "Could not evaluate clause for a rule with missing property for incoming context `" + msg + "`";
  if (kind == "RetrievalError") return "Could not retrieve data from incoming context. Error = `" + msg + "`";
  if (kind == "IncompatibleRetrievalError") return "Types or variable assignments have incompatible types to retrieve `" + msg + "`";
  if (kind == "FileNotFoundError") return "The path `" + msg + "` does not exist";
  if (kind == "FormatError") return "Formatting error when writing " + msg;
  if (kind == "IoError") return "I/O error when reading " + msg;
  if (kind == "RegexError") return "Regex expression parse error for rules file " + msg;
  return msg;
}

void tile_error(const DocBatch& docs, uint32_t doc, const Program& prog, const TileOut& t, ReportError& err) {
  err.set = true;
  R r{docs, prog, docs.serde, docs.base.empty() ? 0 : docs.base[doc]};
  switch (t.err) {
    case E_EMPTY_INCOMPATIBLE:
      err.kind = "IncompatibleError";
      err.msg = std::string("Attempting EMPTY operation on type ") + type_info(t.err_b) + " that does not support it at " + r.path_display(t.err_a);
      break;
    case E_TYPEBLOCK_UNRESOLVED:
      err.kind = "MissingValue";
      err.msg = "Unable to resolve type block query: " + prog.ctx[prog.clauses[t.err_a].f];
      break;
    case E_VAR_MISSING:
      err.kind = "MissingValue";
      err.msg = "Could not resolve variable by name " + prog.var_names[t.err_a] + " across scopes";
      break;
    case E_RULE_MISSING: {
      err.kind = "MissingValue";
      std::string names;
      for (size_t i = 0; i < prog.slot_names.size(); i++) { if (i) names += ", "; names += rust_debug_str(prog.slot_names[i]); }
      err.msg = "Rule " + prog.ctx[prog.clauses[t.err_a].f] + " by that name does not exist, Rule Names = [" + names + "]";
      break;
    }
    case E_PARAM_MISSING: {
      err.kind = "MissingValue";
      std::string names;
      for (size_t i = 0; i < prog.param_rule_names.size(); i++) { if (i) names += ", "; names += rust_debug_str(prog.param_rule_names[i]); }
      err.msg = "Parameterized Rule with name " + prog.ctx[prog.clauses[t.err_a].f] + " was not found, candidate [" + names + "]";
      break;
    }
    case E_PARAM_ARITY:
      err.kind = "IncompatibleError";
      err.msg = "Arity mismatch for called parameter rule " + prog.ctx[prog.clauses[t.err_a].f] + ", expected " +
                std::to_string(t.err_b) + ", got " + std::to_string(prog.clauses[t.err_a].c);
      break;
    case E_INTERP_NON_STRING:   // eval_context.rs:497-518: Debug of key.self_value()
      err.kind = "NotComparable";
      err.msg = "Variable projections inside Query " + slice_display(prog.queries[t.err_b], 0) +
                ", is returning a non-string value for key " + type_info(r.N(t.err_a).kind) + ", (" +
                r.dbg_path(r.path(t.err_a), r.line(t.err_a), r.col(t.err_a)) + ", " + r.debug(t.err_a) + ")";
      break;
    case E_INTERP_QUERY: {      // eval_context.rs:436-443 (the reference displays query[1])
      err.kind = "IncompatibleError";
      const auto& parts = prog.queries[t.err_a];
      std::vector<QueryPart> one(parts.begin() + (parts.size() > 1 ? 1 : 0), parts.begin() + (parts.size() > 1 ? 2 : parts.size()));
      err.msg = "This type of query " + slice_display(one, 0) + " based variable interpolation is not supported map, " +
                slice_display(parts, 0);
      break;
    }
    case E_REGEX_UNSUPPORTED:
      err.kind = "Unsupported";
      err.msg = "unsupported on MI355X path: regex /" + prog.regex_src[t.err_a] + "/ (" + prog.regex[t.err_a].why + ")";
      break;
    case E_HEAP: err.kind = "Unsupported"; err.msg = "MI355X path: per-tile scratch heap exhausted"; break;
    case E_RECORDS: err.kind = "Unsupported"; err.msg = "MI355X path: failure-record buffer exhausted"; break;
    case E_DEPTH: err.kind = "Unsupported"; err.msg = "MI355X path: evaluation depth limit exceeded"; break;
    case E_STACK:
      err.kind = "Unsupported";
      err.msg = "MI355X path: evaluation depth limit exceeded (rules nest deeper than the device lane stack)";
      break;
    default: {
      if (t.err_a == 2) {
        // a filter on a map after a step other than `*`, `[*]` or a key (e.g. `x[0][ ... ]`): the
        // reference's `_ => unreachable!()` (eval_context.rs:752), a panic -- ffi-support's code -1
        // with the panic payload as the message
        err.kind = "Panic";
        err.msg = "internal error: entered unreachable code";
        break;
      }
      static const char* why[] = {"", "variable captures", "filter after this query part", "(unused)",
                                  "join index out of bounds report", "unresolved join keys report", "map key filters (KEYS)",
                                  "functions other than count()", "clause kind"};
      err.kind = "Unsupported";
      err.msg = std::string("unsupported on MI355X path: ") + (t.err_a < 9 ? std::string(why[t.err_a]) : "construct #" + std::to_string(t.err_a) + "/" + std::to_string(t.err_b));
    }
  }
}

namespace {

// FileReport for one data file over every program (CommonStructuredReporter::report,
// structured.rs:99-133); per_file[f] receives program f's not_compliant items when non-null
bool build_file_report(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                       const std::vector<const TileResult*>& tiles, J& fr, std::vector<J>* per_file, ReportError& err) {
  try {
    uint32_t status = ST_SKIP;
    J not_compliant = J::arr();
    std::set<std::string> pass, skip;
    for (size_t f = 0; f < progs.size(); f++) {
      const Program& P = *progs[f];
      const TileResult& T = *tiles[f];
      if (T.out.err) { tile_error(docs, doc, P, T.out, err); return false; }
      R r{docs, P, docs.serde, docs.base[doc], &T.aux};
      Walker w{r, T.recs};
      J items = w.items(0xFFFFFFFFu);
      if (per_file) per_file->push_back(items);
      for (auto& it : items.a) not_compliant.push(std::move(it));
      status = status_and(status, T.out.status);
      for (uint32_t k = 0; k < P.n_rules; k++) {
        const std::string& nm = P.rule_names[P.rule_names.size() - P.n_rules + k];
        if (T.rule_status[k] == ST_PASS) pass.insert(nm);
        else if (T.rule_status[k] == ST_SKIP) skip.insert(nm);
      }
    }
    fr = J::obj();
    fr.add("name", J::str(docs.names[doc]));
    fr.add("metadata", J::obj());
    fr.add("status", J::str(status_str(status)));
    fr.add("not_compliant", std::move(not_compliant));
    J na = J::arr(); for (auto& s : skip) na.push(J::str(s));
    J co = J::arr(); for (auto& s : pass) co.push(J::str(s));
    fr.add("not_applicable", std::move(na));
    fr.add("compliant", std::move(co));
    return true;
  } catch (Fatal& f) {
    err.set = true; err.kind = f.kind; err.msg = f.msg;
    return false;
  }
}

// build_file_report, streamed (JSON): the same object, written as it is walked
bool write_file_report(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                       const std::vector<const TileResult*>& tiles, int indent, TextBuf& out, ReportError& err) {
  const size_t mark = out.size();
  try {
    uint32_t status = ST_SKIP;
    std::set<std::string> pass, skip;
    for (size_t f = 0; f < progs.size(); f++) {
      const Program& P = *progs[f];
      const TileResult& T = *tiles[f];
      if (T.out.err) continue;   // reported in file order below
      status = status_and(status, T.out.status);
      for (uint32_t k = 0; k < P.n_rules; k++) {
        const std::string& nm = P.rule_names[P.rule_names.size() - P.n_rules + k];
        if (T.rule_status[k] == ST_PASS) pass.insert(nm);
        else if (T.rule_status[k] == ST_SKIP) skip.insert(nm);
      }
    }
    JW w(out, indent);
    w.obj();
    w.key("name"); w.str(docs.names[doc]);
    w.key("metadata"); w.obj(); w.end_obj();
    w.key("status"); w.str(status_str(status));
    w.key("not_compliant"); w.arr();
    for (size_t f = 0; f < progs.size(); f++) {
      const TileResult& T = *tiles[f];
      // an earlier file's abort (a value serde cannot write) wins over this tile's error, as in
      // build_file_report's file-order walk
      if (T.out.err) { out.resize(mark); tile_error(docs, doc, *progs[f], T.out, err); return false; }
      R r{docs, *progs[f], docs.serde, docs.base[doc], &T.aux};
      StreamWalker sw{r, T.recs, w};
      sw.items(0xFFFFFFFFu);
    }
    w.end_arr();
    w.key("not_applicable"); w.arr();
    for (auto& x : skip) { w.item(); w.str(x); }
    w.end_arr();
    w.key("compliant"); w.arr();
    for (auto& x : pass) { w.item(); w.str(x); }
    w.end_arr();
    w.end_obj();
    return true;
  } catch (Fatal& f) {
    out.resize(mark);
    err.set = true; err.kind = f.kind; err.msg = f.msg;
    return false;
  }
}

}  // namespace

bool report_json_doc(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                     const std::vector<const TileResult*>& tiles, TextBuf& out, ReportError& err) {
  return write_file_report(docs, doc, progs, tiles, 1, out, err);
}

namespace {

const J* field(const J& o, const char* k) {
  for (auto& kv : o.o) if (kv.first == k) return &kv.second;
  return nullptr;
}

// ClauseReport::get_message (eval_context.rs:1808-1826)
void get_messages(const J& clause, std::vector<const J*>& out) {
  const std::string& kind = clause.o[0].first;
  const J& body = clause.o[0].second;
  if (kind == "Rule" || kind == "Disjunctions") {
    for (auto& ch : field(body, "checks")->a) get_messages(ch, out);
  } else if (kind == "Block") {
    out.push_back(field(body, "messages"));
  } else {
    out.push_back(field(body.o[0].second, "messages"));
  }
}

// ---- YAML: serde_yaml 0.9 over unsafe-libyaml (libyaml 0.2.5), width unlimited, unicode on.
// serde_yaml picks the scalar style of a string: literal when it holds a newline, single-quoted
// when its plain form would resolve to null / bool / int / float (de.rs visit_untagged_scalar),
// otherwise the emitter's choice.
bool yaml_resolves_to_non_string(const std::string& v) {
  if (v.empty() || v == "~" || v == "null" || v == "Null" || v == "NULL") return true;
  if (v == "true" || v == "True" || v == "TRUE" || v == "false" || v == "False" || v == "FALSE") return true;
  if (v.size() >= 2 && v[0] == '+' && (v[1] == '+' || v[1] == '-')) return false;
  auto all = [](const std::string& s, size_t from, const char* set) {
    if (from >= s.size()) return false;
    for (size_t i = from; i < s.size(); i++) if (!strchr(set, s[i])) return false;
    return true;
  };
  // radix-prefixed integers (parse_unsigned_int / parse_negative_int)
  size_t o = (v[0] == '+' || v[0] == '-') ? 1 : 0;
  if (v.size() > o + 2 && v[o] == '0') {
    const char c = v[o + 1];
    if (c == 'x' && all(v, o + 2, "0123456789abcdefABCDEF")) return true;
    if (c == 'o' && all(v, o + 2, "01234567")) return true;
    if (c == 'b' && all(v, o + 2, "01")) return true;
  }
  // .inf / .nan spellings (parse_f64)
  const std::string u = v.substr(v[0] == '+' || v[0] == '-' ? 1 : 0);
  if (u == ".inf" || u == ".Inf" || u == ".INF") return true;
  if (v == ".nan" || v == ".NaN" || v == ".NAN") return true;
  // Rust f64 grammar, finite values: [+-]?(digits(.digits?)?|.digits)([eE][+-]?digits)?
  size_t i = o, n = v.size(), d1 = 0, d2 = 0;
  while (i < n && isdigit((unsigned char)v[i])) { i++; d1++; }
  if (i < n && v[i] == '.') { i++; while (i < n && isdigit((unsigned char)v[i])) { i++; d2++; } }
  if (d1 + d2 == 0) return false;
  if (i < n && (v[i] == 'e' || v[i] == 'E')) {
    i++;
    if (i < n && (v[i] == '+' || v[i] == '-')) i++;
    size_t de = 0;
    while (i < n && isdigit((unsigned char)v[i])) { i++; de++; }
    if (!de) return false;
  }
  if (i != n) return false;
  return std::isfinite(strtod(v.c_str(), nullptr));
}

int yaml_write_handler(void* data, unsigned char* buffer, size_t size) {
  static_cast<std::string*>(data)->append((const char*)buffer, size);
  return 1;
}

struct YamlOut {
  yaml_emitter_t em;
  std::string buf;
  bool ok = true;
  YamlOut() {
    yaml_emitter_initialize(&em);
    yaml_emitter_set_output(&em, yaml_write_handler, &buf);
    yaml_emitter_set_width(&em, -1);
    yaml_emitter_set_unicode(&em, 1);
  }
  ~YamlOut() { yaml_emitter_delete(&em); }
  // one whole YAML stream holding `j` (serde_yaml::to_writer of one value)
  void document(const J& j) {
    yaml_event_t ev;
    yaml_stream_start_event_initialize(&ev, YAML_UTF8_ENCODING); emit(ev);
    yaml_document_start_event_initialize(&ev, nullptr, nullptr, nullptr, 1); emit(ev);
    value(j);
    yaml_document_end_event_initialize(&ev, 1); emit(ev);
    yaml_stream_end_event_initialize(&ev); emit(ev);
    yaml_emitter_flush(&em);
  }
  void emit(yaml_event_t& ev) { if (ok && !yaml_emitter_emit(&em, &ev)) ok = false; }
  void scalar(const std::string& v, yaml_scalar_style_t style) {
    yaml_event_t ev;
    yaml_scalar_event_initialize(&ev, nullptr, nullptr, (yaml_char_t*)v.data(), (int)v.size(), 1, 1, style);
    emit(ev);
  }
  void str(const std::string& v) {
    yaml_scalar_style_t st = YAML_ANY_SCALAR_STYLE;
    if (v.find('\n') != std::string::npos) st = YAML_LITERAL_SCALAR_STYLE;
    else if (yaml_resolves_to_non_string(v)) st = YAML_SINGLE_QUOTED_SCALAR_STYLE;
    scalar(v, st);
  }
  void value(const J& j) {
    yaml_event_t ev;
    switch (j.t) {
      case J::Null: scalar("null", YAML_ANY_SCALAR_STYLE); return;
      case J::Bool: scalar(j.b ? "true" : "false", YAML_ANY_SCALAR_STYLE); return;
      case J::Raw: scalar(j.s, YAML_ANY_SCALAR_STYLE); return;
      case J::Str: str(j.s); return;
      case J::Cmp:
        yaml_sequence_start_event_initialize(&ev, nullptr, nullptr, 1, YAML_BLOCK_SEQUENCE_STYLE);
        emit(ev);
        str(CMP_NAMES[j.op]);
        scalar(j.b ? "true" : "false", YAML_ANY_SCALAR_STYLE);
        yaml_sequence_end_event_initialize(&ev);
        emit(ev);
        return;
      case J::Arr:
        yaml_sequence_start_event_initialize(&ev, nullptr, nullptr, 1, YAML_BLOCK_SEQUENCE_STYLE);
        emit(ev);
        for (auto& x : j.a) value(x);
        yaml_sequence_end_event_initialize(&ev);
        emit(ev);
        return;
      case J::Obj:
        yaml_mapping_start_event_initialize(&ev, nullptr, nullptr, 1, YAML_BLOCK_MAPPING_STYLE);
        emit(ev);
        for (auto& kv : j.o) { str(kv.first); value(kv.second); }
        yaml_mapping_end_event_initialize(&ev);
        emit(ev);
        return;
    }
  }
};

// ---- JUnit: quick_xml writer, indent 4 (reporters/mod.rs:66-420)
std::string xml_escape(const std::string& s) {
  std::string o;
  for (char ch : s) {
    switch (ch) {
      case '&': o += "&amp;"; break;
      case '<': o += "&lt;"; break;
      case '>': o += "&gt;"; break;
      case '\'': o += "&apos;"; break;
      case '"': o += "&quot;"; break;
      default: o.push_back(ch);
    }
  }
  return o;
}

const char* kSarifDescription =
    "AWS CloudFormation Guard is an open-source general-purpose policy-as-code evaluation tool. It provides developers "
    "with a simple-to-use, yet powerful and expressive domain-specific language (DSL) to define policies and enables "
    "developers to validate JSON- or YAML- formatted structured data with those policies.";

std::string sanitize_path(const std::string& p) { return !p.empty() && p[0] == '/' ? p.substr(1) : p; }

// SarifResults::from (sarif.rs:127-160) of one FAILed FileReport: one result per message of every
// not_compliant ClauseReport, in order
void sarif_results(const J& fr, const std::string& name, J& results) {
  for (auto& failure : field(fr, "not_compliant")->a) {
    std::string rule_id;
    if (failure.o[0].first == "Rule") {
      std::string rn = field(failure.o[0].second, "name")->s;
      rule_id = rn.substr(0, rn.find('.'));
      for (auto& ch : rule_id) ch = (char)toupper((unsigned char)ch);
    }
    std::vector<const J*> msgs;
    get_messages(failure, msgs);
    for (const J* m : msgs) {
      int64_t line = m->loc_line < 0 ? 0 : m->loc_line, col = m->loc_col < 0 ? 0 : m->loc_col;
      const J* em = field(*m, "error_message");
      const J* cm = field(*m, "custom_message");
      std::string text = (em->t == J::Str ? em->s : std::string()) + " " + (cm->t == J::Str ? cm->s : std::string());
      J res = J::obj();
      res.add("ruleId", J::str(rule_id));
      res.add("level", J::str("error"));
      J mt = J::obj(); mt.add("text", J::str(text));
      res.add("message", std::move(mt));
      J art = J::obj(); art.add("uri", J::str(sanitize_path(name)));
      J region = J::obj();
      region.add("startLine", J::raw(std::to_string(std::max<int64_t>(line, 1))));
      region.add("startColumn", J::raw(std::to_string(std::max<int64_t>(col, 1))));
      J phys = J::obj(); phys.add("artifactLocation", std::move(art)); phys.add("region", std::move(region));
      J l = J::obj(); l.add("physicalLocation", std::move(phys));
      J locs = J::arr(); locs.push(std::move(l));
      res.add("locations", std::move(locs));
      results.push(std::move(res));
    }
  }
}

// the SARIF report (SarifReport::new, sarif.rs:185-203) with these artifacts and results
J sarif_report(J artifacts, J results) {
  J drv = J::obj();
  drv.add("name", J::str("cfn-guard"));
  drv.add("semanticVersion", J::str("3.1.2"));
  drv.add("fullName", J::str("cfn-guard 3.1.2"));
  drv.add("organization", J::str("Amazon Web Services"));
  drv.add("downloadUri", J::str("https://github.com/aws-cloudformation/cloudformation-guard"));
  drv.add("informationUri", J::str("https://github.com/aws-cloudformation/cloudformation-guard"));
  J sd = J::obj(); sd.add("text", J::str(kSarifDescription));
  drv.add("shortDescription", std::move(sd));
  J tool = J::obj(); tool.add("driver", std::move(drv));
  J run = J::obj();
  run.add("tool", std::move(tool));
  run.add("artifacts", std::move(artifacts));
  run.add("results", std::move(results));
  J runs = J::arr(); runs.push(std::move(run));
  J rep = J::obj();
  rep.add("$schema", J::str("https://docs.oasis-open.org/sarif/sarif/v2.1.0/errata01/os/schemas/sarif-schema-2.1.0.json"));
  rep.add("version", J::str("2.1.0"));
  rep.add("runs", std::move(runs));
  return rep;
}

}  // namespace

bool sarif_doc_results(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                       const std::vector<const TileResult*>& tiles, std::string& out, ReportError& err) {
  J fr;
  if (!build_file_report(docs, doc, progs, tiles, fr, nullptr, err)) return false;
  if (field(fr, "status")->s != "FAIL") return true;
  J results = J::arr();
  sarif_results(fr, docs.names[doc], results);
  for (const J& r : results.a) {
    out += ",\n";
    out.append(8, ' ');
    pretty(r, 4, out);
  }
  return true;
}

void sarif_frame(const std::vector<std::string>& artifact_names, std::string& head, std::string& tail) {
  J artifacts = J::arr();
  for (const std::string& name : artifact_names) {
    J loc = J::obj(); loc.add("uri", J::str(sanitize_path(name)));
    J a = J::obj(); a.add("location", std::move(loc));
    artifacts.push(std::move(a));
  }
  std::string all;
  pretty(sarif_report(std::move(artifacts), J::arr()), 0, all);
  static const char kMark[] = "\"results\": []";
  const size_t at = all.rfind(kMark);
  head = all.substr(0, at + sizeof(kMark) - 2);   // ... "results": [
  tail = all.substr(at + sizeof(kMark) - 2);      // ]\n    }\n  ]\n}
}

struct ReportWriter::Impl {
  int32_t fmt;
  size_t ndocs = 0;
  std::string json;                       // OUT_JSON
  YamlOut* yaml = nullptr;                // OUT_YAML
  J artifacts = J::arr(), results = J::arr();   // OUT_SARIF
  std::set<std::string> seen;
  std::vector<std::string> art_names;     // raw names of `artifacts`, in order
  std::string suites;                     // OUT_JUNIT
  size_t tests = 0, failures = 0;
};

ReportWriter::ReportWriter(int32_t fmt) : p_(new Impl) {
  p_->fmt = fmt;
  if (fmt == OUT_YAML) {
    p_->yaml = new YamlOut();
    yaml_event_t ev;
    yaml_stream_start_event_initialize(&ev, YAML_UTF8_ENCODING);
    p_->yaml->emit(ev);
    yaml_document_start_event_initialize(&ev, nullptr, nullptr, nullptr, 1);
    p_->yaml->emit(ev);
    yaml_sequence_start_event_initialize(&ev, nullptr, nullptr, 1, YAML_BLOCK_SEQUENCE_STYLE);
    p_->yaml->emit(ev);
  }
}

ReportWriter::~ReportWriter() {
  delete p_->yaml;
  delete p_;
}

bool ReportWriter::add(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                       const std::vector<const TileResult*>& tiles, ReportError& err) {
  if (p_->fmt == OUT_JSON) {
    Impl& I = *p_;
    const size_t mark = I.json.size();
    I.json += I.ndocs == 0 ? "[\n" : ",\n";
    I.json.append(2, ' ');
    TextBuf t;
    if (!write_file_report(docs, doc, progs, tiles, 1, t, err)) { I.json.resize(mark); return false; }
    I.json.append(t.data(), t.size());
    I.ndocs++;
    return true;
  }
  J fr;
  std::vector<J> per_file;
  if (!build_file_report(docs, doc, progs, tiles, fr, p_->fmt == OUT_JUNIT ? &per_file : nullptr, err)) return false;
  Impl& I = *p_;
  I.ndocs++;
  switch (I.fmt) {
    case OUT_YAML:
      I.yaml->value(fr);
      break;
    case OUT_SARIF: {
      // SarifRun::from (sarif.rs:29-51): FAILed reports only
      if (field(fr, "status")->s != "FAIL") break;
      const std::string& name = docs.names[doc];
      if (!name.empty() && I.seen.insert(name).second) {
        J loc = J::obj(); loc.add("uri", J::str(sanitize_path(name)));
        J a = J::obj(); a.add("location", std::move(loc));
        I.artifacts.push(std::move(a));
        I.art_names.push_back(name);
      }
      sarif_results(fr, name, I.results);
      break;
    }
    case OUT_JUNIT: {
      // JunitReporter::report (xml.rs:14-80): one test suite per data file, one test case per rules file
      size_t nf = 0;
      std::string cases;
      for (size_t f = 0; f < progs.size(); f++) {
        const std::string rname = xml_escape(progs[f]->file_name);
        I.tests++;
        const uint32_t st = tiles[f]->out.status;
        if (st != ST_FAIL) {
          cases += "        <testcase name=\"" + rname + "\" time=\"0\" status=\"" + (st == ST_PASS ? "pass" : "skip") + "\"/>\n";
          continue;
        }
        nf++;
        // get_test_case (reporters/mod.rs:108-168): the last rule failure names the failure
        std::string fname;
        bool named = false;
        std::string texts;
        size_t ntexts = 0;
        for (auto& failure : per_file[f].a) {
          std::vector<const J*> msgs;
          get_messages(failure, msgs);
          for (const J* m : msgs) {
            if (failure.o[0].first == "Rule") {
              std::string rn = field(failure.o[0].second, "name")->s;
              size_t g = rn.find(".guard/");
              fname = g == std::string::npos ? rn : rn.substr(g + 7);
              named = true;
            }
            const J* cm = field(*m, "custom_message");
            const J* em = field(*m, "error_message");
            if (cm->t == J::Str) { texts += xml_escape(cm->s); ntexts++; }
            if (em->t == J::Str) { texts += xml_escape(em->s); ntexts++; }
          }
        }
        cases += "        <testcase name=\"" + rname + "\" time=\"0\">\n";
        std::string attr = named ? " message=\"" + xml_escape(fname) + "\"" : std::string();
        if (ntexts) cases += "            <failure" + attr + ">" + texts + "</failure>\n";
        else cases += "            <failure" + attr + "/>\n";
        cases += "        </testcase>\n";
      }
      I.failures += nf;
      I.suites += "    <testsuite name=\"" + xml_escape(docs.names[doc]) + "\" errors=\"0\" failures=\"" + std::to_string(nf) +
                  "\" time=\"0\">\n" + cases + "    </testsuite>\n";
      break;
    }
    default:
      I.json += I.ndocs == 1 ? "[\n" : ",\n";
      I.json.append(2, ' ');
      pretty(fr, 1, I.json);
      break;
  }
  return true;
}

void ReportWriter::absorb(ReportWriter& later) {
  Impl& I = *p_;
  Impl& L = *later.p_;
  if (I.fmt != L.fmt || I.fmt == OUT_YAML) throw std::runtime_error("ReportWriter::absorb: unsupported");
  switch (I.fmt) {
    case OUT_SARIF:
      for (size_t k = 0; k < L.art_names.size(); k++)
        if (I.seen.insert(L.art_names[k]).second) { I.artifacts.push(std::move(L.artifacts.a[k])); I.art_names.push_back(L.art_names[k]); }
      for (auto& r : L.results.a) I.results.push(std::move(r));
      break;
    case OUT_JUNIT:
      I.suites += L.suites;
      I.tests += L.tests;
      I.failures += L.failures;
      break;
    default:
      if (L.ndocs) {
        if (I.ndocs) { I.json += ",\n"; I.json.append(L.json, 2, std::string::npos); }
        else I.json = std::move(L.json);
      }
      break;
  }
  I.ndocs += L.ndocs;
  L.ndocs = 0;
}

bool report_batch_writers(const DocBatch& docs, const std::vector<const Program*>& progs, size_t first, size_t ndocs,
                          const std::function<TileResult(size_t doc, size_t file)>& tile, int32_t fmt, unsigned nthreads,
                          std::vector<std::unique_ptr<ReportWriter>>& writers, std::vector<std::string>& yaml_parts,
                          ReportError& err) {
  const size_t nf = progs.size();
  const size_t T = std::max<size_t>(1, std::min<size_t>(nthreads, (ndocs + 255) / 256));
  std::vector<std::unique_ptr<ReportWriter>> w(T);
  std::vector<ReportError> errs(T);
  std::vector<size_t> err_doc(T, SIZE_MAX);
  std::vector<std::string> yaml_out(T);
  auto work = [&](size_t t) {
    const size_t d0 = first + ndocs * t / T, d1 = first + ndocs * (t + 1) / T;
    w[t].reset(new ReportWriter(fmt));
    std::vector<TileResult> trs(nf);
    std::vector<const TileResult*> tp(nf);
    for (size_t d = d0; d < d1; d++) {
      for (size_t f = 0; f < nf; f++) { trs[f] = tile(d, f); tp[f] = &trs[f]; }
      if (!w[t]->add(docs, (uint32_t)d, progs, tp, errs[t])) { err_doc[t] = d; return; }
    }
    if (fmt == OUT_YAML && d1 > d0) yaml_out[t] = w[t]->finish();
  };
  parallel_run(T, work);
  // the first document (in order) whose report aborts decides the error (structured.rs:99-133)
  for (size_t t = 0; t < T; t++) if (err_doc[t] != SIZE_MAX) { err = errs[t]; return false; }
  if (fmt == OUT_YAML) {
    // a block sequence's items are emitted independently: the ranges' streams concatenate
    for (size_t t = 0; t < T; t++) if (first + ndocs * (t + 1) / T > first + ndocs * t / T) yaml_parts.push_back(std::move(yaml_out[t]));
    return true;
  }
  for (auto& x : w) writers.push_back(std::move(x));
  return true;
}

std::string report_writers_finish(int32_t fmt, std::vector<std::unique_ptr<ReportWriter>>& writers,
                                  std::vector<std::string>& yaml_parts) {
  if (fmt == OUT_YAML) {
    if (yaml_parts.empty()) return ReportWriter(fmt).finish();
    std::string out;
    size_t n = 0;
    for (auto& y : yaml_parts) n += y.size();
    out.reserve(n);
    for (auto& y : yaml_parts) out += y;
    return out;
  }
  if (writers.empty()) return ReportWriter(fmt).finish();
  for (size_t t = 1; t < writers.size(); t++) writers[0]->absorb(*writers[t]);
  return writers[0]->finish();
}

bool report_batch(const DocBatch& docs, const std::vector<const Program*>& progs, size_t first, size_t ndocs,
                  const std::function<TileResult(size_t doc, size_t file)>& tile, int32_t fmt, unsigned nthreads,
                  std::string& out, ReportError& err) {
  std::vector<std::unique_ptr<ReportWriter>> w;
  std::vector<std::string> yaml_parts;
  if (!report_batch_writers(docs, progs, first, ndocs, tile, fmt, nthreads, w, yaml_parts, err)) return false;
  out = report_writers_finish(fmt, w, yaml_parts);
  return true;
}

bool report_batch_json_parts(const DocBatch& docs, const std::vector<const Program*>& progs, size_t first, size_t ndocs,
                             const std::function<TileResult(size_t doc, size_t file)>& tile, unsigned nthreads,
                             std::vector<TextBuf>& parts, ReportError& err) {
  const size_t nf = progs.size();
  const size_t T = std::max<size_t>(1, std::min<size_t>(nthreads, (ndocs + 255) / 256));
  // the callers' part buffers are reused (a block loop keeps their pages: no fresh-memory faults)
  parts.resize(T);
  for (auto& p : parts) p.clear();
  std::vector<ReportError> errs(T);
  std::vector<size_t> err_doc(T, SIZE_MAX);
  auto work = [&](size_t t) {
    const size_t d0 = first + ndocs * t / T, d1 = first + ndocs * (t + 1) / T;
    std::vector<TileResult> trs(nf);
    std::vector<const TileResult*> tp(nf);
    // the part is written through a thread-local TextBuf and handed back at the end: the parts'
    // headers sit side by side in `parts`, and a length update per append on a shared cache line
    // made the writers slow each other down (16 threads ran at 2.4x one, tools/gpu_writer_scaling.sh)
    TextBuf o(std::move(parts[t]));
    struct Back { TextBuf& o; TextBuf& slot; ~Back() { slot = std::move(o); } } back{o, parts[t]};
    for (size_t d = d0; d < d1; d++) {
      for (size_t f = 0; f < nf; f++) { trs[f] = tile(d, f); tp[f] = &trs[f]; }
      if (d > d0) o += ",\n";
      o.append(2, ' ');
      if (!write_file_report(docs, (uint32_t)d, progs, tp, 1, o, errs[t])) { err_doc[t] = d; return; }
      // size the part once from its first documents: growing it by doubling copies it again and
      // again and faults its pages in twice
      if (d == d0 + 7 && d1 - d0 > 16) o.reserve(o.size() / 8 * (d1 - d0) / 8 * 9);
    }
  };
  parallel_run(T, work);
  for (size_t t = 0; t < T; t++) if (err_doc[t] != SIZE_MAX) { err = errs[t]; return false; }
  return true;
}

// parts may be empty (a thread with no documents): they contribute nothing
size_t json_parts_count(const std::vector<TextBuf>& parts) {
  size_t k = 0;
  for (auto& p : parts) if (!p.empty()) k++;
  return k;
}

size_t json_parts_size(const std::vector<TextBuf>& parts) {
  const size_t k = json_parts_count(parts);
  if (!k) return 2;   // "[]"
  size_t n = 4 + 2 * (k - 1);   // "[\n" ... "\n]", ",\n" between parts
  for (auto& p : parts) n += p.size();
  return n;
}

char* json_parts_join(const std::vector<TextBuf>& parts) {
  const size_t n = json_parts_size(parts);
  char* buf = (char*)malloc(n + 1);
  if (!buf) throw std::bad_alloc();
  std::vector<const TextBuf*> ne;
  for (auto& p : parts) if (!p.empty()) ne.push_back(&p);
  if (ne.empty()) { memcpy(buf, "[]", 3); return buf; }
  // a large result is one mmap'd chunk of its own: huge pages before the copy first-touches it
  if (n >= kHugeMin) {
    const uintptr_t a = ((uintptr_t)buf + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
    if (a < (uintptr_t)buf + n) madvise((void*)a, (uintptr_t)buf + n - a, MADV_HUGEPAGE);
  }
  std::vector<size_t> off(ne.size());
  size_t o = 2;
  for (size_t k = 0; k < ne.size(); k++) { off[k] = o; o += ne[k]->size() + 2; }
  memcpy(buf, "[\n", 2);
  // each part (and the separator after it) copied by its own thread: one pass over the output
  auto copy = [&](size_t k) {
    memcpy(buf + off[k], ne[k]->data(), ne[k]->size());
    memcpy(buf + off[k] + ne[k]->size(), k + 1 < ne.size() ? ",\n" : "\n]", 2);
  };
  parallel_run(ne.size(), copy);
  buf[n] = 0;
  return buf;
}

std::string ReportWriter::finish() {
  Impl& I = *p_;
  switch (I.fmt) {
    case OUT_YAML: {
      yaml_event_t ev;
      yaml_sequence_end_event_initialize(&ev);
      I.yaml->emit(ev);
      yaml_document_end_event_initialize(&ev, 1);
      I.yaml->emit(ev);
      yaml_stream_end_event_initialize(&ev);
      I.yaml->emit(ev);
      yaml_emitter_flush(&I.yaml->em);
      if (!I.yaml->ok) throw std::runtime_error("YAML emitter error");
      return I.yaml->buf;
    }
    case OUT_SARIF: {
      std::string out;
      pretty(sarif_report(std::move(I.artifacts), std::move(I.results)), 0, out);
      return out;
    }
    case OUT_JUNIT:
      return "<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<testsuites name=\"cfn-guard validate report\" tests=\"" +
             std::to_string(I.tests) + "\" failures=\"" + std::to_string(I.failures) + "\" errors=\"0\" time=\"0\">\n" + I.suites +
             "</testsuites>\n";
    default:
      if (!I.ndocs) return std::string("[]");
      I.json += "\n]";
      return std::move(I.json);
  }
}

std::string test_report(int32_t fmt, const std::string& rules_name, const std::vector<TestSpecFile>& files,
                        int32_t& exit_code) {
  static const char* kStatus[] = {"PASS", "FAIL", "SKIP"};
  exit_code = 0;   // SUCCESS_STATUS_CODE; 7 TEST_FAILURE_STATUS_CODE; 1 TEST_ERROR_STATUS_CODE
  auto statuses = [&](const std::vector<uint32_t>& v) {
    std::string o;
    for (size_t i = 0; i < v.size(); i++) o += (i ? ", " : "") + std::string(kStatus[v[i]]);
    return o;
  };
  if (fmt == OUT_TEXT) {
    // GenericReporter::report (reporters/test/generic.rs:23-63, 105-125)
    std::string out;
    size_t counter = 1;
    for (auto& f : files) {
      if (!f.error.empty()) { out += "Error processing " + f.error + "\n"; exit_code = 1; continue; }
      for (auto& tc : f.cases) {
        out += "Test Case #" + std::to_string(counter++) + "\n";
        if (tc.has_name) out += "Name: " + tc.name + "\n";
        std::vector<std::string> pass, failv;
        for (auto& r : tc.rules) {
          if (r.expected < 0) { out += "  No Test expectation was set for Rule " + r.rule + "\n"; continue; }
          std::string line = r.matched >= 0 ? r.rule + ": Expected = " + kStatus[r.matched]
                                            : r.rule + ": Expected = " + kStatus[r.expected] + ", Evaluated = [" + statuses(r.evaluated) + "]";
          auto& dst = r.matched >= 0 ? pass : failv;
          if (std::find(dst.begin(), dst.end(), line) == dst.end()) dst.push_back(line);   // IndexSet
        }
        out += tc.tree;   // --verbose (generic.rs:116-118): after the rules' lines, before the report
        if (!failv.empty()) { exit_code = 7; out += "  FAIL Rules:\n"; for (auto& l : failv) out += "    " + l + "\n"; }
        if (!pass.empty()) { out += "  PASS Rules:\n"; for (auto& l : pass) out += "    " + l + "\n"; }
        out += "\n";
      }
    }
    return out;
  }
  // StructuredTestReporter (reporters/test/structured.rs) + handle_structured_single_report (test.rs:326-380)
  TestResultIn one;
  one.rules_name = rules_name;
  one.files = files;
  return test_report_list(fmt, std::vector<TestResultIn>{one}, exit_code, true);
}

namespace {
// one TestResult (reporters/test/structured.rs:33-67): Ok {rule_file, test_cases} or Err {rule_file,
// error}; its exit code, its serde object and its JUnit suite (build_test_suite, :69-104)
J test_result(const TestResultIn& in, int32_t& code, std::string& suite, size_t& tests, size_t& failures, size_t& errors) {
  static const char* kStatus[] = {"PASS", "FAIL", "SKIP"};
  auto statuses = [&](const std::vector<uint32_t>& v) {
    std::string o;
    for (size_t i = 0; i < v.size(); i++) o += (i ? ", " : "") + std::string(kStatus[v[i]]);
    return o;
  };
  code = 0;
  const std::string rn = xml_escape(in.rules_name);
  std::string error = in.parse_error;
  if (error.empty())
    for (auto& f : in.files) if (!f.error.empty()) { error = f.error; break; }   // evaluate() returns at the first
  if (!error.empty()) {
    code = 1;
    suite = "    <testsuite name=\"" + rn + "\" errors=\"1\" failures=\"0\" time=\"0\">\n"
            "        <testcase name=\"" + rn + "\" time=\"0\" status=\"error\">\n            <error>" + xml_escape(error) +
            "</error>\n        </testcase>\n    </testsuite>\n";
    tests += 1; errors += 1;
    J e = J::obj(); e.add("rule_file", J::str(in.rules_name)); e.add("error", J::str(error));
    return e;
  }
  J cases = J::arr();
  std::string junit;
  size_t nfail = 0;
  for (auto& f : in.files) {
    for (auto& tc : f.cases) {
      J passed = J::arr(), failed = J::arr(), skipped = J::arr();
      std::string jp, jf;
      const std::string tid = xml_escape(tc.has_name ? tc.name : std::string());
      for (auto& r : tc.rules) {
        if (r.expected < 0) { J sk = J::obj(); sk.add("name", J::str(r.rule)); skipped.push(std::move(sk)); continue; }
        if (r.matched >= 0) {
          J p = J::obj(); p.add("name", J::str(r.rule)); p.add("evaluated", J::str(kStatus[r.matched]));
          passed.push(std::move(p));
          jp += "        <testcase id=\"" + tid + "\" name=\"" + xml_escape(r.rule) + "\" time=\"0\" status=\"pass\"/>\n";
        } else {
          J ev = J::arr();
          for (uint32_t st : r.evaluated) ev.push(J::str(kStatus[st]));
          J p = J::obj(); p.add("name", J::str(r.rule)); p.add("expected", J::str(kStatus[r.expected])); p.add("evaluated", std::move(ev));
          failed.push(std::move(p));
          jf += "        <testcase id=\"" + tid + "\" name=\"" + xml_escape(r.rule) + "\" time=\"0\">\n            <failure>" +
                xml_escape(std::string("Expected = ") + kStatus[r.expected] + ", Evaluated = [" + statuses(r.evaluated) + "]") +
                "</failure>\n        </testcase>\n";
          nfail++;
        }
        tests++;
      }
      if (!failed.a.empty()) code = 7;
      junit += jp + jf;   // build_junit_test_cases: passed rules, then failed rules
      J c = J::obj();
      c.add("name", J::str(tc.has_name ? tc.name : std::string()));
      c.add("passed_rules", std::move(passed));
      c.add("failed_rules", std::move(failed));
      c.add("skipped_rules", std::move(skipped));
      cases.push(std::move(c));
    }
  }
  failures += nfail;
  suite = "    <testsuite name=\"" + rn + "\" errors=\"0\" failures=\"" + std::to_string(nfail) + "\" time=\"0\">\n" + junit +
          "    </testsuite>\n";
  J res = J::obj();
  res.add("rule_file", J::str(in.rules_name));
  res.add("test_cases", std::move(cases));
  return res;
}
}  // namespace

// `cfn-guard test` structured output of one TestResult (single: handle_structured_single_report,
// test.rs:326-380) or of a Vec<TestResult> (handle_structured_directory_report, test.rs:383-456);
// exit code: the TestResults' codes folded with get_exit_code (test.rs:459-472)
std::string test_report_list(int32_t fmt, const std::vector<TestResultIn>& results, int32_t& exit_code, bool single) {
  exit_code = 0;
  J arr = J::arr();
  std::string suites;
  size_t tests = 0, failures = 0, errors = 0;
  for (auto& r : results) {
    int32_t code = 0;
    std::string suite;
    J o = test_result(r, code, suite, tests, failures, errors);
    suites += suite;
    // get_exit_code: SUCCESS takes the result's; TEST_ERROR stays; TEST_FAILURE yields to TEST_ERROR
    if (exit_code == 0) exit_code = code;
    else if (exit_code == 7 && code == 1) exit_code = 1;
    arr.push(std::move(o));
  }
  if (fmt == OUT_JUNIT)
    return "<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<testsuites name=\"cfn-guard test report\" tests=\"" + std::to_string(tests) +
           "\" failures=\"" + std::to_string(failures) + "\" errors=\"" + std::to_string(errors) + "\" time=\"0\">\n" + suites +
           "</testsuites>\n";
  if (fmt == OUT_YAML) {
    YamlOut y;
    if (single) y.document(arr.a[0]); else y.document(arr);
    return y.buf;
  }
  std::string out;
  pretty(single ? arr.a[0] : arr, 0, out);
  return out;
}

namespace {

J status_json(uint32_t s) { return J::str(status_str(s)); }
J block_check(bool alo, uint32_t st) {
  J b = J::obj();
  b.add("at_least_one_matches", J::boolean(alo));
  b.add("status", status_json(st));
  b.add("message", J::null());
  return b;
}
J tagged(const char* k, J v) { J o = J::obj(); o.add(k, std::move(v)); return o; }

// one open event of the verbose tree
// one line of the verbose tree as text (EventRecord Display, display.rs:314-323) and its children
struct TNode {
  std::string line;
  std::vector<TNode> kids;
};

struct VNode {
  uint32_t type = 0, id = NONE;
  std::string ctx;
  J children = J::arr();
  std::vector<TNode> tk;
};

// display_comparison (display.rs:9-11) over CmpOperator's Display (values.rs:58-79)
std::string cmp_text(uint32_t op, bool neg) {
  static const char* names[] = {"EQUALS", "IN", "GREATER THAN", "LESS THAN", "LESS THAN EQUALS", "GREATER THAN EQUALS",
                                "EXISTS", "EMPTY", "IS STRING", "IS LIST", "IS MAP", "IS BOOL", "IS INT", "IS FLOAT", "IS NULL"};
  return std::string(neg ? "not" : "") + " " + (op < 15 ? names[op] : "?");
}

struct VerboseBuilder {
  const R& r;
  const std::string& data_name;
  std::vector<VNode> stack;
  J root;
  bool have_root = false;

  const PClause& pc(uint32_t cid) const { return r.prog.clauses[cid]; }
  const std::string& ctx_d(uint32_t cid) const { return r.prog.ctx[pc(cid).d]; }
  std::string when_ctx(uint32_t cid) const { return (pc(cid).flags & 1u) ? "RuleClause" : "GuardConditionClause"; }

  // text: also build the Display tree (`cfn-guard test --verbose`, validate --verbose)
  bool text = false;
  TNode troot;

  void attach(std::string ctx, J container, J children, std::string disp = std::string(), std::vector<TNode> tk = {}) {
    if (text) {
      TNode t{disp + "[Context=" + ctx + "]", std::move(tk)};
      if (stack.empty()) troot = std::move(t);
      else stack.back().tk.push_back(std::move(t));
    }
    J e = J::obj();
    e.add("context", J::str(ctx));
    e.add("container", std::move(container));
    e.add("children", std::move(children));
    if (stack.empty()) { root = std::move(e); have_root = true; }
    else stack.back().children.push(std::move(e));
  }
  void leaf(std::string ctx, J check, std::string disp = std::string()) {
    attach(std::move(ctx), tagged("ClauseValueCheck", std::move(check)), J::arr(), std::move(disp));
  }

  // QueryResult Display (display.rs:109-126); keep_literal as the serde form of the same record
  std::string qr_text(const QR& q, bool keep_literal) const {
    const uint32_t k = q.meta & 3u;
    if (k == QR_UNRESOLVED) return "(unresolved, " + r.unresolved_display(q) + ")";
    if (keep_literal && k == QR_LITERAL) return "literal, " + r.pav_display(q);
    return "(resolved, " + r.pav_display(q) + ")";
  }
  static std::string st_text(uint32_t st) { return st == ST_PASS ? "PASS" : st == ST_FAIL ? "FAIL" : "SKIP"; }

  // RecordType Display (display.rs:200-311) of a closing container
  std::string close_disp(const Rec& rc) const {
    const std::string st = st_text(rc.y & 0xFFu);
    switch (rc.x) {
      case EV_FILE: return "File(" + data_name + ", Status=" + st + ")";
      case EV_RULE: return "Rule(" + r.prog.rule_names[rc.clause] + ", Status=" + st + ")";
      case EV_RULE_COND: return "Rule/When(Status=" + st + ")";
      case EV_DISJ: return "Disjunction(Status = " + st + ")";
      case EV_GAC: return "GuardClauseBlock(Status = " + st + ")";
      case EV_NAMED:
        if ((rc.y & 0xFFu) == ST_PASS) return "GuardClauseValueCheck(Status=PASS)";
        return "GuardClauseDependentRule(Rule=" + r.prog.ctx[pc(rc.clause).f] + ", Status=FAIL)";
      case EV_BLOCK: return "GuardValueBlockCheck(Status = " + st + ")";
      case EV_WHEN: return "WhenConditionalBlock(Status = " + st + ")";
      case EV_WHEN_COND: return "WhenCondition(Status = " + st + ")";
      case EV_TYPE: return "Type(" + r.prog.ctx[pc(rc.clause).f] + ", Status=" + st + ")";
      case EV_TYPE_COND: return "TypeBlock/When Status=" + st + ")";
      case EV_TYPE_VAL: return "TypeBlock/Block Status=" + st + ")";
      default: return "Filter/ConjunctionsBlock(Status=" + st + ")";
    }
  }

  // eval_conjunction_clauses' context: format!("{}#disjunction", type_name::<T>()) (eval.rs:1980), T
  // the clause type the enclosing container evaluates
  std::string disj_ctx() const {
    const uint32_t pt = stack.empty() ? EV_FILE : stack.back().type;
    const char* t = pt == EV_RULE ? "RuleClause"
                  : (pt == EV_RULE_COND || pt == EV_TYPE_COND || pt == EV_WHEN_COND) ? "WhenGuardClause"
                  : "GuardClause";
    return std::string("cfn_guard::rules::exprs::") + t + "#disjunction";
  }

  std::string open_ctx(const Rec& rc) const {
    switch (rc.x) {
      case EV_FILE: return "File(rules=" + std::to_string(r.prog.n_rules) + ")";
      case EV_RULE: return r.prog.rule_names[rc.clause];
      case EV_RULE_COND: return "Rule#" + r.prog.rule_names[rc.clause] + "/When";
      case EV_DISJ: return disj_ctx();
      case EV_GAC: return "GuardAccessClause#block" + ctx_d(rc.clause);
      case EV_NAMED: case EV_BLOCK: case EV_TYPE: return ctx_d(rc.clause);
      case EV_WHEN: return when_ctx(rc.clause);
      case EV_WHEN_COND: return when_ctx(rc.clause) + "/When";
      case EV_TYPE_COND: return ctx_d(rc.clause) + "/When";
      case EV_TYPE_VAL: return ctx_d(rc.clause) + "/" + std::to_string(rc.y);
      case EV_FILTER_MAP: return "Filter/Map#" + std::to_string(rc.y);
      default: return "Filter/List#" + std::to_string(rc.y);
    }
  }

  J close_container(const Rec& rc) const {
    const uint32_t st = rc.y & 0xFFu;
    const bool alo = (rc.y >> 8) & 1u;
    switch (rc.x) {
      case EV_FILE: {
        J n = J::obj(); n.add("name", J::str(data_name)); n.add("status", status_json(st)); n.add("message", J::null());
        return tagged("FileCheck", std::move(n));
      }
      case EV_RULE: {
        const uint32_t m = rc.from.uref;
        J n = J::obj(); n.add("name", J::str(r.prog.rule_names[rc.clause])); n.add("status", status_json(st));
        n.add("message", m == NONE ? J::null() : J::str(r.prog.msgs[m]));
        return tagged("RuleCheck", std::move(n));
      }
      case EV_RULE_COND: return tagged("RuleCondition", status_json(st));
      case EV_DISJ: return tagged("Disjunction", block_check(true, st));
      case EV_GAC: return tagged("GuardClauseBlockCheck", block_check(alo, st));
      case EV_NAMED: {
        if (st == ST_PASS) return tagged("ClauseValueCheck", J::str("Success"));
        J m = J::obj();
        m.add("rule", J::str(r.prog.ctx[pc(rc.clause).f]));
        m.add("message", J::null());
        m.add("custom_message", r.custom_opt(pc(rc.clause)));
        m.add("status", status_json(ST_FAIL));
        return tagged("ClauseValueCheck", tagged("DependentRule", std::move(m)));
      }
      case EV_BLOCK: return tagged("BlockGuardCheck", block_check(alo, st));
      case EV_WHEN: return tagged("WhenCheck", block_check(false, st));
      case EV_WHEN_COND: return tagged("WhenCondition", status_json(st));
      case EV_TYPE: {
        J t = J::obj(); t.add("type_name", J::str(r.prog.ctx[pc(rc.clause).f])); t.add("block", block_check(false, st));
        return tagged("TypeCheck", std::move(t));
      }
      case EV_TYPE_COND: return tagged("TypeCondition", status_json(st));
      case EV_TYPE_VAL: return tagged("TypeBlock", status_json(st));
      default: return tagged("Filter", status_json(st));
    }
  }

  void run(const RecSpan& recs) {
    for (size_t i = 0; i < recs.size(); i++) {
      const Rec& rc = recs[i];
      const bool mk = rc.clause == NONE;   // a map-key-filter comparison: context "", no custom message
      switch (rc.kind) {
        case REC_EV_OPEN: {
          VNode n; n.type = rc.x; n.id = rc.clause; n.ctx = open_ctx(rc);
          stack.push_back(std::move(n));
          break;
        }
        case REC_EV_CLOSE: {
          if (stack.empty() || stack.back().type != rc.x) throw Fatal{"IncompatibleError", "MI355X path: unbalanced verbose event records"};
          VNode n = std::move(stack.back());
          stack.pop_back();
          attach(std::move(n.ctx), close_container(rc), std::move(n.children), text ? close_disp(rc) : std::string(), std::move(n.tk));
          break;
        }
        case REC_SUCCESS: leaf(mk ? std::string() : ctx_d(rc.clause), J::str("Success"), "GuardClauseValueCheck(Status=PASS)"); break;
        case REC_CMP: {
          const uint32_t op = mk ? (rc.y & 15u) : (pc(rc.clause).flags & 15u);
          const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pc(rc.clause).flags >> 4) & 1u);
          J m = J::obj();
          m.add("comparison", r.comparison(op, neg));
          m.add("from", r.qr_json(rc.from, false));
          m.add("to", rc.to.meta == 0xFFFFFFFFu ? J::null() : r.qr_json(rc.to, false));
          m.add("message", rc.x ? J::str(r.nc_reason(rc)) : J::null());
          m.add("custom_message", mk ? J::null() : r.custom_opt(pc(rc.clause)));
          m.add("status", status_json(ST_FAIL));
          std::string disp;
          if (text)
            disp = "GuardClauseBinaryCheck(Status=FAIL, Comparison=" + cmp_text(op, neg) + ", from=" + qr_text(rc.from, false) +
                   ", to=" + (rc.to.meta == 0xFFFFFFFFu ? std::string() : qr_text(rc.to, false)) + ")";
          leaf(mk ? std::string() : ctx_d(rc.clause), tagged("Comparison", std::move(m)), std::move(disp));
          break;
        }
        case REC_IN: {
          const uint32_t op = mk ? (rc.y & 15u) : (pc(rc.clause).flags & 15u);
          const bool neg = mk ? ((rc.y >> 4) & 1u) : ((pc(rc.clause).flags >> 4) & 1u);
          J to = J::arr();
          std::string tos;   // SliceDisplay (exprs.rs:286-303) of the to values
          uint32_t got = 0;
          auto add_to = [&](const QR& q) {
            to.push(r.qr_json(q, false));
            if (text) tos += (got ? "." : "") + qr_text(q, false);
            got++;
          };
          while (got < rc.x && i + 1 < recs.size() && recs[i + 1].kind == REC_LIST) {
            const Rec& l = recs[++i];
            add_to(l.from);
            if (got < rc.x) add_to(l.to);
          }
          J m = J::obj();
          m.add("comparison", r.comparison(op, neg));
          m.add("from", r.qr_json(rc.from, false));
          m.add("to", std::move(to));
          m.add("message", J::null());
          m.add("custom_message", mk ? J::null() : r.custom_opt(pc(rc.clause)));
          m.add("status", status_json(ST_FAIL));
          std::string disp;
          if (text) {
            std::string fixed;
            for (size_t k = 0; k < tos.size(); k++) { if (tos[k] == '.' && k + 1 < tos.size() && tos[k + 1] == '[') continue; fixed.push_back(tos[k]); }
            disp = "GuardClauseInBinaryCheck(Status=FAIL, Comparison=" + cmp_text(op, neg) + ", from=" + qr_text(rc.from, false) +
                   ", to=" + fixed + ")";
          }
          leaf(mk ? std::string() : ctx_d(rc.clause), tagged("InComparison", std::move(m)), std::move(disp));
          break;
        }
        case REC_UNARY: {
          const PClause& p = pc(rc.clause);
          J v = J::obj();
          v.add("from", r.qr_json(rc.from, true));
          v.add("message", J::null());
          v.add("custom_message", r.custom_opt(p));
          v.add("status", status_json(ST_FAIL));
          J u = J::obj();
          u.add("value", std::move(v));
          u.add("comparison", r.comparison(p.flags & 15u, (p.flags >> 4) & 1u));
          std::string disp;
          if (text)
            disp = "GuardClauseUnaryCheck(Status=FAIL, Comparison=" + cmp_text(p.flags & 15u, (p.flags >> 4) & 1u) +
                   ", Value-At=" + qr_text(rc.from, true) + ")";
          leaf(ctx_d(rc.clause), tagged("Unary", std::move(u)), std::move(disp));
          break;
        }
        case REC_NOVALUE_EMPTY:
          leaf(ctx_d(rc.clause), tagged("NoValueForEmptyCheck", r.custom_opt(pc(rc.clause))),
               "GuardClause(Status=FAIL, Empty, " + r.custom(pc(rc.clause)) + ")");
          break;
        case REC_MISSING_BLOCK_VALUE: {
          // eval.rs:1343-1358: message "Query <query> did not resolve to correct value, reason <reason>"
          const PClause& p = pc(rc.clause);
          const std::string msg = "Query " + slice_display(r.prog.queries[p.a], 0) + " did not resolve to correct value, reason " +
                                  r.reason(rc.from);
          J v = J::obj();
          v.add("from", r.qr_json(rc.from, false));
          v.add("message", J::str(msg));
          v.add("custom_message", J::null());
          v.add("status", status_json(ST_FAIL));
          // display.rs:148-161: the unresolved value's traversed_to path (pointer only)
          const std::string tt = (rc.from.meta & 3u) == QR_UNRESOLVED ? r.path(rc.from.node) : std::string();
          leaf(r.prog.ctx[p.f], tagged("MissingBlockValue", std::move(v)), "GuardBlockValueMissing(Status=FAIL, Reason=" + msg + ", " + tt + ")");
          break;
        }
        default: break;   // report-only records (rule / disjunction brackets) and REC_LIST (consumed above)
      }
    }
    if (!stack.empty() || !have_root) throw Fatal{"IncompatibleError", "MI355X path: incomplete verbose event records"};
  }
};

}  // namespace

bool verbose_tree(const DocBatch& docs, uint32_t doc, const Program& prog, const TileResult& tile, const std::string& data_name,
                  std::string& out, ReportError& err) {
  try {
    if (tile.out.err) { tile_error(docs, doc, prog, tile.out, err); return false; }
    R r{docs, prog, docs.serde, docs.base[doc], &tile.aux};
    VerboseBuilder b{r, data_name, {}, J(), false};
    b.run(tile.recs);
    pretty(b.root, 0, out);
    return true;
  } catch (Fatal& f) {
    err.set = true; err.kind = f.kind; err.msg = f.msg;
    return false;
  }
}

namespace {
// pprint_tree (commands/validate.rs:666-683)
void pprint_tree(const TNode& n, const std::string& prefix, bool last, std::string& out) {
  out += prefix; out += last ? "`- " : "|- "; out += n.line; out += '\n';
  const std::string child = prefix + (last ? "   " : "|  ");
  for (size_t i = 0; i < n.kids.size(); i++) pprint_tree(n.kids[i], child, i + 1 == n.kids.size(), out);
}
}  // namespace

bool verbose_text(const DocBatch& docs, uint32_t doc, const Program& prog, const TileResult& tile, const std::string& data_name,
                  std::string& out, ReportError& err) {
  try {
    if (tile.out.err) { tile_error(docs, doc, prog, tile.out, err); return false; }
    R r{docs, prog, docs.serde, docs.base[doc], &tile.aux};
    VerboseBuilder b{r, data_name, {}, J(), false};
    b.text = true;
    b.run(tile.recs);
    pprint_tree(b.troot, "", true, out);
    return true;
  } catch (Fatal& f) {
    err.set = true; err.kind = f.kind; err.msg = f.msg;
    return false;
  }
}

bool report_document(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                     const std::vector<const TileResult*>& tiles, int indent, std::string& out, ReportError& err) {
  TextBuf t;
  if (!write_file_report(docs, doc, progs, tiles, indent, t, err)) return false;
  out.append(t.data(), t.size());
  return true;
}

#include "console_report.inc"

}  // namespace gg
