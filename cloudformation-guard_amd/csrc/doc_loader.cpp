// Document loader (see doc_loader.h for the reference mapping).
#include "doc_loader.h"

#include <charconv>

#include <yaml.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_map>

#include "host_format.h"

namespace gg {

// ------------------------------------------------------------ Rust parsing ---
// `str::parse::<i64>()`
static bool rust_parse_i64(const std::string& s, int64_t& out) {
  size_t i = 0, n = s.size();
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
  if (i >= n) return false;
  unsigned __int128 v = 0;
  for (; i < n; i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// `str::parse::<f64>()` (Rust dec2flt grammar + inf/infinity/nan, case-insensitive)
static bool rust_parse_f64(const std::string& s, double& out) {
  size_t i = 0, n = s.size();
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
  std::string rest = s.substr(i);
  std::string low;
  for (char c : rest) low.push_back((char)tolower((unsigned char)c));
  if (low == "inf" || low == "infinity") { out = neg ? -INFINITY : INFINITY; return true; }
  if (low == "nan") { out = NAN; return true; }
  size_t j = i, digits = 0;
  while (j < n && isdigit((unsigned char)s[j])) { j++; digits++; }
  if (j < n && s[j] == '.') { j++; while (j < n && isdigit((unsigned char)s[j])) { j++; digits++; } }
  if (digits == 0) return false;
  if (j < n && (s[j] == 'e' || s[j] == 'E')) {
    j++;
    if (j < n && (s[j] == '+' || s[j] == '-')) j++;
    size_t ed = 0;
    while (j < n && isdigit((unsigned char)s[j])) { j++; ed++; }
    if (ed == 0) return false;
  }
  if (j != n) return false;
  out = strtod(s.c_str(), nullptr);
  return true;
}

// ------------------------------------------------------------- temp tree ---
namespace {

struct TN {
  uint32_t kind = K_NULL;
  int64_t i = 0;
  double f = 0;
  std::string s;
  bool bad = false;
  uint32_t line = 0, col = 0;
  std::vector<uint32_t> kids;
  std::vector<std::string> keys;
  std::vector<std::pair<uint32_t, uint32_t>> kmarks;
};

struct Tree {
  std::vector<TN> n;
  uint32_t add(TN&& t) { n.push_back(std::move(t)); return (uint32_t)n.size() - 1; }
};

const char* kShort[][2] = {
    {"Ref", "Ref"}, {"GetAtt", "Fn::GetAtt"}, {"Base64", "Fn::Base64"}, {"Sub", "Fn::Sub"},
    {"GetAZs", "Fn::GetAZs"}, {"ImportValue", "Fn::ImportValue"}, {"Condition", "Condition"},
    {"RefAll", "Fn::RefAll"}, {"Select", "Fn::Select"}, {"Split", "Fn::Split"}, {"Join", "Fn::Join"},
    {"FindInMap", "Fn::FindInMap"}, {"And", "Fn::And"}, {"Equals", "Fn::Equals"},
    {"Contains", "Fn::Contains"}, {"EachMemberIn", "Fn::EachMemberIn"},
    {"EachMemberEquals", "Fn::EachMemberEquals"}, {"ValueOf", "Fn::ValueOf"}, {"If", "Fn::If"},
    {"Not", "Fn::Not"}, {"Or", "Fn::Or"}};
const char* kSingle[] = {"Ref", "Base64", "Sub", "GetAZs", "ImportValue", "GetAtt", "Condition", "RefAll"};
const char* kSeq[] = {"GetAtt", "Sub", "Select", "Split", "Join", "FindInMap", "And", "Equals", "Contains",
                      "EachMemberIn", "EachMemberEquals", "ValueOf", "If", "Not", "Or"};

bool in_set(const char* const* set, size_t n, const std::string& s) {
  for (size_t i = 0; i < n; i++) if (s == set[i]) return true;
  return false;
}
bool is_single(const std::string& s) { return in_set(kSingle, sizeof kSingle / sizeof *kSingle, s); }
bool is_seq(const std::string& s) { return in_set(kSeq, sizeof kSeq / sizeof *kSeq, s); }
std::string long_form(const std::string& s) {
  for (auto& p : kShort) if (s == p[0]) return p[1];
  return s;
}

void split_tag(const std::string& tag, std::string& handle, std::string& suffix) {
  size_t i = 0;
  while (i < tag.size() && tag[i] == '!') i++;
  handle = tag.substr(0, i);
  suffix = tag.substr(i);
}

const char* TYPE_REF_PREFIX = "tag:yaml.org,2002:";

// loader.rs:62-102 (+ handle_type_ref 227-244, handle_single_value_func_ref 197-211)
uint32_t scalar_node(Tree& t, const std::string& val, const char* tag, bool plain, uint32_t line, uint32_t col) {
  TN n; n.line = line; n.col = col;
  if (tag) {
    std::string handle, suffix;
    split_tag(tag, handle, suffix);
    if (handle == "!") {
      if (is_single(suffix)) {
        TN inner; inner.kind = K_STRING; inner.s = val; inner.line = line; inner.col = col;
        uint32_t ii = t.add(std::move(inner));
        n.kind = K_MAP; n.keys.push_back(long_form(suffix)); n.kmarks.push_back({line, col}); n.kids.push_back(ii);
        return t.add(std::move(n));
      }
      n.kind = K_STRING; n.s = val; return t.add(std::move(n));
    }
    if (suffix.rfind(TYPE_REF_PREFIX, 0) == 0) {
      if (suffix == "tag:yaml.org,2002:bool") {
        if (val == "true") { n.kind = K_BOOL; n.i = 1; }
        else if (val == "false") { n.kind = K_BOOL; n.i = 0; }
        else { n.kind = K_STRING; n.s = val; }
      } else if (suffix == "tag:yaml.org,2002:int") {
        int64_t v;
        if (rust_parse_i64(val, v)) { n.kind = K_INT; n.i = v; } else { n.bad = true; n.s = val; }
      } else if (suffix == "tag:yaml.org,2002:float") {
        double v;
        if (rust_parse_f64(val, v)) { n.kind = K_FLOAT; n.f = v; } else { n.bad = true; n.s = val; }
      } else if (suffix == "tag:yaml.org,2002:null") {
        n.kind = K_NULL;
      } else { n.kind = K_STRING; n.s = val; }
      return t.add(std::move(n));
    }
    n.kind = K_STRING; n.s = val; return t.add(std::move(n));
  }
  if (!plain) { n.kind = K_STRING; n.s = val; return t.add(std::move(n)); }
  int64_t iv; double fv;
  if (rust_parse_i64(val, iv)) { n.kind = K_INT; n.i = iv; }
  else if (rust_parse_f64(val, fv)) { n.kind = K_FLOAT; n.f = fv; }
  else if (val == "true" || val == "yes" || val == "on" || val == "y") { n.kind = K_BOOL; n.i = 1; }
  else if (val == "false" || val == "no" || val == "off" || val == "n") { n.kind = K_BOOL; n.i = 0; }
  else {
    std::string low;
    for (char c : val) low.push_back((char)tolower((unsigned char)c));
    if (low == "~" || low == "null") n.kind = K_NULL;
    else { n.kind = K_STRING; n.s = val; }
  }
  return t.add(std::move(n));
}

// serde_yaml 0.9 (YAML 1.2 core) plain scalar resolution
uint32_t serde_yaml_scalar(Tree& t, const std::string& val, bool plain) {
  TN n;
  if (!plain) { n.kind = K_STRING; n.s = val; return t.add(std::move(n)); }
  if (val == "~" || val == "null" || val == "Null" || val == "NULL" || val.empty()) { n.kind = K_NULL; return t.add(std::move(n)); }
  if (val == "true" || val == "True" || val == "TRUE") { n.kind = K_BOOL; n.i = 1; return t.add(std::move(n)); }
  if (val == "false" || val == "False" || val == "FALSE") { n.kind = K_BOOL; n.i = 0; return t.add(std::move(n)); }
  // ints: [-+]?(digits | 0x.. | 0o.. | 0b..)
  {
    size_t i = 0; bool neg = false;
    if (i < val.size() && (val[i] == '+' || val[i] == '-')) { neg = val[i] == '-'; i++; }
    std::string body = val.substr(i);
    int base = 10; size_t start = 0;
    if (body.size() > 2 && body[0] == '0' && (body[1] == 'x' || body[1] == 'o' || body[1] == 'b')) {
      base = body[1] == 'x' ? 16 : body[1] == 'o' ? 8 : 2; start = 2;
    }
    bool ok = start < body.size();
    unsigned __int128 v = 0; bool overflow = false;
    for (size_t j = start; j < body.size() && ok; j++) {
      int d;
      char c = body[j];
      if (c >= '0' && c <= '9') d = c - '0';
      else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
      else { ok = false; break; }
      if (d >= base) { ok = false; break; }
      v = v * base + d;
      if (v > ((unsigned __int128)1 << 64)) overflow = true;
    }
    if (ok) {
      n.kind = K_INT;
      if (!overflow && !neg && v <= (unsigned __int128)INT64_MAX) { n.i = (int64_t)v; return t.add(std::move(n)); }
      if (!overflow && neg && v <= ((unsigned __int128)1 << 63)) { n.i = (int64_t)(-(__int128)v); return t.add(std::move(n)); }
      if (!overflow && !neg && v <= (unsigned __int128)UINT64_MAX) { n.i = (int64_t)(uint64_t)v; return t.add(std::move(n)); }
      n.kind = K_FLOAT; n.f = strtod(val.c_str(), nullptr); return t.add(std::move(n));
    }
  }
  {
    double fv;
    std::string low;
    for (char c : val) low.push_back((char)tolower((unsigned char)c));
    if (low == ".inf" || low == "+.inf") { n.kind = K_FLOAT; n.f = INFINITY; return t.add(std::move(n)); }
    if (low == "-.inf") { n.kind = K_FLOAT; n.f = -INFINITY; return t.add(std::move(n)); }
    if (low == ".nan") { n.kind = K_FLOAT; n.f = NAN; return t.add(std::move(n)); }
    bool okf = !val.empty() && rust_parse_f64(val, fv) && low.find("inf") == std::string::npos && low.find("nan") == std::string::npos;
    if (okf) { n.kind = K_FLOAT; n.f = fv; return t.add(std::move(n)); }
  }
  n.kind = K_STRING; n.s = val; return t.add(std::move(n));
}

constexpr size_t kNoParent = ~(size_t)0;

struct Emitter {
  DocBatch& b;
  Tree& t;
  bool serde;
  uint64_t base;   // global index of the document's first node; stored indices are relative
  void fill(uint32_t ti, size_t slot, size_t parent, uint32_t line, uint32_t col) {
    TN& n = t.n[ti];
    DNode& d = b.nodes[slot];
    d.kind = n.kind; d.count = 0; d.a = 0; d.b = 0; d.parent = parent == kNoParent ? NONE : (uint32_t)(parent - base);
    b.line[slot] = line; b.col[slot] = col;
    switch (n.kind) {
      case K_STRING: {
        d.count = (uint32_t)n.s.size();
        d.a = b.intern(n.s.data(), d.count, fnv1a(n.s.data(), n.s.size()));
        d.b = d.a;   // string id = canonical pool offset (equal ids <=> equal strings)
        break;
      }
      case K_BOOL: d.a = (uint32_t)n.i; break;
      case K_INT: { uint64_t u = (uint64_t)n.i; d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32); break; }
      case K_FLOAT: { uint64_t u; memcpy(&u, &n.f, 8); d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32); break; }
      case K_LIST: {
        uint32_t cnt = (uint32_t)n.kids.size();
        size_t first = b.nodes.size();
        grow(cnt);
        DNode& dd = b.nodes[slot];
        dd.a = (uint32_t)(first - base); dd.count = cnt;
        for (uint32_t j = 0; j < cnt; j++) {
          uint32_t k = t.n[ti].kids[j];
          const TN& kn = t.n[k];
          b.nodes[first + j].key_off = NONE; b.nodes[first + j].key_len = 0; b.nodes[first + j].key_hash = 0;
          fill(k, first + j, slot, serde ? 0 : kn.line, serde ? 0 : kn.col);
        }
        break;
      }
      case K_MAP: {
        // IndexMap<String, _>::insert over the (key, mark) entries: first position, last value
        std::vector<std::string> keys;
        std::vector<std::pair<uint32_t, uint32_t>> kmarks;
        std::vector<uint32_t> vals;
        std::unordered_map<std::string, size_t> pos;
        for (size_t j = 0; j < t.n[ti].keys.size(); j++) {
          const std::string& k = t.n[ti].keys[j];
          auto it = pos.find(k);
          if (it == pos.end()) {
            pos[k] = keys.size(); keys.push_back(k); kmarks.push_back(t.n[ti].kmarks[j]); vals.push_back(t.n[ti].kids[j]);
          } else {
            vals[it->second] = t.n[ti].kids[j];
          }
        }
        uint32_t cnt = (uint32_t)keys.size();
        size_t first = b.nodes.size();
        grow(cnt);
        DNode& dd = b.nodes[slot];
        dd.a = (uint32_t)(first - base); dd.count = cnt;
        const uint32_t nall = (uint32_t)t.n[ti].keys.size();
        if (!serde && nall > cnt) {
          // a repeated key (libyaml loader: the IndexMap is keyed by (key, mark), loader.rs:172-185):
          // MapValue.keys keeps every occurrence while MapValue.values keeps one entry per key
          // (path_value.rs:453-470).  The keys list goes to a block of nall key slots -- key id,
          // length and mark of each occurrence in document order, parent = the map, kind K_NULL,
          // count = nall -- referenced by the map node's `b` (0 = no repeated key; index 0 is the
          // root, never such a block).  `*` captures (accumulate_map's zip of keys with values,
          // eval_context.rs:216) and `keys` filters (:850-856) read it; nothing else does.
          size_t kfirst = b.nodes.size();
          grow(nall);
          b.nodes[slot].b = (uint32_t)(kfirst - base);
          for (uint32_t j = 0; j < nall; j++) {
            const std::string& k = t.n[ti].keys[j];
            DNode& kn = b.nodes[kfirst + j];
            kn.kind = K_NULL; kn.count = nall; kn.a = 0; kn.b = 0; kn.parent = (uint32_t)(slot - base);
            kn.key_len = (uint32_t)k.size();
            kn.key_off = b.intern(k.data(), kn.key_len, fnv1a(k.data(), k.size()));
            kn.key_hash = kn.key_off;
            b.line[kfirst + j] = 0; b.col[kfirst + j] = 0;
            b.kline[kfirst + j] = t.n[ti].kmarks[j].first;
            b.kcol[kfirst + j] = t.n[ti].kmarks[j].second;
          }
        }
        for (uint32_t j = 0; j < cnt; j++) {
          DNode& c = b.nodes[first + j];
          c.key_len = (uint32_t)keys[j].size();
          c.key_off = b.intern(keys[j].data(), c.key_len, fnv1a(keys[j].data(), keys[j].size()));
          c.key_hash = c.key_off;   // key id
          b.kline[first + j] = serde ? 0 : kmarks[j].first;
          b.kcol[first + j] = serde ? 0 : kmarks[j].second;
          const TN& kn = t.n[vals[j]];
          fill(vals[j], first + j, slot, serde ? 0 : kn.line, serde ? 0 : kn.col);
        }
        break;
      }
      default: break;
    }
  }
  void grow(uint32_t cnt) {
    b.grow_zeroed(b.nodes.size() + cnt);
  }
};

bool check_bad(const Tree& t, uint32_t ti, LoadError& err) {
  const TN& n = t.n[ti];
  if (n.bad) {
    err.kind = "ParseError";
    err.msg = "Bad Value encountered parsing incoming file Value = " + n.s + ", Loc = L:" + std::to_string(n.line) +
              ",C:" + std::to_string(n.col);
    return false;
  }
  for (uint32_t k : n.kids) if (!check_bad(t, k, err)) return false;
  return true;
}

bool emit_root(DocBatch& b, Tree& t, uint32_t root, const std::string& name, bool serde, LoadError& err) {
  if (!check_bad(t, root, err)) return false;
  if (t.n.size() > kMaxDocNodes) { err.kind = "IncompatibleError"; err.msg = "document too large for the MI355X arena"; return false; }
  size_t slot = b.nodes.size();
  Emitter e{b, t, serde, (uint64_t)slot};
  e.grow(1);
  b.nodes[slot].key_off = NONE; b.nodes[slot].key_len = 0; b.nodes[slot].key_hash = 0;
  const TN& r = t.n[root];
  uint32_t line = 0, col = 0;
  // root: Path::root() (L0,C0) keeps its location for lists; maps/scalars take their own mark
  if (!serde && r.kind != K_LIST) { line = r.line; col = r.col; }
  e.fill(root, slot, kNoParent, line, col);
  b.roots.push_back(0);
  b.base.push_back(slot);
  b.names.push_back(name);
  return true;
}

// ------------------------------------------------------ libyaml event loop ---
struct YamlParser {
  yaml_parser_t p;
  bool ok;
  YamlParser(const char* text, size_t len) {
    ok = yaml_parser_initialize(&p) != 0;
    yaml_parser_set_encoding(&p, YAML_UTF8_ENCODING);
    yaml_parser_set_input_string(&p, (const unsigned char*)text, len);
  }
  ~YamlParser() { yaml_parser_delete(&p); }
};

std::string ev_scalar(const yaml_event_t& ev) {
  return std::string((const char*)ev.data.scalar.value, ev.data.scalar.length);
}

// Loader::load (loader.rs:31-60): returns root tree node of the first document
bool libyaml_load(const char* text, size_t len, Tree& t, uint32_t& root, LoadError& err) {
  YamlParser yp(text, len);
  std::vector<uint32_t> stack, last_container;
  std::vector<std::pair<size_t, std::pair<std::string, std::pair<uint32_t, uint32_t>>>> func_support;
  for (;;) {
    yaml_event_t ev;
    if (yp.p.error != YAML_NO_ERROR || !yaml_parser_parse(&yp.p, &ev)) {
      err.kind = "ParseError"; err.msg = "error parsing file"; return false;
    }
    uint32_t line = (uint32_t)ev.start_mark.line, col = (uint32_t)ev.start_mark.column;
    bool done = false;
    switch (ev.type) {
      case YAML_STREAM_START_EVENT: case YAML_DOCUMENT_START_EVENT: break;
      case YAML_STREAM_END_EVENT: case YAML_NO_EVENT:
        // the reference keeps polling after STREAM-END and panics (unimplemented!())
        yaml_event_delete(&ev);
        err.kind = "ParseError"; err.msg = "error parsing file"; return false;
      case YAML_DOCUMENT_END_EVENT:
        root = stack.back(); done = true; break;
      case YAML_MAPPING_START_EVENT: {
        TN n; n.kind = K_MAP; n.line = line; n.col = col;
        stack.push_back(t.add(std::move(n)));
        last_container.push_back((uint32_t)stack.size() - 1);
        break;
      }
      case YAML_MAPPING_END_EVENT: {
        uint32_t idx = last_container.back(); last_container.pop_back();
        std::vector<uint32_t> kvs(stack.begin() + idx + 1, stack.end());
        stack.resize(idx + 1);
        uint32_t m = stack.back();
        for (size_t j = 0; j + 1 < kvs.size(); j += 2) {
          const TN& k = t.n[kvs[j]];
          if (k.kind != K_STRING || k.bad) {
            yaml_event_delete(&ev);
            err.kind = "InternalError";
            err.msg = "non string type detected for key in a map at L:" + std::to_string(k.line) + ",C:" +
                      std::to_string(k.col) + ", cfn-guard only supports keys that are string types";
            return false;
          }
          // IndexMap<(String, Location)>::insert
          TN& mm = t.n[m];
          bool replaced = false;
          for (size_t q = 0; q < mm.keys.size(); q++) {
            if (mm.keys[q] == k.s && mm.kmarks[q].first == k.line && mm.kmarks[q].second == k.col) {
              mm.kids[q] = kvs[j + 1]; replaced = true; break;
            }
          }
          if (!replaced) { mm.keys.push_back(k.s); mm.kmarks.push_back({k.line, k.col}); mm.kids.push_back(kvs[j + 1]); }
        }
        break;
      }
      case YAML_SEQUENCE_START_EVENT: {
        if (ev.data.sequence_start.tag) {
          std::string handle, suffix;
          split_tag((const char*)ev.data.sequence_start.tag, handle, suffix);
          if (handle == "!" && is_seq(suffix)) {
            TN nul; nul.kind = K_NULL; nul.line = line; nul.col = col;
            uint32_t ni = t.add(std::move(nul));
            TN m; m.kind = K_MAP; m.line = line; m.col = col;
            m.keys.push_back(long_form(suffix)); m.kmarks.push_back({line, col}); m.kids.push_back(ni);
            stack.push_back(t.add(std::move(m)));
            func_support.push_back({stack.size() - 1, {long_form(suffix), {line, col}}});
          }
        }
        TN n; n.kind = K_LIST; n.line = line; n.col = col;
        stack.push_back(t.add(std::move(n)));
        last_container.push_back((uint32_t)stack.size() - 1);
        break;
      }
      case YAML_SEQUENCE_END_EVENT: {
        uint32_t idx = last_container.back(); last_container.pop_back();
        std::vector<uint32_t> vals(stack.begin() + idx + 1, stack.end());
        stack.resize(idx + 1);
        for (uint32_t v : vals) t.n[stack.back()].kids.push_back(v);
        if (!func_support.empty() && func_support.back().first + 1 == idx) {
          auto fs = func_support.back(); func_support.pop_back();
          uint32_t arr = stack.back(); stack.pop_back();
          TN& mm = t.n[stack.back()];
          if (mm.kind == K_MAP) {
            bool replaced = false;
            for (size_t q = 0; q < mm.keys.size(); q++) {
              if (mm.keys[q] == fs.second.first && mm.kmarks[q] == fs.second.second) { mm.kids[q] = arr; replaced = true; break; }
            }
            if (!replaced) { mm.keys.push_back(fs.second.first); mm.kmarks.push_back(fs.second.second); mm.kids.push_back(arr); }
          }
        }
        break;
      }
      case YAML_SCALAR_EVENT: {
        std::string v = ev_scalar(ev);
        stack.push_back(scalar_node(t, v, (const char*)ev.data.scalar.tag,
                                    ev.data.scalar.style == YAML_PLAIN_SCALAR_STYLE, line, col));
        break;
      }
      case YAML_ALIAS_EVENT:
        yaml_event_delete(&ev);
        err.kind = "ParseError"; err.msg = "Guard does not currently support aliases"; return false;
    }
    yaml_event_delete(&ev);
    if (done) return true;
  }
}

// serde_yaml Value (YAML 1.2) from libyaml events; tags -> handle_tagged_value (values.rs:455-466)
bool serde_yaml_load(const char* text, size_t len, Tree& t, uint32_t& root, std::string& msg) {
  YamlParser yp(text, len);
  struct Frame { bool map; std::vector<uint32_t> items; std::string tag; };
  std::vector<Frame> st;
  st.push_back(Frame{false, {}, ""});
  for (;;) {
    yaml_event_t ev;
    if (yp.p.error != YAML_NO_ERROR || !yaml_parser_parse(&yp.p, &ev)) {
      msg = yp.p.problem ? yp.p.problem : "error parsing YAML"; return false;
    }
    bool done = false;
    auto wrap_tag = [&](uint32_t node, const std::string& tag) -> uint32_t {
      size_t bangs = 0;
      for (char c : tag) if (c == '!') bangs++;
      if (!tag.empty() && tag[0] == '!' && bangs == 1) {
        std::string fn = tag.substr(1);
        if (is_single(fn) || is_seq(fn)) {
          TN m; m.kind = K_MAP; m.keys.push_back(long_form(fn)); m.kmarks.push_back({0, 0}); m.kids.push_back(node);
          return t.add(std::move(m));
        }
      }
      return node;
    };
    switch (ev.type) {
      case YAML_SCALAR_EVENT: {
        std::string v = ev_scalar(ev);
        const char* tg = (const char*)ev.data.scalar.tag;
        bool plain = ev.data.scalar.style == YAML_PLAIN_SCALAR_STYLE;
        uint32_t node;
        if (tg && tg[0] == '!' && std::string(tg) != "!") {
          TN s; s.kind = K_STRING; s.s = v;
          node = wrap_tag(t.add(std::move(s)), tg);
        } else {
          node = serde_yaml_scalar(t, v, plain);
        }
        st.back().items.push_back(node);
        break;
      }
      case YAML_MAPPING_START_EVENT:
        st.push_back(Frame{true, {}, ev.data.mapping_start.tag ? (const char*)ev.data.mapping_start.tag : ""});
        break;
      case YAML_SEQUENCE_START_EVENT:
        st.push_back(Frame{false, {}, ev.data.sequence_start.tag ? (const char*)ev.data.sequence_start.tag : ""});
        break;
      case YAML_MAPPING_END_EVENT: case YAML_SEQUENCE_END_EVENT: {
        Frame f = std::move(st.back()); st.pop_back();
        TN n;
        if (f.map) {
          n.kind = K_MAP;
          for (size_t j = 0; j + 1 < f.items.size(); j += 2) {
            const TN& k = t.n[f.items[j]];
            if (k.kind != K_STRING) { yaml_event_delete(&ev); msg = "non string key"; return false; }
            // serde_yaml 0.9 Mapping::deserialize refuses a repeated key (DuplicateKeyError, "duplicate
            // entry with key {:?}"), so run_checks' YAML fallback fails with a YamlError (code 2);
            // serde_yaml appends a position this loader does not reproduce
            for (const std::string& prev : n.keys)
              if (prev == k.s) { yaml_event_delete(&ev); msg = "duplicate entry with key " + rust_debug_str(k.s); return false; }
            n.keys.push_back(k.s); n.kmarks.push_back({0, 0}); n.kids.push_back(f.items[j + 1]);
          }
        } else {
          n.kind = K_LIST; n.kids = f.items;
        }
        st.back().items.push_back(wrap_tag(t.add(std::move(n)), f.tag));
        break;
      }
      case YAML_ALIAS_EVENT:
        yaml_event_delete(&ev); msg = "aliases are not supported"; return false;
      case YAML_DOCUMENT_END_EVENT: done = true; break;
      case YAML_STREAM_END_EVENT: done = true; break;
      default: break;
    }
    yaml_event_delete(&ev);
    if (done) break;
  }
  if (st.back().items.empty()) { TN n; n.kind = K_NULL; root = t.add(std::move(n)); }
  else root = st.back().items[0];
  return true;
}

// serde_json (preserve_order) strict JSON
struct JsonP {
  const char* s; size_t n; size_t i = 0; Tree& t;
  JsonP(const char* s_, size_t n_, Tree& t_) : s(s_), n(n_), t(t_) {}
  void ws() { while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++; }
  bool str(std::string& out) {
    if (i >= n || s[i] != '"') return false;
    i++;
    while (i < n) {
      unsigned char c = (unsigned char)s[i];
      if (c == '"') { i++; return true; }
      if (c < 0x20) return false;
      if (c == '\\') {
        i++;
        if (i >= n) return false;
        char e = s[i++];
        switch (e) {
          case '"': out.push_back('"'); break;
          case '\\': out.push_back('\\'); break;
          case '/': out.push_back('/'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'n': out.push_back('\n'); break;
          case 'r': out.push_back('\r'); break;
          case 't': out.push_back('\t'); break;
          case 'u': {
            auto hex4 = [&](uint32_t& v) -> bool {
              if (i + 4 > n) return false;
              v = 0;
              for (int k = 0; k < 4; k++) {
                char h = s[i++]; v <<= 4;
                if (h >= '0' && h <= '9') v |= h - '0';
                else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
                else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
                else return false;
              }
              return true;
            };
            uint32_t cp;
            if (!hex4(cp)) return false;
            if (cp >= 0xD800 && cp < 0xDC00) {
              if (i + 2 > n || s[i] != '\\' || s[i + 1] != 'u') return false;
              i += 2;
              uint32_t lo;
              if (!hex4(lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else if (cp >= 0xDC00 && cp <= 0xDFFF) return false;
            utf8_append(out, cp);
            break;
          }
          default: return false;
        }
      } else { out.push_back((char)c); i++; }
    }
    return false;
  }
  bool value(uint32_t& out, int depth) {
    if (depth > 128) return false;
    ws();
    if (i >= n) return false;
    char c = s[i];
    TN node;
    if (c == '{') {
      i++; node.kind = K_MAP; ws();
      if (i < n && s[i] == '}') { i++; out = t.add(std::move(node)); return true; }
      for (;;) {
        ws(); std::string k;
        if (!str(k)) return false;
        ws(); if (i >= n || s[i] != ':') return false; i++;
        uint32_t v; if (!value(v, depth + 1)) return false;
        bool replaced = false;
        for (size_t q = 0; q < node.keys.size(); q++) if (node.keys[q] == k) { node.kids[q] = v; replaced = true; break; }
        if (!replaced) { node.keys.push_back(k); node.kmarks.push_back({0, 0}); node.kids.push_back(v); }
        ws();
        if (i < n && s[i] == ',') { i++; continue; }
        if (i < n && s[i] == '}') { i++; break; }
        return false;
      }
      out = t.add(std::move(node)); return true;
    }
    if (c == '[') {
      i++; node.kind = K_LIST; ws();
      if (i < n && s[i] == ']') { i++; out = t.add(std::move(node)); return true; }
      for (;;) {
        uint32_t v; if (!value(v, depth + 1)) return false;
        node.kids.push_back(v); ws();
        if (i < n && s[i] == ',') { i++; continue; }
        if (i < n && s[i] == ']') { i++; break; }
        return false;
      }
      out = t.add(std::move(node)); return true;
    }
    if (c == '"') { node.kind = K_STRING; if (!str(node.s)) return false; out = t.add(std::move(node)); return true; }
    if (!strncmp(s + i, "true", 4) && i + 4 <= n) { i += 4; node.kind = K_BOOL; node.i = 1; out = t.add(std::move(node)); return true; }
    if (!strncmp(s + i, "false", 5) && i + 5 <= n) { i += 5; node.kind = K_BOOL; node.i = 0; out = t.add(std::move(node)); return true; }
    if (!strncmp(s + i, "null", 4) && i + 4 <= n) { i += 4; node.kind = K_NULL; out = t.add(std::move(node)); return true; }
    // number
    size_t st = i; bool neg = false, isf = false;
    if (s[i] == '-') { neg = true; i++; }
    if (i >= n || !isdigit((unsigned char)s[i])) return false;
    if (s[i] == '0') i++; else while (i < n && isdigit((unsigned char)s[i])) i++;
    if (i < n && s[i] == '.') { isf = true; i++; if (i >= n || !isdigit((unsigned char)s[i])) return false; while (i < n && isdigit((unsigned char)s[i])) i++; }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) { isf = true; i++; if (i < n && (s[i] == '+' || s[i] == '-')) i++; if (i >= n || !isdigit((unsigned char)s[i])) return false; while (i < n && isdigit((unsigned char)s[i])) i++; }
    std::string num(s + st, i - st);
    if (!isf) {
      unsigned __int128 v = 0; bool of = false;
      for (size_t k = neg ? 1 : 0; k < num.size(); k++) { v = v * 10 + (num[k] - '0'); if (v > ((unsigned __int128)1 << 65)) of = true; }
      if (!of) {
        if (neg && v <= ((unsigned __int128)1 << 63)) { node.kind = K_INT; node.i = (int64_t)(-(__int128)v); out = t.add(std::move(node)); return true; }
        if (!neg && v <= (unsigned __int128)UINT64_MAX) { node.kind = K_INT; node.i = (int64_t)(uint64_t)v; out = t.add(std::move(node)); return true; }
      }
    }
    node.kind = K_FLOAT; node.f = strtod(num.c_str(), nullptr);
    if (std::isinf(node.f)) return false;  // serde_json: number out of range
    out = t.add(std::move(node)); return true;
  }
};

}  // namespace

void DocBatch::clear() {
  islots.clear(); ilen.clear(); iused = 0; base.clear();
  nodes.clear(); bytes.clear(); line.clear(); col.clear(); kline.clear(); kcol.clear(); roots.clear(); names.clear();
  serde = false;
}

uint32_t DocBatch::find(const char* p, uint32_t n) const {
  if (islots.empty()) return NONE;
  size_t mask = islots.size() - 1;
  size_t h = fnv1a(p, n) & mask;
  while (islots[h]) {
    if (ilen[h] == n && memcmp(bytes.data() + islots[h] - 1, p, n) == 0) return islots[h] - 1;
    h = (h + 1) & mask;
  }
  return NONE;
}

void DocBatch::intern_reserve() {
  if ((iused + 1) * 2 <= islots.size()) return;
  size_t cap = islots.empty() ? 4096 : islots.size() * 2;
  std::vector<uint32_t> ns(cap, 0), nl(cap, 0);
  for (size_t i = 0; i < islots.size(); i++) {
    if (!islots[i]) continue;
    uint32_t off = islots[i] - 1, len = ilen[i];
    size_t h = fnv1a(bytes.data() + off, len) & (cap - 1);
    while (ns[h]) h = (h + 1) & (cap - 1);
    ns[h] = islots[i]; nl[h] = len;
  }
  islots.swap(ns); ilen.swap(nl);
}

uint32_t DocBatch::intern(const char* p, uint32_t n, uint32_t hash) {
  intern_reserve();
  size_t mask = islots.size() - 1;
  size_t h = hash & mask;
  while (islots[h]) {
    if (ilen[h] == n && memcmp(bytes.data() + islots[h] - 1, p, n) == 0) return islots[h] - 1;
    h = (h + 1) & mask;
  }
  // 16-byte aligned start, zero padding to a 16-byte multiple (device compares in 16-byte chunks);
  // the empty string takes 16 bytes too, so no two distinct strings share an id
  uint32_t off = (uint32_t)bytes.size();
  bytes.append(p, n);
  bytes.append(n ? (16 - (n & 15)) & 15 : 16, '\0');
  islots[h] = off + 1; ilen[h] = n; iused++;
  return off;
}

void DocBatch::adopt(uint32_t off, uint32_t n) {
  intern_reserve();
  size_t mask = islots.size() - 1;
  size_t h = fnv1a(bytes.data() + off, n) & mask;
  while (islots[h]) h = (h + 1) & mask;
  islots[h] = off + 1; ilen[h] = n; iused++;
}

void DocBatch::adopt_bulk(const uint32_t* off, const uint32_t* len, size_t n, unsigned threads) {
  if (!n) return;
  size_t cap = islots.empty() ? 4096 : islots.size();
  while ((iused + n) * 2 > cap) cap *= 2;
  if (cap != islots.size()) {
    // rehash what is there (normally nothing: the device loader fills an empty batch)
    const size_t keep = iused;
    std::vector<uint32_t> old_s, old_l;
    old_s.swap(islots); old_l.swap(ilen);
    islots.assign(cap, 0); ilen.assign(cap, 0);
    iused = 0;
    for (size_t i = 0; i < old_s.size(); i++) if (old_s[i]) adopt(old_s[i] - 1, old_l[i]);
    (void)keep;
  }
  const size_t mask = islots.size() - 1;
  uint32_t* S = islots.data();
  uint32_t* L = ilen.data();
  const char* B = bytes.data();
  threads = std::max(1u, std::min<unsigned>(threads, (unsigned)((n + 65535) / 65536)));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < threads; t++)
    th.emplace_back([=]() {
      for (size_t i = n * t / threads; i < n * (t + 1) / threads; i++) {
        size_t h = fnv1a(B + off[i], len[i]) & mask;
        for (;;) {
          uint32_t expect = 0;
          if (__atomic_compare_exchange_n(&S[h], &expect, off[i] + 1, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
            L[h] = len[i];
            break;
          }
          h = (h + 1) & mask;
        }
      }
    });
  for (auto& x : th) x.join();
  iused += n;
}

std::string DocBatch::path(uint64_t base, uint32_t node) const {
  // JSON-pointer-like path (path_value.rs Path): the node's ancestors' keys / indices, root first
  const DNode* N = nodes.data() + base;
  uint32_t chain[64];
  std::vector<uint32_t> deep;
  size_t n = 0;
  for (uint32_t cur = node; N[cur].parent != NONE; cur = N[cur].parent) {
    if (n < 64) chain[n] = cur; else deep.push_back(cur);
    n++;
  }
  std::string out;
  char num[16];
  for (size_t i = n; i-- > 0;) {
    const uint32_t cur = i < 64 ? chain[i] : deep[i - 64];
    const DNode& p = N[N[cur].parent];
    out.push_back('/');
    if (p.kind == K_MAP) out.append(bytes.data() + N[cur].key_off, N[cur].key_len);
    else { auto r = std::to_chars(num, num + sizeof num, cur - p.a); out.append(num, r.ptr - num); }
  }
  return out;
}

std::string DocBatch::path_display(uint64_t base, uint32_t node) const {
  return path(base, node) + "[L:" + std::to_string(line[base + node]) + ",C:" + std::to_string(col[base + node]) + "]";
}


bool g_json_fast = true;

// ------------------------------------------------------ JSON fast path ---
// Most corpora (CloudFormation JSON, Terraform plan JSON, Config CIs) are strict JSON.  For such a
// document libyaml produces a flow-style event stream whose marks are (line, column) of each
// token's first character and whose plain scalars are exactly the JSON number/true/false/null
// tokens.  This path parses that subset directly into the arena -- same node layout as Emitter
// (each container's children contiguous, blocks in DFS pre-order), same marks, same scalar typing
// -- and returns "not handled" for anything outside the subset it can prove identical: non-ASCII
// or control bytes, tabs/CR, surrogate \u escapes, duplicate keys, a key whose ':' is not on the
// same line within 1000 characters (libyaml simple-key rules), non-container roots, nesting
// deeper than 256.  Unhandled documents take the libyaml path, so results never depend on which
// path ran (tests/test_loader_cpu.py compares both on the corpora).
namespace {

struct JsonFast {
  const char* s;
  size_t n;
  size_t i = 0;
  uint32_t line = 0;
  size_t line_start = 0;
  std::vector<uint32_t> counts;   // pass 1: child count per container, pre-order
  size_t ci = 0;
  std::string sbuf;
  std::vector<uint32_t> khash;    // pass 1 duplicate-key scratch

  JsonFast(const char* t, size_t len) : s(t), n(len) {}

  void ws() {
    while (i < n) {
      char c = s[i];
      if (c == ' ') i++;
      else if (c == '\n') { i++; line++; line_start = i; }
      else break;
    }
  }
  uint32_t col() const { return (uint32_t)(i - line_start); }

  // string token at s[i] == '"'; decodes into sbuf when `decode`
  bool str(bool decode) {
    i++;
    if (decode) sbuf.clear();
    for (;;) {
      if (i >= n) return false;
      unsigned char c = (unsigned char)s[i];
      if (c == '"') { i++; return true; }
      if (c < 0x20 || c > 0x7E) return false;
      if (c != '\\') {
        size_t j = i;
        while (j < n && s[j] != '"' && s[j] != '\\' && (unsigned char)s[j] >= 0x20 && (unsigned char)s[j] <= 0x7E) j++;
        if (decode) sbuf.append(s + i, j - i);
        i = j;
        continue;
      }
      if (i + 1 >= n) return false;
      char e = s[i + 1];
      char out;
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
          if (i + 6 > n) return false;
          uint32_t cp = 0;
          for (int k = 0; k < 4; k++) {
            char h = s[i + 2 + k];
            cp <<= 4;
            if (h >= '0' && h <= '9') cp |= (uint32_t)(h - '0');
            else if (h >= 'a' && h <= 'f') cp |= (uint32_t)(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F') cp |= (uint32_t)(h - 'A' + 10);
            else return false;
          }
          if (cp >= 0xD800 && cp <= 0xDFFF) return false;
          if (decode) utf8_append(sbuf, cp);
          i += 6;
          continue;
        }
        default: return false;
      }
      if (decode) sbuf.push_back(out);
      i += 2;
    }
  }

  // plain token (JSON number / true / false / null): returns its length, 0 if not one
  size_t plain_len() const {
    size_t j = i;
    if (j < n && (s[j] == 't' || s[j] == 'f' || s[j] == 'n')) {
      static const char* words[] = {"true", "false", "null"};
      for (const char* w : words) {
        size_t L = strlen(w);
        if (j + L <= n && memcmp(s + j, w, L) == 0) return L;
      }
      return 0;
    }
    if (j < n && s[j] == '-') j++;
    if (j >= n) return 0;
    if (s[j] == '0') j++;
    else if (s[j] >= '1' && s[j] <= '9') { while (j < n && isdigit((unsigned char)s[j])) j++; }
    else return 0;
    if (j < n && s[j] == '.') {
      j++;
      size_t d = j;
      while (j < n && isdigit((unsigned char)s[j])) j++;
      if (j == d) return 0;
    }
    if (j < n && (s[j] == 'e' || s[j] == 'E')) {
      j++;
      if (j < n && (s[j] == '+' || s[j] == '-')) j++;
      size_t d = j;
      while (j < n && isdigit((unsigned char)s[j])) j++;
      if (j == d) return 0;
    }
    return j - i;
  }
  bool after_plain_ok(size_t j) const {
    return j >= n || s[j] == ' ' || s[j] == '\n' || s[j] == ',' || s[j] == ']' || s[j] == '}';
  }

  // pass 1: validate the subset and record container sizes
  bool v1(int depth) {
    if (depth > 256 || i >= n) return false;
    char c = s[i];
    if (c == '"') return str(false);
    if (c == '{' || c == '[') {
      bool map = c == '{';
      size_t slot = counts.size();
      counts.push_back(0);
      i++;
      ws();
      char close = map ? '}' : ']';
      if (i < n && s[i] == close) { i++; return true; }
      uint32_t cnt = 0;
      size_t kbase = khash.size();
      for (;;) {
        if (map) {
          if (i >= n || s[i] != '"') return false;
          size_t kstart = i;
          uint32_t kline = line;
          if (!str(true)) return false;
          uint32_t h = fnv1a(sbuf.data(), sbuf.size());
          if (khash.size() - kbase <= 64)
            for (size_t q = kbase; q < khash.size(); q++) if (khash[q] == h) return false;  // possible duplicate
          khash.push_back(h);
          while (i < n && s[i] == ' ') i++;
          if (i >= n || s[i] != ':' || line != kline || i - kstart > 1000) return false;
          i++;
          ws();
        }
        if (!v1(depth + 1)) return false;
        cnt++;
        ws();
        if (i < n && s[i] == ',') { i++; ws(); continue; }
        if (i < n && s[i] == close) { i++; break; }
        return false;
      }
      if (khash.size() - kbase > 64) {
        std::sort(khash.begin() + kbase, khash.end());
        for (size_t q = kbase + 1; q < khash.size(); q++) if (khash[q] == khash[q - 1]) return false;
      }
      khash.resize(kbase);
      counts[slot] = cnt;
      return true;
    }
    size_t L = plain_len();
    if (!L || !after_plain_ok(i + L)) return false;
    i += L;
    return true;
  }

  // pass 2: emit into the arena; `slot` already allocated by the parent (global index);
  // stored child/parent indices are relative to the document's first node `dbase`
  uint64_t dbase = 0;
  void v2(DocBatch& b, size_t slot, uint32_t parent) {
    DNode& d = b.nodes[slot];
    d.parent = parent;
    d.count = 0; d.a = 0; d.b = 0;
    char c = s[i];
    if (c == '"') {
      str(true);
      d.kind = K_STRING;
      d.count = (uint32_t)sbuf.size();
      d.a = b.intern(sbuf.data(), d.count, fnv1a(sbuf.data(), sbuf.size()));
      d.b = d.a;
      return;
    }
    if (c == '{' || c == '[') {
      bool map = c == '{';
      uint32_t cnt = counts[ci++];
      size_t first = b.nodes.size();
      size_t sz = first + (size_t)cnt;
      b.nodes.resize(sz); b.line.resize(sz); b.col.resize(sz); b.kline.resize(sz); b.kcol.resize(sz);
      DNode& dd = b.nodes[slot];
      dd.kind = map ? K_MAP : K_LIST;
      dd.a = (uint32_t)(first - dbase); dd.count = cnt;
      i++;
      ws();
      for (uint32_t j = 0; j < cnt; j++) {
        size_t cs = first + j;
        if (map) {
          uint32_t kl = line, kc = col();
          str(true);
          DNode& e = b.nodes[cs];
          e.key_len = (uint32_t)sbuf.size();
          e.key_off = b.intern(sbuf.data(), e.key_len, fnv1a(sbuf.data(), sbuf.size()));
          e.key_hash = e.key_off;
          b.kline[cs] = kl; b.kcol[cs] = kc;
          while (s[i] == ' ') i++;
          i++;  // ':'
          ws();
        } else {
          DNode& e = b.nodes[cs];
          e.key_off = NONE; e.key_len = 0; e.key_hash = 0;
          b.kline[cs] = 0; b.kcol[cs] = 0;
        }
        b.line[cs] = line; b.col[cs] = col();
        v2(b, cs, (uint32_t)(slot - dbase));
        ws();
        i++;  // ',' or the closing bracket
        ws();
      }
      if (!cnt) i++;   // empty container: closing bracket (pass 1 skipped whitespace the same way)
      return;
    }
    size_t L = plain_len();
    std::string tok(s + i, L);
    i += L;
    int64_t iv; double fv;
    if (tok == "true") { d.kind = K_BOOL; d.a = 1; }
    else if (tok == "false") { d.kind = K_BOOL; d.a = 0; }
    else if (tok == "null") { d.kind = K_NULL; }
    else if (rust_parse_i64(tok, iv)) { d.kind = K_INT; uint64_t u = (uint64_t)iv; d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32); }
    else { rust_parse_f64(tok, fv); d.kind = K_FLOAT; uint64_t u; memcpy(&u, &fv, 8); d.a = (uint32_t)u; d.b = (uint32_t)(u >> 32); }
  }
};

}  // namespace

// returns true when the document was loaded by the fast path; false leaves `b` unchanged
static bool load_json_fast(DocBatch& b, const char* text, size_t len, const std::string& name) {
  JsonFast p(text, len);
  p.ws();
  if (p.i >= len || (text[p.i] != '{' && text[p.i] != '[')) return false;
  size_t start = p.i;
  uint32_t sline = p.line, scol = p.col();
  size_t sls = p.line_start;
  if (!p.v1(0)) return false;
  p.ws();
  if (p.i != len) return false;
  if (len + 1 > kMaxDocNodes) return false;
  // pass 2
  p.i = start; p.line = sline; p.line_start = sls; p.ci = 0;
  size_t slot = b.nodes.size();
  p.dbase = slot;
  size_t sz = slot + 1;
  b.nodes.resize(sz); b.line.resize(sz); b.col.resize(sz); b.kline.resize(sz); b.kcol.resize(sz);
  b.nodes[slot].key_off = NONE; b.nodes[slot].key_len = 0; b.nodes[slot].key_hash = 0;
  bool list = text[start] == '[';
  b.line[slot] = list ? 0 : sline; b.col[slot] = list ? 0 : scol;   // emit_root: lists keep Path::root()'s (0,0)
  b.kline[slot] = 0; b.kcol[slot] = 0;
  p.v2(b, slot, NONE);
  b.roots.push_back(0);
  b.base.push_back(slot);
  b.names.push_back(name);
  return true;
}

bool load_document(DocBatch& b, const char* text, size_t len, const std::string& name, LoadMode mode, LoadError& err) {
  Tree t;
  uint32_t root = 0;
  // u32 arena offsets: refuse a document that could push the pool or node count past the cap
  if (b.bytes.size() + len > kMaxPoolBytes) {
    err.kind = "IncompatibleError";
    err.msg = "document batch is full (u32 arena offsets); evaluate it and start a new batch";
    return false;
  }
  if (mode == LOAD_LIBYAML) {
    if (g_json_fast && load_json_fast(b, text, len, name)) return true;
    bool blank = true;
    for (size_t k = 0; k < len; k++) if (!isspace((unsigned char)text[k])) { blank = false; break; }
    if (blank) {
      err.kind = "ParseError";
      err.msg = "Unable to parse a template from data file: " + name + " is empty";
      return false;
    }
    if (!libyaml_load(text, len, t, root, err)) {
      if (err.kind == "InternalError") { err.kind = "ParseError"; return false; }
      size_t l = len < 100 ? len : 100;
      err.kind = "ParseError";
      err.msg = "Error encountered while parsing data file: " + name + ", data beginning with \n" +
                std::string(text, l) + "\n ...";
      return false;
    }
    return emit_root(b, t, root, name, false, err);
  }
  // serde: JSON first, then YAML (commands/helper.rs:30-42)
  JsonP jp(text, len, t);
  bool ok = jp.value(root, 0);
  if (ok) { jp.ws(); ok = jp.i == len; }
  if (!ok) {
    t.n.clear();
    std::string msg;
    if (!serde_yaml_load(text, len, t, root, msg)) {
      err.kind = "YamlError"; err.msg = msg; return false;
    }
  }
  b.serde = true;
  return emit_root(b, t, root, name, true, err);
}

// ------------------------------------------------------ input parameters ---
namespace {
const char* merge_type_info(uint32_t k) {   // PathAwareValue::type_info (path_value.rs:985-1000)
  static const char* t[] = {"null", "String", "Regex", "bool", "int", "float", "char", "array", "map",
                            "range(int, int)", "range(float, float)", "range(char, char)"};
  return k < 12 ? t[k] : "?";
}
}  // namespace

bool merge_into_last(DocBatch& b, size_t d, const DocBatch& P, size_t pd, LoadError& err) {
  const uint64_t base = b.base[d];
  const uint64_t pbase = P.base[pd];
  const uint64_t pend = pd + 1 < P.base.size() ? P.base[pd + 1] : P.nodes.size();
  const uint32_t np = (uint32_t)(pend - pbase);
  const DNode A = P.nodes[pbase + P.roots[pd]];     // self
  const DNode Bn = b.nodes[base + b.roots[d]];       // other
  const uint32_t broot = b.roots[d];
  if (!((A.kind == K_MAP && Bn.kind == K_MAP) || (A.kind == K_LIST && Bn.kind == K_LIST))) {
    err.kind = "IncompatibleError";
    err.msg = std::string("Types are not compatible for merges ") + merge_type_info(A.kind) + ", " + merge_type_info(Bn.kind);
    return false;
  }
  auto pkey = [&](const DNode& e) { return std::string(P.bytes.data() + e.key_off, e.key_len); };
  if (A.kind == K_MAP) {
    // `for (key, value) in other_map.values`: the first of other's keys that self already holds
    std::unordered_map<std::string, int> have;
    for (uint32_t j = 0; j < A.count; j++) have[pkey(P.nodes[pbase + A.a + j])] = 1;
    for (uint32_t j = 0; j < Bn.count; j++) {
      const DNode& e = b.nodes[base + Bn.a + j];
      std::string k(b.bytes.data() + e.key_off, e.key_len);
      if (have.count(k)) { err.kind = "MultipleValues"; err.msg = "Key " + k + ", already exists in map"; return false; }
    }
  }
  const uint64_t rel0 = b.nodes.size() - base;   // relative index of the first appended node
  if (rel0 + np + 8 + 2ull * (A.count + Bn.count) + (A.kind == K_MAP && A.b ? P.nodes[pbase + A.b].count : 0) > kMaxDocNodes) {
    err.kind = "IncompatibleError"; err.msg = "document too large for the MI355X arena"; return false;
  }
  const uint32_t O = (uint32_t)rel0;
  // 1. self's nodes, rebased to O, strings re-interned into b's pool
  b.grow_zeroed(base + rel0 + np);
  std::unordered_map<uint32_t, uint32_t> sid;   // P string id -> b string id
  auto str_id = [&](uint32_t off, uint32_t len) {
    auto it = sid.find(off);
    if (it != sid.end()) return it->second;
    const uint32_t id = b.intern(P.bytes.data() + off, len, fnv1a(P.bytes.data() + off, len));
    sid[off] = id;
    return id;
  };
  for (uint32_t i = 0; i < np; i++) {
    DNode n = P.nodes[pbase + i];
    const size_t g = base + rel0 + i;
    if (n.kind == K_LIST || n.kind == K_MAP) { n.a += O; if (n.kind == K_MAP && n.b) n.b += O; }
    if (n.kind == K_STRING || n.kind == K_REGEX) { n.a = str_id(n.a, n.count); n.b = n.a; }
    if (n.key_off != NONE) { n.key_off = str_id(n.key_off, n.key_len); n.key_hash = n.key_off; }
    if (n.parent != NONE) n.parent += O;
    b.nodes[g] = n;
    b.line[g] = P.line[pbase + i]; b.col[g] = P.col[pbase + i];
    b.kline[g] = P.kline[pbase + i]; b.kcol[g] = P.kcol[pbase + i];
  }
  const uint32_t aroot = O + P.roots[pd];
  const DNode Ar = b.nodes[base + aroot];
  // 2. the merged root, then its entries: self's, then other's (shallow copies: their subtrees stay)
  const uint32_t R = O + np, E = R + 1, n = Ar.count + Bn.count;
  b.grow_zeroed(base + E + n);
  {
    DNode& r = b.nodes[base + R];
    r.kind = Ar.kind; r.count = n; r.a = E; r.b = 0; r.key_off = NONE; r.key_len = 0; r.key_hash = 0; r.parent = NONE;
    b.line[base + R] = b.line[base + aroot]; b.col[base + R] = b.col[base + aroot];   // self's location
  }
  for (uint32_t j = 0; j < n; j++) {
    const bool mine = j < Ar.count;
    const uint64_t src = base + (mine ? Ar.a + j : Bn.a + (j - Ar.count));
    const uint64_t g = base + E + j;
    b.nodes[g] = b.nodes[src];
    b.line[g] = b.line[src]; b.col[g] = b.col[src];
    if (Ar.kind == K_MAP) {
      b.nodes[g].parent = R;
      if (mine) { b.kline[g] = b.kline[src]; b.kcol[g] = b.kcol[src]; }
      else {
        // map.keys.push(String((path.extend_str(&key), key))): other's root path + "/key" at other's location
        b.kline[g] = b.line[base + broot] | kKeyPathExt; b.kcol[g] = b.col[base + broot];
      }
    } else {
      b.kline[g] = 0; b.kcol[g] = 0;
    }
  }
  if (Ar.kind == K_LIST) {
    // vec.extend: the elements keep their own paths (their index in the list they came from), so
    // each side's copies hang under a detached list node whose first child is the side's first copy
    const uint32_t V = E + n;
    b.grow_zeroed(base + V + 2);
    for (uint32_t k = 0; k < 2; k++) {
      DNode& v = b.nodes[base + V + k];
      v.kind = K_LIST; v.count = k ? Bn.count : Ar.count; v.a = k ? E + Ar.count : E; v.parent = NONE;
      v.key_off = NONE; v.key_len = 0; v.key_hash = 0;
    }
    for (uint32_t j = 0; j < n; j++) b.nodes[base + E + j].parent = j < Ar.count ? V : V + 1;
  } else if (Ar.b) {
    // self keeps a key block (a repeated key): the merged keys are self's keys, then other's
    const uint32_t na = b.nodes[base + Ar.b].count, nk = na + Bn.count, K = E + n;
    b.grow_zeroed(base + K + nk);
    for (uint32_t j = 0; j < nk; j++) {
      const uint64_t g = base + K + j;
      const uint64_t src = j < na ? base + Ar.b + j : base + E + Ar.count + (j - na);
      DNode k = b.nodes[src];
      DNode& kn = b.nodes[g];
      kn = DNode{};
      kn.kind = K_NULL; kn.count = nk; kn.parent = R;
      kn.key_off = k.key_off; kn.key_len = k.key_len; kn.key_hash = k.key_hash;
      b.kline[g] = b.kline[src]; b.kcol[g] = b.kcol[src];
    }
    b.nodes[base + R].b = K;
  }
  b.roots[d] = R;
  return true;
}

// test hook: 1 when the fast path accepts `text` and builds exactly the libyaml path's arena,
// 0 when they differ, -1 when the fast path declines (or libyaml fails)
int loader_selfcheck(const char* text, size_t len) {
  DocBatch a, b;
  LoadError e;
  if (!load_json_fast(a, text, len, "x")) return -1;
  bool saved = g_json_fast;
  g_json_fast = false;
  bool ok = load_document(b, text, len, "x", LOAD_LIBYAML, e);
  g_json_fast = saved;
  if (!ok) return -1;
  if (a.nodes.size() != b.nodes.size() || a.bytes != b.bytes || a.roots != b.roots || a.base != b.base || a.line != b.line ||
      a.col != b.col || a.kline != b.kline || a.kcol != b.kcol)
    return 0;
  return memcmp(a.nodes.data(), b.nodes.data(), a.nodes.size() * sizeof(DNode)) == 0 ? 1 : 0;
}

}  // namespace gg
