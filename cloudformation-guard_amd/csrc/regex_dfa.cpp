// Rule regex -> byte DFA (see regex_dfa.h).
#include "regex_dfa.h"

#include <algorithm>
#include <map>
#include <memory>
#include <set>

namespace gg {

namespace {

struct RxErr { std::string why; bool unsupported; };

struct Rng { uint32_t lo, hi; };

struct RNode {
  enum K { Empty, Set, Concat, Alt, Repeat } k = Empty;
  std::vector<Rng> set;                      // code point ranges
  std::vector<std::unique_ptr<RNode>> kids;
  int min = 0, max = -1;                     // Repeat
};

void normalize(std::vector<Rng>& v) {
  std::sort(v.begin(), v.end(), [](const Rng& a, const Rng& b) { return a.lo < b.lo; });
  std::vector<Rng> out;
  for (auto& r : v) {
    if (!out.empty() && r.lo <= out.back().hi + 1) out.back().hi = std::max(out.back().hi, r.hi);
    else out.push_back(r);
  }
  v = out;
}

std::vector<Rng> negate(std::vector<Rng> v) {
  normalize(v);
  std::vector<Rng> out;
  uint32_t next = 0;
  for (auto& r : v) {
    if (r.lo > next) out.push_back({next, r.lo - 1});
    next = r.hi + 1;
  }
  if (next <= 0x10FFFF) out.push_back({next, 0x10FFFF});
  return out;
}

struct RxParser {
  const std::string& p;
  size_t i = 0;
  bool icase = false, dotall = false;
  bool ascii_only = false;
  bool start_anchor = false, end_anchor = false;
  int depth = 0;
  explicit RxParser(const std::string& s) : p(s) {}

  [[noreturn]] void unsup(const std::string& w) { throw RxErr{w, true}; }
  [[noreturn]] void invalid(const std::string& w) { throw RxErr{w, false}; }

  uint32_t next_cp() {
    unsigned char c = (unsigned char)p[i];
    if (c < 0x80) { i++; return c; }
    uint32_t cp; int len;
    if ((c >> 5) == 6) { cp = c & 0x1F; len = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; len = 3; }
    else { cp = c & 0x07; len = 4; }
    for (int k = 1; k < len && i + k < p.size(); k++) cp = (cp << 6) | ((unsigned char)p[i + k] & 0x3F);
    i += len;
    return cp;
  }

  void add_literal(std::vector<Rng>& set, uint32_t cp) {
    set.push_back({cp, cp});
    if (icase) {
      if (cp >= 'a' && cp <= 'z') set.push_back({cp - 32, cp - 32});
      else if (cp >= 'A' && cp <= 'Z') set.push_back({cp + 32, cp + 32});
      if (cp >= 0x80 || cp == 'k' || cp == 'K' || cp == 's' || cp == 'S') ascii_only = true;
    }
  }

  std::vector<Rng> perl_class(char c) {
    std::vector<Rng> s;
    switch (c) {
      case 'd': case 'D': s = {{'0', '9'}}; break;
      case 'w': case 'W': s = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}; break;
      case 's': case 'S': s = {{'\t', '\r'}, {' ', ' '}}; break;
    }
    ascii_only = true;
    if (c == 'D' || c == 'W' || c == 'S') s = negate(s);
    return s;
  }

  uint32_t hex_escape(char kind) {
    // \xNN  \x{...}  \uNNNN  \u{...}  \UNNNNNNNN \U{...}
    int fixed = kind == 'x' ? 2 : kind == 'u' ? 4 : 8;
    uint32_t v = 0;
    auto hexv = [&](char h) -> int {
      if (h >= '0' && h <= '9') return h - '0';
      if (h >= 'a' && h <= 'f') return h - 'a' + 10;
      if (h >= 'A' && h <= 'F') return h - 'A' + 10;
      return -1;
    };
    if (i < p.size() && p[i] == '{') {
      i++;
      int cnt = 0;
      while (i < p.size() && p[i] != '}') { int h = hexv(p[i]); if (h < 0) invalid("bad hex"); v = v * 16 + h; i++; cnt++; }
      if (i >= p.size() || cnt == 0) invalid("bad hex");
      i++;
    } else {
      for (int k = 0; k < fixed; k++) {
        if (i >= p.size()) invalid("bad hex");
        int h = hexv(p[i]); if (h < 0) invalid("bad hex");
        v = v * 16 + h; i++;
      }
    }
    if (v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) invalid("bad code point");
    return v;
  }

  // parses an escape after '\'; returns true + set when it is a class/literal
  std::vector<Rng> escape(bool in_class) {
    if (i >= p.size()) invalid("trailing backslash");
    char c = p[i++];
    std::vector<Rng> s;
    switch (c) {
      case 'd': case 'D': case 'w': case 'W': case 's': case 'S': return perl_class(c);
      case 'n': add_literal(s, '\n'); return s;
      case 't': add_literal(s, '\t'); return s;
      case 'r': add_literal(s, '\r'); return s;
      case 'f': add_literal(s, '\f'); return s;
      case 'v': add_literal(s, '\v'); return s;
      case 'a': add_literal(s, 7); return s;
      case 'x': case 'u': case 'U': add_literal(s, hex_escape(c)); return s;
      case 'p': case 'P': unsup("unicode property class");
      case 'b': case 'B': if (in_class) invalid("\\b in class"); unsup("word boundary");
      case 'A': case 'z': unsup("anchor");  // handled by caller at pattern ends
      case 'k': unsup("backreference");
      default:
        if (c >= '0' && c <= '9') unsup("backreference");
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) invalid("unknown escape");
        add_literal(s, (unsigned char)c);
        return s;
    }
  }

  std::vector<Rng> bracket() {
    // after '['
    bool neg = false;
    std::vector<Rng> set;
    if (i < p.size() && p[i] == '^') { neg = true; i++; }
    bool first = true;
    while (true) {
      if (i >= p.size()) invalid("unclosed class");
      if (p[i] == ']' && !first) { i++; break; }
      first = false;
      if (p[i] == '[') {
        if (i + 1 < p.size() && p[i + 1] == ':') {
          size_t end = p.find(":]", i + 2);
          if (end == std::string::npos) invalid("bad posix class");
          std::string name = p.substr(i + 2, end - i - 2);
          i = end + 2;
          bool pneg = false;
          if (!name.empty() && name[0] == '^') { pneg = true; name = name.substr(1); }
          std::vector<Rng> ps;
          if (name == "alpha") ps = {{'A', 'Z'}, {'a', 'z'}};
          else if (name == "digit") ps = {{'0', '9'}};
          else if (name == "alnum") ps = {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}};
          else if (name == "upper") ps = {{'A', 'Z'}};
          else if (name == "lower") ps = {{'a', 'z'}};
          else if (name == "space") ps = {{'\t', '\r'}, {' ', ' '}};
          else if (name == "xdigit") ps = {{'0', '9'}, {'A', 'F'}, {'a', 'f'}};
          else if (name == "punct") ps = {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}};
          else if (name == "word") ps = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
          else unsup("posix class " + name);
          if (pneg) ps = negate(ps);
          set.insert(set.end(), ps.begin(), ps.end());
          continue;
        }
        unsup("nested class");
      }
      if (p[i] == '&' && i + 1 < p.size() && p[i + 1] == '&') unsup("class intersection");
      if (p[i] == '-' && i + 1 < p.size() && p[i + 1] == '-') unsup("class difference");
      if (p[i] == '~' && i + 1 < p.size() && p[i + 1] == '~') unsup("class symmetric difference");
      // single item
      std::vector<Rng> item;
      uint32_t lo;
      bool is_lit = true;
      if (p[i] == '\\') {
        i++;
        size_t save = i;
        char c = i < p.size() ? p[i] : 0;
        if (c == 'd' || c == 'D' || c == 'w' || c == 'W' || c == 's' || c == 'S') {
          item = escape(true); is_lit = false; lo = 0;
        } else {
          i = save;
          bool ic = icase; icase = false;
          std::vector<Rng> e = escape(true);
          icase = ic;
          lo = e[0].lo;
        }
      } else {
        lo = next_cp();
      }
      if (is_lit && i + 1 < p.size() && p[i] == '-' && p[i + 1] != ']') {
        i++;
        uint32_t hi;
        if (p[i] == '\\') { i++; bool ic = icase; icase = false; std::vector<Rng> e = escape(true); icase = ic; hi = e[0].lo; }
        else hi = next_cp();
        if (hi < lo) invalid("bad range");
        set.push_back({lo, hi});
        if (icase) {
          for (uint32_t c = std::max<uint32_t>(lo, 'a'); c <= std::min<uint32_t>(hi, 'z'); c++) set.push_back({c - 32, c - 32});
          for (uint32_t c = std::max<uint32_t>(lo, 'A'); c <= std::min<uint32_t>(hi, 'Z'); c++) set.push_back({c + 32, c + 32});
          if (hi >= 0x80 || (lo <= 'k' && hi >= 'k') || (lo <= 's' && hi >= 's') || (lo <= 'K' && hi >= 'K') || (lo <= 'S' && hi >= 'S')) ascii_only = true;
        }
      } else if (is_lit) {
        add_literal(set, lo);
      } else {
        set.insert(set.end(), item.begin(), item.end());
      }
    }
    normalize(set);
    if (neg) { set = negate(set); if (icase) ascii_only = true; }
    return set;
  }

  std::unique_ptr<RNode> alt() {
    auto first = concat();
    if (i < p.size() && p[i] == '|') {
      auto n = std::make_unique<RNode>(); n->k = RNode::Alt;
      n->kids.push_back(std::move(first));
      while (i < p.size() && p[i] == '|') { i++; n->kids.push_back(concat()); }
      return n;
    }
    return first;
  }

  std::unique_ptr<RNode> concat() {
    auto n = std::make_unique<RNode>(); n->k = RNode::Concat;
    while (i < p.size() && p[i] != '|' && p[i] != ')') {
      auto atom_ = atom();
      if (!atom_) continue;
      // quantifiers
      while (i < p.size()) {
        int mn = -2, mx = -1;
        char c = p[i];
        if (c == '*') { mn = 0; mx = -1; i++; }
        else if (c == '+') { mn = 1; mx = -1; i++; }
        else if (c == '?') { mn = 0; mx = 1; i++; }
        else if (c == '{') {
          size_t save = i;
          i++;
          auto num = [&](int& v) -> bool {
            size_t s0 = i; v = 0;
            while (i < p.size() && isdigit((unsigned char)p[i])) { v = v * 10 + (p[i] - '0'); if (v > 100000) v = 100000; i++; }
            return i > s0;
          };
          int a, b;
          if (num(a)) {
            if (i < p.size() && p[i] == '}') { mn = a; mx = a; i++; }
            else if (i < p.size() && p[i] == ',') {
              i++;
              if (i < p.size() && p[i] == '}') { mn = a; mx = -1; i++; }
              else if (num(b) && i < p.size() && p[i] == '}') { mn = a; mx = b; i++; if (b < a) invalid("bad repetition"); }
              else { i = save; break; }
            } else { i = save; break; }
          } else { i = save; break; }
        } else break;
        if (i < p.size() && p[i] == '?') i++;          // lazy: same language
        else if (i < p.size() && p[i] == '+') unsup("possessive quantifier");
        if (mn > 1000 || mx > 1000) unsup("large repetition");
        auto r = std::make_unique<RNode>(); r->k = RNode::Repeat; r->min = mn; r->max = mx;
        r->kids.push_back(std::move(atom_));
        atom_ = std::move(r);
      }
      n->kids.push_back(std::move(atom_));
    }
    return n;
  }

  std::unique_ptr<RNode> set_node(std::vector<Rng> s) {
    auto n = std::make_unique<RNode>(); n->k = RNode::Set; normalize(s); n->set = s; return n;
  }

  std::unique_ptr<RNode> atom() {
    char c = p[i];
    if (c == '(') {
      i++;
      bool save_icase = icase, save_dotall = dotall;
      if (i < p.size() && p[i] == '?') {
        i++;
        if (i >= p.size()) invalid("bad group");
        char g = p[i];
        if (g == '=' || g == '!') unsup("lookahead");
        if (g == '<' && i + 1 < p.size() && (p[i + 1] == '=' || p[i + 1] == '!')) unsup("lookbehind");
        if (g == '>') unsup("atomic group");
        if (g == 'P' || g == '<') {
          // named group (?P<name>...) / (?<name>...)
          size_t close = p.find('>', i);
          if (close == std::string::npos) invalid("bad group name");
          i = close + 1;
        } else {
          // flags
          bool neg = false;
          bool scoped = false;
          while (i < p.size() && p[i] != ')' && p[i] != ':') {
            char f = p[i++];
            if (f == '-') { neg = true; continue; }
            if (f == 'i') icase = !neg;
            else if (f == 's') dotall = !neg;
            else if (f == 'x' || f == 'm' || f == 'U' || f == 'R' || f == 'u') unsup(std::string("flag ") + f);
            else invalid("bad flag");
          }
          if (i >= p.size()) invalid("bad group");
          if (p[i] == ')') { i++; return nullptr; }  // flags apply to the rest of the enclosing group
          scoped = true;
          i++;  // ':'
          (void)scoped;
        }
      }
      depth++;
      auto inner = alt();
      depth--;
      if (i >= p.size() || p[i] != ')') invalid("unclosed group");
      i++;
      icase = save_icase; dotall = save_dotall;
      return inner;
    }
    if (c == ')') invalid("unopened group");
    if (c == '[') { i++; return set_node(bracket()); }
    if (c == '.') {
      i++;
      if (dotall) return set_node({{0, 0x10FFFF}});
      return set_node({{0, 9}, {11, 0x10FFFF}});
    }
    if (c == '^') {
      if (i == 0) { start_anchor = true; i++; return nullptr; }
      unsup("mid-pattern ^");
    }
    if (c == '$') {
      if (i + 1 == p.size() && depth == 0) { end_anchor = true; i++; return nullptr; }
      unsup("mid-pattern $");
    }
    if (c == '\\') {
      i++;
      if (i < p.size() && p[i] == 'A') { if (i == 1) { start_anchor = true; i++; return nullptr; } unsup("mid-pattern \\A"); }
      if (i < p.size() && p[i] == 'z') { if (i + 1 == p.size() && depth == 0) { end_anchor = true; i++; return nullptr; } unsup("mid-pattern \\z"); }
      return set_node(escape(false));
    }
    if (c == '*' || c == '+' || c == '?') invalid("repetition operator missing expression");
    std::vector<Rng> s;
    add_literal(s, next_cp());
    return set_node(s);
  }
};

// ------------------------------------------------------------------ NFA ----
struct NState { int type; uint8_t lo, hi; int out, out2; };  // type 0 byte, 1 split, 2 match, 3 eps
struct Nfa {
  std::vector<NState> s;
  int add(int type, uint8_t lo = 0, uint8_t hi = 0, int out = -1, int out2 = -1) {
    s.push_back({type, lo, hi, out, out2});
    return (int)s.size() - 1;
  }
};
struct Frag { int start; std::vector<int*> outs; };

void utf8_encode(uint32_t cp, uint8_t* b, int& n) {
  if (cp < 0x80) { b[0] = (uint8_t)cp; n = 1; }
  else if (cp < 0x800) { b[0] = 0xC0 | (cp >> 6); b[1] = 0x80 | (cp & 0x3F); n = 2; }
  else if (cp < 0x10000) { b[0] = 0xE0 | (cp >> 12); b[1] = 0x80 | ((cp >> 6) & 0x3F); b[2] = 0x80 | (cp & 0x3F); n = 3; }
  else { b[0] = 0xF0 | (cp >> 18); b[1] = 0x80 | ((cp >> 12) & 0x3F); b[2] = 0x80 | ((cp >> 6) & 0x3F); b[3] = 0x80 | (cp & 0x3F); n = 4; }
}

void utf8_seqs(uint32_t lo, uint32_t hi, std::vector<std::vector<std::pair<uint8_t, uint8_t>>>& out) {
  if (lo > hi) return;
  if (lo <= 0xDFFF && hi >= 0xD800) {
    if (lo < 0xD800) utf8_seqs(lo, 0xD7FF, out);
    if (hi > 0xDFFF) utf8_seqs(0xE000, hi, out);
    return;
  }
  const uint32_t maxes[] = {0x7F, 0x7FF, 0xFFFF};
  for (uint32_t m : maxes) if (lo <= m && hi > m) { utf8_seqs(lo, m, out); utf8_seqs(m + 1, hi, out); return; }
  if (hi <= 0x7F) { out.push_back({{(uint8_t)lo, (uint8_t)hi}}); return; }
  for (int k = 1; k < 4; k++) {
    uint32_t m = (1u << (6 * k)) - 1;
    if ((lo & ~m) != (hi & ~m)) {
      if ((lo & m) != 0) { utf8_seqs(lo, lo | m, out); utf8_seqs((lo | m) + 1, hi, out); return; }
      if ((hi & m) != m) { utf8_seqs(lo, (hi & ~m) - 1, out); utf8_seqs(hi & ~m, hi, out); return; }
    }
  }
  uint8_t a[4], b[4]; int na, nb;
  utf8_encode(lo, a, na); utf8_encode(hi, b, nb);
  std::vector<std::pair<uint8_t, uint8_t>> seq;
  for (int k = 0; k < na; k++) seq.push_back({a[k], b[k]});
  out.push_back(seq);
}

struct Builder {
  Nfa& nfa;
  // returns (start, list of dangling out pointers as state indices + which field)
  struct F { int start; std::vector<std::pair<int, int>> outs; };  // (state, field 0/1)
  void patch(const F& f, int target) {
    for (auto& o : f.outs) { if (o.second == 0) nfa.s[o.first].out = target; else nfa.s[o.first].out2 = target; }
  }
  F eps() { int s = nfa.add(3); return F{s, {{s, 0}}}; }
  F build(const RNode& n) {
    switch (n.k) {
      case RNode::Empty: return eps();
      case RNode::Set: {
        std::vector<std::vector<std::pair<uint8_t, uint8_t>>> seqs;
        for (auto& r : n.set) utf8_seqs(r.lo, r.hi, seqs);
        if (seqs.empty()) {  // empty class never matches
          int s = nfa.add(0, 1, 0);  // lo > hi: impossible
          return F{s, {{s, 0}}};
        }
        // alternation of byte sequences
        std::vector<F> alts;
        for (auto& sq : seqs) {
          int first = -1, prev = -1;
          for (auto& br : sq) {
            int st = nfa.add(0, br.first, br.second);
            if (first < 0) first = st;
            if (prev >= 0) nfa.s[prev].out = st;
            prev = st;
          }
          alts.push_back(F{first, {{prev, 0}}});
        }
        return alt_of(alts);
      }
      case RNode::Concat: {
        if (n.kids.empty()) return eps();
        F f = build(*n.kids[0]);
        for (size_t k = 1; k < n.kids.size(); k++) {
          F g = build(*n.kids[k]);
          patch(f, g.start);
          f.outs = g.outs;
        }
        return f;
      }
      case RNode::Alt: {
        std::vector<F> alts;
        for (auto& k : n.kids) alts.push_back(build(*k));
        return alt_of(alts);
      }
      case RNode::Repeat: {
        const RNode& c = *n.kids[0];
        F acc = eps();
        for (int k = 0; k < n.min; k++) { F g = build(c); patch(acc, g.start); acc.outs = g.outs; }
        if (n.max < 0) {
          F g = build(c);
          int sp = nfa.add(1, 0, 0, g.start, -1);
          patch(g, sp);
          patch(acc, sp);
          return F{acc.start, {{sp, 1}}};
        }
        for (int k = n.min; k < n.max; k++) {
          F g = build(c);
          int sp = nfa.add(1, 0, 0, g.start, -1);
          patch(acc, sp);
          std::vector<std::pair<int, int>> outs = g.outs;
          outs.push_back({sp, 1});
          acc = F{acc.start, outs};
        }
        return acc;
      }
    }
    return eps();
  }
  F alt_of(std::vector<F>& alts) {
    if (alts.size() == 1) return alts[0];
    F cur = alts.back();
    for (int k = (int)alts.size() - 2; k >= 0; k--) {
      int sp = nfa.add(1, 0, 0, alts[k].start, cur.start);
      std::vector<std::pair<int, int>> outs = alts[k].outs;
      outs.insert(outs.end(), cur.outs.begin(), cur.outs.end());
      cur = F{sp, outs};
    }
    return cur;
  }
};

void closure(const Nfa& nfa, std::set<int>& st) {
  std::vector<int> stack(st.begin(), st.end());
  while (!stack.empty()) {
    int x = stack.back(); stack.pop_back();
    const NState& s = nfa.s[x];
    if (s.type == 1 || s.type == 3) {
      for (int o : {s.out, s.out2}) if (o >= 0 && !st.count(o)) { st.insert(o); stack.push_back(o); }
    }
  }
}

}  // namespace

CompiledRegex compile_regex(const std::string& pattern) {
  CompiledRegex out;
  RxParser ps(pattern);
  std::unique_ptr<RNode> ast;
  try {
    ast = ps.alt();
    if (ps.i < pattern.size()) throw RxErr{"unopened group", false};
  } catch (RxErr& e) {
    out.why = e.why;
    if (e.unsupported) { out.unsupported = true; return out; }
    out.valid = false; return out;
  }
  out.ascii_only = ps.ascii_only;
  out.end_anchored = ps.end_anchor;
  Nfa nfa;
  Builder b{nfa};
  Builder::F f = b.build(*ast);
  int m = nfa.add(2);
  b.patch(f, m);
  int nstart = f.start;

  // subset construction; state 0 = dead
  std::map<std::set<int>, uint32_t> ids;
  std::vector<std::set<int>> sets;
  sets.push_back({});
  ids[{}] = 0;
  std::set<int> s0 = {nstart};
  closure(nfa, s0);
  auto intern = [&](const std::set<int>& s) -> uint32_t {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    uint32_t id = (uint32_t)sets.size();
    ids[s] = id; sets.push_back(s);
    return id;
  };
  out.start = intern(s0);
  std::vector<std::array<uint16_t, 256>> table;
  table.push_back({});
  table[0].fill(0);
  for (size_t cur = 1; cur < sets.size(); cur++) {
    if (sets.size() > 4000) { out.unsupported = true; out.why = "DFA too large"; return out; }
    std::array<uint16_t, 256> row;
    for (int byte = 0; byte < 256; byte++) {
      std::set<int> nx;
      for (int x : sets[cur]) {
        const NState& s = nfa.s[x];
        if (s.type == 0 && byte >= s.lo && byte <= s.hi) nx.insert(s.out);
      }
      if (!ps.start_anchor) nx.insert(nstart);   // unanchored search
      closure(nfa, nx);
      row[byte] = (uint16_t)intern(nx);
    }
    if (table.size() <= cur) table.resize(cur + 1);
    table[cur] = row;
  }
  out.nstates = (uint32_t)sets.size();
  out.table.resize((size_t)out.nstates * 256);
  for (uint32_t st = 0; st < out.nstates; st++)
    for (int byte = 0; byte < 256; byte++) out.table[(size_t)st * 256 + byte] = st < table.size() ? table[st][byte] : 0;
  out.accept.resize(out.nstates);
  for (uint32_t st = 0; st < out.nstates; st++) out.accept[st] = sets[st].count(m) ? 1 : 0;
  return out;
}

int dfa_match(const CompiledRegex& rx, const char* s, size_t n) {
  if (!rx.valid || rx.unsupported) return -1;
  if (rx.ascii_only) for (size_t k = 0; k < n; k++) if ((unsigned char)s[k] >= 0x80) return -1;
  uint32_t st = rx.start;
  if (!rx.end_anchored && rx.accept[st]) return 1;
  for (size_t k = 0; k < n; k++) {
    st = rx.table[(size_t)st * 256 + (unsigned char)s[k]];
    if (st == 0) return 0;
    if (!rx.end_anchored && rx.accept[st]) return 1;
  }
  return rx.accept[st] ? 1 : 0;
}

}  // namespace gg
