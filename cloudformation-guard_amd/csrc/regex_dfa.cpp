// Rule regex -> byte DFA (see regex_dfa.h).
#include "regex_dfa.h"

#include <algorithm>
#include <array>
#include <map>
#include <memory>
#include <functional>
#include <set>
#include <unordered_map>

#include "unicode_tables.h"

namespace gg {

namespace {

struct RxErr { std::string why; bool unsupported; };

struct Rng { uint32_t lo, hi; };

struct RNode {
  enum K { Empty, Set, Concat, Alt, Repeat, AssertStart, AssertEnd, WordB, NotWordB } k = Empty;
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

std::vector<Rng> table_set(const uint32_t (*t)[2], uint32_t n) {
  std::vector<Rng> v(n);
  for (uint32_t i = 0; i < n; i++) v[i] = {t[i][0], t[i][1]};
  return v;
}

// members of cp's simple-case-folding class (CaseFolding.txt C + S), cp included
void add_fold(std::vector<Rng>& out, uint32_t cp) {
  size_t lo = 0, hi = uni::kFoldCp_N;
  while (lo < hi) { size_t m = (lo + hi) / 2; if (uni::kFoldCp[m][0] < cp) lo = m + 1; else hi = m; }
  if (lo < uni::kFoldCp_N && uni::kFoldCp[lo][0] == cp) {
    const uint32_t* cl = uni::kFoldClass[uni::kFoldCp[lo][1]];
    for (uint32_t k = 0; k < cl[1]; k++) { uint32_t m = uni::kFoldMembers[cl[0] + k]; out.push_back({m, m}); }
  }
}

// ClassUnicode::case_fold_simple (regex-syntax hir::ClassUnicode): every member of the set widened
// to its folding class
void fold_closure(std::vector<Rng>& set) {
  normalize(set);
  std::vector<Rng> add;
  for (const Rng& r : set) {
    size_t lo = 0, hi = uni::kFoldCp_N;
    while (lo < hi) { size_t m = (lo + hi) / 2; if (uni::kFoldCp[m][0] < r.lo) lo = m + 1; else hi = m; }
    for (size_t k = lo; k < uni::kFoldCp_N && uni::kFoldCp[k][0] <= r.hi; k++) add_fold(add, uni::kFoldCp[k][0]);
  }
  set.insert(set.end(), add.begin(), add.end());
  normalize(set);
}

struct RxParser {
  const std::string& p;
  size_t i = 0;
  bool icase = false, dotall = false;
  int depth = 0;
  bool has_word = false;   // \b or \B appears: the DFA tracks whether the previous character was a word one
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
    if (icase) add_fold(set, cp);   // (?i): simple case folding (regex-syntax hir translate)
  }

  // Unicode perl classes (regex-syntax unicode::perl_digit / perl_space / perl_word); they are
  // closed under simple case folding, so (?i) leaves them unchanged
  std::vector<Rng> perl_class(char c) {
    std::vector<Rng> s;
    switch (c) {
      case 'd': case 'D': s = table_set(uni::kDigit, uni::kDigit_N); break;
      case 'w': case 'W': s = table_set(uni::kWord, uni::kWord_N); break;
      case 's': case 'S': s = table_set(uni::kSpace, uni::kSpace_N); break;
    }
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
      case 'b': case 'B': invalid("\\b in class");   // outside a class: atom() (an assertion)
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
      } else if (is_lit) {
        add_literal(set, lo);
      } else {
        set.insert(set.end(), item.begin(), item.end());
      }
    }
    // unicode_fold_and_negate: fold the whole class under (?i), then negate
    if (icase) fold_closure(set);
    normalize(set);
    if (neg) set = negate(set);
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

  std::unique_ptr<RNode> assert_node(RNode::K k) {
    auto n = std::make_unique<RNode>(); n->k = k; return n;
  }
  std::unique_ptr<RNode> end_node() {
    size_t j = i;
    int d = depth;
    while (j < p.size() && p[j] == ')' && d > 0) { j++; d--; }
    if (!(j == p.size() || (p[j] == '|' && d == 0))) unsup("mid-pattern end anchor");
    return assert_node(RNode::AssertEnd);
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
    // `^` / `\A`: an assertion the NFA passes only at offset 0 (closure at_start); `$` / `\z`
    // (non-multiline: end of text) only where nothing can follow it -- the end of the pattern or
    // of a top-level alternative, possibly through closing groups -- where it marks the state as
    // accepting at the end of the haystack
    if (c == '^') { i++; return assert_node(RNode::AssertStart); }
    if (c == '$') { i++; return end_node(); }
    if (c == '\\') {
      i++;
      if (i < p.size() && p[i] == 'A') { i++; return assert_node(RNode::AssertStart); }
      if (i < p.size() && p[i] == 'z') { i++; return end_node(); }
      // Unicode word boundary / not a word boundary (regex-syntax Look::WordUnicode / WordUnicodeNegate):
      // \w on one side and not on the other, the text's ends counting as non-word
      if (i < p.size() && (p[i] == 'b' || p[i] == 'B')) { has_word = true; return assert_node(p[i++] == 'b' ? RNode::WordB : RNode::NotWordB); }
      return set_node(escape(false));
    }
    if (c == '*' || c == '+' || c == '?') invalid("repetition operator missing expression");
    std::vector<Rng> s;
    add_literal(s, next_cp());
    return set_node(s);
  }
};

// ------------------------------------------------------------------ NFA ----
// The automaton runs over code-point classes, not bytes: the code points are partitioned into
// classes whose members every character set of the regex treats alike (\\w + literals: a handful
// of classes), so the DFA table is nstates x nclasses and stays small enough for LDS even for the
// Unicode perl classes.  The matcher decodes UTF-8 and maps a code point to its class through a
// 128-entry ASCII table, or a binary search over the class boundaries above U+007F.
// type 0 class set, 1 split, 2 match, 3 epsilon, 4 start-of-text assertion, 5 match at end of text,
// 6 word boundary (\b), 7 not a word boundary (\B)
struct NState { int type; int cset; int out, out2; };
struct Nfa {
  std::vector<NState> s;
  std::vector<std::vector<uint8_t>> csets;   // per class-set state: membership per class
  int add(int type, int cset = -1, int out = -1, int out2 = -1) {
    s.push_back({type, cset, out, out2});
    return (int)s.size() - 1;
  }
};

void collect_sets(const RNode& n, std::vector<const RNode*>& out) {
  if (n.k == RNode::Set) out.push_back(&n);
  for (auto& k : n.kids) collect_sets(*k, out);
}

struct Builder {
  Nfa& nfa;
  const std::map<const RNode*, int>& cset_of;
  struct F { int start; std::vector<std::pair<int, int>> outs; };  // dangling (state, field 0/1)
  void patch(const F& f, int target) {
    for (auto& o : f.outs) { if (o.second == 0) nfa.s[o.first].out = target; else nfa.s[o.first].out2 = target; }
  }
  F eps() { int s = nfa.add(3); return F{s, {{s, 0}}}; }
  F build(const RNode& n) {
    switch (n.k) {
      case RNode::Empty: return eps();
      case RNode::Set: { int s = nfa.add(0, cset_of.at(&n)); return F{s, {{s, 0}}}; }
      case RNode::AssertStart: { int s = nfa.add(4); return F{s, {{s, 0}}}; }
      case RNode::AssertEnd: { int s = nfa.add(5); return F{s, {}}; }
      case RNode::WordB: { int s = nfa.add(6); return F{s, {{s, 0}}}; }
      case RNode::NotWordB: { int s = nfa.add(7); return F{s, {{s, 0}}}; }
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
          int sp = nfa.add(1, -1, g.start, -1);
          patch(g, sp);
          patch(acc, sp);
          return F{acc.start, {{sp, 1}}};
        }
        for (int k = n.min; k < n.max; k++) {
          F g = build(c);
          int sp = nfa.add(1, -1, g.start, -1);
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
      int sp = nfa.add(1, -1, alts[k].start, cur.start);
      std::vector<std::pair<int, int>> outs = alts[k].outs;
      outs.insert(outs.end(), cur.outs.begin(), cur.outs.end());
      cur = F{sp, outs};
    }
    return cur;
  }
};

// epsilon closure, in place; `mark` is a scratch bitmap over NFA states (cleared on return).
// Start-of-text assertions pass only for the closure taken at offset 0; word-boundary assertions only
// when `look` says the position satisfies them (bit 0: \b holds, bit 1: \B holds) -- a state's closure
// stops at them until the next character (or the end of the text) decides.
void closure(const Nfa& nfa, std::vector<int>& st, std::vector<uint8_t>& mark, bool at_start, uint32_t look = 0) {
  for (int x : st) mark[x] = 1;
  for (size_t k = 0; k < st.size(); k++) {
    const NState& s = nfa.s[st[k]];
    if (s.type == 1 || s.type == 3 || (s.type == 4 && at_start) || (s.type == 6 && (look & 1)) || (s.type == 7 && (look & 2)))
      for (int o : {s.out, s.out2}) if (o >= 0 && !mark[o]) { mark[o] = 1; st.push_back(o); }
  }
  for (int x : st) mark[x] = 0;
  std::sort(st.begin(), st.end());
}

struct VecHash {
  size_t operator()(const std::vector<int>& v) const {
    size_t h = 1469598103934665603ull;
    for (int x : v) h = (h ^ (size_t)x) * 1099511628211ull;
    return h;
  }
};


// The NFA simulation for a regex whose DFA exceeds the limits (CompiledRegex::nfa; layout in regex_dfa.h).
// Only class-set states (type 0) carry bits: the live set after a character is the union of the follow
// sets F[s] of the live states whose class set holds it, plus Z (a match may start at every offset) --
// the same sets the subset construction interns, unioned per step instead of tabulated.  Word assertions
// would need the previous character's kind in every closure; such a regex stays refused.
CompiledRegex& nfa_fallback(CompiledRegex& out, const Nfa& nfa, int nstart, uint32_t ncls0,
                            const std::vector<std::pair<uint32_t, uint32_t>>& ivals, bool has_word, const char* why) {
  auto refuse = [&](std::string w) -> CompiledRegex& { out.unsupported = true; out.why = std::move(w); return out; };
  if (has_word) return refuse(std::string(why) + " (with word assertions)");
  std::vector<int> bit(nfa.s.size(), -1), setst;
  for (size_t k = 0; k < nfa.s.size(); k++) if (nfa.s[k].type == 0) { bit[k] = (int)setst.size(); setst.push_back((int)k); }
  const uint32_t m = (uint32_t)setst.size();
  if (m > kNfaMaxStates) return refuse(std::string(why) + "; NFA too large");
  const uint32_t W = m ? (m + 31) / 32 : 1;
  uint32_t nb = 0;
  for (size_t k = 0; k < ivals.size(); k++)
    if (ivals[k].first >= 128 && (k == 0 || ivals[k - 1].first < 128 || ivals[k - 1].second != ivals[k].second)) nb++;
  const size_t words = kNfaHdr + 2 * (size_t)W + m + (size_t)m * W + (size_t)ncls0 * W + 128 + 2 * (size_t)nb;
  if (words > (1u << 20)) return refuse(std::string(why) + "; NFA tables too large");
  std::vector<uint32_t>& T = out.nfa_tab;
  T.assign(words, 0);
  T[kNfaM] = m; T[kNfaW] = W; T[kNfaCls] = ncls0; T[kNfaNb] = nb;
  const size_t oS0 = kNfaHdr, oZ = oS0 + W, oFL = oZ + W, oF = oFL + m, oM = oF + (size_t)m * W, oA = oM + (size_t)ncls0 * W,
               oB = oA + 128;
  std::vector<uint8_t> mark(nfa.s.size(), 0);
  // a closure as (bitset at `at`, flags)
  auto put = [&](std::vector<int> st, bool at_start, size_t at) -> uint32_t {
    closure(nfa, st, mark, at_start);
    uint32_t fl = 0;
    for (int x : st) {
      const int t = nfa.s[x].type;
      if (t == 0) T[at + bit[x] / 32] |= 1u << (bit[x] % 32);
      else if (t == 2) fl |= 1;
      else if (t == 5) fl |= 2;
    }
    return fl;
  };
  T[kNfaStartFlags] = put({nstart}, true, oS0);
  T[kNfaAgainFlags] = put({nstart}, false, oZ);
  for (uint32_t j = 0; j < m; j++) {
    const NState& s = nfa.s[setst[j]];
    T[oFL + j] = s.out >= 0 ? put({s.out}, false, oF + (size_t)j * W) : 0;
  }
  for (uint32_t c = 0; c < ncls0; c++)
    for (uint32_t j = 0; j < m; j++)
      if (nfa.csets[nfa.s[setst[j]].cset][c]) T[oM + (size_t)c * W + j / 32] |= 1u << (j % 32);
  size_t r = 0;
  for (size_t k = 0; k < ivals.size(); k++) {
    if (ivals[k].first < 128) { T[oA + ivals[k].first] = ivals[k].second; continue; }
    if (k == 0 || ivals[k - 1].first < 128 || ivals[k - 1].second != ivals[k].second) {
      T[oB + 2 * r] = ivals[k].first; T[oB + 2 * r + 1] = ivals[k].second; r++;
    }
  }
  out.nfa = true;
  out.nstates = m;
  out.ncls = ncls0;
  out.why = why;
  return out;
}

}  // namespace

uint32_t regex_class_of(const CompiledRegex& rx, uint32_t cp) {
  if (cp < 128) return rx.ascii[cp];
  // last boundary whose start <= cp (bounds[0].first == 128)
  size_t lo = 0, hi = rx.bounds.size();
  while (hi - lo > 1) { size_t m = (lo + hi) / 2; if (rx.bounds[m].first <= cp) lo = m; else hi = m; }
  return rx.bounds[lo].second;
}

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
  // ---- code-point classes: elementary intervals keyed by the set of Set nodes containing them
  std::vector<const RNode*> sets_n;
  collect_sets(*ast, sets_n);
  // word assertions: \w is one more partitioning set, so every class is all word or all non-word
  // characters (it builds no NFA state)
  RNode word_set;
  word_set.k = RNode::Set;
  if (ps.has_word) {
    word_set.set = table_set(uni::kWord, uni::kWord_N);
    normalize(word_set.set);
    sets_n.push_back(&word_set);
  }
  std::vector<uint32_t> cuts = {0, 128, 0x110000};
  for (auto* n : sets_n) for (auto& r : n->set) { cuts.push_back(r.lo); cuts.push_back(r.hi + 1); }
  for (uint32_t c = 1; c < 128; c++) cuts.push_back(c);   // ASCII: one interval per code point
  std::sort(cuts.begin(), cuts.end());
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  std::map<std::vector<uint8_t>, uint32_t> sig_cls;
  std::vector<std::vector<uint8_t>> cls_sig;
  std::vector<std::pair<uint32_t, uint32_t>> ivals;   // (start, class)
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    const uint32_t lo = cuts[k];
    std::vector<uint8_t> sig(sets_n.size(), 0);
    for (size_t j = 0; j < sets_n.size(); j++) {
      const auto& v = sets_n[j]->set;   // normalized, sorted
      auto it = std::upper_bound(v.begin(), v.end(), lo, [](uint32_t x, const Rng& r) { return x < r.lo; });
      if (it != v.begin() && (it - 1)->hi >= lo) sig[j] = 1;
    }
    auto it = sig_cls.find(sig);
    if (it == sig_cls.end()) {
      it = sig_cls.emplace(sig, (uint32_t)cls_sig.size()).first;
      cls_sig.push_back(sig);
    }
    ivals.push_back({lo, it->second});
  }
  const uint32_t ncls0 = (uint32_t)cls_sig.size();
  Nfa nfa;
  std::map<const RNode*, int> cset_of;
  for (size_t j = 0; j < sets_n.size(); j++) {
    std::vector<uint8_t> mem(ncls0, 0);
    for (uint32_t c = 0; c < ncls0; c++) mem[c] = cls_sig[c][j];
    cset_of[sets_n[j]] = (int)nfa.csets.size();
    nfa.csets.push_back(mem);
  }
  Builder b{nfa, cset_of};
  Builder::F f = b.build(*ast);
  int m = nfa.add(2);
  b.patch(f, m);
  const int nstart = f.start;
  if (ncls0 > 250) return nfa_fallback(out, nfa, nstart, ncls0, ivals, ps.has_word, "too many character classes");

  // ---- subset construction over the classes (state 0 = dead)
  // With word assertions (regex-automata's look-behind state) a DFA state is (NFA states closed up to the
  // word assertions, whether the previous character was a word character; the start state marked apart,
  // as start-of-text assertions still pass there): a transition on class c first extends the closure
  // through the assertions the boundary between the previous character and c satisfies -- a match found
  // there (ending before c) leads to the accepting sink -- then steps on c.  At the end of the text the
  // closure extends with the end counted as a non-word character (accept flag 2).
  const bool hw = ps.has_word;
  std::vector<uint8_t> cls_word(ncls0, 0);
  if (hw) for (uint32_t c = 0; c < ncls0; c++) cls_word[c] = cls_sig[c][sets_n.size() - 1];
  static const int kPrevWord = -1, kStartMark = -2, kMatchSink = -3;
  std::vector<uint8_t> mark(nfa.s.size(), 0);
  std::unordered_map<std::vector<int>, uint32_t, VecHash> ids;
  std::vector<std::vector<int>> sets;
  sets.push_back({});
  ids[{}] = 0;
  std::vector<int> s0 = {nstart};
  closure(nfa, s0, mark, true);
  if (hw) s0.push_back(kStartMark);   // previous "character" = start of text: non-word
  auto intern = [&](std::vector<int>& st) -> uint32_t {
    auto it = ids.find(st);
    if (it != ids.end()) return it->second;
    uint32_t id = (uint32_t)sets.size();
    ids.emplace(st, id);
    sets.push_back(st);
    return id;
  };
  uint32_t start = intern(s0);
  uint32_t sink = 0;
  if (hw) { std::vector<int> m1 = {kMatchSink}; sink = intern(m1); }
  // split a state key into (NFA states, previous-char-is-word, is-start, is-sink)
  auto parts = [&](const std::vector<int>& key, std::vector<int>& st, bool& pw, bool& at0, bool& sk) {
    st.clear(); pw = at0 = sk = false;
    for (int x : key) {
      if (x == kPrevWord) pw = true;
      else if (x == kStartMark) at0 = true;
      else if (x == kMatchSink) sk = true;
      else st.push_back(x);
    }
  };
  std::vector<std::vector<uint32_t>> table(1, std::vector<uint32_t>(ncls0, 0));
  std::vector<int> here, ex;
  for (size_t cur = 1; cur < sets.size(); cur++) {
    if (sets.size() > 4000) return nfa_fallback(out, nfa, nstart, ncls0, ivals, hw, "DFA too large");
    bool pw, at0, sk;
    parts(sets[cur], here, pw, at0, sk);
    std::vector<uint32_t> row(ncls0);
    for (uint32_t c = 0; c < ncls0; c++) {
      if (sk) { row[c] = (uint32_t)cur; continue; }
      const std::vector<int>* from = &here;
      if (hw) {
        ex = here;
        const bool cw = cls_word[c] != 0;
        closure(nfa, ex, mark, at0, pw != cw ? 1u : 2u);
        bool matched = false;
        for (int x : ex) if (nfa.s[x].type == 2) matched = true;
        if (matched) { row[c] = sink; continue; }
        from = &ex;
      }
      std::vector<int> nx;
      for (int x : *from) {
        const NState& s = nfa.s[x];
        if (s.type == 0 && nfa.csets[s.cset][c]) nx.push_back(s.out);
      }
      nx.push_back(nstart);   // unanchored search: a match may start at every offset
      std::sort(nx.begin(), nx.end());
      nx.erase(std::unique(nx.begin(), nx.end()), nx.end());
      closure(nfa, nx, mark, false);
      if (hw && cls_word[c]) nx.push_back(kPrevWord);
      row[c] = intern(nx);
    }
    table.push_back(row);
  }
  // accept flags: 1 = a match ends here (is_match is decided), 2 = a match ends here if the
  // haystack ends here (`$`, or a word assertion the end of the text satisfies)
  const size_t nd = sets.size();
  std::vector<uint8_t> acc(nd, 0);
  for (size_t st = 1; st < nd; st++) {
    bool pw, at0, sk;
    parts(sets[st], here, pw, at0, sk);
    if (sk) { acc[st] = 1; continue; }
    for (int x : here) { if (nfa.s[x].type == 2) acc[st] |= 1; else if (nfa.s[x].type == 5) acc[st] |= 2; }
    if (hw && !(acc[st] & 1)) {
      ex = here;
      closure(nfa, ex, mark, at0, pw ? 1u : 2u);   // the end of the text is a non-word position
      for (int x : ex) if (nfa.s[x].type == 2 || nfa.s[x].type == 5) acc[st] |= 2;
    }
  }
  // ---- Moore minimisation (block 0 stays the dead state)
  std::vector<uint32_t> blk(nd);
  for (size_t st = 0; st < nd; st++) blk[st] = st == 0 ? 0 : 1 + acc[st];
  size_t nblk = std::set<uint32_t>(blk.begin(), blk.end()).size();
  for (;;) {
    std::map<std::vector<uint32_t>, uint32_t> ids2;
    std::vector<uint32_t> nb(nd), key(ncls0 + 1);
    for (size_t st = 0; st < nd; st++) {
      key[0] = blk[st];
      for (uint32_t c = 0; c < ncls0; c++) key[c + 1] = blk[table[st][c]];
      auto it = ids2.find(key);
      if (it == ids2.end()) it = ids2.emplace(key, (uint32_t)ids2.size()).first;
      nb[st] = it->second;
    }
    const uint32_t dead = nb[0];
    for (auto& x : nb) x = x == dead ? 0 : (x < dead ? x + 1 : x);
    blk = nb;
    if (ids2.size() == nblk) break;
    nblk = ids2.size();
  }
  // ---- merge classes that every minimal state treats alike; emit
  const uint32_t nmin = (uint32_t)nblk;
  std::vector<std::vector<uint32_t>> mt(nmin, std::vector<uint32_t>(ncls0, 0));
  std::vector<uint8_t> macc(nmin, 0);
  for (size_t st = 0; st < nd; st++) {
    for (uint32_t c = 0; c < ncls0; c++) mt[blk[st]][c] = blk[table[st][c]];
    macc[blk[st]] = acc[st];
  }
  std::map<std::vector<uint32_t>, uint32_t> col_ids;
  std::vector<uint32_t> cmap(ncls0);
  for (uint32_t c = 0; c < ncls0; c++) {
    std::vector<uint32_t> col(nmin);
    for (uint32_t st = 0; st < nmin; st++) col[st] = mt[st][c];
    auto it = col_ids.find(col);
    if (it == col_ids.end()) it = col_ids.emplace(col, (uint32_t)col_ids.size()).first;
    cmap[c] = it->second;
  }
  out.nstates = nmin;
  out.start = blk[start];
  out.accept = macc;
  out.ncls = (uint32_t)col_ids.size();
  out.table.assign((size_t)nmin * out.ncls, 0);
  for (uint32_t st = 0; st < nmin; st++)
    for (uint32_t c = 0; c < ncls0; c++) out.table[(size_t)st * out.ncls + cmap[c]] = (uint16_t)mt[st][c];
  for (auto& iv : ivals) {
    const uint32_t c = cmap[iv.second];
    if (iv.first < 128) out.ascii[iv.first] = (uint8_t)c;
    else if (out.bounds.empty() || out.bounds.back().second != c) out.bounds.push_back({iv.first, c});
  }
  return out;
}

// host restatement of the device nfa_run (eval_core.inc)
int nfa_match(const CompiledRegex& rx, const char* s, size_t n) {
  const uint32_t* T = rx.nfa_tab.data();
  const uint32_t m = T[kNfaM], W = T[kNfaW], ncls = T[kNfaCls], nb = T[kNfaNb];
  const uint32_t *S0 = T + kNfaHdr, *Z = S0 + W, *FL = Z + W, *F = FL + m, *M = F + (size_t)m * W, *A = M + (size_t)ncls * W,
                 *B = A + 128;
  uint32_t cur[kNfaMaxWords], nx[kNfaMaxWords];
  for (uint32_t w = 0; w < W; w++) cur[w] = S0[w];
  uint32_t cf = T[kNfaStartFlags];
  if (cf & 1) return 1;
  uint32_t cp = 0, need = 0;
  for (size_t k = 0; k < n; k++) {
    const uint8_t by = (uint8_t)s[k];
    if (by < 0x80) { cp = by; need = 0; }
    else if (by >= 0xC0) { need = by >= 0xF0 ? 3 : by >= 0xE0 ? 2 : 1; cp = by & (0x3Fu >> need); continue; }
    else { cp = (cp << 6) | (by & 0x3Fu); if (--need) continue; }
    uint32_t cls;
    if (cp < 128) cls = A[cp];
    else {
      uint32_t lo = 0, hi = nb;
      while (hi - lo > 1) { const uint32_t md = (lo + hi) / 2; if (B[2 * md] <= cp) lo = md; else hi = md; }
      cls = B[2 * lo + 1];
    }
    uint32_t nf = T[kNfaAgainFlags];
    for (uint32_t w = 0; w < W; w++) nx[w] = Z[w];
    for (uint32_t w = 0; w < W; w++) {
      uint32_t x = cur[w] & M[(size_t)cls * W + w];
      while (x) {
        const uint32_t j = w * 32 + (uint32_t)__builtin_ctz(x);
        x &= x - 1;
        nf |= FL[j];
        const uint32_t* f = F + (size_t)j * W;
        for (uint32_t v = 0; v < W; v++) nx[v] |= f[v];
      }
    }
    if (nf & 1) return 1;
    for (uint32_t w = 0; w < W; w++) cur[w] = nx[w];
    cf = nf;
  }
  return (cf & 2) ? 1 : 0;
}

int dfa_match(const CompiledRegex& rx, const char* s, size_t n) {
  if (!rx.valid || rx.unsupported) return -1;
  if (rx.nfa) return nfa_match(rx, s, n);
  uint32_t st = rx.start;
  if (rx.accept[st] & 1) return 1;
  uint32_t cp = 0, need = 0;
  for (size_t k = 0; k < n; k++) {
    const uint8_t by = (uint8_t)s[k];
    if (by < 0x80) { cp = by; need = 0; }
    else if (by >= 0xC0) { need = by >= 0xF0 ? 3 : by >= 0xE0 ? 2 : 1; cp = by & (0x3Fu >> need); continue; }
    else { cp = (cp << 6) | (by & 0x3Fu); if (--need) continue; }
    st = rx.table[(size_t)st * rx.ncls + regex_class_of(rx, cp)];
    if (st == 0) return 0;
    if (rx.accept[st] & 1) return 1;
  }
  return rx.accept[st] ? 1 : 0;
}

}  // namespace gg
