// Rule regex -> byte DFA (host compile, device match).
//
// The reference compiles each regex with fancy-regex 0.13.0 (over regex 1.11.1 / regex-syntax
// 0.8.5) at every comparison and calls `is_match` (unanchored search):
// guard/src/rules/path_value.rs:255,263,1074-1077.  Here each distinct regex is compiled once
// per rules file to a DFA over UTF-8 bytes whose transition table is staged in LDS on device.
//
// Constructs fancy-regex supports but a DFA cannot (look-around, back-references, atomic
// groups, \b, mid-pattern anchors) are NOT silently approximated: the regex is marked
// unsupported and evaluating it raises an explicit "unsupported on MI355X path" error.
// Perl classes \d \w \s and (?i) are Unicode-aware as in regex-syntax (unicode_tables.h).  The
// DFA runs over code-point classes (table = nstates x nclasses); the matcher decodes UTF-8.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "guard_types.h"

namespace gg {

struct CompiledRegex {
  bool valid = true;          // syntactically valid (else: rules parse error)
  bool unsupported = false;   // valid but not DFA-compilable here
  uint32_t nstates = 0;       // state 0 = dead
  uint32_t start = 0;
  uint32_t ncls = 0;          // code-point classes
  uint8_t ascii[128] = {0};   // class of each ASCII code point
  std::vector<std::pair<uint32_t, uint32_t>> bounds;   // (first code point, class) runs above U+007F
  std::vector<uint16_t> table;   // nstates * ncls
  std::vector<uint8_t> accept;   // nstates: 1 = match (decided), 2 = match if the haystack ends here
  // No DFA within the limits (more than 4000 states or 250 classes): the epsilon-free NFA is simulated
  // instead, one bitset of live states stepped per character (nfa_match, device nfa_run).  nstates / ncls
  // then count NFA states / classes; table, accept, ascii, bounds are unused.  Layout: guard_types.h kNfa*.
  bool nfa = false;
  std::vector<uint32_t> nfa_tab;
  std::string why;
};

CompiledRegex compile_regex(const std::string& pattern);

uint32_t regex_class_of(const CompiledRegex& rx, uint32_t cp);
// host reference matcher over the compiled DFA (used by host-side unit tests)
int dfa_match(const CompiledRegex& rx, const char* s, size_t n);  // 1 match, 0 no, -1 unsupported

}  // namespace gg
