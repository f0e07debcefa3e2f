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
// Unicode-dependent classes (\d \w \s, case folding beyond ASCII) are compiled for ASCII and
// marked "ascii_only": matching a haystack that contains non-ASCII bytes raises the same
// explicit error instead of guessing.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace gg {

struct CompiledRegex {
  bool valid = true;          // syntactically valid (else: rules parse error)
  bool unsupported = false;   // valid but not DFA-compilable here
  bool ascii_only = false;
  bool end_anchored = false;
  uint32_t nstates = 0;       // state 0 = dead
  uint32_t start = 0;
  std::vector<uint16_t> table;   // nstates * 256
  std::vector<uint8_t> accept;   // nstates
  std::string why;
};

CompiledRegex compile_regex(const std::string& pattern);

// host reference matcher over the compiled DFA (used by host-side unit tests)
int dfa_match(const CompiledRegex& rx, const char* s, size_t n);  // 1 match, 0 no, -1 unsupported

}  // namespace gg
