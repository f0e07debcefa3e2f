// Compiled rules file: device program blob + host-side tables the reporter needs.
// Lowering of RulesFile (guard/src/rules/exprs.rs:276-284) to flat arrays.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "doc_loader.h"
#include "guard_types.h"
#include "regex_dfa.h"
#include "rules_ast.h"

namespace gg {

struct Program {
  std::string file_name;
  std::vector<uint32_t> blob;          // ProgHeader + sections (uploaded to HBM)
  ProgHeader hdr{};

  // host tables (reporter / error messages)
  std::vector<std::string> ctx;        // context strings (clause.d / clause.f)
  std::vector<std::string> msgs;       // custom messages (clause.e)
  std::vector<std::vector<QueryPart>> queries;   // per query id: parts (remaining-query display)
  std::vector<std::string> rule_names;           // per rule id
  std::vector<std::string> slot_names;           // per name slot
  std::vector<std::string> var_names;            // per var id
  std::vector<std::string> param_rule_names;     // per param rule id
  std::vector<uint32_t> param_rule_nparams;
  std::vector<std::string> type_names;           // per typeblock clause id (indexed by clause)
  std::vector<std::string> unsupported;          // messages for C_UNSUPPORTED / unsupported regex
  std::vector<CompiledRegex> regex;
  std::vector<std::string> regex_src;
  DocBatch lit;                                  // literal arena (paths "" / "/0" ... , L:0,C:0)
  std::vector<DRange> ranges;
  std::vector<PClause> clauses;                  // host copy
  std::vector<PQuery> pqueries;
  std::vector<PPart> parts;
  std::vector<PStr> strs;
  std::string str_bytes;
  uint32_t n_rules = 0;

  std::string query_remaining(uint32_t qid, uint32_t step) const { return slice_display(queries[qid], step); }
};

// Compiles a parsed rules file; returns false + message on a (regex) validation failure that the
// reference reports as a rules parse error.
bool compile_program(const RulesFile& rf, const std::string& file_name, Program& out, std::string& err);

void key_alternates(const std::string& key, std::string out[7]);

}  // namespace gg
