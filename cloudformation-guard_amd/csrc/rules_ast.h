// Guard rules AST (host side) -- mirrors guard/src/rules/exprs.rs:12-284.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace gg {

// literal value (values.rs:81-95 `Value`), later placed in the literal arena
struct LitValue {
  enum K { Null, String, Regex, Bool, Int, Float, Char, List, Map, RangeInt, RangeFloat, RangeChar } k = Null;
  std::string s;        // String / Regex
  bool b = false;
  int64_t i = 0;
  double f = 0;
  uint32_t ch = 0;      // Char
  std::vector<LitValue> items;                       // List
  std::vector<std::pair<std::string, LitValue>> kv;  // Map (deduped, insertion order)
  // ranges
  int64_t ilo = 0, ihi = 0; double flo = 0, fhi = 0; uint32_t clo = 0, chi = 0; uint8_t incl = 0;
};

struct FileLoc { uint32_t line = 0, column = 0; std::string file; };

struct Clause;
struct FuncExpr;
using Disj = std::vector<std::shared_ptr<Clause>>;
using Conj = std::vector<Disj>;

struct QueryPart {
  enum K { This, Key, Index, AllValues, AllIndices, Filter, MapKeyFilter } k = Key;
  std::string key;                // Key / capture name (AllValues/AllIndices/Filter/MapKeyFilter)
  bool has_name = false;
  int32_t index = 0;
  std::shared_ptr<Conj> filter;   // Filter
  // MapKeyFilter
  std::string mk_op; bool mk_not = false;
  std::shared_ptr<struct LetValue> mk_with;
};

struct AccessQuery { std::vector<QueryPart> parts; bool match_all = true; };

struct LetValue {
  enum K { Value, Access, Func } k = Value;
  LitValue value;
  AccessQuery access;
  std::shared_ptr<FuncExpr> func;
};

struct FuncExpr { std::string name; std::vector<LetValue> params; FileLoc loc; };

struct LetExpr { std::string var; LetValue value; };

struct Block { std::vector<LetExpr> assignments; Conj conjunctions; };

struct TypeBlock;

// GuardClause / WhenGuardClause / RuleClause flattened into one node type
struct Clause {
  enum K { Access, NamedRule, ParamRule, BlockClause, WhenBlock, TypeBlockK } k = Access;
  bool rule_level = false;   // WhenBlock: RuleClause::WhenBlock ("RuleClause") vs GuardClause ("GuardConditionClause")
  // Access
  AccessQuery query;
  std::string op; bool op_not = false; bool negation = false;
  bool has_rhs = false; LetValue rhs;
  bool has_msg = false; std::string msg;
  FileLoc loc;
  // NamedRule / ParamRule
  std::string rule; std::vector<LetValue> params;
  // BlockClause (query above) / WhenBlock
  Block block; bool not_empty = false;
  Conj conditions;
  // TypeBlock
  std::shared_ptr<TypeBlock> tb;
};

struct TypeBlock {
  std::string type_name;
  bool has_conditions = false;
  Conj conditions;
  Block block;
  AccessQuery query;   // Resources.*[ Type == "<type_name>" ]
};

struct Rule { std::string name; bool has_conditions = false; Conj conditions; Block block; };
struct ParamRule { std::vector<std::string> params; Rule rule; };

struct RulesFile {
  std::vector<LetExpr> assignments;
  std::vector<Rule> rules;
  std::vector<ParamRule> param_rules;
};

// Returns false on a parse error (msg filled); `empty` set for a comment-only file.
bool parse_rules_file(const std::string& text, const std::string& file_name, RulesFile& out, bool& empty,
                      std::string& msg);

// context-string helpers (exprs.rs:286-393)
std::string slice_display(const std::vector<QueryPart>& parts, size_t from = 0);
std::string gac_display(const Clause& c);
std::string file_location_display(const FileLoc& l);
std::string value_only_display(const LitValue& v);

}  // namespace gg
