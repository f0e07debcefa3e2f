// Shared host/device data layout for the MI355X batch evaluator.
//
// Document arena (columnar, one per batch of documents, resident in HBM):
//   DNode[]  -- 32 B per value node.  A map's / list's children are contiguous.
//   bytes[]  -- string pool (scalar strings and map keys, UTF-8, not NUL terminated)
// Rules program (one per rules file): flat arrays of PPart/PQuery/PClause/... plus a
// literal arena in the same DNode format.  A node reference (u32) with bit 31 set
// addresses the literal arena, otherwise the document arena.
//
// Reference mapping:
//   DNode           <- PathAwareValue            guard/src/rules/path_value.rs:171-185
//   PPart           <- QueryPart                 guard/src/rules/exprs.rs:64-73
//   PClause         <- GuardClause/RuleClause    exprs.rs:224-268
//   QR              <- QueryResult / UnResolved  guard/src/rules/mod.rs:165-177
//   Rec             <- RecordType (failure subset) mod.rs:278-355
#pragma once
#include <stdint.h>

namespace gg {

enum Kind : uint32_t {
  K_NULL = 0, K_STRING = 1, K_REGEX = 2, K_BOOL = 3, K_INT = 4, K_FLOAT = 5, K_CHAR = 6,
  K_LIST = 7, K_MAP = 8, K_RANGE_INT = 9, K_RANGE_FLOAT = 10, K_RANGE_CHAR = 11,
};

static const uint32_t NONE = 0xFFFFFFFFu;
// resource-type column entries (eval_kernel.hip resource_type_kernel): a string id, or
static const uint32_t TIX_UNDECIDED = 0xFFFFFFFFu;   // not a map / no exact `Type` key / Type is a list
static const uint32_t TIX_NOT_STRING = 0xFFFFFFFEu;  // `Type` present but neither string nor list
static const uint32_t LIT_BIT = 0x80000000u;

struct DNode {
  uint32_t kind;     // Kind
  uint32_t count;    // containers: #children; string/regex: byte length
  uint32_t a;        // containers: first child; string/regex: byte offset; int/float: low word;
                     // bool: 0/1; char: code point; range: index into range table
  uint32_t b;        // int/float: high word; string: hash32 of the bytes; regex: regex id
  uint32_t key_off;  // when the parent is a map: key byte offset (else NONE)
  uint32_t key_len;
  uint32_t key_hash;
  uint32_t parent;   // parent node (NONE for a root); host uses it to rebuild JSON pointers
};

// Device arena node (16 B): what the evaluator reads of a DNode, half its size so a map's entries
// and a key scan's batch share fewer cache lines.  kc = kind | count << 4 (count < 2^28); a, b as in
// DNode; key_hash = the key id of a map entry (DNode.key_hash == DNode.key_off for document nodes;
// 0 for other nodes).  DNode.key_len lives in a separate cold column (read only when a map key is
// used as a value); DNode.parent and the marks stay on the host.  Built from the host arena at
// upload by pack_nodes_kernel.
struct DNodeP {
  uint32_t kc, a, b, key_hash;
};
static const uint32_t kMaxPackedCount = (1u << 28) - 1;

struct DRange {      // RangeType<T> (values.rs:232-278)
  uint64_t lo, hi;   // i64 / f64 bits / char code point
  uint32_t incl;     // LOWER_INCLUSIVE=1 | UPPER_INCLUSIVE=2
  uint32_t kind;
};

// ---------------------------------------------------------------- program ---
enum PartKind : uint32_t {
  P_THIS = 0, P_KEY = 1, P_KEY_INDEX = 2, P_KEY_VAR = 3, P_VAR_HEAD = 4, P_INDEX = 5,
  P_ALL_VALUES = 6, P_ALL_INDICES = 7, P_FILTER = 8, P_MAP_KEY_FILTER = 9,
};

struct PStr { uint32_t off, len, hash, pad; };

struct PPart {
  uint32_t kind;
  uint32_t a;   // KEY: pstr id; KEY_INDEX/INDEX: (int32) index; KEY_VAR/VAR_HEAD: var id;
                // ALL_*: capture var id or NONE; FILTER: conj id
  uint32_t b;   // KEY: first of 7 converter-alternate pstr ids (alts[]); FILTER: capture var id
  uint32_t c;
};

struct PQuery { uint32_t first, n, match_all, pad; };

enum ClauseKind : uint32_t {
  C_ACCESS = 0, C_NAMED = 1, C_BLOCK = 2, C_WHEN = 3, C_TYPEBLOCK = 4, C_PARAM = 5,
  C_UNSUPPORTED = 6,
};

enum CmpOp : uint32_t {
  OP_EQ = 0, OP_IN = 1, OP_GT = 2, OP_LT = 3, OP_LE = 4, OP_GE = 5, OP_EXISTS = 6, OP_EMPTY = 7,
  OP_IS_STRING = 8, OP_IS_LIST = 9, OP_IS_MAP = 10, OP_IS_BOOL = 11, OP_IS_INT = 12,
  OP_IS_FLOAT = 13, OP_IS_NULL = 14,
};

enum RhsKind : uint32_t { RHS_NONE = 0, RHS_LITERAL = 1, RHS_QUERY = 2, RHS_FUNC = 3 };

struct PClause {
  uint32_t kind;
  uint32_t flags;   // ACCESS: op | not<<4 | negation<<5 | rhs_kind<<8 | empty_on_expr<<12
                    // NAMED/PARAM: negation; BLOCK: not_empty
  uint32_t a;       // ACCESS/BLOCK/TYPEBLOCK: query id; NAMED: name slot; WHEN: cond conj;
                    // PARAM: param-rule id; UNSUPPORTED: message id
  uint32_t b;       // ACCESS: rhs (literal node ref | query id | func id); BLOCK/WHEN/TYPEBLOCK: block id;
                    // PARAM: first arg (PLet-shaped LetValue list)
  uint32_t c;       // TYPEBLOCK: cond conj or NONE; PARAM: nargs
  uint32_t d;       // host: context string id
  uint32_t e;       // host: custom message id (NONE if none)
  uint32_t f;       // host: secondary context id
};

struct PRange2 { uint32_t first, n; };      // conj -> disj ids ; disj -> clause ids
struct PBlock { uint32_t first_let, nlets, conj, is_rule_level; };
enum LetKind : uint32_t { L_LITERAL = 0, L_QUERY = 1, L_FUNC = 2 };
struct PLet { uint32_t var, kind, id, pad; };   // id: literal node ref | query id | func id
struct PRule { uint32_t name_slot, cond, block, pad; };
struct PFunc { uint32_t fname, first_arg, nargs, pad; };   // args: PLet (var unused)
struct PParamRule { uint32_t rule, first_param, nparams, pad; }; // params: var ids in vars[]
// regex DFA (regex_dfa.h) over code-point classes, in the program's u16 DFA section (offsets in
// u16 units): next-state table at `table` (nstates x ncls), accept flags at `accept` (u16 per state:
// 1 = match decided, 2 = match at the end of the haystack), the ASCII class map at `ascii` (128
// bytes) and, at `bounds`, flags >> 8 u32 words (first code point << 8 | class) sorted by code point
// for the classes above U+007F.  flags bit 0: unsupported on the MI355X path.
// flags: bit 0 unsupported, bit 1 NFA simulation (table = its u32 tables, kNfa* layout), bits 8.. class runs
struct PRegex { uint32_t table, nstates, start, flags, ncls, accept, ascii, bounds; };

// nfa_tab layout (u32 words): header [kNfaM] states m, [kNfaW] words per bitset W = ceil(m / 32),
// [kNfaCls] classes, [kNfaNb] class runs above U+007F, [kNfaStartFlags] / [kNfaAgainFlags] flags of S0 / Z;
// then S0[W] (closure of the start state at offset 0), Z[W] (its closure elsewhere: the unanchored
// restart), FL[m] (flags of each state's follow set), F[m][W] (follow set of each state: the closure of
// its successor), M[ncls][W] (states whose class set holds the class), ascii[128] (class per ASCII code
// point), runs[nb][2] (first code point, class).  Flags: 1 = the match state is in the set, 2 = an
// end-of-text assertion is (a match if the haystack ends here).
enum : uint32_t { kNfaM = 0, kNfaW = 1, kNfaCls = 2, kNfaNb = 3, kNfaStartFlags = 4, kNfaAgainFlags = 5, kNfaHdr = 8,
                  kNfaMaxStates = 1024, kNfaMaxWords = kNfaMaxStates / 32 };


enum FuncName : uint32_t { F_COUNT = 0, F_OTHER = 1 };

struct ProgHeader {
  uint32_t magic, nwords;
  uint32_t off_strs, n_strs;
  uint32_t off_parts, n_parts;
  uint32_t off_queries, n_queries;
  uint32_t off_clauses, n_clauses;
  uint32_t off_conjs, n_conjs;
  uint32_t off_disjs, n_disjs;
  uint32_t off_clause_refs, n_clause_refs;
  uint32_t off_disj_refs, n_disj_refs;
  uint32_t off_blocks, n_blocks;
  uint32_t off_lets, n_lets;
  uint32_t off_rules, n_rules;
  uint32_t off_name_rules, n_name_rules;   // per name slot: PRange2 into name_rule_ids
  uint32_t off_name_rule_ids, n_name_rule_ids;
  uint32_t off_funcs, n_funcs;
  uint32_t off_params, n_params;
  uint32_t off_param_vars, n_param_vars;
  uint32_t off_alts, n_alts;
  uint32_t off_regex, n_regex;
  uint32_t off_dfa, n_dfa;
  uint32_t off_lit_nodes, n_lit_nodes;     // DNode as 8 words
  uint32_t off_lit_ranges, n_lit_ranges;   // DRange as 6 words
  uint32_t off_bytes, n_bytes;             // program bytes (pstr + literal strings), packed 4/word
  uint32_t root_block;                     // file-level lets (conj unused)
  uint32_t n_vars;
  uint32_t n_name_slots;
  uint32_t max_lets;
};

// ------------------------------------------------------------ query result ---
enum QrKind : uint32_t { QR_RESOLVED = 0, QR_LITERAL = 1, QR_UNRESOLVED = 2, QR_SYNTH_INT = 3 };

enum Reason : uint32_t {
  R_NONE = 0, R_INDEX_OOB = 1, R_NO_MORE_ENTRIES = 2, R_KEY_INDEX_NOT_ARRAY = 3,
  R_VAR_INDEX_OOB = 4, R_VAR_KEYS_UNRESOLVED = 5, R_LOCATE_KEY = 6, R_LOCATE_KEY_LIST = 7,
  R_KEY_NOT_FOUND = 8, R_NOT_STRUCT = 9, R_INDEX_NOT_ARRAY = 10, R_FILTER_NOT_STRUCT = 11,
  R_MAPFILTER_NOT_STRUCT = 12,
};

struct QR {
  uint32_t node;   // resolved/literal node ref, or traversed_to for unresolved,
                   // or (SYNTH_INT) the node whose path the value carries (NONE = root path)
  uint32_t meta;   // kind (bits 0-1) | reason << 8
  uint32_t uref;   // unresolved: query id << 12 | remaining-query start step; SYNTH_INT: value lo
  uint32_t aux;    // reason operand; SYNTH_INT: value hi
};

// ----------------------------------------------------------------- records ---
enum RecKind : uint32_t {
  REC_RULE_OPEN = 1, REC_RULE_CLOSE = 2, REC_DISJ_OPEN = 3, REC_DISJ_CLOSE = 4,
  REC_BLOCK_EMPTY = 5, REC_MISSING_BLOCK_VALUE = 6, REC_UNARY = 7, REC_NOVALUE_EMPTY = 8,
  REC_DEPENDENT_RULE = 9, REC_CMP = 10, REC_IN = 11, REC_LIST = 12,
  REC_AUX = 13,   // side record (TileOut.pad0 of them after the tile's records): join-key lists of R4 / R5
  // verbose kernel only (the EventRecord tree, rules/mod.rs:278-355): every event is recorded, in
  // evaluation order -- container opens / closes and one leaf per value check (failure records
  // above, REC_SUCCESS for ClauseCheck::Success)
  REC_EV_OPEN = 14,    // clause: rule / clause id (NONE for file, disjunction, filter); x: EvType; y: TypeBlock value index | filter #conjunctions
  REC_EV_CLOSE = 15,   // clause, x as the open; y: status | at_least_one_matches << 8; from.uref: RuleCheck custom message id
  REC_SUCCESS = 16,    // clause id (NONE: a map-key-filter comparison, context "")
};

enum EvType : uint32_t {
  EV_FILE = 0, EV_RULE = 1, EV_RULE_COND = 2, EV_DISJ = 3, EV_GAC = 4, EV_NAMED = 5, EV_BLOCK = 6, EV_WHEN = 7,
  EV_WHEN_COND = 8, EV_TYPE = 9, EV_TYPE_COND = 10, EV_TYPE_VAL = 11, EV_FILTER_MAP = 12, EV_FILTER_LIST = 13,
};

// NotComparable reasons carried in Rec.x for REC_CMP
enum NcReason : uint32_t {
  NC_NONE = 0, NC_TYPES = 1, NC_FLOAT = 2, NC_STRING_IN = 3, NC_CONTAINED_IN = 4,
};

struct Rec {        // 48 B
  uint32_t kind;
  uint32_t clause;  // clause id (RULE_OPEN: rule id)
  uint32_t x;       // REC_CMP: NcReason; REC_IN: #to entries; RULE_OPEN: custom message id
  uint32_t y;
  QR from;
  QR to;            // REC_CMP: kind bits == 3 + meta high bit => "no to"
};

// ------------------------------------------------------------------ errors ---
enum ErrKind : uint32_t {
  E_OK = 0, E_UNSUPPORTED = 1, E_HEAP = 2, E_EMPTY_INCOMPATIBLE = 3, E_TYPEBLOCK_UNRESOLVED = 4,
  E_VAR_MISSING = 5, E_RULE_MISSING = 6, E_INTERP_NON_STRING = 7, E_INTERP_QUERY = 8,
  E_PARAM_MISSING = 9, E_PARAM_ARITY = 10, E_NO_RHS = 11, E_RECORDS = 12, E_DEPTH = 13,
  E_REGEX_UNSUPPORTED = 14, E_STACK = 15,
};

// per-tile result header written by the kernel
struct TileOut {
  uint32_t status;     // file status: 0 PASS 1 FAIL 2 SKIP
  uint32_t err;        // ErrKind
  uint32_t err_a, err_b;
  uint32_t rec_off;    // offset into the global record arena
  uint32_t rec_n;      // failure records; then pad0 side records (REC_AUX and their pairs)
  uint32_t pad0, pad1;
};

static const uint32_t ST_PASS = 0, ST_FAIL = 1, ST_SKIP = 2;

}  // namespace gg
