// Device-side evaluator state shared by the kernel TU and the host launcher.
#pragma once
#include <stdint.h>

#include "guard_types.h"

namespace gg {

struct DevProg {
  const PStr* strs;
  const PPart* parts;
  const PQuery* queries;
  const PClause* clauses;
  const PRange2* conjs;
  const PRange2* disjs;
  const uint32_t* clause_refs;
  const uint32_t* disj_refs;
  const PBlock* blocks;
  const PLet* lets;
  const PRule* rules;
  const PRange2* name_rules;
  const uint32_t* name_rule_ids;
  const PFunc* funcs;
  const PParamRule* params;
  const uint32_t* param_vars;
  const uint32_t* alts;
  const PRegex* regex;
  const uint16_t* dfa;
  const DNode* lit_nodes;
  const DRange* lit_ranges;
  const char* bytes;
  uint32_t root_block;
  uint32_t top_first;     // first top-level rule id
  uint32_t n_top;         // number of top-level rules
  uint32_t n_slots;
  uint32_t n_rules_total;
  uint32_t n_vars;        // variable ids (root-scope resolved-variable table: lets + captures)
  const uint32_t* blob;   // device blob the pointers above index into
  uint32_t lds_words;     // words the kernels stage in LDS: the whole blob when it fits the window,
                          // else everything before the regex DFA tables
  uint32_t dfa_lds;       // set by stage_program: the DFA tables were staged (dfa points into LDS)
  // is_match memo (eval_core.inc regex_match_ref): per regex of this program, 2 bits per 16-B slot of
  // the document string pool (0 unknown, 1 no match, 2 match) -- a regex's answer is a function of
  // the interned string alone, and a corpus repeats its strings across documents.  Null: no memo.
  uint32_t* rx_memo;
  uint32_t memo_words;    // words per regex
};

struct DevBatch {
  const DNodeP* nodes;     // packed device arena (guard_types.h DNodeP)
  const uint32_t* klen;    // per node: DNode.key_len (cold column)
  const char* bytes;
  const uint32_t* roots;   // per doc: root node (document-relative)
  const uint64_t* base;    // per doc: global index of the document's first node
  uint32_t ndocs;
  // CloudFormation resource-type column: for each document whose root has a `Resources` map,
  // tix[tix_off[d] + j] describes entry j of that map (TIX_* or the string id of its `Type`).
  // Built once per upload by resource_type_kernel; `Resources.*[ Type == '...' ]` filters read it
  // instead of walking every resource's entries.
  const uint32_t* res_map;   // per doc: document-relative node of root.Resources (map), or NONE
  const uint32_t* tix_off;   // per doc: first column entry
  uint32_t* tix;
  uint32_t type_key;         // string id of "Type" (NONE if no document has the key)
};

struct LaunchArgs {
  DevBatch docs;
  // lane-mode batch order: position p of the (chunk-major) document order evaluates document
  // order[p]; null = identity.  Tiles stay indexed by document, so results do not depend on it.
  const uint32_t* order;
  const DevProg* progs;    // per rules file
  uint32_t nfiles;
  uint32_t ntiles;         // ndocs * nfiles (tile = doc * nfiles + file)
  uint32_t tile_base;      // first tile index of this launch
  uint8_t* heaps;          // per wave slot scratch
  uint32_t heap_bytes;
  uint32_t nslots;         // number of wave slots (= grid size)
  TileOut* tiles;          // [ntiles]
  uint8_t* rule_status;    // [ntiles * max_top] 0 PASS 1 FAIL 2 SKIP
  uint32_t max_top;
  Rec* recs;               // global record arena
  uint32_t rec_cap;
  uint32_t* rec_cursor;    // atomic bump
  uint32_t* tile_cursor;   // atomic work queues: [0] lane-mode batches, [1] wave-mode tiles
  uint8_t* lane_heaps;     // lane mode: per lane scratch
  uint32_t lane_heap_bytes;
  uint32_t* retry_list;    // tiles the lane kernel hands to the wave kernel (null: wave kernel runs all)
  uint32_t* retry_count;
  uint32_t wave_frames_bytes;  // wave mode: frame region at the start of each wave heap
  uint32_t wave_recs_bytes;    // wave mode: record staging region after it
  uint32_t* retry2_list;       // tiles the wave pass hands to the large-heap pass (null: none)
  uint32_t* retry2_count;
  uint32_t* xcd_cursor;       // lane mode: one batch queue per XCD ([8])
  uint32_t lds_prog_words;    // program staging window (dynamic LDS, words; multiple of 4)
  uint32_t rec_chunk;         // lane mode: record slots per lane reserved per batch (direct writes; 0: off)
  uint32_t lane_recs_bytes;   // lane mode: record staging bytes per lane (a multiple of 48; after the 4 KB frames)
  uint32_t lane_docs;         // lane mode: documents per batch (lanes 0 .. lane_docs-1 of a wave; 64 or fewer)
  uint32_t lane_group;        // lane mode: lanes per document (1, or 64 / lane_docs: a document's lanes run its
                              // tile in step and split its list fan-outs' filter tests, eval_core.inc coop_chunk)
  uint32_t stack_guard;       // lane-stack bytes past which a recursion step ends the tile with E_STACK
                              // (capi.cpp: the device's stack limit minus the deepest uncheck-ed call chain)
  unsigned long long* stats;   // stats build variant: [0,8) counters, [8] tiles, [9,18) cycles per category
};

}  // namespace gg
