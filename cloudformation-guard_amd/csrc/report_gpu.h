// The structured JSON report rendered on the MI355X (BASELINE north_star: "the reporter (device status
// bitmaps to structured JSON/SARIF)").
//
// Restates, on the device, what reporter.cpp's streamed JSON writer (write_file_report / StreamWalker /
// JW) writes for a document: CommonStructuredReporter::report's FileReport per data file
// (reporters/validate/structured.rs:99-133), its not_compliant ClauseReports from the failure records
// (eval_context.rs:1965-2435 report_all_failed_clauses_for_rules / simplified_json_from_root), serde's
// pretty layout (2-space indent, "[]" / "{}" when empty) and the message texts (Display of
// PathAwareValue / UnResolved, display.rs:33-107).  One lane renders one document, twice: a size pass
// and a write pass at the offsets their scan gives (pool strings read 16 bytes at a time).  A document the device writer does not cover (a float,
// Debug-formatted reasons, map keys or count() values as values, ranges / chars, nesting past 48) is
// flagged in the size pass and written by the host writer at its position, so the bytes never depend on
// which writer ran.
#pragma once
#include <stdint.h>

#include "guard_types.h"

namespace gg {

struct RStr { uint32_t off, len; };

// one rules file's reporter tables (Program's host tables: context strings, custom messages, rule names,
// remaining-query texts, the literal arena with its parents and marks)
struct RProg {
  const char* text;          // every RStr of this struct indexes it
  const RStr* ctx;           // Program::ctx
  const RStr* msgs;          // Program::msgs
  const RStr* rule_names;    // Program::rule_names (by rule id)
  const uint32_t* rem_first; // per query id: first (query, step) entry
  const RStr* rem;           // Program::query_remaining(qid, step), steps 0 .. nparts
  const RStr* pkey;          // queries[qid][step].key
  const int32_t* pidx;       // queries[qid][step].index
  const PClause* clauses;
  const DNode* lit;          // literal arena (host layout: parent links, offsets into lit_bytes)
  const char* lit_bytes;
  const uint32_t* lit_line;
  const uint32_t* lit_col;
  uint32_t n_clauses, n_lit, n_rule_names, n_queries, n_ctx, n_msgs, pad0, pad1;
};

struct RenderArgs {
  // the document arena (packed nodes, key lengths, pool) and the reporter's per-node columns
  const DNodeP* nodes;
  const uint32_t* klen;
  const char* pool;
  const uint32_t* parent;
  const uint32_t* line;
  const uint32_t* col;
  const uint64_t* base;          // per document
  uint64_t n_nodes;              // arena nodes (bounds of every document reference)
  // evaluation results, as the evaluation kernels left them in HBM (records contiguous or strided in
  // their lane's chunk: TileOut.rec_off / pad1)
  const RProg* progs;
  uint32_t nfiles, max_top;
  const TileOut* tiles;
  const uint8_t* rule_status;
  const Rec* recs;
  // not_applicable / compliant: the distinct top-level rule names of all files, sorted; rank r is held
  // by the (file, rule) pairs fk[first[r] .. first[r] + n[r]) (file << 16 | top rule index)
  const char* sname_text;
  const RStr* sname;
  const uint32_t* sname_first;
  const uint32_t* sname_n;
  const uint32_t* sname_fk;
  uint32_t n_sname;
  // this block: documents [doc0, doc0 + ndocs); the report's first document is report_first (no ",\n")
  uint32_t doc0, ndocs, report_first, pad;
  const char* names;             // the block's document names, concatenated
  const uint64_t* name_off;      // [ndocs + 1]
  uint64_t* sizes;               // size pass: bytes per document, kHostDoc | reason for the host writer
  const uint64_t* offsets;       // write pass: each device document's offset in the block's text
  char* out;
};

static const uint64_t kHostDoc = 1ull << 63;

}  // namespace gg
