// Device records -> structured FileReport JSON (byte-exact serde_json pretty output).
// Restates report_all_failed_clauses_for_rules / simplified_json_from_root
// (guard/src/rules/eval_context.rs:1965-2435) and FileReport::combine (:1630-1640) over the
// compact failure records emitted by the kernel.
#pragma once
#include <string>
#include <vector>

#include "doc_loader.h"
#include "guard_types.h"
#include "program.h"

namespace gg {

struct TileResult {
  TileOut out;
  std::vector<uint8_t> rule_status;  // per top-level rule
  std::vector<Rec> recs;
};

struct ReportError { bool set = false; std::string kind, msg; };

// One FileReport object for (doc, all programs) -- tiles[f] is the tile of program f.
// Appends pretty JSON (indent level `indent`) to out.  Returns false + err on an abort.
bool report_document(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                     const std::vector<const TileResult*>& tiles, int indent, std::string& out, ReportError& err);

// error text for a tile error (Error Display, guard/src/rules/errors.rs:11-54)
void tile_error(const DocBatch& docs, uint32_t doc, const Program& prog, const TileOut& t, ReportError& err);

std::string error_display(const std::string& kind, const std::string& msg);

}  // namespace gg
