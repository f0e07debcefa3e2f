// GPU document loader: strict-JSON documents -> the columnar node arena,
// parsed on the MI355X.  Produces exactly the arena the host JSON fast path builds
// (doc_loader.cpp load_json_fast: same node layout, marks and scalar typing), with string ids
// interned batch-wide on the device.  Replaces, for JSON input, the reference's
// Loader::load + PathAwareValue::try_from (guard/src/rules/libyaml/loader.rs:31-195,
// guard/src/rules/path_value.rs:414-478).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "doc_loader.h"

namespace gg {

struct GpuLoadStats {
  double kernel_ms = 0;        // parse + intern kernels (HIP events)
  double h2d_ms = 0, d2h_ms = 0;
  uint64_t text_bytes = 0, nodes = 0, distinct_strings = 0, pool_bytes = 0;
  uint32_t table_retries = 0;   // intern-table doublings
  uint64_t refused_docs = 0;    // documents outside the device subset, built by the host loader
};

// Appends `n` documents (texts[i] of lens[i] bytes, named names[i]) to the EMPTY batch `out`.
// A document outside the subset the device parser proves identical to the host loader (libyaml-only
// syntax, duplicate keys, nesting past 64, a float beyond the exact fast path, a raw character libyaml
// reads specially) is refused on its own: with `refused` non-null its index is appended there and
// `out` holds an empty placeholder for it (the caller builds it with the host loader); with
// `refused` null the whole batch is refused.  Returns false with `why` set when the batch is refused
// (batch-wide limits, or strict mode); `out` is then unchanged.  With `keep_nodes` non-null the
// device copy of out.nodes (dev_alloc'ed, out.nodes.size() DNodes) is handed to the caller, who
// frees it with dev_free (dev_cache.h): the session packs its arena from it instead of uploading the nodes again.
//
// With `resident` non-null as well (and no document refused) the per-node columns stay in HBM: out.nodes,
// line, col, kline, kcol are left EMPTY, the device copies are handed over in *resident (node count
// st.nodes; the caller owns every pointer, dev_free), and only the pool, the intern index, bases and names
// reach the host.  The session copies the columns down when a host consumer first needs them
// (capi.cpp ensure_host_arena); a job whose reports are all rendered on the device never does.
struct ResidentArena {
  uint32_t* line = nullptr;    // per node mark
  uint32_t* col = nullptr;
  uint32_t* kline = nullptr;   // per map-entry node: its key's mark
  uint32_t* kcol = nullptr;
  uint64_t nodes = 0;          // 0: the columns came down to the host (out is complete)
};
bool gpu_load_json(DocBatch& out, const char* const* texts, const size_t* lens, const std::vector<std::string>& names,
                   size_t n, GpuLoadStats& st, std::string& why, std::vector<uint32_t>* refused = nullptr,
                   void** keep_nodes = nullptr, ResidentArena* resident = nullptr);

}  // namespace gg
