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
};

// Appends `n` documents (texts[i] of lens[i] bytes, named names[i]) to the EMPTY batch `out`.
// Returns false with `why` set when any document is outside the subset the device parser proves
// identical to the host loader (the caller then loads the batch on the host); `out` is unchanged.
bool gpu_load_json(DocBatch& out, const char* const* texts, const size_t* lens, const std::vector<std::string>& names,
                   size_t n, GpuLoadStats& st, std::string& why);

}  // namespace gg
