// Synthetic CloudFormation-shaped corpus generator (see synth_corpus.cpp).
#pragma once
#include <cstdint>
#include <string>

namespace gg {
// JSON text of synthetic template `index` with `n_resources` resources (synth.py cfn_doc).
void cfn_synth_doc(uint64_t index, int n_resources, std::string& out);
// the same template as block-style YAML (synth.py cfn_yaml_doc)
void cfn_synth_yaml_doc(uint64_t index, int n_resources, std::string& out);
}  // namespace gg
