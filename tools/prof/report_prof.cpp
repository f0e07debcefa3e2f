// Host report-writer profiling harness (diagnostic, CPU only; not part of the library).
// Loads the cfg-2 rule pack and synthetic templates 0..N-1, reads a GPU run's results saved by
// gg_session_save_results (tools/report_replay.py save), and renders the structured JSON report
// with one thread, R times.  Build: make -C tools/prof (g++ -pg for gprof).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <dirent.h>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
#include <algorithm>

#include "doc_loader.h"
#include "program.h"
#include "reporter.h"
#include "rules_ast.h"
#include "synth_corpus.h"

using namespace gg;

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: report_prof RESULTS NDOCS PACKDIR [REPEAT]\n"); return 2; }
  const char* path = argv[1];
  const size_t nd = (size_t)atoll(argv[2]);
  const std::string pack = argv[3];
  const int rep = argc > 4 ? atoi(argv[4]) : 1;
  std::vector<std::string> files;
  if (DIR* d = opendir(pack.c_str())) {
    while (dirent* e = readdir(d)) { std::string n = e->d_name; if (n.size() > 6 && n.substr(n.size() - 6) == ".guard") files.push_back(n); }
    closedir(d);
  }
  std::sort(files.begin(), files.end());
  std::vector<Program> progs(files.size());
  for (size_t i = 0; i < files.size(); i++) {
    std::ifstream f(pack + "/" + files[i]);
    std::stringstream ss; ss << f.rdbuf();
    RulesFile rf; bool empty = false; std::string perr;
    if (!parse_rules_file(ss.str(), files[i], rf, empty, perr) || !compile_program(rf, files[i], progs[i], perr)) {
      fprintf(stderr, "rules %s: %s\n", files[i].c_str(), perr.c_str()); return 1;
    }
  }
  DocBatch docs;
  std::string text;
  for (size_t i = 0; i < nd; i++) {
    cfn_synth_doc(i, 50, text);
    LoadError le;
    if (!load_document(docs, text.data(), text.size(), "synthetic-" + std::to_string(i) + ".json", LOAD_LIBYAML, le)) {
      fprintf(stderr, "load %zu: %s\n", i, le.msg.c_str()); return 1;
    }
  }
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "cannot read %s\n", path); return 1; }
  uint64_t h[4];
  if (fread(h, sizeof h, 1, f) != 1 || h[1] != nd * progs.size()) { fprintf(stderr, "results do not match\n"); return 1; }
  std::vector<TileOut> tiles(h[1]);
  std::vector<uint8_t> rs(h[1] * h[2]);
  std::vector<Rec> recs(h[3]);
  if (fread(tiles.data(), sizeof(TileOut), h[1], f) != h[1] || fread(rs.data(), 1, rs.size(), f) != rs.size() ||
      fread(recs.data(), sizeof(Rec), h[3], f) != h[3]) { fprintf(stderr, "short read\n"); return 1; }
  fclose(f);
  std::vector<const Program*> pp;
  for (auto& p : progs) pp.push_back(&p);
  const size_t nf = pp.size(), max_top = h[2];
  auto tile = [&](size_t d, size_t fi) { return tile_view(tiles.data(), rs.data(), max_top, recs.data(), d * nf + fi); };
  size_t bytes = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < rep; r++) {
    std::vector<TextBuf> parts;
    ReportError re;
    if (!report_batch_json_parts(docs, pp, 0, nd, tile, 1, parts, re)) { fprintf(stderr, "report error %s\n", re.msg.c_str()); return 1; }
    bytes = json_parts_size(parts);
  }
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / rep;
  printf("%zu bytes in %.3f s = %.3f GB/s (1 thread)\n", bytes, s, bytes / s / 1e9);
  return 0;
}
