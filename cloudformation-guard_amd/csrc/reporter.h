// Device records -> structured FileReport JSON (byte-exact serde_json pretty output).
// Restates report_all_failed_clauses_for_rules / simplified_json_from_root
// (guard/src/rules/eval_context.rs:1965-2435) and FileReport::combine (:1630-1640) over the
// compact failure records emitted by the kernel.
#pragma once
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "doc_loader.h"
#include "guard_types.h"
#include "program.h"

namespace gg {

// Runs work(0) .. work(n - 1), work(0) on the calling thread and the others on their own threads.
// An exception escaping a worker (std::bad_alloc on a large report, a writer's runtime_error) would
// otherwise reach std::terminate on that thread; each is caught, all threads are joined, and the
// lowest-indexed worker's exception is rethrown on the caller, where the C API turns it into an
// extern_err_t.
template <class F>
void parallel_run(size_t n, F&& work) {
  std::vector<std::exception_ptr> ex(n);
  auto guarded = [&](size_t t) {
    try { work(t); } catch (...) { ex[t] = std::current_exception(); }
  };
  std::vector<std::thread> th;
  th.reserve(n ? n - 1 : 0);
  for (size_t t = 1; t < n; t++) th.emplace_back(guarded, t);
  if (n) guarded(0);
  for (auto& x : th) x.join();
  for (auto& e : ex) if (e) std::rethrow_exception(e);
}

// Non-owning view of one tile's device results (the session's fetched buffers).
struct RecSpan {
  const Rec* p = nullptr;
  size_t n = 0;
  size_t size() const { return n; }
  const Rec& operator[](size_t i) const { return p[i]; }
};
struct TileResult {
  TileOut out{};
  const uint8_t* rule_status = nullptr;  // per top-level rule
  RecSpan recs;                          // failure records, in evaluation order
  RecSpan aux;                           // side records (join-key lists of unresolved reasons R4 / R5)
};
// the view of tile t inside fetched session buffers (rec_n records, then pad0 aux records)
inline TileResult tile_view(const TileOut* tiles, const uint8_t* rule_status, size_t max_top, const Rec* recs, size_t t) {
  TileResult r;
  r.out = tiles[t];
  r.rule_status = rule_status + t * max_top;
  r.recs.p = recs + r.out.rec_off; r.recs.n = r.out.rec_n;
  r.aux.p = recs + r.out.rec_off + r.out.rec_n; r.aux.n = r.out.pad0;
  return r;
}

struct ReportError { bool set = false; std::string kind, msg; };

// One FileReport object for (doc, all programs) -- tiles[f] is the tile of program f.
// Appends pretty JSON (indent level `indent`) to out.  Returns false + err on an abort.
bool report_document(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                     const std::vector<const TileResult*>& tiles, int indent, std::string& out, ReportError& err);

// guard-ffi run_checks(verbose = true) (commands/helper.rs:62-64): the serde pretty EventRecord tree
// (rules/mod.rs:165-355, eval_context.rs:990-997) from the verbose kernel's event records of one tile.
bool verbose_tree(const DocBatch& docs, uint32_t doc, const Program& prog, const TileResult& tile, const std::string& data_name,
                  std::string& out, ReportError& err);

// error text for a tile error (Error Display, guard/src/rules/errors.rs:11-54)
void tile_error(const DocBatch& docs, uint32_t doc, const Program& prog, const TileOut& t, ReportError& err);

std::string error_display(const std::string& kind, const std::string& msg);

// `validate --structured -o {json|yaml|sarif|junit}` writers over the same FileReports
// (reporters/validate/structured.rs:99-133, sarif.rs, xml.rs + reporters/mod.rs).
enum OutFormat : int32_t { OUT_JSON = 0, OUT_YAML = 1, OUT_SARIF = 2, OUT_JUNIT = 3 };

// `cfn-guard test` (commands/test.rs, reporters/test/{generic,structured}.rs): per test case, the
// rules grouped by name in first-appearance order with their expected / evaluated statuses.
enum : int32_t { OUT_TEXT = 4 };   // the test command's default single-line-summary text report
struct TestRuleResult {
  std::string rule;
  int32_t expected = -1;              // ST_*; -1: no expectation set for the rule
  int32_t matched = -1;               // get_status_result: the matched status, -1 = FAIL
  std::vector<uint32_t> evaluated;    // statuses seen before the match (FAIL: all of them)
};
// print_verbose_tree (commands/validate.rs:685-687) of a verbose-kernel tile: the EventRecord tree
// as Display lines (display.rs:128-328)
bool verbose_text(const DocBatch& docs, uint32_t doc, const Program& prog, const TileResult& tile, const std::string& data_name,
                  std::string& out, ReportError& err);

// `cfn-guard validate` without --structured (commands/validate.rs:690-758): one (data file, rules file)
// pair's console output -- the summary table (-S), the CFN / Terraform / generic single-line reporter
// (-o single-line-summary) or the pair's FileReport (-o json / yaml), then --verbose's EventRecord tree
// and --print-json.  `tile` is the throughput kernel's tile of the pair, `vtile` the verbose kernel's;
// `text` the data file's source (the CFN reporter prints code around failing values).
struct ConsoleOptions {
  uint32_t summary = 2;            // SummaryType bits: 1 PASS, 2 FAIL, 4 SKIP (0: -S none)
  int32_t format = OUT_TEXT;       // OUT_TEXT (single-line-summary), OUT_JSON or OUT_YAML
  bool verbose = false, print_json = false;
};
bool console_report(const DocBatch& docs, uint32_t doc, const std::string& text, const Program& prog,
                    const TileResult& tile, const TileResult& vtile, const ConsoleOptions& opt, std::string& out,
                    ReportError& err);

struct TestCaseResult {
  bool has_name = false;
  std::string name;
  std::vector<TestRuleResult> rules;
  std::string tree;                   // --verbose: the case's EventRecord tree as text (verbose_text)
};
struct TestSpecFile {
  std::string error;                  // non-empty: the spec file did not parse (Error Display)
  std::vector<TestCaseResult> cases;
};
std::string test_report(int32_t fmt, const std::string& rules_name, const std::vector<TestSpecFile>& files,
                        int32_t& exit_code);
// one rules file's TestResult: its spec files' results, or parse_error (the rules file did not parse)
struct TestResultIn {
  std::string rules_name;
  std::vector<TestSpecFile> files;
  std::string parse_error;
};
// structured (json / yaml / junit) report of one TestResult (single) or of a Vec<TestResult>
std::string test_report_list(int32_t fmt, const std::vector<TestResultIn>& results, int32_t& exit_code, bool single);

class ReportWriter {
 public:
  explicit ReportWriter(int32_t fmt);
  ~ReportWriter();
  ReportWriter(const ReportWriter&) = delete;
  ReportWriter& operator=(const ReportWriter&) = delete;
  // one data file; tiles[f] is its tile of program f.  false + err on an aborting error.
  bool add(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
           const std::vector<const TileResult*>& tiles, ReportError& err);
  std::string finish();
  // appends the documents of `later` (a writer over the next contiguous documents); JSON, SARIF
  // and JUnit only
  void absorb(ReportWriter& later);

 private:
  struct Impl;
  Impl* p_;
};

// SARIF around the device-rendered results (capi.cpp device_report_sarif): one FAILed document's
// SarifResults, each as ",\n" + the results array's indent + the pretty object (the device writer's
// layout; the report's first comma is dropped), nothing for another status; and the report's text before
// and after the results' items for these artifacts (FAILed documents' first-seen non-empty names).
bool sarif_doc_results(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                       const std::vector<const TileResult*>& tiles, std::string& out, ReportError& err);
void sarif_frame(const std::vector<std::string>& artifact_names, std::string& head, std::string& tail);

// The structured report of documents [first, first + ndocs) rendered on `nthreads` host threads over
// contiguous document ranges; byte-identical to one ReportWriter fed in order.  tile(d, f) gives
// document d's tile of program f.
bool report_batch(const DocBatch& docs, const std::vector<const Program*>& progs, size_t first, size_t ndocs,
                  const std::function<TileResult(size_t doc, size_t file)>& tile, int32_t fmt, unsigned nthreads,
                  std::string& out, ReportError& err);

// report_batch in two halves, so several shards' reports join into one: the unfinished writers of
// documents [first, first + ndocs) in order (JSON / SARIF / JUnit), or for YAML each range's finished
// stream (a block sequence's items concatenate).  report_writers_finish absorbs the writers in order
// (or joins the YAML streams) -- the bytes one writer fed every document in order writes.
bool report_batch_writers(const DocBatch& docs, const std::vector<const Program*>& progs, size_t first, size_t ndocs,
                          const std::function<TileResult(size_t doc, size_t file)>& tile, int32_t fmt, unsigned nthreads,
                          std::vector<std::unique_ptr<ReportWriter>>& writers, std::vector<std::string>& yaml_parts,
                          ReportError& err);
std::string report_writers_finish(int32_t fmt, std::vector<std::unique_ptr<ReportWriter>>& writers,
                                  std::vector<std::string>& yaml_parts);

// Growable text buffer for the streamed JSON writer: malloc / realloc storage (large blocks grow by
// mremap, without a copy) and std::string's append interface, so fragment appends are an inline bounds
// check and a memcpy instead of a std::string::append call each.
struct TextBuf {
  char* p = nullptr;
  size_t n = 0, cap = 0;
  TextBuf() = default;
  TextBuf(const TextBuf&) = delete;
  TextBuf& operator=(const TextBuf&) = delete;
  TextBuf(TextBuf&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
  TextBuf& operator=(TextBuf&& o) noexcept { std::swap(p, o.p); std::swap(n, o.n); std::swap(cap, o.cap); return *this; }
  ~TextBuf() { release(); }
  // storage: malloc below kHugeMin, then huge-page backed mmap regions (doc_loader.h huge_alloc) grown
  // by mremap, which moves the pages without copying them
  void release() {
    if (cap >= kHugeMin) huge_free(p, cap); else free(p);
    p = nullptr; n = cap = 0;
  }
  void reserve(size_t k) {
    if (k <= cap) return;
    size_t nc = cap * 2 > k ? cap * 2 : k;
    if (nc < 4096) nc = 4096;
    char* q;
    if (nc < kHugeMin) {
      q = (char*)realloc(p, nc);
      if (!q) throw std::bad_alloc();
    } else {
      nc = (nc + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
      if (cap >= kHugeMin) {
        void* r = mremap(p, cap, nc, MREMAP_MAYMOVE);
        if (r == MAP_FAILED) throw std::bad_alloc();
        q = (char*)r;
        madvise(q + cap, nc - cap, MADV_HUGEPAGE);
      } else {
        q = (char*)huge_alloc(nc);
        if (n) memcpy(q, p, n);
        free(p);
      }
    }
    p = q; cap = nc;
  }
  // kSlack bytes past the end are always allocated, so short copies may store whole 8 / 16-byte
  // words past the new end (they are overwritten by later appends or ignored)
  static constexpr size_t kSlack = 64;
  char* grow(size_t k) { if (n + k + kSlack > cap) reserve(n + k + kSlack); char* r = p + n; n += k; return r; }
  void push_back(char c) { *grow(1) = c; }
  void append(const char* s, size_t k) {
    char* d = grow(k);
    if (k >= 8 && k <= 16) {   // two overlapping words: no libc call for the writer's many short tokens
      uint64_t a, b;
      memcpy(&a, s, 8); memcpy(&b, s + k - 8, 8);
      memcpy(d, &a, 8); memcpy(d + k - 8, &b, 8);
    } else if (k >= 4 && k < 8) {
      uint32_t a, b;
      memcpy(&a, s, 4); memcpy(&b, s + k - 4, 4);
      memcpy(d, &a, 4); memcpy(d + k - 4, &b, 4);
    } else if (k < 4) {
      for (size_t i = 0; i < k; i++) d[i] = s[i];
    } else {
      memcpy(d, s, k);
    }
  }
  void append(size_t k, char c) {
    char* d = grow(k);
    if (c == ' ' && k <= 256) {   // indentation: 16-byte stores of spaces (may run into the slack)
      static const char sp[16] = {' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' '};
      for (size_t i = 0; i < k; i += 16) {
        if (n - k + i + 16 > cap) { memset(d + i, ' ', k - i); break; }
        memcpy(d + i, sp, 16);
      }
    } else if (k) {
      memset(d, c, k);
    }
  }
  TextBuf& operator+=(char c) { push_back(c); return *this; }
  TextBuf& operator+=(const char* s) { append(s, strlen(s)); return *this; }
  TextBuf& operator+=(const std::string& s) { append(s.data(), s.size()); return *this; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const char* data() const { return p; }
  void resize(size_t m) { if (m <= n) n = m; else append(m - n, '\0'); }
  void clear() { n = 0; }
};

// JSON only, for large reports: the FileReports of documents [first, first + ndocs) rendered on
// `nthreads` host threads into contiguous parts, not concatenated.  The report's text is
// "[\n" + parts joined by ",\n" + "\n]" ("[]" with no parts): json_parts_size is its length,
// json_parts_join a malloc'd NUL-terminated copy built in one parallel pass.
bool report_batch_json_parts(const DocBatch& docs, const std::vector<const Program*>& progs, size_t first, size_t ndocs,
                             const std::function<TileResult(size_t doc, size_t file)>& tile, unsigned nthreads,
                             std::vector<TextBuf>& parts, ReportError& err);
size_t json_parts_size(const std::vector<TextBuf>& parts);
// one document's FileReport, streamed JSON at indent 1 (what report_batch_json_parts writes per document,
// without the separator and the two leading spaces); false + err on an abort
bool report_json_doc(const DocBatch& docs, uint32_t doc, const std::vector<const Program*>& progs,
                     const std::vector<const TileResult*>& tiles, TextBuf& out, ReportError& err);
size_t json_parts_count(const std::vector<TextBuf>& parts);   // non-empty parts
char* json_parts_join(const std::vector<TextBuf>& parts);

}  // namespace gg
