// C ABI + HIP runtime for the MI355X evaluator.
//
// Drop-in boundary (guard-ffi/src/lib.rs:32-47, guard-ffi/example/cfn_guard.h):
//   char* cfn_guard_run_checks(validate_input_t data, validate_input_t rules, _Bool verbose, extern_err_t* err)
//   void  cfn_guard_free_string(char*)
// plus a batched entry point (`validate --structured -o json` over many documents and rules files)
// and a session API used by bench.py / tests (documents resident in HBM across evaluations).
//
// There is no CPU evaluation path: every evaluation launches guard_eval_kernel on the GPU, and the
// library reports an explicit error when no HIP device is present.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <unordered_map>
#include <unordered_set>

#include "../../include/cfn_guard_mi355x.h"
#include "dev_cache.h"
#include "host_pinned.h"
#include "doc_loader.h"
#include "eval_device.h"
#include "host_format.h"
#include "json_gpu.h"
#include "eisel_lemire.h"
#include "program.h"
#include "report_gpu.h"
#include "reporter.h"
#include "synth_corpus.h"

namespace gg {
__global__ void guard_eval_kernel(LaunchArgs A);
__global__ void guard_eval_verbose_kernel(LaunchArgs A);
__global__ void guard_eval_lanes_kernel(LaunchArgs A);
// the same kernels with the regex NFA simulation (eval_kernel_nfa.hip), for programs that need it
__global__ void guard_eval_kernel_nfa(LaunchArgs A);
__global__ void guard_eval_verbose_kernel_nfa(LaunchArgs A);
__global__ void guard_eval_lanes_kernel_nfa(LaunchArgs A);
__global__ void resource_type_kernel(DevBatch D);
__global__ void shape_key_kernel(DevBatch D, const uint32_t* top8, unsigned long long* key);
void device_segmented_order(const unsigned long long* key, uint32_t* order, uint32_t n, const uint32_t* seg_host,
                            uint32_t nseg, hipStream_t st);
__global__ void root_resources_kernel(const DNode* nodes, const uint64_t* base, const uint32_t* roots, uint32_t nd, uint32_t rkey,
                                      uint32_t* rmap, uint32_t* cnt);
__global__ void pack_nodes_kernel(const DNode* in, DNodeP* out, uint32_t* klen, uint32_t* parent, uint64_t n, uint32_t* bad);
__global__ void report_kernel(RenderArgs A, uint32_t write);
__global__ void report_sarif_kernel(RenderArgs A, uint32_t write);
void d2h_push(void* dst, const void* src, size_t bytes, hipStream_t st, int blocks);
__global__ void rec_block_sums_kernel(const TileOut* tiles, uint32_t n, uint32_t* bsum);
__global__ void rec_scan_sums_kernel(uint32_t* bsum, uint32_t nb, uint32_t* total);
__global__ void rec_compact_kernel(const TileOut* tiles, uint32_t n, const uint32_t* bsum, const Rec* src, Rec* dst,
                                   uint32_t* dense_off);
__global__ void rule_count_kernel(const TileOut* tiles, const uint8_t* rule_status, const DevProg* progs, uint32_t nfiles,
                                  uint32_t ntiles, uint32_t max_top, unsigned long long* counts);
}

using namespace gg;

namespace {

char* dup_str(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  return p;
}

int32_t ffi_code(const std::string& kind) {
  static const char* names[] = {"", "JsonError", "YamlError", "FormatError", "IoError", "ParseError", "RegexError",
                                "MissingProperty", "MissingVariable", "MultipleValues", "IncompatibleRetrievalError",
                                "IncompatibleError", "NotComparable", "ConversionError", "Errors", "RetrievalError",
                                "MissingValue", "FileNotFoundError", "IllegalArguments"};
  for (int i = 1; i < 19; i++) if (kind == names[i]) return i;
  if (kind == "XMLError") return 20;
  return -1;   // InternalError / unsupported: ffi-support's panic code
}

void set_err(extern_err_t* err, int32_t code, const std::string& msg) {
  if (!err) return;
  err->code = code;
  err->message = code ? dup_str(msg) : nullptr;
}

// code 0 with a message: an informational verdict (the device loader's refusal / difference)
void set_note(extern_err_t* err, const std::string& msg) {
  if (!err) return;
  err->code = 0;
  err->message = dup_str(msg);
}

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_) + " at " #x); } } while (0)

// Device contexts, created lazily per HIP device under one mutex ("device contexts
// created lazily and guarded by a mutex").  The single-device entry points use the process default
// device: the device current on the first calling thread -- torch.cuda.set_device(LOCAL_RANK) in a
// one-process-per-GPU job -- or GG_DEVICE.  cfn_guard_validate_batch_devices names its devices.
static constexpr int kMaxDevices = 64;
static size_t default_stack_bytes() {
  return getenv("GG_STACK_BYTES") ? (size_t)atol(getenv("GG_STACK_BYTES")) : (size_t)16384;
}
// The evaluator checks its lane stack pointer where it recurses (eval_core.inc stack_low); between two
// checks a call chain can grow the stack by at most this much.  tools/stack_budget.py derives the bound from
// the product ISA (per-function frames and call edges; round 6: 1056 B, the wave kernel's eval_conj ->
// parameterized rule -> eval_rule -> eval_conj chain, 1104 B in the NFA variant) and checks that this margin
// covers it.
static constexpr size_t kStackMargin = 3072;
struct DeviceState {
  bool ready = false;
  int ncu = 256;
  uint32_t stack_guard = 16384 - (uint32_t)kStackMargin;
};
struct Devices {
  std::mutex mu;
  int count = -1;    // visible devices (-1: not probed yet)
  int def = -1;      // process default device (-1: not resolved yet)
  DeviceState dev[kMaxDevices];
  // under mu: probes the devices once, initialises device d
  bool init(int d, std::string& why) {
    if (count < 0) {
      int n = 0;
      if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
      count = std::min(n, kMaxDevices);
    }
    if (count == 0) { why = "no HIP device available (the MI355X path has no CPU fallback)"; return false; }
    if (d < 0 || d >= count) { why = "HIP device " + std::to_string(d) + " out of range (" + std::to_string(count) + " visible)"; return false; }
    DeviceState& D = dev[d];
    if (D.ready) return true;
    if (hipSetDevice(d) != hipSuccess) { why = "hipSetDevice failed"; return false; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) == hipSuccess) D.ncu = prop.multiProcessorCount;
    // the recursive evaluator (eval_recursive.inc: eval_conj <-> clauses, filters, rule references) needs a
    // dynamic lane stack: 16 KB for every kernel variant, the NFA one included (its simulation is a leaf
    // call, eval_core.inc nfa_match_*), set once and never raised; GG_STACK_BYTES overrides.  The kernels'
    // stack guard is what the runtime actually granted minus kStackMargin.
    hipDeviceSetLimit(hipLimitStackSize, default_stack_bytes());
    size_t granted = 0;
    if (hipDeviceGetLimit(&granted, hipLimitStackSize) != hipSuccess || !granted) granted = default_stack_bytes();
    D.stack_guard = granted > kStackMargin + 1024 ? (uint32_t)(granted - kStackMargin) : 1024u;
    D.ready = true;
    return true;
  }
  int resolve_default(std::string& why) {
    if (def >= 0) return def;
    int d = 0;
    if (const char* e = getenv("GG_DEVICE")) d = atoi(e);
    else if (hipGetDevice(&d) != hipSuccess) d = 0;
    if (!init(d, why)) { if (why.find("out of range") != std::string::npos) why = "GG_DEVICE / current device out of range"; return -1; }
    def = d;
    return d;
  }
};
Devices g_devs;
int dev_ncu(int d) { return g_devs.dev[d >= 0 && d < kMaxDevices ? d : 0].ncu; }
uint32_t dev_stack_guard(int d) { return g_devs.dev[d >= 0 && d < kMaxDevices ? d : 0].stack_guard; }

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  size_t cap = 0;
  // ensures room for `count` elements (contents undefined); an allocation large enough is kept, so
  // pooled buffers serve later calls without hipMalloc / hipFree
  void alloc(size_t count) {
    n = count;
    if (count <= cap && p) return;
    // a growing buffer may still be read by work queued on its session's stream: hipFree waits for it --
    // for the whole device, so a pooled set growing in a streamed batch waited for the other chunk's report
    // (chunk 3's upload 2.8 s instead of 50 ms, 7.7-9.3 s per 1 M templates against 5.1-5.3 s when no set grew,
    // profiles/r06zf_stream_*).  Growth is made rare: a buffer of 1 MB or more asks for 1/8 headroom (the next
    // chunk's arena is a few percent larger or smaller), and the capacity is the cache's whole size class.
    dev_free_sync(p);
    p = nullptr;
    n = count;
    cap = 0;
    if (count) {
      const size_t want = count * sizeof(T) >= ((size_t)1 << 20) ? count + count / 8 : count;
      HIPCHK(dev_alloc(&p, want * sizeof(T)));
      cap = std::max(want, dev_cache_class(want * sizeof(T)) / sizeof(T));
    }
  }
  // alloc with headroom: a growing buffer is reallocated rarely (hipFree synchronises the whole device,
  // which would serialise the device reporter's overlapped render and copy-out)
  void alloc_grow(size_t count) {
    if (count <= cap && p) { n = count; return; }
    alloc(count + count / 4 + 64);
    n = count;
  }
  void upload(const T* src, size_t count, hipStream_t s) {
    alloc(count);
    if (count) HIPCHK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s));
  }
  // after every stream that used the buffer is drained (~DeviceBufs destroys its streams first)
  void release() { dev_free(p); p = nullptr; n = 0; cap = 0; }
  size_t bytes() const { return cap * sizeof(T); }
  ~DBuf() { release(); }
};

// String ids of a rules program against a document batch: a program string (query key, case
// converted key, string literal, literal map key) gets the batch's id for the same text, or an id
// above every pool offset (shared by equal texts) when no document has it, so the device compares
// program and document strings by id.  Patches a copy of the blob.
struct StringIds {
  std::unordered_map<std::string, uint32_t> absent;
  uint32_t id(const DocBatch& docs, const char* p, uint32_t n) {
    uint32_t off = docs.find(p, n);
    if (off != NONE) return off;
    auto it = absent.find(std::string(p, n));
    if (it != absent.end()) return it->second;
    uint32_t v = 0xF0000000u + (uint32_t)absent.size();
    absent.emplace(std::string(p, n), v);
    return v;
  }
};

std::vector<uint32_t> canonical_blob(const Program& prog, const DocBatch& docs, StringIds& ids) {
  std::vector<uint32_t> b = prog.blob;
  const ProgHeader& h = prog.hdr;
  const char* pb = (const char*)(prog.blob.data() + h.off_bytes);
  PStr* strs = (PStr*)(b.data() + h.off_strs);
  for (uint32_t i = 0; i < h.n_strs; i++) strs[i].hash = ids.id(docs, pb + strs[i].off, strs[i].len);
  DNode* lit = (DNode*)(b.data() + h.off_lit_nodes);
  for (uint32_t i = 0; i < h.n_lit_nodes; i++) {
    if (lit[i].kind == K_STRING) lit[i].b = ids.id(docs, pb + lit[i].a, lit[i].count);
    if (lit[i].key_off != NONE) lit[i].key_hash = ids.id(docs, pb + lit[i].key_off, lit[i].key_len);
  }
  return b;
}

struct GpuProgram {
  Program prog;
  DBuf<uint32_t> blob;
  DevProg dp{};
  std::vector<uint32_t> staged;   // canonical copy of prog.blob (kept alive for the async upload)
  void upload(hipStream_t s, const DocBatch& docs, StringIds& ids) {
    staged = canonical_blob(prog, docs, ids);
    blob.upload(staged.data(), staged.size(), s);
    const uint32_t* b = blob.p;
    const ProgHeader& h = prog.hdr;
    dp.strs = (const PStr*)(b + h.off_strs);
    dp.parts = (const PPart*)(b + h.off_parts);
    dp.queries = (const PQuery*)(b + h.off_queries);
    dp.clauses = (const PClause*)(b + h.off_clauses);
    dp.conjs = (const PRange2*)(b + h.off_conjs);
    dp.disjs = (const PRange2*)(b + h.off_disjs);
    dp.clause_refs = b + h.off_clause_refs;
    dp.disj_refs = b + h.off_disj_refs;
    dp.blocks = (const PBlock*)(b + h.off_blocks);
    dp.lets = (const PLet*)(b + h.off_lets);
    dp.rules = (const PRule*)(b + h.off_rules);
    dp.name_rules = (const PRange2*)(b + h.off_name_rules);
    dp.name_rule_ids = b + h.off_name_rule_ids;
    dp.funcs = (const PFunc*)(b + h.off_funcs);
    dp.params = (const PParamRule*)(b + h.off_params);
    dp.param_vars = b + h.off_param_vars;
    dp.alts = b + h.off_alts;
    dp.regex = (const PRegex*)(b + h.off_regex);
    dp.dfa = (const uint16_t*)(b + h.off_dfa);
    dp.lit_nodes = (const DNode*)(b + h.off_lit_nodes);
    dp.lit_ranges = (const DRange*)(b + h.off_lit_ranges);
    dp.bytes = (const char*)(b + h.off_bytes);
    dp.root_block = h.root_block;
    dp.top_first = prog.blob[sizeof(ProgHeader) / 4];
    dp.n_top = prog.blob[sizeof(ProgHeader) / 4 + 1];
    dp.n_slots = h.n_name_slots;
    dp.n_rules_total = h.n_rules;
    dp.n_vars = h.n_vars;
    dp.blob = b;
    dp.lds_words = h.nwords;   // stage_program falls back to the words before the DFA tables
    dp.dfa_lds = 0;
  }
};

// Device state of one evaluation: arena, programs, scratch heaps, records, tallies, a stream and
// launch events.  Borrowed by a session at upload and returned to a small pool when it ends, so
// repeated FFI calls (guard-lambda, the fuzzers: one document per call) reuse allocations, events
// and streams instead of hipMalloc'ing ~100 MB per call; concurrent callers each hold their own.
struct DeviceBufs {
  DBuf<DNodeP> d_nodes;         // packed device arena
  DBuf<uint32_t> d_klen;        // per node key length (cold)
  DBuf<uint32_t> d_parent;      // per node parent (device reporter: JSON pointers)
  DBuf<uint32_t> d_line, d_col; // per node marks (device reporter), uploaded at its first use
  DBuf<uint8_t> d_rtab;         // device reporter tables (RProg sections, sorted rule names)
  DBuf<RProg> d_rprogs;
  // per block set (two: one renders while the other is copied out): names, sizes, offsets, slots,
  // overflow area, contiguous text
  struct RenderSet {
    DBuf<char> names, text;
    DBuf<uint64_t> name_off, sizes, offs;
  } rset[2];
  hipStream_t copy_stream = nullptr;
  // shader copy-out (d2h_push) with CU masks: the copy kernel on push_stream's CUs, the report's render
  // kernels on render_stream's (the rest), so the two do not share a CU (GG_PUSH_CUS)
  hipStream_t push_stream = nullptr, render_stream = nullptr;
  int push_cus = -1;
  char* pinned = nullptr;       // host staging for report text (kPinnedBytes)
  static constexpr size_t kPinnedBytes = (size_t)256 << 20;
  DBuf<char> d_bytes;
  DBuf<uint32_t> d_roots;
  DBuf<uint64_t> d_base;
  DBuf<uint32_t> d_res_map;     // per doc: root.Resources node (resource-type column, DevBatch)
  DBuf<uint32_t> d_tix_off;
  DBuf<uint32_t> d_order;       // lane-mode document order (shape-sorted batches), empty = identity
  DBuf<uint32_t> d_tix;
  DBuf<DevProg> d_progs;
  DBuf<uint32_t> d_rx_memo;     // regex is_match memo over the string pool (DevProg::rx_memo)
  DBuf<uint8_t> d_heaps;        // wave mode: one heap per wave slot
  DBuf<uint8_t> d_lane_heaps;   // lane mode: one heap per lane
  DBuf<uint32_t> d_retry;       // tiles handed from lane mode to wave mode
  DBuf<uint8_t> d_big_heaps;    // large-heap wave pass (allocated the first time a tile needs it)
  DBuf<uint32_t> d_retry2;      // tiles handed from the wave pass to the large-heap pass
  DBuf<TileOut> d_tiles;
  DBuf<uint8_t> d_rule_status;
  DBuf<Rec> d_recs;
  DBuf<Rec> d_recs_dense;       // session_fetch: the records compacted into tile order
  DBuf<uint32_t> d_dense_off;   // ... and each tile's offset in it
  DBuf<uint32_t> d_bsum;        // compaction block sums (+ total)
  DBuf<uint32_t> d_counters;
  DBuf<unsigned long long> d_counts;   // per (file, top rule) x {PASS, FAIL, SKIP, error}
  DBuf<unsigned long long> d_stats;    // diagnostic counters (stats build variant)
  hipStream_t stream = nullptr;
  int device = 0;               // the HIP device every buffer above lives on
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evq;   // launch brackets, reused
  explicit DeviceBufs(int d) : device(d) { HIPCHK(hipSetDevice(d)); HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)); }
  ~DeviceBufs() {
    hipSetDevice(device);
    if (pinned) pinned_free(pinned);
    if (copy_stream) hipStreamDestroy(copy_stream);
    if (push_stream) hipStreamDestroy(push_stream);
    if (render_stream) hipStreamDestroy(render_stream);
    for (auto& pr : evq) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
    if (stream) hipStreamDestroy(stream);
  }
  // every device buffer back to the device block cache (the stream, events and pinned staging stay)
  void release_device() {
    d_nodes.release(); d_klen.release(); d_parent.release(); d_line.release(); d_col.release(); d_rtab.release(); d_rprogs.release();
    // GG_KEEP_RENDER=1 (diagnostic): the report's text buffers stay with the set (copy-out rate A/B)
    static const bool keep_render = getenv("GG_KEEP_RENDER") && atoi(getenv("GG_KEEP_RENDER")) != 0;
    if (!keep_render)
      for (auto& r : rset) { r.names.release(); r.text.release(); r.name_off.release(); r.sizes.release(); r.offs.release(); }
    d_bytes.release(); d_roots.release(); d_base.release(); d_res_map.release(); d_tix_off.release(); d_order.release(); d_tix.release();
    d_progs.release(); d_rx_memo.release(); d_heaps.release(); d_lane_heaps.release(); d_retry.release(); d_big_heaps.release();
    d_retry2.release(); d_tiles.release(); d_rule_status.release(); d_recs.release(); d_recs_dense.release(); d_dense_off.release();
    d_bsum.release(); d_counters.release(); d_counts.release(); d_stats.release();
  }
  size_t bytes() const {
    return d_nodes.bytes() + d_klen.bytes() + d_parent.bytes() + d_line.bytes() + d_col.bytes() + d_rtab.bytes() +
           rset[0].text.bytes() + rset[1].text.bytes() + d_bytes.bytes() + d_roots.bytes() + d_base.bytes() + d_res_map.bytes() +
           d_tix_off.bytes() + d_tix.bytes() + d_progs.bytes() + d_rx_memo.bytes() + d_heaps.bytes() + d_lane_heaps.bytes() + d_retry.bytes() +
           d_big_heaps.bytes() + d_retry2.bytes() + d_tiles.bytes() + d_rule_status.bytes() + d_recs.bytes() +
           d_recs_dense.bytes() + d_dense_off.bytes() + d_bsum.bytes() +
           d_counters.bytes() + d_counts.bytes() + d_stats.bytes();
  }
};

struct BufPool {
  std::mutex mu;
  std::vector<DeviceBufs*> free;
  static constexpr size_t kMaxFree = 8;               // idle sets kept
  static constexpr size_t kMaxKeepBytes = 1ull << 30; // larger sets (batch jobs) keep no device buffers
};
BufPool g_pool[kMaxDevices];   // one per device: a set's buffers and stream belong to its device

DeviceBufs* acquire_bufs(int d) {
  {
    std::lock_guard<std::mutex> lk(g_pool[d].mu);
    if (!g_pool[d].free.empty()) { DeviceBufs* b = g_pool[d].free.back(); g_pool[d].free.pop_back(); return b; }
  }
  return new DeviceBufs(d);
}

void release_bufs(DeviceBufs* b) {
  if (!b) return;
  hipSetDevice(b->device);
  if (hipStreamSynchronize(b->stream) == hipSuccess && (!b->copy_stream || hipStreamSynchronize(b->copy_stream) == hipSuccess) &&
      (!b->push_stream || hipStreamSynchronize(b->push_stream) == hipSuccess) &&
      (!b->render_stream || hipStreamSynchronize(b->render_stream) == hipSuccess)) {
    // a larger set (a batch job) keeps only its stream, events and pinned staging: its device buffers go
    // to the block cache, where the next batch's allocations find them (deleting the set would
    // hipHostFree the staging, which waits for the device to go idle)
    if (b->bytes() > BufPool::kMaxKeepBytes) b->release_device();
    std::lock_guard<std::mutex> lk(g_pool[b->device].mu);
    if (g_pool[b->device].free.size() < BufPool::kMaxFree) { g_pool[b->device].free.push_back(b); return; }
  }
  delete b;
}

}  // namespace

// ------------------------------------------------------------------ session ---
struct gg_session {
  DocBatch docs;
  std::vector<std::unique_ptr<GpuProgram>> progs;
  std::vector<std::string> parse_errors;   // rules files that failed to parse (exit code 5)
  std::unique_ptr<DocBatch> params;        // merged input parameters (validate -i), one document
  int device = -1;                         // HIP device (-1: the process default, resolved at first use)
  // device residency: buffers borrowed from the device's pool at upload (DeviceBufs)
  DeviceBufs* dv = nullptr;
  uint32_t type_key = NONE;
  bool has_order = false;   // d_order holds a lane-mode document order (shape-sorted batches)
  size_t ncounts = 0;
  hipStream_t stream = nullptr;        // caller stream (e.g. torch's current stream); null = the buffers' own stream
  hipEvent_t ev0 = nullptr, ev1 = nullptr;   // brackets of the most recent launch (= dv->evq[nq - 1])
  size_t nq = 0;
  // the device loader's copy of docs.nodes[0, dev_nodes_n) (hipMalloc'ed): the next upload packs the
  // arena from it instead of sending the nodes over PCIe again, then frees it
  void* dev_nodes = nullptr;
  size_t dev_nodes_n = 0;
  // device-resident arena (gpu_load_json ResidentArena): docs.nodes / line / col / kline / kcol are
  // empty on the host and live in HBM (dev_nodes, resident.*) until a host consumer needs them
  // (ensure_host_arena); dev_nodes then outlives the upload
  ResidentArena resident;
  std::mutex arena_mu;
  unsigned long long* ext_counts = nullptr;   // caller-owned device tally buffer (RCCL all-reduce)
  bool launched = false;
  std::vector<unsigned long long> counts;
  bool uploaded = false;
  uint32_t max_top = 1;
  uint32_t nslots = 0;            // wave-mode grid
  uint32_t lane_slots = 0;        // lane-mode grid (waves)
  uint32_t lane_docs = 64;        // lane mode: documents per batch (session_upload)
  uint32_t lane_group = 1;        // lane mode: lanes per document (64 / lane_docs in lane groups, else 1)
  uint32_t heap_bytes = 512 * 1024;
  static constexpr uint32_t kWaveFrames = 16 * 1024, kWaveRecs = 64 * 1024;
  // large-heap pass (rare: documents with thousands of failing clause values or deep nesting)
  static constexpr uint32_t kBigHeap = 32u << 20, kBigFrames = 1u << 20, kBigRecs = 16u << 20, kBigSlots = 8;
  uint32_t lane_heap_bytes = 64 * 1024;
  uint32_t lane_heap_set = 0;     // gg_session_configure's lane heap (0: sized at upload)
  uint32_t lane_recs_bytes = 24576;   // record staging per lane (eval_core.inc RECS_BYTES by default)
  uint32_t lds_prog_words = 2048;              // per-launch program staging window (words)
  static constexpr uint32_t kMaxLdsProgWords = 4096;   // 16 KB
  int32_t mode = 0;               // 0: lane mode + wave-mode retry; 1: wave mode only
  bool verbose = false;           // wave mode recording the EventRecord tree (guard_eval_verbose_kernel)
  size_t rec_cap = 0;
  uint32_t rec_chunk = 0;         // lane mode: direct record slots per lane per batch (eval_core.inc rec_store)
  size_t rx_memo_words = 0;       // words of the regex is_match memo (0: none)
  bool rx_memo_per_launch = false;   // zero the memo before every launch (bench: no warm memo across steps)
  bool marks_on_device = false;   // d_line / d_col hold docs.line / docs.col (device reporter)
  bool fetched_on_device = false; // the fetched results are the device's (tiles, dense records): it can report them
  // session_fetch leaves the dense records on the device (the streamed batch: its device report reads
  // them there); ensure_host_arena copies them down for a host writer.  recs_pending: not copied yet.
  bool defer_recs = false;
  bool recs_pending = false;
  uint32_t recs_total = 0;
  bool rtab_ready = false;        // d_rtab / d_rprogs built for the current programs
  int32_t device_report = -1;     // 1: JSON reports rendered on the device, 0: host, -1: GG_DEVICE_REPORT (default 1)
  // device reporter: the sorted rule-name tables inside d_rtab (render_tables)
  const char* r_sname_text = nullptr;
  const RStr* r_sname = nullptr;
  const uint32_t *r_sname_first = nullptr, *r_sname_n = nullptr, *r_sname_fk = nullptr;
  uint32_t r_nsname = 0;
  // results
  std::vector<TileOut> tiles;
  std::vector<uint8_t> rule_status;
  std::vector<Rec> recs;
  bool evaluated = false;
  double last_kernel_ms = 0;
  std::string last_error;
  ~gg_session() {
    if (device >= 0) hipSetDevice(device);
    // work enqueued on a caller stream (gg_session_set_stream) may still read or write these buffers:
    // drain it before the set goes back to the pool, where the next session's uploads reuse it
    if (dv && stream) hipStreamSynchronize(stream);
    release_bufs(dv);
    dev_free(dev_nodes);
    for (uint32_t* p : {resident.line, resident.col, resident.kline, resident.kcol}) dev_free(p);
  }
};

namespace {

// makes device `d` (-1: the process default) current on this host thread, creating its context on
// first use; *out receives the ordinal.  The current device is per host thread: FFI callers may arrive
// on any thread.
bool ensure_device(std::string& why, int d = -1, int* out = nullptr) {
  std::lock_guard<std::mutex> lk(g_devs.mu);
  if (d < 0) { d = g_devs.resolve_default(why); if (d < 0) return false; }
  else if (!g_devs.init(d, why)) return false;
  if (hipSetDevice(d) != hipSuccess) { why = "hipSetDevice failed"; return false; }
  if (out) *out = d;
  return true;
}

// the session's device current on this thread (resolving the process default on first use)
void bind_device(gg_session* s) {
  std::string why;
  if (!ensure_device(why, s->device, &s->device)) throw std::runtime_error(why);
}

// arena nodes of the session's documents, on the host or resident in HBM
size_t arena_nodes(const gg_session* s) { return s->resident.nodes ? (size_t)s->resident.nodes : s->docs.nodes.size(); }

// Copies a device-resident arena's columns down to the host batch (the host writers, tile errors, host
// loads appended to the session need them); a no-op once they are there.  Thread-safe per session.
void compact_records_to_host(gg_session* s);
void ensure_host_arena(gg_session* s) {
  std::lock_guard<std::mutex> lk(s->arena_mu);
  if (s->recs_pending) {   // host writers read the records as well: compacted, in tile order
    bind_device(s);
    compact_records_to_host(s);
  }
  if (!s->resident.nodes) return;
  bind_device(s);
  const size_t N = s->resident.nodes;
  if (!s->dev_nodes || s->dev_nodes_n != N) throw std::runtime_error("resident arena: its node copy is gone");
  DocBatch& D = s->docs;
  std::thread a([&]() { D.nodes.resize(N); });
  std::thread b([&]() { D.line.resize(N); D.col.resize(N); });
  D.kline.resize(N); D.kcol.resize(N);
  a.join(); b.join();
  HIPCHK(hipMemcpy(D.nodes.data(), s->dev_nodes, N * sizeof(DNode), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(D.line.data(), s->resident.line, N * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(D.col.data(), s->resident.col, N * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(D.kline.data(), s->resident.kline, N * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(D.kcol.data(), s->resident.kcol, N * 4, hipMemcpyDeviceToHost));
  for (uint32_t* p : {s->resident.line, s->resident.col, s->resident.kline, s->resident.kcol}) dev_free(p);
  s->resident = ResidentArena{};
  // the upload packed its arena already: the unpacked copy is no longer needed
  if (s->uploaded) { dev_free(s->dev_nodes); s->dev_nodes = nullptr; s->dev_nodes_n = 0; }
}

void session_upload(gg_session* s) {
  bind_device(s);
  const bool trace = getenv("GG_LOAD_TRACE") != nullptr;
  const auto tu = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (trace) fprintf(stderr, "[upload] %-22s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tu).count());
  };
  if (s->dv && s->dv->device != s->device) { release_bufs(s->dv); s->dv = nullptr; HIPCHK(hipSetDevice(s->device)); }
  if (!s->dv) s->dv = acquire_bufs(s->device);
  hipStream_t st = s->dv->stream;
  {
    // host arena (32 B nodes) -> device arena (16 B packed nodes + key-length column)
    const size_t n = arena_nodes(s);
    // lane-mode tiles address their document by a 32-bit global node index (eval_core.inc Ctx)
    if (n >= 0xFFFFFFFFull) throw std::runtime_error("batch too large for one session: split it (>= 2^32 arena nodes)");
    DBuf<DNode> tmp;
    const DNode* src = nullptr;
    if (s->dev_nodes && s->dev_nodes_n <= n) {
      // the device loader's nodes are already in HBM: only nodes the host appended since (documents
      // the device refused, built by the host loader) cross PCIe
      if (s->dev_nodes_n == n) {
        src = (const DNode*)s->dev_nodes;
      } else {
        tmp.alloc(n);
        HIPCHK(hipMemcpyAsync(tmp.p, s->dev_nodes, s->dev_nodes_n * sizeof(DNode), hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(tmp.p + s->dev_nodes_n, s->docs.nodes.data() + s->dev_nodes_n,
                              (n - s->dev_nodes_n) * sizeof(DNode), hipMemcpyHostToDevice, st));
        src = tmp.p;
      }
    } else {
      tmp.upload(s->docs.nodes.data(), n, st);
      src = tmp.p;
    }
    s->dv->d_nodes.alloc(std::max<size_t>(n, 1));
    s->dv->d_klen.alloc(std::max<size_t>(n, 1));
    s->dv->d_parent.alloc(std::max<size_t>(n, 1));
    s->marks_on_device = false;
    s->rtab_ready = false;
    s->fetched_on_device = false;
    s->recs_pending = false;
    DBuf<uint32_t> bad;
    bad.alloc(1);
    HIPCHK(hipMemsetAsync(bad.p, 0, 4, st));
    if (n) {
      const uint32_t blocks = (uint32_t)std::min<size_t>((n + 255) / 256, (size_t)dev_ncu(s->device) * 64);
      hipLaunchKernelGGL(pack_nodes_kernel, dim3(blocks), dim3(256), 0, st, src, s->dv->d_nodes.p, s->dv->d_klen.p, s->dv->d_parent.p,
                         (uint64_t)n, bad.p);
      HIPCHK(hipGetLastError());
    }
    uint32_t b = 0;
    HIPCHK(hipMemcpyAsync(&b, bad.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (s->dev_nodes && !s->resident.nodes) { dev_free(s->dev_nodes); s->dev_nodes = nullptr; s->dev_nodes_n = 0; }
    if (b & 1u) throw std::runtime_error("a string or container is too large for the device arena (count >= 2^28)");
    if (b & 2u) throw std::runtime_error("arena invariant broken: a map entry's key offset is not its key id");
    if (b & 4u) throw std::runtime_error("arena invariant broken: a string id is not a 16-byte pool slot");
    mark("packed");
  }
  s->dv->d_bytes.upload(s->docs.bytes.data(), s->docs.bytes.size() ? s->docs.bytes.size() : 1, st);
  s->dv->d_roots.upload(s->docs.roots.data(), s->docs.roots.size(), st);
  s->dv->d_base.upload(s->docs.base.data(), s->docs.base.size(), st);
  {
    // resource-type column layout: root.Resources of every document and its entry count
    const DocBatch& D = s->docs;
    const uint32_t rkey = D.find("Resources", 9);
    s->type_key = D.find("Type", 4);
    size_t nd = D.ndocs();
    std::vector<uint32_t> rmap(std::max<size_t>(nd, 1), NONE), toff(std::max<size_t>(nd, 1), 0);   // one entry at least: the uploads below
    size_t total = 0;
    // a resident arena: the first documents' nodes (the type-frequency sample below) come down, and the
    // root scan runs on the device (root_resources_kernel, json_gpu.hip)
    std::vector<DNode> sample;
    const DNode* HN = D.nodes.data();
    const size_t nsample = std::min<size_t>(nd, 4096);
    if (s->resident.nodes && nd) {
      const size_t sn = nsample < nd ? (size_t)D.base[nsample] : (size_t)s->resident.nodes;
      sample.resize(std::max<size_t>(sn, 1));
      HIPCHK(hipMemcpyAsync(sample.data(), s->dev_nodes, sn * sizeof(DNode), hipMemcpyDeviceToHost, st));
      HN = sample.data();
      if (rkey != NONE && s->type_key != NONE) {
        DBuf<uint32_t> d_rm, d_cnt;
        d_rm.alloc(nd); d_cnt.alloc(nd);
        hipLaunchKernelGGL(root_resources_kernel, dim3(std::min<uint32_t>((uint32_t)((nd + 255) / 256), dev_ncu(s->device) * 16)),
                           dim3(256), 0, st, (const DNode*)s->dev_nodes, s->dv->d_base.p, s->dv->d_roots.p, (uint32_t)nd, rkey,
                           d_rm.p, d_cnt.p);
        HIPCHK(hipGetLastError());
        std::vector<uint32_t> cnt(nd);
        HIPCHK(hipMemcpyAsync(rmap.data(), d_rm.p, nd * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(cnt.data(), d_cnt.p, nd * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (size_t d = 0; d < nd; d++) { toff[d] = (uint32_t)total; total += cnt[d]; }
      }
      HIPCHK(hipStreamSynchronize(st));
    } else if (rkey != NONE && s->type_key != NONE) {
      for (size_t d = 0; d < nd; d++) {
        const DNode* N = D.nodes.data() + D.base[d];
        const DNode& root = N[D.roots[d]];
        toff[d] = (uint32_t)total;
        if (root.kind != K_MAP) continue;
        for (uint32_t k = 0; k < root.count; k++) {
          const DNode& e = N[root.a + k];
          if (e.key_hash != rkey) continue;
          if (e.kind == K_MAP) { rmap[d] = root.a + k; total += e.count; }
          break;
        }
      }
    }
    mark("resource map");
    if (total > 0xFFFFFFF0u) { std::fill(rmap.begin(), rmap.end(), NONE); total = 0; }
    s->has_order = false;

    s->dv->d_res_map.upload(rmap.data(), std::max<size_t>(nd, 1), st);
    s->dv->d_tix_off.upload(toff.data(), std::max<size_t>(nd, 1), st);
    s->dv->d_tix.alloc(std::max<size_t>(total, 1));
    // the column is a property of the documents (the Type string id of each Resources entry), so it
    // is built once per upload with the packed arena, not per evaluation
    if (s->type_key != NONE && nd) {
      DevBatch B{};
      B.nodes = s->dv->d_nodes.p; B.klen = s->dv->d_klen.p; B.bytes = s->dv->d_bytes.p; B.roots = s->dv->d_roots.p;
      B.base = s->dv->d_base.p; B.ndocs = (uint32_t)nd;
      B.res_map = s->dv->d_res_map.p; B.tix_off = s->dv->d_tix_off.p; B.tix = s->dv->d_tix.p; B.type_key = s->type_key;
      const uint32_t blocks = std::min<uint32_t>((B.ndocs + 3) / 4, dev_ncu(s->device) * 16);
      hipLaunchKernelGGL(resource_type_kernel, dim3(blocks), dim3(256), 0, st, B);
      HIPCHK(hipGetLastError());
      if (trace) { HIPCHK(hipStreamSynchronize(st)); mark("type column kernel"); }
      // Shape-sorted batches: the lane kernel's 64 lanes run in lock-step, so a batch costs the union
      // of its documents' paths.  Documents are ordered by their counts of the 8 most frequent Type
      // strings (taken from the first documents; most frequent first) inside each XCD's eighth of the
      // chunks -- every XCD keeps a representative share -- so a batch's documents have similar shapes
      // (cfg-2: lane kernel 56.4 -> 49.9 ms, profiles/r02_ab_inline.log).  Results do not depend on the
      // order: tiles stay indexed by document.  GG_SHAPE_SORT=0 keeps load order.
      const bool sort_on = !getenv("GG_SHAPE_SORT") || atoi(getenv("GG_SHAPE_SORT")) != 0;
      if (sort_on && nd > 64) {
        std::unordered_map<uint32_t, uint32_t> freq, tlen;
        for (size_t d = 0; d < nsample; d++) {
          if (rmap[d] == NONE) continue;
          const DNode* N = HN + D.base[d];
          const DNode& m = N[rmap[d]];
          for (uint32_t j = 0; j < m.count; j++) {
            const DNode& r = N[m.a + j];
            if (r.kind != K_MAP) continue;
            for (uint32_t k = 0; k < r.count; k++) {
              const DNode& e = N[r.a + k];
              if (e.key_hash == s->type_key && e.kind == K_STRING) { freq[e.b]++; tlen[e.b] = e.count; break; }
            }
          }
        }
        // rank: types the rules files name (as a literal) first -- by how many files name them --
        // then by frequency, so the primary sort key aligns the most-checked resource type
        mark("type sample");
        std::vector<std::pair<uint32_t, uint32_t>> top(freq.begin(), freq.end());
        std::unordered_map<uint32_t, uint32_t> named;
        for (auto& tp : top) {
          const std::string tstr(D.bytes.data() + tp.first, tlen[tp.first]);
          uint32_t nf = 0;
          for (auto& gp : s->progs) if (!tstr.empty() && gp->prog.lit.bytes.find(tstr) != std::string::npos) nf++;
          named[tp.first] = nf;
        }
        std::sort(top.begin(), top.end(), [&](auto& a, auto& b) {
          if (named[a.first] != named[b.first]) return named[a.first] > named[b.first];
          return a.second != b.second ? a.second > b.second : a.first < b.first;
        });
        uint32_t top8[8];
        for (int i = 0; i < 8; i++) top8[i] = i < (int)top.size() ? top[i].first : TIX_UNDECIDED;
        DBuf<uint32_t> d_top;
        d_top.upload(top8, 8, st);
        DBuf<unsigned long long> d_key;
        d_key.alloc(nd);
        hipLaunchKernelGGL(shape_key_kernel, dim3(std::min<uint32_t>((uint32_t)((nd + 255) / 256), dev_ncu(s->device) * 16)), dim3(256), 0, st,
                           B, (const uint32_t*)d_top.p, d_key.p);
        HIPCHK(hipGetLastError());
        mark("shape keys");
        // each XCD's eighth of the 64-document chunks sorted by key on the device, ties in load order
        // (host threads with a comparator reading key[] at random took 0.4-0.6 s at 1M documents)
        const size_t nchunks = (nd + 63) / 64;
        uint32_t seg[9];
        for (size_t x = 0; x <= 8; x++) seg[x] = (uint32_t)std::min(nd, (size_t)(nchunks * x / 8) * 64);
        seg[8] = (uint32_t)nd;
        s->dv->d_order.alloc(nd);
        device_segmented_order(d_key.p, s->dv->d_order.p, (uint32_t)nd, seg, 8, st);
        mark("order sorted");
        s->has_order = true;
      }
    }
    HIPCHK(hipStreamSynchronize(st));   // the host vectors above die at the end of this scope
    mark("type column + order");
  }
  std::vector<DevProg> dps;
  s->max_top = 1;
  StringIds ids;
  // regex is_match memo: 2 bits per 16-B pool slot per regex, zeroed once per upload (the pool and
  // the programs are fixed for the session's life)
  const uint32_t memo_words = (uint32_t)std::min<size_t>(s->docs.bytes.size() / 256 + 1, 0xFFFFFFFFull);
  size_t memo_total = 0;
  for (auto& p : s->progs) memo_total += (size_t)p->prog.hdr.n_regex * memo_words;
  const bool memo_on = memo_total && (!getenv("GG_RX_MEMO") || atoi(getenv("GG_RX_MEMO")) != 0);
  s->rx_memo_words = memo_on ? memo_total : 0;
  if (memo_on) {
    s->dv->d_rx_memo.alloc(memo_total);
    HIPCHK(hipMemsetAsync(s->dv->d_rx_memo.p, 0, memo_total * 4, st));
  }
  size_t memo_off = 0;
  for (auto& p : s->progs) {
    p->upload(st, s->docs, ids);
    p->dp.rx_memo = memo_on && p->prog.hdr.n_regex ? s->dv->d_rx_memo.p + memo_off : nullptr;
    p->dp.memo_words = memo_words;
    if (memo_on) memo_off += (size_t)p->prog.hdr.n_regex * memo_words;
    dps.push_back(p->dp);
    s->max_top = std::max<uint32_t>(s->max_top, p->dp.n_top);
  }
  s->dv->d_progs.upload(dps.data(), dps.size(), st);
  // staging window: the largest program (DFA tables included), capped at kMaxLdsProgWords
  s->lds_prog_words = 4;
  for (auto& p : s->progs) {
    uint32_t w = (uint32_t)p->prog.blob.size();
    if (w > gg_session::kMaxLdsProgWords) w = p->prog.hdr.off_dfa;
    if (w <= gg_session::kMaxLdsProgWords) s->lds_prog_words = std::max(s->lds_prog_words, (w + 3u) & ~3u);
  }
  // A session whose programs need the NFA simulation (a regex past the DFA limits) evaluates in the wave kernel:
  // the lane kernel's NFA variant gave wrong verdicts for a program of three or more NFA-simulated regexes in some
  // builds of round 6 (tests/test_gpu_parity.py test_nfa_regex_pack_vs_oracle) while the wave kernel's matched the
  // oracle in every build; the cause is not found.  GG_NFA_LANES=1 keeps the lane kernel (A/B).
  {
    bool nfa = false;
    for (auto& p : s->progs)
      for (auto& r : p->prog.regex) nfa |= r.nfa;
    if (nfa && s->mode == 0 && !(getenv("GG_NFA_LANES") && atoi(getenv("GG_NFA_LANES")))) s->mode = 1;
  }
  size_t ntiles = s->docs.ndocs() * s->progs.size();
  const bool large_docs = s->docs.ndocs() && arena_nodes(s) / s->docs.ndocs() > 4096;
  // Documents per lane batch: 64 (a wave's lanes, one tile each), or -- for a launch of few large documents
  // (cfg4: 8192 Terraform plans of ~60 K nodes; at 64 per wave they fill 256 waves, one per CU, and one lane
  // walks a whole plan's 2000-entry lists) -- L = 64 / G documents with G lanes each: the G lanes of a
  // document run its tile in step and split every chunk of its filtered list fan-outs (coop_chunk), and the
  // launch fills the machine's 16 waves per CU.  GG_LANE_GROUP sets G (1 turns the groups off), GG_LANE_DOCS
  // sets L with one lane per document (the round-5 sparse batches; A/B).
  s->lane_docs = 64;
  s->lane_group = 1;
  {
    const size_t fill = (size_t)dev_ncu(s->device) * 16;   // waves the lane kernel keeps resident
    if (large_docs && (s->docs.ndocs() + 63) / 64 * s->progs.size() < fill) {
      size_t L = 64;
      while (L > 1 && (s->docs.ndocs() + L - 1) / L * s->progs.size() < fill) L >>= 1;
      s->lane_docs = (uint32_t)L;
      s->lane_group = (uint32_t)(64 / L);
    }
    if (const char* e = getenv("GG_LANE_GROUP")) {
      uint32_t g = 1;
      while (g < 64 && g * 2 <= (uint32_t)std::max(1, atoi(e))) g *= 2;
      s->lane_group = g;
      s->lane_docs = 64 / g;
    }
    if (const char* e = getenv("GG_LANE_DOCS")) { s->lane_docs = (uint32_t)std::min(64, std::max(1, atoi(e))); s->lane_group = 1; }
  }
  size_t nbatches = (s->docs.ndocs() + s->lane_docs - 1) / s->lane_docs * s->progs.size();
  // Lane groups (few large documents, no shape order): documents ordered by arena size inside each XCD's share
  // of the L-document chunks (the kernel's c0 / c1 split), largest first.  A batch's L documents are then of
  // similar size, so its lane groups' loops run similar trip counts, and every XCD queue hands out its largest
  // plans first (longest-first scheduling: the launch does not end on a 2000-resource plan started last).
  // GG_SIZE_ORDER=0 keeps load order.  Results do not depend on the order (tiles stay indexed by document).
  if (s->lane_group > 1 && !s->has_order && s->mode != 1 && s->docs.ndocs() > s->lane_docs &&
      !(getenv("GG_SIZE_ORDER") && atoi(getenv("GG_SIZE_ORDER")) == 0)) {
    const DocBatch& D = s->docs;
    const size_t nd = D.ndocs(), L = s->lane_docs, nchunks = (nd + L - 1) / L, total = arena_nodes(s);
    std::vector<uint32_t> ord(nd);
    std::vector<uint64_t> size(nd);
    for (size_t d = 0; d < nd; d++) {
      ord[d] = (uint32_t)d;
      size[d] = (d + 1 < nd ? (uint64_t)D.base[d + 1] : (uint64_t)total) - (uint64_t)D.base[d];
    }
    for (size_t x = 0; x < 8; x++) {
      const size_t lo = std::min(nd, nchunks * x / 8 * L), hi = std::min(nd, nchunks * (x + 1) / 8 * L);
      std::stable_sort(ord.begin() + lo, ord.begin() + hi, [&](uint32_t a, uint32_t b) { return size[a] > size[b]; });
    }
    s->dv->d_order.upload(ord.data(), nd, st);
    HIPCHK(hipStreamSynchronize(st));   // ord dies at the end of this scope
    s->has_order = true;
  }
  // wave mode: all tiles (mode 1) or only the lane kernel's overflow tiles (mode 0)
  size_t wave_slots = s->mode == 1 ? (size_t)dev_ncu(s->device) * 8 : (size_t)dev_ncu(s->device) * 2;
  uint32_t slots = (uint32_t)std::min<size_t>(std::max<size_t>(ntiles, 1), wave_slots);
  s->nslots = slots;
  s->dv->d_heaps.alloc((size_t)slots * s->heap_bytes);
  // lane-mode grid: waves per CU (default 8 = the kernel's occupancy at 2 waves/SIMD)
  size_t lane_waves_per_cu = 16;   // 4 waves per SIMD (build.py GG_LANE_WAVES_PER_EU); LDS holds 16 at cfg-2 program sizes
  if (const char* e = getenv("GG_LANE_WAVES_PER_CU")) lane_waves_per_cu = std::max(1, atoi(e));
  s->lane_slots = s->mode == 1 ? 0 : (uint32_t)std::min<size_t>(std::max<size_t>(nbatches, 1), (size_t)dev_ncu(s->device) * lane_waves_per_cu);
  // every one of the 8 per-XCD queues needs waves (block b serves queue b % 8)
  if (s->lane_slots) s->lane_slots = (std::max<uint32_t>(s->lane_slots, 8u) + 7u) & ~7u;
  // Few lane batches (a corpus of few, large documents: cfg4's plans) leave most of the lane heaps' memory
  // budget unused while their tiles outgrow 64 KB (hundreds of records, long QR lists) and fall back to
  // the wave kernel one tile per wave: such launches get 256 KB lane heaps with 96 KB of record staging
  // while the heaps stay within kLaneHeapBudget
  // Lane groups: every lane of a document's group holds its own copy of the tile's state, so the 256 KB heaps
  // are budgeted at 48 GB of the MI355X's 288 GB -- the resident waves are capped to fit (3072 = 12 per CU)
  static constexpr size_t kLaneHeapBudget = (size_t)24 << 30, kGroupHeapBudget = (size_t)48 << 30;
  s->lane_heap_bytes = s->lane_heap_set ? s->lane_heap_set : 64u * 1024u;
  s->lane_recs_bytes = 24576;
  if (!s->lane_heap_set && large_docs && s->lane_slots) {
    if (s->lane_group > 1) {
      s->lane_heap_bytes = 256u << 10;
      s->lane_recs_bytes = 2048u * (uint32_t)sizeof(Rec);
      size_t budget = kGroupHeapBudget;
      if (const char* e = getenv("GG_GROUP_HEAP_GB")) budget = (size_t)std::max(1, atoi(e)) << 30;
      const size_t cap = budget / ((size_t)64 * s->lane_heap_bytes) & ~(size_t)7;
      if (s->lane_slots > cap) s->lane_slots = (uint32_t)std::max<size_t>(cap, 8);
    } else if ((size_t)s->lane_slots * 64 * (256u << 10) <= kLaneHeapBudget) {
      s->lane_heap_bytes = 256u << 10;
      s->lane_recs_bytes = 2048u * (uint32_t)sizeof(Rec);
    }
  }
  s->dv->d_lane_heaps.alloc((size_t)s->lane_slots * 64 * s->lane_heap_bytes);
  s->dv->d_retry.alloc(std::max<size_t>(ntiles, 1));
  s->dv->d_retry2.alloc(std::max<size_t>(ntiles, 1));
  s->dv->d_tiles.alloc(std::max<size_t>(ntiles, 1));
  s->dv->d_rule_status.alloc(std::max<size_t>(ntiles * s->max_top, 1));
  // direct record chunks (lane mode): rec_chunk slots per document per batch (lane_docs documents), reserved
  // by every lane batch of a launch.  GG_REC_CHUNK overrides (0: every record staged in the lane heap, the round-3 path); halved
  // until the reservations fit kMaxChunkBytes (<= 8 slots: off)
  s->rec_chunk = 0;
  size_t reserve = 0;
  if (s->mode != 1) {
    const size_t lane_batches = nbatches;
    // 64 slots: cfg-2 42.3 -> 41.4 ms against 32 on one box (16: 42.8, 48: 41.6, 96: 41.5, 128: 41.4,
    // profiles/r04_sweep_rec_chunk.log); the 24 GB reservation cap below halves it for larger launches
    size_t ch = 64;
    // few batches (large documents, hundreds of records per tile): chunks as large as 2 GB of
    // reservations allows, up to 1024 records per lane
    static constexpr size_t kSmallChunkBytes = (size_t)2 << 30;
    const size_t per = s->lane_docs;   // record columns per batch: its documents (eval_kernel.hip rbase)
    if (large_docs && lane_batches && lane_batches * per * 32 * sizeof(Rec) < kSmallChunkBytes)
      ch = std::min<size_t>(1024, kSmallChunkBytes / (lane_batches * per * sizeof(Rec)));
    if (getenv("GG_REC_CHUNK")) ch = (size_t)std::max(0, atoi(getenv("GG_REC_CHUNK")));
    static constexpr size_t kMaxChunkBytes = (size_t)24 << 30;
    while (ch >= 8 && lane_batches * per * ch * sizeof(Rec) > kMaxChunkBytes) ch /= 2;
    if (ch >= 8 && lane_batches * per * ch < 0xC0000000ull) { s->rec_chunk = (uint32_t)ch; reserve = lane_batches * per * ch; }
  }
  s->rec_cap = reserve + std::min<size_t>(std::max<size_t>(ntiles * 48, 4096), (size_t)96 * 1024 * 1024);
  s->rec_cap = std::min<size_t>(s->rec_cap, (size_t)0xFFFFFFF0u);
  s->dv->d_recs.alloc(s->rec_cap);
  s->dv->d_counters.alloc(32);   // [0..6] cursors / counts, [16..23] per-XCD lane-mode queues
  s->dv->d_stats.alloc(32);
  HIPCHK(hipMemsetAsync(s->dv->d_stats.p, 0, 32 * sizeof(unsigned long long), st));
  s->ncounts = s->progs.size() * (s->max_top + 1) * 4;
  if (s->ncounts * sizeof(uint32_t) > 60 * 1024)
    throw std::runtime_error("too many (rules file x rule) tallies for one LDS block; split the rules files across sessions");
  s->dv->d_counts.alloc(std::max<size_t>(s->ncounts, 1));
  HIPCHK(hipStreamSynchronize(st));
  s->uploaded = true;
  mark("programs + buffers");
}

hipStream_t session_stream(gg_session* s) { return s->stream ? s->stream : s->dv->stream; }

// enqueues one evaluation of every tile (and the per-rule tally) on the session stream; no host sync
void session_launch(gg_session* s) {
  bind_device(s);
  hipStream_t st = session_stream(s);
  uint32_t ntiles = (uint32_t)(s->docs.ndocs() * s->progs.size());
  HIPCHK(hipMemsetAsync(s->dv->d_counters.p, 0, 32 * sizeof(uint32_t), st));
  unsigned long long* counts = s->ext_counts ? s->ext_counts : s->dv->d_counts.p;
  HIPCHK(hipMemsetAsync(counts, 0, s->ncounts * sizeof(unsigned long long), st));
  // regex memo policy: by default it is zeroed once per upload and stays warm across launches (a pure
  // function of the interned string); per-launch zeroing makes every launch pay its first DFA runs
  if (s->rx_memo_per_launch && s->rx_memo_words)
    HIPCHK(hipMemsetAsync(s->dv->d_rx_memo.p, 0, s->rx_memo_words * 4, st));
  LaunchArgs A{};
  A.docs.nodes = s->dv->d_nodes.p; A.docs.klen = s->dv->d_klen.p; A.docs.bytes = s->dv->d_bytes.p; A.docs.roots = s->dv->d_roots.p; A.docs.base = s->dv->d_base.p; A.docs.ndocs = (uint32_t)s->docs.ndocs();
  A.docs.res_map = s->dv->d_res_map.p; A.docs.tix_off = s->dv->d_tix_off.p; A.docs.tix = s->dv->d_tix.p; A.docs.type_key = s->type_key;
  A.order = s->has_order ? s->dv->d_order.p : nullptr;
  A.progs = s->dv->d_progs.p; A.nfiles = (uint32_t)s->progs.size();
  A.ntiles = ntiles; A.tile_base = 0;
  A.heaps = s->dv->d_heaps.p; A.heap_bytes = s->heap_bytes; A.nslots = s->nslots;
  A.tiles = s->dv->d_tiles.p; A.rule_status = s->dv->d_rule_status.p; A.max_top = s->max_top;
  A.recs = s->dv->d_recs.p; A.rec_cap = (uint32_t)s->rec_cap;
  A.rec_chunk = s->mode == 1 ? 0u : s->rec_chunk;
  A.rec_cursor = s->dv->d_counters.p; A.tile_cursor = s->dv->d_counters.p + 1;   // [1] lane batches, [2] wave tiles
  A.retry_count = s->dv->d_counters.p + 3;
  A.xcd_cursor = s->dv->d_counters.p + 16;
  A.lane_heaps = s->dv->d_lane_heaps.p; A.lane_heap_bytes = s->lane_heap_bytes; A.lane_recs_bytes = s->lane_recs_bytes;
  A.lane_docs = s->lane_docs;
  // bit 16: no split walks (GG_SPLIT_WALK=0, A/B)
  A.lane_group = s->lane_group | ((getenv("GG_SPLIT_WALK") && atoi(getenv("GG_SPLIT_WALK")) == 0) ? (1u << 16) : 0u);
  A.stack_guard = dev_stack_guard(s->device);
  A.retry_list = s->mode == 1 ? nullptr : s->dv->d_retry.p;
  A.wave_frames_bytes = gg_session::kWaveFrames; A.wave_recs_bytes = gg_session::kWaveRecs;
  A.retry2_list = s->dv->d_retry2.p; A.retry2_count = s->dv->d_counters.p + 4;
  A.stats = s->dv->d_stats.p;
  A.lds_prog_words = s->lds_prog_words;
  if (!ntiles) return;
  if (s->nq == s->dv->evq.size()) {
    std::pair<hipEvent_t, hipEvent_t> pr;
    HIPCHK(hipEventCreate(&pr.first));
    HIPCHK(hipEventCreate(&pr.second));
    s->dv->evq.push_back(pr);
  }
  s->ev0 = s->dv->evq[s->nq].first; s->ev1 = s->dv->evq[s->nq].second; s->nq++;
  HIPCHK(hipEventRecord(s->ev0, st));
  // a regex past the DFA limits (PRegex flags bit 1) selects the kernels with the NFA simulation
  bool nfa = false;
  for (auto& p : s->progs)
    for (auto& r : p->prog.regex) nfa |= r.nfa;
  if (s->mode != 1) {
    hipLaunchKernelGGL(nfa ? guard_eval_lanes_kernel_nfa : guard_eval_lanes_kernel, dim3(s->lane_slots), dim3(64),
                       A.lds_prog_words * 4, st, A);
    HIPCHK(hipGetLastError());
  }
  auto wave_kernel = s->verbose ? (nfa ? guard_eval_verbose_kernel_nfa : guard_eval_verbose_kernel)
                                : (nfa ? guard_eval_kernel_nfa : guard_eval_kernel);
  hipLaunchKernelGGL(wave_kernel, dim3(s->nslots), dim3(64), A.lds_prog_words * 4, st, A);
  HIPCHK(hipGetLastError());
  if (s->dv->d_big_heaps.p) {
    // large-heap pass over the wave pass's overflow list (counters[4]; its cursor is counters[6]);
    // normally empty, so its waves exit at once.  Its 256 MB of heaps exist only once a tile of
    // this session has needed them (session_run)
    LaunchArgs B = A;
    B.retry_list = s->dv->d_retry2.p; B.retry_count = s->dv->d_counters.p + 4; B.tile_cursor = s->dv->d_counters.p + 5;
    B.heaps = s->dv->d_big_heaps.p; B.heap_bytes = gg_session::kBigHeap; B.nslots = gg_session::kBigSlots;
    B.wave_frames_bytes = gg_session::kBigFrames; B.wave_recs_bytes = gg_session::kBigRecs;
    B.retry2_list = nullptr; B.retry2_count = nullptr;
    hipLaunchKernelGGL(wave_kernel, dim3(gg_session::kBigSlots), dim3(64), B.lds_prog_words * 4, st, B);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(s->ev1, st));
  uint32_t cblocks = std::min<uint32_t>((ntiles + 255) / 256, dev_ncu(s->device) * 4);
  hipLaunchKernelGGL(rule_count_kernel, dim3(cblocks), dim3(256), s->ncounts * sizeof(uint32_t), st, s->dv->d_tiles.p,
                     s->dv->d_rule_status.p, s->dv->d_progs.p, A.nfiles, ntiles, s->max_top, counts);
  HIPCHK(hipGetLastError());
  s->launched = true;
}

// waits for the last launch; returns the evaluation kernel's milliseconds (HIP events on its stream)
double session_wait(gg_session* s) {
  if (!s->launched) return 0;
  bind_device(s);
  HIPCHK(hipEventSynchronize(s->ev1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
  s->last_kernel_ms = ms;
  return ms;
}

// kernel ms of every launch since the last drain (synchronises on the last one)
size_t session_drain(gg_session* s, double* out, size_t cap) {
  size_t n = s->nq;
  if (n) bind_device(s);
  if (n) HIPCHK(hipEventSynchronize(s->dv->evq[n - 1].second));
  for (size_t i = 0; i < n; i++) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, s->dv->evq[i].first, s->dv->evq[i].second));
    if (i < cap && out) out[i] = ms;
  }
  s->nq = 0;
  return n;
}

// total records the last launch wanted to publish (may exceed rec_cap)
uint32_t session_records_wanted(gg_session* s) {
  uint32_t nrec = 0;
  HIPCHK(hipStreamSynchronize(session_stream(s)));
  HIPCHK(hipMemcpy(&nrec, s->dv->d_counters.p, 4, hipMemcpyDeviceToHost));
  return nrec;
}

// Compacts every tile's records -- in place in their lane's direct chunk (TileOut.pad1 = stride > 1) or contiguous
// -- into one dense array in tile order and copies it to the host (s->recs), rewriting the host tiles'
// rec_off to the dense offsets.  Only host writers read the dense array: the device reporter reads the
// records where the evaluation left them (report_gpu.hip RecSeq), so a device-rendered report needs no
// compaction at all.
void compact_records_to_host(gg_session* s) {
  const uint32_t ntiles = (uint32_t)s->tiles.size();
  uint32_t total = 0;
  if (ntiles) {
    hipStream_t st = session_stream(s);
    const uint32_t nb = (ntiles + 1023u) / 1024u;
    s->dv->d_bsum.alloc((size_t)nb + 1);
    s->dv->d_dense_off.alloc(ntiles);
    hipLaunchKernelGGL(rec_block_sums_kernel, dim3(nb), dim3(256), 0, st, s->dv->d_tiles.p, ntiles, s->dv->d_bsum.p);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(rec_scan_sums_kernel, dim3(1), dim3(1024), 0, st, s->dv->d_bsum.p, nb, s->dv->d_bsum.p + nb);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&total, s->dv->d_bsum.p + nb, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    s->dv->d_recs_dense.alloc(std::max<size_t>(total, 1));
    hipLaunchKernelGGL(rec_compact_kernel, dim3(nb), dim3(256), 0, st, s->dv->d_tiles.p, ntiles, s->dv->d_bsum.p,
                       s->dv->d_recs.p, s->dv->d_recs_dense.p, s->dv->d_dense_off.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    std::vector<uint32_t> doff(ntiles);
    HIPCHK(hipMemcpy(doff.data(), s->dv->d_dense_off.p, ntiles * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (uint32_t t = 0; t < ntiles; t++) { s->tiles[t].rec_off = doff[t]; s->tiles[t].pad1 = 0; }
  }
  s->recs.resize(total);
  if (total) HIPCHK(hipMemcpy(s->recs.data(), s->dv->d_recs_dense.p, (size_t)total * sizeof(Rec), hipMemcpyDeviceToHost));
  s->recs_total = total;
  s->recs_pending = false;
}

// Statuses, rule statuses and tallies to the host.  The records stay in HBM as the evaluation wrote them
// when the session defers them (defer_recs: the device reporter reads them there; ensure_host_arena
// compacts and copies them once a host writer needs them), else they are compacted and copied now.
void session_fetch(gg_session* s) {
  bind_device(s);
  // the tally kernel runs after ev1 on a non-blocking stream: wait for the whole launch
  hipStream_t st = session_stream(s);
  HIPCHK(hipStreamSynchronize(st));
  uint32_t ntiles = (uint32_t)(s->docs.ndocs() * s->progs.size());
  s->tiles.resize(ntiles);
  s->rule_status.resize((size_t)ntiles * s->max_top);
  if (ntiles) {
    HIPCHK(hipMemcpy(s->tiles.data(), s->dv->d_tiles.p, ntiles * sizeof(TileOut), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(s->rule_status.data(), s->dv->d_rule_status.p, s->rule_status.size(), hipMemcpyDeviceToHost));
  }
  uint64_t total = 0;
  for (const TileOut& t : s->tiles) total += (uint64_t)t.rec_n + t.pad0;
  s->recs_total = (uint32_t)total;
  s->recs.clear();
  s->recs_pending = total != 0;
  if (!s->defer_recs) compact_records_to_host(s);
  s->counts.resize(s->ncounts);
  HIPCHK(hipMemcpy(s->counts.data(), s->ext_counts ? s->ext_counts : s->dv->d_counts.p, s->ncounts * sizeof(unsigned long long),
                   hipMemcpyDeviceToHost));
  s->evaluated = true;
  s->fetched_on_device = ntiles > 0;
}

// one complete evaluation; re-runs when the first pass overflowed the record arena (grown) or left
// tiles for the large-heap pass before its heaps existed (allocated)
double session_run(gg_session* s, bool fetch) {
  double ms = 0;
  // re-runs while a pass needed what did not exist yet: a larger record arena (the cursor counts every
  // reservation and allocation, also of tiles that could not write) or the large-heap pass's heaps (its
  // tiles' records are counted only once it runs, so allocating it can call for a larger arena next)
  for (int pass = 0; pass < 4; pass++) {
    session_launch(s);
    ms = session_wait(s);
    uint32_t cnt[5] = {0, 0, 0, 0, 0};
    HIPCHK(hipStreamSynchronize(session_stream(s)));
    HIPCHK(hipMemcpy(cnt, s->dv->d_counters.p, sizeof(cnt), hipMemcpyDeviceToHost));
    bool again = false;
    if (cnt[0] > s->rec_cap) {
      s->rec_cap = std::min<size_t>((size_t)cnt[0] + cnt[0] / 8 + 1024, (size_t)0xFFFFFFF0u);
      s->dv->d_recs.alloc(s->rec_cap);
      again = true;
    }
    if (cnt[4] && !s->dv->d_big_heaps.p) {
      s->dv->d_big_heaps.alloc((size_t)gg_session::kBigSlots * gg_session::kBigHeap);
      again = true;
    }
    if (!again) break;
  }
  if (fetch) session_fetch(s);
  session_drain(s, nullptr, 0);
  return ms;
}

// host threads for report rendering and host loading: GG_REPORT_THREADS, else the process's CPU share --
// its affinity set, capped by OMP_NUM_THREADS when the host declares an allotment (the MI355X pool: 16
// host CPUs per GPU)
unsigned report_threads() {
  if (const char* e = getenv("GG_REPORT_THREADS")) return (unsigned)std::max(1, atoi(e));
  unsigned n = std::thread::hardware_concurrency();
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0 && CPU_COUNT(&cs) > 0) n = (unsigned)CPU_COUNT(&cs);
  if (const char* o = getenv("OMP_NUM_THREADS")) { const int k = atoi(o); if (k > 0) n = std::min(n, (unsigned)k); }
  return std::max(1u, n ? n : 1u);
}

// ------------------------------------------------------------------ device reporter ---
// The structured JSON report rendered on the session's device (report_gpu.hip): the reporter's tables
// (context strings, messages, rule names, remaining-query texts, literal arena, sorted rule names) built
// once per upload, the marks uploaded at first use, then per block of documents a size pass, offsets, a
// write pass and the text copied out in document order, with the documents the device writer leaves to
// the host (floats, Debug-formatted reasons, ...) written by the host writer at their positions.
bool device_report_on(const gg_session* s) {
  if (s->device_report >= 0) return s->device_report != 0;
  const char* e = getenv("GG_DEVICE_REPORT");
  return !e || atoi(e) != 0;
}

// where report text goes: reserve(n) gives room for the next n bytes, commit(n) takes them
struct ReportSink {
  virtual ~ReportSink() = default;
  virtual char* reserve(size_t n) = 0;
  virtual void commit(size_t n) = 0;
  virtual size_t max_piece() const { return SIZE_MAX; }
  // reserve() hands out page-locked host memory: the device report's copy-out may switch from the copy
  // engine to the shader copy (d2h_push reads the host pointer's device mapping) -- never for pageable memory
  virtual bool pinned() const { return false; }
  void write(const char* p, size_t n) {
    while (n) {
      const size_t k = std::min(n, max_piece());
      memcpy(reserve(k), p, k);
      commit(k);
      p += k; n -= k;
    }
  }
};
// the report as one malloc'd NUL-terminated buffer (grown by realloc: glibc moves large blocks by mremap)
struct BufferSink : ReportSink {
  char* p = nullptr;
  size_t n = 0, cap = 0;
  ~BufferSink() override { free(p); }
  char* reserve(size_t k) override {
    if (n + k + 1 > cap) {
      size_t nc = std::max<size_t>(cap * 2, n + k + 1);
      nc = std::max<size_t>(nc, 1 << 16);
      char* q = (char*)realloc(p, nc);
      if (!q) throw std::bad_alloc();
      p = q; cap = nc;
    }
    return p + n;
  }
  void commit(size_t k) override { n += k; }
  char* take() { reserve(0); p[n] = 0; char* r = p; p = nullptr; n = cap = 0; return r; }
};
// counts the bytes and drops them (end-to-end measurement: the text reaches host memory, then is discarded)
struct CountingSink : ReportSink {
  char* stage;
  size_t stage_bytes;
  uint64_t n = 0;
  CountingSink(char* st, size_t sb) : stage(st), stage_bytes(sb) {}
  char* reserve(size_t) override { return stage; }
  void commit(size_t k) override { n += k; }
  size_t max_piece() const override { return stage_bytes; }
  bool pinned() const override { return true; }   // DeviceBufs::pinned staging
};

struct DevReportStats { uint64_t device_docs = 0, host_docs = 0, bytes = 0; double size_ms = 0, write_ms = 0, d2h_ms = 0, host_ms = 0; };

void render_tables(gg_session* s) {
  if (s->rtab_ready) return;
  std::vector<uint8_t> blob;
  auto put = [&](const void* p, size_t n) -> size_t {
    size_t o = (blob.size() + 15) & ~(size_t)15;
    blob.resize(o + std::max<size_t>(n, 1), 0);
    if (n) memcpy(blob.data() + o, p, n);
    return o;
  };
  struct Offs { size_t text, ctx, msgs, rnames, rem_first, rem, pkey, pidx, clauses, lit, lit_bytes, lit_line, lit_col; uint32_t nc, nl, nr, nq, nx, nm; };
  std::vector<Offs> offs;
  for (auto& gp : s->progs) {
    const Program& P = gp->prog;
    std::string text;
    auto add = [&](const std::string& x) { RStr r{(uint32_t)text.size(), (uint32_t)x.size()}; text += x; return r; };
    std::vector<RStr> ctx, msgs, rn, rem, pkey;
    std::vector<uint32_t> rem_first;
    std::vector<int32_t> pidx;
    for (auto& x : P.ctx) ctx.push_back(add(x));
    for (auto& x : P.msgs) msgs.push_back(add(x));
    for (auto& x : P.rule_names) rn.push_back(add(x));
    for (size_t q = 0; q < P.queries.size(); q++) {
      rem_first.push_back((uint32_t)rem.size());
      const auto& parts = P.queries[q];
      for (size_t st = 0; st <= parts.size(); st++) {
        rem.push_back(add(P.query_remaining((uint32_t)q, (uint32_t)st)));
        pkey.push_back(st < parts.size() ? add(parts[st].key) : RStr{0, 0});
        pidx.push_back(st < parts.size() ? parts[st].index : 0);
      }
    }
    rem_first.push_back((uint32_t)rem.size());
    Offs o;
    o.text = put(text.data(), text.size());
    o.ctx = put(ctx.data(), ctx.size() * sizeof(RStr));
    o.msgs = put(msgs.data(), msgs.size() * sizeof(RStr));
    o.rnames = put(rn.data(), rn.size() * sizeof(RStr));
    o.rem_first = put(rem_first.data(), rem_first.size() * 4);
    o.rem = put(rem.data(), rem.size() * sizeof(RStr));
    o.pkey = put(pkey.data(), pkey.size() * sizeof(RStr));
    o.pidx = put(pidx.data(), pidx.size() * 4);
    o.clauses = put(P.clauses.data(), P.clauses.size() * sizeof(PClause));
    o.lit = put(P.lit.nodes.data(), P.lit.nodes.size() * sizeof(DNode));
    o.lit_bytes = put(P.lit.bytes.data(), P.lit.bytes.size());
    o.lit_line = put(P.lit.line.data(), P.lit.line.size() * 4);
    o.lit_col = put(P.lit.col.data(), P.lit.col.size() * 4);
    o.nc = (uint32_t)P.clauses.size(); o.nl = (uint32_t)P.lit.nodes.size(); o.nr = (uint32_t)P.rule_names.size();
    o.nq = (uint32_t)P.queries.size(); o.nx = (uint32_t)P.ctx.size(); o.nm = (uint32_t)P.msgs.size();
    offs.push_back(o);
  }
  // not_applicable / compliant: the distinct top-level rule names, sorted as std::set<std::string> sorts them
  std::map<std::string, std::vector<uint32_t>> names;
  for (size_t f = 0; f < s->progs.size(); f++) {
    const Program& P = s->progs[f]->prog;
    for (uint32_t k = 0; k < P.n_rules; k++) names[P.rule_names[P.rule_names.size() - P.n_rules + k]].push_back((uint32_t)(f << 16 | k));
  }
  std::string stext;
  std::vector<RStr> sname;
  std::vector<uint32_t> sfirst, sn, sfk;
  for (auto& kv : names) {
    sname.push_back(RStr{(uint32_t)stext.size(), (uint32_t)kv.first.size()});
    stext += kv.first;
    sfirst.push_back((uint32_t)sfk.size());
    sn.push_back((uint32_t)kv.second.size());
    for (uint32_t x : kv.second) sfk.push_back(x);
  }
  const size_t o_stext = put(stext.data(), stext.size()), o_sname = put(sname.data(), sname.size() * sizeof(RStr)),
               o_sfirst = put(sfirst.data(), sfirst.size() * 4), o_sn = put(sn.data(), sn.size() * 4), o_sfk = put(sfk.data(), sfk.size() * 4);
  hipStream_t st = s->dv->stream;
  s->dv->d_rtab.upload(blob.data(), blob.size(), st);
  const uint8_t* b = s->dv->d_rtab.p;
  std::vector<RProg> rp;
  for (auto& o : offs) {
    RProg r{};
    r.text = (const char*)(b + o.text); r.ctx = (const RStr*)(b + o.ctx); r.msgs = (const RStr*)(b + o.msgs);
    r.rule_names = (const RStr*)(b + o.rnames); r.rem_first = (const uint32_t*)(b + o.rem_first); r.rem = (const RStr*)(b + o.rem);
    r.pkey = (const RStr*)(b + o.pkey); r.pidx = (const int32_t*)(b + o.pidx); r.clauses = (const PClause*)(b + o.clauses);
    r.lit = (const DNode*)(b + o.lit); r.lit_bytes = (const char*)(b + o.lit_bytes);
    r.lit_line = (const uint32_t*)(b + o.lit_line); r.lit_col = (const uint32_t*)(b + o.lit_col);
    r.n_clauses = o.nc; r.n_lit = o.nl; r.n_rule_names = o.nr; r.n_queries = o.nq; r.n_ctx = o.nx; r.n_msgs = o.nm;
    rp.push_back(r);
  }
  s->dv->d_rprogs.upload(rp.data(), std::max<size_t>(rp.size(), 1), st);
  s->r_sname_text = (const char*)(b + o_stext); s->r_sname = (const RStr*)(b + o_sname);
  s->r_sname_first = (const uint32_t*)(b + o_sfirst); s->r_sname_n = (const uint32_t*)(b + o_sn);
  s->r_sname_fk = (const uint32_t*)(b + o_sfk); s->r_nsname = (uint32_t)sname.size();
  if (!s->marks_on_device) {
    std::lock_guard<std::mutex> lk(s->arena_mu);
    const size_t n = arena_nodes(s);
    if (s->resident.nodes) {   // the loader's marks are in HBM already
      s->dv->d_line.alloc(std::max<size_t>(n, 1));
      s->dv->d_col.alloc(std::max<size_t>(n, 1));
      HIPCHK(hipMemcpyAsync(s->dv->d_line.p, s->resident.line, n * 4, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpyAsync(s->dv->d_col.p, s->resident.col, n * 4, hipMemcpyDeviceToDevice, st));
    } else {
      s->dv->d_line.upload(s->docs.line.data(), std::max<size_t>(n, 1), st);
      s->dv->d_col.upload(s->docs.col.data(), std::max<size_t>(n, 1), st);
    }
    s->marks_on_device = true;
  }
  if (!s->dv->pinned) {
    s->dv->pinned = (char*)pinned_alloc(DeviceBufs::kPinnedBytes, s->device);
    if (!s->dv->pinned) throw std::runtime_error("pinned host staging: allocation failed");
  }
  HIPCHK(hipStreamSynchronize(st));
  s->rtab_ready = true;
}

// JSON FileReports of documents [first, first + count) into `sink` (each preceded by ",\n" unless it is
// report_first, and by two spaces); the session was evaluated and fetched on its device.  false + err when
// a document's report aborts (the host writer's Fatal; the first such document in order).
//
// Per block of documents (two block sets in flight): the size pass, then the write pass at the offsets;
// a copy thread moves each block to the sink in document order -- device runs by D2H, host-writer
// documents between them -- while the device renders the next block.
// the streamed entries' shader copy-out (device_report_text push_default): workgroups of d2h_push
static constexpr int kStreamPushBlocks = 32;
bool device_report_text(gg_session* s, size_t first, size_t count, size_t report_first, ReportSink& sink, ReportError& err,
                        DevReportStats* stats, int32_t fmt, int push_default = 0) {
  bind_device(s);
  render_tables(s);
  hipStream_t st = s->dv->stream;
  if (!s->dv->copy_stream) HIPCHK(hipStreamCreateWithFlags(&s->dv->copy_stream, hipStreamNonBlocking));
  hipStream_t cst = s->dv->copy_stream;
  // GG_D2H_PUSH=<workgroups>: the copy-out by a shader kernel (d2h_push) instead of the copy engine; the
  // streamed entries default to it (push_default): their copy engines were measured at 27 GB/s where the
  // shader copy holds 50-54 (profiles/r05zc_report_ab_push*.log).  0 = the copy engine.
  const int push_blocks = getenv("GG_D2H_PUSH") ? std::max(0, atoi(getenv("GG_D2H_PUSH"))) : push_default;
  if (push_blocks) {
    // GG_PUSH_CUS=<n>: the copy kernel confined to n CUs and the render kernels to the others
    const int cus = getenv("GG_PUSH_CUS") ? std::max(0, atoi(getenv("GG_PUSH_CUS"))) : 0;
    const int ncu = dev_ncu(s->device);
    if (cus > 0 && cus < ncu) {
      if (s->dv->push_cus != cus) {
        if (s->dv->push_stream) { HIPCHK(hipStreamSynchronize(s->dv->push_stream)); HIPCHK(hipStreamDestroy(s->dv->push_stream)); }
        if (s->dv->render_stream) { HIPCHK(hipStreamSynchronize(s->dv->render_stream)); HIPCHK(hipStreamDestroy(s->dv->render_stream)); }
        std::vector<uint32_t> pm((ncu + 31) / 32, 0u), rm((ncu + 31) / 32, 0u);
        // the copy CUs spread over the mask (every ncu / cus-th CU), the render kernels on the rest
        const int step = ncu / cus;
        for (int c = 0; c < ncu; c++) {
          if (c % step == 0 && c / step < cus) pm[c / 32] |= 1u << (c % 32);
          else rm[c / 32] |= 1u << (c % 32);
        }
        HIPCHK(hipExtStreamCreateWithCUMask(&s->dv->push_stream, (uint32_t)pm.size(), pm.data()));
        HIPCHK(hipExtStreamCreateWithCUMask(&s->dv->render_stream, (uint32_t)rm.size(), rm.data()));
        s->dv->push_cus = cus;
      }
      // the render stream starts after everything already queued on the session's buffer stream
      hipEvent_t ready;
      HIPCHK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
      HIPCHK(hipEventRecord(ready, st));
      HIPCHK(hipStreamWaitEvent(s->dv->render_stream, ready, 0));
      HIPCHK(hipEventDestroy(ready));
      st = s->dv->render_stream;
      cst = s->dv->push_stream;
    }
  }
  const int dev = s->device;
  std::vector<const Program*> progs;
  for (auto& p : s->progs) progs.push_back(&p->prog);
  const size_t nf = progs.size();
  const size_t kBlock = getenv("GG_DREPORT_BLOCK") ? (size_t)std::max(1, atoi(getenv("GG_DREPORT_BLOCK"))) : 65536;
  DevReportStats local;
  DevReportStats& S = stats ? *stats : local;
  // GG_DREPORT_TRACE=1: per-block wall-clock spans of the render and the copy-out on stderr (overlap check)
  const bool trace = getenv("GG_DREPORT_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };

  struct Block {
    size_t d0 = 0, nb = 0;
    std::vector<uint64_t> sizes, offs;
    hipEvent_t done = nullptr;   // compaction finished
  };
  Block blk[2];
  for (auto& b : blk) HIPCHK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
  // copy thread state
  std::mutex mu;
  std::condition_variable cv;
  bool busy[2] = {false, false};    // set i holds a block not yet copied out
  int queued = -1;                  // set index handed to the copy thread (-1: none)
  bool finished = false, failed = false;
  ReportError cerr;
  std::exception_ptr cex;
  std::thread copier([&]() {
    // GG_D2H_ADAPT=0: no switch from a slow copy engine to the shader copy (A/B)
    int use_push = push_blocks;
    const bool adapt = !push_blocks && sink.pinned() && !(getenv("GG_D2H_ADAPT") && atoi(getenv("GG_D2H_ADAPT")) == 0);
    uint64_t engine_bytes = 0;
    double engine_ms = 0;
    try {
      HIPCHK(hipSetDevice(dev));
      for (;;) {
        int set;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return queued >= 0 || finished; });
          if (queued < 0) return;
          set = queued;
          queued = -1;
        }
        cv.notify_all();   // the render loop waits for the hand-off slot to empty
        Block& b = blk[set];
        DeviceBufs::RenderSet& R = s->dv->rset[set];
        const double cw = since();
        HIPCHK(hipEventSynchronize(b.done));
        const double cb = since();
        size_t k = 0;
        while (k < b.nb && !failed) {
          if (b.sizes[k] & kHostDoc) {
            const auto h0 = std::chrono::steady_clock::now();
            ensure_host_arena(s);   // the host writer reads the arena's columns
            const size_t d = b.d0 + k;
            std::vector<TileResult> trs(nf);
            std::vector<const TileResult*> tp(nf);
            for (size_t f = 0; f < nf; f++) {
              trs[f] = tile_view(s->tiles.data(), s->rule_status.data(), s->max_top, s->recs.data(), d * nf + f);
              tp[f] = &trs[f];
            }
            if (fmt == OUT_SARIF) {
              std::string t;
              if (!sarif_doc_results(s->docs, (uint32_t)d, progs, tp, t, cerr)) { failed = true; break; }
              sink.write(t.data(), t.size());
              S.bytes += t.size();
            } else {
              TextBuf t;
              if (d != report_first) t.append(",\n", 2);
              t.append(2, ' ');
              if (!report_json_doc(s->docs, (uint32_t)d, progs, tp, t, cerr)) { failed = true; break; }
              sink.write(t.data(), t.size());
              S.bytes += t.size();
            }
            S.host_docs++;
            S.host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
            k++;
            continue;
          }
          size_t k1 = k;
          uint64_t bytes = 0;
          while (k1 < b.nb && !(b.sizes[k1] & kHostDoc)) { bytes += b.sizes[k1]; k1++; }
          const auto c0 = std::chrono::steady_clock::now();
          uint64_t at = b.offs[k];
          while (bytes) {
            const size_t piece = (size_t)std::min<uint64_t>(bytes, sink.max_piece());
            char* dst = sink.reserve(piece);
            void* ddst = nullptr;
            const auto p0 = std::chrono::steady_clock::now();
            bool engine = false;
            if (use_push && ((uintptr_t)dst & 15u) == 0 && hipHostGetDevicePointer(&ddst, dst, 0) == hipSuccess && ddst) {
              d2h_push(ddst, R.text.p + at, piece, cst, use_push);
              HIPCHK(hipGetLastError());
            } else {
              (void)hipGetLastError();
              HIPCHK(hipMemcpyAsync(dst, R.text.p + at, piece, hipMemcpyDeviceToHost, cst));
              engine = true;
            }
            HIPCHK(hipStreamSynchronize(cst));
            if (engine && adapt) {
              // the copy engine's rate over the report's first GB decides: a slow queue (27 GB/s against
              // 53, profiles/r05x_report_ab.log) hands the rest of the report to the shader copy
              engine_bytes += piece;
              engine_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p0).count();
              if (engine_bytes >= (1ull << 30) && engine_bytes / std::max(engine_ms, 1e-3) < 35e6) use_push = kStreamPushBlocks;
            }
            sink.commit(piece);
            at += piece; bytes -= piece; S.bytes += piece;
          }
          S.d2h_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
          S.device_docs += k1 - k;
          k = k1;
        }
        {
          std::lock_guard<std::mutex> lk(mu);
          busy[set] = false;
        }
        cv.notify_all();
        if (trace) fprintf(stderr, "[dreport] copy  set %d docs %zu: queued %.1f start %.1f end %.1f ms\n", set, b.d0, cw, cb, since());
        if (getenv("GG_PROGRESS"))
          fprintf(stderr, "[device report] %zu / %zu documents, %llu bytes\n", b.d0 + b.nb - first, count, (unsigned long long)S.bytes);
      }
    } catch (...) {
      cex = std::current_exception();
      std::lock_guard<std::mutex> lk(mu);
      failed = true;
      busy[0] = busy[1] = false;
      cv.notify_all();
    }
  });
  struct Join {
    std::thread& t; std::mutex& mu; std::condition_variable& cv; bool& finished; Block* blk;
    ~Join() {
      { std::lock_guard<std::mutex> lk(mu); finished = true; }
      cv.notify_all();
      if (t.joinable()) t.join();
      for (int i = 0; i < 2; i++) if (blk[i].done) hipEventDestroy(blk[i].done);
    }
  } join{copier, mu, cv, finished, blk};

  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0)); HIPCHK(hipEventCreate(&e1));
  struct EvFree { hipEvent_t a, b; ~EvFree() { hipEventDestroy(a); hipEventDestroy(b); } } evf{e0, e1};
  std::vector<char> names;
  std::vector<uint64_t> name_off;
  int set = 0;
  for (size_t d0 = first; d0 < first + count; d0 += kBlock, set ^= 1) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return (!busy[set] && queued < 0) || failed; });
      if (failed) break;
    }
    Block& b = blk[set];
    DeviceBufs::RenderSet& R = s->dv->rset[set];
    const size_t nb = std::min(kBlock, first + count - d0);
    const double rb = since();
    b.d0 = d0; b.nb = nb;
    names.clear(); name_off.assign(1, 0);
    for (size_t k = 0; k < nb; k++) {
      const std::string& nm = s->docs.names[d0 + k];
      names.insert(names.end(), nm.begin(), nm.end());
      name_off.push_back(names.size());
    }
    R.names.alloc_grow(std::max<size_t>(names.size(), 1));
    HIPCHK(hipMemcpyAsync(R.names.p, names.data(), names.size(), hipMemcpyHostToDevice, st));
    R.name_off.alloc_grow(name_off.size());
    HIPCHK(hipMemcpyAsync(R.name_off.p, name_off.data(), name_off.size() * 8, hipMemcpyHostToDevice, st));
    R.sizes.alloc_grow(nb);
    RenderArgs A{};
    A.nodes = s->dv->d_nodes.p; A.klen = s->dv->d_klen.p; A.pool = s->dv->d_bytes.p; A.parent = s->dv->d_parent.p;
    A.line = s->dv->d_line.p; A.col = s->dv->d_col.p; A.base = s->dv->d_base.p; A.n_nodes = arena_nodes(s);
    A.progs = s->dv->d_rprogs.p; A.nfiles = (uint32_t)nf; A.max_top = s->max_top;
    A.tiles = s->dv->d_tiles.p; A.rule_status = s->dv->d_rule_status.p; A.recs = s->dv->d_recs.p;
    A.sname_text = s->r_sname_text; A.sname = s->r_sname; A.sname_first = s->r_sname_first; A.sname_n = s->r_sname_n;
    A.sname_fk = s->r_sname_fk; A.n_sname = s->r_nsname;
    A.doc0 = (uint32_t)d0; A.ndocs = (uint32_t)nb; A.report_first = (uint32_t)std::min<size_t>(report_first, 0xFFFFFFFFu);
    A.names = R.names.p; A.name_off = R.name_off.p; A.sizes = R.sizes.p;
    const uint32_t blocks = (uint32_t)std::min<size_t>((nb + 255) / 256, (size_t)dev_ncu(s->device) * 8);
    HIPCHK(hipEventRecord(e0, st));
    auto kern = fmt == OUT_SARIF ? report_sarif_kernel : report_kernel;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, A, 0u);
    HIPCHK(hipGetLastError());
    b.sizes.resize(nb);
    HIPCHK(hipMemcpyAsync(b.sizes.data(), R.sizes.p, nb * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    b.offs.resize(nb);
    uint64_t dev_bytes = 0;
    for (size_t k = 0; k < nb; k++) {
      b.offs[k] = dev_bytes;
      if (!(b.sizes[k] & kHostDoc)) dev_bytes += b.sizes[k];
    }
    R.text.alloc_grow(std::max<uint64_t>(dev_bytes, 1));
    R.offs.alloc_grow(nb);
    HIPCHK(hipMemcpyAsync(R.offs.p, b.offs.data(), nb * 8, hipMemcpyHostToDevice, st));
    A.out = R.text.p; A.offsets = R.offs.p;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, A, 1u);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventRecord(b.done, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1)); S.write_ms += ms;
    if (trace) fprintf(stderr, "[dreport] render set %d docs %zu: start %.1f end %.1f ms (kernels %.1f ms)\n", set, d0, rb, since(), ms);
    {
      std::lock_guard<std::mutex> lk(mu);
      busy[set] = true;
      queued = set;
    }
    cv.notify_all();
  }
  {
    // wait for the copy thread to drain both sets
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return (!busy[0] && !busy[1] && queued < 0) || failed; });
  }
  if (cex) std::rethrow_exception(cex);
  if (failed) { err = cerr; return false; }
  return true;
}

bool device_report_json(gg_session* s, size_t first, size_t count, size_t report_first, ReportSink& sink, ReportError& err,
                        DevReportStats* stats, int push_default = 0) {
  return device_report_text(s, first, count, report_first, sink, err, stats, OUT_JSON, push_default);
}

// One shard of a structured report: documents [first, first + count) of a fetched session.
struct ShardView {
  gg_session* s;
  size_t first, count;
};

// The structured report (format `fmt`, OutFormat) of shards in order -- each a contiguous document range
// of its own session, together the job's documents in order -- joined into the bytes one session over all
// of them writes: JSON parts concatenated, YAML streams concatenated, SARIF / JUnit writers absorbed in
// order (so a job sharded over devices reports exactly as the one-device run).  false + err for an
// aborting error.  (cstr != null and JSON: the report goes to *cstr, a malloc'd buffer, without an
// intermediate string.)
bool shards_report(const std::vector<ShardView>& sh, std::string& out, int32_t& exit_code, ReportError& err, int32_t fmt,
                   char** cstr) {
  exit_code = sh.empty() || sh[0].s->parse_errors.empty() ? 0 : 5;
  // the first tile in (doc, rules-file) order that raised an error aborts the run (structured.rs:110)
  for (const ShardView& v : sh) {
    const size_t nf = v.s->progs.size();
    for (size_t t = v.first * nf; t < (v.first + v.count) * nf; t++) {
      if (v.s->tiles[t].err) {
        ensure_host_arena(v.s);
        std::vector<const Program*> progs;
        for (auto& p : v.s->progs) progs.push_back(&p->prog);
        tile_error(v.s->docs, (uint32_t)(t / nf), *progs[t % nf], v.s->tiles[t], err);
        exit_code = -1;
        return false;
      }
    }
  }
  out.clear();
  bool anyfail = false;
  bool on_device = fmt == OUT_JSON && cstr && !sh.empty();
  for (const ShardView& v : sh) on_device = on_device && (v.count == 0 || (device_report_on(v.s) && v.s->fetched_on_device));
  if (on_device) {
    // the FileReports rendered on the shards' devices (report_gpu.hip), joined in document order
    BufferSink sink;
    size_t ndocs = 0;
    bool firstdoc = true;
    sink.write("[\n", 2);
    for (const ShardView& v : sh) {
      if (!v.count) continue;
      if (!device_report_json(v.s, v.first, v.count, firstdoc ? v.first : SIZE_MAX, sink, err, nullptr)) { exit_code = -1; return false; }
      firstdoc = false;
      ndocs += v.count;
      const size_t nf = v.s->progs.size();
      for (size_t t = v.first * nf; t < (v.first + v.count) * nf; t++) if (v.s->tiles[t].status == ST_FAIL) anyfail = true;
    }
    if (ndocs) sink.write("\n]", 2);
    else { sink.n = 0; sink.write("[]", 2); }
    *cstr = sink.take();
    if (anyfail && !(fmt == OUT_JUNIT && exit_code == 5)) exit_code = 19;
    return true;
  }
  // GG_DEVICE_SARIF=0: the host writer for SARIF as well
  bool sarif_dev = fmt == OUT_SARIF && cstr && !sh.empty() && !(getenv("GG_DEVICE_SARIF") && atoi(getenv("GG_DEVICE_SARIF")) == 0);
  for (const ShardView& v : sh) sarif_dev = sarif_dev && (v.count == 0 || (device_report_on(v.s) && v.s->fetched_on_device));
  if (sarif_dev) {
    // SarifReport::new (sarif.rs:29-53, 185-203): the artifacts -- the FAILed documents' first-seen
    // non-empty names, from the fetched statuses -- written here, every FAILed document's results rendered
    // on its shard's device (report_gpu.hip rg::file_sarif) and joined in document order
    std::vector<std::string> art;
    std::unordered_set<std::string> seen;
    for (const ShardView& v : sh) {
      const size_t nf = v.s->progs.size();
      for (size_t d = v.first; d < v.first + v.count; d++) {
        uint32_t status = ST_SKIP;
        for (size_t f = 0; f < nf; f++) {
          const uint32_t st = v.s->tiles[d * nf + f].status;   // Status::and (rules/mod.rs:122-133)
          if (status == ST_FAIL) continue;
          status = status == ST_PASS ? (st == ST_FAIL ? ST_FAIL : ST_PASS) : st;
        }
        if (status != ST_FAIL) continue;
        anyfail = true;
        const std::string& name = v.s->docs.names[d];
        if (!name.empty() && seen.insert(name).second) art.push_back(name);
      }
    }
    std::string head, tail;
    sarif_frame(art, head, tail);
    BufferSink sink;
    sink.write(head.data(), head.size());
    // the results' first comma is dropped: "[\n        {" as serde's pretty printer writes it
    struct DropFirst : ReportSink {
      ReportSink& in;
      char* last = nullptr;
      uint64_t n = 0;
      explicit DropFirst(ReportSink& s) : in(s) {}
      char* reserve(size_t k) override { return last = in.reserve(k); }
      void commit(size_t k) override {
        if (!k) return;
        if (n == 0) { memmove(last, last + 1, k - 1); in.commit(k - 1); }
        else in.commit(k);
        n += k;
      }
      size_t max_piece() const override { return in.max_piece(); }
      bool pinned() const override { return in.pinned(); }
    } results(sink);
    for (const ShardView& v : sh) {
      if (!v.count || v.s->progs.empty()) continue;
      if (!device_report_text(v.s, v.first, v.count, SIZE_MAX, results, err, nullptr, OUT_SARIF)) { exit_code = -1; return false; }
    }
    if (results.n) sink.write("\n      ", 7);
    sink.write(tail.data(), tail.size());
    *cstr = sink.take();
    if (anyfail) exit_code = 19;
    return true;
  }
  std::vector<TextBuf> all_parts;
  std::vector<std::unique_ptr<ReportWriter>> writers;
  std::vector<std::string> yaml_parts;
  for (const ShardView& v : sh) {
    gg_session* s = v.s;
    ensure_host_arena(s);   // host writers
    std::vector<const Program*> progs;
    for (auto& p : s->progs) progs.push_back(&p->prog);
    const size_t nf = progs.size();
    auto tile = [&](size_t d, size_t f) {
      return tile_view(s->tiles.data(), s->rule_status.data(), s->max_top, s->recs.data(), d * nf + f);
    };
    bool ok;
    if (fmt == OUT_JSON && cstr) {
      std::vector<TextBuf> parts;
      ok = report_batch_json_parts(s->docs, progs, v.first, v.count, tile, report_threads(), parts, err);
      for (auto& p : parts) all_parts.push_back(std::move(p));
    } else {
      ok = report_batch_writers(s->docs, progs, v.first, v.count, tile, fmt, report_threads(), writers, yaml_parts, err);
    }
    if (!ok) { exit_code = -1; return false; }
    for (size_t t = v.first * nf; t < (v.first + v.count) * nf; t++) if (s->tiles[t].status == ST_FAIL) anyfail = true;
  }
  if (fmt == OUT_JSON && cstr) *cstr = json_parts_join(all_parts);
  else out = report_writers_finish(fmt, writers, yaml_parts);
  // exit code 19 when any rules file FAILed; a rules-file parse error set 5 beforehand
  // (structured.rs:40-43).  CommonStructuredReporter overwrites it with 19 (structured.rs:110-112);
  // JunitReporter::update_exit_code keeps 5 (reporters/mod.rs:97-103, validate/xml.rs:62-66).
  if (anyfail && !(fmt == OUT_JUNIT && exit_code == 5)) exit_code = 19;
  return true;
}

// structured report over (docs x programs) in format `fmt`; documents [first, first + count) only (count
// SIZE_MAX: to the end): the report a run over just those documents writes -- a rank's shard of a
// multi-GPU job (sharding.gather_report stitches them).
bool session_report(gg_session* s, std::string& out, int32_t& exit_code, ReportError& err, int32_t fmt = OUT_JSON,
                    char** cstr = nullptr, size_t first = 0, size_t count = SIZE_MAX) {
  first = std::min(first, s->docs.ndocs());
  const size_t nd = std::min(count, s->docs.ndocs() - first);
  return shards_report({ShardView{s, first, nd}}, out, exit_code, err, fmt, cstr);
}

// Contiguous document ranges, one per shard, balanced by text bytes (a document's arena and work are
// proportional to its text); starts[k] = first document of shard k, starts[nshards] = n.
// Every shard gets at least one document while documents remain (the algorithm of
// sharding.shard_ranges_by_bytes).
void shard_by_bytes(const size_t* lens, size_t n, size_t nshards, size_t* starts) {
  double total = 0;
  for (size_t i = 0; i < n; i++) total += (double)lens[i];
  size_t start = 0;
  double acc = 0;
  for (size_t r = 0; r < nshards; r++) {
    starts[r] = start;
    const double target = total * (double)(r + 1) / (double)nshards;
    size_t end = start;
    while (end < n && (acc + (double)lens[end] <= target || end == start) && n - end > nshards - r - 1) {
      acc += (double)lens[end];
      end++;
    }
    if (r == nshards - 1) { while (end < n) { acc += (double)lens[end]; end++; } }
    start = end;
  }
  starts[nshards] = n;
}

// Appends per-thread batches to dst.  Every distinct string of every part is interned into dst's
// pool first (parts in order), so the merged pool again holds each string once and pool offsets
// stay string ids; then each part's nodes are copied, remapped and rebased by its own thread (the
// arena of a 1M-template corpus is tens of GB).
void merge_batches(DocBatch& dst, std::vector<DocBatch>& parts) {
  size_t np = parts.size();
  std::vector<size_t> nbase(np + 1), rbase(np + 1);
  nbase[0] = dst.nodes.size(); rbase[0] = dst.roots.size();
  for (size_t t = 0; t < np; t++) {
    nbase[t + 1] = nbase[t] + parts[t].nodes.size();
    rbase[t + 1] = rbase[t] + parts[t].roots.size();
  }
  // part pool offset (16-byte granule) -> dst pool offset
  std::vector<std::vector<uint32_t>> remap(np);
  for (size_t t = 0; t < np; t++) {
    const DocBatch& src = parts[t];
    remap[t].assign(src.bytes.size() / 16 + 1, NONE);
    for (size_t i = 0; i < src.islots.size(); i++) {
      if (!src.islots[i]) continue;
      uint32_t off = src.islots[i] - 1, len = src.ilen[i];
      if (dst.bytes.size() + len + 16 > kMaxPoolBytes)
        throw std::runtime_error("document batch is full (u32 string-pool offsets); evaluate it and start a new batch");
      remap[t][off / 16] = dst.intern(src.bytes.data() + off, len, fnv1a(src.bytes.data() + off, len));
    }
  }
  dst.nodes.resize(nbase[np]); dst.line.resize(nbase[np]); dst.col.resize(nbase[np]);
  dst.kline.resize(nbase[np]); dst.kcol.resize(nbase[np]);
  dst.roots.resize(rbase[np]);
  dst.base.resize(rbase[np]);
  for (auto& p : parts) if (p.serde) dst.serde = true;
  // node indices are document-relative, so only string ids and document bases move
  auto work = [&](size_t t) {
    const DocBatch& src = parts[t];
    const uint32_t* rm = remap[t].data();
    size_t nb = nbase[t];
    DNode* out = dst.nodes.data() + nb;
    for (size_t i = 0; i < src.nodes.size(); i++) {
      DNode n = src.nodes[i];
      if (n.kind == K_STRING) { n.a = rm[n.a / 16]; n.b = n.a; }
      if (n.key_off != NONE) { n.key_off = rm[n.key_off / 16]; n.key_hash = n.key_off; }
      out[i] = n;
    }
    size_t nn = src.nodes.size() * sizeof(uint32_t);
    if (nn) {
      memcpy(dst.line.data() + nb, src.line.data(), nn);
      memcpy(dst.col.data() + nb, src.col.data(), nn);
      memcpy(dst.kline.data() + nb, src.kline.data(), nn);
      memcpy(dst.kcol.data() + nb, src.kcol.data(), nn);
    }
    for (size_t r = 0; r < src.roots.size(); r++) {
      dst.roots[rbase[t] + r] = src.roots[r];
      dst.base[rbase[t] + r] = src.base[r] + nb;
    }
  };
  parallel_run(np, work);
  for (auto& p : parts) {
    dst.names.insert(dst.names.end(), std::make_move_iterator(p.names.begin()), std::make_move_iterator(p.names.end()));
    p = DocBatch();
  }
}

void merge_batch(DocBatch& dst, DocBatch& src) {
  std::vector<DocBatch> one(1);
  one[0] = std::move(src);
  merge_batches(dst, one);
}

// Input parameters (validate.rs:317-350): each file loaded like a data file (build_data_file), then
// merged in order, `primary = primary.merge(path_value)?` -- a merge error aborts (no unwrap here)
bool load_params(const validate_input_t* params, size_t n, std::unique_ptr<DocBatch>& out, LoadError& le) {
  out.reset();
  for (size_t i = 0; i < n; i++) {
    const char* t = params[i].content ? params[i].content : "";
    std::unique_ptr<DocBatch> next(new DocBatch());
    if (!load_document(*next, t, strlen(t), params[i].file_name ? params[i].file_name : "", LOAD_LIBYAML, le)) return false;
    if (out && !merge_into_last(*next, 0, *out, 0, le)) return false;
    out = std::move(next);
  }
  return true;
}

// Rust Debug of a merge Error (derived: `Variant("message")`), as `.unwrap()` prints it
std::string merge_error_debug(const LoadError& le) { return le.kind + "(" + rust_debug_str(le.msg) + ")"; }

// merged_data (structured.rs:51-65): `data.clone().merge(file.path_value.clone()).unwrap()` -- a
// merge error is a panic there; here code -1 with the panic message
bool merge_params_last(DocBatch& b, const DocBatch* params, LoadError& le) {
  if (!params || b.ndocs() == 0) return true;
  LoadError me;
  if (merge_into_last(b, b.ndocs() - 1, *params, 0, me)) return true;
  le.kind = "Panic";
  le.msg = "called `Result::unwrap()` on an `Err` value: " + merge_error_debug(me);
  return false;
}

bool add_rules(gg_session* s, const std::string& text, const std::string& name, std::string& perr) {
  RulesFile rf;
  bool empty = false;
  std::string msg;
  if (!parse_rules_file(text, name, rf, empty, msg)) { perr = msg; return false; }
  if (empty) return true;
  auto gp = std::make_unique<GpuProgram>();
  std::string cerr;
  if (!compile_program(rf, name, gp->prog, cerr)) { perr = cerr; return false; }
  s->progs.push_back(std::move(gp));
  return true;
}

}  // namespace

extern "C" {

void cfn_guard_free_string(char* s) { free(s); }

char* cfn_guard_run_checks(validate_input_t data, validate_input_t rules, bool verbose, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why)) { set_err(err, -1, why); return nullptr; }
    gg_session s;
    std::string dname = data.file_name ? data.file_name : "";
    LoadError le;
    const char* text = data.content ? data.content : "";
    if (!load_document(s.docs, text, strlen(text), dname, LOAD_SERDE, le)) {
      if (le.kind == "YamlError") set_err(err, 2, error_display("YamlError", le.msg));
      else set_err(err, 5, error_display("ParseError", "Unable to process data in file " + dname + ", Error " + error_display(le.kind, le.msg) + ","));
      return nullptr;
    }
    std::string rname = rules.file_name ? rules.file_name : "";
    std::string perr;
    const char* rtext = rules.content ? rules.content : "";
    RulesFile rf;
    bool empty = false;
    if (!parse_rules_file(rtext, rname, rf, empty, perr)) { set_err(err, 5, error_display("ParseError", perr)); return nullptr; }
    if (empty) return dup_str("");
    auto gp = std::make_unique<GpuProgram>();
    if (!compile_program(rf, rname, gp->prog, perr)) { set_err(err, 5, error_display("ParseError", perr)); return nullptr; }
    s.progs.push_back(std::move(gp));
    if (verbose) { s.mode = 1; s.verbose = true; }   // one tile, evaluated by the verbose wave kernel
    session_upload(&s);
    session_run(&s, true);
    if (s.tiles[0].err) {
      ReportError re;
      tile_error(s.docs, 0, s.progs[0]->prog, s.tiles[0], re);
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      return nullptr;
    }
    TileResult tr = tile_view(s.tiles.data(), s.rule_status.data(), s.max_top, s.recs.data(), 0);
    std::string out;
    ReportError re;
    if (verbose) {
      if (!verbose_tree(s.docs, 0, s.progs[0]->prog, tr, dname, out, re)) {
        set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
        return nullptr;
      }
      return dup_str(out);
    }
    std::vector<const Program*> progs{&s.progs[0]->prog};
    std::vector<const TileResult*> tp{&tr};
    if (!report_document(s.docs, 0, progs, tp, 0, out, re)) {
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      return nullptr;
    }
    return dup_str(out);
  } catch (std::exception& e) {
    set_err(err, -1, e.what());
    return nullptr;
  }
}

char* cfn_guard_validate_batch(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules, size_t n_rules,
                               int32_t* exit_code, extern_err_t* err) {
  return cfn_guard_validate_batch_format(docs, n_docs, rules, n_rules, OUT_JSON, exit_code, err);
}

char* cfn_guard_validate_batch_format(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                      size_t n_rules, int32_t output_format, int32_t* exit_code, extern_err_t* err) {
  return cfn_guard_validate_batch_params(docs, n_docs, rules, n_rules, nullptr, 0, output_format, exit_code, err);
}

// The batch entries load a batch of at least GG_BATCH_DEVICE_LOAD_MIN documents (64; 0 = never) without input
// parameters with the device loader (JSON and block-style YAML on the MI355X, the rest on host threads at
// their positions); when that path does not take the whole batch -- too few large documents, a document
// the host loader then rejects -- the documents load one by one on the host as before, so a load error is
// still the first failing document's, with the reference's message.
static bool batch_device_load(gg_session* s, const validate_input_t* docs, size_t n_docs, size_t first, size_t count) {
  const char* e = getenv("GG_BATCH_DEVICE_LOAD_MIN");
  const size_t min_docs = e ? (size_t)std::max(0, atoi(e)) : 64;
  if (!min_docs || count < min_docs || s->params || s->docs.ndocs()) return false;
  (void)n_docs;
  std::vector<const char*> t(count), nm(count);
  std::vector<size_t> l(count);
  // the texts' lengths on the host threads (strlen over ~11 GB of templates is a second on one)
  const size_t nt = std::max<size_t>(1, std::min<size_t>(report_threads(), count / 1024 + 1));
  parallel_run(nt, [&](size_t w) {
    for (size_t i = count * w / nt; i < count * (w + 1) / nt; i++) {
      const validate_input_t& d = docs[first + i];
      t[i] = d.content ? d.content : "";
      l[i] = strlen(t[i]);
      nm[i] = d.file_name ? d.file_name : "";
    }
  });
  extern_err_t le{0, nullptr};
  const int32_t rc = gg_session_add_docs_device(s, t.data(), l.data(), nm.data(), count, nullptr, &le);
  if (le.message) free(le.message);
  return rc == 0;
}

char* cfn_guard_validate_batch_params(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                      size_t n_rules, const validate_input_t* params, size_t n_params,
                                      int32_t output_format, int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (output_format < OUT_JSON || output_format > OUT_JUNIT) {
    set_err(err, 18, "IllegalArguments: unknown output format");
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
  if (exit_code) *exit_code = 0;
  try {
    std::string why;
    if (!ensure_device(why)) { set_err(err, -1, why); if (exit_code) *exit_code = -1; return nullptr; }
    gg_session s;
    for (size_t i = 0; i < n_rules; i++) {
      std::string perr;
      std::string name = rules[i].file_name ? rules[i].file_name : "";
      if (!add_rules(&s, rules[i].content ? rules[i].content : "", name, perr))
        s.parse_errors.push_back("Parsing error handling rule file = " + name + ", Error = " + error_display("ParseError", perr) + "\n---");
    }
    // Validate::execute order: data files (validate.rs:274-315), then the parameter files (317-350),
    // then the merge into every data file (structured.rs:51-65, a panic on conflict)
    LoadError pe;
    const bool params_ok = load_params(params, n_params, s.params, pe);
    LoadError panic;
    bool panicked = false;
    const bool on_device = !n_params && batch_device_load(&s, docs, n_docs, 0, n_docs);
    for (size_t i = 0; i < n_docs && !on_device; i++) {
      LoadError le;
      const char* t = docs[i].content ? docs[i].content : "";
      if (!load_document(s.docs, t, strlen(t), docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, le)) {
        set_err(err, ffi_code(le.kind), error_display(le.kind, le.msg));
        if (exit_code) *exit_code = -1;
        return nullptr;
      }
      if (params_ok && !panicked && !merge_params_last(s.docs, s.params.get(), panic)) panicked = true;
    }
    if (!params_ok || panicked) {
      const LoadError& e = !params_ok ? pe : panic;
      set_err(err, ffi_code(e.kind), error_display(e.kind, e.msg));
      if (exit_code) *exit_code = -1;
      return nullptr;
    }
    session_upload(&s);
    session_run(&s, true);
    std::string out;
    char* cs = nullptr;
    int32_t code = 0;
    ReportError re;
    if (!session_report(&s, out, code, re, output_format, &cs)) {
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      if (exit_code) *exit_code = -1;
      return nullptr;
    }
    if (exit_code) *exit_code = code;
    return cs ? cs : dup_str(out);
  } catch (std::exception& e) {
    set_err(err, -1, e.what());
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
}

// ---------------------------------------------------------------- validate over several GPUs ---
// cfn_guard_validate_batch_params with the documents sharded over devices: contiguous ranges balanced by
// text bytes (shard_by_bytes), one host thread per shard that loads its documents (host loader, with the
// input parameters merged), compiles the rules, uploads, evaluates and fetches on its device; then the
// shards' reports join in document order (shards_report).  Error precedence is the one-device call's: the
// first document (in order) that does not load, then a parameter-file error, then the first parameter merge
// panic, then the first erroring tile, then the first report that aborts.
namespace {
char* validate_batch_devices(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules, size_t n_rules,
                             const validate_input_t* params, size_t n_params, int32_t output_format,
                             const std::vector<int>& devices, int32_t* exit_code, extern_err_t* err) {
  const size_t ns = std::max<size_t>(1, std::min(devices.size(), std::max<size_t>(n_docs, 1)));
  std::vector<size_t> lens(n_docs), starts(ns + 1);
  for (size_t i = 0; i < n_docs; i++) lens[i] = docs[i].content ? strlen(docs[i].content) : 0;
  shard_by_bytes(lens.data(), n_docs, ns, starts.data());
  // the input parameters, loaded once (read-only for the shards' merges)
  std::unique_ptr<DocBatch> pbatch;
  LoadError pe;
  const bool params_ok = load_params(params, n_params, pbatch, pe);
  struct Shard {
    gg_session s;
    size_t load_fail = SIZE_MAX, panic_doc = SIZE_MAX;
    LoadError le, panic;
  };
  std::vector<std::unique_ptr<Shard>> sh(ns);
  for (auto& x : sh) x.reset(new Shard());
  // phase 1: load (every shard on its own thread)
  parallel_run(ns, [&](size_t k) {
    Shard& S = *sh[k];
    S.s.device = devices[k];
    for (size_t i = 0; i < n_rules; i++) {
      std::string perr;
      std::string name = rules[i].file_name ? rules[i].file_name : "";
      if (!add_rules(&S.s, rules[i].content ? rules[i].content : "", name, perr))
        S.s.parse_errors.push_back("Parsing error handling rule file = " + name + ", Error = " + error_display("ParseError", perr) + "\n---");
    }
    const bool on_device = !n_params && batch_device_load(&S.s, docs, n_docs, starts[k], starts[k + 1] - starts[k]);
    for (size_t i = starts[k]; i < starts[k + 1] && !on_device; i++) {
      const char* t = docs[i].content ? docs[i].content : "";
      if (!load_document(S.s.docs, t, lens[i], docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, S.le)) {
        S.load_fail = i;
        return;
      }
      if (params_ok && S.panic_doc == SIZE_MAX && !merge_params_last(S.s.docs, pbatch.get(), S.panic)) S.panic_doc = i;
    }
  });
  auto fail_with = [&](const std::string& kind, const std::string& msg) -> char* {
    set_err(err, ffi_code(kind), error_display(kind, msg));
    if (exit_code) *exit_code = -1;
    return nullptr;
  };
  for (auto& x : sh) if (x->load_fail != SIZE_MAX) return fail_with(x->le.kind, x->le.msg);
  if (!params_ok) return fail_with(pe.kind, pe.msg);
  for (auto& x : sh) if (x->panic_doc != SIZE_MAX) return fail_with(x->panic.kind, x->panic.msg);
  // phase 2: evaluate (every shard on its own thread and device)
  parallel_run(ns, [&](size_t k) {
    Shard& S = *sh[k];
    if (S.s.progs.empty() || S.s.docs.ndocs() == 0) {
      S.s.tiles.clear(); S.s.rule_status.clear(); S.s.recs.clear(); S.s.evaluated = true;
      return;
    }
    session_upload(&S.s);
    session_run(&S.s, true);
  });
  std::vector<ShardView> views;
  for (auto& x : sh) views.push_back(ShardView{&x->s, 0, x->s.docs.ndocs()});
  std::string out;
  char* cs = nullptr;
  int32_t code = 0;
  ReportError re;
  if (!shards_report(views, out, code, re, output_format, &cs)) return fail_with(re.kind, re.msg);
  if (exit_code) *exit_code = code;
  return cs ? cs : dup_str(out);
}
}  // namespace

// ---------------------------------------------------------------- streamed structured JSON ---
// cfn_guard_validate_batch_format(JSON) for a batch whose report does not fit one string (1 M templates:
// 149 GB): the documents run in chunks of `chunk_docs` on two alternating sessions -- a producer thread
// loads (device JSON / YAML loader), uploads, evaluates and fetches chunk k + 1 while this thread renders
// chunk k on the device and hands its text to `write` in document order (text H2D of the next chunk and
// report D2H of this one share the link in opposite directions).  The bytes written are the one-string
// call's; an abort (a load error, an evaluation error, a failing write) ends the stream with code -1 and
// the error, after the chunks before the failing one were written: the caller drops that prefix.
namespace {
struct CallbackSink : ReportSink {
  cfn_guard_write_fn fn;
  void* ctx;
  char* stage;
  size_t stage_bytes;
  bool failed = false;
  uint64_t n = 0;
  CallbackSink(cfn_guard_write_fn f, void* c, char* st, size_t sb) : fn(f), ctx(c), stage(st), stage_bytes(sb) {}
  char* reserve(size_t) override { return stage; }
  bool pinned() const override { return true; }   // pinned_get staging
  void commit(size_t k) override {
    if (!failed && k && fn(ctx, stage, k) != 0) failed = true;
    n += k;
  }
  size_t max_piece() const override { return stage_bytes; }
};
}  // namespace

namespace {
bool first_load_error(const validate_input_t* docs, size_t from, size_t n, std::string& kind, std::string& msg);
int32_t stream_single(int dev, const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                      size_t n_rules, size_t chunk_docs, cfn_guard_write_fn write, void* ctx,
                      int32_t* exit_code, extern_err_t* err) {
  auto fail = [&](int32_t code, const std::string& msg) { set_err(err, code, msg); if (exit_code) *exit_code = -1; return -1; };
  try {
    HIPCHK(hipSetDevice(dev));
    const size_t chunk = chunk_docs ? chunk_docs : (size_t)262144;
    const size_t nchunks = (n_docs + chunk - 1) / chunk;
    // blocks cached by earlier (larger) calls are of other sizes: freed now, while nothing of this call
    // runs, so that the chunks' own blocks fit under the cache bound and are reused from chunk 3 on
    dev_cache_flush(dev);
    char* stage = nullptr;
    stage = (char*)pinned_get(DeviceBufs::kPinnedBytes, dev);
    if (!stage) throw std::runtime_error("pinned host staging: allocation failed");
    struct StageFree { char* p; int d; ~StageFree() { pinned_put(p, DeviceBufs::kPinnedBytes, d); } } stage_free{stage, dev};
    CallbackSink sink(write, ctx, stage, DeviceBufs::kPinnedBytes);
    // producer / consumer over two slots
    struct Slot {
      std::unique_ptr<gg_session> s;
      size_t k = SIZE_MAX;     // chunk held
      int state = 0;           // 0 free, 1 ready, 2 failed
      std::string kind, msg;
    } slot[2];
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
    int32_t parse_code = 0;
    // GG_STREAM_TRACE=1: per-chunk wall-clock marks on stderr
    const bool trace = getenv("GG_STREAM_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char* what, size_t k) {
      if (trace) fprintf(stderr, "[stream] %8.1f ms  chunk %zu %s\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), k, what);
    };
    // GG_STREAM_SERIAL=1 (diagnostic): a chunk loads only after the previous one is reported
    const bool serial = getenv("GG_STREAM_SERIAL") != nullptr;
    size_t reported = 0;
    // chunk j's session has been torn down (its buffer set is back in the pool): chunk j + 2 uploads into it
    std::vector<char> torn(nchunks, 0);
    std::thread producer([&]() {
      for (size_t k = 0; k < nchunks; k++) {
        Slot& sl = slot[k & 1];
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return (sl.state == 0 && (!serial || reported == k)) || stop; });
          if (stop) return;
        }
        mark("load start", k);
        std::string kind, msg;
        std::unique_ptr<gg_session> ses(new gg_session());
        try {
          ses->device = dev;
          ses->defer_recs = true;   // the device report reads the records in HBM
          for (size_t i = 0; i < n_rules; i++) {
            std::string perr;
            const std::string name = rules[i].file_name ? rules[i].file_name : "";
            if (!add_rules(ses.get(), rules[i].content ? rules[i].content : "", name, perr))
              ses->parse_errors.push_back("Parsing error handling rule file = " + name + ", Error = " + error_display("ParseError", perr) + "\n---");
          }
          const size_t first = k * chunk, count = std::min(chunk, n_docs - first);
          if (!batch_device_load(ses.get(), docs, n_docs, first, count)) {
            for (size_t i = first; i < first + count; i++) {
              LoadError le;
              const char* t = docs[i].content ? docs[i].content : "";
              if (!load_document(ses->docs, t, strlen(t), docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, le)) {
                kind = le.kind; msg = le.msg;
                break;
              }
            }
          }
          mark("loaded", k);
          if (kind.empty()) {
            if (ses->progs.empty()) {
              ses->tiles.clear(); ses->rule_status.clear(); ses->recs.clear(); ses->evaluated = true;
            } else {
              // the load ran alongside chunk k - 2's teardown; the upload takes that chunk's buffer set (a new set
              // would allocate ~25 GB afresh: chunk 3's upload took 3.8 s instead of 40 ms when it raced the
              // teardown, profiles/r06zj_stream_load_trace.log)
              if (k >= 2) {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return torn[k - 2] || stop; });
              }
              session_upload(ses.get());
              mark("uploaded", k);
              session_run(ses.get(), true);
            }
          }
          mark("evaluated", k);
        } catch (std::exception& e) { kind = "Internal"; msg = e.what(); }
        {
          std::lock_guard<std::mutex> lk(mu);
          sl.s = std::move(ses);
          sl.k = k;
          sl.state = kind.empty() ? 1 : 2;
          sl.kind = kind; sl.msg = msg;
        }
        cv.notify_all();
        if (!kind.empty()) return;
      }
    });
    struct Join {
      std::thread& t; std::mutex& mu; std::condition_variable& cv; bool& stop;
      ~Join() { { std::lock_guard<std::mutex> lk(mu); stop = true; } cv.notify_all(); if (t.joinable()) t.join(); }
    } join{producer, mu, cv, stop};
    // Chunk k's report runs on a thread of its own, so chunk k + 1's report renders its first blocks on the
    // device while chunk k's last blocks copy out (within one chunk the render of the first block and the copy of
    // the last one ran alone).  The bytes stay in document order: a report's sink waits for its turn before it
    // takes the staging (OrderedSink), and the turn passes when the previous chunk's report has returned.  The
    // report thread then frees the chunk's slot for the producer and tears the session down.
    struct Turn {
      std::mutex m;
      std::condition_variable cv;
      size_t turn = 0;
      bool abort = false;
    } turn;
    struct OrderedSink : ReportSink {
      ReportSink& in;
      Turn& t;
      size_t k;
      bool mine = false;
      OrderedSink(ReportSink& s, Turn& tt, size_t kk) : in(s), t(tt), k(kk) {}
      char* reserve(size_t n) override {
        if (!mine) {
          std::unique_lock<std::mutex> lk(t.m);
          t.cv.wait(lk, [&] { return t.turn == k || t.abort; });
          if (t.abort) throw std::runtime_error("stream aborted");
          mine = true;
        }
        return in.reserve(n);
      }
      void commit(size_t n) override { in.commit(n); }
      size_t max_piece() const override { return in.max_piece(); }
      bool pinned() const override { return in.pinned(); }
    };
    struct ChunkReport {
      std::thread th;
      bool ok = true;
      ReportError re;
      std::string internal;
    };
    std::vector<std::unique_ptr<ChunkReport>> reps(nchunks);
    struct JoinReports {
      std::vector<std::unique_ptr<ChunkReport>>& v; Turn& t;
      ~JoinReports() {
        { std::lock_guard<std::mutex> lk(t.m); t.abort = true; }
        t.cv.notify_all();
        for (auto& r : v) if (r && r->th.joinable()) r->th.join();
      }
    } join_reports{reps, turn};
    // the first failed chunk report in document order (joining every report before it), or -1
    // the one-string call loads every data file before it evaluates or reports: a document after chunk j that
    // does not load takes precedence over chunk j's evaluation or report error
    auto later_load_error = [&](size_t j, std::string& k, std::string& m) {
      return first_load_error(docs, std::min(n_docs, (j + 1) * chunk), n_docs, k, m);
    };
    auto first_failure = [&](size_t upto) -> int32_t {
      for (size_t j = 0; j < upto; j++) {
        if (!reps[j]) continue;
        if (reps[j]->th.joinable()) reps[j]->th.join();
        if (!reps[j]->internal.empty()) return fail(-1, reps[j]->internal);
        if (!reps[j]->ok) {
          std::string lk, lm;
          if (later_load_error(j, lk, lm)) return fail(ffi_code(lk), error_display(lk, lm));
          return fail(ffi_code(reps[j]->re.kind), error_display(reps[j]->re.kind, reps[j]->re.msg));
        }
      }
      if (sink.failed) return fail(-1, "the write callback failed");
      return 0;
    };
    bool anyfail = false;
    if (!n_docs) {
      // no documents: "[]", exit 5 when a rules file does not parse (as the one-string call)
      gg_session rs;
      for (size_t i = 0; i < n_rules; i++) {
        std::string perr;
        if (!add_rules(&rs, rules[i].content ? rules[i].content : "", rules[i].file_name ? rules[i].file_name : "", perr))
          parse_code = 5;
      }
      sink.write("[]", 2);
    }
    for (size_t k = 0; k < nchunks; k++) {
      Slot& sl = slot[k & 1];
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return sl.state != 0 && sl.k == k; });
      }
      // chunk k's slot was freed by chunk k - 2's report at its end: that thread is done; join it now (at most
      // three report threads exist at a time, however many chunks) and keep only a failed one's result
      if (k >= 2 && reps[k - 2]) {
        if (reps[k - 2]->th.joinable()) reps[k - 2]->th.join();
        if (!reps[k - 2]->ok || !reps[k - 2]->internal.empty()) {
          if (first_failure(k - 1)) return -1;
        } else {
          reps[k - 2].reset();
        }
      }
      mark("report start", k);
      if (sl.state == 2) {
        if (first_failure(k)) return -1;
        return fail(ffi_code(sl.kind), error_display(sl.kind, sl.msg));
      }
      gg_session* s = sl.s.get();
      if (k == 0) parse_code = s->parse_errors.empty() ? 0 : 5;
      const size_t nf = s->progs.size(), nd = s->docs.ndocs();
      for (size_t t = 0; t < nd * nf; t++) {
        if (s->tiles[t].err) {
          if (first_failure(k)) return -1;
          ensure_host_arena(s);
          std::vector<const Program*> progs;
          for (auto& p : s->progs) progs.push_back(&p->prog);
          ReportError re;
          tile_error(s->docs, (uint32_t)(t / nf), *progs[t % nf], s->tiles[t], re);
          std::string lk, lm;
          if (later_load_error(k, lk, lm)) return fail(ffi_code(lk), error_display(lk, lm));
          return fail(ffi_code(re.kind), error_display(re.kind, re.msg));
        }
        if (s->tiles[t].status == ST_FAIL) anyfail = true;
      }
      if (k == 0) sink.write("[\n", 2);
      reps[k].reset(new ChunkReport());
      ChunkReport* cr = reps[k].get();
      cr->th = std::thread([&, k, s, cr, nf, nd]() {
        OrderedSink osink(sink, turn, k);
        try {
          HIPCHK(hipSetDevice(dev));
          if (nf && device_report_on(s) && s->fetched_on_device) {
            cr->ok = device_report_json(s, 0, nd, k == 0 ? 0 : SIZE_MAX, osink, cr->re, nullptr, kStreamPushBlocks);
          } else {
            // host writer for this chunk: its "[\n" ... "\n]" unwrapped, joined with ",\n"
            std::string out;
            char* cs = nullptr;
            int32_t code = 0;
            cr->ok = session_report(s, out, code, cr->re, OUT_JSON, &cs);
            if (cr->ok) {
              std::string text = cs ? std::string(cs) : out;
              if (text.size() >= 4 && text.compare(0, 2, "[\n") == 0) {
                if (k) osink.write(",\n", 2);
                osink.write(text.data() + 2, text.size() - 4);
              }
            }
            if (cs) free(cs);
          }
        } catch (std::exception& e) {
          cr->internal = e.what();
        }
        mark("reported", k);
        {
          // the turn passes strictly in chunk order: a chunk that wrote nothing (and so never waited in
          // OrderedSink::reserve) still waits for its predecessor before handing the turn on
          std::unique_lock<std::mutex> lk(turn.m);
          if (cr->ok && cr->internal.empty()) {
            turn.cv.wait(lk, [&] { return turn.turn == k || turn.abort; });
            if (!turn.abort) turn.turn = k + 1;
          } else {
            turn.abort = true;   // the chunks after a failed one are not written
          }
        }
        turn.cv.notify_all();
        std::unique_ptr<gg_session> done;
        {
          std::lock_guard<std::mutex> lk(mu);
          done = std::move(slot[k & 1].s);
          slot[k & 1].state = 0;
          slot[k & 1].k = SIZE_MAX;
          reported = k + 1;
        }
        cv.notify_all();
        done.reset();
        {
          std::lock_guard<std::mutex> lk(mu);
          torn[k] = 1;
        }
        cv.notify_all();
        mark("torn down", k);
      });
    }
    if (first_failure(nchunks)) return -1;
    if (nchunks) sink.write("\n]", 2);
    if (sink.failed) return fail(-1, "the write callback failed");
    if (exit_code) *exit_code = anyfail ? 19 : parse_code;
    return 0;
  } catch (std::exception& e) {
    return fail(-1, e.what());
  }
}
}  // namespace

int32_t cfn_guard_validate_batch_stream(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                        size_t n_rules, size_t chunk_docs, cfn_guard_write_fn write, void* ctx,
                                        int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (exit_code) *exit_code = 0;
  if (!write) { set_err(err, 18, "IllegalArguments: no write callback"); if (exit_code) *exit_code = -1; return -1; }
  std::string why;
  int dev = 0;
  if (!ensure_device(why, -1, &dev)) { set_err(err, -1, why); if (exit_code) *exit_code = -1; return -1; }
  return stream_single(dev, docs, n_docs, rules, n_rules, chunk_docs, write, ctx, exit_code, err);
}

// ---------------------------------------------------------------- streamed, several devices ---
// cfn_guard_validate_batch_stream with the chunks spread over a device list (SURVEY.md 8(b) n_gpus, 8(e)):
// chunk k (chunk_docs documents) runs on pipeline k % ndev, a host thread bound to devices[k % ndev], which
// loads, uploads, evaluates and fetches it and renders its JSON report on that device into a host buffer
// of its own; this thread hands the buffers to `write` in chunk order (structured.rs:122-129: one writer,
// documents in order).  A pipeline starts chunk k only once chunk k - 2 ndev has been written, so host
// memory holds at most two chunks' reports per device.  Errors: the first in document order, as the
// one-device stream (load error, erroring tile, report abort), after the chunks before it were written.
namespace {
// chunk k's report text (its "[\n" ... "\n]" unwrapped; ",\n" before it unless k == 0) into `sink`;
// false + re for an abort
bool stream_chunk_report(gg_session* s, size_t k, ReportSink& sink, ReportError& re, bool& anyfail) {
  const size_t nf = s->progs.size(), nd = s->docs.ndocs();
  for (size_t t = 0; t < nd * nf; t++) {
    if (s->tiles[t].err) {
      ensure_host_arena(s);
      std::vector<const Program*> progs;
      for (auto& p : s->progs) progs.push_back(&p->prog);
      tile_error(s->docs, (uint32_t)(t / nf), *progs[t % nf], s->tiles[t], re);
      return false;
    }
    if (s->tiles[t].status == ST_FAIL) anyfail = true;
  }
  if (nf && device_report_on(s) && s->fetched_on_device)
    return device_report_json(s, 0, nd, k == 0 ? 0 : SIZE_MAX, sink, re, nullptr, kStreamPushBlocks);
  std::string out;
  char* cs = nullptr;
  int32_t code = 0;
  if (!session_report(s, out, code, re, OUT_JSON, &cs)) return false;
  std::string text = cs ? std::string(cs) : out;
  if (cs) free(cs);
  if (text.size() >= 4 && text.compare(0, 2, "[\n") == 0) {
    if (k) sink.write(",\n", 2);
    sink.write(text.data() + 2, text.size() - 4);
  }
  return true;
}
// chunk [first, first + count) loaded, evaluated and fetched on `dev`; kind / msg for a load error
std::unique_ptr<gg_session> stream_chunk_session(int dev, const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                                 size_t n_rules, size_t first, size_t count, std::string& kind, std::string& msg) {
  std::unique_ptr<gg_session> ses(new gg_session());
  ses->device = dev;
  ses->defer_recs = true;   // the device report reads the records in HBM
  for (size_t i = 0; i < n_rules; i++) {
    std::string perr;
    const std::string name = rules[i].file_name ? rules[i].file_name : "";
    if (!add_rules(ses.get(), rules[i].content ? rules[i].content : "", name, perr))
      ses->parse_errors.push_back("Parsing error handling rule file = " + name + ", Error = " + error_display("ParseError", perr) + "\n---");
  }
  if (!batch_device_load(ses.get(), docs, n_docs, first, count)) {
    for (size_t i = first; i < first + count; i++) {
      LoadError le;
      const char* t = docs[i].content ? docs[i].content : "";
      if (!load_document(ses->docs, t, strlen(t), docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, le)) {
        kind = le.kind; msg = le.msg;
        return ses;
      }
    }
  }
  if (ses->progs.empty()) {
    ses->tiles.clear(); ses->rule_status.clear(); ses->recs.clear(); ses->evaluated = true;
  } else {
    session_upload(ses.get());
    session_run(ses.get(), true);
  }
  return ses;
}
}  // namespace

namespace {
// A chunk's report lands by D2H in pinned host blocks (a device-to-pageable copy is staged through
// the runtime's bounce buffers at a fraction of the PCIe rate) and goes to the callback from there;
// written blocks are recycled, so after the first chunks no block is allocated or pinned again.
struct PinnedPool {
  static constexpr size_t kBlock = (size_t)64 << 20;
  std::mutex mu;
  std::vector<std::pair<char*, int>> all;   // every block of the call, with its device
  std::vector<char*> avail;
  char* get() {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (!avail.empty()) { char* p = avail.back(); avail.pop_back(); return p; }
    }
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    char* p = (char*)pinned_get(kBlock, dev);   // on the node of the calling pipeline's device
    if (!p) throw std::runtime_error("pinned host block: allocation failed");
    std::lock_guard<std::mutex> lk(mu);
    all.push_back({p, dev});
    return p;
  }
  void put(char* p) { std::lock_guard<std::mutex> lk(mu); avail.push_back(p); }
  ~PinnedPool() { for (auto& b : all) pinned_put(b.first, kBlock, b.second); }
};
struct ChainSink : ReportSink {
  PinnedPool& pool;
  std::vector<std::pair<char*, size_t>> blocks;   // (block, bytes used)
  uint64_t n = 0;
  explicit ChainSink(PinnedPool& p) : pool(p) {}
  char* reserve(size_t k) override {
    if (blocks.empty() || blocks.back().second + k > PinnedPool::kBlock) blocks.push_back({pool.get(), 0});
    return blocks.back().first + blocks.back().second;
  }
  void commit(size_t k) override { blocks.back().second += k; n += k; }
  size_t max_piece() const override { return PinnedPool::kBlock; }
  bool pinned() const override { return true; }
};
}  // namespace

int32_t cfn_guard_validate_batch_stream_devices(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                                size_t n_rules, size_t chunk_docs, const int32_t* devices, size_t n_devices,
                                                cfn_guard_write_fn write, void* ctx, int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (exit_code) *exit_code = 0;
  auto fail = [&](int32_t code, const std::string& msg) { set_err(err, code, msg); if (exit_code) *exit_code = -1; return -1; };
  if (!write) return fail(18, "IllegalArguments: no write callback");
  try {
    std::vector<int> devs;
    std::string why;
    if (devices) {
      for (size_t i = 0; i < n_devices; i++) devs.push_back(devices[i]);
    } else {
      int n = 0;
      if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
      for (int d = 0; d < n; d++) devs.push_back(d);
    }
    if (devs.empty()) return fail(-1, devices ? "IllegalArguments: an empty device list" : "no HIP device available (the MI355X path has no CPU fallback)");
    for (int d : devs)
      if (!ensure_device(why, d)) return fail(-1, why);
    const size_t ndev = devs.size();
    // one device: the one-device stream (its report copied out straight into the callback's staging)
    if (ndev == 1) return stream_single(devs[0], docs, n_docs, rules, n_rules, chunk_docs, write, ctx, exit_code, err);
    const size_t chunk = chunk_docs ? chunk_docs : (size_t)16384;
    const size_t nchunks = (n_docs + chunk - 1) / chunk;
    PinnedPool pool;
    struct Out {
      int state = 0;          // 0 pending, 1 ready, 2 failed
      ChainSink text;
      explicit Out(PinnedPool& p) : text(p) {}
      bool anyfail = false, load_error = false;
      int32_t parse_code = 0;
      std::string kind, msg;
    };
    std::vector<std::unique_ptr<Out>> outs(nchunks);
    for (auto& o : outs) o.reset(new Out(pool));
    std::mutex mu;
    std::condition_variable cv;
    size_t written = 0;
    bool stop = false;
    std::vector<std::thread> pipes;
    for (size_t p = 0; p < std::min(ndev, nchunks); p++) {
      pipes.emplace_back([&, p]() {
        for (size_t k = p; k < nchunks; k += ndev) {
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || k < 2 * ndev || written > k - 2 * ndev; });
            if (stop) return;
          }
          Out& o = *outs[k];
          std::string kind, msg;
          try {
            const size_t first = k * chunk, count = std::min(chunk, n_docs - first);
            std::unique_ptr<gg_session> ses = stream_chunk_session(devs[p], docs, n_docs, rules, n_rules, first, count, kind, msg);
            o.load_error = !kind.empty();
            if (kind.empty()) {
              o.parse_code = ses->parse_errors.empty() ? 0 : 5;
              ReportError re;
              if (!stream_chunk_report(ses.get(), k, o.text, re, o.anyfail)) { kind = re.kind; msg = re.msg; }
            }
          } catch (std::exception& e) { kind = "Internal"; msg = e.what(); }
          {
            std::lock_guard<std::mutex> lk(mu);
            o.kind = kind; o.msg = msg;
            o.state = kind.empty() ? 1 : 2;
          }
          cv.notify_all();
          if (!kind.empty()) return;
        }
      });
    }
    struct JoinAll {
      std::vector<std::thread>& v; std::mutex& mu; std::condition_variable& cv; bool& stop;
      ~JoinAll() { { std::lock_guard<std::mutex> lk(mu); stop = true; } cv.notify_all(); for (auto& t : v) if (t.joinable()) t.join(); }
    } join{pipes, mu, cv, stop};
    char* stage = nullptr;
    HIPCHK(hipHostMalloc((void**)&stage, 1u << 20, hipHostMallocDefault));
    struct StageFree { char* p; ~StageFree() { if (p) hipHostFree(p); } } stage_free{stage};
    CallbackSink sink(write, ctx, stage, 1u << 20);
    int32_t parse_code = 0;
    bool anyfail = false;
    if (!n_docs) {
      gg_session rs;
      for (size_t i = 0; i < n_rules; i++) {
        std::string perr;
        if (!add_rules(&rs, rules[i].content ? rules[i].content : "", rules[i].file_name ? rules[i].file_name : "", perr))
          parse_code = 5;
      }
      sink.write("[]", 2);
    }
    for (size_t k = 0; k < nchunks; k++) {
      Out& o = *outs[k];
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return o.state != 0; });
      }
      if (o.state == 2) {
        // an evaluation or report error yields to a later document that does not load (one-string precedence)
        std::string lk, lm;
        if (!o.load_error && o.kind != "Internal" && first_load_error(docs, std::min(n_docs, (k + 1) * chunk), n_docs, lk, lm))
          return fail(ffi_code(lk), error_display(lk, lm));
        return fail(ffi_code(o.kind), error_display(o.kind, o.msg));
      }
      if (k == 0) { parse_code = o.parse_code; sink.write("[\n", 2); }
      anyfail = anyfail || o.anyfail;
      // the pinned blocks go to the callback as they are (no staging copy), then back to the pool; a
      // failing callback ends the stream
      for (auto& b : o.text.blocks) {
        if (!sink.failed && b.second && write(ctx, b.first, b.second) != 0) sink.failed = true;
        pool.put(b.first);
      }
      o.text.blocks.clear();
      sink.n += o.text.n;
      if (sink.failed) return fail(-1, "the write callback failed");
      {
        std::lock_guard<std::mutex> lk(mu);
        written = k + 1;
      }
      cv.notify_all();
      if (k + 1 == nchunks) sink.write("\n]", 2);
    }
    if (sink.failed) return fail(-1, "the write callback failed");
    if (exit_code) *exit_code = anyfail ? 19 : parse_code;
    return 0;
  } catch (std::exception& e) {
    return fail(-1, e.what());
  }
}

// ------------------------------------------------------- streamed, every format and -i ---
// cfn_guard_validate_batch_stream_ex: the streamed entries with the whole structured contract of the
// one-string call -- output format (structured.rs:122-129: JSON / YAML through serde, SARIF sarif.rs:29-53,
// 127-160, JUnit xml.rs / reporters/mod.rs) and input parameters merged into every data file (validate.rs:317-350,
// structured.rs:51-65) -- over a device list.  JSON without parameters runs the streamed JSON paths above.
// Otherwise chunk k is loaded (host loader + merge when parameters are given, else the device loader),
// evaluated and -- for JSON / YAML, whose documents' texts simply concatenate -- rendered on pipeline k % ndev
// and written in order while later chunks run (host memory: two chunks' reports per device).  SARIF lists its
// artifacts (the FAILed documents' names) before every result and JUnit its totals before every suite, so
// those two hold every chunk's evaluated session on its device (≈20 GB of HBM per 1 M CFN templates, no report
// text) until the last is evaluated; then the frame goes out and each chunk's results / suites follow in
// order, each session released once written.  Errors: the one-string call's error precedence -- a data file
// that does not load (in order) before a parameter-file error, a merge panic, an erroring tile or an aborting
// report -- so on any other failure the documents after the failing chunk are load-checked first.  JSON /
// YAML write the chunks before the failing one (the caller drops that prefix); SARIF / JUnit write nothing.
namespace {
// the first document of [from, n) the host loader rejects, scanned on the host threads
bool first_load_error(const validate_input_t* docs, size_t from, size_t n, std::string& kind, std::string& msg) {
  if (from >= n) return false;
  const size_t nt = std::max<size_t>(1, std::min<size_t>(report_threads(), (n - from) / 256 + 1));
  std::vector<size_t> at(nt, SIZE_MAX);
  std::vector<LoadError> les(nt);
  parallel_run(nt, [&](size_t w) {
    const size_t a = from + (n - from) * w / nt, b = from + (n - from) * (w + 1) / nt;
    for (size_t i = a; i < b; i++) {
      DocBatch tmp;
      const char* t = docs[i].content ? docs[i].content : "";
      if (!load_document(tmp, t, strlen(t), docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, les[w])) { at[w] = i; return; }
    }
  });
  for (size_t w = 0; w < nt; w++)
    if (at[w] != SIZE_MAX) { kind = les[w].kind; msg = les[w].msg; return true; }
  return false;
}

// stream_chunk_session with input parameters: documents on the host loader, each merged with them; a merge
// panic is returned as the chunk's error (panic = true) unless a later document of the chunk does not load
std::unique_ptr<gg_session> stream_chunk_session_params(int dev, const validate_input_t* docs, size_t n_docs,
                                                        const validate_input_t* rules, size_t n_rules, const DocBatch* params,
                                                        size_t first, size_t count, std::string& kind, std::string& msg,
                                                        bool& panic) {
  panic = false;
  if (!params) return stream_chunk_session(dev, docs, n_docs, rules, n_rules, first, count, kind, msg);
  std::unique_ptr<gg_session> ses(new gg_session());
  ses->device = dev;
  ses->defer_recs = true;
  for (size_t i = 0; i < n_rules; i++) {
    std::string perr;
    const std::string name = rules[i].file_name ? rules[i].file_name : "";
    if (!add_rules(ses.get(), rules[i].content ? rules[i].content : "", name, perr))
      ses->parse_errors.push_back("Parsing error handling rule file = " + name + ", Error = " + error_display("ParseError", perr) + "\n---");
  }
  LoadError pan;
  bool panicked = false;
  for (size_t i = first; i < first + count; i++) {
    LoadError le;
    const char* t = docs[i].content ? docs[i].content : "";
    if (!load_document(ses->docs, t, strlen(t), docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, le)) {
      kind = le.kind; msg = le.msg;
      return ses;
    }
    if (!panicked && !merge_params_last(ses->docs, params, pan)) panicked = true;
  }
  if (panicked) { kind = pan.kind; msg = pan.msg; panic = true; return ses; }
  if (ses->progs.empty()) {
    ses->tiles.clear(); ses->rule_status.clear(); ses->recs.clear(); ses->evaluated = true;
  } else {
    session_upload(ses.get());
    session_run(ses.get(), true);
  }
  return ses;
}

// the first erroring tile of an evaluated chunk (false + re), and whether any rules file FAILed
bool chunk_tiles(gg_session* s, ReportError& re, bool& anyfail) {
  const size_t nf = s->progs.size(), nd = s->docs.ndocs();
  for (size_t t = 0; t < nd * nf; t++) {
    if (s->tiles[t].err) {
      ensure_host_arena(s);
      std::vector<const Program*> progs;
      for (auto& p : s->progs) progs.push_back(&p->prog);
      tile_error(s->docs, (uint32_t)(t / nf), *progs[t % nf], s->tiles[t], re);
      return false;
    }
    if (s->tiles[t].status == ST_FAIL) anyfail = true;
  }
  return true;
}

int32_t stream_format(const std::vector<int>& devs, const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                      size_t n_rules, const validate_input_t* params, size_t n_params, int32_t fmt, size_t chunk_docs,
                      cfn_guard_write_fn write, void* ctx, int32_t* exit_code, extern_err_t* err) {
  auto fail = [&](int32_t code, const std::string& msg) { set_err(err, code, msg); if (exit_code) *exit_code = -1; return -1; };
  try {
    std::unique_ptr<DocBatch> pbatch;
    LoadError pe;
    if (!load_params(params, n_params, pbatch, pe)) {
      std::string k, m;
      if (first_load_error(docs, 0, n_docs, k, m)) return fail(ffi_code(k), error_display(k, m));
      return fail(ffi_code(pe.kind), error_display(pe.kind, pe.msg));
    }
    const bool hold = fmt == OUT_SARIF || fmt == OUT_JUNIT;
    const size_t ndev = devs.size();
    const size_t chunk = chunk_docs ? chunk_docs : (ndev > 1 ? (size_t)16384 : (size_t)262144);
    const size_t nchunks = (n_docs + chunk - 1) / chunk;
    PinnedPool pool;
    struct Out {
      int state = 0;          // 0 pending, 1 ready, 2 failed
      ChainSink text;
      std::unique_ptr<gg_session> ses;   // SARIF / JUnit: the evaluated chunk, until it is written
      explicit Out(PinnedPool& p) : text(p) {}
      bool anyfail = false, load_error = false;
      int32_t parse_code = 0;
      std::string kind, msg;
    };
    std::vector<std::unique_ptr<Out>> outs(nchunks);
    for (auto& o : outs) o.reset(new Out(pool));
    std::mutex mu;
    std::condition_variable cv;
    size_t written = 0;
    bool stop = false;
    std::vector<std::thread> pipes;
    for (size_t p = 0; p < std::min(ndev, nchunks); p++) {
      pipes.emplace_back([&, p]() {
        for (size_t k = p; k < nchunks; k += ndev) {
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || hold || k < 2 * ndev || written > k - 2 * ndev; });
            if (stop) return;
          }
          Out& o = *outs[k];
          std::string kind, msg;
          bool load_error = false;
          try {
            HIPCHK(hipSetDevice(devs[p]));
            const size_t first = k * chunk, count = std::min(chunk, n_docs - first);
            bool panic = false;
            std::unique_ptr<gg_session> ses =
                stream_chunk_session_params(devs[p], docs, n_docs, rules, n_rules, pbatch.get(), first, count, kind, msg, panic);
            load_error = !kind.empty() && !panic;
            if (kind.empty()) {
              o.parse_code = ses->parse_errors.empty() ? 0 : 5;
              ReportError re;
              if (fmt == OUT_JSON) {
                if (!stream_chunk_report(ses.get(), k, o.text, re, o.anyfail)) { kind = re.kind; msg = re.msg; }
              } else if (!chunk_tiles(ses.get(), re, o.anyfail)) {
                kind = re.kind; msg = re.msg;
              } else if (hold) {
                o.ses = std::move(ses);
              } else {
                // YAML: a chunk's block-sequence items; the chunks' streams concatenate
                std::string out;
                int32_t code = 0;
                if (!session_report(ses.get(), out, code, re, OUT_YAML)) { kind = re.kind; msg = re.msg; }
                else o.text.write(out.data(), out.size());
              }
            }
          } catch (std::exception& e) { kind = "Internal"; msg = e.what(); }
          {
            std::lock_guard<std::mutex> lk(mu);
            o.kind = kind; o.msg = msg; o.load_error = load_error;
            o.state = kind.empty() ? 1 : 2;
          }
          cv.notify_all();
          if (!kind.empty()) return;
        }
      });
    }
    struct JoinAll {
      std::vector<std::thread>& v; std::mutex& mu; std::condition_variable& cv; bool& stop;
      ~JoinAll() { { std::lock_guard<std::mutex> lk(mu); stop = true; } cv.notify_all(); for (auto& t : v) if (t.joinable()) t.join(); }
    } join{pipes, mu, cv, stop};
    char* stage = (char*)pinned_get(DeviceBufs::kPinnedBytes, devs[0]);
    if (!stage) throw std::runtime_error("pinned host staging: allocation failed");
    struct StageFree { char* p; int d; ~StageFree() { pinned_put(p, DeviceBufs::kPinnedBytes, d); } } stage_free{stage, devs[0]};
    CallbackSink sink(write, ctx, stage, DeviceBufs::kPinnedBytes);
    auto wait_chunk = [&](size_t k) -> Out& {
      Out& o = *outs[k];
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return o.state != 0; });
      return o;
    };
    // chunk k failed: a document after it that does not load takes precedence (unless k's error is one)
    auto fail_chunk = [&](size_t k, Out& o) {
      if (!o.load_error) {
        std::string lk, lm;
        if (o.kind != "Internal" && first_load_error(docs, std::min(n_docs, (k + 1) * chunk), n_docs, lk, lm))
          return fail(ffi_code(lk), error_display(lk, lm));
      }
      return fail(ffi_code(o.kind), error_display(o.kind, o.msg));
    };
    int32_t parse_code = 0;
    bool anyfail = false;
    if (!n_docs) {
      // no documents: the format's empty report (exit 5 when a rules file does not parse)
      gg_session rs;
      for (size_t i = 0; i < n_rules; i++) {
        std::string perr;
        if (!add_rules(&rs, rules[i].content ? rules[i].content : "", rules[i].file_name ? rules[i].file_name : "", perr))
          rs.parse_errors.push_back(perr);
      }
      std::string out;
      int32_t code = 0;
      ReportError re;
      if (!session_report(&rs, out, code, re, fmt)) return fail(ffi_code(re.kind), error_display(re.kind, re.msg));
      sink.write(out.data(), out.size());
      if (sink.failed) return fail(-1, "the write callback failed");
      if (exit_code) *exit_code = code;
      return 0;
    }
    if (!hold) {
      for (size_t k = 0; k < nchunks; k++) {
        Out& o = wait_chunk(k);
        if (o.state == 2) return fail_chunk(k, o);
        if (k == 0) { parse_code = o.parse_code; if (fmt == OUT_JSON) sink.write("[\n", 2); }
        anyfail = anyfail || o.anyfail;
        for (auto& b : o.text.blocks) {
          if (!sink.failed && b.second && write(ctx, b.first, b.second) != 0) sink.failed = true;
          pool.put(b.first);
        }
        o.text.blocks.clear();
        sink.n += o.text.n;
        if (sink.failed) return fail(-1, "the write callback failed");
        {
          std::lock_guard<std::mutex> lk(mu);
          written = k + 1;
        }
        cv.notify_all();
      }
      if (fmt == OUT_JSON) sink.write("\n]", 2);
    } else {
      // every chunk evaluated (or the first failure, in order) before a byte is written
      for (size_t k = 0; k < nchunks; k++) {
        Out& o = wait_chunk(k);
        if (o.state == 2) return fail_chunk(k, o);
        anyfail = anyfail || o.anyfail;
      }
      parse_code = outs[0]->parse_code;
      if (fmt == OUT_SARIF) {
        // SarifReport::new (sarif.rs:29-53, 185-203): the FAILed documents' first-seen non-empty names
        std::vector<std::string> art;
        std::unordered_set<std::string> seen;
        for (auto& op : outs) {
          gg_session* s = op->ses.get();
          const size_t nf = s->progs.size();
          for (size_t d = 0; d < s->docs.ndocs(); d++) {
            uint32_t status = ST_SKIP;
            for (size_t f = 0; f < nf; f++) {
              const uint32_t st = s->tiles[d * nf + f].status;   // Status::and (rules/mod.rs:122-133)
              if (status == ST_FAIL) continue;
              status = status == ST_PASS ? (st == ST_FAIL ? ST_FAIL : ST_PASS) : st;
            }
            if (status != ST_FAIL) continue;
            const std::string& name = s->docs.names[d];
            if (!name.empty() && seen.insert(name).second) art.push_back(name);
          }
        }
        std::string head, tail;
        sarif_frame(art, head, tail);
        sink.write(head.data(), head.size());
        // the results' first comma is dropped ("[\n        {" as serde's pretty printer writes it)
        struct DropFirst : ReportSink {
          ReportSink& in;
          char* last = nullptr;
          uint64_t n = 0;
          explicit DropFirst(ReportSink& s) : in(s) {}
          char* reserve(size_t k) override { return last = in.reserve(k); }
          void commit(size_t k) override {
            if (!k) return;
            if (n == 0) { memmove(last, last + 1, k - 1); in.commit(k - 1); }
            else in.commit(k);
            n += k;
          }
          size_t max_piece() const override { return in.max_piece(); }
          bool pinned() const override { return in.pinned(); }
        } results(sink);
        for (auto& op : outs) {
          gg_session* s = op->ses.get();
          ReportError re;
          if (!s->progs.empty()) {
            if (device_report_on(s) && s->fetched_on_device) {
              if (!device_report_text(s, 0, s->docs.ndocs(), SIZE_MAX, results, re, nullptr, OUT_SARIF, kStreamPushBlocks))
                return fail(ffi_code(re.kind), error_display(re.kind, re.msg));
            } else {
              ensure_host_arena(s);
              std::vector<const Program*> progs;
              for (auto& p : s->progs) progs.push_back(&p->prog);
              const size_t nf = progs.size();
              for (size_t d = 0; d < s->docs.ndocs(); d++) {
                std::vector<TileResult> trs(nf);
                std::vector<const TileResult*> tp(nf);
                for (size_t f = 0; f < nf; f++) {
                  trs[f] = tile_view(s->tiles.data(), s->rule_status.data(), s->max_top, s->recs.data(), d * nf + f);
                  tp[f] = &trs[f];
                }
                std::string t;
                if (!sarif_doc_results(s->docs, (uint32_t)d, progs, tp, t, re)) return fail(ffi_code(re.kind), error_display(re.kind, re.msg));
                results.write(t.data(), t.size());
              }
            }
          }
          if (sink.failed) return fail(-1, "the write callback failed");
          op->ses.reset();
        }
        if (results.n) sink.write("\n      ", 7);
        sink.write(tail.data(), tail.size());
      } else {
        // JunitReporter (xml.rs:14-80): the totals -- one test per (data file, rules file), a failure per FAILed
        // one -- then every chunk's test suites (its own report without the frame)
        size_t tests = 0, failures = 0;
        for (auto& op : outs) {
          gg_session* s = op->ses.get();
          const size_t nf = s->progs.size();
          tests += s->docs.ndocs() * nf;
          for (size_t t = 0; t < s->docs.ndocs() * nf; t++) failures += s->tiles[t].status == ST_FAIL;
        }
        const std::string head = "<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<testsuites name=\"cfn-guard validate report\" tests=\"" +
                                 std::to_string(tests) + "\" failures=\"" + std::to_string(failures) + "\" errors=\"0\" time=\"0\">\n";
        static const char kTail[] = "</testsuites>\n";
        sink.write(head.data(), head.size());
        for (auto& op : outs) {
          std::string out;
          int32_t code = 0;
          ReportError re;
          if (!session_report(op->ses.get(), out, code, re, OUT_JUNIT)) return fail(ffi_code(re.kind), error_display(re.kind, re.msg));
          size_t a = out.find('\n');
          a = a == std::string::npos ? out.size() : out.find('\n', a + 1);
          a = a == std::string::npos ? out.size() : a + 1;
          const size_t tl = sizeof(kTail) - 1;
          const size_t b = out.size() >= a + tl && out.compare(out.size() - tl, tl, kTail) == 0 ? out.size() - tl : out.size();
          if (b > a) sink.write(out.data() + a, b - a);
          if (sink.failed) return fail(-1, "the write callback failed");
          op->ses.reset();
        }
        sink.write(kTail, sizeof(kTail) - 1);
      }
    }
    if (sink.failed) return fail(-1, "the write callback failed");
    // exit code 19 on a FAIL; JUnit keeps 5 over 19 (reporters/mod.rs:97-103)
    int32_t code = parse_code;
    if (anyfail && !(fmt == OUT_JUNIT && parse_code == 5)) code = 19;
    if (exit_code) *exit_code = code;
    return 0;
  } catch (std::exception& e) {
    return fail(-1, e.what());
  }
}
}  // namespace

int32_t cfn_guard_validate_batch_stream_ex(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                           size_t n_rules, const validate_input_t* params, size_t n_params,
                                           int32_t output_format, size_t chunk_docs, const int32_t* devices, size_t n_devices,
                                           cfn_guard_write_fn write, void* ctx, int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (exit_code) *exit_code = 0;
  auto fail = [&](int32_t code, const std::string& msg) { set_err(err, code, msg); if (exit_code) *exit_code = -1; return -1; };
  if (!write) return fail(18, "IllegalArguments: no write callback");
  if (output_format < OUT_JSON || output_format > OUT_JUNIT) return fail(18, "IllegalArguments: unknown output format");
  try {
    std::string why;
    std::vector<int> devs;
    if (devices) {
      for (size_t i = 0; i < n_devices; i++) devs.push_back(devices[i]);
      if (devs.empty()) return fail(-1, "IllegalArguments: an empty device list");
      for (int d : devs)
        if (!ensure_device(why, d)) return fail(-1, why);
    } else {
      int d = 0;
      if (!ensure_device(why, -1, &d)) return fail(-1, why);
      devs.push_back(d);
    }
    if (output_format == OUT_JSON && !n_params) {
      if (devs.size() == 1) return stream_single(devs[0], docs, n_docs, rules, n_rules, chunk_docs, write, ctx, exit_code, err);
      return cfn_guard_validate_batch_stream_devices(docs, n_docs, rules, n_rules, chunk_docs, devs.data(), devs.size(), write, ctx,
                                                     exit_code, err);
    }
    return stream_format(devs, docs, n_docs, rules, n_rules, params, n_params, output_format, chunk_docs, write, ctx, exit_code, err);
  } catch (std::exception& e) {
    return fail(-1, e.what());
  }
}

// synthetic corpora as validate inputs (bench.py's streamed end-to-end job): texts generated on host threads
struct gg_texts {
  std::vector<std::string> text, name;
  std::vector<validate_input_t> in;
};
gg_texts* gg_synth_texts(uint64_t first, size_t n, int32_t n_resources, int32_t format, int32_t nthreads) {
  gg_texts* t = new gg_texts();
  t->text.resize(n); t->name.resize(n); t->in.resize(n);
  if (nthreads < 1) nthreads = 1;
  parallel_run((size_t)nthreads, [&](size_t th) {
    for (size_t i = n * th / nthreads; i < n * (th + 1) / nthreads; i++) {
      if (format == 1) cfn_synth_yaml_doc(first + i, n_resources, t->text[i]);
      else cfn_synth_doc(first + i, n_resources, t->text[i]);
      t->name[i] = "synthetic-" + std::to_string(first + i) + (format == 1 ? ".yaml" : ".json");
    }
  });
  for (size_t i = 0; i < n; i++) { t->in[i].content = t->text[i].c_str(); t->in[i].file_name = t->name[i].c_str(); }
  return t;
}
const validate_input_t* gg_texts_inputs(gg_texts* t) { return t ? t->in.data() : nullptr; }
void gg_texts_free(gg_texts* t) { delete t; }

char* cfn_guard_validate_batch_devices(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                       size_t n_rules, const validate_input_t* params, size_t n_params,
                                       int32_t output_format, const int32_t* devices, size_t n_devices, int32_t* exit_code,
                                       extern_err_t* err) {
  set_err(err, 0, "");
  if (exit_code) *exit_code = 0;
  if (output_format < OUT_JSON || output_format > OUT_JUNIT) {
    set_err(err, 18, "IllegalArguments: unknown output format");
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
  try {
    std::vector<int> devs;
    std::string why;
    if (devices) {
      for (size_t i = 0; i < n_devices; i++) devs.push_back(devices[i]);
    } else {
      int n = 0;
      if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
      for (int d = 0; d < n; d++) devs.push_back(d);
    }
    if (devs.empty()) { set_err(err, -1, devices ? "IllegalArguments: an empty device list" : "no HIP device available (the MI355X path has no CPU fallback)"); if (exit_code) *exit_code = -1; return nullptr; }
    for (int d : devs)
      if (!ensure_device(why, d)) { set_err(err, -1, why); if (exit_code) *exit_code = -1; return nullptr; }
    return validate_batch_devices(docs, n_docs, rules, n_rules, params, n_params, output_format, devs, exit_code, err);
  } catch (std::exception& e) {
    set_err(err, -1, e.what());
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
}

char* cfn_guard_validate_batch_gpus(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                    size_t n_rules, int32_t output_format, int32_t n_gpus, int32_t* exit_code,
                                    extern_err_t* err) {
  if (n_gpus <= 0)
    return cfn_guard_validate_batch_devices(docs, n_docs, rules, n_rules, nullptr, 0, output_format, nullptr, 0, exit_code, err);
  std::vector<int32_t> devs(n_gpus);
  for (int32_t d = 0; d < n_gpus; d++) devs[d] = d;
  return cfn_guard_validate_batch_devices(docs, n_docs, rules, n_rules, nullptr, 0, output_format, devs.data(), devs.size(),
                                          exit_code, err);
}

/* host-only (tests): shard_by_bytes -- starts[0..nshards] of contiguous byte-balanced document ranges */
int32_t gg_shard_by_bytes(const size_t* lens, size_t n, size_t nshards, size_t* starts) {
  if (!nshards || !starts) return -1;
  shard_by_bytes(lens, n, nshards, starts);
  return 0;
}

/* the structured report of a fetched session rendered as the shards [cuts[k], cuts[k+1]) and joined by
 * shards_report -- the multi-device join on one session's results (CPU tests, with loaded results) */
char* gg_session_report_shards(gg_session* s, int32_t output_format, const size_t* cuts, size_t ncuts, int32_t* exit_code,
                               extern_err_t* err) {
  set_err(err, 0, "");
  if (!s->evaluated) { set_err(err, -1, "session not evaluated"); return nullptr; }
  try {
    std::vector<ShardView> v;
    size_t prev = 0;
    for (size_t k = 0; k <= ncuts; k++) {
      const size_t c = k < ncuts ? std::min(cuts[k], s->docs.ndocs()) : s->docs.ndocs();
      if (c < prev) { set_err(err, 18, "IllegalArguments: cuts must not decrease"); return nullptr; }
      v.push_back(ShardView{s, prev, c - prev});
      prev = c;
    }
    std::string out;
    char* cs = nullptr;
    int32_t code = 0;
    ReportError re;
    if (!shards_report(v, out, code, re, output_format, &cs)) {
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      if (exit_code) *exit_code = -1;
      return nullptr;
    }
    if (exit_code) *exit_code = code;
    return cs ? cs : dup_str(out);
  } catch (std::exception& e) { set_err(err, -1, e.what()); return nullptr; }
}

// ---------------------------------------------------------------- validate (console) ---
// `cfn-guard validate [-r]+ [-d]+ [-i]* [-o single-line-summary|json|yaml] [-S ...] [--verbose]
// [--print-json]` without --structured (commands/validate.rs:253-487, 552-596, 690-758).  Every pair is
// evaluated twice on the device -- the throughput kernels (the FileReport the CFN / Terraform reporters
// and -o json / yaml read) and the verbose kernel (the EventRecord tree the summary table, the generic
// reporter, --verbose and --print-json read) -- then reported rules file by rules file, data file by
// data file.  An evaluation error ends the output where the reference's `?` does.
char* cfn_guard_validate_console(const validate_input_t* docs, size_t n_docs, const validate_input_t* rules,
                                 size_t n_rules, const validate_input_t* params, size_t n_params, uint32_t show_summary,
                                 int32_t output_format, uint32_t flags, int32_t* exit_code, char** err_text,
                                 extern_err_t* err) {
  set_err(err, 0, "");
  if (err_text) *err_text = nullptr;
  if (exit_code) *exit_code = 0;
  // validate_construct (validate.rs:203-232): junit / sarif need --structured
  if (output_format != OUT_TEXT && output_format != OUT_JSON && output_format != OUT_YAML) {
    set_err(err, 18, error_display("IllegalArguments", "the structured flag must be set when output is set to junit or sarif"));
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
  std::string out, errs;
  auto finish = [&](int32_t code) -> char* {
    if (exit_code) *exit_code = code;
    if (err_text && !errs.empty()) *err_text = dup_str(errs);
    return dup_str(out);
  };
  try {
    std::string why;
    if (!ensure_device(why)) { set_err(err, -1, why); if (exit_code) *exit_code = -1; return nullptr; }
    gg_session s;
    // data files first (validate.rs:274-315), then the parameter files (317-350): a failure aborts
    // before anything is evaluated
    std::vector<std::string> texts;
    for (size_t i = 0; i < n_docs; i++) {
      LoadError le;
      const char* t = docs[i].content ? docs[i].content : "";
      if (!load_document(s.docs, t, strlen(t), docs[i].file_name ? docs[i].file_name : "", LOAD_LIBYAML, le)) {
        set_err(err, ffi_code(le.kind), error_display(le.kind, le.msg));
        if (exit_code) *exit_code = -1;
        return nullptr;
      }
      texts.emplace_back(t);
    }
    LoadError pe;
    if (!load_params(params, n_params, s.params, pe)) {
      set_err(err, ffi_code(pe.kind), error_display(pe.kind, pe.msg));
      if (exit_code) *exit_code = -1;
      return nullptr;
    }
    // evaluate_against_data_input merges per data file (`data.clone().merge(file)?`): the first data file
    // whose merge fails ends the run there, in the first rules file that is evaluated
    size_t ndocs = s.docs.ndocs();
    LoadError merge_err;
    bool merge_failed = false;
    if (s.params) {
      DocBatch merged;
      for (size_t d = 0; d < s.docs.ndocs() && !merge_failed; d++) {
        // re-append document d alone, then merge the parameters into it
        DocBatch one;
        LoadError le;
        const char* t = texts[d].c_str();
        load_document(one, t, texts[d].size(), s.docs.names[d], LOAD_LIBYAML, le);
        merge_batch(merged, one);
        if (!merge_into_last(merged, merged.ndocs() - 1, *s.params, 0, merge_err)) { merge_failed = true; ndocs = d; }
      }
      if (merge_failed) { merged.roots.pop_back(); merged.base.pop_back(); merged.names.pop_back(); }
      s.docs = std::move(merged);
    }
    // rules files in order: a parse error goes to stderr with exit code 5 (evaluate_rule, 563-572)
    std::vector<int> entry;   // program index, -1 parse error, -2 empty rules file
    for (size_t i = 0; i < n_rules; i++) {
      const std::string name = rules[i].file_name ? rules[i].file_name : "";
      const std::string text = rules[i].content ? rules[i].content : "";
      RulesFile rf;
      bool empty = false;
      std::string perr;
      bool ok = parse_rules_file(text, name, rf, empty, perr);
      if (ok && !empty) {
        auto gp = std::make_unique<GpuProgram>();
        ok = compile_program(rf, name, gp->prog, perr);
        if (ok) { entry.push_back((int)s.progs.size()); s.progs.push_back(std::move(gp)); continue; }
      }
      if (!ok) {
        errs += "Parsing error handling rule file = " + name + ", Error = " + error_display("ParseError", perr) + "\n---\n";
        entry.push_back(-1);
      } else {
        entry.push_back(-2);
      }
    }
    const size_t nf = s.progs.size();
    std::vector<TileOut> tiles;
    std::vector<uint8_t> rstat;
    std::vector<Rec> recs;
    if (nf && s.docs.ndocs()) {
      session_upload(&s);
      session_run(&s, true);
      tiles.swap(s.tiles); rstat.swap(s.rule_status); recs.swap(s.recs);
      s.mode = 1; s.verbose = true;   // the same batch again through the verbose kernel
      session_run(&s, true);
    }
    ConsoleOptions opt;
    opt.summary = show_summary;
    opt.format = output_format;
    opt.verbose = (flags & 1u) != 0;
    opt.print_json = (flags & 2u) != 0;
    int32_t code = 0;
    bool first_eval = true;
    for (int e : entry) {
      if (e == -1) { code = 5; continue; }
      if (e == -2) continue;
      bool fail = false;
      for (size_t d = 0; d < ndocs; d++) {
        const size_t t = d * nf + (size_t)e;
        TileResult tr = tile_view(tiles.data(), rstat.data(), s.max_top, recs.data(), t);
        TileResult vr = tile_view(s.tiles.data(), s.rule_status.data(), s.max_top, s.recs.data(), t);
        ReportError re;
        if (!console_report(s.docs, (uint32_t)d, texts[d], s.progs[e]->prog, tr, vr, opt, out, re)) {
          set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
          errs += "Error occurred " + error_display(re.kind, re.msg);
          return finish(-1);
        }
        if (tr.out.status == ST_FAIL) fail = true;
      }
      if (merge_failed && first_eval) {
        set_err(err, ffi_code(merge_err.kind), error_display(merge_err.kind, merge_err.msg));
        errs += "Error occurred " + error_display(merge_err.kind, merge_err.msg);
        return finish(-1);
      }
      first_eval = false;
      if (fail) code = 19;
    }
    return finish(code);
  } catch (std::exception& e) {
    set_err(err, -1, e.what());
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
}

// ---------------------------------------------------------------- cfn-guard test ---
namespace {

const DNode* map_entry(const DocBatch& D, uint64_t base, const DNode& m, const char* key) {
  if (m.kind != K_MAP) return nullptr;
  const size_t kl = strlen(key);
  for (uint32_t j = 0; j < m.count; j++) {
    const DNode& e = D.nodes[base + m.a + j];
    if (e.key_len == kl && memcmp(D.bytes.data() + e.key_off, key, kl) == 0) return &e;
  }
  return nullptr;
}

std::string node_str(const DocBatch& D, const DNode& n) { return std::string(D.bytes.data() + n.a, n.count); }

struct SpecCase { bool has_name; std::string name; uint32_t input; std::vector<std::pair<std::string, std::string>> expected; };

// Vec<TestSpec> (commands/test.rs:480-484) out of a loaded spec document; false + message on a shape error
bool read_spec(const DocBatch& D, size_t doc, std::vector<SpecCase>& out, std::string& why) {
  const uint64_t base = D.base[doc];
  const DNode& root = D.nodes[base + D.roots[doc]];
  if (root.kind != K_LIST) { why = "invalid type: expected a sequence"; return false; }
  for (uint32_t i = 0; i < root.count; i++) {
    const uint32_t ci = root.a + i;
    const DNode& c = D.nodes[base + ci];
    if (c.kind != K_MAP) { why = "invalid type: expected struct TestSpec"; return false; }
    const DNode* name = map_entry(D, base, c, "name");
    const DNode* input = map_entry(D, base, c, "input");
    const DNode* exp = map_entry(D, base, c, "expectations");
    if (!input) { why = "missing field `input`"; return false; }
    if (!exp) { why = "missing field `expectations`"; return false; }
    const DNode* rules = map_entry(D, base, *exp, "rules");
    if (!rules) { why = "missing field `rules`"; return false; }
    SpecCase sc;
    sc.has_name = name && name->kind == K_STRING;
    if (sc.has_name) sc.name = node_str(D, *name);
    sc.input = (uint32_t)(input - &D.nodes[base]);
    if (rules->kind == K_MAP) {
      for (uint32_t j = 0; j < rules->count; j++) {
        const DNode& e = D.nodes[base + rules->a + j];
        if (e.kind != K_STRING) { why = "invalid type: expected a string"; return false; }
        sc.expected.push_back({std::string(D.bytes.data() + e.key_off, e.key_len), node_str(D, e)});
      }
    }
    out.push_back(std::move(sc));
  }
  return true;
}

int32_t status_of(const std::string& s) { return s == "PASS" ? (int32_t)ST_PASS : s == "FAIL" ? (int32_t)ST_FAIL : s == "SKIP" ? (int32_t)ST_SKIP : -1; }

}  // namespace

namespace {
// One rules file's `cfn-guard test` run on the MI355X (StructuredTestReporter::evaluate /
// GenericReporter::report, reporters/test/*.rs): every spec's test cases in one batch, each test
// case a document whose root is its `input` subtree.  Returns 1 with the spec files' results, 2 for
// a rules file with no rules (Ok(None)), 3 for an unparsable one (perr), 0 for an aborting error (err set).
int run_test_file(const std::string& rname, const char* rtext, const validate_input_t* specs, size_t n_specs,
                  std::vector<TestSpecFile>& files, std::string& perr, extern_err_t* err, bool verbose = false) {
  gg_session s;
  if (!add_rules(&s, rtext, rname, perr)) return 3;
  if (s.progs.empty()) return 2;
  if (verbose) { s.mode = 1; s.verbose = true; }   // every event recorded (the verbose wave kernel)
  files.assign(n_specs, TestSpecFile());
  std::vector<std::vector<SpecCase>> cases(n_specs);
  std::vector<std::pair<size_t, size_t>> tile_of;   // (spec, case) of each evaluated document
  DocBatch& D = s.docs;
  for (size_t k = 0; k < n_specs; k++) {
    const char* t = specs[k].content ? specs[k].content : "";
    const std::string path = specs[k].file_name ? specs[k].file_name : "";
    LoadError le;
    std::string shape;
    const size_t at = D.ndocs();
    bool ok = load_document(D, t, strlen(t), path, LOAD_SERDE, le);
    if (ok && !read_spec(D, at, cases[k], shape)) { ok = false; le.msg = shape; }
    if (!ok) {
      files[k].error = error_display("ParseError", "Unable to process data in file " + path + ", Error " + le.msg + ",");
      if (D.ndocs() > at) { D.roots.pop_back(); D.base.pop_back(); D.names.pop_back(); }
      continue;
    }
    // the spec document itself is not evaluated: one document per test case, rooted at its input,
    // whose paths start at that input (PathAwareValue::try_from(spec.input), generic.rs:75)
    const uint64_t base = D.base[at];
    D.roots.pop_back(); D.base.pop_back(); D.names.pop_back();
    for (size_t c = 0; c < cases[k].size(); c++) D.nodes[base + cases[k][c].input].parent = NONE;
    for (size_t c = 0; c < cases[k].size(); c++) {
      D.roots.push_back(cases[k][c].input);
      D.base.push_back(base);
      D.names.push_back(path);
      tile_of.push_back({k, c});
    }
  }
  if (!s.progs.empty() && D.ndocs()) {
    session_upload(&s);
    session_run(&s, true);
  }
  const Program* P = s.progs.empty() ? nullptr : &s.progs[0]->prog;
  for (size_t d = 0; d < tile_of.size(); d++) {
    const size_t k = tile_of[d].first, c = tile_of[d].second;
    const SpecCase& sc = cases[k][c];
    TestCaseResult tc;
    tc.has_name = sc.has_name;
    tc.name = sc.name;
    if (P) {
      const TileOut& to = s.tiles[d];
      if (to.err) {   // an evaluation error aborts the command (eval_rules_file(..)?)
        ReportError re;
        tile_error(D, (uint32_t)d, *P, to, re);
        set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
        return 0;
      }
      // get_by_rules (reporters/test/mod.rs:7-18): top-level rule records grouped by name
      std::vector<std::string> order;
      std::vector<std::vector<uint32_t>> got;
      for (uint32_t r = 0; r < P->n_rules; r++) {
        const std::string& nm = P->rule_names[P->rule_names.size() - P->n_rules + r];
        size_t g = std::find(order.begin(), order.end(), nm) - order.begin();
        if (g == order.size()) { order.push_back(nm); got.emplace_back(); }
        got[g].push_back(s.rule_status[d * s.max_top + r]);
      }
      for (size_t g = 0; g < order.size(); g++) {
        TestRuleResult rr;
        rr.rule = order[g];
        auto it = std::find_if(sc.expected.begin(), sc.expected.end(), [&](const std::pair<std::string, std::string>& e) { return e.first == order[g]; });
        if (it != sc.expected.end()) {
          rr.expected = status_of(it->second);
          if (rr.expected < 0) {
            set_err(err, 5, error_display("ParseError", "Unable to parse status " + it->second));
            return 0;
          }
          // get_status_result (reporters/test/mod.rs:20-54)
          uint32_t all_skipped = 0;
          for (uint32_t st : got[g]) {
            if (rr.expected == (int32_t)ST_SKIP) { if (st == ST_SKIP) all_skipped++; }
            else if ((int32_t)st == rr.expected) { rr.matched = rr.expected; break; }
            rr.evaluated.push_back(st);
          }
          if (rr.matched < 0 && rr.expected == (int32_t)ST_SKIP && all_skipped == got[g].size()) rr.matched = ST_SKIP;
        }
        tc.rules.push_back(std::move(rr));
      }
      if (verbose) {
        ReportError re;
        TileResult tr = tile_view(s.tiles.data(), s.rule_status.data(), s.max_top, s.recs.data(), d);
        if (!verbose_text(D, (uint32_t)d, *P, tr, "", tc.tree, re)) {   // eval_rules_file(.., None): File(, ..)
          set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
          return 0;
        }
      }
    }
    files[k].cases.push_back(std::move(tc));
  }
  return 1;
}
}  // namespace

namespace {
// test.rs:134-141: --verbose with a structured output, SARIF, unknown formats -> IllegalArguments
bool test_args_ok(int32_t output_format, bool verbose, int32_t* exit_code, extern_err_t* err) {
  if (output_format != OUT_TEXT && output_format != OUT_JSON && output_format != OUT_YAML && output_format != OUT_JUNIT) {
    set_err(err, 18, output_format == OUT_SARIF ? "Cannot provide an output_type of SARIF, SARIF reporter is unsupported."
                                                 : "IllegalArguments: test reports are text, json, yaml or junit");
    if (exit_code) *exit_code = -1;
    return false;
  }
  if (verbose && output_format != OUT_TEXT) {
    set_err(err, 18, "Cannot provide an output_type of JSON, YAML, or JUnit while the verbose flag is set");
    if (exit_code) *exit_code = -1;
    return false;
  }
  return true;
}
}  // namespace

/* `cfn-guard test -r <rules> -t <spec files>` (test.rs:285-380). */
char* cfn_guard_test(validate_input_t rules, const validate_input_t* specs, size_t n_specs, int32_t output_format,
                     int32_t* exit_code, extern_err_t* err) {
  return cfn_guard_test_ex(rules, specs, n_specs, output_format, false, exit_code, err);
}

char* cfn_guard_test_ex(validate_input_t rules, const validate_input_t* specs, size_t n_specs, int32_t output_format,
                        bool verbose, int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (exit_code) *exit_code = 0;
  if (!test_args_ok(output_format, verbose, exit_code, err)) return nullptr;
  try {
    std::string why;
    if (!ensure_device(why)) { set_err(err, -1, why); if (exit_code) *exit_code = -1; return nullptr; }
    const std::string rname = rules.file_name ? rules.file_name : "";
    std::string perr;
    std::vector<TestSpecFile> files;
    const int r = run_test_file(rname, rules.content ? rules.content : "", specs, n_specs, files, perr, err, verbose);
    if (r == 0) { if (exit_code) *exit_code = -1; return nullptr; }
    if (r == 3) {
      // test.rs:300-303 (text): exit code 1; 338-350 (structured TestResult::Err): the report, and
      // handle_structured_single_report's exit_code stays SUCCESS_STATUS_CODE on that branch
      if (exit_code) *exit_code = output_format == OUT_TEXT ? 1 : 0;
      if (output_format == OUT_TEXT) return dup_str("Parse Error on ruleset file " + error_display("ParseError", perr) + "\n");
      std::vector<TestSpecFile> ef(1);
      ef[0].error = error_display("ParseError", perr);
      int32_t code = 0;
      return dup_str(test_report(output_format, rname, ef, code));
    }
    // a rules file with no rules (Ok(None)): nothing is written, exit code 0 (test.rs:315, 366)
    if (r == 2) return dup_str("");
    int32_t code = 0;
    std::string out = test_report(output_format, rname, files, code);
    if (exit_code) *exit_code = code;
    return dup_str(out);
  } catch (std::exception& e) {
    set_err(err, -1, e.what());
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
}

/* `cfn-guard test -d <dir>` (test.rs:143-165): rules file i with its spec_counts[i] spec files, which
 * follow each other in `specs`.  Text: handle_plaintext_directory (test.rs:221-283); json / yaml /
 * junit: handle_structured_directory_report (test.rs:383-456). */
char* cfn_guard_test_dir(const validate_input_t* rules, size_t n_rules, const validate_input_t* specs,
                         const size_t* spec_counts, int32_t output_format, bool verbose, int32_t* exit_code,
                         extern_err_t* err) {
  set_err(err, 0, "");
  if (exit_code) *exit_code = 0;
  if (!test_args_ok(output_format, verbose, exit_code, err)) return nullptr;
  try {
    std::string why;
    if (!ensure_device(why)) { set_err(err, -1, why); if (exit_code) *exit_code = -1; return nullptr; }
    std::string text;
    std::vector<TestResultIn> results;
    int32_t code = 0;
    size_t at = 0;
    for (size_t i = 0; i < n_rules; i++) {
      const std::string rname = rules[i].file_name ? rules[i].file_name : "";
      const size_t ns = spec_counts ? spec_counts[i] : 0;
      const validate_input_t* sp = specs + at;
      at += ns;
      if (!ns) {
        // structured: skipped silently (test.rs:395-397); text: a notice (:229-237)
        if (output_format == OUT_TEXT) text += "Guard File " + rname + " did not have any tests associated, skipping.\n---\n";
        continue;
      }
      if (output_format == OUT_TEXT) text += "Testing Guard File " + rname + "\n";
      std::string perr;
      TestResultIn tr;
      tr.rules_name = rname;
      const int r = run_test_file(rname, rules[i].content ? rules[i].content : "", sp, ns, tr.files, perr, err, verbose);
      if (r == 0) { if (exit_code) *exit_code = -1; return nullptr; }
      if (output_format == OUT_TEXT) {
        if (r == 3) { text += "Parse Error on ruleset file " + error_display("ParseError", perr) + "\n"; code = 7; }
        else if (r == 1) {
          int32_t c = 0;
          text += test_report(OUT_TEXT, rname, tr.files, c);
          if (code == 0) code = c;
        }
        text += "---\n";
        continue;
      }
      if (r == 2) continue;   // Ok(None): no TestResult
      if (r == 3) tr.parse_error = error_display("ParseError", perr);
      results.push_back(std::move(tr));
    }
    if (output_format != OUT_TEXT) text = test_report_list(output_format, results, code, false);
    if (exit_code) *exit_code = code;
    return dup_str(text);
  } catch (std::exception& e) {
    set_err(err, -1, e.what());
    if (exit_code) *exit_code = -1;
    return nullptr;
  }
}

// ------------------------------------------------------------- session API ---
gg_session* gg_session_new(void) { return new gg_session(); }
void gg_session_free(gg_session* s) { delete s; }

void gg_session_set_stream(gg_session* s, void* stream) { s->stream = (hipStream_t)stream; }

int32_t gg_session_set_device(gg_session* s, int32_t device) {
  if (s->dv || s->dev_nodes || device < -1) return -1;   // before anything is on a device
  s->device = device;
  return 0;
}

int32_t gg_session_configure(gg_session* s, int32_t mode, uint32_t lane_heap_bytes) {
  if (mode != 0 && mode != 1) return -1;
  if (lane_heap_bytes && lane_heap_bytes < 32 * 1024) return -1;   // frames + record staging + tables
  s->mode = mode;
  if (lane_heap_bytes) { s->lane_heap_bytes = lane_heap_bytes; s->lane_heap_set = lane_heap_bytes; }
  s->uploaded = false;
  return 0;
}

int32_t gg_session_set_option(gg_session* s, int32_t option, int64_t value) {
  switch (option) {
    case GG_OPT_RX_MEMO_PER_LAUNCH: s->rx_memo_per_launch = value != 0; return 0;
    case GG_OPT_DEFER_RECORDS: s->defer_recs = value != 0; return 0;
    default: return -1;
  }
}

int32_t gg_session_launch(gg_session* s, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why, s->device, &s->device)) { set_err(err, -1, why); return -1; }
    if (!s->uploaded) session_upload(s);
    // launch / fetch callers (multi-GPU: launch, all-reduce the tallies, fetch) get no second launch,
    // so the large-heap pass must exist from the first one: a tile that outgrows the wave heap is then
    // evaluated, not left with E_HEAP (session_run allocates it lazily and re-launches instead)
    if (!s->dv->d_big_heaps.p) s->dv->d_big_heaps.alloc((size_t)gg_session::kBigSlots * gg_session::kBigHeap);
    session_launch(s);
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

double gg_session_wait(gg_session* s, extern_err_t* err) {
  set_err(err, 0, "");
  std::string why;
  if (!ensure_device(why, s->device, &s->device)) { set_err(err, -1, why); return -1; }
  try { return session_wait(s); } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

int32_t gg_session_fetch(gg_session* s, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why, s->device, &s->device)) { set_err(err, -1, why); return -1; }
    session_wait(s);
    if (session_records_wanted(s) > s->rec_cap) { set_err(err, -1, "record arena overflow: run gg_session_eval first"); return -1; }
    session_fetch(s);
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

// The structured report rendered in blocks of documents and discarded (end-to-end measurement of
// the reporter at sizes whose text would not fit in memory): returns the bytes the report has.
int64_t gg_session_report_bytes(gg_session* s, int32_t output_format, size_t max_docs, int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (!s->evaluated) { set_err(err, -1, "session not evaluated"); return -1; }
  if (output_format != OUT_JSON && output_format != OUT_YAML) { set_err(err, 18, "IllegalArguments: json or yaml"); return -1; }
  try {
    ensure_host_arena(s);
    std::vector<const Program*> progs;
    for (auto& p : s->progs) progs.push_back(&p->prog);
    const size_t nf = progs.size(), nd = max_docs ? std::min(max_docs, s->docs.ndocs()) : s->docs.ndocs();
    for (size_t t = 0; t < s->tiles.size(); t++)
      if (s->tiles[t].err) {
        ReportError re;
        tile_error(s->docs, (uint32_t)(t / nf), *progs[t % nf], s->tiles[t], re);
        set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
        if (exit_code) *exit_code = -1;
        return -1;
      }
    auto tile = [&](size_t d, size_t f) {
      return tile_view(s->tiles.data(), s->rule_status.data(), s->max_top, s->recs.data(), d * nf + f);
    };
    const size_t kBlock = getenv("GG_REPORT_BLOCK") ? (size_t)std::max(1, atoi(getenv("GG_REPORT_BLOCK"))) : 65536;
    int64_t bytes = 0;
    std::string out;
    size_t json_parts = 0;   // JSON: the whole report is "[\n" + every block's parts joined by ",\n" + "\n]"
    std::vector<TextBuf> parts;   // reused across blocks, as a writer streaming to a file reuses its buffers
    for (size_t d0 = 0; d0 < nd; d0 += kBlock) {
      const size_t n = std::min(kBlock, nd - d0);
      ReportError re;
      bool ok;
      if (output_format == OUT_JSON) {
        ok = report_batch_json_parts(s->docs, progs, d0, n, tile, report_threads(), parts, re);
        for (auto& p : parts) bytes += (int64_t)p.size();
        json_parts += json_parts_count(parts);
      } else {
        ok = report_batch(s->docs, progs, d0, n, tile, output_format, report_threads(), out, re);
        bytes += (int64_t)out.size();
      }
      if (!ok) {
        set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
        if (exit_code) *exit_code = -1;
        return -1;
      }
      if (getenv("GG_PROGRESS")) fprintf(stderr, "[report] %zu / %zu documents, %lld bytes\n", d0 + n, nd, (long long)bytes);
    }
    if (output_format == OUT_JSON) bytes += json_parts ? (int64_t)(4 + 2 * (json_parts - 1)) : 2;
    bool anyfail = false;
    for (auto& t : s->tiles) if (t.status == ST_FAIL) anyfail = true;
    if (exit_code) *exit_code = anyfail ? 19 : (s->parse_errors.empty() ? 0 : 5);
    return bytes;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

size_t gg_session_ncounts(gg_session* s) { return s->ncounts; }
void* gg_session_counts_device(gg_session* s) { return s->ext_counts ? (void*)s->ext_counts : s->dv ? (void*)s->dv->d_counts.p : nullptr; }
int64_t gg_session_report_json_device(gg_session* s, size_t max_docs, int32_t* exit_code, double* stats, extern_err_t* err) {
  set_err(err, 0, "");
  if (!s->evaluated || !s->fetched_on_device) { set_err(err, -1, "session not evaluated and fetched on a device"); return -1; }
  try {
    std::vector<const Program*> progs;
    for (auto& p : s->progs) progs.push_back(&p->prog);
    const size_t nf = progs.size(), nd = max_docs ? std::min(max_docs, s->docs.ndocs()) : s->docs.ndocs();
    for (size_t t = 0; t < nd * nf; t++)
      if (s->tiles[t].err) {
        ensure_host_arena(s);
        ReportError re;
        tile_error(s->docs, (uint32_t)(t / nf), *progs[t % nf], s->tiles[t], re);
        set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
        if (exit_code) *exit_code = -1;
        return -1;
      }
    bind_device(s);
    render_tables(s);
    CountingSink sink(s->dv->pinned, DeviceBufs::kPinnedBytes);
    DevReportStats st;
    ReportError re;
    if (!device_report_json(s, 0, nd, 0, sink, re, &st)) {
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      if (exit_code) *exit_code = -1;
      return -1;
    }
    const int64_t bytes = (int64_t)sink.n + (nd ? 4 : 2);   // "[\n" ... "\n]" or "[]"
    bool anyfail = false;
    for (size_t t = 0; t < nd * nf; t++) if (s->tiles[t].status == ST_FAIL) anyfail = true;
    if (exit_code) *exit_code = anyfail ? 19 : (s->parse_errors.empty() ? 0 : 5);
    if (stats) {
      stats[0] = (double)st.device_docs; stats[1] = (double)st.host_docs; stats[2] = st.size_ms; stats[3] = st.write_ms;
      stats[4] = st.d2h_ms; stats[5] = st.host_ms; stats[6] = (double)st.bytes; stats[7] = 0;
    }
    return bytes;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

// The SARIF report of the first max_docs documents (0: all): the artifact list and frame on the host, every
// FAILed document's results rendered on the device (report_sarif_kernel), copied to host memory and dropped
// (measurement, as gg_session_report_json_device).  Returns the report's byte count.
int64_t gg_session_report_sarif_device(gg_session* s, size_t max_docs, int32_t* exit_code, double* stats, extern_err_t* err) {
  set_err(err, 0, "");
  if (!s->evaluated || !s->fetched_on_device) { set_err(err, -1, "session not evaluated and fetched on a device"); return -1; }
  try {
    std::vector<const Program*> progs;
    for (auto& p : s->progs) progs.push_back(&p->prog);
    const size_t nf = progs.size(), nd = max_docs ? std::min(max_docs, s->docs.ndocs()) : s->docs.ndocs();
    for (size_t t = 0; t < nd * nf; t++)
      if (s->tiles[t].err) {
        ensure_host_arena(s);
        ReportError re;
        tile_error(s->docs, (uint32_t)(t / nf), *progs[t % nf], s->tiles[t], re);
        set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
        if (exit_code) *exit_code = -1;
        return -1;
      }
    // SarifReport::new (sarif.rs:29-53): the FAILed documents' first-seen non-empty names
    std::vector<std::string> art;
    std::unordered_set<std::string> seen;
    bool anyfail = false;
    for (size_t d = 0; d < nd; d++) {
      uint32_t status = ST_SKIP;
      for (size_t f = 0; f < nf; f++) {
        const uint32_t st = s->tiles[d * nf + f].status;
        if (status == ST_FAIL) continue;
        status = status == ST_PASS ? (st == ST_FAIL ? ST_FAIL : ST_PASS) : st;
      }
      if (status != ST_FAIL) continue;
      anyfail = true;
      const std::string& name = s->docs.names[d];
      if (!name.empty() && seen.insert(name).second) art.push_back(name);
    }
    std::string head, tail;
    sarif_frame(art, head, tail);
    bind_device(s);
    render_tables(s);
    CountingSink sink(s->dv->pinned, DeviceBufs::kPinnedBytes);
    DevReportStats st;
    ReportError re;
    if (nf && !device_report_text(s, 0, nd, SIZE_MAX, sink, re, &st, OUT_SARIF)) {
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      if (exit_code) *exit_code = -1;
      return -1;
    }
    // the results' first comma is dropped (serde's "[\n        {"), "\n      " closes a non-empty list
    const int64_t bytes = (int64_t)(head.size() + tail.size() + (sink.n ? sink.n - 1 + 7 : 0));
    if (exit_code) *exit_code = anyfail ? 19 : (s->parse_errors.empty() ? 0 : 5);
    if (stats) {
      stats[0] = (double)st.device_docs; stats[1] = (double)st.host_docs; stats[2] = st.size_ms; stats[3] = st.write_ms;
      stats[4] = st.d2h_ms; stats[5] = st.host_ms; stats[6] = (double)st.bytes; stats[7] = (double)art.size();
    }
    return bytes;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

// a native write callback for cfn_guard_validate_batch_stream(_devices) that counts the bytes into *(uint64_t*)ctx
// and drops them (measurement: the report reaches host memory with no consumer cost on the path)
int32_t gg_count_write(void* ctx, const char*, size_t len) {
  if (ctx) *(uint64_t*)ctx += len;
  return 0;
}

int32_t gg_session_set_device_report(gg_session* s, int32_t on) { s->device_report = on < 0 ? -1 : (on ? 1 : 0); return 0; }

void gg_session_bind_counts(gg_session* s, void* dev, size_t n) {
  s->ext_counts = (dev && n >= s->ncounts) ? (unsigned long long*)dev : nullptr;
}
size_t gg_session_drain_kernel_ms(gg_session* s, double* out, size_t cap, extern_err_t* err) {
  set_err(err, 0, "");
  try { return session_drain(s, out, cap); } catch (std::exception& e) { set_err(err, -1, e.what()); return 0; }
}
int32_t gg_session_counts(gg_session* s, uint64_t* out, size_t n) {
  for (size_t i = 0; i < n && i < s->counts.size(); i++) out[i] = s->counts[i];
  return 0;
}

int32_t gg_session_add_rules(gg_session* s, const char* text, const char* name, extern_err_t* err) {
  set_err(err, 0, "");
  std::string perr;
  if (!add_rules(s, text ? text : "", name ? name : "", perr)) {
    s->parse_errors.push_back(perr);
    set_err(err, 5, error_display("ParseError", perr));
    return 5;
  }
  s->uploaded = false;
  return 0;
}

int32_t gg_session_add_docs(gg_session* s, const char* const* texts, const size_t* lens, const char* const* names, size_t n,
                            int32_t mode, int32_t nthreads, extern_err_t* err) {
  set_err(err, 0, "");
  if (nthreads < 1) nthreads = 1;
  std::vector<DocBatch> parts(nthreads);
  std::vector<LoadError> errs(nthreads);
  std::vector<int> failed(nthreads, -1);
  const DocBatch* params = s->params.get();
  auto work = [&](int t) {
    size_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
    DocBatch B;   // thread-local while it grows (no shared cache lines with the neighbours' headers)
    for (size_t i = lo; i < hi; i++) {
      if (!load_document(B, texts[i], lens[i], names ? names[i] : std::string(), (LoadMode)mode, errs[t]) ||
          !merge_params_last(B, params, errs[t])) { failed[t] = (int)i; break; }
    }
    parts[t] = std::move(B);
  };
  try {
    parallel_run((size_t)nthreads, work);
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
  for (int t = 0; t < nthreads; t++) {
    if (failed[t] >= 0) { set_err(err, ffi_code(errs[t].kind), error_display(errs[t].kind, errs[t].msg)); return 5; }
  }
  try {
    ensure_host_arena(s);   // host documents join a device-loaded batch
    merge_batches(s->docs, parts);
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
  s->uploaded = false;
  return 0;
}

int32_t gg_session_set_params(gg_session* s, const char* const* texts, const size_t* lens, const char* const* names,
                              size_t n, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::vector<validate_input_t> in(n);
    std::vector<std::string> tx(n);
    for (size_t i = 0; i < n; i++) {
      tx[i].assign(texts[i], lens[i]);   // NUL-terminated copies (load_params reads C strings)
      in[i].content = tx[i].c_str();
      in[i].file_name = names ? names[i] : "";
    }
    LoadError le;
    if (!load_params(in.data(), n, s->params, le)) {
      set_err(err, ffi_code(le.kind), error_display(le.kind, le.msg));
      return ffi_code(le.kind);
    }
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

int32_t gg_loader_selfcheck(const char* text, size_t len) { return loader_selfcheck(text, len); }

static void dump_node(const DocBatch& D, uint64_t base, uint32_t i, std::string& o) {
  const DNode& n = D.nodes[base + i];
  auto str = [&](uint32_t off, uint32_t len) { return std::string(D.bytes.data() + off, len); };
  switch (n.kind) {
    case K_NULL: o += "Null"; break;
    case K_STRING: o += "String(" + rust_debug_str(str(n.a, n.count)) + ")"; break;
    case K_BOOL: o += n.a ? "Bool(true)" : "Bool(false)"; break;
    case K_INT: o += "Int(" + std::to_string((int64_t)(((uint64_t)n.b << 32) | n.a)) + ")"; break;
    case K_FLOAT: {
      uint64_t u = ((uint64_t)n.b << 32) | n.a;
      double d;
      memcpy(&d, &u, 8);
      o += "Float(" + rust_debug_f64(d) + ")";
      break;
    }
    case K_LIST:
      o += "[";
      for (uint32_t j = 0; j < n.count; j++) { if (j) o += ", "; dump_node(D, base, n.a + j, o); }
      o += "]";
      break;
    case K_MAP:
      o += "{";
      for (uint32_t j = 0; j < n.count; j++) {
        const DNode& e = D.nodes[base + n.a + j];
        if (j) o += ", ";
        o += rust_debug_str(str(e.key_off, e.key_len)) + ": ";
        dump_node(D, base, n.a + j, o);
      }
      o += "}";
      if (n.b) {
        // MapValue.keys of a map with a repeated key: every occurrence with its mark
        const uint32_t nk = D.nodes[base + n.b].count;
        o += " keys [";
        for (uint32_t j = 0; j < nk; j++) {
          const uint64_t g = base + n.b + j;
          if (j) o += ", ";
          o += rust_debug_str(str(D.nodes[g].key_off, D.nodes[g].key_len)) + "@" + std::to_string(D.kline[g]) + ":" +
               std::to_string(D.kcol[g]);
        }
        o += "]";
      }
      break;
    default: o += "?"; break;
  }
}

char* gg_load_dump(const char* text, size_t len, int32_t mode, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    DocBatch D;
    LoadError le;
    if (!load_document(D, text ? text : "", text ? len : 0, "dump", (LoadMode)mode, le)) {
      set_err(err, ffi_code(le.kind), error_display(le.kind, le.msg));
      return nullptr;
    }
    std::string o;
    dump_node(D, D.base[0], D.roots[0], o);
    return dup_str(o);
  } catch (std::exception& e) { set_err(err, -1, e.what()); return nullptr; }
}

// the device loader's float parser (eisel_lemire.h) on the host: 1 = *out holds the correctly rounded
// double of the JSON number s[0..n), 0 = the loader refuses it (its document goes to the host loader)
int32_t gg_parse_f64(const char* s, size_t n, double* out) {
  uint64_t bits = 0;
  if (!parse_json_f64([&](uint64_t k) -> uint32_t { return k < n ? (unsigned char)s[k] : 256u; }, (uint64_t)n, kPow5_128, bits))
    return 0;
  memcpy(out, &bits, 8);
  return 1;
}

int32_t gg_regex_match(const char* pattern, const char* text, size_t len, uint32_t* stats) {
  CompiledRegex rx = compile_regex(pattern ? pattern : "");
  if (stats) { stats[0] = rx.nstates | (rx.nfa ? 0x80000000u : 0u); stats[1] = rx.ncls; }
  if (!rx.valid) return -2;
  return dfa_match(rx, text ? text : "", text ? len : 0);
}

int32_t gg_program_stats(const char* text, const char* name, uint32_t* out) {
  try {
    RulesFile rf;
    bool empty = false;
    std::string msg;
    if (!parse_rules_file(text ? text : "", name ? name : "", rf, empty, msg)) return 5;
    if (empty) return 1;
    Program p;
    if (!compile_program(rf, name ? name : "", p, msg)) return 5;
    if (out) {
      out[0] = (uint32_t)p.blob.size(); out[1] = p.hdr.off_dfa; out[2] = p.hdr.n_regex;
      out[3] = p.hdr.n_clauses; out[4] = p.hdr.n_parts;
    }
    return 0;
  } catch (std::exception&) { return -1; }
}

int32_t gg_parse_rules(const char* text, const char* name, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    RulesFile rf;
    bool empty = false;
    std::string msg;
    if (!parse_rules_file(text ? text : "", name ? name : "", rf, empty, msg)) {
      set_err(err, 5, error_display("ParseError", msg));
      return 5;
    }
    if (empty) return 1;
    Program p;
    if (!compile_program(rf, name ? name : "", p, msg)) {
      set_err(err, 5, error_display("ParseError", msg));
      return 5;
    }
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

size_t gg_synth_cfn_doc(uint64_t index, int32_t n_resources, char* buf, size_t cap) {
  std::string t;
  cfn_synth_doc(index, n_resources, t);
  if (buf && cap) {
    size_t n = std::min(cap - 1, t.size());
    memcpy(buf, t.data(), n);
    buf[n] = 0;
  }
  return t.size();
}

size_t gg_synth_cfn_yaml_doc(uint64_t index, int32_t n_resources, char* buf, size_t cap) {
  std::string t;
  cfn_synth_yaml_doc(index, n_resources, t);
  if (buf && cap) {
    size_t n = std::min(cap - 1, t.size());
    memcpy(buf, t.data(), n);
    buf[n] = 0;
  }
  return t.size();
}

int32_t gg_session_add_synthetic(gg_session* s, uint64_t first, size_t n, int32_t n_resources, int32_t nthreads,
                                 extern_err_t* err) {
  set_err(err, 0, "");
  try {
    if (nthreads < 1) nthreads = 1;
    std::vector<DocBatch> parts(nthreads);
    std::vector<LoadError> errs(nthreads);
    std::vector<int> failed(nthreads, 0);
    auto work = [&](int t) {
      size_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
      std::string text;
      DocBatch B;   // thread-local while it grows (no shared cache lines with the neighbours' headers)
      struct Back { DocBatch& b; DocBatch& slot; ~Back() { slot = std::move(b); } } back{B, parts[t]};
      for (size_t i = lo; i < hi; i++) {
        cfn_synth_doc(first + i, n_resources, text);
        if (!load_document(B, text.data(), text.size(), "synthetic-" + std::to_string(first + i) + ".json",
                           LOAD_LIBYAML, errs[t]) ||
            !merge_params_last(B, s->params.get(), errs[t])) { failed[t] = 1; return; }
        // size the part's columns once from its first documents (the generator's documents are
        // alike) instead of growing them by doubling, which copies them again and again
        if (i == lo + 7 && hi - lo > 16) {
          const size_t est = B.nodes.size() / 8 * (hi - lo) / 16 * 17;
          B.nodes.reserve(est); B.line.reserve(est); B.col.reserve(est); B.kline.reserve(est); B.kcol.reserve(est);
          B.bytes.reserve(B.bytes.size() / 8 * (hi - lo) / 16 * 17);
          B.base.reserve(hi - lo); B.roots.reserve(hi - lo); B.names.reserve(hi - lo);
        }
      }
    };
    parallel_run((size_t)nthreads, work);
    for (int t = 0; t < nthreads; t++)
      if (failed[t]) { set_err(err, ffi_code(errs[t].kind), error_display(errs[t].kind, errs[t].msg)); return 5; }
    ensure_host_arena(s);
    merge_batches(s->docs, parts);
    s->uploaded = false;
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

// ---- device loader ----------------------------------------------------------
static void load_stats(const GpuLoadStats& st, double* out) {
  if (!out) return;
  out[0] = st.kernel_ms; out[1] = (double)st.nodes; out[2] = (double)st.distinct_strings;
  out[3] = (double)st.pool_bytes; out[4] = (double)st.text_bytes; out[5] = st.h2d_ms; out[6] = st.d2h_ms;
  out[7] = (double)st.table_retries; out[8] = (double)st.refused_docs; out[9] = 0;
}

int32_t gg_session_add_docs_device(gg_session* s, const char* const* texts, const size_t* lens, const char* const* names,
                                   size_t n, double* stats, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why, s->device, &s->device)) { set_err(err, -1, why); return -1; }
    if (s->docs.ndocs()) { set_err(err, 18, "IllegalArguments: the device loader fills an empty session"); return -1; }
    if (s->params) { set_note(err, "input parameters are merged by the host loader (gg_session_add_docs)"); return 1; }
    // the device parse is one lane per document: a batch of few, large documents (Terraform plans of
    // thousands of resources) leaves the device nearly idle -- 2048 plans parsed at 0.3 GB/s of text
    // (profiles/r04a_bench_cfg4_lane_2048.json) against ~1 GB/s on 16 host threads -- so such a batch is
    // refused as a whole and the caller loads it on host threads (GG_JSON_FEW_DOCS=0 keeps it on the device)
    {
      uint64_t total = 0;
      for (size_t i = 0; i < n; i++) total += lens[i];
      const bool force = getenv("GG_JSON_FEW_DOCS") && atoi(getenv("GG_JSON_FEW_DOCS")) == 0;
      if (!force && n < (size_t)dev_ncu(s->device) * 64 && n && total / n > (64u << 10)) {
        set_note(err, "too few documents for the lane-per-document device parse (" + std::to_string(n) + " documents of " +
                          std::to_string(total / n) + " bytes on average): load them on host threads");
        return 1;
      }
    }
    std::vector<std::string> nm(n);
    for (size_t i = 0; i < n; i++) nm[i] = names ? names[i] : std::string();
    GpuLoadStats st;
    DocBatch b;
    std::vector<uint32_t> refused;
    void* dev_nodes = nullptr;
    // the arena's columns stay in HBM unless GG_RESIDENT_ARENA=0 (ensure_host_arena brings them down)
    ResidentArena res;
    const bool keep = !getenv("GG_RESIDENT_ARENA") || atoi(getenv("GG_RESIDENT_ARENA")) != 0;
    const auto tl = std::chrono::steady_clock::now();
    if (!gpu_load_json(b, texts, lens, nm, n, st, why, &refused, &dev_nodes, keep ? &res : nullptr)) { set_note(err, why); return 1; }
    struct ResHolder { ResidentArena& r; ~ResHolder() { for (uint32_t* p : {r.line, r.col, r.kline, r.kcol}) dev_free(p); } } rhold{res};
    if (getenv("GG_LOAD_TRACE"))
      fprintf(stderr, "[load] gpu_load_json returned %8.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count());
    struct Holder { void*& p; ~Holder() { dev_free(p); } } hold{dev_nodes};
    const size_t dev_n = b.nodes.size();
    if (!refused.empty()) {
      // the documents the device refused, built by the host loader (libyaml) on host threads and
      // spliced in at their positions: their nodes are appended to the arena, strings re-interned
      // (merge_batches), and their roots / bases moved to the placeholders the device left
      const size_t nt = std::min<size_t>(refused.size(), report_threads());
      std::vector<DocBatch> parts(nt);
      std::vector<LoadError> errs(nt);
      std::vector<int> ok(nt, 1);
      parallel_run(nt, [&](size_t t) {
        for (size_t j = refused.size() * t / nt; j < refused.size() * (t + 1) / nt && ok[t]; j++) {
          const uint32_t d = refused[j];
          if (!load_document(parts[t], texts[d], lens[d], nm[d], LOAD_LIBYAML, errs[t])) ok[t] = 0;
        }
      });
      for (size_t t = 0; t < nt; t++)
        if (!ok[t]) { set_note(err, "host loader: " + error_display(errs[t].kind, errs[t].msg)); return 1; }
      merge_batches(b, parts);
      for (size_t j = 0; j < refused.size(); j++) {
        b.roots[refused[j]] = b.roots[n + j];
        b.base[refused[j]] = b.base[n + j];
      }
      b.roots.resize(n); b.base.resize(n); b.names.resize(n);
    }
    s->docs = std::move(b);
    s->uploaded = false;
    dev_free(s->dev_nodes);
    s->dev_nodes = dev_nodes; s->dev_nodes_n = res.nodes ? (size_t)res.nodes : dev_n;
    dev_nodes = nullptr;
    s->resident = res;
    res = ResidentArena{};
    load_stats(st, stats);
    if (getenv("GG_LOAD_TRACE"))
      fprintf(stderr, "[load] session holds the batch %8.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count());
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

int32_t gg_session_add_synthetic_device_fmt(gg_session* s, uint64_t first, size_t n, int32_t n_resources, int32_t nthreads,
                                            int32_t format, double* stats, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    if (nthreads < 1) nthreads = 1;
    const auto g0 = std::chrono::steady_clock::now();
    std::vector<std::string> texts(n), names(n);
    auto work = [&](int t) {
      for (size_t i = n * t / nthreads; i < n * (t + 1) / nthreads; i++) {
        if (format == 1) cfn_synth_yaml_doc(first + i, n_resources, texts[i]);
        else cfn_synth_doc(first + i, n_resources, texts[i]);
        names[i] = "synthetic-" + std::to_string(first + i) + (format == 1 ? ".yaml" : ".json");
      }
    };
    parallel_run((size_t)nthreads, work);
    std::vector<const char*> p(n), nm(n);
    std::vector<size_t> l(n);
    for (size_t i = 0; i < n; i++) { p[i] = texts[i].data(); l[i] = texts[i].size(); nm[i] = names[i].c_str(); }
    const double gen_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g0).count();
    const int32_t rc = gg_session_add_docs_device(s, p.data(), l.data(), nm.data(), n, stats, err);
    if (stats) stats[9] = gen_ms;
    // the generated text is freed by the threads that allocated it (their own malloc arenas; freeing
    // a million buffers from one thread serialises on the arenas' locks)
    const auto f0 = std::chrono::steady_clock::now();
    parallel_run((size_t)nthreads, [&](size_t t) {
      for (size_t i = n * t / nthreads; i < n * (t + 1) / nthreads; i++) { std::string().swap(texts[i]); std::string().swap(names[i]); }
    });
    if (getenv("GG_LOAD_TRACE"))
      fprintf(stderr, "[load] generated text freed %8.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count());
    return rc;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

int32_t gg_session_add_synthetic_device(gg_session* s, uint64_t first, size_t n, int32_t n_resources, int32_t nthreads,
                                        double* stats, extern_err_t* err) {
  return gg_session_add_synthetic_device_fmt(s, first, n, n_resources, nthreads, 0, stats, err);
}

// Parity of the device loader with the host loader on the same documents: 1 = the same arena up
// to string ids (node kinds, counts, child / parent links, scalars, marks, string bytes, and one
// pool entry per distinct string), 0 = they differ (`err` says where), -1 = the device refused.
int32_t gg_loader_device_check(const char* const* texts, const size_t* lens, size_t n, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why)) { set_err(err, -1, why); return -1; }
    std::vector<std::string> nm(n, "x");
    DocBatch g, h;
    GpuLoadStats st;
    if (!gpu_load_json(g, texts, lens, nm, n, st, why)) { set_note(err, why); return -1; }
    for (size_t i = 0; i < n; i++) {
      LoadError le;
      if (!load_document(h, texts[i], lens[i], "x", LOAD_LIBYAML, le)) { set_note(err, "host loader failed"); return 0; }
    }
    auto differ = [&](const std::string& what, size_t at) { set_note(err, what + " at node " + std::to_string(at)); return 0; };
    if (g.nodes.size() != h.nodes.size()) return differ("node count", 0);
    if (g.base != h.base || g.roots != h.roots) return differ("document bases", 0);
    if (g.iused != h.iused) return differ("distinct strings", 0);
    auto sv = [](const DocBatch& b, uint32_t off, uint32_t len) { return std::string(b.bytes.data() + off, len); };
    for (size_t k = 0; k < h.nodes.size(); k++) {
      const DNode &a = g.nodes[k], &b = h.nodes[k];
      if (a.kind != b.kind || a.count != b.count || a.parent != b.parent || a.key_len != b.key_len) return differ("shape", k);
      if (g.line[k] != h.line[k] || g.col[k] != h.col[k] || g.kline[k] != h.kline[k] || g.kcol[k] != h.kcol[k]) return differ("marks", k);
      if ((a.key_off == NONE) != (b.key_off == NONE)) return differ("key presence", k);
      if (a.key_off != NONE) {
        if (a.key_hash != a.key_off || sv(g, a.key_off, a.key_len) != sv(h, b.key_off, b.key_len)) return differ("key", k);
        if (g.find(g.bytes.data() + a.key_off, a.key_len) != a.key_off) return differ("key index", k);
      }
      if (a.kind == K_STRING) {
        if (a.b != a.a || sv(g, a.a, a.count) != sv(h, b.a, b.count)) return differ("string", k);
        if (g.find(g.bytes.data() + a.a, a.count) != a.a) return differ("string index", k);
      } else if (a.a != b.a || a.b != b.b) {
        return differ("scalar / link", k);
      }
    }
    return 1;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

int32_t gg_session_upload(gg_session* s, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why, s->device, &s->device)) { set_err(err, -1, why); return -1; }
    session_upload(s);
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

// Runs `iters` evaluations of every (doc, rules-file) tile; fills per-iteration kernel ms.
int32_t gg_session_eval(gg_session* s, int32_t iters, double* ms_out, extern_err_t* err) {
  set_err(err, 0, "");
  try {
    std::string why;
    if (!ensure_device(why, s->device, &s->device)) { set_err(err, -1, why); return -1; }
    if (!s->uploaded) session_upload(s);
    for (int32_t i = 0; i < iters; i++) {
      double ms = session_run(s, i == iters - 1);
      if (ms_out) ms_out[i] = ms;
    }
    return 0;
  } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
}

char* gg_session_report(gg_session* s, int32_t* exit_code, extern_err_t* err) {
  return gg_session_report_format(s, OUT_JSON, exit_code, err);
}

char* gg_session_report_format(gg_session* s, int32_t output_format, int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (!s->evaluated) { set_err(err, -1, "session not evaluated"); return nullptr; }
  if (output_format < OUT_JSON || output_format > OUT_JUNIT) { set_err(err, 18, "IllegalArguments: unknown output format"); return nullptr; }
  std::string out;
  char* cs = nullptr;
  int32_t code = 0;
  ReportError re;
  if (!session_report(s, out, code, re, output_format, &cs)) {
    if (exit_code) *exit_code = -1;
    set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
    return nullptr;
  }
  if (exit_code) *exit_code = code;
  return cs ? cs : dup_str(out);
}

char* gg_session_report_range(gg_session* s, int32_t output_format, size_t first, size_t count, int32_t* exit_code,
                              extern_err_t* err) {
  return gg_session_report_range_n(s, output_format, first, count, nullptr, exit_code, err);
}

char* gg_session_report_range_n(gg_session* s, int32_t output_format, size_t first, size_t count, size_t* len,
                                int32_t* exit_code, extern_err_t* err) {
  set_err(err, 0, "");
  if (len) *len = 0;
  if (!s->evaluated) { set_err(err, -1, "session not evaluated"); return nullptr; }
  if (output_format < OUT_JSON || output_format > OUT_JUNIT) { set_err(err, 18, "IllegalArguments: unknown output format"); return nullptr; }
  try {
    std::string out;
    char* cs = nullptr;
    int32_t code = 0;
    ReportError re;
    if (!session_report(s, out, code, re, output_format, &cs, first, count)) {
      if (exit_code) *exit_code = -1;
      set_err(err, ffi_code(re.kind), error_display(re.kind, re.msg));
      return nullptr;
    }
    if (exit_code) *exit_code = code;
    if (len) *len = cs ? strlen(cs) : out.size();
    return cs ? cs : dup_str(out);
  } catch (std::exception& e) { set_err(err, -1, e.what()); return nullptr; }
}

// statistics: 0 ndocs, 1 nfiles, 2 nodes, 3 string bytes, 4 tiles FAIL, 5 tiles PASS, 6 tiles SKIP,
// 7 tiles with error, 8 records, 9 device arena bytes (nodes + strings + roots), 10 first error code,
// 11 record bytes of the last fetch, 12 record capacity, 13 max top rules per file, 14 wave slots, 15 heap bytes/slot
// Diagnostic: an evaluation's results (tile headers, rule statuses, records) to / from a file, so the
// host report writer can be profiled and A/B'd on a CPU against results the GPU produced.  The
// loading session must hold the same rules files and documents, added in the same order.
int32_t gg_session_save_results(gg_session* s, const char* path, extern_err_t* err) {
  set_err(err, 0, "");
  if (!s->evaluated) { set_err(err, -1, "session not evaluated"); return -1; }
  FILE* f = fopen(path, "wb");
  if (!f) { set_err(err, -1, std::string("cannot write ") + path); return -1; }
  try { ensure_host_arena(s); } catch (std::exception& e) { set_err(err, -1, e.what()); return -1; }
  const uint64_t h[4] = {0x47475245ull, s->tiles.size(), s->max_top, s->recs.size()};
  bool ok = fwrite(h, sizeof(h), 1, f) == 1;
  ok = ok && (s->tiles.empty() || fwrite(s->tiles.data(), sizeof(TileOut), s->tiles.size(), f) == s->tiles.size());
  ok = ok && (s->rule_status.empty() || fwrite(s->rule_status.data(), 1, s->rule_status.size(), f) == s->rule_status.size());
  ok = ok && (s->recs.empty() || fwrite(s->recs.data(), sizeof(Rec), s->recs.size(), f) == s->recs.size());
  fclose(f);
  if (!ok) { set_err(err, -1, "short write"); return -1; }
  return 0;
}

int32_t gg_session_load_results(gg_session* s, const char* path, extern_err_t* err) {
  set_err(err, 0, "");
  FILE* f = fopen(path, "rb");
  if (!f) { set_err(err, -1, std::string("cannot read ") + path); return -1; }
  uint64_t h[4];
  bool ok = fread(h, sizeof(h), 1, f) == 1 && h[0] == 0x47475245ull && h[1] == s->docs.ndocs() * s->progs.size();
  if (ok) {
    s->tiles.resize(h[1]); s->max_top = (uint32_t)h[2]; s->rule_status.resize(h[1] * h[2]); s->recs.resize(h[3]);
    ok = (h[1] == 0 || fread(s->tiles.data(), sizeof(TileOut), h[1], f) == h[1]) &&
         (s->rule_status.empty() || fread(s->rule_status.data(), 1, s->rule_status.size(), f) == s->rule_status.size()) &&
         (h[3] == 0 || fread(s->recs.data(), sizeof(Rec), h[3], f) == h[3]);
  }
  fclose(f);
  if (!ok) { set_err(err, -1, "results file does not match this session"); return -1; }
  s->evaluated = true;
  s->fetched_on_device = false;   // host results only: the host writer reports them
  return 0;
}

int64_t gg_session_stat(gg_session* s, int32_t what) {
  switch (what) {
    case 0: return (int64_t)s->docs.ndocs();
    case 1: return (int64_t)s->progs.size();
    case 2: return (int64_t)arena_nodes(s);
    case 3: return (int64_t)s->docs.bytes.size();
    case 4: case 5: case 6: {
      uint32_t want = what == 4 ? ST_FAIL : what == 5 ? ST_PASS : ST_SKIP;
      int64_t c = 0;
      for (auto& t : s->tiles) if (!t.err && t.status == want) c++;
      return c;
    }
    case 7: { int64_t c = 0; for (auto& t : s->tiles) if (t.err) c++; return c; }
    case 8: return (int64_t)std::max<size_t>(s->recs.size(), s->recs_total);
    case 9: return (int64_t)(arena_nodes(s) * sizeof(DNodeP) + s->docs.bytes.size() + s->docs.roots.size() * 12);
    case 10: for (auto& t : s->tiles) if (t.err) return t.err; return 0;
    case 11: return (int64_t)std::max<size_t>(s->recs.size(), s->recs_total) * (int64_t)sizeof(Rec);
    case 12: return (int64_t)s->rec_cap;
    case 13: return (int64_t)s->max_top;
    case 14: return (int64_t)s->nslots;
    case 15: return (int64_t)s->heap_bytes;
    case 16: {   // tiles the lane kernel handed to wave mode in the last launch
      uint32_t v = 0;
      if (s->dv && s->dv->d_counters.p) { bind_device(s); HIPCHK(hipMemcpy(&v, s->dv->d_counters.p + 3, 4, hipMemcpyDeviceToHost)); }
      return v;
    }
    case 17: return (int64_t)s->lane_slots;
    case 18: { size_t m = 0; for (auto& p : s->progs) m = std::max(m, p->prog.blob.size() * 4); return (int64_t)m; }
    case 19: {   // largest program blob without its regex DFA tables (the part staged in LDS)
      size_t m = 0;
      for (auto& p : s->progs) m = std::max(m, p->prog.blob.size() * 4 - (size_t)p->prog.hdr.n_dfa * 2);
      return (int64_t)m;
    }
    case 20: return (int64_t)s->mode;   // 0 lane mode (+ wave retry), 1 wave mode
    case 21: return (int64_t)s->parse_errors.size();   // rules files that did not parse (exit code 5)
    case 22: return (int64_t)s->lane_group;   // lanes per document of the lane kernel (1: one lane per tile)
    case 23: return (int64_t)s->lane_docs;    // documents per lane batch
    default: return -1;
  }
}

// per-tile status (0 PASS 1 FAIL 2 SKIP, 3 error) into out[ndocs * nfiles]
int32_t gg_session_tile_status(gg_session* s, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n && i < s->tiles.size(); i++) out[i] = s->tiles[i].err ? 3 : (uint8_t)s->tiles[i].status;
  return 0;
}

double gg_session_last_kernel_ms(gg_session* s) { return s->last_kernel_ms; }

// diagnostic lane-kernel counters accumulated since upload (all zero unless built with GG_STATS):
// node reads, heap accesses, query_retrieval calls, clause evaluations, frames pushed, records,
// map entries scanned by key lookups, fast-filter tests, tiles
int32_t gg_session_kernel_stats(gg_session* s, uint64_t* out, size_t n) {
  if (!s->dv || !s->dv->d_stats.p) return -1;
  bind_device(s);
  std::vector<unsigned long long> v(32);
  HIPCHK(hipMemcpy(v.data(), s->dv->d_stats.p, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n && i < 32; i++) out[i] = v[i];
  return 0;
}

int32_t gg_device_available(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int64_t gg_device_cache_release(int32_t device) {
  int64_t released = 0;
  for (int d = 0; d < DevCache::kDevs; d++) {
    if (device >= 0 && d != device) continue;
    released += (int64_t)dev_cache_held(d);
    dev_cache_flush(d);
  }
  // the streamed entries' pinned staging blocks (host_pinned.h PinnedCache)
  released += (int64_t)pinned_cache_flush(device);
  return released;
}

}  // extern "C"
