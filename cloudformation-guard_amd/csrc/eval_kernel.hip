// MI355X batch evaluator kernel: one wavefront per (document, rules-file) tile.
//
// The wave interprets the compiled rules program (program.h) over the document arena
// (doc_loader.h).  Control flow is wave-uniform: every lane executes the same interpreter
// steps on identical scalar state (redundant but divergence-free, and every lane only reads
// what it wrote, so no intra-wave fences are needed); map key lookups are wave-cooperative
// (64 children compared per step, first hit via __ballot).  Failure records are staged in the
// wave's scratch heap and published to the global record arena with one atomic per tile.
//
// Function-for-function restatement of the reference evaluation path:
//   eval_rules_file / eval_rule / eval_conjunction_clauses   guard/src/rules/eval.rs:1837-2065
//   eval_type_block_clause / eval_guard_block_clause          eval.rs:1303-1426, 1649-1822
//   eval_when_condition_block / eval_guard_named_clause       eval.rs:1227-1289, 1428-1502
//   eval_guard_access_clause / unary_operation / binary_op    eval.rs:174-405, 765-974, 1077-1225
//   operators (Eq / In / Common / not reverse-diffs)          guard/src/rules/eval/operators.rs
//   query_retrieval_with_converter                            guard/src/rules/eval_context.rs:337-924
//   scopes (Root/Block/Value/ResolvedParameter)               eval_context.rs:1062-1606, eval.rs:1504-1572
//   compare_eq / compare_values / PartialEq                   guard/src/rules/path_value.rs:245-291, 1047-1192
#include <hip/hip_runtime.h>

#include "eval_device.h"

#define DEV __device__ __attribute__((always_inline)) inline
#define DEVN __device__ __attribute__((noinline))
// GG_NFA 1 (eval_kernel_nfa.hip): the evaluator kernels again, with the regex NFA simulation compiled in
// and the names suffixed _nfa; the shared helper kernels are built once, by the GG_NFA 0 unit.
#ifndef GG_NFA
#define GG_NFA 0
#endif
#if GG_NFA
#define GG_KN(x) x##_nfa
#else
#define GG_KN(x) x
#endif
#ifndef GG_STEAL
#define GG_STEAL 1   // cross-XCD batch stealing at the end of a launch (profiles/r02_ab_inline.log)
#endif

namespace gg {
namespace wv {
#define GG_LANE 0
#include "eval_core.inc"
#undef GG_LANE
}  // namespace wv
namespace ln {
#define GG_LANE 1
#include "eval_core.inc"
#undef GG_LANE
}  // namespace ln
namespace vb {
#define GG_LANE 0
#define GG_VERBOSE 1
#include "eval_core.inc"
#undef GG_VERBOSE
#undef GG_LANE
}  // namespace vb

// ------------------------------------------------------------------ kernels ---
// Rules program staging: every section of the file's program blob before the regex DFA tables
// (KBs: clauses, query parts, strings, literals) is copied into the workgroup's LDS and the
// DevProg pointers are rebased onto the copy, so the interpreter's program reads are LDS reads
// instead of dependent global loads.  Programs larger than the LDS window stay in HBM.
// The staging window is dynamic shared memory sized per launch (LaunchArgs::lds_prog_words: the
// largest program of the launch, capped by the host): a small rules pack leaves LDS for occupancy,
// a regex-heavy one gets its DFA tables staged too.

__device__ __attribute__((always_inline)) inline const DevProg* stage_program(const DevProg* G, DevProg* sp, uint4* sblob,
                                                                             uint32_t window) {
  const uint32_t lane = __lane_id();
  __syncthreads();   // the previous batch's reads of the window are complete
  uint32_t n = G->lds_words;
  // the whole blob (regex DFA tables included) when it fits the window, else all but the tables
  const uint32_t dfa_off = (uint32_t)((const uint32_t*)G->dfa - G->blob);
  if (n > window) n = dfa_off;
  if (n > window) return G;
  const uint4* src = (const uint4*)G->blob;
  for (uint32_t i = lane; i < (n + 3u) / 4u; i += 64u) sblob[i] = src[i];
  if (lane == 0) {
    DevProg d = *G;
    const char* gb = (const char*)G->blob;
    const size_t lim = (size_t)n * 4u;
    char* lb = (char*)sblob;
#define GG_REBASE(f) do { size_t o = (size_t)((const char*)d.f - gb); if (o < lim) d.f = (decltype(d.f))(lb + o); } while (0)
    GG_REBASE(strs); GG_REBASE(parts); GG_REBASE(queries); GG_REBASE(clauses); GG_REBASE(conjs); GG_REBASE(disjs);
    GG_REBASE(clause_refs); GG_REBASE(disj_refs); GG_REBASE(blocks); GG_REBASE(lets); GG_REBASE(rules);
    GG_REBASE(name_rules); GG_REBASE(name_rule_ids); GG_REBASE(funcs); GG_REBASE(params); GG_REBASE(param_vars);
    GG_REBASE(alts); GG_REBASE(regex); GG_REBASE(lit_nodes); GG_REBASE(lit_ranges); GG_REBASE(bytes);
    d.dfa_lds = 0;
    if ((size_t)dfa_off * 4u < lim && G->dfa) { GG_REBASE(dfa); d.dfa_lds = 1; }
#undef GG_REBASE
    *sp = d;
  }
  __syncthreads();
  return sp;
}

// Shared per-tile prologue: scratch heap layout, root frame, memo table.  Lane mode: the wave's
// shared values (heap, arena bases, heap layout) are in ln::g_wave (set once per wave); wave mode
// keeps them in the Ctx.
template <typename CtxT>
__device__ __attribute__((always_inline)) inline void tile_ptrs_lane(CtxT& c, const LaunchArgs& A, uint32_t doc) {
  c.dbase = (uint32_t)A.docs.base[doc];
  c.resmap = A.docs.res_map ? A.docs.res_map[doc] : NONE;
  c.tix_off = c.resmap != NONE ? A.docs.tix_off[doc] : NONE;
}
template <typename CtxT>
__device__ __attribute__((always_inline)) inline void tile_ptrs_wave(CtxT& c, const LaunchArgs& A, const DevProg* P,
                                                                     uint32_t doc, uint8_t* heap, uint32_t frames_bytes,
                                                                     uint32_t recs_bytes) {
  c.P = (decltype(c.P))P; c.dn = A.docs.nodes + A.docs.base[doc]; c.kl = A.docs.klen + A.docs.base[doc]; c.db = A.docs.bytes; c.heap = heap;
  c.fcap = frames_bytes; c.rcap = recs_bytes; c.sguard = A.stack_guard;
  c.resmap = A.docs.res_map ? A.docs.res_map[doc] : NONE;
  c.tix = c.resmap != NONE ? A.docs.tix + A.docs.tix_off[doc] : nullptr;
  c.type_key = A.docs.type_key;
}
template <bool LANE, typename CtxT>
__device__ __attribute__((always_inline)) inline void tile_begin(CtxT& c, const LaunchArgs& A, const DevProg* P,
                                                                 uint32_t doc, uint8_t* heap, uint32_t heap_bytes,
                                                                 uint32_t frames_bytes, uint32_t recs_bytes) {
  if constexpr (LANE) tile_ptrs_lane(c, A, doc);
  else tile_ptrs_wave(c, A, P, doc, heap, frames_bytes, recs_bytes);
  c.tmp = frames_bytes + recs_bytes; c.pers = heap_bytes; c.nframes = 0; c.nrec = 0;
  c.err = 0; c.err_a = 0; c.err_b = 0; c.suppress = 0; c.rec_created = 0; c.split = 0; c.nsyn = 0;
  c.ffok = NONE; c.naux = 0;
#ifdef GG_STATS
  for (int i = 0; i < 8; i++) { c.st[i] = 0; c.tdep[i] = 0; }
  for (int i = 0; i < 9; i++) c.tst[i] = 0;
  for (int i = 0; i < 14; i++) c.fc[i] = 0;
  c.tst[8] = __builtin_amdgcn_s_memtime();
#endif
}
template <typename CtxT>
__device__ __attribute__((always_inline)) inline void tile_stats(CtxT& c, const LaunchArgs& A) {
#ifdef GG_STATS
  for (int i = 0; i < 8; i++) atomicAdd(&A.stats[i], (unsigned long long)c.st[i]);
  atomicAdd(&A.stats[8], 1ull);
  c.tst[8] = __builtin_amdgcn_s_memtime() - c.tst[8];
  for (int i = 0; i < 9; i++) atomicAdd(&A.stats[9 + i], c.tst[i]);
  for (int i = 0; i < 14; i++) atomicAdd(&A.stats[18 + i], (unsigned long long)c.fc[i]);
#endif
}

// Lane mode (the throughput path): each lane evaluates one (document, rules file) tile.  A wave
// takes a batch = one rules file x 64 consecutive documents, so all lanes interpret the same
// program over different documents.  Records are published with one atomic per wave (wave
// prefix sum).  Tiles that outgrow the 64 KB lane heap (heap, record staging or frame limits)
// are queued for the wave-mode kernel below instead of failing.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GG_LANE_WAVES_PER_EU))) GG_KN(guard_eval_lanes_kernel)(LaunchArgs A) {
  using namespace ln;
  const uint32_t lane = __lane_id();
  // 64 lanes share one interleaved region (see haddr in eval_core.inc)
  uint8_t* heap = A.lane_heaps + (size_t)blockIdx.x * 64 * A.lane_heap_bytes;
  // XCD-aware work queues: workgroups are dispatched round-robin over the 8 XCDs, so block b runs
  // on XCD b % 8.  Each XCD owns a contiguous eighth of the 64-document chunks and hands out its
  // batches chunk-major, file-minor: the rules files of one chunk run back to back on the same
  // XCD, so the chunk's arena lines fetched by the first file are L2 hits for the others.
  // a batch is lane_docs consecutive documents (64, or fewer for launches of few large documents: fewer
  // lanes of a wave diverge, and more waves share the CUs)
  const uint32_t L = A.lane_docs ? A.lane_docs : 64u;
  // lanes per document: 1, or 64 / L -- the lanes of a document run its tile in step (identical state, one
  // writer) and split its list fan-outs' filter tests (eval_recursive.inc coop_chunk)
  const uint32_t G = (A.lane_group & 0xFFFFu) ? (A.lane_group & 0xFFFFu) : 1u;
  const bool leader = (lane & (G - 1u)) == 0u;
  const uint32_t nchunks = (A.docs.ndocs + L - 1u) / L;
  const uint32_t xcd = blockIdx.x & 7u;
  const uint32_t c0 = (uint32_t)(((uint64_t)nchunks * xcd) / 8u), c1 = (uint32_t)(((uint64_t)nchunks * (xcd + 1u)) / 8u);
  const uint32_t nbatches = (c1 - c0) * A.nfiles;
  // interpreter state lives in LDS (one Ctx per lane), not in the per-lane stack
  __shared__ Ctx s_ctx[64];
  extern __shared__ uint4 s_blob[];
  LCtx& c = *(LCtx*)&s_ctx[lane];
  if (lane == 0) {
    g_wave.heap = heap; g_wave.nodes = A.docs.nodes; g_wave.klen = A.docs.klen; g_wave.db = A.docs.bytes;
    g_wave.tix = A.docs.tix; g_wave.fcap = FRAMES_BYTES; g_wave.rcap = A.lane_recs_bytes; g_wave.type_key = A.docs.type_key;
    g_wave.recs = A.recs; g_wave.rchunk = A.rec_chunk; g_wave.sguard = A.stack_guard;
    g_wave.rstride = L; g_wave.group = G; g_wave.split_on = (A.lane_group >> 16) ? 0u : 1u;
  }
  __syncthreads();
  uint32_t staged = NONE;
  const DevProg* P = nullptr;
#if GG_STEAL
  // a wave whose XCD queue is empty takes batches from the other XCDs' queues, in order, so the
  // launch does not end with one XCD still working through its eighth
  uint32_t qi = 0;
#endif
  for (;;) {
    uint32_t b = 0;
#if GG_STEAL
    const uint32_t q = (xcd + qi) & 7u;
    const uint32_t q0 = (uint32_t)(((uint64_t)nchunks * q) / 8u), q1 = (uint32_t)(((uint64_t)nchunks * (q + 1u)) / 8u);
    if (lane == 0) b = atomicAdd(A.xcd_cursor + q, 1u);
    b = __shfl(b, 0);
    if (b >= (q1 - q0) * A.nfiles) { if (++qi == 8u) break; continue; }
    const uint32_t file = b % A.nfiles, chunk = q0 + b / A.nfiles;
    (void)nbatches; (void)c1;
#else
    if (lane == 0) b = atomicAdd(A.xcd_cursor + xcd, 1u);
    b = __shfl(b, 0);
    if (b >= nbatches) break;
    const uint32_t file = b % A.nfiles, chunk = c0 + b / A.nfiles;
#endif
    const uint32_t pos = chunk * L + lane / G;
    const bool active = lane / G < L && pos < A.docs.ndocs;
    const uint32_t doc = (A.order && active) ? A.order[pos] : pos;
    if (file != staged) { P = stage_program(&A.progs[file], &g_prog, s_blob, A.lds_prog_words); staged = file; }
    const uint32_t tile = doc * A.nfiles + file;
    uint32_t status = ST_SKIP, n = 0;
    if (P != &g_prog) {
      // the program did not fit the LDS window: lane mode reads it through LDS-typed pointers only,
      // so the whole batch goes to the wave kernel
      if (active && leader) A.retry_list[atomicAdd(A.retry_count, 1u)] = tile;
      continue;
    }
    // the batch's direct record chunk: L documents x rec_chunk slots (slot i of document d at base + L i + d),
    // one atomic per wave (eval_core.inc rec_store); a reservation past the arena leaves the lanes without a
    // chunk (their tiles then fail with E_RECORDS if they record anything, and the host re-runs with a larger
    // arena)
    uint32_t rbase = NONE;
    if (A.rec_chunk) {
      if (lane == 0) rbase = atomicAdd(A.rec_cursor, L * A.rec_chunk);
      rbase = __shfl(rbase, 0);
      if ((uint64_t)rbase + (uint64_t)L * A.rec_chunk > A.rec_cap) rbase = NONE;
    }
    c.rbase = rbase == NONE ? NONE : rbase + lane / G;
    c.mute = leader ? 0u : 1u;
    if (active) {
      tile_begin<true>(c, A, P, doc, heap, A.lane_heap_bytes, FRAMES_BYTES, A.lane_recs_bytes);
      c.syn_off = alloc_pers(c, 256 * 16);
      c.wbase = alloc_pers(c, WLEVELS * (uint32_t)sizeof(WLevel)); c.wdepth = 0;
      c.memo = alloc_pers(c, (P->n_slots ? P->n_slots : 1) * 4);
      if (!c.err) for (uint32_t i = 0; i < P->n_slots; i++) u32a(c, c.memo)[i] = 3u;
      c.vtab = alloc_pers(c, (P->n_vars ? P->n_vars : 1) * 16);
      if (!c.err) for (uint32_t i = 0; i < P->n_vars; i++) u32a(c, c.vtab)[i * 4] = 0u;
      push_frame(c, F_ROOT, NONE, A.docs.roots[doc], P->root_block);
      uint32_t fails = 0, passes = 0;
      uint8_t* rs = A.rule_status + (size_t)tile * A.max_top;
      for (uint32_t r = 0; r < P->n_top && !c.err; r++) {
        uint32_t st = run_rule(c, P->top_first + r);
        if (c.err) break;
        if (leader) rs[r] = (uint8_t)st;
        if (st == ST_PASS) passes++; else if (st == ST_FAIL) fails++;
      }
      status = fails ? ST_FAIL : (passes ? ST_PASS : ST_SKIP);
      n = c.err ? 0 : c.nrec + c.naux;
      // records written into a chunk the arena could not hold: the tile is re-run after the host grows it
      if (n && A.rec_chunk && c.rbase == NONE) { c.err = E_RECORDS; n = 0; }
      if (leader) tile_stats(c, A);
    }
    // a tile whose records fit its chunk is published in place; the others (overflow, or no chunks) get a
    // contiguous range: wave-aggregated allocation, one atomic per wave
    const bool in_chunk = active && A.rec_chunk && c.rbase != NONE && n <= A.rec_chunk;
    const uint32_t need = (in_chunk || !leader) ? 0u : n;
    uint32_t incl = need;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      uint32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    uint32_t total = __shfl(incl, 63);
    uint32_t base = 0;
    if (lane == 0 && total) base = atomicAdd(A.rec_cursor, total);
    base = __shfl(base, 0);
    if (active && leader) {
      uint32_t off = base + incl - need;
      bool retry = c.err == E_HEAP || c.err == E_RECORDS || c.err == E_DEPTH;   // not E_STACK: wave frames are larger
      if (retry) A.retry_list[atomicAdd(A.retry_count, 1u)] = tile;
      if (need && off + need > A.rec_cap) { c.err = E_RECORDS; n = 0; }
      const uint32_t naux = n ? c.naux : 0, nrec = n - naux;
      TileOut o;
      o.status = status; o.err = c.err; o.err_a = c.err_a; o.err_b = c.err_b;
      o.rec_n = nrec; o.pad0 = naux;
      if (in_chunk && n) {
        // side records follow the tile's records in its chunk
        for (uint32_t i = 0; i < naux; i++) rec_store(c, nrec + i, stage_load(c, rec_slots(c) - 1 - i));
        o.rec_off = c.rbase; o.pad1 = L;   // slot k at rec_off + L k (session_fetch compacts)
      } else {
#if GG_AB_NOREC != 1 && GG_AB_NOREC != 3   // diagnostic A/B only (2: staging off; 3: copy-out off)
        for (uint32_t i = 0; i < nrec; i++) A.recs[off + i] = rec_load(c, i);
#endif
        for (uint32_t i = 0; i < naux; i++)
          A.recs[off + nrec + i] = stage_load(c, rec_slots(c) - 1 - i);
        o.rec_off = n ? off : 0; o.pad1 = 1;   // contiguous
      }
      A.tiles[tile] = o;
    }
  }
}

// Wave mode: one wavefront per tile, all 64 lanes in lock-step (map lookups are wave-parallel),
// 512 KB heap per wave.  Runs the tiles the lane kernel queued (A.retry_list), or every tile
// when A.retry_list is null.
__global__ void __launch_bounds__(64) GG_KN(guard_eval_kernel)(LaunchArgs A) {
  using namespace wv;
#include "wave_tile_loop.inc"
}

// guard-ffi run_checks(verbose = true): the same wave-mode evaluation recording every event of the
// reference's EventRecord tree (eval_core.inc, GG_VERBOSE); the host renders it (reporter.cpp
// verbose_tree).  Launched only for verbose requests, so the two kernels above keep no trace of it.
__global__ void __launch_bounds__(64) GG_KN(guard_eval_verbose_kernel)(LaunchArgs A) {
  using namespace vb;
#include "wave_tile_loop.inc"
}

}  // namespace gg

#if !GG_NFA
namespace gg {

// Resource-type column (DevBatch::tix): one wavefront per document, lanes over the entries of the
// root's `Resources` map (coalesced reads of the contiguous entry block), each lane looking up its
// resource's exact `Type` key.  Runs once per upload (capi.cpp session_upload): the column depends on
// the documents only.
__global__ void __launch_bounds__(256) resource_type_kernel(DevBatch D) {
  const uint32_t lane = __lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;
  const uint32_t nwaves = gridDim.x * blockDim.x / 64u;
  for (uint32_t d = wave; d < D.ndocs; d += nwaves) {
    const uint32_t rm = D.res_map[d];
    if (rm == NONE) continue;
    const DNodeP* dn = D.nodes + D.base[d];
    const DNodeP m = dn[rm];
    uint32_t* out = D.tix + D.tix_off[d];
    for (uint32_t j = lane; j < (m.kc >> 4); j += 64u) {
      const DNodeP r = dn[m.a + j];
      uint32_t v = TIX_UNDECIDED;
      if ((r.kc & 15u) == K_MAP) {
        for (uint32_t k = 0; k < (r.kc >> 4); k++) {
          const DNodeP e = dn[r.a + k];
          if (e.key_hash != D.type_key) continue;
          const uint32_t ek = e.kc & 15u;
          v = ek == K_STRING ? e.b : (ek == K_LIST ? TIX_UNDECIDED : TIX_NOT_STRING);
          break;
        }
      }
      out[j] = v;
    }
  }
}

// Shape key per document for the lane kernel's batch order (capi.cpp session_upload): its counts of
// the batch's 8 most frequent Type strings, 8 bits each, most frequent first; from the type column.
__global__ void __launch_bounds__(256) shape_key_kernel(DevBatch D, const uint32_t* top8, unsigned long long* key) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = top8[i];
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < D.ndocs; d += gridDim.x * blockDim.x) {
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t rm = D.res_map[d];
    if (rm != NONE) {
      const uint32_t n = D.nodes[D.base[d] + rm].kc >> 4;
      const uint32_t* col = D.tix + D.tix_off[d];
      for (uint32_t j = 0; j < n; j++) {
        const uint32_t v = col[j];
#pragma unroll
        for (int i = 0; i < 8; i++) cnt[i] += v == t[i] ? 1u : 0u;
      }
    }
    unsigned long long k = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) k = (k << 8) | (cnt[i] < 255u ? cnt[i] : 255u);
    key[d] = k;
  }
}

// Per-(rules file, top rule) PASS/FAIL/SKIP tallies over every tile of one evaluation, plus a
// per-file line (index max_top) holding file statuses and errored tiles (status slot 3).
// counts[((file * (max_top + 1) + rule) * 4) + status]; the same buffer is what the multi-GPU
// path all-reduces over RCCL.  LDS-privatised so global atomics are per block.
__global__ void __launch_bounds__(256) rule_count_kernel(const TileOut* tiles, const uint8_t* rule_status,
                                                          const DevProg* progs, uint32_t nfiles, uint32_t ntiles,
                                                          uint32_t max_top, unsigned long long* counts) {
  extern __shared__ uint32_t lds_counts[];
  const uint32_t ncount = nfiles * (max_top + 1) * 4;
  for (uint32_t i = threadIdx.x; i < ncount; i += blockDim.x) lds_counts[i] = 0;
  __syncthreads();
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x) {
    uint32_t file = t % nfiles;
    TileOut o = tiles[t];
    uint32_t base = file * (max_top + 1) * 4;
    if (o.err) { atomicAdd(&lds_counts[base + max_top * 4 + 3], 1u); continue; }
    atomicAdd(&lds_counts[base + max_top * 4 + o.status], 1u);
    uint32_t ntop = progs[file].n_top;
    const uint8_t* rs = rule_status + (size_t)t * max_top;
    for (uint32_t r = 0; r < ntop; r++) atomicAdd(&lds_counts[base + r * 4 + rs[r]], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ncount; i += blockDim.x)
    if (lds_counts[i]) atomicAdd(&counts[i], (unsigned long long)lds_counts[i]);
}

// Record compaction (session_fetch, outside the evaluation): every tile's records -- in place in its
// lane's direct chunk (TileOut.pad1 = stride s > 1: record k at rec_off + s k) or contiguous (pad1 0 / 1) -- are
// copied to dst[dense_off[t] ..), dense_off an exclusive scan of the tiles' record counts (rec_n + pad0),
// so the host receives one dense array in tile order.  Three passes: per-block sums, a one-block scan of
// the block sums, then per-block scan + copy.  The evaluation's buffers are only read (idempotent).
static constexpr uint32_t kScanTiles = 1024;   // tiles per block (256 threads x 4)
__device__ __attribute__((always_inline)) inline uint32_t tile_rec_count(const TileOut* t, uint32_t i, uint32_t n) {
  return i < n ? t[i].rec_n + t[i].pad0 : 0u;
}
__global__ void __launch_bounds__(256) rec_block_sums_kernel(const TileOut* tiles, uint32_t n, uint32_t* bsum) {
  __shared__ uint32_t part[256];
  const uint32_t i0 = blockIdx.x * kScanTiles + threadIdx.x * 4u;
  uint32_t v = 0;
  for (uint32_t k = 0; k < 4; k++) v += tile_rec_count(tiles, i0 + k, n);
  part[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t st = 128; st; st >>= 1) {
    if (threadIdx.x < st) part[threadIdx.x] += part[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = part[0];
}
// one block: bsum[0, nb) -> exclusive offsets in place; total records in *total
__global__ void __launch_bounds__(1024) rec_scan_sums_kernel(uint32_t* bsum, uint32_t nb, uint32_t* total) {
  __shared__ uint32_t sh[1024];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nb; base += 1024u) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < nb ? bsum[i] : 0u;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {
      const uint32_t add = threadIdx.x >= d ? sh[threadIdx.x - d] : 0u;
      __syncthreads();
      sh[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < nb) bsum[i] = carry + sh[threadIdx.x] - v;
    carry += sh[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ void __launch_bounds__(256) rec_compact_kernel(const TileOut* tiles, uint32_t n, const uint32_t* bsum,
                                                          const Rec* src, Rec* dst, uint32_t* dense_off) {
  __shared__ uint32_t sh[256];
  const uint32_t i0 = blockIdx.x * kScanTiles + threadIdx.x * 4u;
  uint32_t c[4], v = 0;
  for (uint32_t k = 0; k < 4; k++) { c[k] = tile_rec_count(tiles, i0 + k, n); v += c[k]; }
  sh[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t d = 1; d < 256u; d <<= 1) {
    const uint32_t add = threadIdx.x >= d ? sh[threadIdx.x - d] : 0u;
    __syncthreads();
    sh[threadIdx.x] += add;
    __syncthreads();
  }
  uint32_t off = bsum[blockIdx.x] + sh[threadIdx.x] - v;
  for (uint32_t k = 0; k < 4; k++) {
    const uint32_t i = i0 + k;
    if (i >= n) break;
    dense_off[i] = off;
    const TileOut t = tiles[i];
    const uint32_t stride = t.pad1 > 1u ? t.pad1 : 1u;
    for (uint32_t r = 0; r < c[k]; r++) dst[off + r] = src[t.rec_off + (size_t)r * stride];
    off += c[k];
  }
}

// Packs the host arena (32 B DNode) into the device arena (16 B DNodeP + key-length column) and the
// parent column the device reporter walks.
// bad[0] = 1: a count past 2^28; 2: a map entry whose key offset is not its key id.
__global__ void __launch_bounds__(256) pack_nodes_kernel(const DNode* in, DNodeP* out, uint32_t* klen, uint32_t* parent,
                                                         uint64_t n, uint32_t* bad) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const DNode d = in[i];
    if (d.count > kMaxPackedCount) atomicOr(bad, 1u);
    if (d.key_off != NONE && d.key_off != d.key_hash) atomicOr(bad, 2u);
    // the regex memo (eval_core.inc regex_match_ref) is keyed by a string's 16-byte pool slot
    if (d.kind == K_STRING && (d.a & 15u)) atomicOr(bad, 4u);
    DNodeP p;
    p.kc = d.kind | (d.count << 4); p.a = d.a; p.b = d.b; p.key_hash = d.key_off != NONE ? d.key_hash : 0u;
    out[i] = p;
    klen[i] = d.key_off != NONE ? d.key_len : 0u;
    parent[i] = d.parent;   // the device reporter's JSON pointers (report_gpu.hip)
  }
}

}  // namespace gg
#endif  // !GG_NFA
