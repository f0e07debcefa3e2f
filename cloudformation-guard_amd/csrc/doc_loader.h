// Document loader: YAML/JSON text -> columnar node arena (host side, then uploaded to HBM).
//
// Replaces the reference's document model construction:
//   Loader::load                       guard/src/rules/libyaml/loader.rs:31-195
//   PathAwareValue::try_from(Marked)   guard/src/rules/path_value.rs:414-478
//   build_data_file                    guard/src/commands/validate.rs:760-787
//   run_checks' serde loader           guard/src/commands/helper.rs:30-42
// The YAML event stream comes from libyaml 0.2.5 (the reference links unsafe-libyaml 0.2.11,
// a transpile of the same C library).
#pragma once
#include <sys/mman.h>

#include <memory>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "guard_types.h"

namespace gg {

// Large host buffers (arena columns: tens of GB at 1M templates; report text: ~150 KB per template)
// are fresh memory the first time they are written, and first-touch page faults on 4 KB pages
// serialise in the kernel: on the MI355X box 16 threads fault fresh memory in at ~15 GB/s, against
// ~200 GB/s with transparent huge pages (tools/prof/fault_bench.c; THP is in `madvise` mode there).
// Buffers from kHugeMin up are mmap'd and marked MADV_HUGEPAGE before anything touches them.
constexpr size_t kHugeMin = 4u << 20;
inline void* huge_alloc(size_t bytes) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  madvise(p, bytes, MADV_HUGEPAGE);
  return p;
}
inline void huge_free(void* p, size_t bytes) { if (p) munmap(p, bytes); }

// Allocator whose value-less construct() default-initialises: resize() of the arena columns (trivial
// element types, every element written right after) skips the zero fill.  At 1M templates the
// columns are ~29 GB, so zero-filling them before the copy doubled the loader's memory traffic.
template <class T>
struct default_init_allocator : std::allocator<T> {
  template <class U> struct rebind { using other = default_init_allocator<U>; };
  using std::allocator<T>::allocator;
  template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
  template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
  // huge-page backed from kHugeMin bytes up (see huge_alloc)
  T* allocate(size_t n) {
    const size_t b = n * sizeof(T);
    return b >= kHugeMin ? (T*)huge_alloc(b) : std::allocator<T>::allocate(n);
  }
  void deallocate(T* p, size_t n) {
    const size_t b = n * sizeof(T);
    if (b >= kHugeMin) huge_free(p, b); else std::allocator<T>::deallocate(p, n);
  }
};
template <class T>
using column = std::vector<T, default_init_allocator<T>>;

// Append-only once a device copy exists: the device loader keeps its HBM copy of nodes[0, n) (and a
// resident arena keeps every column there, capi.cpp ensure_host_arena), and the session's next upload
// packs the evaluator's arena from that copy while the reporter reads the host columns.  Mutators may
// append documents (merge_batches, merge_into_last, grow_zeroed past the end) but must not rewrite an
// existing node; a path that did would have to drop the device copy (gg_session dev_nodes) first.
struct DocBatch {
  column<DNode> nodes;
  std::string bytes;
  column<uint32_t> line, col;            // per node mark (PathAwareValue location)
  column<uint32_t> kline, kcol;          // per map-entry node: its key's mark
  // Node indices inside a document are DOCUMENT-RELATIVE (child/parent fields, roots, records):
  // doc k's nodes are nodes[base[k] .. base[k+1]) and its root is nodes[base[k] + roots[k]].
  // The literal arena of a compiled rules file has no `base` (one implicit document at 0).
  std::vector<uint32_t> roots;           // per document: root node (relative; 0 for loaded docs)
  std::vector<uint64_t> base;            // per document: global index of its first node
  std::vector<std::string> names;        // per document: data file name
  bool serde = false;                    // loaded by the serde (FFI) loader: key paths differ
  // string pool interning: map keys and string scalars repeat heavily across templates
  // ("Properties", "Type", "AWS::S3::Bucket"), so each distinct string is stored once per batch.
  // Offsets are u32: a batch's pool is capped at kMaxPoolBytes (load_document fails beyond it).
  std::vector<uint32_t> islots;          // open addressing: pool offset + 1 (0 = empty)
  std::vector<uint32_t> ilen;            // parallel to islots: string length
  size_t iused = 0;
  // The pool holds each distinct string once per batch (merge_batches re-interns per-thread
  // parts), so a string's pool offset is its id: DNode.b of a string and DNode.key_hash of a map
  // entry carry that id, and the device tests string equality by comparing ids.
  uint32_t intern(const char* p, uint32_t n, uint32_t hash);
  void intern_reserve();                 // grows islots before one more insertion
  uint32_t find(const char* p, uint32_t n) const;   // pool offset of an interned string, or NONE
  // indexes a string already in the pool at `off` (a pool built on the device, json_gpu.hip)
  void adopt(uint32_t off, uint32_t n);
  // adopt() for n strings at once on `threads` host threads: the index is sized once and filled by
  // concurrent linear-probing inserts (compare-and-swap on the slot; no deletions, so every string sits
  // at the first free slot from its hash at its insertion and find() reaches it)
  void adopt_bulk(const uint32_t* off, const uint32_t* len, size_t n, unsigned threads);

  // resizes every per-node column to s nodes, zero-filling new nodes (the columns default-initialise;
  // loaders that do not write every field of a new node use this)
  void grow_zeroed(size_t s) {
    const size_t o = nodes.size();
    nodes.resize(s); line.resize(s); col.resize(s); kline.resize(s); kcol.resize(s);
    for (size_t i = o; i < s; i++) { nodes[i] = DNode{}; line[i] = col[i] = kline[i] = kcol[i] = 0; }
  }
  size_t ndocs() const { return roots.size(); }
  std::string path(uint64_t base, uint32_t node) const;  // JSON pointer ("" for a root)
  std::string path_display(uint64_t base, uint32_t node) const;  // "{pointer}[L:{line},C:{col}]"
  void clear();
};

constexpr size_t kMaxPoolBytes = 0xF0000000u;
constexpr size_t kMaxDocNodes = 0x1FFFFFFFu;   // relative refs share a u32 with the LIT/SYN/KEY flag bits

enum LoadMode { LOAD_LIBYAML = 0, LOAD_SERDE = 1 };

struct LoadError { std::string kind, msg; };

// strict-JSON documents skip libyaml (identical arena; see doc_loader.cpp); tests switch it off
extern bool g_json_fast;
int loader_selfcheck(const char* text, size_t len);

// Appends one document; returns false and fills err on failure (batch unchanged).
bool load_document(DocBatch& b, const char* text, size_t len, const std::string& name,
                   LoadMode mode, LoadError& err);

// kline flag of a map entry: the entry's key PathAwareValue has the map's path + "/key" at the
// location kept in kline/kcol (keys PathAwareValue::merge pushes, path_value.rs:905-907), not the
// map's path at the key's own mark (path_value.rs:459-466)
constexpr uint32_t kKeyPathExt = 0x80000000u;

// `cfn-guard validate -i`: PathAwareValue::merge (path_value.rs:889-919) of `self` = document `pd`
// of P (the input parameters) with `other` = document d of b, which must be b's last document.
// The merged value is built in place after d's nodes (d's own nodes are not touched) and becomes d's
// root (b.roots[d]).  Returns false with err = MultipleValues / IncompatibleError (the reference's
// messages) and b unchanged.
bool merge_into_last(DocBatch& b, size_t d, const DocBatch& P, size_t pd, LoadError& err);

}  // namespace gg
