// Device allocations through a per-device cache of freed blocks.
//
// hipFree waits for the whole device to go idle.  The streamed batch (cfn_guard_validate_batch_stream)
// loads chunk k+1 and tears down chunk k-1's session while chunk k's report kernels and copies run on
// another thread: every hipFree of a loader temporary or a session buffer waited for that report.
// dev_free puts a block on its device's free list instead (the caller has synchronised every stream
// that used it, as before a hipFree); dev_free_on(p, stream) is for a caller that may still have work
// queued on `stream` (an exception unwinding past a loader pass): it records an event there, and the block
// is handed out again only once that event has completed -- the ordering hipFree enforced device-wide,
// enforced per block.  dev_alloc takes a cached block of the same size class whose fence (if any) has
// passed before calling hipMalloc.  A hipMalloc that fails empties the device's list and tries once more.
// GG_DEV_CACHE_GB bounds the bytes a device's list holds (default 48; 0 turns the cache off).  Memory held
// here is invisible to the HIP runtime and to torch's allocator in the same process, so the default stays
// well under the 288 GB of one MI355X -- but above one streamed chunk's buffer set (262 144 templates: ~25 GB
// of lane heaps, record arena and arena columns): with 16 GB the rest of every torn-down set went to hipFree,
// which waits for the device to go idle (the other chunk's report), and the next chunk hipMalloc'd it again.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace gg {

struct DevCache {
  static constexpr int kDevs = 64;
  struct Block { void* p; hipEvent_t fence; };   // fence: null, or the event the block waits for
  std::mutex mu;
  std::multimap<size_t, Block> free_list[kDevs];
  std::vector<hipEvent_t> spare_events[kDevs];
  size_t held[kDevs] = {};
  std::unordered_map<void*, std::pair<int, size_t>> live;   // block -> (device, class bytes)
  size_t cap = 0;
  DevCache() {
    const char* e = getenv("GG_DEV_CACHE_GB");
    // the cap is parsed as a double and scaled before the conversion (GG_DEV_CACHE_GB=0.5 is 512 MB)
    const double gb = e ? atof(e) : 48.0;
    cap = gb > 0 ? (size_t)(gb * (double)(1ull << 30)) : 0;
  }
};

// never destroyed: blocks still cached at exit go with the process (a static destructor calling
// hipFree after the runtime's own teardown is undefined)
inline DevCache& dev_cache() {
  static DevCache* c = new DevCache;
  return *c;
}

// size classes: 8 per octave above 4 KB (at most 12.5% over the request), 256-byte steps below
inline size_t dev_cache_class(size_t b) {
  if (b <= 4096) return (b + 255) & ~(size_t)255;
  size_t p = 1;
  while (p < b) p <<= 1;
  const size_t step = p / 16;
  return (b + step - 1) / step * step;
}

inline size_t dev_cache_held(int dev) {
  DevCache& C = dev_cache();
  std::lock_guard<std::mutex> lk(C.mu);
  return C.held[dev];
}

inline void dev_cache_flush(int dev) {
  DevCache& C = dev_cache();
  std::vector<DevCache::Block> out;
  {
    std::lock_guard<std::mutex> lk(C.mu);
    for (auto& kv : C.free_list[dev]) out.push_back(kv.second);
    C.free_list[dev].clear();
    C.held[dev] = 0;
  }
  for (auto& b : out) {
    if (b.fence) { (void)hipEventSynchronize(b.fence); (void)hipEventDestroy(b.fence); }
    (void)hipFree(b.p);
  }
}

inline hipError_t dev_alloc(void** out, size_t bytes) {
  DevCache& C = dev_cache();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= DevCache::kDevs) dev = 0;
  const size_t c = dev_cache_class(bytes ? bytes : 1);
  {
    std::lock_guard<std::mutex> lk(C.mu);
    auto& fl = C.free_list[dev];
    // the smallest cached block of this class or up to 1.5 x larger: a streamed batch's last, smaller chunk
    // (or any chunk whose counts land a class lower) takes the previous chunk's blocks instead of hipMalloc'ing
    // ~20 GB afresh (2.2-3.8 s, profiles/r06zk_stream_trace.log); the block keeps its own class
    for (auto it = fl.lower_bound(c); it != fl.end() && it->first <= c + c / 2; ++it) {
      // a fenced block is taken only once the work queued before its dev_free_on has completed
      if (it->second.fence) {
        if (hipEventQuery(it->second.fence) != hipSuccess) { (void)hipGetLastError(); continue; }
        C.spare_events[dev].push_back(it->second.fence);
      }
      const size_t have = it->first;
      *out = it->second.p;
      C.held[dev] -= have;
      fl.erase(it);
      C.live[*out] = {dev, have};
      return hipSuccess;
    }
  }
  void* p = nullptr;
  // GG_ALLOC_TRACE=<MB>: every cache miss of at least that size on stderr, with the hipMalloc's wall time
  static const long trace_mb = getenv("GG_ALLOC_TRACE") ? atol(getenv("GG_ALLOC_TRACE")) : -1;
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipMalloc(&p, c);
  if (trace_mb >= 0 && c >= ((size_t)trace_mb << 20)) {
    size_t cached = 0, near = 0;
    {
      std::lock_guard<std::mutex> lk(C.mu);
      cached = C.held[dev];
      auto it = C.free_list[dev].lower_bound(c / 2);
      if (it != C.free_list[dev].end()) near = it->first;
    }
    fprintf(stderr, "[alloc] miss %zu MB on device %d: hipMalloc %.1f ms (cache holds %zu MB, next class >= half: %zu MB)\n",
            c >> 20, dev, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
            cached >> 20, near >> 20);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    dev_cache_flush(dev);
    e = hipMalloc(&p, c);
    if (e != hipSuccess) return e;
  }
  std::lock_guard<std::mutex> lk(C.mu);
  C.live[p] = {dev, c};
  *out = p;
  return hipSuccess;
}

template <class T>
inline hipError_t dev_alloc(T** out, size_t bytes) {
  void* p = nullptr;
  const hipError_t e = dev_alloc(&p, bytes);
  *out = (T*)p;
  return e;
}

// p: from dev_alloc (or null).  fenced: work that may use p is still queued on `stream` (the device current
// on this thread): the block is cached behind an event recorded there; otherwise no stream may still use it.
inline void dev_free_impl(void* p, bool fenced, hipStream_t stream) {
  if (!p) return;
  DevCache& C = dev_cache();
  {
    std::lock_guard<std::mutex> lk(C.mu);
    auto it = C.live.find(p);
    if (it != C.live.end()) {
      const int dev = it->second.first;
      const size_t c = it->second.second;
      C.live.erase(it);
      if (C.held[dev] + c <= C.cap) {
        hipEvent_t ev = nullptr;
        if (fenced) {
          if (!C.spare_events[dev].empty()) { ev = C.spare_events[dev].back(); C.spare_events[dev].pop_back(); }
          else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
          if (!ev || hipEventRecord(ev, stream) != hipSuccess) {
            // no fence could be placed: hipFree's device-wide wait instead of a block of unknown state
            if (ev) (void)hipEventDestroy(ev);
            (void)hipGetLastError();
            goto release;
          }
        }
        C.free_list[dev].emplace(c, DevCache::Block{p, ev});
        C.held[dev] += c;
        return;
      }
    }
  }
release:
  (void)hipFree(p);
}
inline void dev_free(void* p) { dev_free_impl(p, false, nullptr); }
inline void dev_free_on(void* p, hipStream_t stream) { dev_free_impl(p, true, stream); }

// p: from dev_alloc (or null), possibly still in use by queued work: hipFree's device-wide wait
inline void dev_free_sync(void* p) {
  if (!p) return;
  {
    DevCache& C = dev_cache();
    std::lock_guard<std::mutex> lk(C.mu);
    C.live.erase(p);
  }
  (void)hipFree(p);
}

}  // namespace gg
