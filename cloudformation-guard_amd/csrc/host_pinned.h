// Pinned host memory on the NUMA node of a device (the DMA staging of report copies and text uploads).
//
// hipHostMalloc places its pages wherever the calling thread happens to run: on a two-socket host a
// staging buffer on the far socket moves every device-to-host byte across the inter-socket link as well
// as PCIe.  pinned_alloc maps the pages itself, binds them to the device's node (the PCI device's
// numa_node in sysfs), touches them there and registers them with the runtime; without a known node, or
// when any step fails, it falls back to hipHostMalloc.  GG_PINNED_NUMA=0 turns the placement off (A/B).
// The policy is MPOL_PREFERRED: a node short of free memory places the pages elsewhere instead of
// making the first touch reclaim or fail there.
#pragma once

#include <hip/hip_runtime.h>
#include <numaif.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace gg {

// the NUMA node of HIP device `dev` (-1: unknown / single node)
inline int device_numa_node(int dev) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return -1;
  for (char* p = bus; *p; p++) *p = (char)tolower(*p);
  char path[160];
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

struct PinnedRegistry {
  std::mutex mu;
  std::unordered_map<void*, size_t> mapped;   // pinned_alloc'd by mmap + hipHostRegister: bytes
  static PinnedRegistry& get() { static PinnedRegistry r; return r; }
};

inline void* pinned_alloc(size_t bytes, int dev) {
  const char* e = getenv("GG_PINNED_NUMA");
  const int node = (e && atoi(e) == 0) ? -1 : device_numa_node(dev);
  if (getenv("GG_PINNED_TRACE")) fprintf(stderr, "[pinned] %zu bytes for device %d: NUMA node %d\n", bytes, dev, node);
  if (node >= 0 && node < 64) {
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p != MAP_FAILED) {
      unsigned long mask = 1ul << node;
      bool ok = syscall(SYS_mbind, p, bytes, MPOL_PREFERRED, &mask, 64ul, 0u) == 0;
      if (ok) memset(p, 0, bytes);   // first touch: the pages are allocated on the node now
      if (ok) ok = hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess;
      if (ok) {
        PinnedRegistry& r = PinnedRegistry::get();
        std::lock_guard<std::mutex> lk(r.mu);
        r.mapped[p] = bytes;
        return p;
      }
      munmap(p, bytes);
    }
  }
  void* q = nullptr;
  if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return q;
}

inline void pinned_free(void* p) {
  if (!p) return;
  size_t bytes = 0;
  {
    PinnedRegistry& r = PinnedRegistry::get();
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.mapped.find(p);
    if (it != r.mapped.end()) { bytes = it->second; r.mapped.erase(it); }
  }
  if (bytes) {
    (void)hipHostUnregister(p);
    munmap(p, bytes);
  } else {
    (void)hipHostFree(p);
  }
}

// Process-wide cache of pinned blocks by (device, size): the streamed entries take their staging and chunk
// blocks here and give them back at the end of the call instead of unpinning them (pinning 256 MB costs
// ~0.1 s, and the report copy-out of the sessions after a call that unpinned its staging was measured at
// half the rate, profiles/r05x_report_ab.log).  At most GG_PINNED_CACHE_GB per device stay cached (default
// 2: the one-device stream's 256 MB staging, the device loader's two 64 MB bounce buffers per load, and a
// device-list stream's working set of 64 MB blocks); page-
// locked memory is invisible to the rest of the host, so gg_device_cache_release hands it back too
// (pinned_cache_flush).
struct PinnedCache {
  size_t cap;
  std::mutex mu;
  std::unordered_map<uint64_t, std::vector<void*>> free;   // (device << 48 | bytes) -> blocks
  std::unordered_map<int, size_t> cached;                  // device -> bytes in `free`
  PinnedCache() {
    const char* e = getenv("GG_PINNED_CACHE_GB");
    const double gb = e ? atof(e) : 2.0;
    cap = gb > 0 ? (size_t)(gb * (double)(1ull << 30)) : 0;
  }
  static PinnedCache& get() { static PinnedCache* c = new PinnedCache; return *c; }
};
inline void* pinned_get(size_t bytes, int dev) {
  PinnedCache& c = PinnedCache::get();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.free.find(((uint64_t)dev << 48) | bytes);
    if (it != c.free.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      c.cached[dev] -= bytes;
      return p;
    }
  }
  return pinned_alloc(bytes, dev);
}
inline void pinned_put(void* p, size_t bytes, int dev) {
  if (!p) return;
  PinnedCache& c = PinnedCache::get();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.cached[dev] + bytes <= c.cap) {
      c.free[((uint64_t)dev << 48) | bytes].push_back(p);
      c.cached[dev] += bytes;
      return;
    }
  }
  pinned_free(p);
}
// unpins and frees the cached blocks of `dev` (-1: every device); returns the bytes released
inline size_t pinned_cache_flush(int dev) {
  PinnedCache& c = PinnedCache::get();
  std::vector<void*> out;
  size_t bytes = 0;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto it = c.free.begin(); it != c.free.end();) {
      const int d = (int)(it->first >> 48);
      if (dev >= 0 && d != dev) { ++it; continue; }
      const size_t b = (size_t)(it->first & ((1ull << 48) - 1));
      for (void* p : it->second) { out.push_back(p); bytes += b; }
      c.cached[d] = 0;
      it = c.free.erase(it);
    }
  }
  for (void* p : out) pinned_free(p);
  return bytes;
}

}  // namespace gg
