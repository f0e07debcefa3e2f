// Shape-sorted document order (capi.cpp session_upload): the documents of each of 8 contiguous segments
// (one per XCD's share of the lane batches) stably sorted by their 64-bit shape key, on the device -- a
// segmented radix sort of (key, document) pairs (hipCUB over rocPRIM), instead of host threads whose
// comparator reads the key array at random.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_segmented_radix_sort.hpp>

#include "dev_cache.h"

#include <stdexcept>
#include <string>

namespace gg {

namespace {
__global__ void iota_kernel(uint32_t* v, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = i;
}
void chk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e) + " at " + what);
}
}  // namespace

// order[0, n) := documents sorted by key within each segment [seg[k], seg[k + 1]) (k < nseg), ties in
// document order.  key: n device keys (overwritten as scratch is not needed: read only); order: n device
// slots.  Synchronous on `st` when it returns.
void device_segmented_order(const unsigned long long* key, uint32_t* order, uint32_t n, const uint32_t* seg_host,
                            uint32_t nseg, hipStream_t st) {
  if (!n) return;
  uint32_t *vals_in = nullptr, *d_seg = nullptr;
  unsigned long long* keys_out = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  struct Free {
    void** p[4];
    ~Free() { for (auto q : p) gg::dev_free(*q); }
  } fr{{(void**)&vals_in, (void**)&d_seg, (void**)&keys_out, &tmp}};
  chk(gg::dev_alloc(&vals_in, (size_t)n * 4), "order values");
  chk(gg::dev_alloc(&keys_out, (size_t)n * 8), "order keys");
  chk(gg::dev_alloc(&d_seg, (size_t)(nseg + 1) * 4), "order segments");
  chk(hipMemcpyAsync(d_seg, seg_host, (size_t)(nseg + 1) * 4, hipMemcpyHostToDevice, st), "order segments H2D");
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096), dim3(256), 0, st, vals_in, n);
  chk(hipGetLastError(), "iota_kernel");
  chk(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tmp_bytes, key, keys_out, vals_in, order, (int)n, (int)nseg,
                                                  d_seg, d_seg + 1, 0, 64, st),
      "segmented sort (size)");
  chk(gg::dev_alloc(&tmp, tmp_bytes ? tmp_bytes : 1), "segmented sort scratch");
  chk(hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tmp_bytes, key, keys_out, vals_in, order, (int)n, (int)nseg,
                                                  d_seg, d_seg + 1, 0, 64, st),
      "segmented sort");
  chk(hipStreamSynchronize(st), "segmented sort");
}

}  // namespace gg
