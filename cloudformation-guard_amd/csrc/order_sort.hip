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
  // fenced on `st`: an error thrown between the launches and the final synchronisation leaves work queued
  struct Free {
    void** p[4];
    hipStream_t s;
    ~Free() { for (auto q : p) gg::dev_free_on(*q, s); }
  } fr{{(void**)&vals_in, (void**)&d_seg, (void**)&keys_out, &tmp}, st};
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

namespace gg {
namespace {
// Device-to-host copy by the shader (GG_D2H_PUSH=1): each thread reads 16 bytes of the device text (from a
// 4-byte aligned base, funnel-shifted when the source is not 16-byte aligned) and writes them to the pinned
// destination with one 16-byte nontemporal store; the last partial group is written byte by byte.  The
// SDMA engine a copy queue lands on was measured at 27 to 57 GB/s from process to process
// (profiles/r05zb_*); the shader path does not depend on it.
__global__ void __launch_bounds__(256) d2h_push_kernel(const uint32_t* __restrict__ src_base, uint32_t shift_bits,
                                                      const unsigned char* __restrict__ src, uint4* dst,
                                                      size_t n16, size_t nbytes) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t nwords = (nbytes + (shift_bits >> 3) + 3) / 4;   // readable words from src_base
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const size_t w = 4 * i;
    uint32_t a[5];
#pragma unroll
    for (int k = 0; k < 5; k++) a[k] = (w + k < nwords) ? src_base[w + k] : 0u;
    uint4 o;
    if (shift_bits) {
      o.x = __builtin_amdgcn_alignbit(a[1], a[0], shift_bits);
      o.y = __builtin_amdgcn_alignbit(a[2], a[1], shift_bits);
      o.z = __builtin_amdgcn_alignbit(a[3], a[2], shift_bits);
      o.w = __builtin_amdgcn_alignbit(a[4], a[3], shift_bits);
    } else {
      o = make_uint4(a[0], a[1], a[2], a[3]);
    }
    __builtin_nontemporal_store(o.x, &dst[i].x);
    __builtin_nontemporal_store(o.y, &dst[i].y);
    __builtin_nontemporal_store(o.z, &dst[i].z);
    __builtin_nontemporal_store(o.w, &dst[i].w);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (size_t b = n16 * 16; b < nbytes; b++) ((unsigned char*)dst)[b] = src[b];
}
}  // namespace

// bytes from device `src` to pinned host `dst` (device-accessible), enqueued on `st`
void d2h_push(void* dst, const void* src, size_t bytes, hipStream_t st, int blocks) {
  if (!bytes) return;
  const uintptr_t s = (uintptr_t)src;
  const uint32_t* base = (const uint32_t*)(s & ~(uintptr_t)3);
  const uint32_t shift_bits = (uint32_t)(s & 3) * 8;
  const size_t n16 = bytes / 16;
  hipLaunchKernelGGL(d2h_push_kernel, dim3(blocks), dim3(256), 0, st, base, shift_bits, (const unsigned char*)src,
                     (uint4*)dst, n16, bytes);
}
}  // namespace gg
