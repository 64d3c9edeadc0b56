// prims.hpp — device primitives shared by the hot-path kernels (gfx950):
// stream-ordered caching allocator, exclusive scan (u32/u64), stable LSD radix
// sort of (u32 key, u32 value) pairs. Hand-written HIP, wave64 idioms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstddef>

namespace pmd {

// Caching device allocator: freed blocks are kept and reused in stream order
// (per-(device, stream) pools, see prims.hip), so timed loops do not hipMalloc.
// Blocks come from the calling thread's current device.
void* dev_alloc(size_t bytes);
// The device of a stream (the current device for the null stream).
int stream_device(hipStream_t s);
// One entry point's scope: makes `s`'s device (or `device` if >= 0) current
// for the calling thread and `s` the stream of its dev_alloc / dev_free, and
// restores both on exit (RAII). A host thread that never called hipSetDevice
// is on device 0; this keeps every allocation and launch of a call on the
// device of the stream it was given.
struct AllocStream {
  hipStream_t prev;
  int dev = 0;        // the call's device
  int restore = -1;   // device to make current again on exit (-1: unchanged)
  explicit AllocStream(hipStream_t s, int device = -1);
  ~AllocStream();
  AllocStream(const AllocStream&) = delete;
  AllocStream& operator=(const AllocStream&) = delete;
};
void dev_free(void* p);
// Bytes held by live blocks and by idle pooled blocks of device `dev` (-1: all).
void dev_pool_stats(int dev, size_t* live, size_t* cached);
// The process-wide side stream `idx` of a device (created on first use): 0
// the render's caustic gather, 1 the global gather's box build.
hipStream_t side_stream(int dev, int idx = 0);
void dev_cache_trim();

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  explicit DevBuf(size_t count) { alloc(count); }
  ~DevBuf() { reset(); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  void alloc(size_t count) {
    reset();
    n = count;
    p = count ? static_cast<T*>(dev_alloc(count * sizeof(T))) : nullptr;
  }
  void reset() {
    if (p) dev_free(p);
    p = nullptr;
    n = 0;
  }
  T* get() const { return p; }
};

// out[i] = sum_{j<i} in[j]; if total != nullptr, *total (device) = sum of all.
hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total, hipStream_t s);
hipError_t exclusive_scan_u64(const uint64_t* in, uint64_t* out, int64_t n, uint64_t* total, hipStream_t s);

// Stable LSD radix sort on key bits [0, end_bit). Sorted data ends in keys/vals.
hipError_t radix_sort_pairs(uint32_t* keys, uint32_t* vals, int64_t n, int end_bit, hipStream_t s);
// The kd presort: stable sort of positions 0..n-1 by 32-bit keys (read-only),
// writing elems[i] of the sorted positions as four SoA arrays (x, y, z, w). The
// first pass takes the positions implicitly, the last one gathers the elements.
struct SoaOut {
  float* c[4];
};
hipError_t radix_sort_gather_soa(const uint32_t* keys, int64_t n, const float4* elems, const SoaOut& out,
                                 hipStream_t s);

// float -> uint32 whose unsigned order == float order, with -0 == +0.
__host__ __device__ inline uint32_t orderable_key(float f) {
  if (f == 0.0f) f = 0.0f;
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

inline int grid_for(int64_t n, int block) { return (int)((n + block - 1) / block); }

}  // namespace pmd

#define PM_HIP_TRY(expr)                         \
  do {                                           \
    hipError_t _e = (expr);                      \
    if (_e != hipSuccess) return _e;             \
  } while (0)
