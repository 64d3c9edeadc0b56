// prims.hip — caching allocator, exclusive scan, stable radix sort (gfx950).
#include <map>
#include <mutex>
#include <unordered_map>

#include "prims.hpp"

namespace pmd {

// ------------------------------------------------------------ allocator
// Free blocks are pooled per (device, stream): a block returns to the pool of
// the stream that is current (AllocStream) when it is freed, and is handed out
// again only to work on that stream of its own device, so stream order makes
// reuse safe even when two host threads drive two streams (pm_render_begin
// beside the photon trace), and a block never crosses to another GPU when one
// process drives several. A block that outlives an entry point is idle when
// freed (every entry point synchronises its stream), so its pool does not
// matter.
namespace {
struct PoolKey {
  int dev;
  hipStream_t s;
  size_t sz;
  bool operator<(const PoolKey& o) const {
    if (dev != o.dev) return dev < o.dev;
    if (s != o.s) return s < o.s;
    return sz < o.sz;
  }
};
struct Live {
  size_t sz;
  int dev;
};
std::mutex g_mu;
std::multimap<PoolKey, void*> g_free;    // (device, stream, size) -> block
std::unordered_map<void*, Live> g_live;  // block -> (size, device)
thread_local hipStream_t t_stream = nullptr;
size_t round_up(size_t b) {
  size_t r = 256;
  while (r < b) r <<= 1;
  return r;
}
int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) {
    (void)hipGetLastError();
    d = 0;
  }
  return d;
}
}  // namespace

int stream_device(hipStream_t s) {
  if (!s) return current_device();
  hipDevice_t d = 0;
  if (hipStreamGetDevice(s, &d) != hipSuccess) {
    (void)hipGetLastError();
    return current_device();
  }
  return (int)d;
}

AllocStream::AllocStream(hipStream_t s, int device) : prev(t_stream) {
  const int cur = current_device();
  dev = device >= 0 ? device : stream_device(s);
  if (dev != cur && hipSetDevice(dev) == hipSuccess) restore = cur;
  t_stream = s;
}
AllocStream::~AllocStream() {
  t_stream = prev;
  if (restore >= 0) (void)hipSetDevice(restore);
}

void* dev_alloc(size_t bytes) {
  const size_t sz = round_up(bytes ? bytes : 1);
  const int dev = current_device();
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_free.find(PoolKey{dev, t_stream, sz});
    if (it != g_free.end()) {
      void* p = it->second;
      g_free.erase(it);
      g_live[p] = Live{sz, dev};
      return p;
    }
  }
  void* p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) {
    (void)hipGetLastError();
    dev_cache_trim();
    if (hipMalloc(&p, sz) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_live[p] = Live{sz, dev};
  return p;
}

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_live.find(p);
  if (it == g_live.end()) return;
  g_free.emplace(PoolKey{it->second.dev, t_stream, it->second.sz}, p);
  g_live.erase(it);
}

// Releases the current device's idle blocks (after an out-of-memory).
void dev_cache_trim() {
  const int dev = current_device();
  (void)hipDeviceSynchronize();
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto it = g_free.begin(); it != g_free.end();) {
    if (it->first.dev == dev) {
      (void)hipFree(it->second);
      it = g_free.erase(it);
    } else {
      ++it;
    }
  }
}

void dev_pool_stats(int dev, size_t* live, size_t* cached) {
  std::lock_guard<std::mutex> lk(g_mu);
  size_t l = 0, c = 0;
  for (const auto& kv : g_live)
    if (dev < 0 || kv.second.dev == dev) l += kv.second.sz;
  for (const auto& kv : g_free)
    if (dev < 0 || kv.first.dev == dev) c += kv.first.sz;
  if (live) *live = l;
  if (cached) *cached = c;
}

// One non-blocking side stream per device for the life of the process (the
// render's caustic gather): its allocator pool then persists from frame to
// frame (a per-job stream took its temporaries' pool with it).
hipStream_t side_stream(int dev, int idx) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, hipStream_t> streams;
  std::lock_guard<std::mutex> lk(mu);
  const std::pair<int, int> key{dev, idx};
  auto it = streams.find(key);
  if (it != streams.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  streams[key] = s;
  return s;
}

// ------------------------------------------------------------ scan
constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanBlock * kScanItems;

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// block exclusive scan of one value per thread; returns exclusive prefix, *tot = block total
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T& tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int i = 0; i < kScanBlock / 64; i++) {
      T t = sh[i];
      sh[i] = run;
      run += t;
    }
    sh[kScanBlock / 64] = run;
  }
  __syncthreads();
  T r = inc - v + sh[w];
  tot = sh[kScanBlock / 64];
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(const T* in, int64_t n, T* bsum) {
  __shared__ T sh[kScanBlock / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  T acc = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    int64_t i = base + (int64_t)k * kScanBlock + threadIdx.x;
    if (i < n) acc += in[i];
  }
  T tot;
  (void)block_excl_scan<T>(acc, sh, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

template <typename T>
__global__ __launch_bounds__(kScanBlock) void k_scan_down(const T* in, T* out, int64_t n, const T* boff, T* total,
                                                          int nblocks) {
  __shared__ T sh[kScanBlock / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  // each thread owns kScanItems consecutive elements
  T v[kScanItems];
  T acc = 0;
  const int64_t mine = base + (int64_t)threadIdx.x * kScanItems;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    int64_t i = mine + k;
    v[k] = i < n ? in[i] : (T)0;
    acc += v[k];
  }
  T tot;
  T pre = block_excl_scan<T>(acc, sh, tot) + (boff ? boff[blockIdx.x] : (T)0);
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    int64_t i = mine + k;
    if (i < n) out[i] = pre;
    pre += v[k];
  }
  if (total && blockIdx.x == nblocks - 1 && threadIdx.x == kScanBlock - 1) *total = pre;
}

template <typename T>
static hipError_t scan_impl(const T* in, T* out, int64_t n, T* total, hipStream_t s) {
  if (n <= 0) {
    if (total) PM_HIP_TRY(hipMemsetAsync(total, 0, sizeof(T), s));
    return hipSuccess;
  }
  const int nb = (int)((n + kScanTile - 1) / kScanTile);
  if (nb == 1) {
    k_scan_down<T><<<1, kScanBlock, 0, s>>>(in, out, n, nullptr, total, 1);
    return hipGetLastError();
  }
  DevBuf<T> bsum(nb), boff(nb);
  if (!bsum.p || !boff.p) return hipErrorOutOfMemory;
  k_scan_reduce<T><<<nb, kScanBlock, 0, s>>>(in, n, bsum.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(scan_impl<T>(bsum.p, boff.p, nb, nullptr, s));
  k_scan_down<T><<<nb, kScanBlock, 0, s>>>(in, out, n, boff.p, total, nb);
  return hipGetLastError();
}

hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total, hipStream_t s) {
  return scan_impl<uint32_t>(in, out, n, total, s);
}
hipError_t exclusive_scan_u64(const uint64_t* in, uint64_t* out, int64_t n, uint64_t* total, hipStream_t s) {
  return scan_impl<uint64_t>(in, out, n, total, s);
}

// ------------------------------------------------------------ radix sort
// 8-bit digits; tile = 256 threads x 8 rounds. Histogram -> digit-major scan
// -> stable scatter with wave64 ballot multi-split ranking.
constexpr int kSortBlock = 256;
constexpr int kSortRounds = 16;   // 4096 keys per tile: ~16 per digit run on write-out
constexpr int kSortTile = kSortBlock * kSortRounds;

// Per-tile digit histogram: 16 consecutive keys per thread (four 16-B loads),
// per-wave sub-histograms in LDS (less atomic contention), summed at the end.
__global__ __launch_bounds__(kSortBlock) void k_sort_hist(const uint32_t* keys, int64_t n, int shift,
                                                          uint32_t* hist, int nblocks) {
  __shared__ uint32_t h[kSortBlock / 64][256];
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int k = 0; k < kSortBlock / 64; k++) h[k][tid] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile + (int64_t)tid * kSortRounds;
  if (base + kSortRounds <= n) {
    const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
#pragma unroll
    for (int r = 0; r < kSortRounds / 4; r++) {
      const uint4 v = k4[r];
      atomicAdd(&h[w][(v.x >> shift) & 0xFF], 1u);
      atomicAdd(&h[w][(v.y >> shift) & 0xFF], 1u);
      atomicAdd(&h[w][(v.z >> shift) & 0xFF], 1u);
      atomicAdd(&h[w][(v.w >> shift) & 0xFF], 1u);
    }
  } else {
    for (int r = 0; r < kSortRounds; r++)
      if (base + r < n) atomicAdd(&h[w][(keys[base + r] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kSortBlock / 64; k++) c += h[k][tid];
  hist[(int64_t)tid * nblocks + blockIdx.x] = c;
}

// Stable per-tile scatter. Wave w ranks the tile's w-th run of 1024 keys (all
// 16 loads issued up front; ballot multi-split per 64 keys, wave-private digit
// counters in LDS, no block barriers), one barrier turns the per-wave counts
// into offsets (wave w's keys follow wave w-1's in the input, so the order is
// stable), then the tile is ranked into LDS in digit order and written out so
// that consecutive threads store consecutive positions of each digit's run.
// (Loading inside 16 barrier-separated rounds left the pass latency-bound.)
// IOTA: the values are the input positions (not read: the first pass of a sort
// by index). ELEMS != nullptr (the last pass of the kd presort): no keys or
// values are written; each sorted position receives elems[value] as four SoA
// arrays (the gather by sorted index fused into the write-out).
template <bool IOTA, bool SOA>
__global__ __launch_bounds__(kSortBlock) void k_sort_scatter(const uint32_t* __restrict__ keys,
                                                             const uint32_t* __restrict__ vals,
                                                             uint32_t* __restrict__ okeys, uint32_t* __restrict__ ovals,
                                                             int64_t n, int shift, const uint32_t* __restrict__ hist,
                                                             const uint32_t* __restrict__ hoff, int nblocks,
                                                             const float4* __restrict__ elems, SoaOut soa) {
  __shared__ uint32_t lkey[kSortTile], lval[kSortTile];
  __shared__ uint32_t lstart[256], gbase[256];
  __shared__ uint32_t wcnt[kSortBlock / 64][256];
  __shared__ uint32_t wsum[kSortBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int kWaveKeys = kSortTile / (kSortBlock / 64);   // 1024
  constexpr int kSub = kWaveKeys / 64;                      // 16 sub-rounds of 64 keys
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  const int64_t wbase = base + (int64_t)w * kWaveKeys;
  uint32_t kr[kSub], vr[kSub];
#pragma unroll
  for (int r = 0; r < kSub; r++) {
    const int64_t i = wbase + r * 64 + lane;
    kr[r] = i < n ? keys[i] : 0u;
    vr[r] = IOTA ? (uint32_t)i : (i < n ? vals[i] : 0u);
  }
  // local digit starts = exclusive scan of this tile's histogram
  const uint32_t c = hist[(int64_t)tid * nblocks + blockIdx.x];
  uint32_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t up = (uint32_t)__shfl_up((int)incl, o);
    if (lane >= o) incl += up;
  }
  if (lane == 63) wsum[w] = incl;
#pragma unroll
  for (int k = 0; k < kSortBlock / 64; k++) wcnt[k][tid] = 0;
  __syncthreads();
  uint32_t wpre = 0;
#pragma unroll
  for (int k = 0; k < kSortBlock / 64; k++) wpre += k < w ? wsum[k] : 0u;
  lstart[tid] = wpre + incl - c;
  gbase[tid] = hoff[(int64_t)tid * nblocks + blockIdx.x];
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t rk[kSub];
#pragma unroll
  for (int r = 0; r < kSub; r++) {
    const bool valid = wbase + r * 64 + lane < n;
    const uint32_t dg = (kr[r] >> shift) & 0xFF;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t bal = __ballot((dg >> b) & 1);
      peers &= ((dg >> b) & 1) ? bal : ~bal;
    }
    const uint32_t before = wcnt[w][dg];
    const uint32_t lr = (uint32_t)__popcll(peers & lt_mask);
    rk[r] = before + lr;
    if (valid && lr == 0) wcnt[w][dg] = before + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  {  // per-digit offsets of each wave's keys inside the tile
    uint32_t run = lstart[tid];
#pragma unroll
    for (int k = 0; k < kSortBlock / 64; k++) {
      const uint32_t cnt = wcnt[k][tid];
      wcnt[k][tid] = run;
      run += cnt;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSub; r++) {
    if (wbase + r * 64 + lane < n) {
      const uint32_t pos = wcnt[w][(kr[r] >> shift) & 0xFF] + rk[r];
      lkey[pos] = kr[r];
      lval[pos] = vr[r];
    }
  }
  __syncthreads();
  const int tile_n = (int)min((int64_t)kSortTile, n - base);
  for (int p = tid; p < tile_n; p += kSortBlock) {
    const uint32_t key = lkey[p];
    const uint32_t dg = (key >> shift) & 0xFF;
    const uint32_t o = gbase[dg] + (uint32_t)p - lstart[dg];
    if (SOA) {
      const float4 e = elems[lval[p]];
      soa.c[0][o] = e.x;
      soa.c[1][o] = e.y;
      soa.c[2][o] = e.z;
      soa.c[3][o] = e.w;
    } else {
      okeys[o] = key;
      ovals[o] = lval[p];
    }
  }
}

hipError_t radix_sort_pairs(uint32_t* keys, uint32_t* vals, int64_t n, int end_bit, hipStream_t s) {
  if (n <= 1) return hipSuccess;
  const int nb = (int)((n + kSortTile - 1) / kSortTile);
  DevBuf<uint32_t> k2(n), v2(n), hist((size_t)256 * nb), hoff((size_t)256 * nb);
  if (!k2.p || !v2.p || !hist.p || !hoff.p) return hipErrorOutOfMemory;
  uint32_t *ka = keys, *va = vals, *kb = k2.p, *vb = v2.p;
  int passes = 0;
  for (int shift = 0; shift < end_bit; shift += 8, passes++) {
    k_sort_hist<<<nb, kSortBlock, 0, s>>>(ka, n, shift, hist.p, nb);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(exclusive_scan_u32(hist.p, hoff.p, (int64_t)256 * nb, nullptr, s));
    k_sort_scatter<false, false><<<nb, kSortBlock, 0, s>>>(ka, va, kb, vb, n, shift, hist.p, hoff.p, nb, nullptr,
                                                            SoaOut{});
    PM_HIP_TRY(hipGetLastError());
    uint32_t* t = ka; ka = kb; kb = t;
    t = va; va = vb; vb = t;
  }
  if (passes & 1) {
    PM_HIP_TRY(hipMemcpyAsync(keys, ka, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    PM_HIP_TRY(hipMemcpyAsync(vals, va, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  }
  return hipSuccess;
}

hipError_t radix_sort_gather_soa(const uint32_t* keys, int64_t n, const float4* elems, const SoaOut& out,
                                 hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int nb = (int)((n + kSortTile - 1) / kSortTile);
  DevBuf<uint32_t> ka(n), kb(n), va(n), vb(n), hist((size_t)256 * nb), hoff((size_t)256 * nb);
  if (!ka.p || !kb.p || !va.p || !vb.p || !hist.p || !hoff.p) return hipErrorOutOfMemory;
  const uint32_t* kin = keys;
  const uint32_t* vin = nullptr;
  uint32_t *ko = ka.p, *vo = va.p;
  for (int pass = 0; pass < 4; pass++) {
    const int shift = 8 * pass;
    k_sort_hist<<<nb, kSortBlock, 0, s>>>(kin, n, shift, hist.p, nb);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(exclusive_scan_u32(hist.p, hoff.p, (int64_t)256 * nb, nullptr, s));
    if (pass == 0)
      k_sort_scatter<true, false><<<nb, kSortBlock, 0, s>>>(kin, nullptr, ko, vo, n, shift, hist.p, hoff.p, nb,
                                                            nullptr, SoaOut{});
    else if (pass < 3)
      k_sort_scatter<false, false><<<nb, kSortBlock, 0, s>>>(kin, vin, ko, vo, n, shift, hist.p, hoff.p, nb,
                                                             nullptr, SoaOut{});
    else
      k_sort_scatter<false, true><<<nb, kSortBlock, 0, s>>>(kin, vin, nullptr, nullptr, n, shift, hist.p, hoff.p,
                                                            nb, elems, out);
    PM_HIP_TRY(hipGetLastError());
    kin = ko;
    vin = vo;
    ko = ko == ka.p ? kb.p : ka.p;
    vo = vo == va.p ? vb.p : va.p;
  }
  return hipSuccess;
}

}  // namespace pmd
