// kdshard.hip — the global map's kd-tree built across G ranks.
//
// The reference builds one tree on one device (cukd::buildTree, ray-tracer/
// src/hostCode.cu:94-95). With G GPUs every rank holds the same all-gathered
// photons, and rebuilding the whole tree on every rank (the replicated build)
// costs N log N of the G-times-larger map: 311 ms at 8 x 45.4 M photons against
// 35 ms for one GPU's share. Here the top L = ceil(log2 G) + 1 levels are
// selected directly (every rank, redundantly, a few passes over the elements),
// the 2^L subtrees below them are dealt to the ranks (balanced by size: about
// two per rank) and built with the ordinary kd_build, and the built subtrees
// (4-B tags per node: original index << 2 | split dimension) are all-gathered
// and placed into the implicit layout, positions taken from the photons every
// rank already holds. The
// result is the SAME tree as kd_build over all elements (same left-balanced
// ranks, same widest-dimension rule, same (coordinate, original index) order;
// tested bitwise): only who computes which part changes.
//
//   top level l, segment j (size s): dim = widest extent of its elements (the
//   extents kd_build reads from its presorted lists: min / max), median = the
//   element of rank left_size(s) in (orderable_key(coord), index) order, found by
//   an 8-bit radix select on that 64-bit key: two histogram passes over all
//   elements, one compaction of the elements whose top 16 key bits match, six
//   histogram passes over those candidates.
//   subtree j: the elements whose top-level path ends at j (stable compaction,
//   so local order = global index order and ties break the same way), built by
//   kd_build, original indices restored.
#include <algorithm>
#include <cstring>

#include "pm_internal.hpp"

namespace pmd {

constexpr int kShardMaxLevels = 5;   // <= 16 top segments per level, <= 32 subtrees

static inline int left_size_host(int s) {
  if (s <= 1) return 0;
  const int h = 32 - __builtin_clz((unsigned)s);
  const int half = 1 << (h - 2);
  const int full = (1 << (h - 1)) - 1;
  const int last = s - full;
  return (half - 1) + std::min(last, half);
}

__device__ __forceinline__ float shard_coord(const float4 e, int d) { return d == 0 ? e.x : (d == 1 ? e.y : e.z); }

// segment of e among the 2^l segments below the top l levels, or -1 if e is
// one of the top nodes (kd_class: left iff (c, id) < (node c, node id))
__device__ __forceinline__ int top_path(const float4 e, const float4* __restrict__ top, int l) {
  const int id = __float_as_int(e.w);
  int t = 0;
  for (int k = 0; k < l; k++) {
    const float4 nd = top[t];
    const int w = __float_as_int(nd.w), dim = w & 3, nid = (int)((uint32_t)w >> 2);
    if (id == nid) return -1;
    const float c = shard_coord(e, dim), nc = shard_coord(nd, dim);
    const bool left = c < nc || (c == nc && id < nid);
    t = 2 * t + (left ? 1 : 2);
  }
  return t - ((1 << l) - 1);
}

__device__ __forceinline__ uint64_t shard_key(const float4 e, int dim) {
  return ((uint64_t)orderable_key(shard_coord(e, dim)) << 32) | (uint32_t)__float_as_int(e.w);
}

// grid-stride passes over all elements: a fixed grid, one LDS init / flush per block
constexpr int kShardGrid = 2048;

// per-segment min / max of the orderable keys of x, y, z. NR > 0: the first
// levels (<= NR segments) keep per-thread register accumulators (same-address
// LDS atomics from a whole wave serialise: level 0 has one segment); deeper
// levels spread over 8-16 segments and use LDS atomics. One global atomic per
// block, segment and component.
template <int NR>
__global__ void k_shard_bounds(const float4* __restrict__ elems, int64_t n, const float4* __restrict__ top, int l,
                               uint32_t* __restrict__ ob /* [nseg][6] */) {
  __shared__ uint32_t sb[16 * 6];
  const int nseg = 1 << l;
  for (int k = threadIdx.x; k < nseg * 6; k += blockDim.x) sb[k] = (k % 6) < 3 ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  uint32_t acc[NR > 0 ? NR : 1][6];
#pragma unroll
  for (int r = 0; r < (NR > 0 ? NR : 1); r++)
#pragma unroll
    for (int k = 0; k < 6; k++) acc[r][k] = k < 3 ? 0xFFFFFFFFu : 0u;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 e = elems[i];
    const int j = top_path(e, top, l);
    if (j < 0) continue;
    const uint32_t k3[3] = {orderable_key(e.x), orderable_key(e.y), orderable_key(e.z)};
    if (NR > 0) {
#pragma unroll
      for (int r = 0; r < NR; r++) {
        if (j == r) {
#pragma unroll
          for (int d = 0; d < 3; d++) {
            acc[r][d] = min(acc[r][d], k3[d]);
            acc[r][3 + d] = max(acc[r][3 + d], k3[d]);
          }
        }
      }
    } else {
#pragma unroll
      for (int d = 0; d < 3; d++) {
        atomicMin(&sb[6 * j + d], k3[d]);
        atomicMax(&sb[6 * j + 3 + d], k3[d]);
      }
    }
  }
  if (NR > 0) {
#pragma unroll
    for (int r = 0; r < NR; r++) {
      if (r < nseg) {
#pragma unroll
        for (int d = 0; d < 3; d++) {
          if (acc[r][d] != 0xFFFFFFFFu) atomicMin(&sb[6 * r + d], acc[r][d]);
          if (acc[r][3 + d] != 0u) atomicMax(&sb[6 * r + 3 + d], acc[r][3 + d]);
        }
      }
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nseg * 6; k += blockDim.x) {
    if ((k % 6) < 3) {
      if (sb[k] != 0xFFFFFFFFu) atomicMin(&ob[k], sb[k]);
    } else if (sb[k] != 0u) {
      atomicMax(&ob[k], sb[k]);
    }
  }
}

// ShardSel (pm_internal.hpp): per segment the split dimension and the key bits
// above `shift + 8` selected so far

// segment -> (dim, prefix) in LDS (a by-value kernel argument indexed at run
// time would go through private memory)
struct ShardSelLds {
  int dim[16];
  uint64_t prefix[16];
  __device__ __forceinline__ void load(const ShardSel& s) {
    if (threadIdx.x < 16) {
#pragma unroll
      for (int k = 0; k < 16; k++)
        if ((int)threadIdx.x == k) dim[k] = s.dim[k], prefix[k] = s.prefix[k];
    }
  }
};

// 256-bin histogram of key bits [shift, shift + 8) over the elements of each
// segment whose key matches the segment's prefix above them; up to two wave
// rounds merge lanes with the same (segment, bin) before the LDS atomics
__global__ void k_shard_hist(const float4* __restrict__ elems, int64_t n, const float4* __restrict__ top, int l,
                             ShardSel sel, int shift, uint32_t* __restrict__ hist /* [nseg][256] */) {
  __shared__ uint32_t sh[16 * 256];
  __shared__ ShardSelLds ss;
  const int nseg = 1 << l;
  const int lane = threadIdx.x & 63;
  for (int k = threadIdx.x; k < nseg * 256; k += blockDim.x) sh[k] = 0;
  ss.load(sel);
  __syncthreads();
  const int hb = shift + 8;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += step) {
    const int64_t i = base + threadIdx.x;
    int slot = -1;
    if (i < n) {
      const float4 e = elems[i];
      const int j = top_path(e, top, l);
      if (j >= 0) {
        const uint64_t key = shard_key(e, ss.dim[j]);
        if (hb >= 64 || (key >> hb) == (ss.prefix[j] >> hb)) slot = 256 * j + (int)((key >> shift) & 255u);
      }
    }
    for (int round = 0; round < 2; round++) {
      const uint64_t pending = __ballot(slot >= 0);
      if (!pending) break;
      const int sl = __shfl(slot, __builtin_ctzll(pending));
      const uint64_t m = __ballot(slot == sl);
      if (lane == __builtin_ctzll(m)) atomicAdd(&sh[sl], (uint32_t)__popcll(m));
      if (slot == sl) slot = -1;
    }
    if (slot >= 0) atomicAdd(&sh[slot], 1u);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nseg * 256; k += blockDim.x)
    if (sh[k]) atomicAdd(&hist[k], sh[k]);
}

// the matching elements' keys, per segment, into cand[off[j] ...): block-
// aggregated over chunks of kCompactIPT x 256 elements (LDS counts, one global
// atomic per block, segment and chunk)
constexpr int kCompactIPT = 8;
__global__ void k_shard_compact(const float4* __restrict__ elems, int64_t n, const float4* __restrict__ top, int l,
                                ShardSel sel, int hb, const uint64_t* __restrict__ off,
                                unsigned long long* __restrict__ cnt, uint64_t* __restrict__ cand, uint64_t cap) {
  __shared__ ShardSelLds ss;
  __shared__ uint32_t lc[16];
  __shared__ unsigned long long lb[16];
  const int nseg = 1 << l;
  ss.load(sel);
  const int64_t chunk = (int64_t)blockDim.x * kCompactIPT;
  for (int64_t base = (int64_t)blockIdx.x * chunk; base < n; base += (int64_t)gridDim.x * chunk) {
    if (threadIdx.x < 16) lc[threadIdx.x] = 0;
    __syncthreads();
    int j[kCompactIPT];
    uint32_t mine[kCompactIPT];
    uint64_t key[kCompactIPT];
#pragma unroll
    for (int k = 0; k < kCompactIPT; k++) {
      const int64_t i = base + k * blockDim.x + threadIdx.x;
      j[k] = -1;
      key[k] = 0;
      if (i < n) {
        const float4 e = elems[i];
        j[k] = top_path(e, top, l);
        if (j[k] >= 0) {
          key[k] = shard_key(e, ss.dim[j[k]]);
          if ((key[k] >> hb) != (ss.prefix[j[k]] >> hb)) j[k] = -1;
        }
      }
      mine[k] = j[k] >= 0 ? atomicAdd(&lc[j[k]], 1u) : 0u;
    }
    __syncthreads();
    if ((int)threadIdx.x < nseg && lc[threadIdx.x] > 0)
      lb[threadIdx.x] = atomicAdd(&cnt[threadIdx.x], (unsigned long long)lc[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kCompactIPT; k++)
      if (j[k] >= 0) {
        const uint64_t at = off[j[k]] + lb[j[k]] + mine[k];
        if (at < cap) cand[at] = key[k];   // (a distributed selection fed wrong reductions)
      }
  }
}

__global__ void k_shard_cand_hist(const uint64_t* __restrict__ cand, int64_t nc, uint64_t prefix, int shift,
                                  uint32_t* __restrict__ hist /* [256] */) {
  __shared__ uint32_t sh[256];
  for (int k = threadIdx.x; k < 256; k += blockDim.x) sh[k] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nc) {
    const uint64_t key = cand[i];
    const int hb = shift + 8;
    if ((key >> hb) == (prefix >> hb)) atomicAdd(&sh[(int)((key >> shift) & 255u)], 1u);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 256; k += blockDim.x)
    if (sh[k]) atomicAdd(&hist[k], sh[k]);
}

// top node t = 2^l - 1 + j: the selected element, split dimension in the tag
__global__ void k_shard_top_write(const float4* __restrict__ elems, ShardSel sel, int l, float4* __restrict__ top) {
  const int j = threadIdx.x;
  if (j >= (1 << l)) return;
  const int id = (int)(uint32_t)sel.prefix[j];
  const float4 e = elems[id];
  top[(1 << l) - 1 + j] = make_float4(e.x, e.y, e.z, __int_as_float((id << 2) | sel.dim[j]));
}

// subtree of every element (255: a top node), once per plan
__global__ void k_shard_sub(const float4* __restrict__ elems, int64_t n, const float4* __restrict__ top, int L,
                            uint8_t* __restrict__ sub) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int j = top_path(elems[i], top, L);
  sub[i] = j < 0 ? 255 : (uint8_t)j;
}

// Subtree extraction. Once per plan, k_shard_count counts every subtree's
// elements per tile of kShardExtTile and one scan over the (subtree, tile)
// counts, subtree-major, gives each tile's start inside each subtree. A
// subtree's extraction is then ONE pass: it reads the 1-B subtree ids (16 per
// thread, one 16-B load) and only its own elements, ranks them inside the tile
// with a block scan of the per-thread match counts (thread order = index
// order: stable) and writes them out. The earlier per-subtree
// flag / scan / extract passes moved ~21 B per element of the whole map for
// every subtree a rank builds.
constexpr int kShardExtTile = 4096;   // 256 threads x 16 chunks

__global__ __launch_bounds__(256) void k_shard_count(const uint8_t* __restrict__ sub, int64_t n, int nb,
                                                     int64_t tiles, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[32];
  if (threadIdx.x < 32) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kShardExtTile;
  for (int k = 0; k < kShardExtTile / 256; k++) {
    const int64_t e = base + k * 256 + threadIdx.x;
    if (e < n) {
      const int b = sub[e];
      if (b < nb) atomicAdd(&h[b], 1u);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < nb) cnt[threadIdx.x * tiles + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_shard_extract(const float4* __restrict__ elems,
                                                       const uint8_t* __restrict__ subof, int64_t n, int j,
                                                       int64_t tiles, const uint32_t* __restrict__ boff,
                                                       float4* __restrict__ sub, int32_t* __restrict__ gid) {
  // thread t owns elements [16 t, 16 t + 16) of the tile: one 16-B load of
  // their subtree ids, a match mask, and a block scan of the match counts
  __shared__ uint32_t wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t run = boff[(int64_t)j * tiles + blockIdx.x] - boff[(int64_t)j * tiles];
  const int64_t e0 = (int64_t)blockIdx.x * kShardExtTile + (int64_t)threadIdx.x * 16;
  uint32_t wd[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};   // 255: matches no subtree
  if (e0 + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(subof + e0);
    wd[0] = v.x, wd[1] = v.y, wd[2] = v.z, wd[3] = v.w;
  } else {
    for (int k = 0; k < 16 && e0 + k < n; k++)
      wd[k >> 2] = (wd[k >> 2] & ~(0xFFu << (8 * (k & 3)))) | ((uint32_t)subof[e0 + k] << (8 * (k & 3)));
  }
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) m |= (((wd[k >> 2] >> (8 * (k & 3))) & 0xFFu) == (uint32_t)j ? 1u : 0u) << k;
  const uint32_t c = (uint32_t)__popc(m);
  uint32_t x = c;   // inclusive wave scan
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t p = run + x - c;
  for (int v = 0; v < w; v++) p += wsum[v];
  while (m) {
    const int k = __ffs(m) - 1;
    m &= m - 1;
    const float4 el = elems[e0 + k];
    sub[p] = make_float4(el.x, el.y, el.z, __int_as_float((int)p));
    gid[p] = __float_as_int(el.w);
    p++;
  }
}

// built subtree -> 4-B tags (original index << 2 | split dimension): the
// positions travel once, in the photon exchange, not again with the tree
__global__ void k_shard_tags(const float4* __restrict__ nodes, int64_t s, const int32_t* __restrict__ gid,
                             int32_t* __restrict__ tags) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= s) return;
  const int w = __float_as_int(nodes[u].w);
  tags[u] = (gid[(uint32_t)w >> 2] << 2) | (w & 3);
}

// subtree rooted at global node t: local node u (depth d, k-th at that depth)
// -> global (t + 1) 2^d - 1 + k; the position comes from elems[original index]
__global__ void k_shard_place(const float4* __restrict__ elems, const int32_t* __restrict__ tags, int64_t s,
                              int64_t t, float4* __restrict__ nodes) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= s) return;
  const int d = 63 - __clzll((unsigned long long)(u + 1));
  const int64_t k = u + 1 - ((int64_t)1 << d);
  const int w = tags[u];
  const float4 e = elems[(uint32_t)w >> 2];
  nodes[(t + 1) * ((int64_t)1 << d) - 1 + k] = make_float4(e.x, e.y, e.z, __int_as_float(w));
}

// levels for G ranks: ceil(log2 G) + 1, capped: about two subtrees per rank, so
// the caller can balance the left-balanced tree's unequal subtrees (the left
// ones hold the full last level: up to 2x the right ones)
int shard_levels(int world) {
  int L = 0;
  while ((1 << L) < world) L++;
  return std::min(L + 1, kShardMaxLevels);
}

bool shard_ok(int64_t n, int L) { return L >= 1 && L <= kShardMaxLevels && n >= (2ll << L) && n < kMaxMapPhotons; }

// Top L levels: top[0 .. 2^L - 1) and the 2^L subtree sizes (host).
hipError_t kd_shard_top(const float4* elems, int64_t n, int L, float4* top, std::vector<int64_t>& sizes,
                        hipStream_t s) {
  if (!shard_ok(n, L)) return hipErrorInvalidValue;
  std::vector<int64_t> seg{n};
  DevBuf<uint32_t> ob(16 * 6), hist(16 * 256);
  DevBuf<uint64_t> off(16);
  DevBuf<unsigned long long> cnt(16);
  DevBuf<uint64_t> cand;
  if (!ob.p || !hist.p || !off.p || !cnt.p) return hipErrorOutOfMemory;
  const int g = (int)std::min<int64_t>(kShardGrid, (n + 255) / 256);
  for (int l = 0; l < L; l++) {
    const int nseg = 1 << l;
    // widest dimension per segment
    std::vector<uint32_t> hb(nseg * 6);
    for (int k = 0; k < nseg * 6; k++) hb[k] = (k % 6) < 3 ? 0xFFFFFFFFu : 0u;
    PM_HIP_TRY(hipMemcpyAsync(ob.p, hb.data(), 4 * hb.size(), hipMemcpyHostToDevice, s));
    if (nseg <= 4) k_shard_bounds<4><<<g, 256, 0, s>>>(elems, n, top, l, ob.p);
    else k_shard_bounds<0><<<g, 256, 0, s>>>(elems, n, top, l, ob.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(hipMemcpyAsync(hb.data(), ob.p, 4 * hb.size(), hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
    ShardSel sel{};
    std::vector<int64_t> rank(nseg);
    for (int j = 0; j < nseg; j++) {
      float ext[3];
      for (int d = 0; d < 3; d++) {
        auto to_f = [](uint32_t u) {
          const uint32_t bits = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
          float f;
          std::memcpy(&f, &bits, 4);
          return f;
        };
        ext[d] = to_f(hb[6 * j + 3 + d]) - to_f(hb[6 * j + d]);   // last - first of the sorted list
      }
      int dim = 0;
      if (ext[1] > ext[dim]) dim = 1;
      if (ext[2] > ext[dim]) dim = 2;
      sel.dim[j] = dim;
      sel.prefix[j] = 0;
      rank[j] = left_size_host((int)seg[j]);
    }
    // radix select, 8 bits per pass from the top of the 64-bit key
    auto take = [&](const std::vector<uint32_t>& h, int j, int shift) {
      int64_t r = rank[j];
      int b = 0;
      for (; b < 255; b++) {
        if (r < (int64_t)h[256 * j + b]) break;
        r -= h[256 * j + b];
      }
      rank[j] = r;
      sel.prefix[j] |= (uint64_t)b << shift;
      return (int64_t)h[256 * j + b];
    };
    std::vector<uint32_t> hh(nseg * 256);
    std::vector<int64_t> ncand(nseg);
    for (int pass = 0; pass < 2; pass++) {
      const int shift = 56 - 8 * pass;
      PM_HIP_TRY(hipMemsetAsync(hist.p, 0, 4 * 256 * nseg, s));
      k_shard_hist<<<g, 256, 0, s>>>(elems, n, top, l, sel, shift, hist.p);
      PM_HIP_TRY(hipGetLastError());
      PM_HIP_TRY(hipMemcpyAsync(hh.data(), hist.p, 4 * hh.size(), hipMemcpyDeviceToHost, s));
      PM_HIP_TRY(hipStreamSynchronize(s));
      for (int j = 0; j < nseg; j++) ncand[j] = take(hh, j, shift);
    }
    std::vector<uint64_t> ho(nseg);
    int64_t tot = 0;
    for (int j = 0; j < nseg; j++) ho[j] = (uint64_t)tot, tot += ncand[j];
    if ((int64_t)cand.n < tot) cand.alloc(tot);
    if (!cand.p) return hipErrorOutOfMemory;
    PM_HIP_TRY(hipMemcpyAsync(off.p, ho.data(), 8 * nseg, hipMemcpyHostToDevice, s));
    PM_HIP_TRY(hipMemsetAsync(cnt.p, 0, 8 * nseg, s));
    k_shard_compact<<<g, 256, 0, s>>>(elems, n, top, l, sel, 48, off.p, cnt.p, cand.p, (uint64_t)cand.n);
    PM_HIP_TRY(hipGetLastError());
    for (int pass = 2; pass < 8; pass++) {
      const int shift = 56 - 8 * pass;
      PM_HIP_TRY(hipMemsetAsync(hist.p, 0, 4 * 256 * nseg, s));
      for (int j = 0; j < nseg; j++)
        if (ncand[j] > 0)
          k_shard_cand_hist<<<grid_for(ncand[j], 256), 256, 0, s>>>(cand.p + ho[j], ncand[j], sel.prefix[j], shift,
                                                                     hist.p + 256 * j);
      PM_HIP_TRY(hipGetLastError());
      PM_HIP_TRY(hipMemcpyAsync(hh.data(), hist.p, 4 * hh.size(), hipMemcpyDeviceToHost, s));
      PM_HIP_TRY(hipStreamSynchronize(s));
      for (int j = 0; j < nseg; j++) take(hh, j, shift);
    }
    k_shard_top_write<<<1, 64, 0, s>>>(elems, sel, l, top);
    PM_HIP_TRY(hipGetLastError());
    std::vector<int64_t> nxt;
    for (int j = 0; j < nseg; j++) {
      const int64_t ls = left_size_host((int)seg[j]);
      nxt.push_back(ls);
      nxt.push_back(seg[j] - ls - 1);
    }
    seg.swap(nxt);
  }
  sizes = seg;
  return hipStreamSynchronize(s);
}

// ---- distributed top selection (each rank over its OWN photons) -------------
// kd_shard_top reads every element on every rank: at 8 x 45.4 M photons that is
// 16 full passes over 363 M elements per rank (34 ms), all of it replicated. The
// same selection splits over the ranks: every pass (bounds, the two top-byte
// histograms, the six candidate histograms) runs over the rank's own elements
// -- its traced photons, with their GLOBAL indices, so keys and ties are those
// of the gathered map -- and the caller reduces the small pass output across
// ranks (MIN for the bounds, SUM for the histograms) before the next step. The
// host logic is kd_shard_top's; the result (top nodes, subtree sizes) is the
// same on every rank and equal to kd_shard_top's over the gathered elements.
// It needs no exchanged photon, so it runs while the photon all-gather is in
// flight. Top nodes carry only the split coordinate until the gathered
// elements fill them in (kd_shard_top_fix).
__device__ __forceinline__ float shard_kd_coord(float x) { return x != x ? __int_as_float(0x7f800000) : x; }

__global__ void k_shard_local_elems(const pm_photon* __restrict__ a, int64_t na, int64_t aid,
                                    const pm_photon* __restrict__ b, int64_t nb, int64_t bid,
                                    float4* __restrict__ elems) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na + nb) return;
  const pm_photon p = i < na ? a[i] : b[i - na];
  const int64_t id = i < na ? aid + i : bid + (i - na);
  elems[i] = make_float4(shard_kd_coord(p.pos.x), shard_kd_coord(p.pos.y), shard_kd_coord(p.pos.z),
                         __int_as_float((int)id));
}

// pass output -> the caller's int64 reduction buffer (bounds: maxima stored
// inverted so that one MIN reduces both)
__global__ void k_shard_red(const uint32_t* __restrict__ src, int count, int bounds, int64_t* __restrict__ red) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint32_t v = src[k];
  red[k] = (int64_t)(bounds && (k % 6) >= 3 ? ~v : v);
}

__global__ void k_shard_top_fix(const float4* __restrict__ elems, int64_t ntop, float4* __restrict__ top) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntop) return;
  const int w = __float_as_int(top[t].w);
  const float4 e = elems[(uint32_t)w >> 2];
  top[t] = make_float4(e.x, e.y, e.z, __int_as_float(w));
}

static float from_orderable(uint32_t u) {
  const uint32_t bits = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

hipError_t KdTopSel::init(const pm_photon* a, int64_t na, int64_t aid, const pm_photon* b, int64_t nb, int64_t bid,
                          int64_t n_total, int levels, hipStream_t s) {
  if (!shard_ok(n_total, levels)) return hipErrorInvalidValue;
  L = levels;
  n = na + nb;
  seg_total = n_total;
  seg.assign(1, n_total);
  elems.alloc(std::max<int64_t>(n, 1));
  top.alloc((size_t)1 << L);
  ob.alloc(16 * 6);
  hist.alloc(16 * 256);
  off.alloc(16);
  cnt.alloc(16);
  if (!elems.p || !top.p || !ob.p || !hist.p || !off.p || !cnt.p) return hipErrorOutOfMemory;
  if (n > 0) {
    k_shard_local_elems<<<grid_for(n, 256), 256, 0, s>>>(a, na, aid, b, nb, bid, elems.p);
    PM_HIP_TRY(hipGetLastError());
  }
  level = 0;
  pending = -1;
  return hipSuccess;
}

// issue pass `pending` of the current level into red (count, op)
hipError_t KdTopSel::issue(int64_t* red, int64_t* count, int* op, hipStream_t s) {
  const int nseg = 1 << level;
  const int g = (int)std::max<int64_t>(1, std::min<int64_t>(kShardGrid, (n + 255) / 256));
  if (pending == 0) {
    std::vector<uint32_t> hb(nseg * 6);
    for (int k = 0; k < nseg * 6; k++) hb[k] = (k % 6) < 3 ? 0xFFFFFFFFu : 0u;
    PM_HIP_TRY(hipMemcpyAsync(ob.p, hb.data(), 4 * hb.size(), hipMemcpyHostToDevice, s));
    if (n > 0) {
      if (nseg <= 4) k_shard_bounds<4><<<g, 256, 0, s>>>(elems.p, n, top.p, level, ob.p);
      else k_shard_bounds<0><<<g, 256, 0, s>>>(elems.p, n, top.p, level, ob.p);
      PM_HIP_TRY(hipGetLastError());
    }
    k_shard_red<<<grid_for(nseg * 6, 256), 256, 0, s>>>(ob.p, nseg * 6, 1, red);
    *count = nseg * 6;
    *op = 2;
    return hipStreamSynchronize(s);   // hb is read by the copy
  }
  PM_HIP_TRY(hipMemsetAsync(hist.p, 0, 4 * 256 * nseg, s));
  if (pending <= 2) {   // top-byte passes over the elements
    if (n > 0) {
      k_shard_hist<<<g, 256, 0, s>>>(elems.p, n, top.p, level, sel, 56 - 8 * (pending - 1), hist.p);
      PM_HIP_TRY(hipGetLastError());
    }
  } else {   // candidate passes
    const int shift = 56 - 8 * (pending - 1);
    for (int j = 0; j < nseg; j++)
      if (ncand[j] > 0)
        k_shard_cand_hist<<<grid_for(ncand[j], 256), 256, 0, s>>>(cand.p + ho[j], ncand[j], sel.prefix[j], shift,
                                                                   hist.p + 256 * j);
    PM_HIP_TRY(hipGetLastError());
  }
  k_shard_red<<<grid_for(nseg * 256, 256), 256, 0, s>>>(hist.p, nseg * 256, 0, red);
  PM_HIP_TRY(hipGetLastError());
  *count = nseg * 256;
  *op = 1;
  return hipSuccess;
}

// consume the reduced output of pass `pending` (kd_shard_top's host logic)
hipError_t KdTopSel::consume(const int64_t* red, hipStream_t s) {
  const int nseg = 1 << level;
  const int cnt_n = pending == 0 ? nseg * 6 : nseg * 256;
  std::vector<int64_t> h(cnt_n);
  PM_HIP_TRY(hipMemcpyAsync(h.data(), red, 8 * cnt_n, hipMemcpyDeviceToHost, s));
  PM_HIP_TRY(hipStreamSynchronize(s));
  if (pending == 0) {
    rank.assign(nseg, 0);
    for (int j = 0; j < nseg; j++) {
      float ext[3];
      for (int d = 0; d < 3; d++)
        ext[d] = from_orderable((uint32_t)~(uint32_t)h[6 * j + 3 + d]) - from_orderable((uint32_t)h[6 * j + d]);
      int dim = 0;
      if (ext[1] > ext[dim]) dim = 1;
      if (ext[2] > ext[dim]) dim = 2;
      sel.dim[j] = dim;
      sel.prefix[j] = 0;
      rank[j] = left_size_host((int)seg[j]);
    }
    ncand.assign(nseg, 0);
    pending = 1;
    return hipSuccess;
  }
  const int shift = 56 - 8 * (pending - 1);
  for (int j = 0; j < nseg; j++) {   // radix select: the bin holding rank j
    int64_t r = rank[j];
    int b = 0;
    for (; b < 255; b++) {
      if (r < h[256 * j + b]) break;
      r -= h[256 * j + b];
    }
    rank[j] = r;
    sel.prefix[j] |= (uint64_t)b << shift;
    // top-byte passes: the global count under the prefix sizes the candidate
    // buffer (candidate passes keep this rank's own count from the compaction)
    if (pending <= 2) ncand[j] = h[256 * j + b];
  }
  if (pending == 2) {   // the local elements under each 16-bit prefix
    std::vector<uint64_t> hc(nseg, 0);
    PM_HIP_TRY(hipMemsetAsync(cnt.p, 0, 8 * nseg, s));
    // local counts first: an upper bound (the global count) sizes the buffer
    ho.assign(nseg, 0);
    int64_t tot = 0;
    for (int j = 0; j < nseg; j++) ho[j] = (uint64_t)tot, tot += ncand[j];
    if ((int64_t)cand.n < std::max<int64_t>(tot, 1)) cand.alloc(std::max<int64_t>(tot, 1));
    if (!cand.p) return hipErrorOutOfMemory;
    PM_HIP_TRY(hipMemcpyAsync(off.p, ho.data(), 8 * nseg, hipMemcpyHostToDevice, s));
    if (n > 0) {
      const int g = (int)std::max<int64_t>(1, std::min<int64_t>(kShardGrid, (n + 255) / 256));
      k_shard_compact<<<g, 256, 0, s>>>(elems.p, n, top.p, level, sel, 48, off.p, cnt.p, cand.p,
                                          (uint64_t)cand.n);
      PM_HIP_TRY(hipGetLastError());
    }
    PM_HIP_TRY(hipMemcpyAsync(hc.data(), cnt.p, 8 * nseg, hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
    for (int j = 0; j < nseg; j++) ncand[j] = std::min<int64_t>((int64_t)hc[j], ncand[j]);   // this rank's own
  }
  if (pending < 8) {
    pending++;
    return hipSuccess;
  }
  // level done: the selected keys are the top nodes (split coordinate + tag);
  // an index outside the map means the caller's reductions were not the
  // documented ones (every rank, every pass): refuse it rather than place it
  std::vector<float4> ht(nseg);
  for (int j = 0; j < nseg; j++) {
    const uint32_t id = (uint32_t)sel.prefix[j];
    if ((int64_t)id >= seg_total) return hipErrorInvalidValue;
    const float c = from_orderable((uint32_t)(sel.prefix[j] >> 32));
    const uint32_t w = (id << 2) | (uint32_t)sel.dim[j];
    float wf;
    std::memcpy(&wf, &w, 4);
    float4 r = make_float4(0.f, 0.f, 0.f, wf);
    if (sel.dim[j] == 0) r.x = c;
    else if (sel.dim[j] == 1) r.y = c;
    else r.z = c;
    ht[j] = r;
  }
  PM_HIP_TRY(hipMemcpyAsync(top.p + ((1 << level) - 1), ht.data(), sizeof(float4) * nseg, hipMemcpyHostToDevice, s));
  PM_HIP_TRY(hipStreamSynchronize(s));
  std::vector<int64_t> nxt;
  for (int j = 0; j < nseg; j++) {
    const int64_t ls = left_size_host((int)seg[j]);
    nxt.push_back(ls);
    nxt.push_back(seg[j] - ls - 1);
  }
  seg.swap(nxt);
  level++;
  pending = level < L ? 0 : -1;
  return hipSuccess;
}

hipError_t KdTopSel::step(int64_t* red, int64_t* count, int* op, hipStream_t s) {
  *count = 0;
  *op = 0;
  if (level >= L) return hipSuccess;
  if (pending < 0) pending = 0;          // first call: level 0's bounds
  else PM_HIP_TRY(consume(red, s));      // the caller reduced the previous pass
  if (level >= L) return hipSuccess;     // finished
  return issue(red, count, op, s);
}

// The gathered photons -> elements + payload (k_elems_from_rows) and each
// element's subtree (k_shard_sub) in one pass per run of rows: the selection's
// top nodes carry the split coordinates top_path reads.
__global__ void k_shard_elems_classify(const float* __restrict__ rows, int stride, int coff, int64_t n, int64_t id0,
                                       float power, const float4* __restrict__ top, int L,
                                       float4* __restrict__ elems, float4* __restrict__ payload,
                                       uint8_t* __restrict__ sub) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = rows + i * stride;
  const int64_t id = id0 + i;
  const float4 e = make_float4(shard_kd_coord(r[0]), shard_kd_coord(r[1]), shard_kd_coord(r[2]),
                               __int_as_float((int)id));
  elems[id] = e;
  payload[id] = make_float4(r[coff], r[coff + 1], r[coff + 2], power);
  const int j = top_path(e, top, L);
  sub[id] = j < 0 ? 255 : (uint8_t)j;
}

hipError_t kd_shard_elems_classify(const RowRuns& runs, const float4* top, int L, float4* elems, float4* payload,
                                   uint8_t* sub, hipStream_t s) {
  int64_t id0 = 0;
  for (const RowRun& r : runs) {
    if (r.n > 0) {
      k_shard_elems_classify<<<grid_for(r.n, 256), 256, 0, s>>>(r.rows, r.stride, r.coff, r.n, id0, r.power, top, L,
                                                               elems, payload, sub);
      PM_HIP_TRY(hipGetLastError());
    }
    id0 += r.n;
  }
  return hipSuccess;
}

hipError_t kd_shard_top_fix(const float4* elems, float4* top, int L, hipStream_t s) {
  const int64_t ntop = (1ll << L) - 1;
  k_shard_top_fix<<<grid_for(ntop, 64), 64, 0, s>>>(elems, ntop, top);
  return hipGetLastError();
}

// Subtree j below the top L levels, in its local implicit layout with
// original indices in the tags (out: sizes[j] nodes).
hipError_t kd_shard_classify(const float4* elems, int64_t n, int L, const float4* top, uint8_t* sub, hipStream_t s) {
  k_shard_sub<<<grid_for(n, 256), 256, 0, s>>>(elems, n, top, L, sub);
  return hipGetLastError();
}

int64_t kd_shard_tiles(int64_t n) { return (n + kShardExtTile - 1) / kShardExtTile; }

// `expect`: the plan's subtree sizes. k_shard_extract writes each subtree's
// elements into a buffer of exactly that size, so the counts found here must
// agree: a plan whose sizes came from a distributed selection fed the wrong
// reductions (pm_kd_shard_plan_create_from_sel) is refused with
// hipErrorInvalidValue instead of writing past a subtree buffer.
hipError_t kd_shard_offsets(const uint8_t* subof, int64_t n, int nb, const int64_t* expect, uint32_t* boff,
                            hipStream_t s) {
  const int64_t tiles = kd_shard_tiles(n);
  if (n <= 0 || nb < 1 || nb > 32 || tiles > 0x7FFFFFFF || tiles * nb > 0xFFFFFFFFll) return hipErrorInvalidValue;
  DevBuf<uint32_t> cnt(tiles * nb), total(1);
  if (!cnt.p || !total.p) return hipErrorOutOfMemory;
  k_shard_count<<<(int)tiles, 256, 0, s>>>(subof, n, nb, tiles, cnt.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(exclusive_scan_u32(cnt.p, boff, tiles * nb, total.p, s));
  uint32_t start[33];
  for (int j = 0; j < nb; j++)
    PM_HIP_TRY(hipMemcpyAsync(&start[j], boff + (int64_t)j * tiles, 4, hipMemcpyDeviceToHost, s));
  PM_HIP_TRY(hipMemcpyAsync(&start[nb], total.p, 4, hipMemcpyDeviceToHost, s));
  PM_HIP_TRY(hipStreamSynchronize(s));
  for (int j = 0; j < nb; j++)
    if ((int64_t)(start[j + 1] - start[j]) != expect[j]) return hipErrorInvalidValue;
  return hipSuccess;
}

hipError_t kd_shard_subtree(const float4* elems, const uint8_t* subof, const uint32_t* boff, int64_t n, int j,
                            int64_t size, int32_t* out, hipStream_t s) {
  if (size <= 0) return hipSuccess;
  DevBuf<float4> sub(size), nodes(size);
  DevBuf<int32_t> gid(size);
  if (!sub.p || !nodes.p || !gid.p) return hipErrorOutOfMemory;
  const int64_t tiles = kd_shard_tiles(n);
  k_shard_extract<<<(int)tiles, 256, 0, s>>>(elems, subof, n, j, tiles, boff, sub.p, gid.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(kd_build(sub.p, size, nodes.p, s));
  k_shard_tags<<<grid_for(size, 256), 256, 0, s>>>(nodes.p, size, gid.p, out);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);   // scratch buffers are freed on return
}

// Global layout from the top nodes and the subtrees' tags (concatenated in j order).
hipError_t kd_shard_assemble(const float4* elems, const float4* top, int L, const int32_t* tags,
                             const std::vector<int64_t>& sizes, float4* nodes, hipStream_t s) {
  const int64_t ntop = (1ll << L) - 1;
  PM_HIP_TRY(hipMemcpyAsync(nodes, top, sizeof(float4) * ntop, hipMemcpyDeviceToDevice, s));
  int64_t off = 0;
  for (size_t j = 0; j < sizes.size(); j++) {
    if (sizes[j] > 0) {
      k_shard_place<<<grid_for(sizes[j], 256), 256, 0, s>>>(elems, tags + off, sizes[j], ntop + (int64_t)j, nodes);
      PM_HIP_TRY(hipGetLastError());
    }
    off += sizes[j];
  }
  return hipSuccess;
}

}  // namespace pmd
