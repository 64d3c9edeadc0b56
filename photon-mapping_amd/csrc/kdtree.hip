// kdtree.hip — left-balanced implicit kd-tree build for gfx950.
//
// Replaces cukd::buildTree<Photon, Photon_traits> (ray-tracer/src/hostCode.cu:
// 94-95; traits ray-tracer/include/photon.h:23-40, has_explicit_dim): the
// output is the implicit complete binary tree (children 2t+1, 2t+2) whose node
// t holds the element of rank left_size(|subtree|) along the subtree's widest
// dimension, i.e. left subtree <= node <= right subtree on that dimension.
//
// Algorithm (presorted lists, level by level): the points are sorted once per
// dimension (stable radix sort on (coord, index)); every level then splits each
// active subtree range at its left-balanced median — the median element is read
// directly from the list of the chosen dimension and the two OTHER lists are
// stably partitioned around it (segmented count scan over 512-position tiles:
// k_kd_count -> k_kd_chunkscan / k_kd_chunkcarry -> k_kd_part). The split
// dimension's own list is already partitioned (it is sorted on that dimension)
// and is not moved: every list has two buffers and each subtree records which
// buffer holds each of its three lists (SegTab::sel). The lists are SoA (x, y,
// z, original index as four arrays), so the count pass reads only the split
// coordinate (and the index on a coordinate tie). Subtree ranges are identical
// in the three lists; a position's subtree is found from the subtree table
// (k_kd_tileseg + seg_find). Ties are broken by the original index.
#include <algorithm>

#include "pm_internal.hpp"

namespace pmd {

__device__ __forceinline__ int left_size(int s) {
  // complete-tree left subtree size for a subtree of s >= 1 nodes
  if (s <= 1) return 0;
  const int h = 32 - __clz(s);              // levels
  const int half = 1 << (h - 2);            // capacity of left's last level
  const int full = (1 << (h - 1)) - 1;      // nodes above the last level
  const int last = s - full;
  return (half - 1) + min(last, half);
}

__device__ __forceinline__ float coord_of(const float4 e, int d) { return d == 0 ? e.x : (d == 1 ? e.y : e.z); }

// orderable keys of the three coordinates in one pass over the elements
__global__ void k_kd_init_keys(const float4* __restrict__ elems, int64_t n, uint32_t* __restrict__ kx,
                               uint32_t* __restrict__ ky, uint32_t* __restrict__ kz) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 e = elems[i];
  kx[i] = orderable_key(e.x);
  ky[i] = orderable_key(e.y);
  kz[i] = orderable_key(e.z);
}

// The presorted lists: list d (sorted on dimension d) in buffer k (0 / 1) as
// four arrays (x, y, z, original index bits), one allocation of 24 n floats.
struct KdLists {
  float* base;
  int64_t n;
  __host__ __device__ float* comp(int d, int k, int c) const { return base + (int64_t)((d * 2 + k) * 4 + c) * n; }
};

__device__ __forceinline__ float4 kd_elem(const KdLists& Lst, int d, int k, int64_t p) {
  return make_float4(Lst.comp(d, k, 0)[p], Lst.comp(d, k, 1)[p], Lst.comp(d, k, 2)[p], Lst.comp(d, k, 3)[p]);
}

struct SegTab {
  int32_t* b;
  int32_t* s;
  int32_t* ls;
  int32_t* dim;
  float* coord;
  int32_t* id;
  int32_t* sel;   // bit d: buffer of list d for this subtree
};

__global__ void k_kd_seg(KdLists Lst, int level, int64_t cap, SegTab T, float4* out_nodes) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nseg = 1ll << level;
  if (j >= nseg) return;
  const int64_t t = nseg - 1 + j;
  const int b = T.b[t], s = T.s[t];
  const int sel = T.sel[t];
  const int64_t c1 = 2 * t + 1, c2 = 2 * t + 2;
  if (s <= 0) {
    T.ls[t] = -1;
    if (c2 < cap) {
      T.b[c1] = b; T.s[c1] = 0; T.sel[c1] = sel;
      T.b[c2] = b; T.s[c2] = 0; T.sel[c2] = sel;
    }
    return;
  }
  const int ls = left_size(s);
  float ext[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const float* c = Lst.comp(d, (sel >> d) & 1, d);
    ext[d] = c[b + s - 1] - c[b];
  }
  int dim = 0;
  if (ext[1] > ext[dim]) dim = 1;
  if (ext[2] > ext[dim]) dim = 2;
  const float4 e = kd_elem(Lst, dim, (sel >> dim) & 1, b + ls);
  const int id = __float_as_int(e.w);
  T.ls[t] = ls;
  T.dim[t] = dim;
  T.coord[t] = coord_of(e, dim);
  T.id[t] = id;
  out_nodes[t] = make_float4(e.x, e.y, e.z, __int_as_float((id << 2) | dim));
  if (c2 < cap) {
    // the two non-split lists move to the other buffer this level
    const int csel = sel ^ (7 ^ (1 << dim));
    T.b[c1] = b; T.s[c1] = ls; T.sel[c1] = csel;
    T.b[c2] = b + ls + 1; T.s[c2] = s - ls - 1; T.sel[c2] = csel;
  }
}

// class of element e relative to node key (coord, id) along dim: 0 left, 1 node, 2 right
__device__ __forceinline__ int kd_class(const float4 e, int dim, float nc, int nid) {
  const float c = coord_of(e, dim);
  const int id = __float_as_int(e.w);
  if (c < nc || (c == nc && id < nid)) return 0;
  if (id == nid) return 1;
  return 2;
}

// ------------------------------------------------------------------ partition
// Per level: positions are cut into 512-position tiles; the element at each
// position of the two non-split lists is classed against its segment's median
// (L / M / R; the split list and placed positions: 3) and the packed (L, R)
// counts are scanned SEGMENTED (reset at segment starts):
//   k_kd_count     per-tile segmented aggregate (reads the split coordinate,
//                  the index only on a coordinate tie; a block sum of packed
//                  tile-local counts),
//   k_kd_chunkscan / k_kd_chunkcarry  exclusive segmented carry per tile,
//   k_kd_part      block scan of the packed counts + carry -> stable scatter
//                  into the other buffer:
//                  L -> b + #L before it in the segment, M -> b + ls,
//                  R -> b + ls + 1 + #R before it.
// Kernel boundaries order the passes (a decoupled look-back needs agent-scope
// release fences per tile, i.e. L2 write-backs across the 8 XCDs: measured
// 7 ms per level). Traffic per element and level: count 2 x 4 B, part 2 x 16 B
// read + 2 x 16 B written (72 B; the AoS lists that moved all three 16-B lists
// and a segment tag per position took 140 B).
// Occupancy targets (waves per SIMD, 0 = compiler's choice), build-time A/B knobs.
#ifndef PM_KD_PART_WAVES
#define PM_KD_PART_WAVES 8   // 84 -> 64 VGPRs, no spill: kd build 27.4 -> 26.6 ms (5 waves: the default allocation)
#endif
#ifndef PM_KD_COUNT_WAVES
#define PM_KD_COUNT_WAVES 0
#endif
// threads of a partition block; the tile is PM_KD_IPT positions per thread
// (config 3 kd build, AoS lists, round 1: 256 x 4 44.5 ms (count 114 / part 142
// VGPRs), 256 x 2 36.4 ms (58 / 92), 256 x 1 36.6 ms)
#ifndef PM_KD_PART_THREADS
#define PM_KD_PART_THREADS 256
#endif
#ifndef PM_KD_IPT
#define PM_KD_IPT 2
#endif
constexpr int kPartThreads = PM_KD_PART_THREADS;
constexpr int kPartIPT = PM_KD_IPT;
constexpr int kPartTile = kPartThreads * kPartIPT;   // positions per tile
static_assert(kPartTile < 1024, "tile-local counts are packed in 10-bit fields (pack_cls)");

struct SegVal {   // segmented-scan value: packed (L | R << 32) count per list
  uint64_t v[3];
  uint32_t f;     // contains a segment start
};

__device__ __forceinline__ SegVal seg_zero() {
  SegVal r;
  r.v[0] = r.v[1] = r.v[2] = 0;
  r.f = 0;
  return r;
}

__device__ __forceinline__ SegVal seg_combine(const SegVal& a, const SegVal& b) {   // a before b
  SegVal r;
#pragma unroll
  for (int d = 0; d < 3; d++) r.v[d] = b.f ? b.v[d] : a.v[d] + b.v[d];
  r.f = a.f | b.f;
  return r;
}

__device__ __forceinline__ SegVal seg_shfl_up(const SegVal& x, int delta) {
  SegVal r;
#pragma unroll
  for (int d = 0; d < 3; d++) r.v[d] = __shfl_up(x.v[d], delta);
  r.f = (uint32_t)__shfl_up((int)x.f, delta);
  return r;
}

// Block-wide exclusive segmented scan (blockDim = W * 64); also returns the
// block aggregate. `sh` holds W entries.
template <int W>
__device__ __forceinline__ SegVal block_seg_scan(const SegVal& th, SegVal* sh, SegVal& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  SegVal inc = th;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const SegVal up = seg_shfl_up(inc, o);
    if (lane >= o) inc = seg_combine(up, inc);
  }
  if (lane == 63) sh[wave] = inc;
  __syncthreads();
  SegVal ex = seg_shfl_up(inc, 1);
  if (lane == 0) ex = seg_zero();
  SegVal wpre = seg_zero();
  total = seg_zero();
#pragma unroll
  for (int w = 0; w < W; w++) {
    if (w < wave) wpre = seg_combine(wpre, sh[w]);
    total = seg_combine(total, sh[w]);
  }
  __syncthreads();   // sh is reused by the next call
  return seg_combine(wpre, ex);
}

// Segment lookup without a per-position tag array: the segments of a level are
// the heap nodes t = 2^L - 1 + j, j = 0 .. 2^L - 1, left to right with
// non-decreasing starts b_j (a gap between two holds the medians of earlier
// levels: placed positions). k_kd_tileseg finds, per 512-position tile, the
// last segment starting at or before the tile; a block then knows that its
// positions lie in segments jl .. jh (jh: the next tile's first). Up to
// kSegCache records are staged in LDS (the usual case: a global-level segment
// holds >= 1023 positions, so a tile meets one or two); more (the check
// variant's tiny deep segments) fall back to a binary search in global memory.
// This replaced a 4-B tag per position read by both passes and rewritten by
// the part pass, and the per-position dependent loads of the segment record.
constexpr int kSegCache = 8;

struct SegRec {
  int b, s, ls, dim, id, sel;
  float coord;
};

__device__ __forceinline__ SegRec seg_load(const SegTab& T, int64_t t) {
  SegRec r;
  r.b = T.b[t];
  r.s = T.s[t];
  r.ls = T.ls[t];
  r.dim = T.dim[t];
  r.id = T.id[t];
  r.sel = T.sel[t];
  r.coord = T.coord[t];
  return r;
}

__global__ void k_kd_tileseg(const int32_t* __restrict__ tb, int level, int64_t ntiles, int32_t* __restrict__ tile_seg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > ntiles) return;
  const int64_t base = (1ll << level) - 1, nseg = 1ll << level;
  const int64_t p = i < ntiles ? i * kPartTile : INT64_MAX;
  int64_t lo = 0, hi = nseg;   // last j with b_j <= p (b_0 = 0)
  while (hi - lo > 1) {
    const int64_t m = (lo + hi) >> 1;
    if ((int64_t)tb[base + m] <= p) lo = m;
    else hi = m;
  }
  tile_seg[i] = (int32_t)lo;
}

// Per-block view of the segments [jl, jh] that can hold the block's positions.
struct TileSegs {
  int jl, jh;
  bool cached;
  int64_t last_start;   // largest start of a (non-empty) subtree inside the tile, -1: none
};

__device__ __forceinline__ TileSegs tile_segs(const SegTab& T, int level, const int32_t* __restrict__ tile_seg,
                                              SegRec* cache) {
  TileSegs ts;
  ts.jl = tile_seg[blockIdx.x];
  ts.jh = tile_seg[blockIdx.x + 1];
  ts.cached = ts.jh - ts.jl < kSegCache;
  const int64_t base = (1ll << level) - 1;
  const int64_t t0 = (int64_t)blockIdx.x * kPartTile;
  __shared__ long long s_last;
  if (threadIdx.x == 0) s_last = -1;
  __syncthreads();
  for (int j = ts.jl + (int)threadIdx.x; j <= ts.jh; j += blockDim.x) {
    const SegRec r = seg_load(T, base + j);
    if (ts.cached) cache[j - ts.jl] = r;
    if (r.s > 0 && r.b >= t0 && r.b < t0 + kPartTile) atomicMax(&s_last, (long long)r.b);
  }
  __syncthreads();
  ts.last_start = s_last;
  return ts;
}

// segment of position p (false: p is a placed median / outside every segment)
__device__ __forceinline__ bool seg_find(const SegTab& T, int level, const TileSegs& ts, const SegRec* cache,
                                         int64_t p, SegRec& r) {
  if (ts.cached) {
    int k = 0;
    for (int c = 1; c <= ts.jh - ts.jl; c++)
      if ((int64_t)cache[c].b <= p) k = c;
    r = cache[k];
  } else {
    const int64_t base = (1ll << level) - 1;
    int lo = ts.jl, hi = ts.jh + 1;
    while (hi - lo > 1) {
      const int m = (lo + hi) >> 1;
      if ((int64_t)T.b[base + m] <= p) lo = m;
      else hi = m;
    }
    r = seg_load(T, base + lo);
  }
  return r.s > 0 && p >= r.b && p < (int64_t)r.b + r.s;
}

// Striped tiles: item k of thread i sits at position tile*512 + k*256 + i, so
// every wave access covers 64 consecutive positions; the segmented scan runs
// once per k-round, carried across rounds.
struct PartItem {
  int sb, sls, sel;
  bool live;
  uint8_t cls[3];   // 0 L, 1 M, 2 R, 3 not moved (split list / placed / out of range)
};

// Classes of position p in the three lists; KEEP: also load the moved
// elements (into e[d]). The split list is never loaded (positional).
template <bool KEEP>
__device__ __forceinline__ SegVal part_load(const KdLists& Lst, int64_t n, const SegTab& T, int level,
                                            const TileSegs& ts, const SegRec* cache, int64_t p, PartItem& it,
                                            float4 (&e)[3]) {
  SegVal th = seg_zero();
  SegRec r{};
  it.live = p < n && seg_find(T, level, ts, cache, p, r);
  it.sb = r.b;
  it.sls = r.ls;
  it.sel = r.sel;
  const int dim = r.dim, nid = r.id;
  const float nc = r.coord;
  th.f = it.live && p == it.sb;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    int c = 3;
    if (it.live && d != dim) {
      const int k = (it.sel >> d) & 1;
      if (KEEP) {
        e[d] = kd_elem(Lst, d, k, p);
        c = kd_class(e[d], dim, nc, nid);
      } else {
        // count pass: the split coordinate alone decides unless it ties the
        // median's (then the index does; the median itself has c == nc) --
        // kd_class's predicate on the loaded coordinate (positions are never
        // NaN: k_elems_* map NaN to +inf, so == and the sort keys agree)
        const float cv = Lst.comp(d, k, dim)[p];
        if (cv < nc) c = 0;
        else if (!(cv == nc)) c = 2;
        else {
          const int id = __float_as_int(Lst.comp(d, k, 3)[p]);
          c = id < nid ? 0 : (id == nid ? 1 : 2);
        }
      }
    }
    it.cls[d] = (uint8_t)c;
    th.v[d] = c == 0 ? 1ull : (c == 2 ? (1ull << 32) : 0ull);
  }
  return th;
}

// Tile-local counts packed in one u64: list d's L count at bits 20d, its R
// count at bits 20d + 10 (a tile has 512 positions: 10 bits per field).
__device__ __forceinline__ uint64_t pack_cls(const PartItem& it) {
  uint64_t v = 0;
#pragma unroll
  for (int d = 0; d < 3; d++)
    v |= (uint64_t)(it.cls[d] == 0) << (20 * d) | (uint64_t)(it.cls[d] == 2) << (20 * d + 10);
  return v;
}
__device__ __forceinline__ uint32_t field_l(uint64_t v, int d) { return (uint32_t)(v >> (20 * d)) & 1023u; }
__device__ __forceinline__ uint32_t field_r(uint64_t v, int d) { return (uint32_t)(v >> (20 * d + 10)) & 1023u; }

// Block-wide sum of a u64 (blockDim = kPartThreads).
__device__ __forceinline__ uint64_t block_sum_u64(uint64_t v, uint64_t* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int w = 0; w < kPartThreads / 64; w++) t += sh[w];
  return t;
}

// Per-tile segmented aggregate: the (L, R) counts of the positions at or after
// the last subtree start inside the tile (all positions if none starts in it),
// and whether one starts -- a plain wave sum, no scan. One wave per tile (the
// tile's positions striped over its 64 lanes): the pass is bound by each
// tile's dependent loads (tile -> subtree records -> split coordinates), so
// small blocks keep 4x more tiles in flight than a 256-thread tile did.
constexpr int kCountThreads = 64;
constexpr int kCountIPT = kPartTile / kCountThreads;
static_assert(kPartTile % kCountThreads == 0, "count tiles are striped over one wave");
__global__ __launch_bounds__(kCountThreads) PM_WAVES_ATTR(PM_KD_COUNT_WAVES) void k_kd_count(KdLists Lst, int64_t n,
                                                           SegTab T, int level,
                                                           const int32_t* __restrict__ tile_seg,
                                                           SegVal* __restrict__ tile_agg) {
  __shared__ SegRec cache[kSegCache];
  const TileSegs ts = tile_segs(T, level, tile_seg, cache);
  const int64_t base = (int64_t)blockIdx.x * kPartTile + threadIdx.x;
  uint64_t sum = 0;
  float4 dummy[3];
#pragma unroll
  for (int k = 0; k < kCountIPT; k++) {
    PartItem it;
    const int64_t p = base + k * kCountThreads;
    part_load<false>(Lst, n, T, level, ts, cache, p, it, dummy);
    if (p >= ts.last_start) sum += pack_cls(it);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (threadIdx.x == 0) {
    SegVal agg;
#pragma unroll
    for (int d = 0; d < 3; d++) agg.v[d] = (uint64_t)field_l(sum, d) | (uint64_t)field_r(sum, d) << 32;
    agg.f = ts.last_start >= 0;
    tile_agg[blockIdx.x] = agg;
  }
}

// Exclusive segmented prefix over the tile aggregates in two coalesced steps:
// k_kd_chunkscan scans chunks of 1024 tiles (one block each) and records each
// chunk's total; k_kd_chunkcarry scans the chunk totals in place (one block,
// 1024 chunks per round). k_kd_part combines the two carries.
// (A single block walking all tiles cost ~115 us per level.)
constexpr int kChunk = 1024;
__global__ __launch_bounds__(kChunk) void k_kd_chunkscan(const SegVal* __restrict__ agg, int64_t ntiles,
                                                         SegVal* __restrict__ carry, SegVal* __restrict__ chunk_agg) {
  __shared__ SegVal sh[kChunk / 64];
  const int64_t t = (int64_t)blockIdx.x * kChunk + threadIdx.x;
  const SegVal v = t < ntiles ? agg[t] : seg_zero();
  SegVal total;
  const SegVal ex = block_seg_scan<kChunk / 64>(v, sh, total);
  if (t < ntiles) carry[t] = ex;
  if (threadIdx.x == 0) chunk_agg[blockIdx.x] = total;
}

__global__ __launch_bounds__(kChunk) void k_kd_chunkcarry(SegVal* __restrict__ chunk_agg, int nchunks) {
  __shared__ SegVal sh[kChunk / 64];
  SegVal run = seg_zero();
  for (int base = 0; base < nchunks; base += kChunk) {   // one pass up to 2^20 tiles
    const int c = base + (int)threadIdx.x;
    const SegVal v = c < nchunks ? chunk_agg[c] : seg_zero();
    SegVal total;
    const SegVal ex = block_seg_scan<kChunk / 64>(v, sh, total);   // every read precedes its barriers
    if (c < nchunks) chunk_agg[c] = seg_combine(run, ex);
    run = seg_combine(run, total);
  }
}

// Block-wide inclusive scan of a u64 (blockDim = W * 64, W <= 64); total out.
// `sh` holds W + 1 entries: wave totals, then (after wave 0 scanned them) the
// exclusive wave prefixes and the block total, so a thread reads two values
// whatever W is (a per-thread loop over W loads kept 2W VGPRs live).
template <int W = kPartThreads / 64>
__device__ __forceinline__ uint64_t block_scan_u64(uint64_t v, uint64_t* sh, uint64_t& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t up = __shfl_up(v, o);
    if (lane >= o) v += up;
  }
  if (lane == 63) sh[wave] = v;
  __syncthreads();
  if (wave == 0) {
    uint64_t x = lane < W ? sh[lane] : 0ull;
#pragma unroll
    for (int o = 1; o < W; o <<= 1) {
      const uint64_t up = __shfl_up(x, o);
      if (lane >= o) x += up;
    }
    if (lane == W - 1) sh[W] = x;
    const uint64_t ex = __shfl_up(x, 1);
    if (lane < W) sh[lane] = lane == 0 ? 0ull : ex;
  }
  __syncthreads();
  const uint64_t pre = sh[wave];
  total = sh[W];
  __syncthreads();   // sh is reused by the next call
  return pre + v;
}

// Stable scatter of the tile's moving elements: a plain exclusive scan of the
// packed tile-local counts gives each position the counts before it in the
// tile; a subtree that starts inside the tile subtracts the prefix at its
// start, one that started before adds the carry of the earlier tiles.
__global__ __launch_bounds__(kPartThreads) PM_WAVES_ATTR(PM_KD_PART_WAVES) void k_kd_part(KdLists Lst, int64_t n,
                                                          SegTab T, int level,
                                                          const int32_t* __restrict__ tile_seg,
                                                          const SegVal* __restrict__ tile_carry,
                                                          const SegVal* __restrict__ chunk_carry) {
  __shared__ SegRec cache[kSegCache];
  __shared__ uint64_t sh[kPartThreads / 64 + 1];
  __shared__ uint64_t pre[kPartTile];   // exclusive tile-local prefix per position
  const TileSegs ts = tile_segs(T, level, tile_seg, cache);
  const int64_t t0 = (int64_t)blockIdx.x * kPartTile;
  const int64_t base = t0 + threadIdx.x;
  PartItem it[kPartIPT];
  float4 e[kPartIPT][3];
  uint64_t run = 0;
#pragma unroll
  for (int k = 0; k < kPartIPT; k++) {
    part_load<true>(Lst, n, T, level, ts, cache, base + k * kPartThreads, it[k], e[k]);
    const uint64_t v = pack_cls(it[k]);
    uint64_t total;
    const uint64_t inc = block_scan_u64(v, sh, total);
    pre[k * kPartThreads + threadIdx.x] = run + inc - v;
    run += total;
  }
  __syncthreads();
  const SegVal carry = seg_combine(chunk_carry[blockIdx.x / kChunk], tile_carry[blockIdx.x]);
#pragma unroll
  for (int k = 0; k < kPartIPT; k++) {
    const int64_t p = base + k * kPartThreads;
    if (!it[k].live) continue;
    const uint64_t mine = pre[p - t0];
    const bool inside = it[k].sb >= t0;   // the subtree starts in this tile
    const uint64_t before = inside ? mine - pre[it[k].sb - t0] : mine;   // field-wise (prefixes only grow)
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int c = it[k].cls[d];
      if (c == 3) continue;
      int64_t dst;
      if (c == 0) {
        dst = it[k].sb + (int64_t)field_l(before, d) + (inside ? 0 : (int64_t)(uint32_t)carry.v[d]);
      } else if (c == 1) {
        dst = it[k].sb + it[k].sls;
      } else {
        dst = it[k].sb + it[k].sls + 1 + (int64_t)field_r(before, d) +
              (inside ? 0 : (int64_t)(uint32_t)(carry.v[d] >> 32));
      }
      const int ko = ((it[k].sel >> d) & 1) ^ 1;
      Lst.comp(d, ko, 0)[dst] = e[k][d].x;
      Lst.comp(d, ko, 1)[dst] = e[k][d].y;
      Lst.comp(d, ko, 2)[dst] = e[k][d].z;
      Lst.comp(d, ko, 3)[dst] = e[k][d].w;
    }
  }
}

// ------------------------------------------------------------------ local finish
// Once every segment holds <= kLocal - 1 elements (global level L0 = H - kLocalLog),
// one workgroup per segment finishes all remaining levels in LDS: the three
// presorted lists of its range are loaded once (48 KB), and each local level
// picks every sub-segment's widest dimension and median from the lists,
// classes the elements, runs the block-wide segmented scan and scatters in
// place (every thread holds its three elements in registers across the
// barrier). Same rules as the global levels, so the tree is identical; the
// bottom ~10 levels no longer cost a global read + write each.
// PM_KD_LOCAL_LOG: log2 of the workgroup (10: 1024 threads, subtrees of <= 1023
// elements, two workgroups per CU; 9: 512 threads, one more global level, four
// workgroups per CU -- 32 waves either way -- with barriers half as wide and
// 45 instead of 55 sort stages). Measured on config 3: the kd phase 24.0 ms
// with 10, 31.2-31.7 ms with 9 (the extra global level costs more than the
// narrower finish saves); the tree is the same (parity tests pass with both).
#ifndef PM_KD_LOCAL_LOG
#define PM_KD_LOCAL_LOG 10
#endif
constexpr int kLocalLog = PM_KD_LOCAL_LOG;
constexpr int kLocal = 1 << kLocalLog;
// From local level kLocalLog - 6 on every sub-segment has <= 63 elements and
// there are kLocal / 64 of them: sub-segment j is finished by wave j with
// shuffles, a packed wave scan and ds_permute (no block barriers, no LDS);
// same rules, same tree.
constexpr int kLocalWaveLevel = kLocalLog - 6;
static_assert(kLocalLog >= 8 && kLocalLog <= 10, "sub-segment sizes are packed in 10-bit fields");
static_assert(kLocal / 64 == (1 << kLocalWaveLevel), "one wave per wave-level sub-segment");

// The selection build's elements: four SoA arrays (x, y, z, index bits) per
// buffer k (0 / 1), unsorted inside each subtree range.
struct KdSoa {
  float* base;
  int64_t n;
  __host__ __device__ float* comp(int k, int c) const { return base + (int64_t)(k * 4 + c) * n; }
};

// lane ^ stride exchange for stride < 64: DPP quad permutes for 1 and 2 (VALU),
// ds_swizzle's xor mode for 4 .. 16, ds_bpermute for 32
__device__ __forceinline__ int xor_lane(int v, int stride) {
  switch (stride) {
    case 1: return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1, 0, 3, 2]
    case 2: return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2, 3, 0, 1]
    case 4: return __builtin_amdgcn_ds_swizzle(v, 0x1F | (4 << 10));
    case 8: return __builtin_amdgcn_ds_swizzle(v, 0x1F | (8 << 10));
    case 16: return __builtin_amdgcn_ds_swizzle(v, 0x1F | (16 << 10));
    default: return __shfl_xor(v, stride);
  }
}

// min / max over the 64 lanes of a wave, valid in every lane: DPP row shifts
// inside each 16-lane row (identity shifted in), then the four row results
template <bool MAX>
__device__ __forceinline__ uint32_t wave_minmax(uint32_t v) {
  const int id = MAX ? 0 : (int)0xFFFFFFFFu;
  auto op = [](uint32_t a, uint32_t b) { return MAX ? max(a, b) : min(a, b); };
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 15), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 47), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  return op(op(a, b), op(c, d));
}

// u64 min / max over a wave: the high words first, then the low words of the
// lanes that hold the extreme high word
template <bool MAX>
__device__ __forceinline__ uint64_t wave_minmax64(uint64_t v) {
  const uint32_t hi = (uint32_t)(v >> 32);
  const uint32_t h = wave_minmax<MAX>(hi);
  const uint32_t lo = hi == h ? (uint32_t)v : (MAX ? 0u : 0xFFFFFFFFu);
  return (uint64_t)h << 32 | wave_minmax<MAX>(lo);
}

// Block-wide bitonic sort (blockDim = kLocal, one (key, slot) pair per thread,
// ascending over the first n2 threads, n2 a power of two >= 64): strides below
// 64 exchange through wave shuffles, larger ones through LDS (kx / vx).
__device__ __forceinline__ void block_bitonic(uint64_t& k, int& v, int n2, uint64_t* kx, int16_t* vx) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int ls = 1; ls <= kLocalLog; ls++) {   // size 2 .. kLocal, every stride a constant after unrolling
    const int size = 1 << ls;
#pragma unroll
    for (int lst = ls - 1; lst >= 0; lst--) {
      if (size > n2) continue;   // n2 is uniform: the barriers below are reached by all or none
      const int stride = 1 << lst;
      uint64_t pk;
      int pv;
      if (stride >= 64) {
        __syncthreads();   // the previous stage's reads are done
        kx[tid] = k;
        vx[tid] = (int16_t)v;
        __syncthreads();
        pk = kx[tid ^ stride];
        pv = vx[tid ^ stride];
      } else {
        pk = (uint64_t)(uint32_t)xor_lane((int)(uint32_t)k, stride) |
             (uint64_t)(uint32_t)xor_lane((int)(uint32_t)(k >> 32), stride) << 32;
        pv = xor_lane(v, stride);
      }
      const bool up = (tid & size) == 0, lower = (tid & stride) == 0;
      if (lower == up ? pk < k : pk > k) {
        k = pk;
        v = pv;
      }
    }
  }
}

// The three lists' sorts as ONE network (PM_KD_SORT3): every thread carries its
// element's three (key, slot) pairs through the same compare-exchange stages,
// so the stages that exchange through LDS pay their two block barriers once
// for all three lists instead of once per list (30 instead of 90 barriers per
// 1024-element block), and each in-wave stage has three independent chains.
// kx / vx: 3 kLocal u64 and 3 kLocal i16 of LDS scratch.
#ifndef PM_KD_SORT3
#define PM_KD_SORT3 1
#endif
__device__ __forceinline__ void block_bitonic3(uint64_t (&k)[3], int (&v)[3], int n2, uint64_t* kx, int16_t* vx) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int ls = 1; ls <= kLocalLog; ls++) {
    const int size = 1 << ls;
#pragma unroll
    for (int lst = ls - 1; lst >= 0; lst--) {
      if (size > n2) continue;   // uniform
      const int stride = 1 << lst;
      uint64_t pk[3];
      int pv[3];
      if (stride >= 64) {
        __syncthreads();
#pragma unroll
        for (int d = 0; d < 3; d++) {
          kx[d * kLocal + tid] = k[d];
          vx[d * kLocal + tid] = (int16_t)v[d];
        }
        __syncthreads();
#pragma unroll
        for (int d = 0; d < 3; d++) {
          pk[d] = kx[d * kLocal + (tid ^ stride)];
          pv[d] = vx[d * kLocal + (tid ^ stride)];
        }
      } else {
#pragma unroll
        for (int d = 0; d < 3; d++) {
          pk[d] = (uint64_t)(uint32_t)xor_lane((int)(uint32_t)k[d], stride) |
                  (uint64_t)(uint32_t)xor_lane((int)(uint32_t)(k[d] >> 32), stride) << 32;
          pv[d] = xor_lane(v[d], stride);
        }
      }
      const bool up = (tid & size) == 0, lower = (tid & stride) == 0;
#pragma unroll
      for (int d = 0; d < 3; d++) {
        if (lower == up ? pk[d] < k[d] : pk[d] > k[d]) {
          k[d] = pk[d];
          v[d] = pv[d];
        }
      }
    }
  }
}

// The wave levels of a local finish: sub-segment j of local level KB (<= 63
// elements, positions b0 .. b0 + sz0 - 1) is finished by wave j with shuffles,
// a packed wave scan and ds_permute (no block barriers, no LDS). e[d]: this
// lane's element in list d (the sub-segment sorted by (coordinate d, index));
// nodes go to stage[] by local heap index. (The lists come by value: an array
// parameter let the callee's selects of e[dim] become loads through a selected
// address, which kept e[] in scratch once inlined.)
__device__ __forceinline__ void local_wave_levels(float4 e0, float4 e1, float4 e2, int lane, int j, int KB, int H,
                                                  int b0, int sz0, float4* stage) {
  float4 e[3] = {e0, e1, e2};
  const bool active = lane < sz0;
  const int p = b0 + lane;                       // this lane's position (fixed)
  int b = b0, sz = sz0;                          // this lane's segment
  int lnode = (1 << KB) - 1 + j;                // local heap index of this lane's segment
  bool placed = !active;
  for (int k = KB; k < H && sz0 > 0; k++) {
    const int ls = placed ? 0 : left_size(sz);
    // segment extents and median from the lanes holding them (all lanes shuffle)
    const int lf = placed ? lane : b - b0, ll = placed ? lane : b + sz - 1 - b0;
    float ext[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const float c = coord_of(e[d], d);
      ext[d] = __shfl(c, ll) - __shfl(c, lf);
    }
    int dim = 0;
    if (ext[1] > ext[dim]) dim = 1;
    if (ext[2] > ext[dim]) dim = 2;
    // per component: a select of whole float4s indexed e[] dynamically,
    // which kept e[] in scratch for the whole wave phase
    const bool d0 = dim == 0, d1 = dim == 1;
    const float4 sel = make_float4(d0 ? e[0].x : (d1 ? e[1].x : e[2].x), d0 ? e[0].y : (d1 ? e[1].y : e[2].y),
                                   d0 ? e[0].z : (d1 ? e[1].z : e[2].z), d0 ? e[0].w : (d1 ? e[1].w : e[2].w));
    const int lm = placed ? lane : b + ls - b0;
    const float4 m = make_float4(__shfl(sel.x, lm), __shfl(sel.y, lm), __shfl(sel.z, lm), __shfl(sel.w, lm));
    const int nid = __float_as_int(m.w);
    const float nc = coord_of(m, dim);
    if (!placed && p == b + ls) stage[lnode] = make_float4(m.x, m.y, m.z, __int_as_float((nid << 2) | dim));
    if (k + 1 == H) break;
    // class per list, packed (L, R) counts: list d at bits 14d (L) and 14d + 7 (R)
    uint8_t c[3];
    uint64_t cnt = 0;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      c[d] = placed ? 3 : (uint8_t)kd_class(e[d], dim, nc, nid);
      cnt |= (uint64_t)(c[d] == 0) << (14 * d) | (uint64_t)(c[d] == 2) << (14 * d + 7);
    }
    uint64_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t up = __shfl_up(inc, o);
      if (lane >= o) inc += up;
    }
    const int lb = b - b0 - 1;   // lane before the segment (-1: none)
    const uint64_t before = __shfl(inc, lb < 0 ? 0 : lb);
    const uint64_t ex = inc - cnt - (lb < 0 || placed ? 0ull : before);
    // forward permute of the three elements to their positions in the segment
#pragma unroll
    for (int d = 0; d < 3; d++) {
      int dst = p;
      if (c[d] == 0) dst = b + (int)((ex >> (14 * d)) & 127);
      else if (c[d] == 1) dst = b + ls;
      else if (c[d] == 2) dst = b + ls + 1 + (int)((ex >> (14 * d + 7)) & 127);
      const int a = (dst - b0) * 4;
      e[d].x = __int_as_float(__builtin_amdgcn_ds_permute(a, __float_as_int(e[d].x)));
      e[d].y = __int_as_float(__builtin_amdgcn_ds_permute(a, __float_as_int(e[d].y)));
      e[d].z = __int_as_float(__builtin_amdgcn_ds_permute(a, __float_as_int(e[d].z)));
      e[d].w = __int_as_float(__builtin_amdgcn_ds_permute(a, __float_as_int(e[d].w)));
    }
    // positional segment update
    if (!placed) {
      if (p < b + ls) {
        sz = ls;
        lnode = 2 * lnode + 1;
      } else if (p == b + ls) {
        placed = true;
      } else {
        b = b + ls + 1;
        sz = sz - ls - 1;
        lnode = 2 * lnode + 2;
      }
    }
  }
}

// SORT (the selection build): the subtree's elements arrive unsorted in E; the
// three lists are made in LDS by sorting (orderable coordinate, index) keys,
// the presort's order. Otherwise they are loaded from the presorted lists.
template <bool SORT>
__global__ __launch_bounds__(kLocal) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_kd_local(KdLists Lst, KdSoa E,
                                                                                           int L0, SegTab T,
                                                                                           float4* __restrict__ nodes) {
  __shared__ float4 buf[3][kLocal];
  __shared__ int16_t tag[kLocal];
  constexpr int NS = 1 << kLocalWaveLevel;   // sub-segments at the wave level
  __shared__ int16_t sb[2][NS], ss[2][NS];   // sub-segment start / size, ping-pong by level
  __shared__ int16_t sls[NS / 2];
  __shared__ uint8_t sdim[NS / 2];
  __shared__ float sco[NS / 2];
  __shared__ int32_t sid[NS / 2];
  __shared__ uint64_t sh[kLocal / 64 + 1];
  __shared__ uint64_t spre[1 << kLocalWaveLevel];   // packed-count prefix at each sub-segment's start
  __shared__ float4 stage[kLocal];   // this subtree's nodes by local heap index (w = -1: none)
  const int tid = threadIdx.x;
  const int64_t t = ((int64_t)1 << L0) - 1 + blockIdx.x;
  const int B = T.b[t], S = T.s[t];
  if (S <= 0) return;
  if (SORT) {
    const int k0 = L0 & 1;
    float4 me = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < S) {
      me = make_float4(E.comp(k0, 0)[B + tid], E.comp(k0, 1)[B + tid], E.comp(k0, 2)[B + tid], E.comp(k0, 3)[B + tid]);
      buf[2][tid] = me;
    }
    int n2 = 64;
    while (n2 < S) n2 <<= 1;
    if (PM_KD_SORT3) {
      // scratch: buf[0] and buf[1] (written only after the sort), 24 KB of keys
      // then 6 KB of slots
      uint64_t* kx = reinterpret_cast<uint64_t*>(&buf[0][0]);
      int16_t* vx = reinterpret_cast<int16_t*>(kx + 3 * kLocal);
      uint64_t k[3];
      int v[3];
#pragma unroll
      for (int d = 0; d < 3; d++) {
        k[d] = tid < S ? (uint64_t)orderable_key(coord_of(me, d)) << 32 | (uint32_t)__float_as_int(me.w) : ~0ull;
        v[d] = tid;
      }
#ifndef PM_KD_DIAG_NOSORT
      block_bitonic3(k, v, n2, kx, vx);
#endif
      __syncthreads();   // buf[2] written; every exchange read
      // (loads only under tid < S: a select between an LDS element and a
      // register value compiled to a flat load through scratch)
      float4 x0, x1, x2;
      if (tid < S) {
        x0 = buf[2][v[0]];
        x1 = buf[2][v[1]];
        x2 = buf[2][v[2]];
      }
      __syncthreads();
      if (tid < S) {
        buf[0][tid] = x0;
        buf[1][tid] = x1;
        buf[2][tid] = x2;
      }
    } else {
      uint64_t* kx = reinterpret_cast<uint64_t*>(stage);   // scratch until stage is set below
#pragma unroll 1
      for (int d = 0; d < 3; d++) {
        uint64_t k = tid < S ? (uint64_t)orderable_key(coord_of(me, d)) << 32 | (uint32_t)__float_as_int(me.w) : ~0ull;
        int v = tid;
        block_bitonic(k, v, n2, kx, tag);
        __syncthreads();   // buf[2] written; every exchange read
        float4 x;
        if (tid < S) x = buf[2][v];
        if (d == 2) __syncthreads();
        if (tid < S) buf[d][tid] = x;
      }
    }
    __syncthreads();
  } else {
    const int sel = T.sel[t];
    if (tid < S) {
#pragma unroll
      for (int d = 0; d < 3; d++) buf[d][tid] = kd_elem(Lst, d, (sel >> d) & 1, B + tid);
    }
  }
  tag[tid] = tid < S ? 0 : -1;
  stage[tid] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  if (tid == 0) {
    sb[0][0] = 0;
    ss[0][0] = (int16_t)S;
  }
  const int H = 32 - __clz(S);   // levels of this subtree
  const int KB = min(H, kLocalWaveLevel);   // block-wide levels; the rest run per wave
  for (int k = 0; k < KB; k++) {
    const int cur = k & 1;
    const int nsub = 1 << k;
    __syncthreads();
    // sub-segment roots of this level
    if (tid < nsub) {
      const int b = sb[cur][tid], sz = ss[cur][tid];
      int ls = 0;
      if (sz > 0) {
        ls = left_size(sz);
        float ext[3];
#pragma unroll
        for (int d = 0; d < 3; d++) ext[d] = coord_of(buf[d][b + sz - 1], d) - coord_of(buf[d][b], d);
        int dim = 0;
        if (ext[1] > ext[dim]) dim = 1;
        if (ext[2] > ext[dim]) dim = 2;
        const float4 e = buf[dim][b + ls];
        const int id = __float_as_int(e.w);
        sdim[tid] = (uint8_t)dim;
        sco[tid] = coord_of(e, dim);
        sid[tid] = id;
        stage[(1 << k) - 1 + tid] = make_float4(e.x, e.y, e.z, __int_as_float((id << 2) | dim));
      }
      sls[tid] = (int16_t)ls;
      if (k + 1 < H) {
        const int nxt = cur ^ 1;
        sb[nxt][2 * tid] = (int16_t)b;
        ss[nxt][2 * tid] = (int16_t)(sz > 0 ? ls : 0);
        sb[nxt][2 * tid + 1] = (int16_t)(b + ls + 1);
        ss[nxt][2 * tid + 1] = (int16_t)(sz > 0 ? sz - ls - 1 : 0);
      }
    }
    if (k + 1 == H) break;
    __syncthreads();
    // class, scan of the packed counts (10 bits per field: a sub-segment holds
    // <= 1023) and in-place stable scatter of the three lists; counts before a
    // position in its sub-segment = its exclusive prefix - the prefix at the
    // sub-segment's start (block levels: <= 8 sub-segments)
    const int j = tag[tid];
    float4 e[3];
    uint8_t c[3];
    uint64_t v = 0;
    int b = 0, ls = 0;
    if (j >= 0) {
      b = sb[cur][j];
      ls = sls[j];
    }
#pragma unroll
    for (int d = 0; d < 3; d++) {
      e[d] = buf[d][tid];
      c[d] = j < 0 ? 3 : (uint8_t)kd_class(e[d], sdim[j >= 0 ? j : 0], sco[j >= 0 ? j : 0], sid[j >= 0 ? j : 0]);
      v |= (uint64_t)(c[d] == 0) << (20 * d) | (uint64_t)(c[d] == 2) << (20 * d + 10);
    }
    uint64_t total;
    const uint64_t inc = block_scan_u64<kLocal / 64>(v, sh, total);   // ends with a barrier: all reads done
    if (j >= 0 && tid == b) spre[j] = inc - v;
    __syncthreads();
    const uint64_t before = inc - v - (j >= 0 ? spre[j] : 0ull);
#pragma unroll
    for (int d = 0; d < 3; d++) {
      int dst;
      if (c[d] == 3) dst = tid;
      else if (c[d] == 0) dst = b + (int)field_l(before, d);
      else if (c[d] == 1) dst = b + ls;
      else dst = b + ls + 1 + (int)field_r(before, d);
      if (tid < S) buf[d][dst] = e[d];
    }
    if (j >= 0) tag[tid] = (int16_t)(tid < b + ls ? 2 * j : (tid == b + ls ? -1 : 2 * j + 1));
  }
  __syncthreads();
#ifdef PM_KD_DIAG_NOWAVE
  if (false) {
#else
  if (KB < H) {
#endif
    // ---- wave phase: sub-segment j of local level KB (<= 63 elements) -> wave j
    const int lane = tid & 63, j = tid >> 6;
    const int cur = KB & 1;
    const int b0 = sb[cur][j], sz0 = ss[cur][j];
    float4 e[3];
#pragma unroll
    for (int d = 0; d < 3; d++) e[d] = lane < sz0 ? buf[d][b0 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    local_wave_levels(e[0], e[1], e[2], lane, j, KB, H, b0, sz0, stage);
  }
  // ---- write-out: nodes leave LDS once, level by level (contiguous heap ranges);
  // a global store inside the level loop made every block barrier wait for it
  __syncthreads();
  const float4 nd = stage[tid];
  if (__float_as_int(nd.w) >= 0) {
    const int k = 31 - __clz(tid + 1);
    nodes[(t + 1) * ((int64_t)1 << k) - 1 + (tid + 1 - (1 << k))] = nd;
  }
}

// Local finish of the selection build without sorting the three lists
// (PM_KD_LOCAL_SEL): the block levels (local levels 0 ..
// KB - 1, <= 8 sub-segments) SELECT each sub-segment's median like the global
// levels do, on ONE unsorted list in LDS:
//   extents   the orderable-key min / max of every sub-segment's elements
//             (wave reductions, one LDS atomic per wave and sub-segment);
//   histogram 1024 bins per level shared by the sub-segments, the coordinate
//             key scaled to the sub-segment's key range (monotone: equal keys
//             share a bin, bins follow the order); the bin holding rank
//             left_size(sz) is found by one wave per sub-segment;
//   rank      that bin's elements are appended to a candidate list as unique
//             (key, index) keys, and each ranks itself among them;
//   partition every element moves to its child range (unstable: one LDS
//             atomic per wave, sub-segment and side; the order inside a range
//             does not matter, the median is defined by rank).
// The wave levels then sort each <= 63-element sub-segment's three lists in its
// wave (a 64-lane bitonic network, no barriers) and run local_wave_levels as
// the sorting finish does. Same rules, same medians, same tree; the sort of
// 1,024 keys x 3 lists it replaces was 3.0 of k_kd_local<true>'s 6.6 ms per
// config-3 frame (profiles/r06/r06b_kd_local_nosort_diag.txt).
#ifndef PM_KD_LOCAL_SEL
#define PM_KD_LOCAL_SEL 1
#endif
constexpr int kLocalBins = 1024;   // histogram bins per block level (all sub-segments)
// PM_KD_DIAG_TIME (diagnostic builds only): thread 0 of each local-finish
// workgroup stamps clock64() at its phase boundaries; pm_diag_kd_stamps copies
// them out (tools/kd_local_diag.py).
#ifdef PM_KD_DIAG_TIME
constexpr int kDiagBlocks = 1 << 16, kDiagStamps = 8;
__device__ unsigned long long g_kd_stamp[kDiagBlocks * kDiagStamps];
#define KD_STAMP(i)                                                                            \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kDiagBlocks) g_kd_stamp[blockIdx.x * kDiagStamps + (i)] = clock64(); \
  } while (0)
#else
#define KD_STAMP(i) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ uint32_t key_of(const float4 e, int d) { return orderable_key(coord_of(e, d)); }
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// In-wave bitonic sort (ascending) of one (key, slot) pair per lane, 64 lanes.
__device__ __forceinline__ void wave_bitonic(uint64_t& k, int& v, int lane) {
#pragma unroll
  for (int ls = 1; ls <= 6; ls++) {
    const int size = 1 << ls;
#pragma unroll
    for (int lst = ls - 1; lst >= 0; lst--) {
      const int stride = 1 << lst;
      const uint64_t pk = (uint64_t)(uint32_t)xor_lane((int)(uint32_t)k, stride) |
                          (uint64_t)(uint32_t)xor_lane((int)(uint32_t)(k >> 32), stride) << 32;
      const int pv = xor_lane(v, stride);
      const bool up = (lane & size) == 0, lower = (lane & stride) == 0;
      if (lower == up ? pk < k : pk > k) {
        k = pk;
        v = pv;
      }
    }
  }
}

__global__ __launch_bounds__(kLocal) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_kd_local_sel(
    KdSoa E, int L0, SegTab T, float4* __restrict__ nodes) {
  constexpr int NS = 1 << kLocalWaveLevel;   // sub-segments at the wave level
  constexpr int NB = NS / 2;                  // <= sub-segments at a block level
  __shared__ float4 buf[kLocal];              // the elements by position
  __shared__ float4 stage[kLocal];            // this subtree's nodes by local heap index (w = -1: none)
  __shared__ uint32_t hist[kLocalBins];
  __shared__ uint64_t cand[kLocal];           // a sub-segment's candidates at its own positions
  __shared__ uint32_t kmin[2][NB][3], kmax[2][NB][3];   // per level parity
  __shared__ int16_t sb[2][NS], ss[2][NS];
  __shared__ int16_t sls[NB];
  __shared__ uint32_t sbin[NB], srank[NB], scnt[NB], sl[NB], sr[NB];
  __shared__ float sco[NB];
  __shared__ int32_t sid[NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t t = ((int64_t)1 << L0) - 1 + blockIdx.x;
  const int B = T.b[t], S = T.s[t];
  if (S <= 0) return;
  const int k0 = L0 & 1;
  KD_STAMP(0);
  float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid < S) e = make_float4(E.comp(k0, 0)[B + tid], E.comp(k0, 1)[B + tid], E.comp(k0, 2)[B + tid], E.comp(k0, 3)[B + tid]);
  int j = tid < S ? 0 : -1;   // sub-segment of this position (-1: placed or empty)
  stage[tid] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  for (int i = tid; i < kLocalBins; i += kLocal) hist[i] = 0;
  if (tid < 2 * NB * 3) {
    (&kmin[0][0][0])[tid] = 0xFFFFFFFFu;
    (&kmax[0][0][0])[tid] = 0u;
  }
  if (tid == 0) {
    sb[0][0] = 0;
    ss[0][0] = (int16_t)S;
  }
  const int H = 32 - __clz(S);                 // levels of this subtree
  const int KB = min(H, kLocalWaveLevel);      // block levels; the rest run per wave
  __syncthreads();
  // extents of this position's sub-segment at level k (parity par): per wave,
  // one reduction and one LDS atomic per sub-segment present
  auto extents = [&](int par) {
    uint64_t todo = __builtin_amdgcn_ballot_w64(j >= 0);
    while (todo) {
      const int l = __ffsll((long long)todo) - 1;
      const int sj = __builtin_amdgcn_readlane(j, l);
      const bool m = j == sj;
      todo &= ~__builtin_amdgcn_ballot_w64(m);
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const uint32_t kd = key_of(e, d);
        const uint32_t mn = wave_minmax<false>(m ? kd : 0xFFFFFFFFu), mx = wave_minmax<true>(m ? kd : 0u);
        if (lane == l) {
          atomicMin(&kmin[par][sj][d], mn);
          atomicMax(&kmax[par][sj][d], mx);
        }
      }
    }
  };
  extents(0);
  KD_STAMP(1);
  for (int k = 0; k < KB; k++) {
    const int cur = k & 1, nsub = 1 << k, nbin = kLocalBins >> k;
    __syncthreads();   // extents complete
    // split dimension, key range and bin of this position's element
    int dim = 0;
    uint32_t key = 0, bin = 0;
    if (j >= 0) {
      float ext[3];
#pragma unroll
      for (int d = 0; d < 3; d++) ext[d] = unkey(kmax[cur][j][d]) - unkey(kmin[cur][j][d]);
      if (ext[1] > ext[dim]) dim = 1;
      if (ext[2] > ext[dim]) dim = 2;
      const uint32_t lo = kmin[cur][j][dim], hi = kmax[cur][j][dim];
      key = key_of(e, dim);
      const float scale = (float)nbin / ((float)(hi - lo) + 1.f);
      bin = min((uint32_t)nbin - 1u, (uint32_t)((float)(key - lo) * scale));
      atomicAdd(&hist[j * nbin + bin], 1u);
    }
    __syncthreads();   // histogram complete
    // wave w < nsub: sub-segment w's bin holding rank ls; its children's ranges
    if (wave < nsub) {
      const int sz = ss[cur][wave], b = sb[cur][wave];
      const int ls = sz > 0 ? left_size(sz) : 0;
      if (sz > 0) {
        constexpr int PER = kLocalBins / 64;   // bins per lane at level 0
        const int per = PER >> k;              // nbin / 64 (>= 2 at the block levels)
        uint32_t c[PER];
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < PER; q++) {
          c[q] = q < per ? hist[wave * nbin + lane * per + q] : 0u;
          sum += c[q];
        }
        uint32_t inc = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t up = __shfl_up(inc, o);
          if (lane >= o) inc += up;
        }
        const uint32_t exl = inc - sum;
        // the lane whose bins cover rank ls
        if (exl <= (uint32_t)ls && (uint32_t)ls < inc) {
          uint32_t acc = exl, fb = 0, rr = 0;
          bool found = false;
#pragma unroll
          for (int q = 0; q < PER; q++) {
            if (!found && q < per && (uint32_t)ls < acc + c[q]) {
              fb = (uint32_t)(lane * per + q);
              rr = (uint32_t)ls - acc;
              found = true;
            }
            acc += c[q];
          }
          sbin[wave] = fb;
          srank[wave] = rr;
        }
      }
      if (lane == 0) {
        sls[wave] = (int16_t)ls;
        scnt[wave] = 0;
        sl[wave] = 0;
        sr[wave] = 0;
        if (k + 1 < H) {
          const int nxt = cur ^ 1;
          sb[nxt][2 * wave] = (int16_t)b;
          ss[nxt][2 * wave] = (int16_t)(sz > 0 ? ls : 0);
          sb[nxt][2 * wave + 1] = (int16_t)(b + ls + 1);
          ss[nxt][2 * wave + 1] = (int16_t)(sz > 0 ? sz - ls - 1 : 0);
        }
      }
    }
    __syncthreads();   // bins found
    // the found bin's elements: unique (key, index) candidates
    const int idx = __float_as_int(e.w);
    const uint64_t ck = (uint64_t)key << 32 | (uint32_t)idx;
    const bool isc = j >= 0 && bin == sbin[j];
    const int cb = j >= 0 ? sb[cur][j] : 0;
    if (isc) cand[cb + atomicAdd(&scnt[j], 1u)] = ck;
    for (int i = tid; i < kLocalBins; i += kLocal) hist[i] = 0;   // this level's histogram is read; the next starts at zero
    if (tid < NB * 3) {   // the next level's extents start empty
      (&kmin[cur ^ 1][0][0])[tid] = 0xFFFFFFFFu;
      (&kmax[cur ^ 1][0][0])[tid] = 0u;
    }
    __syncthreads();   // candidates complete
    if (isc) {
      const uint32_t m = scnt[j];
      uint32_t r = 0;
      for (uint32_t i = 0; i < m; i++) r += cand[cb + i] < ck ? 1u : 0u;
      if (r == srank[j]) {
        sco[j] = coord_of(e, dim);
        sid[j] = idx;
        stage[(1 << k) - 1 + j] = make_float4(e.x, e.y, e.z, __int_as_float((idx << 2) | dim));
      }
    }
    if (k + 1 == H) break;
    __syncthreads();   // medians known
    // partition (unstable): left -> [b, b + ls), median -> b + ls, right -> [b + ls + 1, b + sz)
    int dst = tid;
    int cls = 3;
    if (j >= 0) cls = kd_class(e, dim, sco[j], sid[j]);
    {
      uint64_t todo = __builtin_amdgcn_ballot_w64(j >= 0);
      while (todo) {
        const int l = __ffsll((long long)todo) - 1;
        const int sj = __builtin_amdgcn_readlane(j, l);
        const bool m = j == sj;
        todo &= ~__builtin_amdgcn_ballot_w64(m);
        const uint64_t ml = __builtin_amdgcn_ballot_w64(m && cls == 0), mr = __builtin_amdgcn_ballot_w64(m && cls == 2);
        uint32_t bl = 0, br = 0;
        if (lane == l) {
          if (ml) bl = atomicAdd(&sl[sj], (uint32_t)__popcll(ml));
          if (mr) br = atomicAdd(&sr[sj], (uint32_t)__popcll(mr));
        }
        bl = (uint32_t)__builtin_amdgcn_readlane((int)bl, l);
        br = (uint32_t)__builtin_amdgcn_readlane((int)br, l);
        if (m) {
          const int b = sb[cur][sj], ls = sls[sj];
          const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
          if (cls == 0) dst = b + (int)bl + __popcll(ml & lt);
          else if (cls == 1) dst = b + ls;
          else dst = b + ls + 1 + (int)br + __popcll(mr & lt);
        }
      }
    }
    // the position's sub-segment after the move (positions keep their meaning)
    int nj = -1;
    if (j >= 0) {
      const int b = sb[cur][j], ls = sls[j];
      nj = tid < b + ls ? 2 * j : (tid == b + ls ? -1 : 2 * j + 1);
    }
    // (buf was last read at the previous level's reload, several barriers ago)
    if (tid < S) buf[dst] = e;
    __syncthreads();
    if (tid < S) e = buf[tid];
    j = nj;
    extents(cur ^ 1);
    if (k < 4) KD_STAMP(2 + k);
  }
  if (KB < H) {
    __syncthreads();
    // ---- wave levels: sub-segment `wave` of local level KB, sorted in the wave
    const int cur = KB & 1;
    const int b0 = sb[cur][wave], sz0 = ss[cur][wave];
    const float4 el = lane < sz0 ? buf[b0 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 es[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
      uint64_t kk = lane < sz0 ? (uint64_t)key_of(el, d) << 32 | (uint32_t)__float_as_int(el.w) : ~0ull;
      int v = lane;
      wave_bitonic(kk, v, lane);
      es[d] = make_float4(__shfl(el.x, v), __shfl(el.y, v), __shfl(el.z, v), __shfl(el.w, v));
    }
    KD_STAMP(6);
    local_wave_levels(es[0], es[1], es[2], lane, wave, KB, H, b0, sz0, stage);
  }
  // ---- write-out: nodes leave LDS once, level by level (contiguous heap ranges)
  __syncthreads();
  const float4 nd = stage[tid];
  if (__float_as_int(nd.w) >= 0) {
    const int k = 31 - __clz(tid + 1);
    nodes[(t + 1) * ((int64_t)1 << k) - 1 + (tid + 1 - (1 << k))] = nd;
  }
  KD_STAMP(7);
}

// ------------------------------------------------------------------ selection build
// The production build (round 3): no presort. The elements stay unsorted in
// their subtree ranges (SoA, ping-pong by level) and every global level
//   k_ks_seg      picks each subtree's split dimension from its extents (the
//                 orderable-key min / max of its elements, reduced by the
//                 previous level's partition) -- the same float extents the
//                 presorted lists give (first and last element);
//   k_ks_hist / k_ks_find / k_ks_compact / k_ks_cand
//                 select the element of rank left_size(s) in (coordinate,
//                 index) order: a 256-bin histogram of the coordinate scaled to
//                 the subtree's range (monotone in the coordinate, so equal
//                 coordinates share a bin and bins follow the order), the bin
//                 holding the rank, a compaction of that bin's elements into
//                 the subtree's own range of a candidate buffer as the unique
//                 keys K = (orderable(coord) - min) << idbits | index, and one
//                 workgroup per subtree that radix-selects among them (8-bit
//                 digits while more than 256 match, then a sort in LDS);
//   k_ks_part     moves every element to its child range (unstable: one atomic
//                 per wave and (subtree, side) reserves slots; the order inside
//                 a range does not matter, the median is defined by rank) and
//                 reduces the children's extents.
// Per element and level: 4 B (histogram) + 4 B (compaction) + 16 B read and
// 16 B written (partition), against the presorted build's 72 B plus its
// 12-pass presort. Once subtrees hold <= 1023 elements, k_kd_local<true> sorts
// each one's three lists in LDS and finishes it like the presorted build.
// Same medians, same tree: the check variant keeps the presorted build, and
// tests/test_gpu_check_variant.py compares the two bit for bit.
#ifndef PM_KS_IPT
#define PM_KS_IPT 8   // positions per thread of the per-position selection kernels
#endif
#ifndef PM_KS_NSUB
#define PM_KS_NSUB 4   // sub-tiles per block (one subtree prologue for all of them)
#endif
#ifndef PM_KS_THREADS
#define PM_KS_THREADS 256   // threads per block of the per-position selection kernels
#endif
constexpr int kSelThreads = PM_KS_THREADS;
constexpr int kSelIPT = PM_KS_IPT;
constexpr int kSelTile = kSelThreads * kSelIPT;   // positions per sub-tile
constexpr int kSelNSub = PM_KS_NSUB;
constexpr int kSelBlock = kSelTile * kSelNSub;    // positions per block
constexpr int kSelCache = 4 + 2 * kSelNSub;       // subtrees staged per block (global-level subtrees hold >= 1023)
constexpr int kCandThreads = 256;                  // k_ks_cand: LDS sort of <= 256 keys
#ifndef PM_KS_CANDCAP
#define PM_KS_CANDCAP 65536
#endif
constexpr int kCandCap = PM_KS_CANDCAP;            // larger candidate sets: grid-wide radix passes first

struct SelTab {
  uint32_t* ext[2];   // per subtree: orderable min x, y, z, max x, y, z (by level parity)
  int32_t* dim;       // split dimension (-1: empty subtree)
  uint32_t* kmin;     // orderable min along dim
  float* vlo;         // first pass: bin = (coord - vlo) * vsc, clamped to 0 .. 255
  float* vsc;
  int32_t* vbin;      // the bin holding the median
  uint32_t* rank;     // the median's rank (inside vbin after k_ks_find)
  int32_t* tb;        // key bits
  uint64_t* med;      // the median's key
  uint32_t* hist;     // 256 bins per subtree
  uint32_t* cnt;      // partition slots taken: left, right per subtree
  uint32_t* ccnt;     // candidates per subtree
  uint64_t* cand;     // candidate keys, subtree j's at [b_j, b_j + ccnt_j)
  uint64_t* cmin;     // range of the subtree's candidate keys
  uint64_t* cmax;
  int32_t* cshift;    // candidate radix select: key bits still to select,
  uint64_t* cprefix;  //   the selected bits above them,
  uint32_t* cmatch;   //   and how many candidates carry them
  uint64_t* cand2;    // large sets: the keys left after the grid passes, at [b_j, b_j + cnt2_j)
  uint32_t* cnt2;
  int idbits;
};

__device__ __forceinline__ float key_float(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ int bitlen32(uint32_t x) { return x ? 32 - __clz((int)x) : 0; }
// monotone non-decreasing in c (float subtraction and scaling round
// monotonically; NaN from inf * 0 lands in bin 0 with everything else)
__device__ __forceinline__ int vbin_of(float c, float lo, float sc) {
  const float t = (c - lo) * sc;
  return t >= 255.f ? 255 : (t > 0.f ? (int)t : 0);
}

// The bin of a 256-bin histogram (4 bins per lane of one wave) that holds
// rank `rank`: returns false if none does; r = the rank inside the bin, cb =
// its count.
__device__ __forceinline__ bool wave_pick_bin(uint4 c4, uint32_t rank, int& bin, uint32_t& r, uint32_t& cb) {
  const int lane = threadIdx.x & 63;
  const uint32_t sum = c4.x + c4.y + c4.z + c4.w;
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t up = (uint32_t)__shfl_up((int)inc, o);
    if (lane >= o) inc += up;
  }
  const uint32_t ex = inc - sum;
  const uint64_t hit = __ballot(ex <= rank && rank < inc);
  if (!hit || lane != __ffsll((unsigned long long)hit) - 1) return false;
  r = rank - ex;
  bin = 0;
  cb = c4.x;
  if (r >= c4.x) {
    r -= c4.x;
    bin = 1;
    cb = c4.y;
    if (r >= c4.y) {
      r -= c4.y;
      bin = 2;
      cb = c4.z;
      if (r >= c4.z) {
        r -= c4.z;
        bin = 3;
        cb = c4.w;
      }
    }
  }
  bin += 4 * lane;
  return true;
}

// root: elements -> SoA buffer 0, extents of the whole set (one atomic per wave)
constexpr int kInitBlocks = 2048;   // grid-stride: few blocks, few same-address atomics
__global__ __launch_bounds__(256) void k_ks_init(const float4* __restrict__ elems, int64_t n, KdSoa E,
                                                 uint32_t* __restrict__ ext) {
  uint32_t mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0u, 0u, 0u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)kInitBlocks * 256) {
    const float4 e = elems[i];
    E.comp(0, 0)[i] = e.x;
    E.comp(0, 1)[i] = e.y;
    E.comp(0, 2)[i] = e.z;
    E.comp(0, 3)[i] = e.w;
    const float c[3] = {e.x, e.y, e.z};
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const uint32_t kk = orderable_key(c[d]);
      mn[d] = min(mn[d], kk);
      mx[d] = max(mx[d], kk);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; d++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn[d] = min(mn[d], (uint32_t)__shfl_xor((int)mn[d], o));
      mx[d] = max(mx[d], (uint32_t)__shfl_xor((int)mx[d], o));
    }
  }
  __shared__ uint32_t wmn[4][3], wmx[4][3];   // blockDim = 256
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int d = 0; d < 3; d++) wmn[w][d] = mn[d], wmx[w][d] = mx[d];
  }
  __syncthreads();
  if (threadIdx.x < 3) {   // one atomic per block and component
    const int d = threadIdx.x;
    const uint32_t a = min(min(wmn[0][d], wmn[1][d]), min(wmn[2][d], wmn[3][d]));
    const uint32_t b = max(max(wmx[0][d], wmx[1][d]), max(wmx[2][d], wmx[3][d]));
    atomicMin(&ext[d], a);
    atomicMax(&ext[3 + d], b);
  }
}

// per subtree of level L: split dimension, selection state, children ranges,
// the children's extent accumulators and the counters reset
__global__ void k_ks_seg(int level, int64_t cap, SegTab T, SelTab S) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nseg = 1ll << level;
  if (j >= nseg) return;
  const int64_t t = nseg - 1 + j;
  const int b = T.b[t], s = T.s[t];
  const int64_t c1 = 2 * t + 1, c2 = 2 * t + 2;
  uint32_t* nx = S.ext[(level + 1) & 1];
#pragma unroll
  for (int c = 0; c < 2; c++) {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      nx[(2 * j + c) * 6 + d] = 0xFFFFFFFFu;
      nx[(2 * j + c) * 6 + 3 + d] = 0u;
    }
    S.cnt[2 * j + c] = 0;
  }
  S.ccnt[j] = 0;
  S.cmin[j] = ~0ull;
  S.cmax[j] = 0ull;
  S.cnt2[j] = 0;
  if (s <= 0) {
    S.dim[j] = -1;
    T.ls[t] = -1;
    if (c2 < cap) {
      T.b[c1] = b; T.s[c1] = 0;
      T.b[c2] = b; T.s[c2] = 0;
    }
    return;
  }
  const int ls = left_size(s);
  const uint32_t* ex = S.ext[level & 1] + j * 6;
  float ext[3];
#pragma unroll
  for (int d = 0; d < 3; d++) ext[d] = key_float(ex[3 + d]) - key_float(ex[d]);
  int dim = 0;
  if (ext[1] > ext[dim]) dim = 1;
  if (ext[2] > ext[dim]) dim = 2;
  const float lo = key_float(ex[dim]), range = ext[dim];
  S.dim[j] = dim;
  S.kmin[j] = ex[dim];
  S.vlo[j] = lo;
  S.vsc[j] = range > 0.f ? 256.f / range : 0.f;   // inf range: 0 (one bin)
  S.tb[j] = bitlen32(ex[3 + dim] - ex[dim]) + S.idbits;
  S.rank[j] = (uint32_t)ls;
  T.ls[t] = ls;
  T.dim[t] = dim;
  if (c2 < cap) {
    T.b[c1] = b; T.s[c1] = ls;
    T.b[c2] = b + ls + 1; T.s[c2] = s - ls - 1;
  }
}

// a subtree as the per-position kernels see it
struct SelRec {
  int b, s, dim, vbin;
  uint32_t kmin;
  float vlo, vsc;
  uint64_t med;
  int cb[2];   // children starts (k_ks_part)
};

__device__ __forceinline__ SelRec sel_load(const SegTab& T, const SelTab& S, int level, int j, bool med) {
  const int64_t t = (1ll << level) - 1 + j;
  SelRec r;
  r.b = T.b[t];
  r.s = T.s[t];
  r.dim = S.dim[j];
  r.kmin = S.kmin[j];
  r.vlo = S.vlo[j];
  r.vsc = S.vsc[j];
  r.vbin = S.vbin[j];
  r.med = med ? S.med[j] : 0ull;
  r.cb[0] = med ? T.b[2 * t + 1] : 0;
  r.cb[1] = med ? T.b[2 * t + 2] : 0;
  return r;
}

// slot (j - jl) of position p in a cached tile, -1: a placed median / past n
__device__ __forceinline__ int sel_slot(const SelRec* cache, int nslot, int64_t p) {
  int k = 0;
  for (int c = 1; c < nslot; c++)
    if ((int64_t)cache[c].b <= p) k = c;
  const SelRec& r = cache[k];
  return (r.s > 0 && p >= r.b && p < (int64_t)r.b + r.s) ? k : -1;
}

// the subtrees a kSelTile-position block can meet: jl .. jh (tile_seg);
// staged in LDS when there are few (always, in practice: global-level subtrees
// hold >= 1023 elements)
struct SelTile {
  int jl, jh;
  bool cached;
};

__device__ __forceinline__ SelTile sel_tile(const SegTab& T, const SelTab& S, int level, bool med,
                                            const int32_t* __restrict__ tile_seg, SelRec* cache) {
  SelTile st;
  st.jl = tile_seg[blockIdx.x];
  st.jh = tile_seg[blockIdx.x + 1];
  st.cached = st.jh - st.jl < kSelCache;
  if (st.cached)
    for (int j = st.jl + (int)threadIdx.x; j <= st.jh; j += blockDim.x)
      cache[j - st.jl] = sel_load(T, S, level, j, med);
  __syncthreads();
  return st;
}

// subtree of position p (-1: a placed median / outside every subtree)
__device__ __forceinline__ int sel_find(const SegTab& T, const SelTab& S, int level, bool med, const SelTile& st,
                                        const SelRec* cache, int64_t p, SelRec& r) {
  int j;
  if (st.cached) {
    int k = 0;
    for (int c = 1; c <= st.jh - st.jl; c++)
      if ((int64_t)cache[c].b <= p) k = c;
    r = cache[k];
    j = st.jl + k;
  } else {
    const int64_t base = (1ll << level) - 1;
    int lo = st.jl, hi = st.jh + 1;
    while (hi - lo > 1) {
      const int m = (lo + hi) >> 1;
      if ((int64_t)T.b[base + m] <= p) lo = m;
      else hi = m;
    }
    r = sel_load(T, S, level, lo, med);
    j = lo;
  }
  return (r.s > 0 && p >= r.b && p < (int64_t)r.b + r.s) ? j : -1;
}

// k_kd_tileseg for a runtime tile size
__global__ void k_kd_tileseg_n(const int32_t* __restrict__ tb, int level, int64_t ntiles, int tile,
                               int32_t* __restrict__ tile_seg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > ntiles) return;
  const int64_t base = (1ll << level) - 1, nseg = 1ll << level;
  const int64_t p = i < ntiles ? i * tile : INT64_MAX;
  int64_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const int64_t m = (lo + hi) >> 1;
    if ((int64_t)tb[base + m] <= p) lo = m;
    else hi = m;
  }
  tile_seg[i] = (int32_t)lo;
}

// (slot, bin) groups of a wave merged before the atomic: up to `rounds` leader
// rounds, then one atomic per remaining lane
__device__ __forceinline__ void merged_add(uint32_t* base, int key, int rounds) {
  const int lane = threadIdx.x & 63;
  uint64_t todo = __ballot(key >= 0);
  for (int r = 0; todo && r < rounds; r++) {
    const int l = __ffsll((unsigned long long)todo) - 1;
    const int kl = __shfl(key, l);
    const uint64_t same = __ballot(key == kl) & todo;
    if (lane == l) atomicAdd(&base[kl], (uint32_t)__popcll(same));
    if ((same >> lane) & 1) key = -1;
    todo &= ~same;
  }
  if (key >= 0) atomicAdd(&base[key], 1u);
}

// first selection pass: 256-bin histograms of the scaled coordinate, per
// block in LDS, flushed with one atomic per used bin. Every item's load is
// issued before any is used (the per-item atomics would otherwise serialise
// the loads behind them).
__global__ __launch_bounds__(kSelThreads) void k_ks_hist(KdSoa E, int64_t n, SegTab T, SelTab S, int level,
                                                         const int32_t* __restrict__ tile_seg) {
  __shared__ SelRec cache[kSelCache];
  __shared__ uint32_t lh[kSelCache * 256];
  const SelTile st = sel_tile(T, S, level, false, tile_seg, cache);
  const int k = level & 1;
  const int64_t t0 = (int64_t)blockIdx.x * kSelBlock;
  if (!st.cached) {   // never at global levels (subtrees of >= 1023 elements); kept general
    for (int it = 0; it < kSelIPT * kSelNSub; it++) {
      const int64_t p = t0 + it * kSelThreads + threadIdx.x;
      SelRec r;
      const int j = p < n ? sel_find(T, S, level, false, st, cache, p, r) : -1;
      if (j >= 0) atomicAdd(&S.hist[(int64_t)j * 256 + vbin_of(E.comp(k, r.dim)[p], r.vlo, r.vsc)], 1u);
    }
    return;
  }
  const int nslot = st.jh - st.jl + 1;
  for (int i = threadIdx.x; i < nslot * 256; i += kSelThreads) lh[i] = 0;
  __syncthreads();
  for (int sub = 0; sub < kSelNSub; sub++) {
    const int64_t ts = t0 + (int64_t)sub * kSelTile;
    int sl[kSelIPT];
    float cv[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      const int64_t p = ts + it * kSelThreads + threadIdx.x;
      sl[it] = p < n ? sel_slot(cache, nslot, p) : -1;
    }
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {   // every load issued before any is used
      const int64_t p = ts + it * kSelThreads + threadIdx.x;
      cv[it] = E.comp(k, cache[sl[it] < 0 ? 0 : sl[it]].dim)[sl[it] < 0 ? 0 : p];
    }
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      int key = -1;
      if (sl[it] >= 0) {
        const SelRec& r = cache[sl[it]];
        key = sl[it] * 256 + vbin_of(cv[it], r.vlo, r.vsc);
      }
      merged_add(lh, key, 2);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nslot * 256; i += kSelThreads) {
    const uint32_t c = lh[i];
    if (c) atomicAdd(&S.hist[(int64_t)st.jl * 256 + i], c);
  }
}

// one wave per subtree: the bin holding the median's rank (its rank inside
// the bin kept); the bins are cleared for the next use
__global__ __launch_bounds__(64) void k_ks_find(SelTab S) {
  const int j = blockIdx.x, lane = threadIdx.x;
  if (S.dim[j] < 0) return;
  uint32_t* h = S.hist + (int64_t)j * 256;
  const uint4 c4 = reinterpret_cast<const uint4*>(h)[lane];
  reinterpret_cast<uint4*>(h)[lane] = make_uint4(0u, 0u, 0u, 0u);
  uint32_t r, cb;
  int bin;
  if (!wave_pick_bin(c4, S.rank[j], bin, r, cb)) return;
  S.vbin[j] = bin;
  S.rank[j] = r;
}

// the median bin's elements -> the subtree's candidate range, as keys, with
// the range of those keys (per block in LDS, one atomic per block and subtree)
__global__ __launch_bounds__(kSelThreads) void k_ks_compact(KdSoa E, int64_t n, SegTab T, SelTab S, int level,
                                                            const int32_t* __restrict__ tile_seg) {
  __shared__ SelRec cache[kSelCache];
  __shared__ uint32_t lcc[kSelCache], lbase[kSelCache];
  __shared__ unsigned long long lkmin[kSelCache], lkmax[kSelCache];
  const SelTile st = sel_tile(T, S, level, false, tile_seg, cache);
  const int k = level & 1;
  const int lane = threadIdx.x & 63;
  const int64_t t0 = (int64_t)blockIdx.x * kSelBlock;
  if (!st.cached) {   // never at global levels; kept general
    for (int it = 0; it < kSelIPT * kSelNSub; it++) {
      const int64_t p = t0 + it * kSelThreads + threadIdx.x;
      SelRec r;
      const int j = p < n ? sel_find(T, S, level, false, st, cache, p, r) : -1;
      if (j < 0) continue;
      const float c = E.comp(k, r.dim)[p];
      if (vbin_of(c, r.vlo, r.vsc) != r.vbin) continue;
      const uint64_t key = (uint64_t)(orderable_key(c) - r.kmin) << S.idbits | (uint32_t)__float_as_int(E.comp(k, 3)[p]);
      S.cand[(int64_t)r.b + atomicAdd(&S.ccnt[j], 1u)] = key;
      atomicMin((unsigned long long*)&S.cmin[j], (unsigned long long)key);
      atomicMax((unsigned long long*)&S.cmax[j], (unsigned long long)key);
    }
    return;
  }
  const int nslot = st.jh - st.jl + 1;
  if (threadIdx.x < nslot) {
    lkmin[threadIdx.x] = ~0ull;
    lkmax[threadIdx.x] = 0ull;
  }
  uint64_t kmn0 = ~0ull, kmx0 = 0ull, kmn1 = ~0ull, kmx1 = 0ull;   // key range of slots 0 / 1 (this lane)
  for (int sub = 0; sub < kSelNSub; sub++) {
    const int64_t ts = t0 + (int64_t)sub * kSelTile;
    if (threadIdx.x < nslot) lcc[threadIdx.x] = 0;
    int sl[kSelIPT];
    float cv[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      const int64_t p = ts + it * kSelThreads + threadIdx.x;
      sl[it] = p < n ? sel_slot(cache, nslot, p) : -1;
    }
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      const int64_t p = ts + it * kSelThreads + threadIdx.x;
      cv[it] = E.comp(k, cache[sl[it] < 0 ? 0 : sl[it]].dim)[sl[it] < 0 ? 0 : p];
    }
#pragma unroll
    for (int it = 0; it < kSelIPT; it++)
      if (sl[it] >= 0 && vbin_of(cv[it], cache[sl[it]].vlo, cache[sl[it]].vsc) != cache[sl[it]].vbin) sl[it] = -1;
    uint32_t idv[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      const int64_t p = ts + it * kSelThreads + threadIdx.x;
      idv[it] = sl[it] >= 0 ? (uint32_t)__float_as_int(E.comp(k, 3)[p]) : 0u;
    }
    __syncthreads();   // lcc reset (and the previous sub-tile's lbase reads) done
    uint64_t key[kSelIPT];
    uint32_t rk[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      const int g = sl[it];
      key[it] = g >= 0 ? (uint64_t)(orderable_key(cv[it]) - cache[g].kmin) << S.idbits | idv[it] : 0ull;
      rk[it] = 0;
      if (g == 0) kmn0 = min(kmn0, key[it]), kmx0 = max(kmx0, key[it]);
      else if (g == 1) kmn1 = min(kmn1, key[it]), kmx1 = max(kmx1, key[it]);
      else if (g > 1) {
        atomicMin(&lkmin[g], (unsigned long long)key[it]);
        atomicMax(&lkmax[g], (unsigned long long)key[it]);
      }
      uint64_t todo = __ballot(g >= 0);
      while (todo) {
        const int l = __ffsll((unsigned long long)todo) - 1;
        const int gl = __shfl(g, l);
        const uint64_t same = __ballot(g == gl) & todo;
        uint32_t base = 0;
        if (lane == l) base = atomicAdd(&lcc[gl], (uint32_t)__popcll(same));
        base = (uint32_t)__shfl((int)base, l);
        if ((same >> lane) & 1) rk[it] = base + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
        todo &= ~same;
      }
    }
    __syncthreads();
    if (threadIdx.x < nslot) {
      const uint32_t c = lcc[threadIdx.x];
      lbase[threadIdx.x] = c ? atomicAdd(&S.ccnt[st.jl + threadIdx.x], c) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kSelIPT; it++)
      if (sl[it] >= 0) S.cand[(int64_t)cache[sl[it]].b + lbase[sl[it]] + rk[it]] = key[it];
  }
  {
    const uint64_t a0 = wave_minmax64<false>(kmn0), b0 = wave_minmax64<true>(kmx0);
    const uint64_t a1 = wave_minmax64<false>(kmn1), b1 = wave_minmax64<true>(kmx1);
    if (lane == 0) {
      if (a0 <= b0) atomicMin(&lkmin[0], (unsigned long long)a0), atomicMax(&lkmax[0], (unsigned long long)b0);
      if (a1 <= b1) atomicMin(&lkmin[1], (unsigned long long)a1), atomicMax(&lkmax[1], (unsigned long long)b1);
    }
  }
  __syncthreads();
  if (threadIdx.x < nslot && lkmin[threadIdx.x] <= lkmax[threadIdx.x]) {
    const int j = st.jl + threadIdx.x;
    atomicMin((unsigned long long*)&S.cmin[j], lkmin[threadIdx.x]);
    atomicMax((unsigned long long*)&S.cmax[j], lkmax[threadIdx.x]);
  }
}

// candidate selection state: the digits above the highest bit in which the
// subtree's candidate keys differ are common to all of them
__global__ void k_ks_cinit(int64_t nseg, SelTab S) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nseg || S.dim[j] < 0) return;
  const uint64_t a = S.cmin[j], b = S.cmax[j];
  const int sh = (a ^ b) ? 64 - __clzll((long long)(a ^ b)) : 0;
  S.cshift[j] = sh;
  S.cprefix[j] = sh >= 64 ? 0ull : a >> sh;
  S.cmatch[j] = S.ccnt[j];
}

// a radix pass over a large candidate set, spread over gridDim.x blocks per
// subtree (subtrees with <= kCandCap matching keys are left to k_ks_cand)
__global__ __launch_bounds__(kSelThreads) void k_ks_chist(int level, SegTab T, SelTab S) {
  __shared__ uint32_t h[256];
  const int j = blockIdx.y;
  if (S.dim[j] < 0) return;
  const int shift = S.cshift[j];
  if (S.cmatch[j] <= (uint32_t)kCandCap || shift <= 0) return;
  const uint64_t prefix = S.cprefix[j];
  const int w = min(8, shift);
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t total = S.ccnt[j];
  const uint32_t per = (total + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = blockIdx.x * per, hi = min(total, lo + per);
  const uint64_t* cand = S.cand + T.b[(1ll << level) - 1 + j];
  for (uint32_t i0 = lo; i0 < hi; i0 += kSelThreads) {
    const uint32_t i = i0 + threadIdx.x;
    int bin = -1;
    if (i < hi) {
      const uint64_t key = cand[i];
      if ((key >> shift) == prefix) bin = (int)((key >> (shift - w)) & ((1u << w) - 1u));
    }
    merged_add(h, bin, 2);
  }
  __syncthreads();
  const uint32_t c = h[threadIdx.x];
  if (c) atomicAdd(&S.hist[(int64_t)j * 256 + threadIdx.x], c);
}

__global__ __launch_bounds__(64) void k_ks_cfind(SelTab S) {
  const int j = blockIdx.x;
  if (S.dim[j] < 0) return;
  const int shift = S.cshift[j];
  if (S.cmatch[j] <= (uint32_t)kCandCap || shift <= 0) return;
  uint32_t* h = S.hist + (int64_t)j * 256;
  const uint4 c4 = reinterpret_cast<const uint4*>(h)[threadIdx.x];
  reinterpret_cast<uint4*>(h)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
  uint32_t r, cb;
  int bin;
  if (!wave_pick_bin(c4, S.rank[j], bin, r, cb)) return;
  const int w = min(8, shift);
  S.cprefix[j] = S.cprefix[j] << w | (uint64_t)bin;
  S.cshift[j] = shift - w;
  S.rank[j] = r;
  S.cmatch[j] = cb;
}

// large sets after the grid passes: the keys still matching -> cand2 (one
// atomic per wave)
__global__ __launch_bounds__(kSelThreads) void k_ks_cgather(int level, SegTab T, SelTab S) {
  const int j = blockIdx.y, lane = threadIdx.x & 63;
  if (S.dim[j] < 0 || S.ccnt[j] <= (uint32_t)kCandCap) return;
  const int shift = S.cshift[j];
  const uint64_t prefix = S.cprefix[j];
  const uint32_t total = S.ccnt[j];
  const uint32_t per = (total + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = blockIdx.x * per, hi = min(total, lo + per);
  const int64_t b = T.b[(1ll << level) - 1 + j];
  const uint64_t* cand = S.cand + b;
  for (uint32_t i0 = lo; i0 < hi; i0 += kSelThreads) {
    const uint32_t i = i0 + threadIdx.x;
    uint64_t key = 0;
    bool take = false;
    if (i < hi) {
      key = cand[i];
      take = (key >> shift) == prefix;
    }
    const uint64_t m = __ballot(take);
    if (!m) continue;
    const int l = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == l) base = atomicAdd(&S.cnt2[j], (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, l);
    if (take) S.cand2[b + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = key;
  }
}

// The candidate of rank `rank` among the `total` keys at cand (global) whose
// bits above `shift` equal `prefix` (c of them): while more than kCandThreads
// match, an 8-bit radix pass over them (LDS histogram); then the matching keys
// are sorted in LDS. Writes the median's key and its node (position from
// elems[index]). Called by a whole kCandThreads-thread workgroup.
struct CandShared {
  uint32_t h[256];
  uint64_t lk[kCandThreads], kx[kCandThreads];
  int16_t vx[kCandThreads];
  uint64_t prefix;
  uint32_t rank, cnt;
  int shift;
};
__device__ __forceinline__ void cand_pick(CandShared& sh, const uint64_t* cand, uint32_t total, uint32_t rank,
                                          uint32_t c, uint64_t prefix, int shift, int j, int64_t t, SegTab T,
                                          SelTab S, const float4* __restrict__ elems, float4* __restrict__ nodes) {
  const int tid = threadIdx.x;
  while (c > kCandThreads && shift > 0) {   // keys are unique: c == 1 once shift == 0
    const int w = min(8, shift);
    sh.h[tid] = 0;
    if (tid == 0) {   // a rank outside the histogram ends the loop (never, with consistent counts)
      sh.prefix = prefix;
      sh.rank = rank;
      sh.cnt = 0;
      sh.shift = 0;
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < total; i0 += kCandThreads) {
      const uint32_t i = i0 + tid;
      int bin = -1;
      if (i < total) {
        const uint64_t key = cand[i];
        if ((key >> shift) == prefix) bin = (int)((key >> (shift - w)) & ((1u << w) - 1u));
      }
      merged_add(sh.h, bin, 2);
    }
    __syncthreads();
    if (tid < 64) {
      const uint4 c4 = reinterpret_cast<const uint4*>(sh.h)[tid];
      uint32_t r, cb;
      int bin;
      if (wave_pick_bin(c4, rank, bin, r, cb)) {
        sh.prefix = prefix << w | (uint64_t)bin;
        sh.rank = r;
        sh.cnt = cb;
        sh.shift = shift - w;
      }
    }
    __syncthreads();
    prefix = sh.prefix;
    rank = sh.rank;
    c = sh.cnt;
    shift = sh.shift;
    __syncthreads();
  }
  if (tid == 0) sh.cnt = 0;
  __syncthreads();
  for (uint32_t i = tid; i < total; i += kCandThreads) {
    const uint64_t key = cand[i];
    if ((key >> shift) == prefix) {
      const uint32_t o = atomicAdd(&sh.cnt, 1u);
      if (o < kCandThreads) sh.lk[o] = key;
    }
  }
  __syncthreads();
  c = min(sh.cnt, (uint32_t)kCandThreads);
  int n2 = 64;
  while (n2 < (int)c) n2 <<= 1;
  uint64_t key = tid < (int)c ? sh.lk[tid] : ~0ull;
  int v = tid;
  block_bitonic(key, v, n2, sh.kx, sh.vx);
  if (tid == (int)rank) {
    S.med[j] = key;
    const int id = (int)(key & ((1ull << S.idbits) - 1ull));
    const int dim = S.dim[j];
    const float4 e = elems[id];
    T.id[t] = id;
    T.coord[t] = coord_of(e, dim);
    nodes[t] = make_float4(e.x, e.y, e.z, __int_as_float((id << 2) | dim));
  }
}

// one workgroup per subtree: the candidate of the median's rank (after the
// grid-wide passes for large sets)
__global__ __launch_bounds__(kCandThreads) void k_ks_cand(int level, SegTab T, SelTab S,
                                                          const float4* __restrict__ elems,
                                                          float4* __restrict__ nodes, bool gathered) {
  __shared__ CandShared sh;
  const int j = blockIdx.x;
  if (S.dim[j] < 0) return;
  const int64_t t = (1ll << level) - 1 + j;
  const bool big = gathered && S.ccnt[j] > (uint32_t)kCandCap;   // k_ks_cgather ran for it
  const uint64_t* cand = (big ? S.cand2 : S.cand) + T.b[t];
  const uint32_t total = big ? S.cnt2[j] : S.ccnt[j];
  cand_pick(sh, cand, total, S.rank[j], S.cmatch[j], S.cprefix[j], S.cshift[j], j, t, T, S, elems, nodes);
}

// Deep levels (subtrees of <= kSegSelMax elements, enough of them to fill the
// GPU): one workgroup per subtree does the whole selection over its own
// contiguous range -- histogram, bin pick, compaction of the bin's keys into
// its candidate range (with their key range), cand_pick -- in one launch
// instead of five, reading the split coordinate twice (the second time from L2).
constexpr int kSegSelMax = 1 << 17;
#ifndef PM_KS_SEGSEL_MIN
// subtrees per level for k_ks_segsel (fewer workgroups underfill the GPU).
// Round 6, config 3 (profiles/r06/r06j_*): 512 sent level 9 (512 subtrees of
// ~89 k elements, 2 workgroups per CU) here at 2.2 ms; 1024 gives it to the
// grid-wide passes: kd phase -0.3 ms; 2048: no further change
#define PM_KS_SEGSEL_MIN 1024
#endif
constexpr int64_t kSegSelMinSegs = PM_KS_SEGSEL_MIN;
#ifndef PM_KS_SEGSEL_U
#define PM_KS_SEGSEL_U 8
#endif
__global__ __launch_bounds__(kCandThreads) void k_ks_segsel(KdSoa E, int level, SegTab T, SelTab S,
                                                            const float4* __restrict__ elems,
                                                            float4* __restrict__ nodes) {
  __shared__ CandShared sh;
  __shared__ int s_bin;
  __shared__ uint32_t s_rank, s_cb, s_n;
  __shared__ unsigned long long s_kmin, s_kmax;
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  if (S.dim[j] < 0) return;
  const int64_t t = (1ll << level) - 1 + j;
  const int b = T.b[t], s = T.s[t], dim = S.dim[j];
  const uint32_t kmin = S.kmin[j];
  const float lo = S.vlo[j], sc = S.vsc[j];
  const int k = level & 1;
  const float* cd = E.comp(k, dim) + b;
  const float* ci = E.comp(k, 3) + b;
  sh.h[tid] = 0;
  if (tid == 0) {
    s_bin = -1;
    s_n = 0;
    s_kmin = ~0ull;
    s_kmax = 0ull;
  }
  __syncthreads();
  constexpr int U = PM_KS_SEGSEL_U;   // loads in flight per thread
  for (int i0 = 0; i0 < s; i0 += U * kCandThreads) {
    float cv[U];
#pragma unroll
    for (int q = 0; q < U; q++) {
      const int i = i0 + q * kCandThreads + tid;
      cv[q] = i < s ? cd[i] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; q++) {
      const int i = i0 + q * kCandThreads + tid;
      merged_add(sh.h, i < s ? vbin_of(cv[q], lo, sc) : -1, 2);
    }
  }
  __syncthreads();
  if (tid < 64) {
    const uint4 c4 = reinterpret_cast<const uint4*>(sh.h)[tid];
    uint32_t r, cb;
    int bin;
    if (wave_pick_bin(c4, S.rank[j], bin, r, cb)) {
      s_bin = bin;
      s_rank = r;
      s_cb = cb;
    }
  }
  __syncthreads();
  const int bin = s_bin;
  if (bin < 0) return;   // inconsistent counts (never): leave the node unwritten
  uint64_t* cand = S.cand + b;
  uint64_t kmn = ~0ull, kmx = 0ull;
  for (int i0 = 0; i0 < s; i0 += U * kCandThreads) {
    float cv[U];
#pragma unroll
    for (int q = 0; q < U; q++) {
      const int i = i0 + q * kCandThreads + tid;
      cv[q] = i < s ? cd[i] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; q++) {
      const int i = i0 + q * kCandThreads + tid;
      const bool take = i < s && vbin_of(cv[q], lo, sc) == bin;
      const uint64_t m = __ballot(take);
      if (!m) continue;
      const int l = __ffsll((unsigned long long)m) - 1;
      uint32_t base = 0;
      if (lane == l) base = atomicAdd(&s_n, (uint32_t)__popcll(m));
      base = (uint32_t)__shfl((int)base, l);
      if (take) {
        const uint64_t key = (uint64_t)(orderable_key(cv[q]) - kmin) << S.idbits | (uint32_t)__float_as_int(ci[i]);
        cand[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = key;
        kmn = min(kmn, key);
        kmx = max(kmx, key);
      }
    }
  }
  kmn = wave_minmax64<false>(kmn);
  kmx = wave_minmax64<true>(kmx);
  if (lane == 0 && kmn <= kmx) {
    atomicMin(&s_kmin, (unsigned long long)kmn);
    atomicMax(&s_kmax, (unsigned long long)kmx);
  }
  __syncthreads();   // the candidates (global, this workgroup's) and their range are complete
  const uint64_t a = s_kmin, z = s_kmax;
  const int shift = (a ^ z) ? 64 - __clzll((long long)(a ^ z)) : 0;
  cand_pick(sh, cand, s_cb, s_rank, s_cb, shift >= 64 ? 0ull : a >> shift, shift, j, t, T, S, elems, nodes);
}

// every element to its child range; the children's extents reduced per lane
// (the block's first two subtrees), per block in LDS, then one atomic per
// block, child and component. All loads are issued first.
#ifndef PM_KS_PART_WAVES
#define PM_KS_PART_WAVES 0   // occupancy target of k_ks_part (0: compiler's choice)
#endif
__global__ __launch_bounds__(kSelThreads) PM_WAVES_ATTR(PM_KS_PART_WAVES) void k_ks_part(KdSoa E, int64_t n, SegTab T,
                                                                                      SelTab S, int level,
                                                         const int32_t* __restrict__ tile_seg) {
  __shared__ SelRec cache[kSelCache];
  __shared__ uint32_t lcnt[kSelCache * 2], lbase[kSelCache * 2];
  __shared__ uint32_t lext[kSelCache * 2][6];
  const SelTile st = sel_tile(T, S, level, true, tile_seg, cache);
  const int k = level & 1, ko = k ^ 1;
  const int lane = threadIdx.x & 63;
  const int64_t t0 = (int64_t)blockIdx.x * kSelBlock;
  if (!st.cached) {   // never at global levels; kept general
    for (int it = 0; it < kSelIPT * kSelNSub; it++) {
      const int64_t p = t0 + it * kSelThreads + threadIdx.x;
      SelRec r;
      const int j = p < n ? sel_find(T, S, level, true, st, cache, p, r) : -1;
      if (j < 0) continue;
      const float4 e = make_float4(E.comp(k, 0)[p], E.comp(k, 1)[p], E.comp(k, 2)[p], E.comp(k, 3)[p]);
      const uint64_t key = (uint64_t)(orderable_key(coord_of(e, r.dim)) - r.kmin) << S.idbits |
                           (uint32_t)__float_as_int(e.w);
      if (key == r.med) continue;
      const int side = key < r.med ? 0 : 1;
      const int64_t dst = (int64_t)r.cb[side] + atomicAdd(&S.cnt[2 * j + side], 1u);
      uint32_t* nx = S.ext[(level + 1) & 1] + (2 * (int64_t)j + side) * 6;
      const uint32_t ok[3] = {orderable_key(e.x), orderable_key(e.y), orderable_key(e.z)};
      for (int d = 0; d < 3; d++) {
        atomicMin(&nx[d], ok[d]);
        atomicMax(&nx[3 + d], ok[d]);
      }
      E.comp(ko, 0)[dst] = e.x;
      E.comp(ko, 1)[dst] = e.y;
      E.comp(ko, 2)[dst] = e.z;
      E.comp(ko, 3)[dst] = e.w;
    }
    return;
  }
  const int nslot = st.jh - st.jl + 1;
  for (int i = threadIdx.x; i < nslot * 2; i += kSelThreads) {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      lext[i][d] = 0xFFFFFFFFu;
      lext[i][3 + d] = 0u;
    }
  }
  uint32_t amn[4][3], amx[4][3];   // groups 0..3 = slot 0 / 1 x side
#pragma unroll
  for (int g = 0; g < 4; g++)
#pragma unroll
    for (int d = 0; d < 3; d++) amn[g][d] = 0xFFFFFFFFu, amx[g][d] = 0u;
  for (int sub = 0; sub < kSelNSub; sub++) {
    const int64_t ts = t0 + (int64_t)sub * kSelTile;
    for (int i = threadIdx.x; i < nslot * 2; i += kSelThreads) lcnt[i] = 0;
    int sl[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      const int64_t p = ts + it * kSelThreads + threadIdx.x;
      sl[it] = p < n ? sel_slot(cache, nslot, p) : -1;
    }
    float4 e[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {   // every load issued before any is used
      const int64_t p = sl[it] < 0 ? 0 : ts + it * kSelThreads + threadIdx.x;
      e[it] = make_float4(E.comp(k, 0)[p], E.comp(k, 1)[p], E.comp(k, 2)[p], E.comp(k, 3)[p]);
    }
    __syncthreads();   // lcnt reset (and the previous sub-tile's lbase reads) done
    int grp[kSelIPT];   // slot * 2 + side, -1: not moved
    uint32_t rk[kSelIPT];
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      int g = -1;
      if (sl[it] >= 0) {
        const SelRec& r = cache[sl[it]];
        const uint64_t key = (uint64_t)(orderable_key(coord_of(e[it], r.dim)) - r.kmin) << S.idbits |
                             (uint32_t)__float_as_int(e[it].w);
        if (key != r.med) g = sl[it] * 2 + (key < r.med ? 0 : 1);   // the median is already a node
      }
      grp[it] = g;
      rk[it] = 0;
      uint64_t todo = __ballot(g >= 0);
      while (todo) {
        const int l = __ffsll((unsigned long long)todo) - 1;
        const int gl = __shfl(g, l);
        const uint64_t same = __ballot(g == gl) & todo;
        uint32_t base = 0;
        if (lane == l) base = atomicAdd(&lcnt[gl], (uint32_t)__popcll(same));
        base = (uint32_t)__shfl((int)base, l);
        if ((same >> lane) & 1) rk[it] = base + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
        todo &= ~same;
      }
      if (g >= 0) {
        const uint32_t ok[3] = {orderable_key(e[it].x), orderable_key(e[it].y), orderable_key(e[it].z)};
        if (g < 4) {
#pragma unroll
          for (int q = 0; q < 4; q++)
#pragma unroll
            for (int d = 0; d < 3; d++) {
              amn[q][d] = g == q ? min(amn[q][d], ok[d]) : amn[q][d];
              amx[q][d] = g == q ? max(amx[q][d], ok[d]) : amx[q][d];
            }
        } else {
#pragma unroll
          for (int d = 0; d < 3; d++) {
            atomicMin(&lext[g][d], ok[d]);
            atomicMax(&lext[g][3 + d], ok[d]);
          }
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nslot * 2; i += kSelThreads) {
      const uint32_t cn = lcnt[i];
      lbase[i] = (uint32_t)cache[i >> 1].cb[i & 1] + (cn ? atomicAdd(&S.cnt[2 * (st.jl + (i >> 1)) + (i & 1)], cn) : 0u);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kSelIPT; it++) {
      if (grp[it] < 0) continue;
      const int64_t dst = (int64_t)lbase[grp[it]] + rk[it];
      E.comp(ko, 0)[dst] = e[it].x;
      E.comp(ko, 1)[dst] = e[it].y;
      E.comp(ko, 2)[dst] = e[it].z;
      E.comp(ko, 3)[dst] = e[it].w;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const uint32_t mn = wave_minmax<false>(amn[q][d]), mx = wave_minmax<true>(amx[q][d]);
      if (lane == 0 && q < nslot * 2 && mn <= mx) {
        atomicMin(&lext[q][d], mn);
        atomicMax(&lext[q][3 + d], mx);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nslot * 2; i += kSelThreads) {
    if (lext[i][0] > lext[i][3]) continue;   // nothing went to this child from here
    uint32_t* nx = S.ext[(level + 1) & 1] + (2 * (int64_t)(st.jl + (i >> 1)) + (i & 1)) * 6;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      atomicMin(&nx[d], lext[i][d]);
      atomicMax(&nx[3 + d], lext[i][3 + d]);
    }
  }
}

static hipError_t kd_build_sel(const float4* elems, int64_t n, float4* nodes, hipStream_t s) {
  int H = 0;
  while ((1ll << H) <= n) H++;          // levels = floor(log2 n) + 1
  const int L0 = std::max(0, H - kLocalLog);   // subtrees at L0 hold <= kLocal - 1 elements
  const int64_t cap = 1ll << (L0 + 1);  // subtree records down to level L0
  int idbits = 1;
  while ((1ll << idbits) < n) idbits++;
  const int64_t nsc = 1ll << L0;        // subtrees at L0 (children of the last global level)
  const bool global = L0 > 0;
  DevBuf<float> soa((size_t)8 * n);
  DevBuf<int32_t> tb(cap), ts(cap), tls(cap), tdim(cap), tid(cap), tsel(cap);
  DevBuf<float> tco(cap), vlo(nsc), vsc(nsc);
  DevBuf<uint32_t> ext((size_t)12 * nsc), kmin(nsc), rank(nsc), hist((size_t)256 * nsc), cnt(2 * nsc), ccnt(nsc);
  DevBuf<int32_t> sdim(nsc), vbin(nsc), stb(nsc);
  DevBuf<uint64_t> med(nsc), cand(global ? n : 0), cmin(nsc), cmax(nsc), cprefix(nsc);
  DevBuf<int32_t> cshift(nsc);
  DevBuf<uint32_t> cmatch(nsc), cnt2(nsc);
  const bool bigsets = (1ll << H) > kCandCap;   // some subtree may exceed kCandCap candidates
  DevBuf<uint64_t> cand2(global && bigsets ? n : 0);
  const int64_t ntiles = (n + kSelBlock - 1) / kSelBlock;
  DevBuf<int32_t> tile_seg(ntiles + 1);
  if (!soa.p || !tb.p || !ts.p || !tls.p || !tdim.p || !tid.p || !tsel.p || !tco.p || !vlo.p || !vsc.p || !ext.p ||
      !kmin.p || !rank.p || !hist.p || !cnt.p || !ccnt.p || !sdim.p || !vbin.p || !stb.p || !med.p ||
      !tile_seg.p || !cmin.p || !cmax.p || !cprefix.p || !cshift.p || !cmatch.p || !cnt2.p ||
      (global && !cand.p) || (global && bigsets && !cand2.p))
    return hipErrorOutOfMemory;
  const KdSoa E{soa.p, n};
  SegTab T{tb.p, ts.p, tls.p, tdim.p, tco.p, tid.p, tsel.p};
  SelTab S{{ext.p, ext.p + 6 * nsc}, sdim.p, kmin.p, vlo.p, vsc.p, vbin.p, rank.p, stb.p, med.p, hist.p, cnt.p,
           ccnt.p, cand.p, cmin.p, cmax.p, cshift.p, cprefix.p, cmatch.p, cand2.p, cnt2.p, idbits};
  const int32_t root[2] = {0, (int32_t)n};
  PM_HIP_TRY(hipMemcpyAsync(tb.p, &root[0], 4, hipMemcpyHostToDevice, s));
  PM_HIP_TRY(hipMemcpyAsync(ts.p, &root[1], 4, hipMemcpyHostToDevice, s));
  const uint32_t ext0[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
  PM_HIP_TRY(hipMemcpyAsync(ext.p, ext0, sizeof(ext0), hipMemcpyHostToDevice, s));
  if (global) PM_HIP_TRY(hipMemsetAsync(hist.p, 0, sizeof(uint32_t) * 256 * (size_t)(nsc / 2), s));
  k_ks_init<<<(int)std::min<int64_t>(kInitBlocks, grid_for(n, 256)), 256, 0, s>>>(elems, n, E, ext.p);
  PM_HIP_TRY(hipGetLastError());
  for (int L = 0; L < L0; L++) {
    const int64_t nseg = 1ll << L;
    k_ks_seg<<<grid_for(nseg, 256), 256, 0, s>>>(L, cap, T, S);
    PM_HIP_TRY(hipGetLastError());
    k_kd_tileseg_n<<<grid_for(ntiles + 1, 256), 256, 0, s>>>(tb.p, L, ntiles, kSelBlock, tile_seg.p);
    PM_HIP_TRY(hipGetLastError());
    if ((1ll << (H - L)) <= kSegSelMax && nseg >= kSegSelMinSegs) {   // deep level: one workgroup per subtree
      k_ks_segsel<<<(int)nseg, kCandThreads, 0, s>>>(E, L, T, S, elems, nodes);
      PM_HIP_TRY(hipGetLastError());
      k_ks_part<<<(int)ntiles, kSelThreads, 0, s>>>(E, n, T, S, L, tile_seg.p);
      PM_HIP_TRY(hipGetLastError());
      continue;
    }
    k_ks_hist<<<(int)ntiles, kSelThreads, 0, s>>>(E, n, T, S, L, tile_seg.p);
    PM_HIP_TRY(hipGetLastError());
    k_ks_find<<<(int)nseg, 64, 0, s>>>(S);
    PM_HIP_TRY(hipGetLastError());
    k_ks_compact<<<(int)ntiles, kSelThreads, 0, s>>>(E, n, T, S, L, tile_seg.p);
    PM_HIP_TRY(hipGetLastError());
    k_ks_cinit<<<grid_for(nseg, 256), 256, 0, s>>>(nseg, S);
    PM_HIP_TRY(hipGetLastError());
    const bool big = (1ll << (H - L)) > kCandCap;   // a subtree may hold more than kCandCap candidates
    if (big) {
      const dim3 g(std::max(1, 1024 >> L), (unsigned)nseg);
      for (int pass = 0; pass < 8; pass++) {   // <= 61 key bits: every set reaches one key
        k_ks_chist<<<g, kSelThreads, 0, s>>>(L, T, S);
        PM_HIP_TRY(hipGetLastError());
        k_ks_cfind<<<(int)nseg, 64, 0, s>>>(S);
        PM_HIP_TRY(hipGetLastError());
      }
      k_ks_cgather<<<g, kSelThreads, 0, s>>>(L, T, S);
      PM_HIP_TRY(hipGetLastError());
    }
    k_ks_cand<<<(int)nseg, kCandThreads, 0, s>>>(L, T, S, elems, nodes, big);
    PM_HIP_TRY(hipGetLastError());
    k_ks_part<<<(int)ntiles, kSelThreads, 0, s>>>(E, n, T, S, L, tile_seg.p);
    PM_HIP_TRY(hipGetLastError());
  }
  if (PM_KD_LOCAL_SEL) k_kd_local_sel<<<(int)nsc, kLocal, 0, s>>>(E, L0, T, nodes);
  else k_kd_local<true><<<(int)nsc, kLocal, 0, s>>>(KdLists{}, E, L0, T, nodes);
  return hipGetLastError();
}

#ifndef PM_KD_SEL
#define PM_KD_SEL 1   // the selection build (production); 0: the presorted build only
#endif
// Below this size the presorted build is faster (the selection build's ~10
// launches per level dominate). Round 3 (tools/kd_probe.py): 45.4 M elements
// 21.4 vs 24.5 ms, 10 M 6.0 vs 5.7 ms, 1 M 2.0 vs 1.0 ms: 2^24. Round 5, the
// current kernels (tools/kd_size_probe.py, uniform random points, selection vs
// presorted): 2.2 M 1.99 vs 1.55 ms, 3 M 2.10 vs 1.85, 4 M 2.25 vs 2.25, 6 M
// 3.17 vs 3.46, 8 M 3.60 vs 4.21, 12 M 5.84 vs 6.33, 16.8 M 6.81 vs 8.60: 2^22
// (the 8-rank subtrees of 2^24 - 1 elements now take the selection build).
// Same tree either way.
#ifndef PM_KD_SEL_MIN
#define PM_KD_SEL_MIN (1 << 22)
#endif

static hipError_t kd_build_lists(const float4* elems, int64_t n, float4* nodes, hipStream_t s);

hipError_t kd_build(const float4* elems, int64_t n, float4* nodes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n >= kMaxMapPhotons) return hipErrorInvalidValue;
  // the check variant keeps the presorted build (the identical-tree tests
  // compare the two libraries)
  if (PM_KD_SEL && !PM_CHECK_VARIANT && n >= PM_KD_SEL_MIN) return kd_build_sel(elems, n, nodes, s);
  return kd_build_lists(elems, n, nodes, s);
}

// The presorted build (rounds 1-2; the check variant's).
static hipError_t kd_build_lists(const float4* elems, int64_t n, float4* nodes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n >= kMaxMapPhotons) return hipErrorInvalidValue;
  int H = 0;
  while ((1ll << H) <= n) H++;          // levels = floor(log2 n) + 1
  const int64_t cap = 1ll << (H + 1);
  DevBuf<float> lists((size_t)24 * n);
  if (!lists.p) return hipErrorOutOfMemory;
  const KdLists Lst{lists.p, n};
  {
    // presort: list d = the elements stably sorted on (orderable coordinate d,
    // index); keys of all three coordinates in one pass, the index implicit in
    // the first radix pass and the gather of the elements fused into the last
    DevBuf<uint32_t> keys((size_t)3 * n);
    if (!keys.p) return hipErrorOutOfMemory;
    k_kd_init_keys<<<grid_for(n, 256), 256, 0, s>>>(elems, n, keys.p, keys.p + n, keys.p + 2 * n);
    PM_HIP_TRY(hipGetLastError());
    for (int d = 0; d < 3; d++) {
      const SoaOut out{{Lst.comp(d, 0, 0), Lst.comp(d, 0, 1), Lst.comp(d, 0, 2), Lst.comp(d, 0, 3)}};
      PM_HIP_TRY(radix_sort_gather_soa(keys.p + (int64_t)d * n, n, elems, out, s));
    }
  }
  DevBuf<int32_t> tb(cap), ts(cap), tls(cap), tdim(cap), tid(cap), tsel(cap);
  DevBuf<float> tco(cap);
  const int64_t ntiles = (n + kPartTile - 1) / kPartTile;
  const int nchunks = (int)((ntiles + kChunk - 1) / kChunk);
  DevBuf<SegVal> tagg(ntiles), tcarry(ntiles), ccarry(nchunks);
  DevBuf<int32_t> tile_seg(ntiles + 1);
  if (!tb.p || !ts.p || !tls.p || !tdim.p || !tid.p || !tsel.p || !tco.p || !tagg.p || !tcarry.p || !ccarry.p ||
      !tile_seg.p)
    return hipErrorOutOfMemory;
  SegTab T{tb.p, ts.p, tls.p, tdim.p, tco.p, tid.p, tsel.p};
  const int32_t root[3] = {0, (int32_t)n, 0};
  PM_HIP_TRY(hipMemcpyAsync(tb.p, &root[0], 4, hipMemcpyHostToDevice, s));
  PM_HIP_TRY(hipMemcpyAsync(ts.p, &root[1], 4, hipMemcpyHostToDevice, s));
  PM_HIP_TRY(hipMemcpyAsync(tsel.p, &root[2], 4, hipMemcpyHostToDevice, s));
  // segments at L0 hold <= 1023 elements; the check variant keeps every level
  // global (the identical-tree test compares the two libraries)
  const int L0 = PM_CHECK_VARIANT ? H : std::max(0, H - kLocalLog);
  for (int L = 0; L < H; L++) {
    if (L == L0) {
      k_kd_local<false><<<(int)(1ll << L0), kLocal, 0, s>>>(Lst, KdSoa{}, L0, T, nodes);
      PM_HIP_TRY(hipGetLastError());
      break;
    }
    const int64_t nseg = 1ll << L;
    k_kd_seg<<<grid_for(nseg, 256), 256, 0, s>>>(Lst, L, cap, T, nodes);
    PM_HIP_TRY(hipGetLastError());
    if (L == H - 1) break;   // last level: every remaining subtree has one node
    k_kd_tileseg<<<grid_for(ntiles + 1, 256), 256, 0, s>>>(tb.p, L, ntiles, tile_seg.p);
    PM_HIP_TRY(hipGetLastError());
    k_kd_count<<<(int)ntiles, kCountThreads, 0, s>>>(Lst, n, T, L, tile_seg.p, tagg.p);
    PM_HIP_TRY(hipGetLastError());
    k_kd_chunkscan<<<nchunks, kChunk, 0, s>>>(tagg.p, ntiles, tcarry.p, ccarry.p);
    PM_HIP_TRY(hipGetLastError());
    k_kd_chunkcarry<<<1, kChunk, 0, s>>>(ccarry.p, nchunks);
    PM_HIP_TRY(hipGetLastError());
    k_kd_part<<<(int)ntiles, kPartThreads, 0, s>>>(Lst, n, T, L, tile_seg.p, tcarry.p, ccarry.p);
    PM_HIP_TRY(hipGetLastError());
  }
  return hipSuccess;
}


// ---------------------------------------------------------------- helpers for the C-ABI
// A NaN coordinate becomes +inf (include/pm.h): the photon sorts last, compares
// consistently in every pass (NaN compares false both ways, so the float
// classification and the sort keys would disagree), and is never within a
// gather radius.
__device__ __forceinline__ float kd_coord(float x) { return x != x ? __int_as_float(0x7f800000) : x; }

// one run of photon rows -> elements [id0, id0 + n) and their payload
__global__ void k_elems_from_rows(const float* __restrict__ rows, int stride, int coff, int64_t n, int64_t id0,
                                  float power, float4* __restrict__ elems, float4* __restrict__ payload) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = rows + i * stride;
  elems[id0 + i] = make_float4(kd_coord(r[0]), kd_coord(r[1]), kd_coord(r[2]), __int_as_float((int)(id0 + i)));
  payload[id0 + i] = make_float4(r[coff], r[coff + 1], r[coff + 2], power);
}

__global__ void k_elems_from_kd(const pm_kd_photon* in, int64_t n, float4* elems) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  elems[i] = make_float4(kd_coord(in[i].pos.x), kd_coord(in[i].pos.y), kd_coord(in[i].pos.z),
                         __int_as_float((int)i));
}

__global__ void k_kd_reorder(const pm_kd_photon* src, const float4* nodes, int64_t n, pm_kd_photon* dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int w = __float_as_int(nodes[t].w);
  pm_kd_photon p = src[(uint32_t)w >> 2];
  p.split_dim = (uint8_t)(w & 3);
  dst[t] = p;
}

__global__ void k_map_export(const float4* nodes, const float4* payload, int64_t n, pm_kd_photon* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float4 nd = nodes[t];
  const int w = __float_as_int(nd.w);
  const float4 pl = payload[(uint32_t)w >> 2];
  pm_kd_photon p;
  p.pos = {nd.x, nd.y, nd.z};
  p.dir = {0.f, 0.f, 0.f};
  p.color = {pl.x, pl.y, pl.z};
  p.power = pl.w;
  p.quantized_normal[0] = p.quantized_normal[1] = p.quantized_normal[2] = 0;
  p.split_dim = (uint8_t)(w & 3);
  out[t] = p;
}

// wave-reduced first: one atomic per wave and component (same-address global
// atomics serialise at one L2 channel)
__global__ void k_bounds(const float4* elems, int64_t n, unsigned* ob) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0u, 0u, 0u};
  if (i < n) {
    const float4 e = elems[i];
    const float c[3] = {e.x, e.y, e.z};
#pragma unroll
    for (int k = 0; k < 3; k++) mn[k] = mx[k] = orderable_key(c[k]);
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn[k] = min(mn[k], (uint32_t)__shfl_xor((int)mn[k], o));
      mx[k] = max(mx[k], (uint32_t)__shfl_xor((int)mx[k], o));
    }
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      atomicMin(&ob[k], mn[k]);
      atomicMax(&ob[3 + k], mx[k]);
    }
  }
}

__global__ void k_bounds_final(const unsigned* ob, pm_box* box) {
  float v[6];
  for (int k = 0; k < 6; k++) {
    const uint32_t u = ob[k];
    const uint32_t bits = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    v[k] = __uint_as_float(bits);
  }
  box->lower = {v[0], v[1], v[2]};
  box->upper = {v[3], v[4], v[5]};
}

int64_t rows_total(const RowRuns& runs) {
  int64_t n = 0;
  for (const RowRun& r : runs) n += r.n;
  return n;
}

hipError_t launch_elems_from_rows(const RowRuns& runs, float4* elems, float4* payload, hipStream_t s) {
  int64_t id0 = 0;
  for (const RowRun& r : runs) {
    if (r.n > 0) {
      k_elems_from_rows<<<grid_for(r.n, 256), 256, 0, s>>>(r.rows, r.stride, r.coff, r.n, id0, r.power, elems,
                                                          payload);
      PM_HIP_TRY(hipGetLastError());
    }
    id0 += r.n;
  }
  return hipSuccess;
}

hipError_t kd_build_records(pm_kd_photon* d, int64_t n, pm_box* bounds, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  DevBuf<float4> elems(n), nodes(n);
  DevBuf<pm_kd_photon> copy(n);
  if (!elems.p || !nodes.p || !copy.p) return hipErrorOutOfMemory;
  k_elems_from_kd<<<grid_for(n, 256), 256, 0, s>>>(d, n, elems.p);
  PM_HIP_TRY(hipGetLastError());
  if (bounds) {
    DevBuf<unsigned> ob(6);
    const unsigned init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    PM_HIP_TRY(hipMemcpyAsync(ob.p, init, sizeof(init), hipMemcpyHostToDevice, s));
    k_bounds<<<grid_for(n, 256), 256, 0, s>>>(elems.p, n, ob.p);
    PM_HIP_TRY(hipGetLastError());
    k_bounds_final<<<1, 1, 0, s>>>(ob.p, bounds);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(hipStreamSynchronize(s));
  }
  PM_HIP_TRY(kd_build(elems.p, n, nodes.p, s));
  PM_HIP_TRY(hipMemcpyAsync(copy.p, d, sizeof(pm_kd_photon) * n, hipMemcpyDeviceToDevice, s));
  k_kd_reorder<<<grid_for(n, 256), 256, 0, s>>>(copy.p, nodes.p, n, d);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

hipError_t launch_map_export(const pm_photon_map* m, pm_kd_photon* out, hipStream_t s) {
  if (m->n <= 0) return hipSuccess;
  k_map_export<<<grid_for(m->n, 256), 256, 0, s>>>(m->nodes.p, m->payload.p, m->n, out);
  return hipGetLastError();
}

}  // namespace pmd

#ifdef PM_KD_DIAG_TIME
extern "C" int pm_diag_kd_stamps(unsigned long long* out, long long n) {
  if (n > (long long)pmd::kDiagBlocks * pmd::kDiagStamps) n = (long long)pmd::kDiagBlocks * pmd::kDiagStamps;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pmd::g_kd_stamp), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif
