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
// directly from the list of the chosen dimension and the three lists are
// stably partitioned around it with one fused flag pass, one u64 scan and one
// scatter. Subtree ranges are identical in the three lists, so a single tag
// array tracks subtree membership. Ties are broken by the original index.
#include <algorithm>
#include <cstdlib>

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

__global__ void k_kd_init_keys(const float4* elems, int64_t n, int d, uint32_t* keys, uint32_t* vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = orderable_key(coord_of(elems[i], d));
  vals[i] = (uint32_t)i;
}

__global__ void k_kd_gather(const float4* elems, const uint32_t* order, int64_t n, float4* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = elems[order[i]];
}

struct SegTab {
  int32_t* b;
  int32_t* s;
  int32_t* ls;
  int32_t* dim;
  float* coord;
  int32_t* id;
};

__global__ void k_kd_seg(const float4* l0, const float4* l1, const float4* l2, int level, int64_t cap, SegTab T,
                         float4* out_nodes) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nseg = 1ll << level;
  if (j >= nseg) return;
  const int64_t t = nseg - 1 + j;
  const int b = T.b[t], s = T.s[t];
  const int64_t c1 = 2 * t + 1, c2 = 2 * t + 2;
  if (s <= 0) {
    T.ls[t] = -1;
    if (c2 < cap) {
      T.b[c1] = b; T.s[c1] = 0;
      T.b[c2] = b; T.s[c2] = 0;
    }
    return;
  }
  const int ls = left_size(s);
  const float4* L[3] = {l0, l1, l2};
  float ext[3];
#pragma unroll
  for (int d = 0; d < 3; d++) ext[d] = coord_of(L[d][b + s - 1], d) - coord_of(L[d][b], d);
  int dim = 0;
  if (ext[1] > ext[dim]) dim = 1;
  if (ext[2] > ext[dim]) dim = 2;
  const float4 e = L[dim][b + ls];
  const int id = __float_as_int(e.w);
  T.ls[t] = ls;
  T.dim[t] = dim;
  T.coord[t] = coord_of(e, dim);
  T.id[t] = id;
  out_nodes[t] = make_float4(e.x, e.y, e.z, __int_as_float((id << 2) | dim));
  if (c2 < cap) {
    T.b[c1] = b; T.s[c1] = ls;
    T.b[c2] = b + ls + 1; T.s[c2] = s - ls - 1;
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

__global__ void k_kd_flags(const float4* l0, const float4* l1, const float4* l2, const int32_t* tag, int64_t n,
                           SegTab T, uint64_t* flags) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int t = tag[p];
  if (t < 0) {
    flags[p] = 0;
    flags[n + p] = 0;
    flags[2 * n + p] = 0;
    return;
  }
  const int dim = T.dim[t];
  const float nc = T.coord[t];
  const int nid = T.id[t];
  const float4 e[3] = {l0[p], l1[p], l2[p]};
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const int c = kd_class(e[d], dim, nc, nid);
    flags[(int64_t)d * n + p] = c == 0 ? 1ull : (c == 2 ? (1ull << 32) : 0ull);
  }
}

__global__ void k_kd_scatter(const float4* l0, const float4* l1, const float4* l2, float4* o0, float4* o1, float4* o2,
                             const int32_t* tag, int64_t n, SegTab T, const uint64_t* pre) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int t = tag[p];
  const float4* L[3] = {l0, l1, l2};
  float4* O[3] = {o0, o1, o2};
  if (t < 0) {
#pragma unroll
    for (int d = 0; d < 3; d++) O[d][p] = L[d][p];
    return;
  }
  const int b = T.b[t], ls = T.ls[t], dim = T.dim[t];
  const float nc = T.coord[t];
  const int nid = T.id[t];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const float4 e = L[d][p];
    const int c = kd_class(e, dim, nc, nid);
    const uint64_t pp = pre[(int64_t)d * n + p], pb = pre[(int64_t)d * n + b];
    int64_t np;
    if (c == 0)
      np = b + (int64_t)((uint32_t)pp - (uint32_t)pb);
    else if (c == 1)
      np = b + ls;
    else
      np = b + ls + 1 + (int64_t)((uint32_t)(pp >> 32) - (uint32_t)(pb >> 32));
    O[d][np] = e;
  }
}

__global__ void k_kd_tag(int32_t* tag, int64_t n, SegTab T) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int t = tag[p];
  if (t < 0) return;
  const int mid = T.b[t] + T.ls[t];
  tag[p] = p < mid ? 2 * t + 1 : (p == mid ? -1 : 2 * t + 2);
}

hipError_t kd_build(const float4* elems, int64_t n, float4* nodes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n >= (1ll << 30)) return hipErrorInvalidValue;
  int H = 0;
  while ((1ll << H) <= n) H++;          // levels = floor(log2 n) + 1
  const int64_t cap = 1ll << (H + 1);
  DevBuf<float4> la[3], lb[3];
  for (int d = 0; d < 3; d++) {
    la[d].alloc(n);
    lb[d].alloc(n);
    if (!la[d].p || !lb[d].p) return hipErrorOutOfMemory;
  }
  {
    DevBuf<uint32_t> keys(n), vals(n);
    if (!keys.p || !vals.p) return hipErrorOutOfMemory;
    for (int d = 0; d < 3; d++) {
      k_kd_init_keys<<<grid_for(n, 256), 256, 0, s>>>(elems, n, d, keys.p, vals.p);
      PM_HIP_TRY(hipGetLastError());
      PM_HIP_TRY(radix_sort_pairs(keys.p, vals.p, n, 32, s));
      k_kd_gather<<<grid_for(n, 256), 256, 0, s>>>(elems, vals.p, n, la[d].p);
      PM_HIP_TRY(hipGetLastError());
    }
  }
  DevBuf<int32_t> tb(cap), ts(cap), tls(cap), tdim(cap), tid(cap), tag(n);
  DevBuf<float> tco(cap);
  DevBuf<uint64_t> flags((size_t)3 * n), pre((size_t)3 * n);
  if (!tb.p || !ts.p || !tls.p || !tdim.p || !tid.p || !tag.p || !tco.p || !flags.p || !pre.p)
    return hipErrorOutOfMemory;
  SegTab T{tb.p, ts.p, tls.p, tdim.p, tco.p, tid.p};
  const int32_t root[2] = {0, (int32_t)n};
  PM_HIP_TRY(hipMemcpyAsync(tb.p, &root[0], 4, hipMemcpyHostToDevice, s));
  PM_HIP_TRY(hipMemcpyAsync(ts.p, &root[1], 4, hipMemcpyHostToDevice, s));
  PM_HIP_TRY(hipMemsetAsync(tag.p, 0, sizeof(int32_t) * n, s));
  float4* cur[3] = {la[0].p, la[1].p, la[2].p};
  float4* nxt[3] = {lb[0].p, lb[1].p, lb[2].p};
  for (int L = 0; L < H; L++) {
    const int64_t nseg = 1ll << L;
    k_kd_seg<<<grid_for(nseg, 256), 256, 0, s>>>(cur[0], cur[1], cur[2], L, cap, T, nodes);
    PM_HIP_TRY(hipGetLastError());
    if (L == H - 1) break;   // last level: every remaining subtree has one node
    k_kd_flags<<<grid_for(n, 256), 256, 0, s>>>(cur[0], cur[1], cur[2], tag.p, n, T, flags.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(exclusive_scan_u64(flags.p, pre.p, 3 * n, nullptr, s));
    k_kd_scatter<<<grid_for(n, 256), 256, 0, s>>>(cur[0], cur[1], cur[2], nxt[0], nxt[1], nxt[2], tag.p, n, T,
                                                   pre.p);
    PM_HIP_TRY(hipGetLastError());
    k_kd_tag<<<grid_for(n, 256), 256, 0, s>>>(tag.p, n, T);
    PM_HIP_TRY(hipGetLastError());
    for (int d = 0; d < 3; d++) {
      float4* t = cur[d];
      cur[d] = nxt[d];
      nxt[d] = t;
    }
  }
  return hipSuccess;
}

// ---------------------------------------------------------------- buckets
__global__ void k_kd_buckets(const float4* nodes, int64_t n, int first, int nb, int levels, float4* out) {
  const int slots = (1 << levels) - 1;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)nb * slots) return;
  const int64_t b = i / slots;
  const int sl = (int)(i % slots);
  const int lvl = 31 - __clz(sl + 1);            // level inside the subtree
  const int j = sl + 1 - (1 << lvl);             // position in that level
  const int64_t root = first + b;
  const int64_t t = ((root + 1) << lvl) - 1 + j;  // implicit index of the node
  out[i] = t < n ? nodes[t] : make_float4(INFINITY, INFINITY, INFINITY, __int_as_float(-1));
}

hipError_t kd_make_buckets(pm_photon_map* m, hipStream_t s) {
  const int64_t n = m->n;
  m->bucket_first = INT32_MAX;
  m->bucket_slots = 0;
  m->bucket_data.reset();
  int B = kBucketLevels;
  if (const char* e = std::getenv("PM_KD_BUCKET_LEVELS")) B = std::atoi(e);   // tuning knob; 0 = off
  if (n <= 0 || B <= 0) return hipSuccess;
  int H = 0;
  while ((1ll << H) <= n) H++;                   // levels
  const int lb = H > B ? H - B : 0;
  const int levels = H - lb;
  const int first = (1 << lb) - 1;
  const int nb = (int)std::min<int64_t>(1ll << lb, std::max<int64_t>(0, n - first));
  const int slots = (1 << levels) - 1;
  m->bucket_data.alloc((size_t)nb * slots);
  if (!m->bucket_data.p) return hipErrorOutOfMemory;
  k_kd_buckets<<<grid_for((int64_t)nb * slots, 256), 256, 0, s>>>(m->nodes.p, n, first, nb, levels,
                                                                 m->bucket_data.p);
  PM_HIP_TRY(hipGetLastError());
  m->bucket_first = first;
  m->bucket_slots = slots;
  return hipSuccess;
}

// ---------------------------------------------------------------- helpers for the C-ABI
__global__ void k_elems_from_photons(const pm_photon* a, int64_t na, const pm_photon* b, int64_t nb, float pa,
                                     float pb, float4* elems, float4* payload) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na + nb) return;
  const pm_photon p = i < na ? a[i] : b[i - na];
  elems[i] = make_float4(p.pos.x, p.pos.y, p.pos.z, __int_as_float((int)i));
  payload[i] = make_float4(p.color.x, p.color.y, p.color.z, i < na ? pa : pb);
}

__global__ void k_elems_from_kd(const pm_kd_photon* in, int64_t n, float4* elems) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  elems[i] = make_float4(in[i].pos.x, in[i].pos.y, in[i].pos.z, __int_as_float((int)i));
}

__global__ void k_kd_reorder(const pm_kd_photon* src, const float4* nodes, int64_t n, pm_kd_photon* dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int w = __float_as_int(nodes[t].w);
  pm_kd_photon p = src[w >> 2];
  p.split_dim = (uint8_t)(w & 3);
  dst[t] = p;
}

__global__ void k_map_export(const float4* nodes, const float4* payload, int64_t n, pm_kd_photon* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float4 nd = nodes[t];
  const int w = __float_as_int(nd.w);
  const float4 pl = payload[w >> 2];
  pm_kd_photon p;
  p.pos = {nd.x, nd.y, nd.z};
  p.dir = {0.f, 0.f, 0.f};
  p.color = {pl.x, pl.y, pl.z};
  p.power = pl.w;
  p.quantized_normal[0] = p.quantized_normal[1] = p.quantized_normal[2] = 0;
  p.split_dim = (uint8_t)(w & 3);
  out[t] = p;
}

__global__ void k_bounds(const float4* elems, int64_t n, unsigned* ob) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 e = elems[i];
  const float c[3] = {e.x, e.y, e.z};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    atomicMin(&ob[k], orderable_key(c[k]));
    atomicMax(&ob[3 + k], orderable_key(c[k]));
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

hipError_t launch_elems_from_photons(const pm_photon* a, int64_t na, const pm_photon* b, int64_t nb, float pa,
                                     float pb, float4* elems, float4* payload, hipStream_t s) {
  if (na + nb <= 0) return hipSuccess;
  k_elems_from_photons<<<grid_for(na + nb, 256), 256, 0, s>>>(a, na, b, nb, pa, pb, elems, payload);
  return hipGetLastError();
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
