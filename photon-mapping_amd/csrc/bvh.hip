// bvh.hip — LBVH build (Karras 2012) and ray-query kernels for gfx950.
//
// Replaces the OptiX GAS+IAS build of common/src/world.cpp:3-58 (loadGeometry:
// one build input per mesh, owlGroupBuildAccel) and the RT-core traversal
// behind every owl::traceRay / optixTrace. Pipeline: 30-bit Morton codes of
// triangle centroids -> stable radix sort -> PLOC clustering (default) or the
// Karras hierarchy + bottom-up refit (agent-scope release/acquire hand-off
// between sibling threads) into 64-B BVH2 nodes that carry both child boxes ->
// greedy top-down collapse into 128-B BVH4 nodes (one cache line = four box
// tests), which the traversal uses.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "pm_internal.hpp"

namespace pmd {

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void k_morton(const float4* tri, int n, float3 lo, float3 inv_ext, uint32_t* codes, uint32_t* idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 a = tri[3 * i], b = tri[3 * i + 1], c = tri[3 * i + 2];
  const float cx = (a.x + b.x + c.x) / 3.0f, cy = (a.y + b.y + c.y) / 3.0f, cz = (a.z + b.z + c.z) / 3.0f;
  const float fx = fminf(fmaxf((cx - lo.x) * inv_ext.x * 1024.0f, 0.0f), 1023.0f);
  const float fy = fminf(fmaxf((cy - lo.y) * inv_ext.y * 1024.0f, 0.0f), 1023.0f);
  const float fz = fminf(fmaxf((cz - lo.z) * inv_ext.z * 1024.0f, 0.0f), 1023.0f);
  codes[i] = (expand_bits((uint32_t)fx) << 2) | (expand_bits((uint32_t)fy) << 1) | expand_bits((uint32_t)fz);
  idx[i] = (uint32_t)i;
}

__global__ void k_gather_tris(const float4* src, const uint32_t* order, int n, float4* dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t o = order[i];
  dst[3 * i] = src[3 * o];
  dst[3 * i + 1] = src[3 * o + 1];
  dst[3 * i + 2] = src[3 * o + 2];
}

__device__ __forceinline__ int delta(const uint32_t* codes, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint32_t ci = codes[i], cj = codes[j];
  if (ci == cj) return 32 + __clz((uint32_t)(i ^ j));
  return __clz(ci ^ cj);
}

// Karras 2012, Fig. 4: internal node i covers [min(i,j), max(i,j)], split gamma.
__global__ void k_hierarchy(const uint32_t* codes, int n, int4* child, int* parent_int, int* parent_leaf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = (delta(codes, n, i, i + 1) - delta(codes, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(codes, n, i, i - d);
  int lmax = 2;
  while (delta(codes, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(codes, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(codes, n, i, j);
  int s = 0;
  int t = l;
  do {
    t = (t + 1) >> 1;
    if (delta(codes, n, i, i + (s + t) * d) > dnode) s += t;
  } while (t > 1);
  const int gamma = i + s * d + min(d, 0);
  const int lo = min(i, j), hi = max(i, j);
  int left, right;
  if (lo == gamma) {
    left = ~gamma;
    parent_leaf[gamma] = i;
  } else {
    left = gamma;
    parent_int[gamma] = i;
  }
  if (hi == gamma + 1) {
    right = ~(gamma + 1);
    parent_leaf[gamma + 1] = i;
  } else {
    right = gamma + 1;
    parent_int[gamma + 1] = i;
  }
  child[i] = make_int4(left, right, 0, 0);
}

__device__ __forceinline__ void write_child_box(float4* nodes, int node, int side, const float b[6]) {
  // node layout: n0 = (lx0, lx1, ly0, ly1), n1 = (lz0, lz1, rx0, rx1), n2 = (ry0, ry1, rz0, rz1)
  float* f = reinterpret_cast<float*>(&nodes[4 * node]);
  const int base = side == 0 ? 0 : 6;
#pragma unroll
  for (int k = 0; k < 6; k++) f[base + k] = b[k];
}

// Bottom-up refit: each leaf walks up; the second arriving child of a node
// unions both boxes. Hand-off per cdna_hip_programming.md Guideline 16:
// plain stores -> release fence -> asm vmcnt(0) -> relaxed agent atomic;
// consumer: atomic returns -> acquire fence -> loads.
__global__ void k_refit(const float4* tri, int n, float pad, float4* nodes, const int4* child,
                        const int* parent_int, const int* parent_leaf, unsigned* flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 a = tri[3 * i], b = tri[3 * i + 1], c = tri[3 * i + 2];
  float bx[6] = {fminf(fminf(a.x, b.x), c.x) - pad, fmaxf(fmaxf(a.x, b.x), c.x) + pad,
                 fminf(fminf(a.y, b.y), c.y) - pad, fmaxf(fmaxf(a.y, b.y), c.y) + pad,
                 fminf(fminf(a.z, b.z), c.z) - pad, fmaxf(fmaxf(a.z, b.z), c.z) + pad};
  int p = parent_leaf[i];
  int me = ~i;
  for (;;) {
    const int4 ch = child[p];
    write_child_box(nodes, p, ch.x == me ? 0 : 1, bx);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(&flags[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float* f = reinterpret_cast<const float*>(&nodes[4 * p]);
    float u[6];
    u[0] = fminf(__hip_atomic_load(&f[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&f[6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    u[1] = fmaxf(__hip_atomic_load(&f[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&f[7], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    u[2] = fminf(__hip_atomic_load(&f[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&f[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    u[3] = fmaxf(__hip_atomic_load(&f[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&f[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    u[4] = fminf(__hip_atomic_load(&f[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&f[10], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    u[5] = fmaxf(__hip_atomic_load(&f[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&f[11], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
    for (int k = 0; k < 6; k++) bx[k] = u[k];
    if (p == 0) return;
    me = p;
    p = parent_int[p];
  }
}

__global__ void k_pack_children(float4* nodes, const int4* child, int nn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  nodes[4 * i + 3] = *reinterpret_cast<const float4*>(&child[i]);
}

// ---------------------------------------------------------------- PLOC
// Parallel locally-ordered clustering (Meister & Bittner 2018), the default
// binary builder (PM_BVH=lbvh selects the Karras hierarchy + refit above): the
// leaves in Morton order are the initial clusters; every iteration each cluster
// finds its nearest neighbour within +-r positions (surface area of
// the merged box; ties to the lower index), mutual pairs merge into a new node,
// survivors are compacted in order. Node ids are handed out from n-2 down, so
// the last merge (the root) is node 0, as collapse_bvh4 expects. Deterministic.
// A tree closer to SAH quality only changes the traversal's speed: hits are
// argmin (t, triangle id) whatever the tree.
constexpr int kPlocRadius = 32;   // LDS window; the search radius r <= kPlocRadius (PM_PLOC_RADIUS)
constexpr int kPlocBlock = 256;
constexpr int kPlocDefaultRadius = 8;   // config 3 frame: r 8 168.2 ms, 16 168.5, 24 173.3, 32 175.4 (LBVH 176.4); at 137 ms: r 2 137.5, 4 138.1, 8 136.9, 16 137.2, 32 140.3

struct Clu {   // cluster: box (lo.xyz, code bits) (hi.xyz, -)
  float4 lo, hi;
};

__device__ __forceinline__ float merged_area(const Clu& a, const Clu& b) {
  const float dx = fmaxf(a.hi.x, b.hi.x) - fminf(a.lo.x, b.lo.x);
  const float dy = fmaxf(a.hi.y, b.hi.y) - fminf(a.lo.y, b.lo.y);
  const float dz = fmaxf(a.hi.z, b.hi.z) - fminf(a.lo.z, b.lo.z);
  return dx * dy + dy * dz + dz * dx;
}

__global__ void k_ploc_leaves(const float4* tri, int n, float pad, Clu* c) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 a = tri[3 * i], b = tri[3 * i + 1], d = tri[3 * i + 2];
  Clu u;
  u.lo = make_float4(fminf(fminf(a.x, b.x), d.x) - pad, fminf(fminf(a.y, b.y), d.y) - pad,
                     fminf(fminf(a.z, b.z), d.z) - pad, __int_as_float(~i));
  u.hi = make_float4(fmaxf(fmaxf(a.x, b.x), d.x) + pad, fmaxf(fmaxf(a.y, b.y), d.y) + pad,
                     fmaxf(fmaxf(a.z, b.z), d.z) + pad, 0.f);
  c[i] = u;
}

__global__ __launch_bounds__(kPlocBlock) void k_ploc_nn(const Clu* __restrict__ c, int m, int r,
                                                        int* __restrict__ nn) {
  __shared__ Clu sc[kPlocBlock + 2 * kPlocRadius];
  const int b0 = blockIdx.x * kPlocBlock - kPlocRadius;
  for (int k = threadIdx.x; k < kPlocBlock + 2 * kPlocRadius; k += kPlocBlock) {
    const int g = b0 + k;
    if (g >= 0 && g < m) sc[k] = c[g];
  }
  __syncthreads();
  const int i = blockIdx.x * kPlocBlock + threadIdx.x;
  if (i >= m) return;
  const Clu me = sc[threadIdx.x + kPlocRadius];
  float best = INFINITY;
  int bj = -1;
  for (int d = -r; d <= r; d++) {
    const int j = i + d;
    if (d == 0 || j < 0 || j >= m) continue;
    const float a = merged_area(me, sc[threadIdx.x + kPlocRadius + d]);
    if (a < best) {   // ascending j: ties keep the lower index
      best = a;
      bj = j;
    }
  }
  nn[i] = bj;
}

// merge_lo: i is the lower index of a mutual pair; keep: i survives the compaction
__global__ void k_ploc_flags(const int* __restrict__ nn, int m, uint32_t* __restrict__ merge_lo,
                             uint32_t* __restrict__ keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int j = nn[i];
  const bool mutual = j >= 0 && nn[j] == i;
  merge_lo[i] = mutual && i < j;
  keep[i] = !(mutual && i > j);
}

__global__ void k_ploc_merge(Clu* __restrict__ c, const int* __restrict__ nn, int m,
                             const uint32_t* __restrict__ merge_lo, const uint32_t* __restrict__ moff, int top,
                             float4* __restrict__ bin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !merge_lo[i]) return;
  const Clu a = c[i], b = c[nn[i]];
  const int node = top - 1 - (int)moff[i];
  float* f = reinterpret_cast<float*>(&bin[4 * node]);   // (l box, r box), then child codes
  f[0] = a.lo.x; f[1] = a.hi.x; f[2] = a.lo.y; f[3] = a.hi.y; f[4] = a.lo.z; f[5] = a.hi.z;
  f[6] = b.lo.x; f[7] = b.hi.x; f[8] = b.lo.y; f[9] = b.hi.y; f[10] = b.lo.z; f[11] = b.hi.z;
  bin[4 * node + 3] = make_float4(a.lo.w, b.lo.w, 0.f, 0.f);
  Clu u;
  u.lo = make_float4(fminf(a.lo.x, b.lo.x), fminf(a.lo.y, b.lo.y), fminf(a.lo.z, b.lo.z), __int_as_float(node));
  u.hi = make_float4(fmaxf(a.hi.x, b.hi.x), fmaxf(a.hi.y, b.hi.y), fmaxf(a.hi.z, b.hi.z), 0.f);
  c[i] = u;
}

__global__ void k_ploc_compact(const Clu* __restrict__ c, int m, const uint32_t* __restrict__ keep,
                               const uint32_t* __restrict__ koff, Clu* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !keep[i]) return;
  out[koff[i]] = c[i];
}

static hipError_t build_ploc(const float4* tri, int n, float pad, float4* bin, hipStream_t s) {
  DevBuf<Clu> ca(n), cb(n);
  DevBuf<int> nn(n);
  DevBuf<uint32_t> mlo(n), moff(n), keep(n), koff(n), tot(2);
  if (!ca.p || !cb.p || !nn.p || !mlo.p || !moff.p || !keep.p || !koff.p || !tot.p) return hipErrorOutOfMemory;
  k_ploc_leaves<<<grid_for(n, 256), 256, 0, s>>>(tri, n, pad, ca.p);
  PM_HIP_TRY(hipGetLastError());
  Clu *cur = ca.p, *nxt = cb.p;
  const int r = kPlocDefaultRadius;
  int m = n, top = n - 1;   // internal node ids top-1 .. 0
  while (m > 1) {
    k_ploc_nn<<<grid_for(m, kPlocBlock), kPlocBlock, 0, s>>>(cur, m, r, nn.p);
    PM_HIP_TRY(hipGetLastError());
    k_ploc_flags<<<grid_for(m, 256), 256, 0, s>>>(nn.p, m, mlo.p, keep.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(exclusive_scan_u32(mlo.p, moff.p, m, tot.p, s));
    PM_HIP_TRY(exclusive_scan_u32(keep.p, koff.p, m, tot.p + 1, s));
    k_ploc_merge<<<grid_for(m, 256), 256, 0, s>>>(cur, nn.p, m, mlo.p, moff.p, top, bin);
    PM_HIP_TRY(hipGetLastError());
    k_ploc_compact<<<grid_for(m, 256), 256, 0, s>>>(cur, m, keep.p, koff.p, nxt);
    PM_HIP_TRY(hipGetLastError());
    uint32_t h[2] = {0, 0};
    PM_HIP_TRY(hipMemcpyAsync(h, tot.p, sizeof(h), hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
    if (h[0] == 0) return hipErrorUnknown;   // cannot happen: the closest pair is mutual
    top -= (int)h[0];
    m = (int)h[1];
    std::swap(cur, nxt);
  }
  return top == 0 ? hipStreamSynchronize(s) : hipErrorUnknown;
}

// ---------------------------------------------------------------- BVH4 collapse
// The binary LBVH is collapsed top-down into 4-wide nodes (128 B, one cache
// line: SoA child boxes + 4 child codes). A BVH4 node adopts the two children
// of its binary node, then repeatedly opens the internal candidate with the
// largest surface area until it holds 4 (Wald et al. 2008 style greedy
// collapse). One level of the BVH4 per launch pair; node ids are assigned by
// an exclusive scan so the layout is deterministic.
__device__ __forceinline__ float box_area(const float b[6]) {
  const float dx = b[1] - b[0], dy = b[3] - b[2], dz = b[5] - b[4];
  return dx * dy + dy * dz + dz * dx;
}

__global__ void k_collapse_open(const float4* __restrict__ bin, const int2* __restrict__ frontier, int nf,
                                float4* __restrict__ q, uint32_t* __restrict__ cnt) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nf) return;
  const int2 fr = frontier[f];
  int code[4];
  float box[4][6];
  const float* nb = reinterpret_cast<const float*>(&bin[4 * fr.x]);
  const int4 c2 = *reinterpret_cast<const int4*>(&bin[4 * fr.x + 3]);
  code[0] = c2.x;
  code[1] = c2.y;
#pragma unroll
  for (int k = 0; k < 6; k++) box[0][k] = nb[k], box[1][k] = nb[6 + k];
  int m = 2;
  for (int it = 0; it < 2; it++) {
    int best = -1;
    float barea = -1.0f;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      if (c < m && code[c] >= 0) {
        const float a = box_area(box[c]);
        if (a > barea) barea = a, best = c;
      }
    }
    if (best < 0) break;
    const float* ob = reinterpret_cast<const float*>(&bin[4 * code[best]]);
    const int4 oc = *reinterpret_cast<const int4*>(&bin[4 * code[best] + 3]);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      if (c == best) {
        code[c] = oc.x;
#pragma unroll
        for (int k = 0; k < 6; k++) box[c][k] = ob[k];
      } else if (c == m) {
        code[c] = oc.y;
#pragma unroll
        for (int k = 0; k < 6; k++) box[c][k] = ob[6 + k];
      }
    }
    m++;
  }
  uint32_t internal = 0;
  float* qn = reinterpret_cast<float*>(&q[8 * (int64_t)fr.y]);
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const bool used = c < m;
    if (used && code[c] >= 0) internal++;
#pragma unroll
    for (int k = 0; k < 6; k++) qn[4 * k + c] = used ? box[c][k] : 0.0f;   // k: lo.x hi.x lo.y hi.y lo.z hi.z
    reinterpret_cast<int*>(qn)[24 + c] = used ? code[c] : kBvhEmpty;       // patched by k_collapse_link
    reinterpret_cast<int*>(qn)[28 + c] = 0;
  }
  cnt[f] = internal;
}

__global__ void k_collapse_link(const int2* __restrict__ frontier, int nf, const uint32_t* __restrict__ off,
                                int base, float4* __restrict__ q, int2* __restrict__ next) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nf) return;
  const int2 fr = frontier[f];
  int4* cp = reinterpret_cast<int4*>(&q[8 * (int64_t)fr.y + 6]);
  int4 c = *cp;
  int o = (int)off[f];
  int* cc = reinterpret_cast<int*>(&c);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (cc[k] >= 0) {
      next[o] = make_int2(cc[k], base + o);
      cc[k] = base + o;
      o++;
    }
  }
  *cp = c;
}

// decoded plane of a quantised box: p + q s (q s exact, one rounding)
__device__ __forceinline__ float q_decode(float p, uint32_t q, float sc) { return p + (float)q * sc; }

// PM_BVH_Q4: the float BVH4 node (8 x float4) -> 64 B (4 x float4, see
// traverse_step4): corner p = min of the used children's lo, per-axis scale
// s = 2^e with 255 s >= the children's extent, each child plane rounded
// outwards (floor / ceil, then stepped until the float decode p + q s encloses
// the padded float plane), so culling stays conservative and results stay
// bitwise (argmin (t, id) does not depend on the visit order).
__global__ void k_quantize4(const float4* __restrict__ f, int nn, float4* __restrict__ q) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  const float4* fn = f + 8 * (int64_t)i;
  const float4 lo4[3] = {fn[0], fn[2], fn[4]}, hi4[3] = {fn[1], fn[3], fn[5]};
  const int4 ch = *reinterpret_cast<const int4*>(&fn[6]);
  const int cd[4] = {ch.x, ch.y, ch.z, ch.w};
  auto comp = [](const float4& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); };
  float p[3];
  uint32_t eb[3], ql[3] = {0, 0, 0}, qh[3] = {0, 0, 0};
  for (int a = 0; a < 3; a++) {
    float lo = INFINITY, hi = -INFINITY;
    for (int c = 0; c < 4; c++)
      if (cd[c] != kBvhEmpty) lo = fminf(lo, comp(lo4[a], c)), hi = fmaxf(hi, comp(hi4[a], c));
    if (!(lo <= hi)) lo = hi = 0.f;   // no used child
    p[a] = lo;
    const double ext = (double)hi - (double)lo;
    int e = 1;
    if (ext > 0.0) {
      int k;
      frexp(ext / 255.0, &k);
      e = k + 127;
    }
    e = e < 1 ? 1 : e;
    while (e < 254 && q_decode(p[a], 255u, __uint_as_float((uint32_t)e << 23)) < hi) e++;
    eb[a] = (uint32_t)e;
    const float sc = __uint_as_float((uint32_t)e << 23);
    const double inv = 1.0 / (double)sc;
    for (int c = 0; c < 4; c++) {
      if (cd[c] == kBvhEmpty) continue;
      const float bl = comp(lo4[a], c), bh = comp(hi4[a], c);
      uint32_t l = (uint32_t)fmin(fmax(floor(((double)bl - (double)p[a]) * inv), 0.0), 255.0);
      uint32_t u = (uint32_t)fmin(fmax(ceil(((double)bh - (double)p[a]) * inv), 0.0), 255.0);
      while (l > 0 && q_decode(p[a], l, sc) > bl) l--;
      while (u < 255 && q_decode(p[a], u, sc) < bh) u++;
      ql[a] |= l << (8 * c);
      qh[a] |= u << (8 * c);
    }
  }
  float4* qn = q + 4 * (int64_t)i;
  qn[0] = make_float4(p[0], p[1], p[2], __uint_as_float(eb[0] | eb[1] << 8 | eb[2] << 16));
  qn[1] = fn[6];
  qn[2] = make_float4(__uint_as_float(ql[0]), __uint_as_float(ql[1]), __uint_as_float(ql[2]), __uint_as_float(qh[0]));
  qn[3] = make_float4(__uint_as_float(qh[1]), __uint_as_float(qh[2]), 0.f, 0.f);
}

static hipError_t collapse_bvh(const float4* bin, int nbin, pm_scene* sc, hipStream_t s) {
  sc->nodes.alloc((size_t)8 * nbin);
  DevBuf<int2> fa(nbin), fb(nbin);
  DevBuf<uint32_t> cnt(nbin), off(nbin), total(1);
  if (!sc->nodes.p || !fa.p || !fb.p || !cnt.p || !off.p || !total.p) return hipErrorOutOfMemory;
  const int2 root = make_int2(0, 0);
  PM_HIP_TRY(hipMemcpyAsync(fa.p, &root, sizeof(int2), hipMemcpyHostToDevice, s));
  int nf = 1, alloc = 1, depth = 0;
  int2 *cur = fa.p, *nxt = fb.p;
  while (nf > 0) {
    depth++;
    k_collapse_open<<<grid_for(nf, 256), 256, 0, s>>>(bin, cur, nf, sc->nodes.p, cnt.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(exclusive_scan_u32(cnt.p, off.p, nf, total.p, s));
    k_collapse_link<<<grid_for(nf, 256), 256, 0, s>>>(cur, nf, off.p, alloc, sc->nodes.p, nxt);
    PM_HIP_TRY(hipGetLastError());
    uint32_t t = 0;
    PM_HIP_TRY(hipMemcpyAsync(&t, total.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
    alloc += (int)t;
    nf = (int)t;
    std::swap(cur, nxt);
  }
  sc->nnodes = alloc;
  sc->depth = depth;
  if (kBvhQ4) {
    DevBuf<float4> qn((size_t)4 * alloc);
    if (!qn.p) return hipErrorOutOfMemory;
    k_quantize4<<<grid_for(alloc, 256), 256, 0, s>>>(sc->nodes.p, alloc, qn.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(hipStreamSynchronize(s));
    std::swap(sc->nodes.p, qn.p);
    std::swap(sc->nodes.n, qn.n);
  }
  return hipSuccess;
}

hipError_t build_lbvh(pm_scene* sc, const std::vector<float4>& th, hipStream_t s) {
  const int n = sc->ntri;
  if (n == 0) {
    sc->nnodes = 0;
    sc->depth = 0;
    return hipSuccess;
  }
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  float clo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, chi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = 0; i < n; i++) {
    const float4 v[3] = {th[3 * i], th[3 * i + 1], th[3 * i + 2]};
    float c[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++) {
      const float vx = v[k].x, vy = v[k].y, vz = v[k].z;
      lo[0] = std::min(lo[0], vx); hi[0] = std::max(hi[0], vx);
      lo[1] = std::min(lo[1], vy); hi[1] = std::max(hi[1], vy);
      lo[2] = std::min(lo[2], vz); hi[2] = std::max(hi[2], vz);
      c[0] += vx; c[1] += vy; c[2] += vz;
    }
    for (int k = 0; k < 3; k++) {
      clo[k] = std::min(clo[k], c[k] / 3.0f);
      chi[k] = std::max(chi[k], c[k] / 3.0f);
    }
  }
  float ext = 0.f;
  for (int k = 0; k < 3; k++) ext = std::max(ext, hi[k] - lo[k]);
  const float pad = ext * 1e-5f + 1e-20f;
  sc->bounds = {{lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}};

  DevBuf<float4> tri_orig((size_t)3 * n);
  sc->tri.alloc((size_t)3 * n);
  const int nn = std::max(1, n - 1);
  DevBuf<float4> bin((size_t)4 * nn);   // binary LBVH, collapsed into sc->nodes below
  if (!tri_orig.p || !sc->tri.p || !bin.p) return hipErrorOutOfMemory;
  PM_HIP_TRY(hipMemcpyAsync(tri_orig.p, th.data(), sizeof(float4) * 3 * n, hipMemcpyHostToDevice, s));
  if (n == 1) {
    PM_HIP_TRY(hipMemcpyAsync(sc->tri.p, tri_orig.p, sizeof(float4) * 3, hipMemcpyDeviceToDevice, s));
    const float4 a = th[0], b = th[1], c = th[2];
    float bx[6] = {std::min({a.x, b.x, c.x}) - pad, std::max({a.x, b.x, c.x}) + pad,
                   std::min({a.y, b.y, c.y}) - pad, std::max({a.y, b.y, c.y}) + pad,
                   std::min({a.z, b.z, c.z}) - pad, std::max({a.z, b.z, c.z}) + pad};
    float node[16];
    for (int k = 0; k < 6; k++) node[k] = bx[k], node[6 + k] = bx[k];
    const int ch[4] = {~0, ~0, 0, 0};
    std::memcpy(&node[12], ch, 16);
    PM_HIP_TRY(hipMemcpyAsync(bin.p, node, 64, hipMemcpyHostToDevice, s));
    return collapse_bvh(bin.p, nn, sc, s);
  }
  DevBuf<uint32_t> codes(n), order(n);
  DevBuf<int4> child(nn);
  DevBuf<int> pint(nn), pleaf(n);
  DevBuf<unsigned> flags(nn);
  if (!codes.p || !order.p || !child.p || !pint.p || !pleaf.p || !flags.p) return hipErrorOutOfMemory;
  float3 clo3 = make_float3(clo[0], clo[1], clo[2]);
  float3 inv = make_float3(chi[0] > clo[0] ? 1.0f / (chi[0] - clo[0]) : 0.f,
                           chi[1] > clo[1] ? 1.0f / (chi[1] - clo[1]) : 0.f,
                           chi[2] > clo[2] ? 1.0f / (chi[2] - clo[2]) : 0.f);
  k_morton<<<grid_for(n, 256), 256, 0, s>>>(tri_orig.p, n, clo3, inv, codes.p, order.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(radix_sort_pairs(codes.p, order.p, n, 30, s));
  k_gather_tris<<<grid_for(n, 256), 256, 0, s>>>(tri_orig.p, order.p, n, sc->tri.p);
  PM_HIP_TRY(hipGetLastError());
  // production: PLOC clustering; the check variant builds the Karras LBVH below
  // (a different tree: closest hits are argmin (t, id), so results must not move)
  if (!PM_CHECK_VARIANT) {
    PM_HIP_TRY(build_ploc(sc->tri.p, n, pad, bin.p, s));
    return collapse_bvh(bin.p, nn, sc, s);
  }
  PM_HIP_TRY(hipMemsetAsync(pint.p, 0, sizeof(int) * nn, s));
  k_hierarchy<<<grid_for(n - 1, 256), 256, 0, s>>>(codes.p, n, child.p, pint.p, pleaf.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(hipMemsetAsync(flags.p, 0, sizeof(unsigned) * nn, s));
  k_refit<<<grid_for(n, 256), 256, 0, s>>>(sc->tri.p, n, pad, bin.p, child.p, pint.p, pleaf.p, flags.p);
  PM_HIP_TRY(hipGetLastError());
  k_pack_children<<<grid_for(nn, 256), 256, 0, s>>>(bin.p, child.p, nn);
  PM_HIP_TRY(hipGetLastError());
  return collapse_bvh(bin.p, nn, sc, s);
}

// ---------------------------------------------------------------- queries
constexpr int kQBlock = 128;

template <bool ANY>
__global__ __launch_bounds__(kQBlock) void k_query(DevScene S, const pm_ray* rays, int64_t n, pm_hit* hits,
                                                   int32_t* occ, int* overflow) {
  __shared__ int stack[kStackDepth * kQBlock];
  const int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x;
  if (i >= n) return;
  const pm_ray R = rays[i];
  Ray r;
  ray_prep(r, mk(R.origin), mk(R.direction));
  HitInfo h = traverse<ANY>(S, r, R.tmin, R.tmax, stack + threadIdx.x, kQBlock, overflow);
  if (ANY) {
    occ[i] = h.slot >= 0 ? 1 : 0;
  } else {
    pm_hit o;
    if (h.slot < 0) {
      o.t = INFINITY;
      o.mesh = o.prim = o.tri = -1;
    } else {
      const float4 a = S.tri[3 * h.slot], b = S.tri[3 * h.slot + 1];
      o.t = h.t;
      o.mesh = __float_as_int(a.w);
      o.prim = __float_as_int(b.w);
      o.tri = h.gid;
    }
    hits[i] = o;
  }
}

hipError_t launch_query(pm_scene* sc, const pm_ray* rays, int64_t n, pm_hit* hits, int32_t* occ, bool any,
                        hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (any)
    k_query<true><<<grid_for(n, kQBlock), kQBlock, 0, s>>>(sc->view(), rays, n, hits, occ, sc->overflow.p);
  else
    k_query<false><<<grid_for(n, kQBlock), kQBlock, 0, s>>>(sc->view(), rays, n, hits, occ, sc->overflow.p);
  return hipGetLastError();
}

}  // namespace pmd
