// render.hip — final gather render for gfx950 (stage 2).
//
// Restates simpleRayGen / tracePath / ray_colour (ray-tracer/cuda/deviceCode.cu:
// 25-231) and reflect_or_refract_ray / calculate_refracted / specularBrdf
// (ray-tracer/cuda/shading.h:20-91) as a wavefront pipeline:
//   1. k_paths        per pixel: the camera path; writes per-vertex records
//                     and the caustic query, and EMITS the shadow rays and the
//                     20 final-gather rays per vertex into fixed slots. The
//                     first vertex of each sample has a fixed slot; later ones
//                     take continuation slots (wave-aggregated atomic) linked
//                     by `next`, so no counting pass replays the paths;
//      k_diffuse_rays / k_shadow_rays trace them (lean traversal kernels at
//                     high occupancy), k_direct sums the direct light in the
//                     reference's order.
//   2. compaction of valid queries, k_gather (knn.hip) per query.
//   3. k_resolve      per pixel: replays ray_colour's colour arithmetic in the
//                     reference's order with the gathered radiance, following
//                     each sample's vertex links.
// Gathers never steer control flow, so this is bitwise the megakernel result.
// Reference UB is defined as in SURVEY §5.1-18: per-pixel hit record and the
// diffuse rays' hit records are zero-initialised; a miss keeps the stale record.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>

#include "pm_internal.hpp"

namespace pmd {

constexpr int kRBlock = 128;
constexpr uint32_t VF_MISS = 1u, VF_LAST = 2u;

struct LightR {
  float4 pos;   // xyz, power (float)
  float4 rgb;
};

struct RenderArgs {
  int32_t W, H, spp, depth;
  int32_t caustic_k;   // host side only: neighbours of the caustic gather
  int32_t tile_rank, tile_count, tiles_x, my_tiles;
  v3 cam_pos, d00, du, dv, sky;
  const LightR* lights;
  int32_t nl;
};

struct HitRec {
  v3 hitpoint, normal;
  float4 m0, m1;   // (albedo, diffuse), (specular, transmission, ior, 0)
};

__device__ __forceinline__ bool pixel_of(const RenderArgs& A, int64_t tid, int& px, int& py) {
  const int64_t lt = tid >> 8;
  if (lt >= A.my_tiles) return false;
  const int64_t tile = (int64_t)A.tile_rank + lt * A.tile_count;
  const int ty = (int)(tile / A.tiles_x), tx = (int)(tile % A.tiles_x);
  const int p = (int)(tid & 255);
  px = tx * 16 + (p & 15);
  py = ty * 16 + (p >> 4);
  return px < A.W && py < A.H;
}

// closestHit (deviceCode.cu:233-253)
__device__ __forceinline__ bool trace_closest(const DevScene& S, v3 o, v3 d, float tmin, float tmax, HitRec& hr,
                                              int* st, int* overflow) {
  Ray r;
  ray_prep(r, o, d);
  const HitInfo h = traverse<false>(S, r, tmin, tmax, st, kRBlock, overflow);
  if (h.slot < 0) return false;
  const int mesh = __float_as_int(S.tri[3 * h.slot].w);
  hr.m0 = S.mat[2 * mesh];
  hr.m1 = S.mat[2 * mesh + 1];
  hr.hitpoint = add(o, mulf(d, h.t));
  const v3 n = tri_normal(S, h.slot);
  hr.normal = dot(d, n) < 0.f ? n : neg(n);
  hr.normal = normalize(hr.normal);
  return true;
}

// shading.h:20-55 (Random by value)
__device__ __forceinline__ v3 calculate_refracted(const HitRec& hr, v3 rd, v3 n, uint32_t rng) {
  v3 outward, refracted = {0.f, 0.f, 0.f};
  float ni, R, cosine;
  const float ior = hr.m1.z;
  if (dot(rd, n) > 0.f) {
    outward = neg(n);
    ni = ior;
    cosine = dot(rd, n);
    cosine = sqrtf(1.f - ior * ior * (1.f - cosine * cosine));
  } else {
    outward = n;
    ni = 1.f / ior;
    cosine = -dot(rd, n);
  }
  if (refract_uv(rd, outward, ni, refracted))
    R = schlick(cosine, ior);
  else
    R = 1.f;
  if (lcg_next(rng) < R) return reflect(rd, n);
  return refracted;
}
// shading.h:57-80 (Random by value)
__device__ __forceinline__ v3 reflect_or_refract(const HitRec& hr, v3 rd, v3 n, uint32_t rng, bool& absorbed,
                                                 float& coef) {
  absorbed = false;
  const float r = lcg_next(rng);
  if (r < hr.m1.x) {
    coef = hr.m1.x;
    return reflect(rd, n);
  }
  if (r < hr.m1.x + hr.m1.y) {
    coef = hr.m1.y;
    return calculate_refracted(hr, rd, n, rng);
  }
  coef = 0.f;
  absorbed = true;
  return {0.f, 0.f, 0.f};
}

// deviceCode.cu:112-120: the RNG use of one diffuse sample (direction only)
__device__ __forceinline__ v3 diffuse_direction(v3 normal_at_hit, uint32_t& rng) {
  const v3 n = normalize(normal_at_hit);
  v3 rv, rdir;
  do {
    rv = random_unit_vector(rng);
    rdir = add(n, rv);
  } while (near_zero(rdir));
  return normalize(rdir);
}

__device__ __forceinline__ v3 camera_dir(const RenderArgs& A, int px, int py, uint32_t& rng) {
  const float ex = lcg_next(rng);   // vec2f(rnd(), rnd()) evaluated left to right
  const float ey = lcg_next(rng);
  const float su = ((float)px + ex) / (float)A.W;
  const float sv = ((float)py + ey) / (float)A.H;
  return normalize(add(add(A.d00, smul(su, A.du)), smul(sv, A.dv)));
}

struct PathOut {
  float4* vdirect;    // direct term (or sky colour for a miss)
  float4* vatt;       // attenuation at this vertex
  float4* valb;       // albedo at this vertex
  uint32_t* vflags;
  float4* cq;         // caustic query (hitpoint, diffuse_brdf)
  uint32_t* cvalid;
  float4* gq;         // [20 * v + j] global query (hitpoint, brdf)
  float4* galb;       // [20 * v + j] albedo of the diffuse hit
  uint32_t* gvalid;   // k_paths: diffuse ray emitted; k_diffuse_rays: query valid
  float4* gdir;       // [20 * v + j] diffuse ray direction (origin = cq[v].xyz)
  float4* sray;       // [nl * v + l] shadow ray (direction, tmax); w < 0: not cast
  float4* sterm;      // [nl * v + l] (ldn, inv, bs, 0) of the direct-light term
  uint32_t* svis;     // [nl * v + l] 1 = light visible
  unsigned long long* rays;
  int32_t* next;      // next vertex of the same sample, -1 after the last
  uint32_t* ovf;      // continuation-slot counter (slots nbase + k)
  int64_t nbase;      // first vertex of (thread t, sample s) is slot t * spp + s
  int64_t cap;        // continuation slots available
};

// Vertex slots without a counting pass: the first vertex of (thread t, sample
// s) is slot t * spp + s; a path that continues takes its next slot from the
// continuation area (one atomic per wave and depth step) and links it with
// O.next. Every per-vertex kernel is order-agnostic and k_resolve follows the
// links, so results do not depend on the slot order. (The counting pass replayed
// every camera path once more: ~3.3 ms, mostly the latency chain of the few
// long specular paths.) Threads outside the image mark their base slots empty.
__global__ __launch_bounds__(kRBlock) PM_WAVES_ATTR(PM_PATHS_WAVES) void k_paths(DevScene S, RenderArgs A, PathOut O,
                                                   int* overflow) {
  __shared__ int stack[kStackDepth * kRBlock];
  const int64_t tid = (int64_t)blockIdx.x * kRBlock + threadIdx.x;
  int px, py;
  const bool valid = pixel_of(A, tid, px, py);
  uint32_t nrays = 0;
  if (!valid && (tid >> 8) < A.my_tiles) {
    for (int s = 0; s < A.spp; s++) {
      const int64_t v = tid * A.spp + s;
      O.vflags[v] = VF_MISS | VF_LAST;
      O.cvalid[v] = 0;
      O.next[v] = -1;
#pragma unroll 1
      for (int j = 0; j < kNumDiffuseSamples; j++) O.gvalid[v * kNumDiffuseSamples + j] = 0;
      for (int l = 0; l < A.nl; l++) O.sray[v * A.nl + l] = make_float4(0.f, 0.f, 0.f, -1.f);
    }
  }
  if (valid) {
    int* st = stack + threadIdx.x;
    uint32_t rng = lcg_init((uint32_t)px, (uint32_t)py);
    HitRec hr;
    hr.hitpoint = hr.normal = {0.f, 0.f, 0.f};
    hr.m0 = hr.m1 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < A.spp; s++) {
      int64_t v = tid * A.spp + s;
      v3 ro = A.cam_pos;
      v3 rd = camera_dir(A, px, py, rng);
      v3 att = {1.f, 1.f, 1.f};
      for (int d = 0; d < A.depth; d++) {
        nrays++;
        const bool hit = trace_closest(S, ro, rd, kEPS, kINFTY, hr, st, overflow);
        O.vatt[v] = make_float4(att.x, att.y, att.z, 0.f);
        uint32_t fl = 0;
        if (!hit) {
          fl |= VF_MISS;
          O.vdirect[v] = make_float4(A.sky.x, A.sky.y, A.sky.z, 0.f);
          O.cvalid[v] = 0;
  #pragma unroll 1
          for (int j = 0; j < kNumDiffuseSamples; j++) O.gvalid[(int64_t)v * kNumDiffuseSamples + j] = 0;
          // no shadow rays from a miss (k_shadow_rays / k_direct skip w < 0)
          for (int l = 0; l < A.nl; l++) O.sray[v * A.nl + l] = make_float4(0.f, 0.f, 0.f, -1.f);
        } else {
          const v3 albedo = {hr.m0.x, hr.m0.y, hr.m0.z};
          const float diffuse_brdf = hr.m0.w / kPI;
          // direct light (deviceCode.cu:145-171): the shadow rays are cast by
          // k_shadow_rays; the per-light term is kept so that k_direct sums it
          // in the reference's order with the visibility
          for (int l = 0; l < A.nl; l++) {
            const LightR L = A.lights[l];
            const v3 org = hr.hitpoint;
            v3 ldir = sub(v3{L.pos.x, L.pos.y, L.pos.z}, org);
            const float dist = norm3(ldir);
            ldir = normalize(ldir);
            const float ldn = dot(ldir, hr.normal);
            const int64_t si = v * A.nl + l;
            if (ldn < 0.f) {
              O.sray[si] = make_float4(0.f, 0.f, 0.f, -1.f);
              continue;
            }
            nrays++;
            // specularBrdf (shading.h:82-91)
            const float sb = near_zero(sub(reflect(ldir, hr.normal), rd)) ? hr.m1.x : 0.f;
            const float inv = 1.f / (dist * dist);
            O.sray[si] = make_float4(ldir.x, ldir.y, ldir.z, dist * (1.f - kEPS));
            O.sterm[si] = make_float4(ldn, inv, diffuse_brdf + sb, 0.f);
          }
          O.valb[v] = make_float4(albedo.x, albedo.y, albedo.z, 0.f);
          O.cq[v] = make_float4(hr.hitpoint.x, hr.hitpoint.y, hr.hitpoint.z, diffuse_brdf);
          O.cvalid[v] = 1;
          // the 20 final-gather rays (deviceCode.cu:112-131): directions here (RNG
          // order unchanged), traversal in k_diffuse_rays
          for (int j = 0; j < kNumDiffuseSamples; j++) {
            const int64_t gi = (int64_t)v * kNumDiffuseSamples + j;
            uint32_t cast = 0;
            if (diffuse_brdf > 0.f) {
              const v3 rdir = diffuse_direction(hr.normal, rng);
              O.gdir[gi] = make_float4(rdir.x, rdir.y, rdir.z, 0.f);
              nrays++;
              cast = 1;
            }
            O.gvalid[gi] = cast;
          }
        }
        bool absorbed;
        float coef;
        const v3 od = reflect_or_refract(hr, rd, hr.normal, rng, absorbed, coef);
        const bool last = absorbed || d == A.depth - 1;
        if (last) fl |= VF_LAST;
        O.vflags[v] = fl;
        // continuation slot (wave-aggregated atomic)
        const uint64_t m = __ballot(!last);
        int64_t nv = -1;
        if (m) {
          const int lane = threadIdx.x & 63;
          const int leader = __ffsll((long long)m) - 1;
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(O.ovf, (uint32_t)__popcll(m));
          base = (uint32_t)__shfl((int)base, leader);
          const uint32_t k = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
          if (!last) nv = (int64_t)k < O.cap ? O.nbase + (int64_t)k : -1;   // full: the host reruns
        }
        O.next[v] = (int32_t)nv;
        if (last || nv < 0) break;
        v = nv;
        att = mulv(att, smul(coef, v3{hr.m0.x, hr.m0.y, hr.m0.z}));
        ro = hr.hitpoint;
        rd = od;
      }
    }
  }
  // one atomic per wave (every lane reaches here; lanes outside the image add 0)
  unsigned long long nr = nrays;
  for (int o = 32; o > 0; o >>= 1) nr += (unsigned long long)__shfl_xor((long long)nr, o);
  if ((threadIdx.x & 63) == 0 && nr) atomicAdd(O.rays, nr);
}

// Final-gather rays: closest hit from the vertex; a hit with a diffuse
// material yields a global-map query (hitpoint, brdf) and its albedo
// (closestHit + deviceCode.cu:120-129).
#ifndef PM_RAYS_LDS_PAD
#define PM_RAYS_LDS_PAD 0   // extra LDS bytes per ray-pool workgroup (caps workgroups per CU)
#endif
#ifndef PM_RAYS_WAVES
#define PM_RAYS_WAVES 8   // occupancy target of k_diffuse_rays / k_shadow_rays (0: compiler's choice; 8 with 64-B nodes)
#endif
__global__ __launch_bounds__(kRBlock) PM_WAVES_ATTR(PM_RAYS_WAVES) void k_diffuse_rays(DevScene S, const float4* __restrict__ cq,
                                                          const float4* __restrict__ gdir, int64_t ng,
                                                          uint32_t* __restrict__ gvalid, float4* __restrict__ gq,
                                                          float4* __restrict__ galb, int* overflow) {
  __shared__ int stack[kStackDepth * kRBlock];
  const int64_t gi = (int64_t)blockIdx.x * kRBlock + threadIdx.x;
  if (gi >= ng || !gvalid[gi]) return;
  const float4 c = cq[gi / kNumDiffuseSamples];
  const float4 dd = gdir[gi];
  const v3 o = {c.x, c.y, c.z}, d = {dd.x, dd.y, dd.z};
  Ray r;
  ray_prep(r, o, d);
  const HitInfo h = traverse<false>(S, r, 3 * kEPS, kINFTY, stack + threadIdx.x, kRBlock, overflow);
  uint32_t ok = 0;
  if (h.slot >= 0) {
    const int mesh = __float_as_int(S.tri[3 * h.slot].w);
    const float4 m0 = S.mat[2 * mesh];
    if (m0.w > 0.f) {
      const v3 hp = add(o, mulf(d, h.t));
      gq[gi] = make_float4(hp.x, hp.y, hp.z, m0.w / kPI);
      galb[gi] = make_float4(m0.x, m0.y, m0.z, 0.f);
      ok = 1;
    }
  }
  gvalid[gi] = ok;
}

// Shadow rays (TERMINATE_ON_FIRST_HIT): visible = no hit in (eps, dist (1 - eps)).
__global__ __launch_bounds__(kRBlock) PM_WAVES_ATTR(PM_RAYS_WAVES) void k_shadow_rays(DevScene S, const float4* __restrict__ cq,
                                                         const float4* __restrict__ sray, int nl, int64_t ns,
                                                         uint32_t* __restrict__ svis, int* overflow) {
  __shared__ int stack[kStackDepth * kRBlock];
  const int64_t si = (int64_t)blockIdx.x * kRBlock + threadIdx.x;
  if (si >= ns) return;
  const float4 sr = sray[si];
  if (sr.w < 0.f) return;
  const float4 c = cq[si / nl];
  Ray r;
  ray_prep(r, v3{c.x, c.y, c.z}, v3{sr.x, sr.y, sr.z});
  const HitInfo h = traverse<true>(S, r, kEPS, sr.w, stack + threadIdx.x, kRBlock, overflow);
  svis[si] = h.slot >= 0 ? 0u : 1u;
}

// Ray-pool versions of k_diffuse_rays / k_shadow_rays (PM_RAY_POOL, see
// traverse_pool): same per-ray results.
#ifndef PM_RAY_POOL
#define PM_RAY_POOL 1
#endif
__global__ __launch_bounds__(kRBlock) PM_WAVES_ATTR(PM_RAYS_WAVES) void k_diffuse_rays_pool(
    DevScene S, const float4* __restrict__ cq, const float4* __restrict__ gdir, int64_t ng,
    uint32_t* __restrict__ gvalid, float4* __restrict__ gq, float4* __restrict__ galb, int* overflow, int chunk) {
  __shared__ int stack[kStackDepth * kRBlock];
  __shared__ int lnext;
  if (threadIdx.x == 0) lnext = 0;
  __syncthreads();
  traverse_pool<false>(
      S, stack + threadIdx.x, kRBlock, overflow, ng, chunk, &lnext,
      [&](int64_t gi, Ray& r, float& tmin, float& tmax) {
        if (!gvalid[gi]) return false;
        const float4 c = cq[gi / kNumDiffuseSamples];
        const float4 dd = gdir[gi];
        ray_prep(r, v3{c.x, c.y, c.z}, v3{dd.x, dd.y, dd.z});
        tmin = 3 * kEPS;
        tmax = kINFTY;
        return true;
      },
      [&](int64_t gi, const Ray& r, const HitInfo& h) {
        uint32_t ok = 0;
        if (h.slot >= 0) {
          const int mesh = __float_as_int(S.tri[3 * h.slot].w);
          const float4 m0 = S.mat[2 * mesh];
          if (m0.w > 0.f) {
            const v3 hp = add(r.o, mulf(r.d, h.t));
            gq[gi] = make_float4(hp.x, hp.y, hp.z, m0.w / kPI);
            galb[gi] = make_float4(m0.x, m0.y, m0.z, 0.f);
            ok = 1;
          }
        }
        gvalid[gi] = ok;
      });
}

__global__ __launch_bounds__(kRBlock) PM_WAVES_ATTR(PM_RAYS_WAVES) void k_shadow_rays_pool(
    DevScene S, const float4* __restrict__ cq, const float4* __restrict__ sray, int nl, int64_t ns,
    uint32_t* __restrict__ svis, int* overflow, int chunk) {
  __shared__ int stack[kStackDepth * kRBlock];
  __shared__ int lnext;
  if (threadIdx.x == 0) lnext = 0;
  __syncthreads();
  traverse_pool<true>(
      S, stack + threadIdx.x, kRBlock, overflow, ns, chunk, &lnext,
      [&](int64_t si, Ray& r, float& tmin, float& tmax) {
        const float4 sr = sray[si];
        if (sr.w < 0.f) return false;
        const float4 c = cq[si / nl];
        ray_prep(r, v3{c.x, c.y, c.z}, v3{sr.x, sr.y, sr.z});
        tmin = kEPS;
        tmax = sr.w;
        return true;
      },
      [&](int64_t si, const Ray&, const HitInfo& h) { svis[si] = h.slot >= 0 ? 0u : 1u; });
}

// Direct light of each hit vertex, summed over the lights in order exactly as
// deviceCode.cu:145-171 (vis * power * ldn * inv * brdf * rgb), times albedo.
__global__ __launch_bounds__(256) void k_direct(RenderArgs A, int64_t nv, const uint32_t* __restrict__ vflags,
                                                const float4* __restrict__ valb, const float4* __restrict__ sray,
                                                const float4* __restrict__ sterm, const uint32_t* __restrict__ svis,
                                                float4* __restrict__ vdirect) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nv || (vflags[v] & VF_MISS)) return;
  v3 direct = {0.f, 0.f, 0.f};
  for (int l = 0; l < A.nl; l++) {
    const int64_t si = v * A.nl + l;
    if (sray[si].w < 0.f) continue;
    const LightR L = A.lights[l];
    const float4 t = sterm[si];
    const float vis = svis[si] ? 1.f : 0.f;
    const float pw = L.pos.w;
    const float ldn = t.x, inv = t.y, bs = t.z;
    direct = add(direct, v3{vis * pw * ldn * inv * bs * L.rgb.x, vis * pw * ldn * inv * bs * L.rgb.y,
                            vis * pw * ldn * inv * bs * L.rgb.z});
  }
  const float4 ab = valb[v];
  const v3 dt = mulv(v3{ab.x, ab.y, ab.z}, direct);
  vdirect[v] = make_float4(dt.x, dt.y, dt.z, 0.f);
}

__global__ void k_compact_q(const float4* q, const uint32_t* valid, const uint32_t* idx, int64_t n, float4* dense) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (valid[i]) dense[idx[i]] = q[i];
}

// 30-bit Morton code of each query position (scene bounds) + identity permutation
// Query walk order (PM_QUERY_ORDER): 0 Morton, 1 Hilbert. A 3-D Hilbert key
// (Skilling, "Programming the Hilbert curve", AIP Conf. Proc. 707, 2004: axes
// to transpose, then the transpose's bits interleaved) never jumps between
// distant cells the way Morton order does at its power-of-two seams, so the 64
// queries of a wave and a follower's leaders lie closer together.
// PM_QUERY_BITS per axis (3 x bits of key: the radix sort runs ceil(3 bits / 8)
// passes); queries sharing a cell keep their dense (pixel, sample) order.
#ifndef PM_QUERY_ORDER
#define PM_QUERY_ORDER 1
#endif
#ifndef PM_QUERY_BITS
#define PM_QUERY_BITS 10
#endif
constexpr int kQueryBits = PM_QUERY_BITS;
static_assert(kQueryBits >= 1 && kQueryBits <= 10, "3 x PM_QUERY_BITS must fit the 30-bit spread");
__device__ __forceinline__ uint32_t query_cell(float c, float lo, float inv) {
  constexpr float cells = (float)(1u << kQueryBits);
  return (uint32_t)fminf(fmaxf((c - lo) * inv * cells, 0.0f), cells - 1.0f);
}
__device__ __forceinline__ uint32_t hilbert_key(float x, float y, float z, float3 lo, float3 inv) {
  uint32_t X0 = query_cell(x, lo.x, inv.x), X1 = query_cell(y, lo.y, inv.y), X2 = query_cell(z, lo.z, inv.z);
  // inverse undo (every loop has constant bounds: the coordinates stay in registers)
#pragma unroll
  for (uint32_t Q = 1u << (kQueryBits - 1); Q > 1; Q >>= 1) {
    const uint32_t P = Q - 1;
    // i = 0: X0 & Q ? invert X0 : exchange X0 with itself (a no-op)
    if (X0 & Q) X0 ^= P;
    if (X1 & Q) {
      X0 ^= P;
    } else {
      const uint32_t t = (X0 ^ X1) & P;
      X0 ^= t;
      X1 ^= t;
    }
    if (X2 & Q) {
      X0 ^= P;
    } else {
      const uint32_t t = (X0 ^ X2) & P;
      X0 ^= t;
      X2 ^= t;
    }
  }
  // Gray encode
  X1 ^= X0;
  X2 ^= X1;
  uint32_t t = 0;
#pragma unroll
  for (uint32_t Q = 1u << (kQueryBits - 1); Q > 1; Q >>= 1)
    if (X2 & Q) t ^= Q - 1;
  X0 ^= t;
  X1 ^= t;
  X2 ^= t;
  return (spread3(X0) << 2) | (spread3(X1) << 1) | spread3(X2);
}
__device__ __forceinline__ uint32_t morton_key(float x, float y, float z, float3 lo, float3 inv) {
  return (spread3(query_cell(x, lo.x, inv.x)) << 2) | (spread3(query_cell(y, lo.y, inv.y)) << 1) |
         spread3(query_cell(z, lo.z, inv.z));
}

__global__ void k_query_morton(const float4* q, int64_t n, float3 lo, float3 inv, uint32_t* keys, uint32_t* perm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = q[i];
  keys[i] = PM_QUERY_ORDER == 1 ? hilbert_key(p.x, p.y, p.z, lo, inv) : morton_key(p.x, p.y, p.z, lo, inv);
  perm[i] = (uint32_t)i;
}
// Gathers run in Morton order of the query points (a pure permutation:
// results are bitwise unchanged) so the lanes of a wave walk the same kd-tree
// nodes; k_gather reads and writes through the permutation. The sort needs only
// the scene bounds, so it belongs to render_begin.
struct SortedQueries {
  DevBuf<uint32_t> keys, perm;   // perm: Morton order of the dense queries
  const float4* dense = nullptr;
  int64_t n = 0;
};

static hipError_t sort_queries(const float4* dense, int64_t n, const pm_box& bb, SortedQueries& Q, hipStream_t s) {
  Q.n = n;
  Q.dense = dense;
  if (n <= 0) return hipSuccess;
  Q.keys.alloc(n);
  Q.perm.alloc(n);
  if (!Q.keys.p || !Q.perm.p) return hipErrorOutOfMemory;
  const float3 lo = make_float3(bb.lower.x, bb.lower.y, bb.lower.z);
  const float ex = bb.upper.x - bb.lower.x, ey = bb.upper.y - bb.lower.y, ez = bb.upper.z - bb.lower.z;
  const float3 inv = make_float3(ex > 0.f ? 1.0f / ex : 0.f, ey > 0.f ? 1.0f / ey : 0.f, ez > 0.f ? 1.0f / ez : 0.f);
  k_query_morton<<<grid_for(n, 256), 256, 0, s>>>(dense, n, lo, inv, Q.keys.p, Q.perm.p);
  PM_HIP_TRY(hipGetLastError());
  return radix_sort_pairs(Q.keys.p, Q.perm.p, n, 3 * kQueryBits, s);
}

static hipError_t gather_sorted(const pm_photon_map* m, SortedQueries& Q, float4* res, int tag, hipStream_t s,
                                int k = kKNearest) {
  if (Q.n <= 0) return hipSuccess;
  // lanes take the queries in Morton order and write each result in place
  if (k == kKNearest) PM_HIP_TRY(launch_gather(m, Q.dense, Q.n, res, s, tag, Q.perm.p));
  else PM_HIP_TRY(launch_gather_k(m, Q.dense, Q.n, res, s, k, Q.perm.p));
  return hipSuccess;
}

// Per-vertex colour (deviceCode.cu:173-231's vertex term): the 20 final-gather
// samples of 64 consecutive vertices are read by the whole block (flags,
// albedo, gather result: consecutive lanes, consecutive samples), their
// products staged in LDS, then one lane per vertex sums them in sample order,
// exactly as the per-pixel walk did. (One lane per vertex reading its own
// 80-B flag row and 320-B albedo row, 64 rows apart across the wave, made the
// old single-kernel resolve ~1 ms for ~1.6 GB.)
constexpr int kVcVerts = 64;
constexpr int kVcSamples = kVcVerts * kNumDiffuseSamples;
__global__ __launch_bounds__(256) void k_vertex_colour(PathOut O, int64_t nv, const uint32_t* __restrict__ cidx,
                                                       const float4* __restrict__ cres,
                                                       const uint32_t* __restrict__ gidx,
                                                       const float4* __restrict__ gres, float4* __restrict__ vcol) {
  __shared__ float prod[3][kVcSamples];
  __shared__ uint8_t pvalid[kVcSamples];
  const int64_t v0 = (int64_t)blockIdx.x * kVcVerts;
  const int64_t nvb = nv - v0 < kVcVerts ? nv - v0 : kVcVerts;
  const int64_t ns = nvb * kNumDiffuseSamples;
  for (int i = threadIdx.x; i < kVcSamples; i += blockDim.x) {
    uint32_t ok = 0;
    if (i < ns) {
      const int64_t gi = v0 * kNumDiffuseSamples + i;
      ok = O.gvalid[gi];
      if (ok) {
        const float4 g4 = gres[gidx[gi]];   // valid samples are consecutive in gres
        const float4 al = O.galb[gi];
        const v3 p = mulv(v3{g4.x, g4.y, g4.z}, v3{al.x, al.y, al.z});
        prod[0][i] = p.x;
        prod[1][i] = p.y;
        prod[2][i] = p.z;
      }
    }
    pvalid[i] = (uint8_t)ok;
  }
  __syncthreads();
  const int lv = threadIdx.x;
  if (lv >= nvb) return;
  const int64_t v = v0 + lv;
  const uint32_t fl = O.vflags[v];
  v3 c;
  if (fl & VF_MISS) {
    const float4 sk = O.vdirect[v];
    c = {sk.x, sk.y, sk.z};
  } else {
    const float4 c4 = cres[cidx[v]];
    const v3 caustics = {c4.x, c4.y, c4.z};
    v3 diffuse = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kNumDiffuseSamples; j++) {
      const int i = lv * kNumDiffuseSamples + j;
      if (pvalid[i]) diffuse = add(diffuse, v3{prod[0][i], prod[1][i], prod[2][i]});
    }
    diffuse = divf(diffuse, (float)kNumDiffuseSamples);
    const float4 ab = O.valb[v];
    diffuse = mulv(diffuse, v3{ab.x, ab.y, ab.z});
    const float4 d4 = O.vdirect[v];
    c = {kDiffuseFactor * diffuse.x + kCausticsFactor * caustics.x + kDirectLightFactor * d4.x,
         kDiffuseFactor * diffuse.y + kCausticsFactor * caustics.y + kDirectLightFactor * d4.y,
         kDiffuseFactor * diffuse.z + kCausticsFactor * caustics.z + kDirectLightFactor * d4.z};
  }
  vcol[v] = make_float4(c.x, c.y, c.z, 0.f);
}

// ray_colour's accumulation along each camera path: colour += c_v * att_v.
__global__ __launch_bounds__(256) void k_resolve(RenderArgs A, PathOut O, const float4* __restrict__ vcol,
                                                 uint32_t* rgba, float* rgb) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int px, py;
  if (!pixel_of(A, tid, px, py)) return;
  v3 fc = {0.f, 0.f, 0.f};
  for (int s = 0; s < A.spp && A.depth > 0; s++) {
    v3 colour = {0.f, 0.f, 0.f};
    for (int64_t v = tid * A.spp + s; v >= 0;) {
      const uint32_t fl = O.vflags[v];
      const float4 a4 = O.vatt[v];
      const float4 c4 = vcol[v];
      colour = add(colour, mulv(v3{c4.x, c4.y, c4.z}, v3{a4.x, a4.y, a4.z}));
      if (fl & VF_LAST) break;
      v = O.next[v];
    }
    fc = add(fc, colour);
  }
  fc = mulf(fc, 1.f / (float)A.spp);
  const int y = A.H - py;
  if (y >= A.H) return;   // pixelID.y == 0 writes past the buffer in the reference: dropped
  const int64_t ofs = (int64_t)px + (int64_t)A.W * y;
  rgba[ofs] = make_rgba(fc);
  if (rgb) {
    rgb[3 * ofs] = fc.x;
    rgb[3 * ofs + 1] = fc.y;
    rgb[3 * ofs + 2] = fc.z;
  }
}

}  // namespace pmd

// Everything of a frame's render that does not depend on the photon maps:
// camera paths, shadow / final-gather rays, direct light, compacted and
// Morton-sorted gather queries. Held between pm_render_begin and
// pm_render_finish so that it can overlap the photon trace and kd-tree build
// (on another stream).
struct pm_render_job {
  pmd::RenderArgs A;
  pmd::DevBuf<pmd::LightR> dl;
  int64_t nthreads = 0, NV = 0, NG = 0, NS = 0, nbase = 0, cap = 0;
  pmd::DevBuf<uint32_t> ovf;
  pmd::DevBuf<int32_t> next;
  pmd::DevBuf<float4> vdirect, vatt, valb, cq, gq, galb, gdir, sray, sterm, cdense, gdense, cres, gres;
  pmd::DevBuf<uint32_t> vflags, cvalid, gvalid, cidx, gidx, ctot, gtot, svis;
  pmd::DevBuf<unsigned long long> rays;
  pmd::SortedQueries cs, gs;
  pm_render_stats stats{};
  pm_scene* scene = nullptr;
  bool finished = false;
  hipStream_t begun_on = nullptr;   // render_begin's stream: the job's buffers return to its allocator pool
  int device = 0;                   // begun_on's device
  const pm_photon_map* caustic_map = nullptr;   // set once the caustic gather ran (render_gather_caustic)
};

namespace pmd {

pm_render_job* render_job_new(pm_scene* sc, hipStream_t s) {
  pm_render_job* J = new (std::nothrow) pm_render_job();
  if (J) {
    J->scene = sc;
    J->begun_on = s;
    J->device = stream_device(s);
  }
  return J;
}
// The job's buffers go back to the pool of the stream they were taken from:
// freed under the destroying thread's stream (none outside an entry point),
// a caller that begins every frame's job on a side stream would never get them
// back there (each begin a fresh hipMalloc, until memory runs out).
void render_job_delete(pm_render_job* J) {
  if (!J) return;
  AllocStream pool(J->begun_on, J->device);
  delete J;
}
const pm_render_stats& render_job_stats(const pm_render_job* J) { return J->stats; }
pm_scene* render_job_scene(const pm_render_job* J) { return J->scene; }
int render_job_device(const pm_render_job* J) { return J->device; }
// The job's dense gather queries (pos, brdf) and results (radiance, 0) of one
// map: which 0 = global (final gather), 1 = caustic.
void render_job_queries(const pm_render_job* J, int which, const float4** q, const float4** res, int64_t* n) {
  const pmd::SortedQueries& Q = which == 0 ? J->gs : J->cs;
  *q = Q.n > 0 ? Q.dense : nullptr;
  *res = Q.n > 0 ? (which == 0 ? J->gres.p : J->cres.p) : nullptr;
  *n = Q.n;
}
bool render_job_finished(const pm_render_job* J) { return J->finished; }
void render_job_mark_finished(pm_render_job* J) { J->finished = true; }
const pm_photon_map* render_job_caustic_map(const pm_render_job* J) { return J->caustic_map; }

hipError_t render_begin(pm_scene* sc, const pm_render_params* P, const pm_light* lights, int nl, pm_render_job* J,
                        hipStream_t s) {
  RenderArgs& A = J->A;
  A.W = P->width;
  A.H = P->height;
  A.spp = P->samples_per_pixel;
  A.depth = P->max_depth;
  A.caustic_k = P->caustic_k > 0 ? P->caustic_k : kKNearest;
  A.tile_rank = P->tile_count > 1 ? P->tile_rank : 0;
  A.tile_count = P->tile_count > 1 ? P->tile_count : 1;
  A.tiles_x = (A.W + 15) / 16;
  const int tiles_y = (A.H + 15) / 16;
  const int64_t ntiles = (int64_t)A.tiles_x * tiles_y;
  A.my_tiles = (int32_t)(ntiles > A.tile_rank ? (ntiles - A.tile_rank + A.tile_count - 1) / A.tile_count : 0);
  A.cam_pos = mk(P->camera.pos);
  A.d00 = mk(P->camera.dir_00);
  A.du = mk(P->camera.dir_du);
  A.dv = mk(P->camera.dir_dv);
  A.sky = mk(P->sky_colour);
  A.nl = nl;
  std::vector<LightR> lh(nl > 0 ? nl : 1);
  for (int i = 0; i < nl; i++) {
    lh[i].pos = make_float4(lights[i].pos.x, lights[i].pos.y, lights[i].pos.z, (float)lights[i].power);
    lh[i].rgb = make_float4(lights[i].rgb.x, lights[i].rgb.y, lights[i].rgb.z, 0.f);
  }
  J->dl.alloc(lh.size());
  if (!J->dl.p) return hipErrorOutOfMemory;
  PM_HIP_TRY(hipMemcpyAsync(J->dl.p, lh.data(), sizeof(LightR) * lh.size(), hipMemcpyHostToDevice, s));
  A.lights = J->dl.p;
  const int64_t nthreads = (int64_t)A.my_tiles * 256;
  J->nthreads = nthreads;
  if (nthreads == 0) return hipStreamSynchronize(s);
  const DevScene S = sc->view();
  const int64_t nbase = A.depth > 0 ? nthreads * A.spp : 0;
  J->nbase = nbase;
  J->ovf.alloc(1);
  J->rays.alloc(1);
  J->ctot.alloc(1);
  J->gtot.alloc(1);
  if (!J->ovf.p || !J->rays.p || !J->ctot.p || !J->gtot.p) return hipErrorOutOfMemory;
  // continuation slots: a guess first (one per sample, or the last frame's
  // need); if it was short, k_paths reruns with a larger area
  static thread_local int64_t last_need = 0;
  int64_t cap = std::max<int64_t>(std::max<int64_t>(nbase, last_need + last_need / 8), 4096);
#if PM_CHECK_VARIANT
  cap = 1;   // check variant: the first guess is always short, so every render exercises the rerun
#endif
  uint32_t used = 0;
  for (int attempt = 0;; attempt++) {
    const int64_t NV = nbase + cap, NG = NV * kNumDiffuseSamples, NS = NV * nl;
    for (auto* b : {&J->vdirect, &J->vatt, &J->valb, &J->cq}) b->alloc(NV);
    for (auto* b : {&J->gq, &J->galb, &J->gdir}) b->alloc(NG);
    for (auto* b : {&J->vflags, &J->cvalid, &J->cidx}) b->alloc(NV);
    for (auto* b : {&J->gvalid, &J->gidx}) b->alloc(NG);
    J->next.alloc(NV);
    J->sray.alloc(NS);
    J->sterm.alloc(NS);
    J->svis.alloc(NS);
    if (NV > 0 && (!J->vdirect.p || !J->vatt.p || !J->valb.p || !J->cq.p || !J->gq.p || !J->galb.p ||
                   !J->vflags.p || !J->cvalid.p || !J->gvalid.p || !J->cidx.p || !J->gidx.p || !J->gdir.p ||
                   !J->next.p))
      return hipErrorOutOfMemory;
    if (NS > 0 && (!J->sray.p || !J->sterm.p || !J->svis.p)) return hipErrorOutOfMemory;
    if (nbase == 0) break;
    PathOut O{J->vdirect.p, J->vatt.p, J->valb.p, J->vflags.p, J->cq.p, J->cvalid.p, J->gq.p, J->galb.p,
              J->gvalid.p,  J->gdir.p, J->sray.p, J->sterm.p, J->svis.p, J->rays.p,  J->next.p, J->ovf.p,
              nbase,        cap};
    PhaseTimer tm(PH_PATHS, s);
    PM_HIP_TRY(hipMemsetAsync(J->rays.p, 0, 8, s));
    PM_HIP_TRY(hipMemsetAsync(J->ovf.p, 0, 4, s));
    k_paths<<<grid_for(nthreads, kRBlock), kRBlock, 0, s>>>(S, A, O, sc->overflow.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(hipMemcpyAsync(&used, J->ovf.p, 4, hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
    if ((int64_t)used <= cap) break;
    // paths cut short by a full area stopped requesting slots, so `used` is a
    // lower bound: grow geometrically, then fall back to the worst case
    const int64_t worst = nbase * std::max(A.depth - 1, 1);
    if (cap >= worst) return hipErrorUnknown;   // cannot happen: every path fits
    cap = attempt < 3 ? std::min(worst, std::max<int64_t>(2 * (int64_t)used, 4 * cap)) : worst;
  }
  last_need = used;
  J->cap = cap;
  const int64_t NV = nbase + (int64_t)used, NG = NV * kNumDiffuseSamples, NS = NV * nl;
  J->NV = NV;
  J->NG = NG;
  J->NS = NS;
  uint32_t NC = 0, NGv = 0;
  {
    PhaseTimer tm(PH_PATHS, s);
    if (NG > 0) {
      if (PM_RAY_POOL)
        k_diffuse_rays_pool<<<grid_for(NG, pool_chunk(NG, kRBlock)), kRBlock, PM_RAYS_LDS_PAD, s>>>(
            S, J->cq.p, J->gdir.p, NG, J->gvalid.p, J->gq.p, J->galb.p, sc->overflow.p, pool_chunk(NG, kRBlock));
      else
        k_diffuse_rays<<<grid_for(NG, kRBlock), kRBlock, 0, s>>>(S, J->cq.p, J->gdir.p, NG, J->gvalid.p, J->gq.p,
                                                                 J->galb.p, sc->overflow.p);
      PM_HIP_TRY(hipGetLastError());
    }
    if (NS > 0) {
      if (PM_RAY_POOL)
        k_shadow_rays_pool<<<grid_for(NS, pool_chunk(NS, kRBlock)), kRBlock, PM_RAYS_LDS_PAD, s>>>(
            S, J->cq.p, J->sray.p, nl, NS, J->svis.p, sc->overflow.p, pool_chunk(NS, kRBlock));
      else
        k_shadow_rays<<<grid_for(NS, kRBlock), kRBlock, 0, s>>>(S, J->cq.p, J->sray.p, nl, NS, J->svis.p,
                                                                sc->overflow.p);
      PM_HIP_TRY(hipGetLastError());
    }
    if (NV > 0) {
      k_direct<<<grid_for(NV, 256), 256, 0, s>>>(A, NV, J->vflags.p, J->valb.p, J->sray.p, J->sterm.p, J->svis.p,
                                                 J->vdirect.p);
      PM_HIP_TRY(hipGetLastError());
    }
    PM_HIP_TRY(exclusive_scan_u32(J->cvalid.p, J->cidx.p, NV, J->ctot.p, s));
    PM_HIP_TRY(exclusive_scan_u32(J->gvalid.p, J->gidx.p, NG, J->gtot.p, s));
    PM_HIP_TRY(hipMemcpyAsync(&NC, J->ctot.p, 4, hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipMemcpyAsync(&NGv, J->gtot.p, 4, hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
  }
  J->cdense.alloc(NC);
  J->gdense.alloc(NGv);
  J->cres.alloc(NC);
  J->gres.alloc(NGv);
  if ((NC && (!J->cdense.p || !J->cres.p)) || (NGv && (!J->gdense.p || !J->gres.p))) return hipErrorOutOfMemory;
  {
    PhaseTimer tm(PH_PATHS, s);
    if (NV) {
      k_compact_q<<<grid_for(NV, 256), 256, 0, s>>>(J->cq.p, J->cvalid.p, J->cidx.p, NV, J->cdense.p);
      PM_HIP_TRY(hipGetLastError());
      k_compact_q<<<grid_for(NG, 256), 256, 0, s>>>(J->gq.p, J->gvalid.p, J->gidx.p, NG, J->gdense.p);
      PM_HIP_TRY(hipGetLastError());
    }
    PM_HIP_TRY(sort_queries(J->cdense.p, NC, sc->bounds, J->cs, s));
    PM_HIP_TRY(sort_queries(J->gdense.p, NGv, sc->bounds, J->gs, s));
  }
  unsigned long long nr = 0;
  PM_HIP_TRY(hipMemcpyAsync(&nr, J->rays.p, 8, hipMemcpyDeviceToHost, s));
  PM_HIP_TRY(hipStreamSynchronize(s));
  int64_t px = 0;
  for (int64_t t = 0; t < A.my_tiles; t++) {
    const int64_t tile = A.tile_rank + t * A.tile_count;
    const int ty = (int)(tile / A.tiles_x), tx = (int)(tile % A.tiles_x);
    px += (int64_t)std::min(16, A.W - tx * 16) * std::min(16, A.H - ty * 16);
  }
  J->stats.pixels = px;
  J->stats.path_vertices = (A.depth > 0 ? px * A.spp : 0) + (int64_t)used;
  J->stats.caustic_queries = NC;
  J->stats.global_queries = NGv;
  J->stats.rays = (int64_t)nr;
  return hipSuccess;
}

// The caustic gather alone, ahead of render_finish: it needs only the caustic
// map, so a frame can run it beside the global map's trace and build.
hipError_t render_gather_caustic(pm_render_job* J, const pm_photon_map* cmap, hipStream_t s) {
  if (J->nthreads > 0) {
    PM_HIP_TRY(gather_sorted(cmap, J->cs, J->cres.p, 0, s, J->A.caustic_k));
    PM_HIP_TRY(hipStreamSynchronize(s));
  }
  J->caustic_map = cmap;
  return hipSuccess;
}

hipError_t render_finish(pm_render_job* J, const pm_photon_map* gmap, const pm_photon_map* cmap, uint32_t* rgba,
                         float* rgb, hipStream_t s) {
  if (J->nthreads == 0) return hipSuccess;
  {
    // The two gathers are independent: unless render_gather_caustic already
    // ran it, the caustic one runs on a side stream beside the global one. The
    // global map's leader launch (every 16th query) ends with its slowest
    // waves while most of the GPU idles -- on the Cornell box (config 2) 231k
    // leaders, fewer waves than the GPU holds, and a few leaders walk
    // thousands of nodes -- and the caustic gather fills it.
    // The global gather is enqueued first: a k != 50 caustic gather
    // synchronises its own stream before it returns.
    // (The global gather's own time comes from events read after the final
    // synchronisation: a host wait between the two would serialise them.)
    // The side stream is the device's process-wide one, so the pool of the
    // side gather's temporaries persists from frame to frame.
    PhaseTimer tm(PH_GATHER, s);
    const bool side = J->caustic_map == nullptr;
    hipStream_t side_s = side ? side_stream(stream_device(s)) : nullptr;
    if (side && !side_s) return hipErrorOutOfMemory;
    hipEvent_t ready = nullptr, done = nullptr, g0 = nullptr, g1 = nullptr;
    hipError_t e = hipEventCreate(&g0);
    if (e == hipSuccess) e = hipEventCreate(&g1);
    if (side) {
      if (e == hipSuccess) e = hipEventCreateWithFlags(&ready, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventRecord(ready, s);
      if (e == hipSuccess) e = hipStreamWaitEvent(side_s, ready, 0);
    }
    if (e == hipSuccess) e = hipEventRecord(g0, s);
    if (e == hipSuccess) e = gather_sorted(gmap, J->gs, J->gres.p, 1, s);
    if (e == hipSuccess) e = hipEventRecord(g1, s);
    if (side) {
      if (e == hipSuccess) {
        AllocStream side_pool(side_s);   // the side gather's temporaries belong to its stream
        e = gather_sorted(cmap, J->cs, J->cres.p, 0, side_s, J->A.caustic_k);
      }
      if (e == hipSuccess) e = hipEventRecord(done, side_s);
      if (e == hipSuccess) e = hipStreamWaitEvent(s, done, 0);
    }
    if (e == hipSuccess) e = hipEventSynchronize(g1);
    float ms = 0.f;
    if (e == hipSuccess && hipEventElapsedTime(&ms, g0, g1) == hipSuccess) record_phase_us(PH_GATHER_GLOBAL, ms * 1e3);
    if (e != hipSuccess && side) (void)hipStreamSynchronize(side_s);   // no side work outlives a failed call
    for (hipEvent_t ev : {ready, done, g0, g1})
      if (ev) (void)hipEventDestroy(ev);
    PM_HIP_TRY(e);
  }
  PathOut O{J->vdirect.p, J->vatt.p, J->valb.p, J->vflags.p, J->cq.p, J->cvalid.p, J->gq.p, J->galb.p,
            J->gvalid.p,  J->gdir.p, J->sray.p, J->sterm.p, J->svis.p, J->rays.p,  J->next.p, J->ovf.p,
            J->nbase,     J->cap};
  {
    PhaseTimer tm(PH_RESOLVE, s);
    DevBuf<float4> vcol(J->NV);
    if (J->NV > 0 && !vcol.p) return hipErrorOutOfMemory;
    if (J->NV > 0) {
      k_vertex_colour<<<(int)((J->NV + kVcVerts - 1) / kVcVerts), 256, 0, s>>>(O, J->NV, J->cidx.p, J->cres.p,
                                                                               J->gidx.p, J->gres.p, vcol.p);
      PM_HIP_TRY(hipGetLastError());
    }
    k_resolve<<<grid_for(J->nthreads, 256), 256, 0, s>>>(J->A, O, vcol.p, rgba, rgb);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(hipStreamSynchronize(s));   // vcol is freed on scope exit
  }
  return hipStreamSynchronize(s);
}

}  // namespace pmd
