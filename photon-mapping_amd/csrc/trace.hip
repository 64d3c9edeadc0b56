// trace.hip — photon emission and bounce (stage 1) for gfx950.
//
// One fused launch over every light's photons replaces the per-light
// owlRayGenLaunch2D loop (photon-mapping/src/hostCode.cu:72-90, :112-138):
// global photon index g = light offset + id, RNG seeded with the per-light id
// exactly as pointLightRayGen's prd.random.init(id.x, 0) (deviceCode.cu:59).
// The bounce loop follows shootPhoton / shootCausticsPhoton (:25-52), the
// closest-hit program triangleMeshClosestHit (:113-131) and the scatter
// functions (:74-111). The atomicAdd deposit (:10-17) is replaced by
// deterministic slots: deposit k of photon i lands in slots[k][i] (coalesced
// across the wave), then a scan + compaction writes the canonical
// (g, bounce) order.
#include <algorithm>
#include <cstdlib>
#include <utility>

#include "pm_internal.hpp"

namespace pmd {

constexpr int kTBlock = 128;

// Each lane traces several photons back to back (i, i + stride, ...): when a
// photon's path ends the lane immediately starts its next photon, so a wave
// is not held by its longest path (path lengths range over 1..max_depth).
constexpr int kPhotonsPerLane = 8;

__global__ __launch_bounds__(kTBlock) PM_WAVES_ATTR(PM_TRACE_WAVES) void k_trace_photons(DevScene S, const LightDev* lights, const int64_t* loff,
                                                           int nl, int64_t g_lo, int64_t np, int maxd,
                                                           int caustic, pm_photon* slots, uint32_t* cnt,
                                                           int* overflow) {
  __shared__ int stack[kStackDepth * kTBlock];
  const int64_t stride = (int64_t)gridDim.x * kTBlock;
  int64_t i = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
  int* st = stack + threadIdx.x;
  const float tmin = kEPS;
  bool alive = false;
  uint32_t rng = 0, n = 0;
  int b = 0;
  v3 color = {0.f, 0.f, 0.f}, o = {0.f, 0.f, 0.f}, d = {0.f, 0.f, 0.f};
  for (;;) {
    if (!alive) {
      if (i >= np) break;
      // pointLightRayGen (photon-mapping/cuda/deviceCode.cu:54-72)
      const int64_t g = g_lo + i;
      int l = 0;
      while (l < nl - 1 && g >= loff[l + 1]) l++;
      const uint32_t id = (uint32_t)(g - loff[l]);
      const LightDev L = lights[l];
      rng = lcg_init(id, 0u);
      color = {L.rgb.x, L.rgb.y, L.rgb.z};
      emit_photon(L.rgb.w, v3{L.pos.x, L.pos.y, L.pos.z}, v3{L.nrm.x, L.nrm.y, L.nrm.z}, L.nrm.w, rng, o, d);
      n = 0;
      b = 0;
      alive = true;
    }
    // one owl::traceRay + triangleMeshClosestHit (deviceCode.cu:113-131)
    Ray r;
    ray_prep(r, o, d);
    const HitInfo h = traverse<false>(S, r, tmin, kPhotonTmax, st, kTBlock, overflow);
    int ev;
    v3 so = {0.f, 0.f, 0.f}, sd = {0.f, 0.f, 0.f}, sc = {0.f, 0.f, 0.f};
    if (h.slot < 0) {
      ev = EV_MISS;
    } else {
      const int mesh = __float_as_int(S.tri[3 * h.slot].w);
      const float4 m0 = S.mat[2 * mesh], m1 = S.mat[2 * mesh + 1];
      const float pd = m0.w;
      const float ps = m1.x + pd;
      const float pt = m1.y + ps;
      const float rp = lcg_next(rng);
      const v3 hp = add(o, smul(h.t, d));
      const v3 albedo = {m0.x, m0.y, m0.z};
      if (rp < pd) {
        ev = EV_DIFFUSE;
        so = hp;
        sd = cosine_sample_hemisphere(tri_normal(S, h.slot), rng);
        sc = mulv(albedo, color);
      } else if (rp < ps) {
        ev = EV_SPECULAR;
        so = hp;
        sd = reflect(d, tri_normal(S, h.slot));
        sc = mulv(albedo, color);
      } else if (rp < pt) {
        ev = EV_REFRACT;
        so = hp;
        sd = refract_ior(d, tri_normal(S, h.slot), m1.z);
        sc = mulv(albedo, color);
      } else {
        ev = EV_ABSORBED;
      }
    }
    // shootPhoton / shootCausticsPhoton deposit + continuation (deviceCode.cu:25-52)
    if (b > 0 && ev == EV_DIFFUSE) {
      pm_photon p;
      p.pos = {so.x, so.y, so.z};
      p.dir = {sd.x, sd.y, sd.z};
      p.power = 0;
      p.color = {color.x, color.y, color.z};
      slots[(int64_t)n * np + i] = p;
      n++;
    }
    const bool cont = caustic ? ((ev & (EV_SPECULAR | EV_REFRACT)) != 0) : (ev == EV_DIFFUSE);
    b++;
    if (!cont || b >= maxd) {
      cnt[i] = n;
      alive = false;
      i += stride;
    } else {
      o = so;
      d = sd;
      color = sc;
    }
  }
}

// ------------------------------------------------------------------ wavefront
// The same photon paths as k_trace_photons, split per bounce into a lean
// closest-hit kernel (k_ph_trace: traversal only, high occupancy) and a shading
// kernel (k_ph_shade: event, deposit, continuation). Surviving rays are
// appended to the next bounce's list with one atomic per wave; deposits go to
// slots[n][photon] exactly as in the fused kernel, so the output does not
// depend on the order in which rays are processed.
struct PhotonRay {   // 48 B
  float4 o;          // origin, rng state (bits)
  float4 d;          // direction, photon index (bits)
  float4 c;          // colour, (deposits << 8 | bounce) (bits)
};

__global__ __launch_bounds__(256) void k_ph_gen(const LightDev* __restrict__ lights, const int64_t* __restrict__ loff,
                                                int nl, int64_t g_lo, int64_t np, PhotonRay* __restrict__ rays) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  // pointLightRayGen (photon-mapping/cuda/deviceCode.cu:54-72)
  const int64_t g = g_lo + i;
  int l = 0;
  while (l < nl - 1 && g >= loff[l + 1]) l++;
  const uint32_t id = (uint32_t)(g - loff[l]);
  const LightDev L = lights[l];
  uint32_t rng = lcg_init(id, 0u);
  v3 o, d;
  emit_photon(L.rgb.w, v3{L.pos.x, L.pos.y, L.pos.z}, v3{L.nrm.x, L.nrm.y, L.nrm.z}, L.nrm.w, rng, o, d);
  PhotonRay r;
  r.o = make_float4(o.x, o.y, o.z, __uint_as_float(rng));
  r.d = make_float4(d.x, d.y, d.z, __uint_as_float((uint32_t)i));
  r.c = make_float4(L.rgb.x, L.rgb.y, L.rgb.z, __uint_as_float(0u));
  rays[i] = r;
}

__global__ __launch_bounds__(kTBlock) void k_ph_trace(DevScene S, const PhotonRay* __restrict__ rays, int64_t n,
                                                      float2* __restrict__ hits, int* overflow) {
  __shared__ int stack[kStackDepth * kTBlock];
  const int64_t i = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
  if (i >= n) return;
  const float4 o = rays[i].o, d = rays[i].d;
  Ray r;
  ray_prep(r, v3{o.x, o.y, o.z}, v3{d.x, d.y, d.z});
  const HitInfo h = traverse<false>(S, r, kEPS, kPhotonTmax, stack + threadIdx.x, kTBlock, overflow);
  hits[i] = make_float2(h.t, __int_as_float(h.slot));
}

// PM_RAY_POOL (build knob, default on): the bounce rays go through the chunked
// ray pool (traverse_pool) instead of one ray per lane.
#ifndef PM_RAY_POOL
#define PM_RAY_POOL 1
#endif
#ifndef PM_TPOOL_WAVES
#define PM_TPOOL_WAVES 0   // occupancy target of k_ph_trace_pool (0: compiler's choice)
#endif
__global__ __launch_bounds__(kTBlock) PM_WAVES_ATTR(PM_TPOOL_WAVES) void k_ph_trace_pool(DevScene S, const PhotonRay* __restrict__ rays, int64_t n,
                                                           float2* __restrict__ hits, int* overflow, int chunk) {
  __shared__ int stack[kStackDepth * kTBlock];
  __shared__ int lnext;
  if (threadIdx.x == 0) lnext = 0;
  __syncthreads();
  traverse_pool<false>(
      S, stack + threadIdx.x, kTBlock, overflow, n, chunk, &lnext,
      [&](int64_t i, Ray& r, float& tmin, float& tmax) {
        const float4 o = rays[i].o, d = rays[i].d;
        ray_prep(r, v3{o.x, o.y, o.z}, v3{d.x, d.y, d.z});
        tmin = kEPS;
        tmax = kPhotonTmax;
        return true;
      },
      [&](int64_t i, const Ray&, const HitInfo& h) { hits[i] = make_float2(h.t, __int_as_float(h.slot)); });
}

// Surviving rays are appended with ONE atomic per 1024-thread block (a
// same-address atomic per wave serialised at one L2 channel: ~2/3 of the
// kernel). With `keys`, the next bounce's sort key (top `mbits` of the origin's
// Morton code) is written beside the ray.
constexpr int kShadeBlock = 1024;

__global__ __launch_bounds__(kShadeBlock) void k_ph_shade(DevScene S, const PhotonRay* __restrict__ in,
                                                          int64_t n_in, const float2* __restrict__ hits,
                                                          PhotonRay* __restrict__ out,
                                                          uint32_t* __restrict__ count_out, int64_t np, int maxd,
                                                          int caustic, pm_photon* __restrict__ slots,
                                                          uint32_t* __restrict__ cnt, uint32_t* __restrict__ keys,
                                                          float3 klo, float3 kinv, int mbits) {
  __shared__ uint32_t wcount[kShadeBlock / 64];
  __shared__ uint32_t block_base;
  const int64_t i = (int64_t)blockIdx.x * kShadeBlock + threadIdx.x;
  bool keep = false;
  PhotonRay nr;
  if (i < n_in) {
    const PhotonRay pr = in[i];
    const float2 hh = hits[i];
    const int slot = __float_as_int(hh.y);
    uint32_t rng = __float_as_uint(pr.o.w);
    const uint32_t pi = __float_as_uint(pr.d.w);
    const uint32_t nb = __float_as_uint(pr.c.w);
    uint32_t n = nb >> 8;
    const int b = (int)(nb & 0xFF);
    const v3 o = {pr.o.x, pr.o.y, pr.o.z}, d = {pr.d.x, pr.d.y, pr.d.z}, color = {pr.c.x, pr.c.y, pr.c.z};
    int ev;
    v3 so = {0.f, 0.f, 0.f}, sd = {0.f, 0.f, 0.f}, sc = {0.f, 0.f, 0.f};
    // triangleMeshClosestHit (deviceCode.cu:113-131)
    if (slot < 0) {
      ev = EV_MISS;
    } else {
      const int mesh = __float_as_int(S.tri[3 * slot].w);
      const float4 m0 = S.mat[2 * mesh], m1 = S.mat[2 * mesh + 1];
      const float pd = m0.w;
      const float ps = m1.x + pd;
      const float pt = m1.y + ps;
      const float rp = lcg_next(rng);
      const v3 hp = add(o, smul(hh.x, d));
      const v3 albedo = {m0.x, m0.y, m0.z};
      if (rp < pd) {
        ev = EV_DIFFUSE;
        so = hp;
        sd = cosine_sample_hemisphere(tri_normal(S, slot), rng);
        sc = mulv(albedo, color);
      } else if (rp < ps) {
        ev = EV_SPECULAR;
        so = hp;
        sd = reflect(d, tri_normal(S, slot));
        sc = mulv(albedo, color);
      } else if (rp < pt) {
        ev = EV_REFRACT;
        so = hp;
        sd = refract_ior(d, tri_normal(S, slot), m1.z);
        sc = mulv(albedo, color);
      } else {
        ev = EV_ABSORBED;
      }
    }
    // shootPhoton / shootCausticsPhoton (deviceCode.cu:25-52)
    if (b > 0 && ev == EV_DIFFUSE) {
      pm_photon p;
      p.pos = {so.x, so.y, so.z};
      p.dir = {sd.x, sd.y, sd.z};
      p.power = 0;
      p.color = {color.x, color.y, color.z};
      slots[(int64_t)n * np + pi] = p;
      n++;
    }
    const bool cont = caustic ? ((ev & (EV_SPECULAR | EV_REFRACT)) != 0) : (ev == EV_DIFFUSE);
    if (!cont || b + 1 >= maxd) {
      cnt[pi] = n;
    } else {
      keep = true;
      nr.o = make_float4(so.x, so.y, so.z, __uint_as_float(rng));
      nr.d = make_float4(sd.x, sd.y, sd.z, __uint_as_float(pi));
      nr.c = make_float4(sc.x, sc.y, sc.z, __uint_as_float((n << 8) | (uint32_t)(b + 1)));
    }
  }
  // block-aggregated append
  const uint64_t m = __ballot(keep);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wcount[wave] = (uint32_t)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kShadeBlock / 64; w++) tot += wcount[w];
    block_base = tot ? atomicAdd(count_out, tot) : 0u;
  }
  __syncthreads();
  if (!keep) return;
  uint32_t off = block_base;
  for (int w = 0; w < wave; w++) off += wcount[w];
  const uint32_t dst = off + (uint32_t)__popcll(m & ((1ull << lane) - 1));
  out[dst] = nr;
  if (keys) keys[dst] = morton30(nr.o.x, nr.o.y, nr.o.z, klo, kinv) >> (30 - mbits);
}

// Bounce rays reordered by the Morton code of their origin (PM_TRACE_SORT,
// default on): neighbouring lanes then start in the same BVH region. The order
// of rays never changes a result (deposits go to slots[n][photon]).
__global__ void k_iota(uint32_t* __restrict__ perm, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) perm[i] = (uint32_t)i;
}

__global__ void k_ray_permute(const PhotonRay* __restrict__ src, const uint32_t* __restrict__ perm, int64_t n,
                              PhotonRay* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src[perm[i]];
}

hipError_t launch_trace_wavefront(pm_scene* sc, const LightDev* d_lights, const int64_t* d_loff, int nl,
                                  int64_t g_lo, int64_t np, int maxd, int caustic, pm_photon* slots, uint32_t* cnt,
                                  hipStream_t s) {
  // PM_TRACE_SORT=1: Morton-sort each bounce's rays by origin. Config 3 (trace ms), before the
  // chunked ray pool: unsorted 57.8, 30 bits 55.6, 24 bits 54.9, 16 bits 54.6 (two radix passes),
  // 21 bits + direction octant 54.6. With the pool the sort no longer pays: unsorted 29.5, 16 bits
  // 31.2, 24 bits 32.2, 8 bits 32.3, so it is off by default.
  const char* senv = std::getenv("PM_TRACE_SORT");
  const bool sort_rays = senv && std::atoi(senv) != 0;
  const char* benv = std::getenv("PM_TRACE_SORT_BITS");
  const int mbits = benv ? std::min(30, std::max(8, std::atoi(benv))) : 16;
  DevBuf<PhotonRay> ra(np), rb(np);
  DevBuf<float2> hits(np);
  DevBuf<uint32_t> counts(1), keys, perm;
  if (!ra.p || !rb.p || !hits.p || !counts.p) return hipErrorOutOfMemory;
  if (sort_rays) {
    keys.alloc(np);
    perm.alloc(np);
    if (!keys.p || !perm.p) return hipErrorOutOfMemory;
  }
  const pm_box& bb = sc->bounds;
  const float3 lo = make_float3(bb.lower.x, bb.lower.y, bb.lower.z);
  const float ex = bb.upper.x - bb.lower.x, ey = bb.upper.y - bb.lower.y, ez = bb.upper.z - bb.lower.z;
  const float3 inv = make_float3(ex > 0.f ? 1.0f / ex : 0.f, ey > 0.f ? 1.0f / ey : 0.f, ez > 0.f ? 1.0f / ez : 0.f);
  k_ph_gen<<<grid_for(np, 256), 256, 0, s>>>(d_lights, d_loff, nl, g_lo, np, ra.p);
  PM_HIP_TRY(hipGetLastError());
  PhotonRay *cur = ra.p, *nxt = rb.p;
  int64_t live = np;
  for (int b = 0; b < maxd && live > 0; b++) {
    const bool last = b + 1 >= maxd;
    const bool sort_next = sort_rays && !last;
    PM_HIP_TRY(hipMemsetAsync(counts.p, 0, sizeof(uint32_t), s));
    if (PM_RAY_POOL)
      k_ph_trace_pool<<<grid_for(live, pool_chunk(live, kTBlock)), kTBlock, 0, s>>>(sc->view(), cur, live, hits.p,
                                                                                    sc->overflow.p, pool_chunk(live, kTBlock));
    else
      k_ph_trace<<<grid_for(live, kTBlock), kTBlock, 0, s>>>(sc->view(), cur, live, hits.p, sc->overflow.p);
    PM_HIP_TRY(hipGetLastError());
    k_ph_shade<<<grid_for(live, kShadeBlock), kShadeBlock, 0, s>>>(sc->view(), cur, live, hits.p, nxt, counts.p, np,
                                                                   maxd, caustic, slots, cnt,
                                                                   sort_next ? keys.p : nullptr, lo, inv, mbits);
    PM_HIP_TRY(hipGetLastError());
    if (last) break;
    uint32_t nl_host = 0;
    PM_HIP_TRY(hipMemcpyAsync(&nl_host, counts.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PM_HIP_TRY(hipStreamSynchronize(s));
    live = nl_host;
    if (sort_next && live > 1) {
      k_iota<<<grid_for(live, 256), 256, 0, s>>>(perm.p, live);
      PM_HIP_TRY(hipGetLastError());
      PM_HIP_TRY(radix_sort_pairs(keys.p, perm.p, live, mbits, s));
      // the input rays of this bounce are dead: sorted rays go there
      k_ray_permute<<<grid_for(live, 256), 256, 0, s>>>(nxt, perm.p, live, cur);
      PM_HIP_TRY(hipGetLastError());
    } else {
      std::swap(cur, nxt);
    }
  }
  // keep the scratch alive until the stream has consumed it (DevBuf frees on scope exit)
  return hipStreamSynchronize(s);
}

// Compaction into the canonical (photon, bounce) order. A block's 256 photons own
// one contiguous output range: their deposits are read row by row (coalesced),
// staged in LDS at their output offsets and written out as consecutive floats;
// a block whose range exceeds the stage writes directly (same positions).
constexpr int kCompactStage = 1536;   // records (60 KB)
static_assert(sizeof(pm_photon) == 10 * sizeof(float), "pm_photon is staged as 10 floats");
__global__ __launch_bounds__(256) void k_compact_photons(const pm_photon* slots, const uint32_t* cnt,
                                                         const uint32_t* off, int64_t np, pm_photon* out) {
  __shared__ float stage[kCompactStage * 10];
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + threadIdx.x;
  const int64_t ilast = (i0 + blockDim.x < np ? i0 + blockDim.x : np) - 1;
  const uint32_t c = i < np ? cnt[i] : 0u, o = i < np ? off[i] : 0u;
  const uint32_t b0 = off[i0], b1 = off[ilast] + cnt[ilast];   // block's output range
  const uint32_t total = b1 - b0;
  if (total > (uint32_t)kCompactStage) {
    for (uint32_t k = 0; k < c; k++) out[(int64_t)o + k] = slots[(int64_t)k * np + i];
    return;
  }
  for (uint32_t k = 0; k < c; k++) {
    const pm_photon ph = slots[(int64_t)k * np + i];
    const float* f = reinterpret_cast<const float*>(&ph);
    float* d = stage + (size_t)(o - b0 + k) * 10;
#pragma unroll
    for (int w = 0; w < 10; w++) d[w] = f[w];
  }
  __syncthreads();
  float* of = reinterpret_cast<float*>(out + b0);
  for (uint32_t w = threadIdx.x; w < total * 10; w += blockDim.x) of[w] = stage[w];
}

hipError_t launch_trace_chunk(pm_scene* sc, const LightDev* d_lights, const int64_t* d_loff, int nl, int64_t g_lo,
                              int64_t np, int maxd, int caustic, pm_photon* slots, uint32_t* cnt, hipStream_t s) {
  if (np <= 0) return hipSuccess;
  if (maxd <= 0) return hipMemsetAsync(cnt, 0, sizeof(uint32_t) * np, s);
  // wavefront trace by default (57.5 vs 69.9 ms on config 3); PM_TRACE_WAVEFRONT=0
  // selects the fused per-lane kernel (A/B)
  const char* wf = std::getenv("PM_TRACE_WAVEFRONT");
  if (!wf || std::atoi(wf) != 0)
    return launch_trace_wavefront(sc, d_lights, d_loff, nl, g_lo, np, maxd, caustic, slots, cnt, s);
  const int blocks = grid_for((np + kPhotonsPerLane - 1) / kPhotonsPerLane, kTBlock);
  k_trace_photons<<<blocks, kTBlock, 0, s>>>(sc->view(), d_lights, d_loff, nl, g_lo, np, maxd, caustic, slots, cnt,
                                             sc->overflow.p);
  return hipGetLastError();
}

hipError_t launch_compact(const pm_photon* slots, const uint32_t* cnt, const uint32_t* off, int64_t np,
                          pm_photon* out, hipStream_t s) {
  if (np <= 0) return hipSuccess;
  k_compact_photons<<<grid_for(np, 256), 256, 0, s>>>(slots, cnt, off, np, out);
  return hipGetLastError();
}

}  // namespace pmd
