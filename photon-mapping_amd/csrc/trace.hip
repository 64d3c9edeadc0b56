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
#include "pm_internal.hpp"

namespace pmd {

constexpr int kTBlock = 128;

struct LightDev {
  float4 pos;   // xyz
  float4 rgb;   // xyz
};

// Each lane traces several photons back to back (i, i + stride, ...): when a
// photon's path ends the lane immediately starts its next photon, so a wave
// is not held by its longest path (path lengths range over 1..max_depth).
constexpr int kPhotonsPerLane = 8;

__global__ __launch_bounds__(kTBlock) void k_trace_photons(DevScene S, const LightDev* lights, const int64_t* loff,
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
      o = {L.pos.x, L.pos.y, L.pos.z};
      d = random_point_in_unit_sphere(rng);
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

__global__ void k_compact_photons(const pm_photon* slots, const uint32_t* cnt, const uint32_t* off, int64_t np,
                                  pm_photon* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  const uint32_t c = cnt[i], o = off[i];
  for (uint32_t k = 0; k < c; k++) out[(int64_t)o + k] = slots[(int64_t)k * np + i];
}

hipError_t launch_trace_chunk(pm_scene* sc, const LightDev* d_lights, const int64_t* d_loff, int nl, int64_t g_lo,
                              int64_t np, int maxd, int caustic, pm_photon* slots, uint32_t* cnt, hipStream_t s) {
  if (np <= 0) return hipSuccess;
  if (maxd <= 0) return hipMemsetAsync(cnt, 0, sizeof(uint32_t) * np, s);
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
