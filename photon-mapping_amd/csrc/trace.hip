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
#include <utility>

#include "pm_internal.hpp"

namespace pmd {

constexpr int kTBlock = 128;

// ------------------------------------------------------------------ wavefront
// Photon paths split per bounce into a lean closest-hit kernel
// (k_ph_trace_pool: traversal only, high occupancy, lanes refilled from a
// per-workgroup chunk of rays) and a shading kernel (k_ph_shade: event,
// deposit, continuation). Surviving rays are appended to the next bounce's
// list with one atomic per block; deposits go to slots[n][photon], so the
// output does not depend on the order in which rays are processed. (A fused
// per-lane kernel measured 70 vs 57.5 ms on config 3, a Morton sort of each
// bounce's rays 31.2 vs 29.5 ms with the ray pool: both removed.)
// The live-ray counts stay on the device (live[b] = rays entering bounce b):
// every bounce's grid is sized for all np rays and the blocks past live[b]
// retire at once, so the bounce loop never waits on the host.
struct PhotonRay {   // 48 B
  float4 o;          // origin, rng state (bits)
  float4 d;          // direction, photon index (bits)
  float4 c;          // colour, (deposits << 8 | bounce) (bits)
};

// Emission of photon i of this call (global index g_lo + i): pointLightRayGen
// (photon-mapping/cuda/deviceCode.cu:54-72), RNG seeded with the per-light id.
__device__ __forceinline__ void ph_emit(const LightDev* __restrict__ lights, const int64_t* __restrict__ loff, int nl,
                                        int64_t g, uint32_t& rng, v3& o, v3& d, v3& color) {
  int l = 0;
  while (l < nl - 1 && g >= loff[l + 1]) l++;
  const uint32_t id = (uint32_t)(g - loff[l]);
  const LightDev L = lights[l];
  rng = lcg_init(id, 0u);
  emit_photon(L.rgb.w, v3{L.pos.x, L.pos.y, L.pos.z}, v3{L.nrm.x, L.nrm.y, L.nrm.z}, L.nrm.w, rng, o, d);
  color = v3{L.rgb.x, L.rgb.y, L.rgb.z};
}

// One photon event at the end of a segment (t, slot: the closest hit; slot < 0:
// miss): triangleMeshClosestHit (deviceCode.cu:113-131) picks the event, and
// shootPhoton / shootCausticsPhoton (:25-52) deposit and decide whether the path
// goes on. Deposit k of photon pi lands in slots[k][pi]; a path that ends writes
// its deposit count to cnt[pi]. Returns true with the continuation (so, sd, and
// the scattered colour in `color`) when the path goes on to bounce b + 1.
__device__ __forceinline__ bool ph_event(const DevScene& S, v3 o, v3 d, float t, int slot, uint32_t& rng, v3& color,
                                         uint32_t& n, int b, uint32_t pi, int64_t np, int maxd, int caustic,
                                         pm_photon* __restrict__ slots, uint32_t* __restrict__ cnt, v3& so, v3& sd) {
  int ev;
  v3 sc = {0.f, 0.f, 0.f};
  so = sd = v3{0.f, 0.f, 0.f};
  if (slot < 0) {
    ev = EV_MISS;
  } else {
    const int mesh = __float_as_int(S.tri[3 * slot].w);
    const float4 m0 = S.mat[2 * mesh], m1 = S.mat[2 * mesh + 1];
    const float pd = m0.w;
    const float ps = m1.x + pd;
    const float pt = m1.y + ps;
    const float rp = lcg_next(rng);
    const v3 hp = add(o, smul(t, d));
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
    return false;
  }
  color = sc;
  return true;
}

__global__ __launch_bounds__(256) void k_ph_gen(const LightDev* __restrict__ lights, const int64_t* __restrict__ loff,
                                                int nl, int64_t g_lo, int64_t np, PhotonRay* __restrict__ rays) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  // pointLightRayGen (photon-mapping/cuda/deviceCode.cu:54-72)
  uint32_t rng;
  v3 o, d, c;
  ph_emit(lights, loff, nl, g_lo + i, rng, o, d, c);
  PhotonRay r;
  r.o = make_float4(o.x, o.y, o.z, __uint_as_float(rng));
  r.d = make_float4(d.x, d.y, d.z, __uint_as_float((uint32_t)i));
  r.c = make_float4(c.x, c.y, c.z, __uint_as_float(0u));
  rays[i] = r;
}

#ifndef PM_TPOOL_WAVES
#define PM_TPOOL_WAVES 8   // occupancy target of k_ph_trace_pool (0: compiler's choice; 8 measured best with 64-B nodes)
#endif
__global__ __launch_bounds__(kTBlock) PM_WAVES_ATTR(PM_TPOOL_WAVES) void k_ph_trace_pool(
    DevScene S, const PhotonRay* __restrict__ rays, const uint32_t* __restrict__ live, float2* __restrict__ hits,
    int* overflow) {
  __shared__ int stack[kStackDepth * kTBlock];
  __shared__ int lnext;
  const int64_t n = *live;
  const int chunk = pool_chunk(n, kTBlock);   // the grid covers it for any n <= np (pool_grid)
  if ((int64_t)blockIdx.x * chunk >= n) return;
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

// Surviving rays are appended with ONE atomic per block (a same-address atomic
// per wave serialised at one L2 channel: ~2/3 of the kernel).
#ifndef PM_SHADE_BLOCK
#define PM_SHADE_BLOCK 256
#endif
constexpr int kShadeBlock = PM_SHADE_BLOCK;

__global__ __launch_bounds__(kShadeBlock) void k_ph_shade(DevScene S, const PhotonRay* __restrict__ in,
                                                          const uint32_t* __restrict__ live,
                                                          const float2* __restrict__ hits,
                                                          PhotonRay* __restrict__ out,
                                                          uint32_t* __restrict__ count_out, int64_t np, int maxd,
                                                          int caustic, pm_photon* __restrict__ slots,
                                                          uint32_t* __restrict__ cnt) {
  __shared__ uint32_t wcount[kShadeBlock / 64];
  __shared__ uint32_t block_base;
  const int64_t n_in = *live;
  if ((int64_t)blockIdx.x * kShadeBlock >= n_in) return;   // whole block past the live rays (uniform)
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
    v3 color = {pr.c.x, pr.c.y, pr.c.z}, so, sd;
    if (ph_event(S, v3{pr.o.x, pr.o.y, pr.o.z}, v3{pr.d.x, pr.d.y, pr.d.z}, hh.x, slot, rng, color, n, b, pi, np,
                 maxd, caustic, slots, cnt, so, sd)) {
      keep = true;
      nr.o = make_float4(so.x, so.y, so.z, __uint_as_float(rng));
      nr.d = make_float4(sd.x, sd.y, sd.z, __uint_as_float(pi));
      nr.c = make_float4(color.x, color.y, color.z, __uint_as_float((n << 8) | (uint32_t)(b + 1)));
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
}

// ------------------------------------------------------------------ fused paths
// PM_TRACE_FUSED: one launch per chunk instead of emission + two per bounce.
// A persistent grid (PM_TPATH_BLOCKS workgroups per CU) takes photons from a
// global counter; each lane traces a photon's whole path: emission, then per
// segment the same closest-hit traversal as k_ph_trace_pool and the same event
// as k_ph_shade (ph_event), continuing with the scattered ray until the path
// ends, then takes the next photon. Lanes whose segment is done wait until
// PM_PATH_EVENT_MIN of them (or all the wave's non-idle lanes) are, and the
// wave runs their events together; idle lanes are refilled together (one
// atomic per wave). Deposits land in slots[k][photon] as before, so the output
// is the wavefront path's bit for bit (the check variant library keeps the
// wavefront path: tests/test_gpu_check_variant.py compares the two; the budget
// variant runs this kernel with a 4-entry LDS stack against production). The
// kernel holds every wave slot it gets until the last path ends, so the frame
// starts the render's ray kernels after it (pm_amd.dist FrameConfig.
// begin_after_trace); the cap below can leave slots and VGPRs to other streams
// instead (measured slower). Config 3's global trace alone:
// ~16-17 ms (the wavefront path: ~27 ms).
#ifndef PM_TRACE_FUSED
#define PM_TRACE_FUSED 1
#endif
#ifndef PM_PATH_EVENT_MIN
#define PM_PATH_EVENT_MIN 16
#endif
#ifndef PM_TPATH_WAVES
#define PM_TPATH_WAVES 7
#endif
// Workgroups of kTBlock threads per CU (14: every slot 72 VGPRs allow, 7 waves
// per SIMD). Config 3 frames (ms) with the render begin beside the trace, caps
// 6 / 8 / 10 / 14: 97.7 / 97.0 / 97.0 / 98.4 (wavefront trace: 96.5); with the
// render begin after the trace (FrameConfig.begin_after_trace, now the
// default): 8 / 10 / 14: 99.1 / 97.9 / 93.8-94.3.
#ifndef PM_TPATH_BLOCKS
#define PM_TPATH_BLOCKS 14
#endif
__global__ __launch_bounds__(kTBlock) PM_WAVES_ATTR(PM_TPATH_WAVES) void k_ph_paths(
    DevScene S, const LightDev* __restrict__ lights, int nl, PathSet A, PathSet B, int maxd,
    unsigned long long* __restrict__ next, int* overflow) {
  __shared__ int stack[kStackDepth * kTBlock];
  int* const st = stack + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int64_t np = A.np + B.np;   // photons [0, A.np) are set A's, the rest set B's
  int spill[kSpillDepth > 0 ? kSpillDepth : 1];
  Ray r;
  HitInfo h{kPhotonTmax, -1, -1};
  int node = 0, sp = 0, b = 0;
  int64_t pi = -1;      // this lane's photon (-1: idle), an index over both sets
  bool pend = false;    // its segment's traversal is done, the event not yet run
  uint32_t rng = 0, n = 0;
  v3 color = {0.f, 0.f, 0.f};
  bool drained = false;
  for (;;) {
    const uint64_t pm = __ballot(pend);
    if (pm != 0 && (__popcll(pm) >= PM_PATH_EVENT_MIN || __ballot(pi >= 0 && !pend) == 0)) {
      if (pend) {
        const bool inb = pi >= A.np;
        v3 so, sd;
        if (ph_event(S, r.o, r.d, h.t, h.slot, rng, color, n, b, (uint32_t)(inb ? pi - A.np : pi), inb ? B.np : A.np,
                     maxd, inb ? B.caustic : A.caustic, inb ? B.slots : A.slots, inb ? B.cnt : A.cnt, so, sd)) {
          ray_prep(r, so, sd);
          h = HitInfo{kPhotonTmax, -1, -1};
          node = 0;
          sp = 0;
          b++;
        } else {
          pi = -1;
        }
        pend = false;
      }
    }
    const uint64_t idle = __ballot(pi < 0);
    const int nidle = __popcll(idle);
    if (!drained && nidle >= PM_POOL_REFILL) {
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(next, (unsigned long long)nidle);
      base = __shfl(base, 0);
      if (base + (unsigned long long)nidle >= (unsigned long long)np) drained = true;
      if (pi < 0) {
        const int64_t i = (int64_t)base + __popcll(idle & lt_mask);
        if (i < np) {
          const bool inb = i >= A.np;
          v3 o, d;
          ph_emit(lights, inb ? B.loff : A.loff, nl, inb ? B.g_lo + (i - A.np) : A.g_lo + i, rng, o, d, color);
          ray_prep(r, o, d);
          h = HitInfo{kPhotonTmax, -1, -1};
          node = 0;
          sp = 0;
          b = 0;
          n = 0;
          pi = i;
          pend = S.ntri <= 0;   // empty scene: a miss at once
        }
      }
    }
    if (__ballot(pi >= 0) == 0) {
      if (drained) break;
      continue;
    }
    if (pi >= 0 && !pend && traverse_step<false>(S, r, kEPS, kPhotonTmax, st, kTBlock, spill, node, sp, h, overflow))
      pend = true;
  }
}

// One persistent launch over both sets (B.np may be 0): set A's photons are
// taken first, so set B's (the frame passes the caustic set, whose paths end
// at their first diffuse hit) fill the tail that A's long paths leave.
static hipError_t launch_trace_fused(pm_scene* sc, const LightDev* d_lights, int nl, const PathSet& A,
                                     const PathSet& B, int maxd, hipStream_t s) {
  int cus = 0;   // of the stream's device (a process may drive several)
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, stream_device(s)) != hipSuccess || cus <= 0)
    cus = 256;
  DevBuf<unsigned long long> next(1);
  if (!next.p) return hipErrorOutOfMemory;
  PM_HIP_TRY(hipMemsetAsync(next.p, 0, sizeof(unsigned long long), s));
  const int64_t want = (A.np + B.np + kTBlock - 1) / kTBlock;
  const int grid = (int)std::min<int64_t>(want, (int64_t)cus * PM_TPATH_BLOCKS);
  k_ph_paths<<<grid, kTBlock, 0, s>>>(sc->view(), d_lights, nl, A, B, maxd, next.p, sc->overflow.p);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);   // the counter is freed on return
}

__global__ void k_live_init(uint32_t* __restrict__ live, int nlive, uint32_t np) {
  const int i = (int)threadIdx.x;
  if (i < nlive) live[i] = i == 0 ? np : 0u;
}

hipError_t launch_trace_wavefront(pm_scene* sc, const LightDev* d_lights, const int64_t* d_loff, int nl,
                                  int64_t g_lo, int64_t np, int maxd, int caustic, pm_photon* slots, uint32_t* cnt,
                                  hipStream_t s) {
  DevBuf<PhotonRay> ra(np), rb(np);
  DevBuf<float2> hits(np);
  DevBuf<uint32_t> live(maxd + 1);
  if (!ra.p || !rb.p || !hits.p || !live.p) return hipErrorOutOfMemory;
  k_live_init<<<1, 64 * ((maxd + 64) / 64), 0, s>>>(live.p, maxd + 1, (uint32_t)np);
  PM_HIP_TRY(hipGetLastError());
  k_ph_gen<<<grid_for(np, 256), 256, 0, s>>>(d_lights, d_loff, nl, g_lo, np, ra.p);
  PM_HIP_TRY(hipGetLastError());
  PhotonRay *cur = ra.p, *nxt = rb.p;
  const int tgrid = (int)pool_grid(np, kTBlock);
  for (int b = 0; b < maxd; b++) {
    k_ph_trace_pool<<<tgrid, kTBlock, 0, s>>>(sc->view(), cur, live.p + b, hits.p, sc->overflow.p);
    PM_HIP_TRY(hipGetLastError());
    k_ph_shade<<<grid_for(np, kShadeBlock), kShadeBlock, 0, s>>>(sc->view(), cur, live.p + b, hits.p, nxt,
                                                                 live.p + b + 1, np, maxd, caustic, slots, cnt);
    PM_HIP_TRY(hipGetLastError());
    std::swap(cur, nxt);
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
  return launch_trace_sets(sc, d_lights, nl, PathSet{d_loff, g_lo, np, caustic, slots, cnt}, PathSet{}, maxd, s);
}

hipError_t launch_trace_sets(pm_scene* sc, const LightDev* d_lights, int nl, PathSet A, PathSet B, int maxd,
                             hipStream_t s) {
  if (A.np < 0 || B.np < 0 || A.np + B.np > 0xFFFFFFFFll)   // photon ids and live counts are 32-bit
    return hipErrorInvalidValue;
  if (A.np + B.np == 0) return hipSuccess;
  if (maxd <= 0) {
    if (A.np > 0) PM_HIP_TRY(hipMemsetAsync(A.cnt, 0, sizeof(uint32_t) * A.np, s));
    if (B.np > 0) PM_HIP_TRY(hipMemsetAsync(B.cnt, 0, sizeof(uint32_t) * B.np, s));
    return hipSuccess;
  }
  if (PM_TRACE_FUSED) {
    if (A.np == 0) std::swap(A, B);
    return launch_trace_fused(sc, d_lights, nl, A, B, maxd, s);
  }
  // the wavefront path (check variant): one set after the other
  for (const PathSet* P : {&A, &B})
    if (P->np > 0)
      PM_HIP_TRY(launch_trace_wavefront(sc, d_lights, P->loff, nl, P->g_lo, P->np, maxd, P->caustic, P->slots, P->cnt,
                                        s));
  return hipSuccess;
}

hipError_t launch_compact(const pm_photon* slots, const uint32_t* cnt, const uint32_t* off, int64_t np,
                          pm_photon* out, hipStream_t s) {
  if (np <= 0) return hipSuccess;
  k_compact_photons<<<grid_for(np, 256), 256, 0, s>>>(slots, cnt, off, np, out);
  return hipGetLastError();
}

}  // namespace pmd
