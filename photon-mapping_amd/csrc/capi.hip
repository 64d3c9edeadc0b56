// capi.hip — the extern "C" boundary of libpm_hip.so (declared in include/pm.h).
//
// Mirrors the reference's host-side entry points for the hot path:
//   pm_scene_create      <- loadGeometry (common/src/world.cpp:3-58)
//   pm_trace_photons     <- runNormal / runCaustics / runPointLightRayGen
//                           (photon-mapping/src/hostCode.cu:72-138)
//   pm_photon_map_create <- loadPhotons (ray-tracer/src/hostCode.cu:54-99)
//   pm_kdtree_build      <- cukd::buildTree (ray-tracer/src/hostCode.cu:94-95)
//   pm_knn / pm_gather   <- KNearestPhotons / gatherPhotons (ray-tracer/cuda/shading.h)
//   pm_render            <- owlRayGenLaunch2D(simpleRayGen) (ray-tracer/src/hostCode.cu:231-237)
// Every compute entry point runs on the GPU; without a device it returns
// PM_ERR_NO_DEVICE (there is no CPU fallback).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "pm_internal.hpp"

namespace pmd {

hipError_t launch_query(pm_scene* sc, const pm_ray* rays, int64_t n, pm_hit* hits, int32_t* occ, bool any,
                        hipStream_t s);
hipError_t photons_quantize(pm_photon* ph, int64_t n, hipStream_t s);
hipError_t photon_view(pm_scene* sc, const pm_photon* ph, int64_t n, const pm_viewer_params& P, uint32_t* rgba,
                       hipStream_t s);
hipError_t launch_trace_chunk(pm_scene* sc, const LightDev* d_lights, const int64_t* d_loff, int nl, int64_t g_lo,
                              int64_t np, int maxd, int caustic, pm_photon* slots, uint32_t* cnt, hipStream_t s);
hipError_t launch_compact(const pm_photon* slots, const uint32_t* cnt, const uint32_t* off, int64_t np,
                          pm_photon* out, hipStream_t s);
hipError_t kd_build_records(pm_kd_photon* d, int64_t n, pm_box* bounds, hipStream_t s);
hipError_t launch_map_export(const pm_photon_map* m, pm_kd_photon* out, hipStream_t s);
hipError_t launch_knn(const pm_photon_map* m, const pm_float3* q, int64_t nq, int k, float radius, int32_t* ids,
                      float* d2, float* maxd2, hipStream_t s);
hipError_t launch_gather_api(const pm_photon_map* m, const pm_float3* pts, const float* brdf, int64_t nq,
                             pm_float3* out, hipStream_t s, int k);
hipError_t render_begin(pm_scene* sc, const pm_render_params* P, const pm_light* lights, int nl, pm_render_job* J,
                        hipStream_t s);
hipError_t render_finish(pm_render_job* J, const pm_photon_map* gmap, const pm_photon_map* cmap, uint32_t* rgba,
                         float* rgb, hipStream_t s);
pm_render_job* render_job_new(pm_scene* sc, hipStream_t s);
void render_job_delete(pm_render_job* J);
const pm_render_stats& render_job_stats(const pm_render_job* J);
pm_scene* render_job_scene(const pm_render_job* J);
int render_job_device(const pm_render_job* J);
void render_job_queries(const pm_render_job* J, int which, const float4** q, const float4** res, int64_t* n);
bool render_job_finished(const pm_render_job* J);
void render_job_mark_finished(pm_render_job* J);
const pm_photon_map* render_job_caustic_map(const pm_render_job* J);
hipError_t render_gather_caustic(pm_render_job* J, const pm_photon_map* cmap, hipStream_t s);

namespace {
std::mutex g_phase_mu;   // guards g_render_stats
// phase timers are per host thread: a caller that drives two streams from two
// threads (the caustic pass beside the global trace) reads each call's own time
thread_local double g_phase_us[PH_COUNT] = {0};
pm_render_stats g_render_stats{};
}  // namespace

void record_phase_us(int phase, double us) {
  if (phase >= 0 && phase < PH_COUNT) g_phase_us[phase] += us;
}
static void reset_phase(int phase) {
  if (phase >= 0 && phase < PH_COUNT) g_phase_us[phase] = 0;
}

PhaseTimer::PhaseTimer(int ph, hipStream_t st) : s(st), phase(ph) {
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
    a = b = nullptr;
    return;
  }
  (void)hipEventRecord(a, s);
}
PhaseTimer::~PhaseTimer() {
  if (!a) return;
  (void)hipEventRecord(b, s);
  if (hipEventSynchronize(b) == hipSuccess) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) == hipSuccess) record_phase_us(phase, (double)ms * 1000.0);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

}  // namespace pmd

using namespace pmd;

namespace {

int map_err(hipError_t e) {
  if (e == hipSuccess) return PM_OK;
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return PM_ERR_OOM;
  if (e == hipErrorInvalidValue) return PM_ERR_INVALID;
  if (e == hipErrorNoDevice) return PM_ERR_NO_DEVICE;
  std::fprintf(stderr, "pm: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
  return PM_ERR_HIP;
}

int require_device() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return PM_ERR_NO_DEVICE;
  }
  return PM_OK;
}

int check_overflow(pm_scene* sc, hipStream_t s) {
  int ov = 0;
  if (hipMemcpyAsync(&ov, sc->overflow.p, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return PM_ERR_HIP;
  return ov ? PM_ERR_OVERFLOW : PM_OK;
}

// A handle belongs to the device it was created on; a call whose stream is on
// another device is refused (PM_ERR_DEVICE) instead of launching kernels that
// would read that GPU's memory from this one.
#define PM_SAME_DEVICE(scope, obj)                                   \
  do {                                                               \
    if ((obj) && (obj)->device != (scope).dev) return PM_ERR_DEVICE; \
  } while (0)

// A caller's device pointer that lives on another device than the call's.
bool ptr_elsewhere(const void* p, int dev) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;   // not a HIP allocation (e.g. host memory): nothing to compare
  }
  return a.type == hipMemoryTypeDevice && a.device != dev;
}

#define PM_PTR_DEVICE(scope, ptr)                                 \
  do {                                                            \
    if (ptr_elsewhere((ptr), (scope).dev)) return PM_ERR_DEVICE;  \
  } while (0)

#define PM_TRY_ST(expr)             \
  do {                              \
    int _st = map_err(expr);        \
    if (_st != PM_OK) return _st;   \
  } while (0)

// the runs of two pm_photon arrays (a ++ b)
RowRuns runs_of(const pm_photon* a, int64_t na, float pa, const pm_photon* b, int64_t nb, float pb) {
  RowRuns r;
  if (na > 0) r.push_back({reinterpret_cast<const float*>(a), 10, 7, na, pa});
  if (nb > 0) r.push_back({reinterpret_cast<const float*>(b), 10, 7, nb, pb});
  return r;
}

// the runs of a pm_photon_rows set (NULL: none); false on a malformed descriptor
bool runs_of_rows(const pm_photon_rows* x, float power, RowRuns& out) {
  if (!x) return true;
  if (x->nseg < 0 || x->nseg > PM_ROWS_MAX_SEGS || x->row_floats < 6 || x->color_offset < 3 ||
      x->color_offset > x->row_floats - 3 || x->reserved != 0)
    return false;
  for (int k = 0; k < x->nseg; k++) {
    if (x->seg_row0[k] < 0 || x->seg_count[k] < 0) return false;
    if (x->seg_count[k] == 0) continue;
    if (!x->d_rows) return false;
    out.push_back({x->d_rows + x->seg_row0[k] * x->row_floats, x->row_floats, x->color_offset, x->seg_count[k], power});
  }
  return true;
}

// every run's rows on the call's device
bool runs_elsewhere(const RowRuns& runs, int dev) {
  for (const RowRun& r : runs)
    if (ptr_elsewhere(r.rows, dev)) return true;
  return false;
}

}  // namespace

extern "C" {

int pm_abi_version(void) { return PM_ABI_VERSION; }

const char* pm_status_string(int st) {
  switch (st) {
    case PM_OK: return "ok";
    case PM_ERR_INVALID: return "invalid argument";
    case PM_ERR_HIP: return "HIP runtime error";
    case PM_ERR_OOM: return "device out of memory";
    case PM_ERR_NO_DEVICE: return "no HIP device";
    case PM_ERR_IO: return "I/O error";
    case PM_ERR_CAPACITY: return "output capacity too small";
    case PM_ERR_OVERFLOW: return "traversal stack overflow";
    case PM_ERR_DEVICE: return "handle or buffer on another device than the stream";
    default: return "unknown status";
  }
}

int pm_device_count(int32_t* count) {
  if (!count) return PM_ERR_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  *count = n;
  return PM_OK;
}

int pm_last_phase_us(int32_t phase, double* us) {
  if (!us || phase < 0 || phase >= PH_COUNT) return PM_ERR_INVALID;
  *us = g_phase_us[phase];
  return PM_OK;
}

int pm_device_pool_stats(int32_t device, int64_t* live_bytes, int64_t* cached_bytes) {
  size_t l = 0, c = 0;
  dev_pool_stats(device, &l, &c);
  if (live_bytes) *live_bytes = (int64_t)l;
  if (cached_bytes) *cached_bytes = (int64_t)c;
  return PM_OK;
}

// ------------------------------------------------------------------ scene
int pm_device_alloc(size_t bytes, void** d_ptr) {
  if (!d_ptr) return PM_ERR_INVALID;
  *d_ptr = nullptr;
  if (int st = require_device()) return st;
  if (bytes == 0) return PM_OK;
  return map_err(hipMalloc(d_ptr, bytes));
}

int pm_device_free(void* d_ptr) {
  if (!d_ptr) return PM_OK;
  return map_err(hipFree(d_ptr));
}

int pm_copy_to_device(void* d_dst, const void* h_src, size_t bytes) {
  if (bytes == 0) return PM_OK;
  if (!d_dst || !h_src) return PM_ERR_INVALID;
  if (int st = require_device()) return st;
  return map_err(hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice));
}

int pm_copy_to_host(void* h_dst, const void* d_src, size_t bytes) {
  if (bytes == 0) return PM_OK;
  if (!h_dst || !d_src) return PM_ERR_INVALID;
  if (int st = require_device()) return st;
  return map_err(hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost));
}

int pm_scene_create(const pm_mesh* meshes, int32_t num_meshes, pm_scene** out) {
  if (!out || num_meshes < 0 || (num_meshes > 0 && !meshes)) return PM_ERR_INVALID;
  *out = nullptr;
  int st = require_device();
  if (st != PM_OK) return st;
  std::vector<float4> th;
  std::vector<float4> mh;
  int64_t gid = 0;
  for (int m = 0; m < num_meshes; m++) {
    const pm_mesh& M = meshes[m];
    if (M.num_triangles < 0 || M.num_vertices < 0 || (M.num_triangles > 0 && (!M.indices || !M.vertices)))
      return PM_ERR_INVALID;
    for (int j = 0; j < M.num_triangles; j++, gid++) {
      const pm_int3 ix = M.indices[j];
      const int32_t id3[3] = {ix.x, ix.y, ix.z};
      for (int k = 0; k < 3; k++)
        if (id3[k] < 0 || id3[k] >= M.num_vertices) return PM_ERR_INVALID;
      const pm_float3 A = M.vertices[ix.x], B = M.vertices[ix.y], C = M.vertices[ix.z];
      float wa, wb, wc;
      const int32_t im = m, ip = j, ig = (int32_t)gid;
      std::memcpy(&wa, &im, 4);
      std::memcpy(&wb, &ip, 4);
      std::memcpy(&wc, &ig, 4);
      th.push_back(make_float4(A.x, A.y, A.z, wa));
      th.push_back(make_float4(B.x, B.y, B.z, wb));
      th.push_back(make_float4(C.x, C.y, C.z, wc));
    }
    const pm_material& mt = M.material;
    mh.push_back(make_float4(mt.albedo.x, mt.albedo.y, mt.albedo.z, mt.diffuse));
    mh.push_back(make_float4(mt.specular, mt.transmission, mt.refraction_idx, 0.f));
  }
  if (gid >= (1ll << 31)) return PM_ERR_INVALID;
  pm_scene* sc = new pm_scene;
  sc->device = stream_device(nullptr);
  sc->ntri = (int32_t)gid;
  sc->nmesh = num_meshes;
  for (int m = 0; m < num_meshes; m++) sc->host_mat.push_back(meshes[m].material);
  hipStream_t s = nullptr;
  sc->mat.alloc(std::max<size_t>(mh.size(), 2));
  sc->overflow.alloc(1);
  if (!sc->mat.p || !sc->overflow.p) {
    delete sc;
    return PM_ERR_OOM;
  }
  hipError_t e = hipSuccess;
  if (!mh.empty()) e = hipMemcpyAsync(sc->mat.p, mh.data(), sizeof(float4) * mh.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemsetAsync(sc->overflow.p, 0, sizeof(int32_t), s);
  reset_phase(PH_BVH);
  if (e == hipSuccess) {
    PhaseTimer tm(PH_BVH, s);
    e = build_lbvh(sc, th, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete sc;
    return map_err(e);
  }
  *out = sc;
  return PM_OK;
}

int pm_scene_stats_get(const pm_scene* sc, pm_scene_stats* o) {
  if (!sc || !o) return PM_ERR_INVALID;
  o->num_triangles = sc->ntri;
  o->num_nodes = sc->nnodes;
  o->num_meshes = sc->nmesh;
  o->max_depth = sc->depth;
  o->bounds = sc->bounds;
  return PM_OK;
}

int pm_scene_destroy(pm_scene* sc) {
  if (sc) {
    AllocStream pool(nullptr, sc->device);
    delete sc;
  }
  return PM_OK;
}

int pm_scene_intersect(pm_scene* sc, const pm_ray* rays, int64_t n, pm_hit* hits, void* stream) {
  if (!sc || n < 0 || (n > 0 && (!rays || !hits))) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, sc);
  PM_PTR_DEVICE(alloc_scope, rays);
  PM_PTR_DEVICE(alloc_scope, hits);
  PM_TRY_ST(launch_query(sc, rays, n, hits, nullptr, false, s));
  return check_overflow(sc, s);
}

int pm_scene_occluded(pm_scene* sc, const pm_ray* rays, int64_t n, int32_t* occ, void* stream) {
  if (!sc || n < 0 || (n > 0 && (!rays || !occ))) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, sc);
  PM_PTR_DEVICE(alloc_scope, rays);
  PM_PTR_DEVICE(alloc_scope, occ);
  PM_TRY_ST(launch_query(sc, rays, n, nullptr, occ, true, s));
  return check_overflow(sc, s);
}

// ------------------------------------------------------------------ stage 1
int pm_photons_per_light(const pm_light* lights, int32_t nl, int64_t casted, int64_t* counts) {
  if (nl < 0 || (nl > 0 && (!lights || !counts))) return PM_ERR_INVALID;
  // computePhotonsPerWatt (hostCode.cu:102-110): int photonsPerWatt = int / double
  double total = 0;
  for (int i = 0; i < nl; i++) total += lights[i].power;
  if (!(total > 0.0)) {
    for (int i = 0; i < nl; i++) counts[i] = 0;
    return PM_OK;
  }
  const int ppw = (int)((double)(int)casted / total);
  for (int i = 0; i < nl; i++) counts[i] = (int64_t)(int)(lights[i].power * ppw);   // hostCode.cu:86
  return PM_OK;
}

static int shard_range(const pm_light* lights, int32_t nl, const pm_trace_params* p, std::vector<int64_t>& loff,
                       int64_t& lo, int64_t& hi) {
  if (!p || p->shard_count < 1 || p->shard_rank < 0 || p->shard_rank >= p->shard_count || p->max_depth < 0 ||
      p->max_depth > 255 || p->casted_photons < 0)
    return PM_ERR_INVALID;
  std::vector<int64_t> cnt(nl > 0 ? nl : 1, 0);
  int st = pm_photons_per_light(lights, nl, p->casted_photons, cnt.data());
  if (st != PM_OK) return st;
  loff.assign(nl + 1, 0);
  for (int i = 0; i < nl; i++) loff[i + 1] = loff[i] + std::max<int64_t>(cnt[i], 0);
  const int64_t tot = loff[nl];
  lo = tot * p->shard_rank / p->shard_count;
  hi = tot * (p->shard_rank + 1) / p->shard_count;
  return PM_OK;
}

int pm_trace_capacity(const pm_light* lights, int32_t nl, const pm_trace_params* p, int64_t* capacity) {
  if (!capacity) return PM_ERR_INVALID;
  std::vector<int64_t> loff;
  int64_t lo, hi;
  int st = shard_range(lights, nl, p, loff, lo, hi);
  if (st != PM_OK) return st;
  const int per = p->caustics_mode ? 1 : std::max(p->max_depth - 1, 0);
  *capacity = (hi - lo) * per;
  return PM_OK;
}

int pm_trace_photons(pm_scene* sc, const pm_light* lights, int32_t nl, const pm_trace_params* p, pm_photon* d_out,
                     int64_t capacity, int64_t* count, void* stream) {
  if (!sc || !count || capacity < 0) return PM_ERR_INVALID;
  *count = 0;
  std::vector<int64_t> loff;
  int64_t lo, hi;
  int st = shard_range(lights, nl, p, loff, lo, hi);
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, sc);
  PM_PTR_DEVICE(alloc_scope, d_out);
  reset_phase(PH_TRACE);
  reset_phase(PH_COMPACT);
  const int maxd = p->max_depth;
  const int per = p->caustics_mode ? 1 : std::max(maxd - 1, 0);
  const int64_t np_total = hi - lo;
  if (np_total <= 0 || per == 0 || nl == 0) return PM_OK;
  std::vector<LightDev> lh(nl);
  for (int i = 0; i < nl; i++) {
    lh[i].pos = make_float4(lights[i].pos.x, lights[i].pos.y, lights[i].pos.z, 0.f);
    lh[i].rgb = make_float4(lights[i].rgb.x, lights[i].rgb.y, lights[i].rgb.z,
                            lights[i].source_type == PM_SQUARE_LIGHT ? 1.f : 0.f);
    lh[i].nrm = make_float4(lights[i].normal.x, lights[i].normal.y, lights[i].normal.z,
                            (float)lights[i].side_length);
  }
  DevBuf<LightDev> dl(nl);
  DevBuf<int64_t> dloff(nl + 1);
  if (!dl.p || !dloff.p) return PM_ERR_OOM;
  PM_TRY_ST(hipMemcpyAsync(dl.p, lh.data(), sizeof(LightDev) * nl, hipMemcpyHostToDevice, s));
  PM_TRY_ST(hipMemcpyAsync(dloff.p, loff.data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
  // chunk so that the deposit slots stay below ~16 GB (of 288): config 3's 10 M
  // photons run as ONE chunk (at ~3 GB they ran as 8.3 M + 1.7 M, and the small
  // chunk's late bounces could not fill the GPU)
  int64_t chunk = std::min<int64_t>(np_total, std::max<int64_t>(1 << 16, (int64_t)16e9 / (40ll * per)));
  chunk = std::min<int64_t>(chunk, 1ll << 26);
  DevBuf<pm_photon> slots((size_t)chunk * per);
  DevBuf<uint32_t> cnt(chunk), off(chunk), tot(1);
  if (!slots.p || !cnt.p || !off.p || !tot.p) return PM_ERR_OOM;
  int64_t written = 0;
  bool over = false;
  for (int64_t g0 = lo; g0 < hi; g0 += chunk) {
    const int64_t np = std::min(chunk, hi - g0);
    {
      PhaseTimer tm(PH_TRACE, s);
      PM_TRY_ST(launch_trace_chunk(sc, dl.p, dloff.p, nl, g0, np, maxd, p->caustics_mode ? 1 : 0, slots.p, cnt.p,
                                   s));
    }
    uint32_t t = 0;
    {
      PhaseTimer tm(PH_COMPACT, s);
      PM_TRY_ST(exclusive_scan_u32(cnt.p, off.p, np, tot.p, s));
      PM_TRY_ST(hipMemcpyAsync(&t, tot.p, 4, hipMemcpyDeviceToHost, s));
      PM_TRY_ST(hipStreamSynchronize(s));
      if (!over && written + (int64_t)t <= capacity && d_out) {
        PM_TRY_ST(launch_compact(slots.p, cnt.p, off.p, np, d_out + written, s));
      } else {
        over = true;
      }
    }
    written += t;
  }
  PM_TRY_ST(hipStreamSynchronize(s));
  *count = written;
  st = check_overflow(sc, s);
  if (st != PM_OK) return st;
  return over ? PM_ERR_CAPACITY : PM_OK;
}

// Both photon sets of a frame in ONE launch (runNormal + runCaustics,
// photon-mapping/src/hostCode.cu:112-138): each set's photons, order and
// capacity behaviour are exactly those of its own pm_trace_photons call.
static void light_devs(const pm_light* lights, int nl, std::vector<LightDev>& lh) {
  lh.resize(nl);
  for (int i = 0; i < nl; i++) {
    lh[i].pos = make_float4(lights[i].pos.x, lights[i].pos.y, lights[i].pos.z, 0.f);
    lh[i].rgb = make_float4(lights[i].rgb.x, lights[i].rgb.y, lights[i].rgb.z,
                            lights[i].source_type == PM_SQUARE_LIGHT ? 1.f : 0.f);
    lh[i].nrm = make_float4(lights[i].normal.x, lights[i].normal.y, lights[i].normal.z,
                            (float)lights[i].side_length);
  }
}

int pm_trace_photon_sets(pm_scene* sc, const pm_light* lights, int32_t nl, const pm_trace_params* params,
                         pm_photon* const* d_out, const int64_t* capacity, int64_t* count, void* stream) {
  if (!sc || !params || !d_out || !capacity || !count) return PM_ERR_INVALID;
  count[0] = count[1] = 0;
  std::vector<int64_t> loff[2];
  int64_t lo[2], hi[2], np[2];
  int per[2];
  for (int k = 0; k < 2; k++) {
    if (capacity[k] < 0) return PM_ERR_INVALID;
    const int st = shard_range(lights, nl, &params[k], loff[k], lo[k], hi[k]);
    if (st != PM_OK) return st;
    per[k] = params[k].caustics_mode ? 1 : std::max(params[k].max_depth - 1, 0);
    np[k] = (per[k] > 0 && nl > 0) ? hi[k] - lo[k] : 0;
  }
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, sc);
  PM_PTR_DEVICE(alloc_scope, d_out[0]);
  PM_PTR_DEVICE(alloc_scope, d_out[1]);
  // the deposit slots of both sets within the one-chunk budget (as
  // pm_trace_photons' ~16 GB), one max_depth; else one call per set
  const bool one = params[0].max_depth == params[1].max_depth && np[0] + np[1] <= 0xFFFFFFFFll &&
                   (np[0] * per[0] + np[1] * per[1]) * 40 <= (int64_t)16e9;
  if (!one) {
    hipEvent_t a = nullptr, b = nullptr;
    PM_TRY_ST(hipEventCreate(&a));
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      return PM_ERR_HIP;
    }
    (void)hipEventRecord(a, s);
    double compact = 0.0;
    int st = PM_OK;
    for (int k = 0; k < 2 && (st == PM_OK || st == PM_ERR_CAPACITY); k++) {
      const int sk = pm_trace_photons(sc, lights, nl, &params[k], d_out[k], capacity[k], &count[k], stream);
      compact += g_phase_us[PH_COMPACT];
      if (st == PM_OK) st = sk;
    }
    (void)hipEventRecord(b, s);
    float ms = 0.f;
    if (hipEventSynchronize(b) == hipSuccess && hipEventElapsedTime(&ms, a, b) == hipSuccess) {
      g_phase_us[PH_TRACE] = (double)ms * 1000.0;
      g_phase_us[PH_COMPACT] = compact;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return st;
  }
  reset_phase(PH_TRACE);
  reset_phase(PH_COMPACT);
  if (np[0] + np[1] == 0) return PM_OK;
  std::vector<LightDev> lh;
  light_devs(lights, nl, lh);
  DevBuf<LightDev> dl(nl);
  DevBuf<int64_t> dloff0(nl + 1), dloff1(nl + 1);
  DevBuf<pm_photon> slots0((size_t)np[0] * per[0]), slots1((size_t)np[1] * per[1]);
  DevBuf<uint32_t> cnt0(np[0]), cnt1(np[1]), off0(np[0]), off1(np[1]), tot(2);
  if (!dl.p || !dloff0.p || !dloff1.p || (np[0] && (!slots0.p || !cnt0.p || !off0.p)) ||
      (np[1] && (!slots1.p || !cnt1.p || !off1.p)) || !tot.p)
    return PM_ERR_OOM;
  PM_TRY_ST(hipMemcpyAsync(dl.p, lh.data(), sizeof(LightDev) * nl, hipMemcpyHostToDevice, s));
  PM_TRY_ST(hipMemcpyAsync(dloff0.p, loff[0].data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
  PM_TRY_ST(hipMemcpyAsync(dloff1.p, loff[1].data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
  PM_TRY_ST(hipMemsetAsync(tot.p, 0, 2 * sizeof(uint32_t), s));
  const PathSet A{dloff0.p, lo[0], np[0], params[0].caustics_mode ? 1 : 0, slots0.p, cnt0.p};
  const PathSet B{dloff1.p, lo[1], np[1], params[1].caustics_mode ? 1 : 0, slots1.p, cnt1.p};
  uint32_t t[2] = {0, 0};
  bool over[2] = {false, false};
  {
    // PH_TRACE: the trace WINDOW, the launch's start to the last compaction's
    // end (one stream); PH_COMPACT: the scans and compactions alone
    PhaseTimer win(PH_TRACE, s);
    PM_TRY_ST(launch_trace_sets(sc, dl.p, nl, A, B, params[0].max_depth, s));
    PhaseTimer tc(PH_COMPACT, s);
    if (np[0]) PM_TRY_ST(exclusive_scan_u32(cnt0.p, off0.p, np[0], tot.p, s));
    if (np[1]) PM_TRY_ST(exclusive_scan_u32(cnt1.p, off1.p, np[1], tot.p + 1, s));
    PM_TRY_ST(hipMemcpyAsync(t, tot.p, sizeof(t), hipMemcpyDeviceToHost, s));
    PM_TRY_ST(hipStreamSynchronize(s));
    const PathSet* sets[2] = {&A, &B};
    const uint32_t* offs[2] = {off0.p, off1.p};
    for (int k = 0; k < 2; k++) {
      if (!np[k]) continue;
      if ((int64_t)t[k] <= capacity[k] && d_out[k])
        PM_TRY_ST(launch_compact(sets[k]->slots, sets[k]->cnt, offs[k], np[k], d_out[k], s));
      else
        over[k] = true;
    }
  }
  PM_TRY_ST(hipStreamSynchronize(s));
  count[0] = t[0];
  count[1] = t[1];
  const int st = check_overflow(sc, s);
  if (st != PM_OK) return st;
  return (over[0] || over[1]) ? PM_ERR_CAPACITY : PM_OK;
}

// ------------------------------------------------------------------ stage 2
int pm_kdtree_build(pm_kd_photon* d, int64_t n, pm_box* bounds, void* stream) {
  if (n < 0 || (n > 0 && !d) || n >= kMaxMapPhotons) return PM_ERR_INVALID;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_PTR_DEVICE(alloc_scope, d);
  PM_PTR_DEVICE(alloc_scope, bounds);
  reset_phase(PH_KDBUILD);
  PhaseTimer tm(PH_KDBUILD, s);
  return map_err(kd_build_records(d, n, bounds, s));
}

static int map_create_runs(const RowRuns& runs, pm_photon_map** out, void* stream) {
  *out = nullptr;
  const int64_t n = rows_total(runs);
  if (n >= kMaxMapPhotons) return PM_ERR_INVALID;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  if (runs_elsewhere(runs, alloc_scope.dev)) return PM_ERR_DEVICE;
  pm_photon_map* m = new pm_photon_map;
  m->made_on = s;
  m->device = alloc_scope.dev;
  m->n = n;
  if (n > 0) {
    m->nodes.alloc(n);
    m->payload.alloc(n);
    DevBuf<float4> elems(n);
    if (!m->nodes.p || !m->payload.p || !elems.p) {
      delete m;
      return PM_ERR_OOM;
    }
    reset_phase(PH_KDBUILD);
    hipError_t e;
    {
      PhaseTimer tm(PH_KDBUILD, s);
      e = launch_elems_from_rows(runs, elems.p, m->payload.p, s);
      if (e == hipSuccess) e = kd_build(elems.p, n, m->nodes.p, s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      delete m;
      return map_err(e);
    }
  }
  *out = m;
  return PM_OK;
}

int pm_photon_map_create(const pm_photon* a, int64_t na, float pa, const pm_photon* b, int64_t nb, float pb,
                         pm_photon_map** out, void* stream) {
  if (!out || na < 0 || nb < 0 || (na > 0 && !a) || (nb > 0 && !b)) return PM_ERR_INVALID;
  return map_create_runs(runs_of(a, na, pa, b, nb, pb), out, stream);
}

int pm_photon_map_create_rows(const pm_photon_rows* a, float pa, const pm_photon_rows* b, float pb,
                              pm_photon_map** out, void* stream) {
  RowRuns runs;
  if (!out || !runs_of_rows(a, pa, runs) || !runs_of_rows(b, pb, runs)) return PM_ERR_INVALID;
  return map_create_runs(runs, out, stream);
}

int pm_photon_map_size(const pm_photon_map* m, int64_t* n) {
  if (!m || !n) return PM_ERR_INVALID;
  *n = m->n;
  return PM_OK;
}

int pm_photon_map_export(const pm_photon_map* m, pm_kd_photon* d_out, void* stream) {
  if (!m || (m->n > 0 && !d_out)) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, m);
  PM_PTR_DEVICE(alloc_scope, d_out);
  PM_TRY_ST(launch_map_export(m, d_out, s));
  return map_err(hipStreamSynchronize(s));
}

int pm_photon_map_destroy(pm_photon_map* m) {
  if (m) {
    // back to the pool of the stream it was built on (a map built on a side
    // stream every frame would otherwise hipMalloc anew each time)
    AllocStream pool(m->made_on, m->device);
    delete m;
  }
  return PM_OK;
}

// ---- sharded global-map build (kdshard.hip)
struct pm_kd_shard_plan {
  DevBuf<float4> elems, payload, top;
  DevBuf<uint8_t> sub;   // subtree of every element (255: a top node)
  DevBuf<uint32_t> boff;  // per-tile subtree starts (kd_shard_offsets), made by the first build
  std::mutex boff_mu;     // builds of one plan may run from several host threads (streams) at once
  int64_t n = 0;
  int L = 0;   // 0: not split
  std::vector<int64_t> sizes;
  hipStream_t made_on = nullptr;
  int device = 0;
};

static int plan_create_runs(const RowRuns& runs, int32_t world, pm_kd_shard_plan** out, void* stream) {
  *out = nullptr;
  const int64_t n = rows_total(runs);
  if (n >= kMaxMapPhotons) return PM_ERR_INVALID;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  if (runs_elsewhere(runs, alloc_scope.dev)) return PM_ERR_DEVICE;
  pm_kd_shard_plan* p = new pm_kd_shard_plan;
  p->made_on = s;
  p->device = alloc_scope.dev;
  p->n = n;
  hipError_t e = hipSuccess;
  if (n > 0) {
    p->elems.alloc(n);
    p->payload.alloc(n);
    if (!p->elems.p || !p->payload.p) {
      delete p;
      return PM_ERR_OOM;
    }
    reset_phase(PH_KDBUILD);
    PhaseTimer tm(PH_KDBUILD, s);
    e = launch_elems_from_rows(runs, p->elems.p, p->payload.p, s);
    const int L = shard_levels(world);
    if (e == hipSuccess && world > 1 && shard_ok(n, L)) {
      p->top.alloc((size_t)1 << L);
      if (!p->top.p) e = hipErrorOutOfMemory;
      if (e == hipSuccess) e = kd_shard_top(p->elems.p, n, L, p->top.p, p->sizes, s);
      if (e == hipSuccess) {
        p->sub.alloc(n);
        e = p->sub.p ? kd_shard_classify(p->elems.p, n, L, p->top.p, p->sub.p, s) : hipErrorOutOfMemory;
      }
      if (e == hipSuccess) p->L = L;
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete p;
    return map_err(e);
  }
  *out = p;
  return PM_OK;
}

int pm_kd_shard_plan_create(const pm_photon* a, int64_t na, float pa, const pm_photon* b, int64_t nb, float pb,
                            int32_t world, pm_kd_shard_plan** out, void* stream) {
  if (!out || na < 0 || nb < 0 || world < 1 || (na > 0 && !a) || (nb > 0 && !b)) return PM_ERR_INVALID;
  return plan_create_runs(runs_of(a, na, pa, b, nb, pb), world, out, stream);
}

int pm_kd_shard_plan_create_rows(const pm_photon_rows* a, float pa, const pm_photon_rows* b, float pb, int32_t world,
                                 pm_kd_shard_plan** out, void* stream) {
  RowRuns runs;
  if (!out || world < 1 || !runs_of_rows(a, pa, runs) || !runs_of_rows(b, pb, runs)) return PM_ERR_INVALID;
  return plan_create_runs(runs, world, out, stream);
}

int pm_kd_shard_subtrees(const pm_kd_shard_plan* p, int32_t* count, int64_t* sizes) {
  if (!p || !count) return PM_ERR_INVALID;
  *count = p->L > 0 ? (int32_t)p->sizes.size() : 0;
  if (sizes)
    for (int32_t j = 0; j < *count; j++) sizes[j] = p->sizes[j];
  return PM_OK;
}

int pm_kd_shard_build(pm_kd_shard_plan* p, int32_t j, int32_t* d_tags, void* stream) {
  if (!p || p->L == 0 || j < 0 || j >= (int32_t)p->sizes.size() || (p->sizes[j] > 0 && !d_tags))
    return PM_ERR_INVALID;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, p);
  PM_PTR_DEVICE(alloc_scope, d_tags);
  reset_phase(PH_KDBUILD);
  hipError_t e;
  {
    PhaseTimer tm(PH_KDBUILD, s);
    e = hipSuccess;
    {
      // the offsets are made once, by the first build (kd_shard_offsets
      // synchronises its stream, so a build on another stream may use them
      // as soon as the lock is released)
      std::lock_guard<std::mutex> lk(p->boff_mu);
      if (!p->boff.p) {
        p->boff.alloc((size_t)kd_shard_tiles(p->n) * p->sizes.size());
        e = p->boff.p ? kd_shard_offsets(p->sub.p, p->n, (int)p->sizes.size(), p->sizes.data(), p->boff.p, s)
                      : hipErrorOutOfMemory;
        if (e != hipSuccess) p->boff.reset();
      }
    }
    if (e == hipSuccess) e = kd_shard_subtree(p->elems.p, p->sub.p, p->boff.p, p->n, j, p->sizes[j], d_tags, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return map_err(e);
}

int pm_photon_map_create_sharded(pm_kd_shard_plan* p, const int32_t* subs, pm_photon_map** out, void* stream) {
  if (!p || !out || (p->L > 0 && !subs)) return PM_ERR_INVALID;
  *out = nullptr;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, p);
  PM_PTR_DEVICE(alloc_scope, subs);
  pm_photon_map* m = new pm_photon_map;
  m->made_on = s;
  m->device = alloc_scope.dev;
  m->n = p->n;
  hipError_t e = hipSuccess;
  if (p->n > 0) {
    m->nodes.alloc(p->n);
    if (!m->nodes.p) {
      delete m;
      return PM_ERR_OOM;
    }
    reset_phase(PH_KDBUILD);
    {
      PhaseTimer tm(PH_KDBUILD, s);
      if (p->L > 0)
        e = kd_shard_assemble(p->elems.p, p->top.p, p->L, subs, p->sizes, m->nodes.p, s);
      else
        e = kd_build(p->elems.p, p->n, m->nodes.p, s);
    }
    std::swap(m->payload.p, p->payload.p);   // the plan's payload moves into the map
    std::swap(m->payload.n, p->payload.n);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess || (p->n > 0 && !m->payload.p)) {
    delete m;
    return e != hipSuccess ? map_err(e) : PM_ERR_INVALID;   // a plan's payload moves once
  }
  *out = m;
  return PM_OK;
}

int pm_kd_shard_plan_destroy(pm_kd_shard_plan* p) {
  if (p) {
    AllocStream pool(p->made_on, p->device);
    delete p;
  }
  return PM_OK;
}

// ---- distributed top selection (kdshard.hip, KdTopSel)
struct pm_kd_top_sel {
  KdTopSel sel;
  int64_t n_total = 0;
  bool split = false;
  hipStream_t made_on = nullptr;
  int device = 0;
};

int pm_kd_top_sel_create(const pm_photon* a, int64_t na, int64_t a_first, const pm_photon* b, int64_t nb,
                         int64_t b_first, int64_t n_total, int32_t world, pm_kd_top_sel** out, void* stream) {
  if (!out || na < 0 || nb < 0 || a_first < 0 || b_first < 0 || world < 1 || (na > 0 && !a) || (nb > 0 && !b) ||
      n_total < 0 || n_total >= kMaxMapPhotons || a_first + na > n_total || b_first + nb > n_total)
    return PM_ERR_INVALID;
  *out = nullptr;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_PTR_DEVICE(alloc_scope, a);
  PM_PTR_DEVICE(alloc_scope, b);
  pm_kd_top_sel* h = new pm_kd_top_sel;
  h->made_on = s;
  h->device = alloc_scope.dev;
  h->n_total = n_total;
  const int L = shard_levels(world);
  hipError_t e = hipSuccess;
  if (world > 1 && shard_ok(n_total, L)) {
    h->split = true;
    reset_phase(PH_KDBUILD);
    PhaseTimer tm(PH_KDBUILD, s);
    e = h->sel.init(a, na, a_first, b, nb, b_first, n_total, L, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete h;
    return map_err(e);
  }
  *out = h;
  return PM_OK;
}

int pm_kd_top_sel_step(pm_kd_top_sel* h, int64_t* d_buf, int64_t* count, int32_t* op, void* stream) {
  if (!h || !d_buf || !count || !op) return PM_ERR_INVALID;
  *count = 0;
  *op = 0;
  if (!h->split) return PM_OK;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, h);
  PM_PTR_DEVICE(alloc_scope, d_buf);
  reset_phase(PH_KDBUILD);
  int o = 0;
  hipError_t e;
  {
    PhaseTimer tm(PH_KDBUILD, s);
    e = h->sel.step(d_buf, count, &o, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  *op = o;
  return map_err(e);
}

static int plan_from_sel_runs(const pm_kd_top_sel* h, const RowRuns& runs, pm_kd_shard_plan** out, void* stream) {
  const int64_t n = rows_total(runs);
  if (n != h->n_total || (h->split && h->sel.level < h->sel.L))
    return PM_ERR_INVALID;   // the gathered map, after the last step
  *out = nullptr;
  int st = require_device();
  if (st != PM_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, h);
  if (runs_elsewhere(runs, alloc_scope.dev)) return PM_ERR_DEVICE;
  pm_kd_shard_plan* p = new pm_kd_shard_plan;
  p->made_on = s;
  p->device = alloc_scope.dev;
  p->n = n;
  hipError_t e = hipSuccess;
  if (n > 0) {
    p->elems.alloc(n);
    p->payload.alloc(n);
    if (!p->elems.p || !p->payload.p) {
      delete p;
      return PM_ERR_OOM;
    }
    reset_phase(PH_KDBUILD);
    PhaseTimer tm(PH_KDBUILD, s);
    if (!h->split) {
      e = launch_elems_from_rows(runs, p->elems.p, p->payload.p, s);
    } else {
      // elements, payload and subtrees in one pass over the gathered photons
      // (the selection's top nodes hold the split coordinates), then the top
      // nodes' full positions from the elements
      const int L = h->sel.L;
      p->top.alloc((size_t)1 << L);
      p->sub.alloc(n);
      if (!p->top.p || !p->sub.p) e = hipErrorOutOfMemory;
      if (e == hipSuccess) e = kd_shard_elems_classify(runs, h->sel.top.p, L, p->elems.p, p->payload.p, p->sub.p, s);
      if (e == hipSuccess)
        e = hipMemcpyAsync(p->top.p, h->sel.top.p, sizeof(float4) * (((size_t)1 << L) - 1), hipMemcpyDeviceToDevice,
                           s);
      if (e == hipSuccess) e = kd_shard_top_fix(p->elems.p, p->top.p, L, s);
      if (e == hipSuccess) {
        p->sizes = h->sel.seg;
        p->L = L;
      }
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete p;
    return map_err(e);
  }
  *out = p;
  return PM_OK;
}

int pm_kd_shard_plan_create_from_sel(const pm_kd_top_sel* h, const pm_photon* a, int64_t na, float pa,
                                     const pm_photon* b, int64_t nb, float pb, pm_kd_shard_plan** out,
                                     void* stream) {
  if (!h || !out || na < 0 || nb < 0 || (na > 0 && !a) || (nb > 0 && !b)) return PM_ERR_INVALID;
  return plan_from_sel_runs(h, runs_of(a, na, pa, b, nb, pb), out, stream);
}

int pm_kd_shard_plan_create_from_sel_rows(const pm_kd_top_sel* h, const pm_photon_rows* a, float pa,
                                          const pm_photon_rows* b, float pb, pm_kd_shard_plan** out, void* stream) {
  RowRuns runs;
  if (!h || !out || !runs_of_rows(a, pa, runs) || !runs_of_rows(b, pb, runs)) return PM_ERR_INVALID;
  return plan_from_sel_runs(h, runs, out, stream);
}

int pm_kd_top_sel_destroy(pm_kd_top_sel* h) {
  if (h) {
    AllocStream pool(h->made_on, h->device);
    delete h;
  }
  return PM_OK;
}

int pm_knn(const pm_photon_map* m, const pm_float3* q, int64_t nq, int32_t k, float max_radius, int32_t* ids,
           float* d2, float* maxd2, void* stream) {
  if (!m || nq < 0 || k < 1 || k > 256 || (nq > 0 && (!q || !ids)) || !(max_radius >= 0.f)) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, m);
  PM_PTR_DEVICE(alloc_scope, q);
  PM_PTR_DEVICE(alloc_scope, ids);
  PM_TRY_ST(launch_knn(m, q, nq, k, max_radius, ids, d2, maxd2, s));
  return map_err(hipStreamSynchronize(s));
}

int pm_gather(const pm_photon_map* m, const pm_float3* pts, const float* brdf, int64_t nq, pm_float3* out,
              void* stream) {
  if (!m || nq < 0 || (nq > 0 && (!pts || !brdf || !out))) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, m);
  PM_PTR_DEVICE(alloc_scope, pts);
  PM_PTR_DEVICE(alloc_scope, out);
  reset_phase(PH_GATHER);
  PhaseTimer tm(PH_GATHER, s);
  return map_err(launch_gather_api(m, pts, brdf, nq, out, s, kKNearest));
}

int pm_gather_k(const pm_photon_map* m, const pm_float3* pts, const float* brdf, int64_t nq, int32_t k,
                pm_float3* out, void* stream) {
  if (!m || nq < 0 || k < 1 || k > 256 || (nq > 0 && (!pts || !brdf || !out))) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, m);
  PM_PTR_DEVICE(alloc_scope, pts);
  PM_PTR_DEVICE(alloc_scope, out);
  reset_phase(PH_GATHER);
  PhaseTimer tm(PH_GATHER, s);
  return map_err(launch_gather_api(m, pts, brdf, nq, out, s, k));
}

int pm_camera_setup(pm_float3 from, pm_float3 at, pm_float3 up, float fovy, int32_t w, int32_t h, pm_camera* o) {
  if (!o || w <= 0 || h <= 0) return PM_ERR_INVALID;
  // setupCamera (ray-tracer/src/hostCode.cu:100-108), owl vec3f arithmetic
  struct V {
    float x, y, z;
  };
  auto sub = [](V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; };
  auto add = [](V a, V b) { return V{a.x + b.x, a.y + b.y, a.z + b.z}; };
  auto smul = [](float s, V a) { return V{s * a.x, s * a.y, s * a.z}; };
  auto dot = [](V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
  auto cross = [](V a, V b) { return V{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; };
  auto norm = [&](V v) {
    const float r = 1.0f / std::sqrt(dot(v, v));
    return V{v.x * r, v.y * r, v.z * r};
  };
  const float aspect = (float)w / (float)h;
  const float cf = std::cos(fovy);
  const V F{from.x, from.y, from.z}, A{at.x, at.y, at.z}, U{up.x, up.y, up.z};
  V d00 = norm(sub(A, F));
  const V du = smul(cf * aspect, norm(cross(d00, U)));
  const V dv = smul(cf, norm(cross(du, d00)));
  d00 = sub(d00, smul(0.5f, add(du, dv)));
  o->pos = from;
  o->dir_00 = {d00.x, d00.y, d00.z};
  o->dir_du = {du.x, du.y, du.z};
  o->dir_dv = {dv.x, dv.y, dv.z};
  return PM_OK;
}

static bool render_params_ok(const pm_scene* sc, const pm_render_params* P, const pm_light* lights, int32_t nl) {
  return sc && P && nl >= 0 && (nl == 0 || lights) && P->width > 0 && P->height > 0 && P->samples_per_pixel > 0 &&
         P->max_depth >= 0 && !(P->tile_count > 1 && (P->tile_rank < 0 || P->tile_rank >= P->tile_count)) &&
         P->caustic_k >= 0 && P->caustic_k <= 256;
}

int pm_render_begin(pm_scene* sc, const pm_render_params* P, const pm_light* lights, int32_t nl, pm_render_job** out,
                    void* stream) {
  if (!out) return PM_ERR_INVALID;
  *out = nullptr;
  if (!render_params_ok(sc, P, lights, nl)) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, sc);
  reset_phase(PH_PATHS);
  pm_render_job* J = render_job_new(sc, s);
  if (!J) return PM_ERR_OOM;
  hipError_t e = render_begin(sc, P, lights, nl, J, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    render_job_delete(J);
    return map_err(e);
  }
  const int st = check_overflow(sc, s);
  if (st != PM_OK) {
    render_job_delete(J);
    return st;
  }
  *out = J;
  return PM_OK;
}

int pm_render_gather_caustic(pm_render_job* J, const pm_photon_map* cmap, void* stream) {
  if (!J || !cmap || render_job_finished(J) || render_job_caustic_map(J)) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  if (render_job_device(J) != alloc_scope.dev) return PM_ERR_DEVICE;
  PM_SAME_DEVICE(alloc_scope, cmap);
  reset_phase(PH_GATHER);
  {
    PhaseTimer tm(PH_GATHER, s);
    PM_TRY_ST(render_gather_caustic(J, cmap, s));
  }
  return PM_OK;
}

int pm_render_finish(pm_render_job* J, const pm_photon_map* gmap, const pm_photon_map* cmap, uint32_t* rgba,
                     float* rgb, void* stream) {
  if (!J || !gmap || !rgba || render_job_finished(J)) return PM_ERR_INVALID;
  const pm_photon_map* early = render_job_caustic_map(J);
  if (early ? (cmap && cmap != early) : !cmap) return PM_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  if (render_job_device(J) != alloc_scope.dev) return PM_ERR_DEVICE;
  PM_SAME_DEVICE(alloc_scope, gmap);
  PM_SAME_DEVICE(alloc_scope, cmap);
  PM_PTR_DEVICE(alloc_scope, rgba);
  PM_PTR_DEVICE(alloc_scope, rgb);
  reset_phase(PH_GATHER); reset_phase(PH_RESOLVE); reset_phase(PH_GATHER_GLOBAL);
  render_job_mark_finished(J);
  PM_TRY_ST(render_finish(J, gmap, cmap, rgba, rgb, s));
  PM_TRY_ST(hipStreamSynchronize(s));
  {
    std::lock_guard<std::mutex> lk(g_phase_mu);
    g_render_stats = render_job_stats(J);
  }
  return check_overflow(render_job_scene(J), s);
}

int pm_render_job_queries(const pm_render_job* J, int32_t which, float* d_queries, float* d_results,
                          int64_t capacity, int64_t* count, void* stream) {
  if (!J || !count || (which != 0 && which != 1) || capacity < 0) return PM_ERR_INVALID;
  const float4 *q = nullptr, *res = nullptr;
  int64_t n = 0;
  render_job_queries(J, which, &q, &res, &n);
  *count = n;
  if (!d_queries && !d_results) return PM_OK;   // size query
  if (capacity < n) return PM_ERR_CAPACITY;
  if (d_results && !render_job_finished(J)) return PM_ERR_INVALID;   // no results before finish
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  if (render_job_device(J) != alloc_scope.dev) return PM_ERR_DEVICE;
  PM_PTR_DEVICE(alloc_scope, d_queries);
  PM_PTR_DEVICE(alloc_scope, d_results);
  if (n == 0) return PM_OK;
  if (d_queries) PM_TRY_ST(hipMemcpyAsync(d_queries, q, sizeof(float4) * n, hipMemcpyDeviceToDevice, s));
  if (d_results) PM_TRY_ST(hipMemcpyAsync(d_results, res, sizeof(float4) * n, hipMemcpyDeviceToDevice, s));
  return map_err(hipStreamSynchronize(s));
}

int pm_render_job_destroy(pm_render_job* J) {
  render_job_delete(J);
  return PM_OK;
}

int pm_render(pm_scene* sc, const pm_render_params* P, const pm_light* lights, int32_t nl,
              const pm_photon_map* gmap, const pm_photon_map* cmap, uint32_t* rgba, float* rgb, void* stream) {
  if (!render_params_ok(sc, P, lights, nl) || !gmap || !cmap || !rgba) return PM_ERR_INVALID;
  pm_render_job* J = nullptr;
  int st = pm_render_begin(sc, P, lights, nl, &J, stream);
  if (st != PM_OK) return st;
  st = pm_render_finish(J, gmap, cmap, rgba, rgb, stream);
  render_job_delete(J);
  return st;
}

int pm_photon_view(pm_scene* sc, const pm_photon* d_photons, int64_t n, const pm_viewer_params* P, uint32_t* d_rgba,
                   void* stream) {
  if (!sc || !P || n < 0 || (n > 0 && !d_photons) || n > INT32_MAX || P->width <= 0 || P->height <= 0 || !d_rgba)
    return PM_ERR_INVALID;
  if (int st = require_device()) return st;
  hipStream_t s = (hipStream_t)stream;
  AllocStream alloc_scope(s);
  PM_SAME_DEVICE(alloc_scope, sc);
  PM_PTR_DEVICE(alloc_scope, d_photons);
  PM_PTR_DEVICE(alloc_scope, d_rgba);
  PM_TRY_ST(photon_view(sc, d_photons, n, *P, d_rgba, s));
  return check_overflow(sc, s);
}

int pm_photons_quantize(pm_photon* d, int64_t n, void* stream) {
  if (n < 0 || (n > 0 && !d)) return PM_ERR_INVALID;
  if (int st = require_device()) return st;
  AllocStream alloc_scope((hipStream_t)stream);
  PM_PTR_DEVICE(alloc_scope, d);
  return map_err(photons_quantize(d, n, (hipStream_t)stream));
}

int pm_render_stats_get(pm_render_stats* o) {
  if (!o) return PM_ERR_INVALID;
  std::lock_guard<std::mutex> lk(g_phase_mu);
  *o = g_render_stats;
  return PM_OK;
}

}  // extern "C"
