/*
 * pm.h — C-ABI of the MI355X-native photon-mapping hot path (libpm_hip.so).
 *
 * This is the drop-in boundary for the three reference boundaries named in
 * SURVEY.md §8(b):
 *   B1  process / CLI contract  -> the `photon-mapping`, `photonMapping`,
 *       `rayTracer` binaries built on top of this library (tools/).
 *   B2  OWL/OptiX device-program ABI (photon-mapping/include/deviceCode.h:8-43,
 *       ray-tracer/include/deviceCode.h:10-64, common/src/mesh.h:15-20)
 *       -> pm_scene_*, pm_trace_photons, pm_render.
 *   B3  cudaKDTree template API (ray-tracer/src/hostCode.cu:94-95,
 *       ray-tracer/cuda/shading.h:11-18) -> pm_kdtree_build, pm_knn.
 *
 * Conventions (all entry points):
 *   - extern "C", plain pointers and sizes; no torch / HIP types.
 *   - every call returns an int status (PM_OK == 0); no aborts.
 *   - pointers prefixed d_ are DEVICE pointers (caller-owned, e.g. torch
 *     tensors or hipMalloc); h_ / plain pointers are host memory.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *     Calls that return a host-visible scalar (counts) synchronise the stream.
 *   - devices: a call that takes a stream runs on THAT stream's device. For
 *     the duration of the call it makes that device current for the calling
 *     host thread (a thread that never chose a device is on device 0) and
 *     restores the previous one on return, so a side thread driving GPU r's
 *     stream allocates and launches on GPU r. A NULL stream means the calling
 *     thread's current device. Calls without a stream (pm_scene_create,
 *     pm_device_alloc, ...) use the calling thread's current device.
 *   - handles (pm_scene, pm_photon_map, pm_kd_shard_plan, pm_render_job) own
 *     their device memory and belong to the device they were created on;
 *     passing one, or a caller's device buffer, with a stream of another
 *     device returns PM_ERR_DEVICE (nothing is launched).
 *   - single-threaded per handle.
 * There is NO CPU fallback: every compute entry point runs HIP kernels for
 * gfx950 and fails with PM_ERR_NO_DEVICE when no GPU is present.
 */
#ifndef PM_H_
#define PM_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PM_ABI_VERSION 6

enum pm_status {
  PM_OK = 0,
  PM_ERR_INVALID = 1,     /* bad argument / shape                          */
  PM_ERR_HIP = 2,         /* HIP runtime error                             */
  PM_ERR_OOM = 3,         /* device allocation failed                      */
  PM_ERR_NO_DEVICE = 4,   /* no gfx950 device visible                      */
  PM_ERR_IO = 5,          /* file could not be opened / parsed             */
  PM_ERR_CAPACITY = 6,    /* output buffer too small (count still written) */
  PM_ERR_OVERFLOW = 7,    /* traversal stack overflow inside a kernel      */
  PM_ERR_DEVICE = 8       /* handle / buffer on another device than the stream */
};

typedef struct { float x, y, z; } pm_float3;
typedef struct { int32_t x, y, z; } pm_int3;

/* common/src/mesh.h:6-12  (28 B) */
typedef struct {
  pm_float3 albedo;
  float diffuse, specular, transmission, refraction_idx;
} pm_material;

/* common/src/mesh.h:22-27 (Mesh) + mesh.h:15-20 (TrianglesGeomData). */
typedef struct {
  const pm_float3* vertices;   /* host */
  int32_t num_vertices;
  const pm_int3* indices;      /* host, per-mesh vertex indices */
  int32_t num_triangles;
  pm_material material;
} pm_mesh;

/* common/src/world.h:11-27 (LightSource, 64 B). POINT_LIGHT is the
 * reference's emitter (pointLightRayGen). SQUARE_LIGHT is declared by the
 * reference but never emitted there; this build defines it: the photon origin
 * is uniform on the side_length square centred at pos, perpendicular to
 * normal (basis t1 = normalize(cross(a, n)), t2 = cross(n, t1), a = (0,1,0) if
 * |n.x| > 0.9 else (1,0,0); two RNG draws), the direction a cosine lobe about
 * normal. lights.txt lines with 11 values "x y z r g b power nx ny nz side"
 * load as SQUARE_LIGHT. The final-gather render lights every source as a point
 * at pos, as the reference's direct-light loop does. */
enum { PM_POINT_LIGHT = 0, PM_SQUARE_LIGHT = 1 };
typedef struct {
  int32_t source_type;
  pm_float3 pos;
  double power;
  pm_float3 rgb;
  pm_float3 normal;
  double side_length;
  int32_t num_photons;
} pm_light;

/* photon-mapping/include/photon.h:5-11 (40 B) — stage-1 output record. */
typedef struct {
  pm_float3 pos;
  pm_float3 dir;
  int32_t power;               /* never written by the reference */
  pm_float3 color;
} pm_photon;

/* ray-tracer/include/photon.h:11-21 (44 B) — cudaKDTree data record. */
typedef struct {
  pm_float3 pos;
  pm_float3 dir;
  pm_float3 color;
  float power;
  uint8_t quantized_normal[3];
  uint8_t split_dim;
} pm_kd_photon;

/* cukd::box_t<float3> */
typedef struct { pm_float3 lower, upper; } pm_box;

/* common/src/camera.h:5-10 */
typedef struct { pm_float3 pos, dir_00, dir_du, dir_dv; } pm_camera;

/* A ray for the traversal entry points (owl::Ray: origin, direction, tmin, tmax). */
typedef struct { pm_float3 origin; float tmin; pm_float3 direction; float tmax; } pm_ray;
/* Closest-hit record: t, mesh (OWL geom index) and primitive (optixGetPrimitiveIndex). */
typedef struct { float t; int32_t mesh; int32_t prim; int32_t tri; } pm_hit;

/* ---- library / device ---------------------------------------------------- */
int pm_abi_version(void);
const char* pm_status_string(int status);
/* Number of visible HIP devices (0 on a host without a GPU; never fails). */
int pm_device_count(int32_t* count);
/* Microseconds of the last kernel(s) of a phase, measured with hipEvents on
 * the stream the kernels ran on, as seen by the calling host thread (each
 * thread reads the phases of its own last calls). phase: 0 trace, 1
 * compaction, 2 kd-build, 3 render-paths, 4 knn-gather (all), 5 resolve, 6
 * bvh-build, 7 the global-map gather launch alone (the dominant kernel). */
int pm_last_phase_us(int32_t phase, double* us);
/* Device memory for callers without HIP headers (the CLI, cgo / JNI / ctypes
 * bindings): hipMalloc / hipFree / synchronous hipMemcpy on the current device. */
int pm_device_alloc(size_t bytes, void** d_ptr);
int pm_device_free(void* d_ptr);
int pm_copy_to_device(void* d_dst, const void* h_src, size_t bytes);
int pm_copy_to_host(void* h_dst, const void* d_src, size_t bytes);
/* The library's caching allocator on `device` (-1: all devices): bytes held by
 * live blocks (owned by handles or in use by a running call) and by idle
 * pooled blocks kept for reuse. Steady-state frames do not grow either. */
int pm_device_pool_stats(int32_t device, int64_t* live_bytes, int64_t* cached_bytes);

/* ---- scene (world.cpp:3-58 loadGeometry; OptiX GAS+IAS -> HIP LBVH) ------- */
typedef struct pm_scene pm_scene;
typedef struct {
  int64_t num_triangles;
  int64_t num_nodes;          /* BVH4 nodes (collapsed from the binary LBVH) */
  int32_t num_meshes;
  int32_t max_depth;          /* BVH4 levels */
  pm_box bounds;
} pm_scene_stats;

int pm_scene_create(const pm_mesh* meshes, int32_t num_meshes, pm_scene** out);
int pm_scene_stats_get(const pm_scene* scene, pm_scene_stats* out);
int pm_scene_destroy(pm_scene* scene);
/* Closest hit (optixTrace without any-hit) for n rays; miss -> t=+inf, ids -1. */
int pm_scene_intersect(pm_scene* scene, const pm_ray* d_rays, int64_t n,
                       pm_hit* d_hits, void* stream);
/* Shadow rays (TERMINATE_ON_FIRST_HIT): d_occluded[i] = 1 if any hit in (tmin,tmax). */
int pm_scene_occluded(pm_scene* scene, const pm_ray* d_rays, int64_t n,
                      int32_t* d_occluded, void* stream);

/* ---- stage 1: photon emission + bounce ----------------------------------
 * photon-mapping/src/hostCode.cu:72-138 (runPointLightRayGen, runNormal,
 * runCaustics), photon-mapping/cuda/deviceCode.cu:10-136.
 * Output order is deterministic: (light, photon id, bounce); the reference's
 * atomicAdd order (deviceCode.cu:11) is nondeterministic, so parity is on this
 * canonical order (a permutation of the reference's multiset). */
typedef struct {
  int64_t casted_photons;      /* photon-mapper.casted_{diffuse,caustics}_photons */
  int32_t max_depth;           /* photon-mapper.max_depth */
  int32_t caustics_mode;       /* 0 = runNormal, 1 = runCaustics */
  int32_t shard_rank;          /* photon-index sharding across GPUs (0..count-1) */
  int32_t shard_count;         /* 1 = whole job */
} pm_trace_params;

/* Photons launched per light: n_L = int(P_L * int(casted / sum P)) (hostCode.cu:86,102-110). */
int pm_photons_per_light(const pm_light* lights, int32_t num_lights,
                         int64_t casted_photons, int64_t* h_counts /* num_lights */);
/* Worst-case number of stored photons for this shard (capacity to allocate). */
int pm_trace_capacity(const pm_light* lights, int32_t num_lights,
                      const pm_trace_params* params, int64_t* capacity);
/* Trace and compact. d_out receives *count photons (device). If capacity is
 * too small PM_ERR_CAPACITY is returned with *count set to the needed size. */
int pm_trace_photons(pm_scene* scene, const pm_light* lights, int32_t num_lights,
                     const pm_trace_params* params, pm_photon* d_out,
                     int64_t capacity, int64_t* count, void* stream);

/* Both photon sets of a frame (runNormal + runCaustics, hostCode.cu:112-138)
 * in ONE persistent launch: params[0] / params[1] (each its own casted count,
 * mode and shard) trace into d_out[0] / d_out[1] exactly the photons, order,
 * counts (count[k]) and PM_ERR_CAPACITY behaviour of two pm_trace_photons
 * calls. Set 0's photons are taken first, so set 1's fill the tail of its
 * long paths (the frame passes the diffuse set first, the caustic set second).
 * Phases: 0 = the trace window (the launch through the last compaction), 1 =
 * the compactions. Sets whose deposit slots exceed one chunk, or whose
 * max_depth differ, are traced one after the other (same results). */
int pm_trace_photon_sets(pm_scene* scene, const pm_light* lights, int32_t num_lights,
                         const pm_trace_params* params /* [2] */, pm_photon* const* d_out /* [2] */,
                         const int64_t* capacity /* [2] */, int64_t* count /* [2] */, void* stream);

/* ---- stage 2a: kd-tree (cukd::buildTree, hostCode.cu:94-95) -------------- */
/* In place: reorders d_photons into a left-balanced implicit kd-tree (children
 * 2i+1, 2i+2) with split_dim set per node (has_explicit_dim, photon.h:23-40);
 * writes the point bounds to *d_bounds (device) if non-NULL. */
int pm_kdtree_build(pm_kd_photon* d_photons, int64_t n, pm_box* d_bounds, void* stream);

/* Photon map = kd-tree + gather payload, built from stage-1 photon arrays the
 * way loadPhotons does (hostCode.cu:54-99): map = a[0..na) (power_a) ++
 * b[0..nb) (power_b). Original index = position in that concatenation.
 * A NaN position coordinate is taken as +inf by every tree build (this one,
 * pm_kdtree_build, the sharded build): such a photon sorts last and is never
 * within a gather radius (cukd leaves NaN undefined). */
typedef struct pm_photon_map pm_photon_map;
int pm_photon_map_create(const pm_photon* d_a, int64_t na, float power_a,
                         const pm_photon* d_b, int64_t nb, float power_b,
                         pm_photon_map** out, void* stream);
/* Photon ROWS: the photons of one set as nseg segments of row_floats-float
 * rows in one device buffer, concatenated in segment order: segment s is rows
 * [seg_row0[s], seg_row0[s] + seg_count[s]) of d_rows; the position is floats
 * 0..2 of a row and the colour floats color_offset..color_offset+2. A
 * pm_photon array is {10, 7, one segment}. The N > 1 exchange
 * all-gathers (position, colour) rows padded to the largest rank's count into
 * one buffer, rank r at rows [r m, r m + n_r): {6, 3, world segments} hands that
 * buffer to the maps as it is, with no compaction and no re-expansion to
 * pm_photon. Original index = position in the concatenation, as for the
 * pm_photon calls (a ++ b). A NULL set has no photons. */
#define PM_ROWS_MAX_SEGS 32
typedef struct {
  const float* d_rows;
  int32_t row_floats;          /* >= 6 */
  int32_t color_offset;        /* >= 3, color_offset + 3 <= row_floats */
  int32_t nseg;                /* 0 .. PM_ROWS_MAX_SEGS */
  int32_t reserved;            /* 0 */
  int64_t seg_row0[PM_ROWS_MAX_SEGS];
  int64_t seg_count[PM_ROWS_MAX_SEGS];
} pm_photon_rows;
/* pm_photon_map_create over photon rows (the same map as over the concatenated
 * pm_photon arrays, bit for bit). */
int pm_photon_map_create_rows(const pm_photon_rows* a, float power_a, const pm_photon_rows* b, float power_b,
                              pm_photon_map** out, void* stream);
int pm_photon_map_size(const pm_photon_map* map, int64_t* n);
/* Copy the map out in kd order as reference kd records (power, split_dim set). */
int pm_photon_map_export(const pm_photon_map* map, pm_kd_photon* d_out, void* stream);
int pm_photon_map_destroy(pm_photon_map* map);

/* ---- stage 2a across G ranks (replaces the replicated buildTree)
 * Every rank holds the same all-gathered photons (pm_photon_map_create's
 * arguments). pm_kd_shard_plan_create selects the top L = min(ceil(log2 G) + 1, 5)
 * levels of the global tree on every rank; the caller deals the 2^L subtrees
 * to ranks (any deterministic assignment, e.g. balanced by size), each rank
 * builds its own (pm_kd_shard_build: one 4-B tag per node, original index << 2
 * | split dimension, in the subtree's own implicit layout), the caller
 * all-gathers them, concatenated in subtree order, and
 * pm_photon_map_create_sharded places them (positions from the photons). The map equals
 * pm_photon_map_create's bit for bit. A plan with 0 subtrees (map too small
 * to split, or G == 1) builds the whole tree in pm_photon_map_create_sharded. */
typedef struct pm_kd_shard_plan pm_kd_shard_plan;
int pm_kd_shard_plan_create(const pm_photon* d_a, int64_t na, float power_a,
                            const pm_photon* d_b, int64_t nb, float power_b,
                            int32_t world, pm_kd_shard_plan** out, void* stream);
/* *count = number of subtrees (2^L or 0); h_sizes (count entries) may be NULL. */
int pm_kd_shard_subtrees(const pm_kd_shard_plan* plan, int32_t* count, int64_t* h_sizes);
/* Builds of different subtrees of one plan may run at the same time from
 * several host threads, each on its own stream (the rank's subtrees side by
 * side); the call returns when its stream is done. */
int pm_kd_shard_build(pm_kd_shard_plan* plan, int32_t subtree, int32_t* d_tags /* size */,
                      void* stream);
/* d_tags: all subtrees' tags in subtree order (NULL if count == 0). */
int pm_photon_map_create_sharded(pm_kd_shard_plan* plan, const int32_t* d_tags,
                                 pm_photon_map** out, void* stream);
/* pm_kd_shard_plan_create over photon rows (see pm_photon_rows). */
int pm_kd_shard_plan_create_rows(const pm_photon_rows* a, float power_a, const pm_photon_rows* b, float power_b,
                                 int32_t world, pm_kd_shard_plan** out, void* stream);
int pm_kd_shard_plan_destroy(pm_kd_shard_plan* plan);

/* Distributed top selection: the same top L levels and subtree sizes as
 * pm_kd_shard_plan_create, computed from every rank's OWN photons before the
 * exchange (each rank reads 1/G of the elements; no photon crosses ranks).
 * d_a / d_b: this rank's photons of the two sets; a_first / b_first: the index
 * of d_a[0] / d_b[0] in the gathered map (diffuse ++ caustic, rank order, so
 * b_first = all ranks' diffuse count + the caustic count of lower ranks);
 * n_total: the gathered map's size. Drive it with pm_kd_top_sel_step until
 * *op == 0: each call consumes the reduction of the previous pass and issues
 * the next into d_buf (int64, capacity PM_KD_TOP_SEL_BUF), whose first *count
 * entries the caller reduces in place across all ranks -- *op 1: SUM, 2: MIN --
 * before the next call (every rank runs the same number of steps). Then
 * pm_kd_shard_plan_create_from_sel takes the gathered photons (as
 * pm_kd_shard_plan_create would) and the rest is unchanged. A selection with
 * no split (G == 1 or a small map) finishes at once and gives a plan with 0
 * subtrees. */
#define PM_KD_TOP_SEL_BUF 4096
typedef struct pm_kd_top_sel pm_kd_top_sel;
int pm_kd_top_sel_create(const pm_photon* d_a, int64_t na, int64_t a_first,
                         const pm_photon* d_b, int64_t nb, int64_t b_first,
                         int64_t n_total, int32_t world, pm_kd_top_sel** out, void* stream);
int pm_kd_top_sel_step(pm_kd_top_sel* sel, int64_t* d_buf, int64_t* count, int32_t* op,
                       void* stream);
int pm_kd_shard_plan_create_from_sel(const pm_kd_top_sel* sel,
                                     const pm_photon* d_a, int64_t na, float power_a,
                                     const pm_photon* d_b, int64_t nb, float power_b,
                                     pm_kd_shard_plan** out, void* stream);
/* the same over the gathered photon rows (the exchange's padded buffer) */
int pm_kd_shard_plan_create_from_sel_rows(const pm_kd_top_sel* sel, const pm_photon_rows* a, float power_a,
                                          const pm_photon_rows* b, float power_b, pm_kd_shard_plan** out,
                                          void* stream);
int pm_kd_top_sel_destroy(pm_kd_top_sel* sel);

/* ---- stage 2b: kNN + radiance estimate ----------------------------------
 * cukd::stackBased::knn<HeapCandidateList<k>> (shading.h:11-18): exact k
 * nearest photons with d^2 < max_radius^2, ordered by (d^2, original index);
 * empty slots id -1. d_maxd2[q] = k-th d^2, or max_radius^2 if fewer found.
 * d_ids / d_d2 are [nq][k] (d_d2 may be NULL). k <= 256. */
int pm_knn(const pm_photon_map* map, const pm_float3* d_queries, int64_t nq,
           int32_t k, float max_radius, int32_t* d_ids, float* d_d2,
           float* d_maxd2, void* stream);
/* gatherPhotons (shading.h:93-121), k = 50, radius 100, cone filter 1.1. */
int pm_gather(const pm_photon_map* map, const pm_float3* d_points,
              const float* d_brdf, int64_t nq, pm_float3* d_out, void* stream);
/* The same estimate over the k nearest (1 <= k <= 256; SURVEY §8d config 5
 * gathers caustics with k = 200). k = 50 is pm_gather. */
int pm_gather_k(const pm_photon_map* map, const pm_float3* d_points,
                const float* d_brdf, int64_t nq, int32_t k, pm_float3* d_out, void* stream);

/* ---- stage 2c: render (simpleRayGen, ray-tracer/cuda/deviceCode.cu:25-231) */
typedef struct {
  int32_t width, height;       /* ray-tracer.fb_size */
  int32_t samples_per_pixel;   /* ray-tracer.samples_per_pixel */
  int32_t max_depth;           /* ray-tracer.depth */
  pm_camera camera;
  pm_float3 sky_colour;        /* ray-tracer.sky_colour */
  int32_t tile_rank;           /* image-tile sharding (16x16 tiles round robin) */
  int32_t tile_count;          /* 1 = whole image */
  int32_t caustic_k;           /* neighbours of the caustic gather: 0 = the reference's
                                  K = 50 (shading.h:7); up to 256 (config 5: 200) */
} pm_render_params;

/* setupCamera (ray-tracer/src/hostCode.cu:100-108), cos(fovy) scaling kept. */
int pm_camera_setup(pm_float3 look_from, pm_float3 look_at, pm_float3 look_up,
                    float fovy, int32_t width, int32_t height, pm_camera* out);
/* Renders into d_rgba (uint32 [H][W], row H-y layout of deviceCode.cu:224-230;
 * rows/tiles not rendered are left untouched) and, if non-NULL, d_rgb
 * (float [H][W][3], same layout, the pre-quantisation colour). */
int pm_render(pm_scene* scene, const pm_render_params* params,
              const pm_light* lights, int32_t num_lights,
              const pm_photon_map* global_map, const pm_photon_map* caustic_map,
              uint32_t* d_rgba, float* d_rgb, void* stream);
typedef struct {
  int64_t pixels, path_vertices, caustic_queries, global_queries, rays;
} pm_render_stats;
int pm_render_stats_get(pm_render_stats* out);

/* pm_render in two halves, so that the map-independent half overlaps the
 * photon trace and kd-tree build of the same frame (run it on another stream
 * from another host thread). pm_render_begin traces the camera paths, the
 * shadow and final-gather rays and the direct light, and sorts the gather
 * queries; it reads only the scene. pm_render_finish runs the two gathers
 * against the maps and resolves the pixels. begin + finish gives exactly
 * pm_render's image. The job owns device memory until destroyed; finish may
 * be called once. Overflow in either half is reported as PM_ERR_OVERFLOW. */
typedef struct pm_render_job pm_render_job;
int pm_render_begin(pm_scene* scene, const pm_render_params* params,
                    const pm_light* lights, int32_t num_lights,
                    pm_render_job** out, void* stream);
int pm_render_finish(pm_render_job* job, const pm_photon_map* global_map,
                     const pm_photon_map* caustic_map, uint32_t* d_rgba,
                     float* d_rgb, void* stream);
/* Optional, between begin and finish: run the job's caustic gather now (it
 * needs only the caustic map, e.g. beside the global map's trace and build;
 * synchronous on `stream`). pm_render_finish then runs only the global gather
 * and takes caustic_map = NULL or this same map. Once per job. */
int pm_render_gather_caustic(pm_render_job* job, const pm_photon_map* caustic_map,
                             void* stream);
/* A job's gather queries and, once pm_render_finish ran, their results:
 * which 0 = the global map's (final-gather) queries, 1 = the caustic ones.
 * d_queries [count][4] = (hit point xyz, brdf), d_results [count][4] =
 * (radiance estimate xyz, 0), in the job's dense query order; either may be
 * NULL (both NULL: *count only). Lets a caller check a frame's gathers against
 * an independent kNN (the parity tests) or reuse them. */
int pm_render_job_queries(const pm_render_job* job, int32_t which, float* d_queries,
                          float* d_results, int64_t capacity, int64_t* count, void* stream);
int pm_render_job_destroy(pm_render_job* job);

/* ---- photon viewer (photon-viewer/; debug splat) --------
 * loadPhotons' projection (photon-viewer/src/hostCode.cu:53-75: glm lookAt x
 * perspective(fovy, W/H, 0.1, 1000), z < 0 dropped, pixel = (int((x/w + 1)
 * 0.5 W), H - int((y/w + 1) 0.5 H))) + photonViewerRayGen (photon-viewer/cuda/
 * deviceCode.cu:10-38): a photon inside the frame whose visibility ray from
 * look_from (tmin 0, tmax = |pos - eye| - 1e-4 in double) hits nothing paints
 * make_rgba(color) over a 0xFF000000 frame. Several photons on one pixel: the
 * highest index wins (the reference's order is a race). d_rgba is [H][W]. */
typedef struct {
  pm_float3 look_from, look_at, look_up;
  float fovy;
  int32_t width, height;
} pm_viewer_params;
int pm_photon_view(pm_scene* scene, const pm_photon* d_photons, int64_t n, const pm_viewer_params* params,
                   uint32_t* d_rgba, void* stream);

/* ---- host-side boundary I/O (no GPU needed) ------------------------------ */
/* config.toml (configLoader.h:8-19; keys of photon-mapping/src/hostCode.cu:153-158
 * and ray-tracer/src/hostCode.cu:193-206). Strings are NUL-terminated. */
typedef struct {
  pm_float3 look_from, look_at, look_up; float fovy;
  char photons_file[512], caustics_photons_file[512], model_path[512];
  pm_float3 sky_colour; char output_filename[512];
  int32_t fb_width, fb_height, samples_per_pixel, depth;
  char viewer_output_filename[512], viewer_caustics_output_filename[512];
  int32_t viewer_fb_width, viewer_fb_height;
  int64_t casted_diffuse_photons, casted_caustics_photons; int32_t max_depth;
  uint32_t present_mask;       /* bit i set = key i found (see pm_config_key_name) */
  char error[512];
} pm_config;
int pm_config_load(const char* path, pm_config* out);
const char* pm_config_key_name(int32_t i);

/* Scene ingest (assetImporter.cxx:16-205): GLB (glTF 2.0 binary) or OBJ,
 * BFS node flatten with node*parent transforms, per-mesh position dedup,
 * <dir>/lights.txt, <stem>.mtl by material name; '/' and '\\' both accepted. */
typedef struct pm_scene_data pm_scene_data;
int pm_scene_data_load(const char* path, pm_scene_data** out);
int pm_scene_data_counts(const pm_scene_data* s, int32_t* num_meshes,
                         int32_t* num_lights, int64_t* num_vertices,
                         int64_t* num_triangles);
/* Borrowed views into the loaded scene (valid until pm_scene_data_free). */
int pm_scene_data_meshes(const pm_scene_data* s, const pm_mesh** meshes);
int pm_scene_data_lights(const pm_scene_data* s, const pm_light** lights);
int pm_scene_data_mesh_name(const pm_scene_data* s, int32_t i, const char** name);
int pm_scene_data_free(pm_scene_data* s);

/* Photon text files (photon-mapping/src/hostCode.cu:31-49 writer, %.6f, 9
 * values per line; ray-tracer/src/hostCode.cu:26-52 reader). */
int pm_photons_write_txt(const char* path, const pm_photon* h_photons, int64_t n);
int pm_photons_read_txt(const char* path, pm_photon** h_out, int64_t* n); /* free with pm_free */
/* stbi_write_png(path, W, H, 4, rgba, W*4) (ray-tracer/src/hostCode.cu:240). */
int pm_write_png_rgba(const char* path, const uint32_t* h_rgba, int32_t w, int32_t h);
/* In-memory equivalent of write_txt -> read_txt on device photons: each of
 * the 9 written floats becomes the float the %.6f text parses back to, power
 * is zeroed (values with |x| >= 9e9 are outside the exact range). */
int pm_photons_quantize(pm_photon* d_photons, int64_t n, void* stream);
/* Binary photon file (faster than the text contract): "PMPHOTN1", int64 n,
 * n x 40-B pm_photon records, little endian. */
int pm_photons_write_bin(const char* path, const pm_photon* h_photons, int64_t n);
int pm_photons_read_bin(const char* path, pm_photon** h_out, int64_t* n); /* free with pm_free */
void pm_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* PM_H_ */
