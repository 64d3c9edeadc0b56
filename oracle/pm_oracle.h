/*
 * pm_oracle.h — CPU ORACLE for the photon-mapping hot path. TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker. The product (libpm_hip.so)
 * never links or calls it.
 *
 * PARITY UNPINNED against reference outputs: the reference (CUDA + OptiX 7 +
 * OWL + cudaKDTree, empty submodules) cannot be built or run here and ships no
 * golden vectors. This oracle is a scalar C restatement of the
 * reference algorithm, each function citing the reference file:line it
 * follows; where the reference depends on upstream code that is absent (OWL
 * LCG, OptiX intersection, cudaKDTree) the published algorithm is restated and
 * the choices are listed in DESIGN.md §2 ("arithmetic spec"). It is pinned by
 * known-answer tests (tests/test_oracle_*.py) and by the golden fixtures it
 * generates (tests/golden/, script tests/golden/make_golden.py).
 *
 * Types are those of include/pm.h (layout only).
 */
#ifndef PM_ORACLE_H_
#define PM_ORACLE_H_
#include <stdint.h>
#include "../include/pm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* Photon id's emission (origin, direction) of one light, RNG seeded (id, 0). */
void orc_emit_photon(const pm_light* light, uint32_t id, float o[3], float d[3]);
typedef struct orc_map orc_map;

/* --- scalar kernels exposed for known-answer tests --- */
uint32_t orc_lcg_init(uint32_t v0, uint32_t v1);
float orc_lcg_next(uint32_t* state);
float orc_acosf(float x);
float orc_sinf(float x);
float orc_cosf(float x);
void orc_random_point_in_unit_sphere(uint32_t* state, float out[3]);
void orc_refract(const float in[3], const float n[3], float ior, float out[3]);

/* --- scene: brute force or own BVH (use_bvh) --- */
int orc_scene_create(const pm_mesh* meshes, int32_t num_meshes, int32_t use_bvh,
                     orc_scene** out);
void orc_scene_destroy(orc_scene* s);
int64_t orc_scene_num_triangles(const orc_scene* s);
int orc_intersect(const orc_scene* s, const pm_ray* rays, int64_t n, pm_hit* hits);
int orc_occluded(const orc_scene* s, const pm_ray* rays, int64_t n, int32_t* occ);

/* --- stage 1 --- */
int orc_photons_per_light(const pm_light* lights, int32_t nl, int64_t casted, int64_t* counts);
int orc_trace_photons(const orc_scene* s, const pm_light* lights, int32_t nl,
                      const pm_trace_params* p, int32_t nthreads,
                      pm_photon* out, int64_t capacity, int64_t* count);
/* trace only photons with global index in [g_lo, g_hi) (bounded samples) */
int orc_trace_photon_range(const orc_scene* s, const pm_light* lights, int32_t nl,
                           const pm_trace_params* p, int64_t g_lo, int64_t g_hi,
                           int32_t nthreads, pm_photon* out, int64_t capacity,
                           int64_t* count);

/* --- stage 2 --- */
/* cukd::buildTree's in-place left-balanced layout (ray-tracer/src/hostCode.cu:
 * 94-95): tags[t] = original index << 2 | split dim of node t
 * of the implicit tree over n points (pos: x, y, z at pos[i*stride]). */
int orc_kd_left_balanced(const float* pos, int64_t stride, int64_t n, int32_t nthreads, int32_t* tags);
/* complete-tree left subtree size of a subtree of s nodes */
int64_t orc_left_size(int64_t s);
/* threads used by orc_map_create's kd build (default 1) */
void orc_set_build_threads(int32_t n);
int orc_map_create(const pm_photon* a, int64_t na, float power_a,
                   const pm_photon* b, int64_t nb, float power_b, orc_map** out);
void orc_map_destroy(orc_map* m);
/* Alternative specifications of the gather (a bound on this build's unpinned
 * choices; NOT the parity spec): flags 0 = production; else
 * ORC_SPEC_HEAP (2, required) | ORC_SPEC_DOMAIN_DIM (1) | ORC_SPEC_FMA (4).
 * Later gathers and renders through m follow it. */
int orc_map_set_spec(orc_map* m, int32_t flags, int32_t nthreads);
int orc_knn(const orc_map* m, const pm_float3* q, int64_t nq, int32_t k,
            float max_radius, int32_t nthreads, int32_t* ids, float* d2, float* maxd2);
int orc_gather(const orc_map* m, const pm_float3* pts, const float* brdf,
               int64_t nq, int32_t nthreads, pm_float3* out);
int orc_gather_k(const orc_map* m, const pm_float3* pts, const float* brdf,
                 int64_t nq, int32_t k, int32_t nthreads, pm_float3* out);
int orc_camera_setup(pm_float3 look_from, pm_float3 look_at, pm_float3 look_up,
                     float fovy, int32_t w, int32_t h, pm_camera* out);
/* Renders rows [row_lo, row_hi) of launch indices (pixelID.y); whole image if
 * row_hi <= row_lo. rgba/rgb use the [H][W] layout of pm_render. */
int orc_render(const orc_scene* s, const pm_render_params* p, const pm_light* lights,
               int32_t nl, const orc_map* gmap, const orc_map* cmap,
               int32_t row_lo, int32_t row_hi, int32_t nthreads,
               uint32_t* rgba, float* rgb, pm_render_stats* stats);

/* The value each float takes after the %.6f text write + strtof read back. */
void orc_quantize6(const float* in, float* out, int64_t n);

/* Photon viewer splat (see pm_photon_view in include/pm.h). M is column-major. */
void orc_viewer_matrix(const pm_viewer_params* params, float M[16]);
int orc_photon_view(const orc_scene* s, const pm_photon* photons, int64_t n, const pm_viewer_params* params,
                    uint32_t* rgba);

#ifdef __cplusplus
}
#endif
#endif
