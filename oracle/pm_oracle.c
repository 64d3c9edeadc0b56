/*
 * pm_oracle.c — CPU ORACLE (test infrastructure only; see pm_oracle.h).
 * Scalar C restatement of the reference photon-mapping hot path.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 * PARITY UNPINNED against reference outputs (reference unbuildable here).
 *
 * Arithmetic spec shared with the HIP product: IEEE float32,
 * round-to-nearest, no FMA contraction, correctly rounded / and sqrt, own
 * polynomial acos/sin/cos, normalize(v) = v * (1/sqrt(dot(v,v))), watertight
 * ray-triangle test, closest hit = argmin (t, global triangle index).
 */
#define _GNU_SOURCE
#include "pm_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define EPS 1e-3f                    /* common/cuda/helpers.h:8 */
#define PI_F ((float)3.141592653)    /* helpers.h:9 */
#define INFTY_F 1e10f                /* helpers.h:7 */
#define PHOTON_TMAX 1e30f            /* owl::Ray default tmax (upstream OWL) */
#define K_NEAREST 50                 /* ray-tracer/cuda/shading.h:7 */
#define K_MAX_DISTANCE 100.0f        /* shading.h:8 */
#define CONE_FILTER_C 1.1f           /* shading.h:9 */
#define NUM_DIFFUSE_SAMPLES 20       /* ray-tracer/cuda/deviceCode.cu:15 */
#define DIRECT_LIGHT_FACTOR 0.8f     /* deviceCode.cu:10 */
#define CAUSTICS_FACTOR 0.08f        /* deviceCode.cu:11 */
#define DIFFUSE_FACTOR 0.2f          /* deviceCode.cu:12 */

enum { EV_MISS = 0, EV_ABSORBED = 1, EV_DIFFUSE = 2, EV_SPECULAR = 4, EV_REFRACT = 8 };

/* ------------------------------------------------------------------------ */
/* vec3 (owl::vec3f semantics, evaluation order left to right)               */
typedef struct { float x, y, z; } v3;
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mulf(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return V3(s * a.x, s * a.y, s * a.z); }
static inline v3 mulv(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 divf(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
  return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* owl normalize = v * rsqrt(dot(v,v)); spec: rsqrt := 1/sqrtf */
static inline v3 normalize(v3 v) { return mulf(v, 1.0f / sqrtf(dot(v, v))); }
static inline float norm3(v3 v) { return sqrtf(dot(v, v)); }   /* helpers.h:23-25 */
static inline v3 fromp(pm_float3 p) { return V3(p.x, p.y, p.z); }
static inline pm_float3 top3(v3 v) { pm_float3 p = {v.x, v.y, v.z}; return p; }
/* helpers.h:15-17 (signed test, kept) */
static inline int near_zero(v3 v) { return v.x < EPS && v.y < EPS && v.z < EPS; }

/* ------------------------------------------------------------------------ */
/* owl::LCG<16> (upstream owl/common/math/random.h): TEA init + LCG draw.    */
uint32_t orc_lcg_init(uint32_t val0, uint32_t val1) {
  uint32_t v0 = val0, v1 = val1, s0 = 0;
  for (int n = 0; n < 16; n++) {
    s0 += 0x9e3779b9u;
    v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
    v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
  }
  return v0;
}
float orc_lcg_next(uint32_t* state) {
  *state = 1664525u * *state + 1013904223u;
  return (float)(*state & 0x00FFFFFFu) / (float)0x01000000;
}

/* ------------------------------------------------------------------------ */
/* Deterministic trig (spec DESIGN.md §2; replaces CUDA acosf/sinf/cosf).    */
float orc_acosf(float x) {
  /* Abramowitz & Stegun 4.4.46 on |x|, reflected for x < 0. */
  float ax = fabsf(x);
  float p = -0.0012624911f;
  p = p * ax + 0.0066700901f;
  p = p * ax + -0.0170881256f;
  p = p * ax + 0.0308918810f;
  p = p * ax + -0.0501743046f;
  p = p * ax + 0.0889789874f;
  p = p * ax + -0.2145988016f;
  p = p * ax + 1.5707963050f;
  float r = sqrtf(1.0f - ax) * p;
  return x < 0.0f ? 3.14159274f - r : r;
}
static void sincos_spec(float x, float* s, float* c) {
  /* Cody-Waite reduction by pi/2 (3-part constant), cephes kernels. */
  float q = rintf(x * 0.636619772f);
  int k = (int)q;
  float r = x - q * 1.5703125f;
  r = r - q * 4.837512969970703125e-4f;
  r = r - q * 7.549789954891882e-8f;
  float r2 = r * r;
  float sp = -1.9515295891e-4f;
  sp = sp * r2 + 8.3321608736e-3f;
  sp = sp * r2 + -1.6666654611e-1f;
  sp = sp * r2;
  sp = sp * r;
  sp = sp + r;
  float cp = 2.443315711809948e-5f;
  cp = cp * r2 + -1.388731625493765e-3f;
  cp = cp * r2 + 4.166664568298827e-2f;
  cp = cp * (r2 * r2);
  cp = (1.0f - 0.5f * r2) + cp;
  switch (k & 3) {
    case 0: *s = sp; *c = cp; break;
    case 1: *s = cp; *c = -sp; break;
    case 2: *s = -sp; *c = -cp; break;
    default: *s = -cp; *c = sp; break;
  }
}
float orc_sinf(float x) { float s, c; sincos_spec(x, &s, &c); return s; }
float orc_cosf(float x) { float s, c; sincos_spec(x, &s, &c); return c; }

/* helpers.h:27-34 randomPointInUnitSphere */
static v3 random_point_in_unit_sphere(uint32_t* st) {
  const float u = orc_lcg_next(st);
  const float v = orc_lcg_next(st);
  const float theta = 2.f * PI_F * u;
  const float phi = orc_acosf(2.f * v - 1.f);
  float sp, cp, st_, ct;
  sincos_spec(phi, &sp, &cp);
  sincos_spec(theta, &st_, &ct);
  return V3(sp * ct, sp * st_, cp);
}
void orc_random_point_in_unit_sphere(uint32_t* state, float out[3]) {
  v3 r = random_point_in_unit_sphere(state);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
/* helpers.h:36-43 randomUnitVector */
static v3 random_unit_vector(uint32_t* st) {
  v3 v;
  do {
    v.x = 2.f * orc_lcg_next(st) - 1.f;
    v.y = 2.f * orc_lcg_next(st) - 1.f;
    v.z = 2.f * orc_lcg_next(st) - 1.f;
  } while (dot(v, v) >= 1.f);
  return normalize(v);
}
/* helpers.h:45-47 */
static v3 cosine_sample_hemisphere(v3 n, uint32_t* st) {
  return normalize(add(n, mulf(random_point_in_unit_sphere(st), (1 - EPS))));
}
/* helpers.h:49-51 */
static v3 reflect(v3 i, v3 n) { return sub(i, mulf(n, 2.f * dot(i, n))); }
/* helpers.h:57-74 (normal not flipped on exit — kept) */
static v3 refract_ior(v3 in, v3 n, float ior) {
  float cos_theta = -dot(in, n);
  float mu;
  if (cos_theta > 0.f) {
    mu = 1.f / ior;
  } else {
    mu = ior;
    cos_theta = -cos_theta;
  }
  const float cos_phi = 1.f - mu * mu * (1.f - cos_theta * cos_theta);
  if (cos_phi >= 0) return add(smul(mu, in), smul(mu * cos_theta - sqrtf(cos_phi), n));
  return reflect(in, n);
}
void orc_refract(const float in[3], const float n[3], float ior, float out[3]) {
  v3 r = refract_ior(V3(in[0], in[1], in[2]), V3(n[0], n[1], n[2]), ior);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
/* helpers.h:91-106 refract(v, n, ni_over_nt, &refracted) */
static int refract_uv(v3 v, v3 n, float ni, v3* refracted) {
  const v3 uv = normalize(v);
  const float dt = dot(uv, n);
  const float disc = 1.0f - ni * ni * (1 - dt * dt);
  if (disc > 0.f) {
    *refracted = sub(smul(ni, sub(uv, mulf(n, dt))), mulf(n, sqrtf(disc)));
    return 1;
  }
  return 0;
}
/* helpers.h:108-112: double arithmetic; pow(x,5) := ((x*x)*(x*x))*x */
static float schlick(float cosv, float ior) {
  float r0 = (float)((1. - (double)ior) / (1. + (double)ior));
  r0 = r0 * r0;
  double x = 1. - (double)cosv;
  double x2 = x * x;
  double p5 = (x2 * x2) * x;
  return (float)((double)r0 + (1. - (double)r0) * p5);
}

/* ------------------------------------------------------------------------ */
/* Scene: triangles + optional own BVH (conservative culling).               */
typedef struct { float lo[3], hi[3]; int32_t left, count; } onode;
struct orc_scene {
  int64_t ntri;
  float* tri;          /* ntri * 9: A, B, C world-space */
  int32_t* mesh;
  int32_t* prim;
  pm_material* mat;
  int32_t nmesh;
  int use_bvh;
  onode* nodes;
  int32_t nnodes;
  int32_t* order;
  float pad;
};

typedef struct {
  v3 o, d, inv;
  int kx, ky, kz;
  float Sx, Sy, Sz;
} rayp;

static void ray_prep(rayp* r, v3 o, v3 d) {
  r->o = o; r->d = d;
  float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  int kz = ax > ay ? (ax > az ? 0 : 2) : (ay > az ? 1 : 2);
  int kx = kz + 1; if (kx == 3) kx = 0;
  int ky = kx + 1; if (ky == 3) ky = 0;
  float dd[3] = {d.x, d.y, d.z};
  if (dd[kz] < 0.0f) { int t = kx; kx = ky; ky = t; }
  r->kx = kx; r->ky = ky; r->kz = kz;
  r->Sx = dd[kx] / dd[kz];
  r->Sy = dd[ky] / dd[kz];
  r->Sz = 1.0f / dd[kz];
  float iv[3];
  for (int i = 0; i < 3; i++) {
    float c = dd[i];
    if (fabsf(c) < 1e-20f) c = copysignf(1e-20f, c);
    iv[i] = 1.0f / c;
  }
  r->inv = V3(iv[0], iv[1], iv[2]);
}

/* Watertight ray/triangle (Woop, Benthin, Wald 2013) — stands in for the
 * OptiX built-in triangle test used by every optixTrace/owl::traceRay call. */
static int wt_hit(const float* t9, const rayp* r, float* tout) {
  const float oo[3] = {r->o.x, r->o.y, r->o.z};
  float A[3], B[3], C[3];
  for (int i = 0; i < 3; i++) {
    A[i] = t9[i] - oo[i];
    B[i] = t9[3 + i] - oo[i];
    C[i] = t9[6 + i] - oo[i];
  }
  const int kx = r->kx, ky = r->ky, kz = r->kz;
  const float Ax = A[kx] - r->Sx * A[kz], Ay = A[ky] - r->Sy * A[kz];
  const float Bx = B[kx] - r->Sx * B[kz], By = B[ky] - r->Sy * B[kz];
  const float Cx = C[kx] - r->Sx * C[kz], Cy = C[ky] - r->Sy * C[kz];
  float U = Cx * By - Cy * Bx;
  float Vv = Ax * Cy - Ay * Cx;
  float W = Bx * Ay - By * Ax;
  if (U == 0.0f || Vv == 0.0f || W == 0.0f) {
    double CxBy = (double)Cx * (double)By, CyBx = (double)Cy * (double)Bx;
    U = (float)(CxBy - CyBx);
    double AxCy = (double)Ax * (double)Cy, AyCx = (double)Ay * (double)Cx;
    Vv = (float)(AxCy - AyCx);
    double BxAy = (double)Bx * (double)Ay, ByAx = (double)By * (double)Ax;
    W = (float)(BxAy - ByAx);
  }
  if ((U < 0.0f || Vv < 0.0f || W < 0.0f) && (U > 0.0f || Vv > 0.0f || W > 0.0f)) return 0;
  const float det = U + Vv + W;
  if (det == 0.0f) return 0;
  const float Az = r->Sz * A[kz], Bz = r->Sz * B[kz], Cz = r->Sz * C[kz];
  const float T = U * Az + Vv * Bz + W * Cz;
  *tout = T / det;
  return 1;
}

static int box_hit(const onode* n, const rayp* r, float tmin, float tmax) {
  float t0x = (n->lo[0] - r->o.x) * r->inv.x, t1x = (n->hi[0] - r->o.x) * r->inv.x;
  float t0y = (n->lo[1] - r->o.y) * r->inv.y, t1y = (n->hi[1] - r->o.y) * r->inv.y;
  float t0z = (n->lo[2] - r->o.z) * r->inv.z, t1z = (n->hi[2] - r->o.z) * r->inv.z;
  float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
  float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
  return tn <= tf;
}

static int cmp_axis;
static const float* cmp_cent;
static int cmp_idx(const void* a, const void* b) {
  int ia = *(const int32_t*)a, ib = *(const int32_t*)b;
  float ca = cmp_cent[ia * 3 + cmp_axis], cb = cmp_cent[ib * 3 + cmp_axis];
  if (ca < cb) return -1;
  if (ca > cb) return 1;
  return ia < ib ? -1 : (ia > ib);
}

static int32_t bvh_build_rec(orc_scene* s, const float* cent, int32_t lo, int32_t hi) {
  int32_t id = s->nnodes++;
  onode* n = &s->nodes[id];
  for (int k = 0; k < 3; k++) { n->lo[k] = FLT_MAX; n->hi[k] = -FLT_MAX; }
  for (int32_t i = lo; i < hi; i++) {
    const float* t = &s->tri[(int64_t)s->order[i] * 9];
    for (int v = 0; v < 3; v++)
      for (int k = 0; k < 3; k++) {
        n->lo[k] = fminf(n->lo[k], t[v * 3 + k]);
        n->hi[k] = fmaxf(n->hi[k], t[v * 3 + k]);
      }
  }
  for (int k = 0; k < 3; k++) { n->lo[k] -= s->pad; n->hi[k] += s->pad; }
  if (hi - lo <= 4) {
    n->left = lo;
    n->count = hi - lo;
    return id;
  }
  float ext[3];
  for (int k = 0; k < 3; k++) ext[k] = n->hi[k] - n->lo[k];
  cmp_axis = ext[0] > ext[1] ? (ext[0] > ext[2] ? 0 : 2) : (ext[1] > ext[2] ? 1 : 2);
  cmp_cent = cent;
  qsort(&s->order[lo], (size_t)(hi - lo), sizeof(int32_t), cmp_idx);
  int32_t mid = lo + (hi - lo) / 2;
  n->count = 0;
  bvh_build_rec(s, cent, lo, mid);                       /* left = id + 1 */
  int32_t right = bvh_build_rec(s, cent, mid, hi);
  s->nodes[id].left = right;
  return id;
}

int orc_scene_create(const pm_mesh* meshes, int32_t nm, int32_t use_bvh, orc_scene** out) {
  if (!out || nm < 0) return PM_ERR_INVALID;
  orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
  int64_t nt = 0;
  for (int i = 0; i < nm; i++) nt += meshes[i].num_triangles;
  s->ntri = nt;
  s->nmesh = nm;
  s->tri = (float*)malloc(sizeof(float) * 9 * (size_t)(nt > 0 ? nt : 1));
  s->mesh = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nt > 0 ? nt : 1));
  s->prim = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nt > 0 ? nt : 1));
  s->mat = (pm_material*)malloc(sizeof(pm_material) * (size_t)(nm > 0 ? nm : 1));
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  int64_t t = 0;
  for (int m = 0; m < nm; m++) {
    s->mat[m] = meshes[m].material;
    for (int j = 0; j < meshes[m].num_triangles; j++, t++) {
      const pm_int3 ix = meshes[m].indices[j];
      const int32_t id3[3] = {ix.x, ix.y, ix.z};
      for (int v = 0; v < 3; v++) {
        if (id3[v] < 0 || id3[v] >= meshes[m].num_vertices) { orc_scene_destroy(s); return PM_ERR_INVALID; }
        pm_float3 p = meshes[m].vertices[id3[v]];
        s->tri[t * 9 + v * 3 + 0] = p.x;
        s->tri[t * 9 + v * 3 + 1] = p.y;
        s->tri[t * 9 + v * 3 + 2] = p.z;
        lo[0] = fminf(lo[0], p.x); lo[1] = fminf(lo[1], p.y); lo[2] = fminf(lo[2], p.z);
        hi[0] = fmaxf(hi[0], p.x); hi[1] = fmaxf(hi[1], p.y); hi[2] = fmaxf(hi[2], p.z);
      }
      s->mesh[t] = m;
      s->prim[t] = j;
    }
  }
  float ext = 0.f;
  for (int k = 0; k < 3; k++) if (nt > 0) ext = fmaxf(ext, hi[k] - lo[k]);
  s->pad = ext * 1e-5f + 1e-20f;
  s->use_bvh = use_bvh && nt > 0;
  if (s->use_bvh) {
    float* cent = (float*)malloc(sizeof(float) * 3 * (size_t)nt);
    for (int64_t i = 0; i < nt; i++)
      for (int k = 0; k < 3; k++)
        cent[i * 3 + k] = (s->tri[i * 9 + k] + s->tri[i * 9 + 3 + k] + s->tri[i * 9 + 6 + k]) / 3.0f;
    s->order = (int32_t*)malloc(sizeof(int32_t) * (size_t)nt);
    for (int64_t i = 0; i < nt; i++) s->order[i] = (int32_t)i;
    s->nodes = (onode*)malloc(sizeof(onode) * (size_t)(2 * nt + 1));
    s->nnodes = 0;
    bvh_build_rec(s, cent, 0, (int32_t)nt);
    free(cent);
  }
  *out = s;
  return PM_OK;
}

void orc_scene_destroy(orc_scene* s) {
  if (!s) return;
  free(s->tri); free(s->mesh); free(s->prim); free(s->mat);
  free(s->nodes); free(s->order);
  free(s);
}
int64_t orc_scene_num_triangles(const orc_scene* s) { return s->ntri; }

/* closest hit in (tmin, tmax): argmin (t, triangle index). Returns tri or -1. */
static int64_t closest_hit(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, float* tbest) {
  rayp r;
  ray_prep(&r, o, d);
  float bt = tmax;
  int64_t bid = -1;
  if (!s->use_bvh) {
    for (int64_t i = 0; i < s->ntri; i++) {
      float t;
      if (!wt_hit(&s->tri[i * 9], &r, &t)) continue;
      if (!(t > tmin && t < tmax)) continue;
      if (bid < 0 || t < bt || (t == bt && i < bid)) { bt = t; bid = i; }
    }
  } else {
    int32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
      const onode* n = &s->nodes[stack[--sp]];
      float lim = bid < 0 ? tmax : bt * 1.00001f;
      if (!box_hit(n, &r, tmin, lim)) continue;
      if (n->count > 0) {
        for (int32_t j = 0; j < n->count; j++) {
          int64_t i = s->order[n->left + j];
          float t;
          if (!wt_hit(&s->tri[i * 9], &r, &t)) continue;
          if (!(t > tmin && t < tmax)) continue;
          if (bid < 0 || t < bt || (t == bt && i < bid)) { bt = t; bid = i; }
        }
      } else {
        int32_t self = (int32_t)(n - s->nodes);
        stack[sp++] = n->left;
        stack[sp++] = self + 1;
      }
    }
  }
  *tbest = bt;
  return bid;
}

static int any_hit(const orc_scene* s, v3 o, v3 d, float tmin, float tmax) {
  rayp r;
  ray_prep(&r, o, d);
  if (!s->use_bvh) {
    for (int64_t i = 0; i < s->ntri; i++) {
      float t;
      if (wt_hit(&s->tri[i * 9], &r, &t) && t > tmin && t < tmax) return 1;
    }
    return 0;
  }
  int32_t stack[128];
  int sp = 0;
  stack[sp++] = 0;
  while (sp) {
    const onode* n = &s->nodes[stack[--sp]];
    if (!box_hit(n, &r, tmin, tmax * 1.00001f)) continue;
    if (n->count > 0) {
      for (int32_t j = 0; j < n->count; j++) {
        int64_t i = s->order[n->left + j];
        float t;
        if (wt_hit(&s->tri[i * 9], &r, &t) && t > tmin && t < tmax) return 1;
      }
    } else {
      int32_t self = (int32_t)(n - s->nodes);
      stack[sp++] = n->left;
      stack[sp++] = self + 1;
    }
  }
  return 0;
}

int orc_intersect(const orc_scene* s, const pm_ray* rays, int64_t n, pm_hit* hits) {
  for (int64_t i = 0; i < n; i++) {
    float t;
    int64_t id = closest_hit(s, fromp(rays[i].origin), fromp(rays[i].direction),
                             rays[i].tmin, rays[i].tmax, &t);
    if (id < 0) {
      hits[i].t = INFINITY; hits[i].mesh = -1; hits[i].prim = -1; hits[i].tri = -1;
    } else {
      hits[i].t = t; hits[i].mesh = s->mesh[id]; hits[i].prim = s->prim[id]; hits[i].tri = (int32_t)id;
    }
  }
  return PM_OK;
}
int orc_occluded(const orc_scene* s, const pm_ray* rays, int64_t n, int32_t* occ) {
  for (int64_t i = 0; i < n; i++)
    occ[i] = any_hit(s, fromp(rays[i].origin), fromp(rays[i].direction), rays[i].tmin, rays[i].tmax);
  return PM_OK;
}

/* helpers.h:76-85 getPrimitiveNormal (unflipped geometric normal) */
static v3 prim_normal(const orc_scene* s, int64_t tri) {
  const float* t = &s->tri[tri * 9];
  v3 A = V3(t[0], t[1], t[2]), B = V3(t[3], t[4], t[5]), C = V3(t[6], t[7], t[8]);
  return normalize(cross(sub(B, A), sub(C, A)));
}

/* ------------------------------------------------------------------------ */
/* tiny parallel-for                                                          */
typedef void (*pf_fn)(void* ctx, int64_t lo, int64_t hi);
typedef struct { pf_fn fn; void* ctx; int64_t n, chunk; int64_t next; pthread_mutex_t mu; } pf_t;
static void* pf_worker(void* a) {
  pf_t* p = (pf_t*)a;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    int64_t lo = p->next;
    p->next += p->chunk;
    pthread_mutex_unlock(&p->mu);
    if (lo >= p->n) break;
    int64_t hi = lo + p->chunk < p->n ? lo + p->chunk : p->n;
    p->fn(p->ctx, lo, hi);
  }
  return NULL;
}
static void parallel_for(int64_t n, int64_t chunk, int nthreads, pf_fn fn, void* ctx) {
  if (n <= 0) return;
  if (nthreads <= 1) { fn(ctx, 0, n); return; }
  pf_t p;
  p.fn = fn; p.ctx = ctx; p.n = n; p.chunk = chunk > 0 ? chunk : 1; p.next = 0;
  pthread_mutex_init(&p.mu, NULL);
  pthread_t th[256];
  if (nthreads > 256) nthreads = 256;
  for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, pf_worker, &p);
  for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&p.mu);
}

/* ------------------------------------------------------------------------ */
/* Stage 1: photon tracer                                                     */
/* photon-mapping/src/hostCode.cu:102-110 + :86 */
int orc_photons_per_light(const pm_light* lights, int32_t nl, int64_t casted, int64_t* counts) {
  double total = 0;
  for (int i = 0; i < nl; i++) total += lights[i].power;
  if (!(total > 0.0)) { for (int i = 0; i < nl; i++) counts[i] = 0; return PM_OK; }
  int ppw = (int)((double)(int)casted / total);
  for (int i = 0; i < nl; i++) counts[i] = (int64_t)(int)(lights[i].power * ppw);
  return PM_OK;
}

typedef struct {
  const orc_scene* s;
  const pm_light* lights;
  int32_t nl;
  const int64_t* loff;   /* nl+1 prefix of per-light counts */
  int64_t g_lo;
  int32_t maxd, caustic;
  pm_photon* slots;      /* [g - g_lo][maxd] */
  uint8_t* cnt;
} trace_ctx;

/* photon-mapping/cuda/deviceCode.cu:54-72 (raygen) + :25-52 (bounce loops)
 * + :113-131 (closest hit) + :74-111 (scatter) + :10-17 (deposit). */
/* Emission: point light = pointLightRayGen (deviceCode.cu:54-72); SQUARE_LIGHT
 * = this build's definition (the reference declares the type only, world.h:
 * 8-24): origin uniform on the side x side square about pos in the basis
 * t1 = normalize(cross(a, n)), t2 = cross(n, t1), a = (0,1,0) if |n.x| > 0.9
 * else (1,0,0) (two draws), direction = cosine lobe about n. */
static void emit_photon(const pm_light* L, uint32_t* rng, v3* o, v3* d) {
  if (L->source_type == PM_SQUARE_LIGHT) {
    const v3 n = normalize(fromp(L->normal));
    const v3 a = fabsf(n.x) > 0.9f ? V3(0.f, 1.f, 0.f) : V3(1.f, 0.f, 0.f);
    const v3 t1 = normalize(cross(a, n));
    const v3 t2 = cross(n, t1);
    const float side = (float)L->side_length;
    const float u = orc_lcg_next(rng);
    const float w = orc_lcg_next(rng);
    *o = add(add(fromp(L->pos), smul((u - 0.5f) * side, t1)), smul((w - 0.5f) * side, t2));
    *d = cosine_sample_hemisphere(n, rng);
  } else {
    *o = fromp(L->pos);
    *d = random_point_in_unit_sphere(rng);
  }
}

void orc_emit_photon(const pm_light* L, uint32_t id, float o[3], float d[3]) {
  uint32_t rng = orc_lcg_init(id, 0);
  v3 oo, dd;
  emit_photon(L, &rng, &oo, &dd);
  o[0] = oo.x; o[1] = oo.y; o[2] = oo.z;
  d[0] = dd.x; d[1] = dd.y; d[2] = dd.z;
}

static void trace_one(const trace_ctx* c, int64_t g) {
  int l = 0;
  while (g >= c->loff[l + 1]) l++;
  const uint32_t id = (uint32_t)(g - c->loff[l]);
  const pm_light* L = &c->lights[l];
  uint32_t rng = orc_lcg_init(id, 0);
  v3 color = fromp(L->rgb);
  v3 o, d;
  emit_photon(L, &rng, &o, &d);
  const float tmin = EPS;
  pm_photon* out = &c->slots[(g - c->g_lo) * c->maxd];
  int n = 0;
  for (int i = 0; i < c->maxd; i++) {
    float t;
    int64_t tri = closest_hit(c->s, o, d, tmin, PHOTON_TMAX, &t);
    int ev;
    v3 so = {0, 0, 0}, sd = {0, 0, 0}, sc = {0, 0, 0};
    if (tri < 0) {
      ev = EV_MISS;
    } else {
      const pm_material* m = &c->s->mat[c->s->mesh[tri]];
      const float pd = m->diffuse;
      const float ps = m->specular + pd;
      const float pt = m->transmission + ps;
      const float rp = orc_lcg_next(&rng);
      const v3 hp = add(o, smul(t, d));
      const v3 albedo = fromp(m->albedo);
      if (rp < pd) {
        ev = EV_DIFFUSE;
        so = hp;
        sd = cosine_sample_hemisphere(prim_normal(c->s, tri), &rng);
        sc = mulv(albedo, color);
      } else if (rp < ps) {
        ev = EV_SPECULAR;
        so = hp;
        sd = reflect(d, prim_normal(c->s, tri));
        sc = mulv(albedo, color);
      } else if (rp < pt) {
        ev = EV_REFRACT;
        so = hp;
        sd = refract_ior(d, prim_normal(c->s, tri), m->refraction_idx);
        sc = mulv(albedo, color);
      } else {
        ev = EV_ABSORBED;
      }
    }
    if (!c->caustic) {
      if (ev == EV_DIFFUSE) {
        if (i > 0) {
          pm_photon* p = &out[n++];
          p->pos = top3(so); p->dir = top3(sd); p->power = 0; p->color = top3(color);
        }
        o = so; d = sd; color = sc;
      } else {
        break;
      }
    } else {
      if (i > 0 && ev == EV_DIFFUSE) {
        pm_photon* p = &out[n++];
        p->pos = top3(so); p->dir = top3(sd); p->power = 0; p->color = top3(color);
      }
      if (ev & (EV_SPECULAR | EV_REFRACT)) {
        o = so; d = sd; color = sc;
      } else {
        break;
      }
    }
  }
  c->cnt[g - c->g_lo] = (uint8_t)n;
}
static void trace_range(void* ctx, int64_t lo, int64_t hi) {
  const trace_ctx* c = (const trace_ctx*)ctx;
  for (int64_t i = lo; i < hi; i++) trace_one(c, c->g_lo + i);
}

int orc_trace_photon_range(const orc_scene* s, const pm_light* lights, int32_t nl,
                           const pm_trace_params* p, int64_t g_lo, int64_t g_hi,
                           int32_t nthreads, pm_photon* out, int64_t capacity, int64_t* count) {
  if (!s || !p || !count || nl < 0 || p->max_depth < 0 || p->max_depth > 255) return PM_ERR_INVALID;
  int64_t* cnts = (int64_t*)calloc((size_t)nl + 1, sizeof(int64_t));
  int64_t* loff = (int64_t*)calloc((size_t)nl + 2, sizeof(int64_t));
  orc_photons_per_light(lights, nl, p->casted_photons, cnts);
  for (int i = 0; i < nl; i++) loff[i + 1] = loff[i] + (cnts[i] > 0 ? cnts[i] : 0);
  loff[nl + 1] = INT64_MAX;
  if (g_hi > loff[nl]) g_hi = loff[nl];
  if (g_lo < 0) g_lo = 0;
  int64_t np = g_hi > g_lo ? g_hi - g_lo : 0;
  int maxd = p->max_depth;
  trace_ctx c;
  c.s = s; c.lights = lights; c.nl = nl; c.loff = loff; c.g_lo = g_lo;
  c.maxd = maxd; c.caustic = p->caustics_mode;
  c.slots = (pm_photon*)malloc(sizeof(pm_photon) * (size_t)(np * (maxd > 0 ? maxd : 1) + 1));
  c.cnt = (uint8_t*)calloc((size_t)np + 1, 1);
  parallel_for(np, 256, nthreads, trace_range, &c);
  int64_t total = 0;
  for (int64_t i = 0; i < np; i++) total += c.cnt[i];
  *count = total;
  int st = PM_OK;
  if (total > capacity || (total > 0 && !out)) {
    st = PM_ERR_CAPACITY;
  } else {
    int64_t w = 0;
    for (int64_t i = 0; i < np; i++)
      for (int j = 0; j < c.cnt[i]; j++) out[w++] = c.slots[i * maxd + j];
  }
  free(c.slots); free(c.cnt); free(cnts); free(loff);
  return st;
}

int orc_trace_photons(const orc_scene* s, const pm_light* lights, int32_t nl,
                      const pm_trace_params* p, int32_t nthreads,
                      pm_photon* out, int64_t capacity, int64_t* count) {
  if (!p || p->shard_count < 1 || p->shard_rank < 0 || p->shard_rank >= p->shard_count)
    return PM_ERR_INVALID;
  int64_t* cnts = (int64_t*)calloc((size_t)nl + 1, sizeof(int64_t));
  orc_photons_per_light(lights, nl, p->casted_photons, cnts);
  int64_t tot = 0;
  for (int i = 0; i < nl; i++) tot += cnts[i] > 0 ? cnts[i] : 0;
  free(cnts);
  int64_t lo = tot * p->shard_rank / p->shard_count;
  int64_t hi = tot * (p->shard_rank + 1) / p->shard_count;
  return orc_trace_photon_range(s, lights, nl, p, lo, hi, nthreads, out, capacity, count);
}

/* ------------------------------------------------------------------------ */
/* Stage 2: photon map (own kd-tree, exact kNN by (d^2, original index))      */
struct orc_map {
  int64_t n;
  float* pos;      /* n*3 */
  float* col;      /* n*3 */
  float* pw;       /* n   */
  int32_t* idx;    /* kd order -> original index */
  int32_t* node_lo; int32_t* node_hi; int8_t* node_dim; float* node_split; int32_t nnodes;
  struct orc_refkd* ref;   /* orc_map_set_spec: the alternative specification, or NULL */
};

/* ray-tracer/src/hostCode.cu:54-83 loadPhotons: map = a (power_a) ++ b (power_b).
 * Build: median split on the widest dimension in (coord, original index) order,
 * found by quickselect (O(n) per level; the subtree MEMBERSHIP equals a full
 * sort's, so the tree is independent of the selection method), subtrees built
 * in parallel threads near the root (the CPU baseline uses every core). */
static inline int kd_less(const float* pos, int dim, int32_t a, int32_t b) {
  const float ca = pos[(int64_t)a * 3 + dim], cb = pos[(int64_t)b * 3 + dim];
  return ca < cb || (ca == cb && a < b);
}
/* rearranges v[0..n) so that v[k] is the k-th smallest and v[<k] <= v[k] <= v[>k] */
static void kd_select(const float* pos, int dim, int32_t* v, int64_t n, int64_t k) {
  int64_t lo = 0, hi = n - 1;
  while (hi > lo) {
    /* median-of-three pivot */
    const int64_t mid = lo + (hi - lo) / 2;
    int32_t a = v[lo], b = v[mid], c = v[hi], pv;
    if (kd_less(pos, dim, a, b)) pv = kd_less(pos, dim, b, c) ? b : (kd_less(pos, dim, a, c) ? c : a);
    else pv = kd_less(pos, dim, a, c) ? a : (kd_less(pos, dim, b, c) ? c : b);
    int64_t i = lo, j = hi;
    while (i <= j) {
      while (kd_less(pos, dim, v[i], pv)) i++;
      while (kd_less(pos, dim, pv, v[j])) j--;
      if (i <= j) {
        const int32_t t = v[i]; v[i] = v[j]; v[j] = t;
        i++; j--;
      }
    }
    if (k <= j) hi = j;
    else if (k >= i) lo = i;
    else return;
  }
}
typedef struct { orc_map* m; int32_t node; int64_t lo, hi; int par; } kd_task;
static void kd_build(orc_map* m, int32_t node, int64_t lo, int64_t hi, int par);
static void* kd_build_thread(void* arg) {
  kd_task* t = (kd_task*)arg;
  kd_build(t->m, t->node, t->lo, t->hi, t->par);
  return NULL;
}
/* Node layout: implicit binary tree over the idx array, leaves <= 8 points.
 * par > 1: build the left child in a new thread (par/2 threads each side). */
static void kd_build(orc_map* m, int32_t node, int64_t lo, int64_t hi, int par) {
  m->node_lo[node] = (int32_t)lo;
  m->node_hi[node] = (int32_t)hi;
  if (hi - lo <= 8 || 2 * node + 2 >= m->nnodes) { m->node_dim[node] = -1; return; }
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = lo; i < hi; i++)
    for (int k = 0; k < 3; k++) {
      float v = m->pos[(int64_t)m->idx[i] * 3 + k];
      mn[k] = fminf(mn[k], v); mx[k] = fmaxf(mx[k], v);
    }
  int dim = 0;
  for (int k = 1; k < 3; k++) if (mx[k] - mn[k] > mx[dim] - mn[dim]) dim = k;
  const int64_t mid = lo + (hi - lo) / 2;
  kd_select(m->pos, dim, &m->idx[lo], hi - lo, mid - lo);
  m->node_dim[node] = (int8_t)dim;
  m->node_split[node] = m->pos[(int64_t)m->idx[mid] * 3 + dim];
  if (par > 1 && hi - lo > 65536) {
    kd_task t = {m, 2 * node + 1, lo, mid, par / 2};
    pthread_t th;
    if (pthread_create(&th, NULL, kd_build_thread, &t) == 0) {
      kd_build(m, 2 * node + 2, mid, hi, par - par / 2);
      pthread_join(th, NULL);
      return;
    }
  }
  kd_build(m, 2 * node + 1, lo, mid, 1);
  kd_build(m, 2 * node + 2, mid, hi, 1);
}

/* threads of the map build (orc_set_build_threads; default 1) */
static int orc_build_threads = 1;
void orc_set_build_threads(int32_t n) { orc_build_threads = n < 1 ? 1 : (n > 256 ? 256 : n); }

int orc_map_create(const pm_photon* a, int64_t na, float power_a,
                   const pm_photon* b, int64_t nb, float power_b, orc_map** out) {
  if (!out || na < 0 || nb < 0) return PM_ERR_INVALID;
  orc_map* m = (orc_map*)calloc(1, sizeof(orc_map));
  int64_t n = na + nb;
  m->n = n;
  m->pos = (float*)malloc(sizeof(float) * 3 * (size_t)(n + 1));
  m->col = (float*)malloc(sizeof(float) * 3 * (size_t)(n + 1));
  m->pw = (float*)malloc(sizeof(float) * (size_t)(n + 1));
  m->idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
  for (int64_t i = 0; i < n; i++) {
    const pm_photon* p = i < na ? &a[i] : &b[i - na];
    m->pos[i * 3 + 0] = p->pos.x; m->pos[i * 3 + 1] = p->pos.y; m->pos[i * 3 + 2] = p->pos.z;
    m->col[i * 3 + 0] = p->color.x; m->col[i * 3 + 1] = p->color.y; m->col[i * 3 + 2] = p->color.z;
    m->pw[i] = i < na ? power_a : power_b;
    m->idx[i] = (int32_t)i;
  }
  int32_t nn = 1;
  while ((int64_t)nn * 8 < n * 2 && nn < (1 << 26)) nn *= 2;
  m->nnodes = 2 * nn;
  m->node_lo = (int32_t*)calloc((size_t)m->nnodes, sizeof(int32_t));
  m->node_hi = (int32_t*)calloc((size_t)m->nnodes, sizeof(int32_t));
  m->node_dim = (int8_t*)calloc((size_t)m->nnodes, sizeof(int8_t));
  m->node_split = (float*)calloc((size_t)m->nnodes, sizeof(float));
  kd_build(m, 0, 0, n, orc_build_threads);
  *out = m;
  return PM_OK;
}
static void refkd_destroy(struct orc_refkd* r);
void orc_map_destroy(orc_map* m) {
  if (!m) return;
  refkd_destroy(m->ref);
  free(m->pos); free(m->col); free(m->pw); free(m->idx);
  free(m->node_lo); free(m->node_hi); free(m->node_dim); free(m->node_split);
  free(m);
}

/* ------------------------------------------------------------------------ */
/* The left-balanced layout of cukd::buildTree<Photon, Photon_traits>
 * (ray-tracer/src/hostCode.cu:94-95; traits ray-tracer/include/photon.h:23-40,
 * has_explicit_dim), as THIS BUILD SPECIFIES it: the layout
 * tests are spec-pinned, cukd-unpinned. cudaKDTree is an empty submodule in
 * the reference, and two of the rules below are this build's own choices:
 *   - the split dimension comes from the extent of the subtree's own POINTS;
 *     cudaKDTree's explicit-dim builders may take it from the node's domain
 *     box instead (the world bounds, which the reference passes as
 *     globalPhotonsBounds, clipped at every ancestor's split plane);
 *   - ties between equal coordinates break by original index (the
 *     reference's thrust sort leaves their order unspecified).
 * The rules:
 *   - the tree is the implicit complete binary tree, children 2t+1 / 2t+2, over
 *     the n records in place; subtree t holds s elements, its root the element
 *     of rank left_size(s) (complete-tree left subtree size), the left child the
 *     ls smaller elements, the right child the rest;
 *   - order along dimension d = (orderable float key of coordinate d, original
 *     index): -0.0 and +0.0 are one key, NaN is taken as +inf (include/pm.h);
 *   - split dimension = the widest extent max - min (f32, from the subtree's
 *     smallest and largest key), first dimension on a tie; written per node
 *     (Photon_traits::set_dim, photon.h:36-39).
 * This is an independent recursive restatement (quickselect per subtree), not
 * the HIP level-by-level build; node t's output tag is orig << 2 | dim. */
typedef struct { uint32_t k[3]; int32_t id; } lb_elem;

static inline uint32_t lb_key(float f) {
  if (f != f) f = INFINITY;
  if (f == 0.0f) f = 0.0f;
  uint32_t u;
  memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
static inline float lb_unkey(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static inline uint64_t lb_ord(const lb_elem* e, int d) { return (uint64_t)e->k[d] << 32 | (uint32_t)e->id; }

int64_t orc_left_size(int64_t s) {
  if (s <= 1) return 0;
  int h = 0;
  while (((int64_t)1 << h) <= s) h++;            /* levels */
  const int64_t half = (int64_t)1 << (h - 2);     /* left subtree's last-level capacity */
  const int64_t full = ((int64_t)1 << (h - 1)) - 1;
  const int64_t last = s - full;
  return (half - 1) + (last < half ? last : half);
}

/* v[0..n): v[k] = rank-k element in (key d, index) order, smaller ones before it */
static void lb_select(lb_elem* v, int64_t n, int64_t k, int d) {
  int64_t lo = 0, hi = n - 1;
  while (hi > lo) {
    const int64_t mid = lo + (hi - lo) / 2;
    const uint64_t a = lb_ord(&v[lo], d), b = lb_ord(&v[mid], d), c = lb_ord(&v[hi], d);
    const uint64_t pv = a < b ? (b < c ? b : (a < c ? c : a)) : (a < c ? a : (b < c ? c : b));
    int64_t i = lo, j = hi;
    while (i <= j) {
      while (lb_ord(&v[i], d) < pv) i++;
      while (pv < lb_ord(&v[j], d)) j--;
      if (i <= j) {
        const lb_elem t = v[i]; v[i] = v[j]; v[j] = t;
        i++; j--;
      }
    }
    if (k <= j) hi = j;
    else if (k >= i) lo = i;
    else return;
  }
}

typedef struct { lb_elem* e; int32_t* tags; int64_t t, lo, hi; int par; } lb_task;
static void lb_build(lb_elem* e, int32_t* tags, int64_t t, int64_t lo, int64_t hi, int par);
static void* lb_thread(void* arg) {
  lb_task* k = (lb_task*)arg;
  lb_build(k->e, k->tags, k->t, k->lo, k->hi, k->par);
  return NULL;
}
static void lb_build(lb_elem* e, int32_t* tags, int64_t t, int64_t lo, int64_t hi, int par) {
  for (;;) {
    const int64_t s = hi - lo;
    if (s <= 0) return;
    uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    for (int64_t i = lo; i < hi; i++)
      for (int d = 0; d < 3; d++) {
        const uint32_t k = e[i].k[d];
        if (k < mn[d]) mn[d] = k;
        if (k > mx[d]) mx[d] = k;
      }
    float ext[3];
    for (int d = 0; d < 3; d++) ext[d] = lb_unkey(mx[d]) - lb_unkey(mn[d]);
    int dim = 0;
    if (ext[1] > ext[dim]) dim = 1;
    if (ext[2] > ext[dim]) dim = 2;
    const int64_t ls = orc_left_size(s);
    lb_select(&e[lo], s, ls, dim);
    tags[t] = (int32_t)((uint32_t)e[lo + ls].id << 2 | (uint32_t)dim);
    if (par > 1 && s > 65536) {
      lb_task k = {e, tags, 2 * t + 1, lo, lo + ls, par / 2};
      pthread_t th;
      if (pthread_create(&th, NULL, lb_thread, &k) == 0) {
        lb_build(e, tags, 2 * t + 2, lo + ls + 1, hi, par - par / 2);
        pthread_join(th, NULL);
        return;
      }
    }
    lb_build(e, tags, 2 * t + 1, lo, lo + ls, 1);
    t = 2 * t + 2;   /* right subtree: iterate */
    lo = lo + ls + 1;
  }
}

int orc_kd_left_balanced(const float* pos, int64_t stride, int64_t n, int32_t nthreads, int32_t* tags) {
  if (n < 0 || stride < 3 || (n > 0 && (!pos || !tags)) || n >= ((int64_t)1 << 30)) return PM_ERR_INVALID;
  if (n == 0) return PM_OK;
  lb_elem* e = (lb_elem*)malloc(sizeof(lb_elem) * (size_t)n);
  if (!e) return PM_ERR_INVALID;
  for (int64_t i = 0; i < n; i++) {
    for (int d = 0; d < 3; d++) e[i].k[d] = lb_key(pos[i * stride + d]);
    e[i].id = (int32_t)i;
  }
  lb_build(e, tags, 0, 0, n, nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads));
  free(e);
  return PM_OK;
}

typedef struct { float d2; int32_t id; } cand;
static inline int cand_less(cand a, cand b) { return a.d2 < b.d2 || (a.d2 == b.d2 && a.id < b.id); }
typedef struct { cand* h; int k, cnt; float r2; } heap_t;
static void heap_push(heap_t* H, cand c) {
  if (!(c.d2 < H->r2)) return;
  if (H->cnt < H->k) {
    int i = H->cnt++;
    H->h[i] = c;
    while (i > 0) {
      int p = (i - 1) / 2;
      if (cand_less(H->h[p], H->h[i])) { cand t = H->h[p]; H->h[p] = H->h[i]; H->h[i] = t; i = p; }
      else break;
    }
    return;
  }
  if (!cand_less(c, H->h[0])) return;
  H->h[0] = c;
  int i = 0;
  for (;;) {
    int l = 2 * i + 1, r = l + 1, b = i;
    if (l < H->k && cand_less(H->h[b], H->h[l])) b = l;
    if (r < H->k && cand_less(H->h[b], H->h[r])) b = r;
    if (b == i) break;
    cand t = H->h[b]; H->h[b] = H->h[i]; H->h[i] = t; i = b;
  }
}
static inline float heap_bound(const heap_t* H) { return H->cnt < H->k ? H->r2 : H->h[0].d2; }

static void knn_rec(const orc_map* m, int32_t node, const float q[3], heap_t* H) {
  if (m->node_dim[node] < 0) {
    for (int32_t i = m->node_lo[node]; i < m->node_hi[node]; i++) {
      int32_t pid = m->idx[i];
      const float* p = &m->pos[(int64_t)pid * 3];
      /* cukd sqrDistance == dot(q - p, q - p) */
      float dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
      cand c = {dx * dx + dy * dy + dz * dz, pid};
      heap_push(H, c);
    }
    return;
  }
  int dim = m->node_dim[node];
  float diff = q[dim] - m->node_split[node];
  int32_t nearc = diff < 0.f ? 2 * node + 1 : 2 * node + 2;
  int32_t farc = diff < 0.f ? 2 * node + 2 : 2 * node + 1;
  knn_rec(m, nearc, q, H);
  if (diff * diff <= heap_bound(H)) knn_rec(m, farc, q, H);
}
static int cmp_cand(const void* a, const void* b) {
  cand x = *(const cand*)a, y = *(const cand*)b;
  return cand_less(x, y) ? -1 : (cand_less(y, x) ? 1 : 0);
}
/* k nearest, sorted ascending by (d2, id); returns max d2 (radius^2 if not full) */
static float knn_one(const orc_map* m, const float q[3], int k, float radius, cand* buf) {
  heap_t H = {buf, k, 0, radius * radius};
  if (m->n > 0) knn_rec(m, 0, q, &H);
  float r2 = heap_bound(&H);
  qsort(buf, (size_t)H.cnt, sizeof(cand), cmp_cand);
  for (int i = H.cnt; i < k; i++) { buf[i].d2 = H.r2; buf[i].id = -1; }
  return r2;
}

typedef struct {
  const orc_map* m; const pm_float3* q; int k; float radius;
  int32_t* ids; float* d2; float* maxd2;
} knn_ctx;
static void knn_range(void* vc, int64_t lo, int64_t hi) {
  knn_ctx* c = (knn_ctx*)vc;
  cand* buf = (cand*)malloc(sizeof(cand) * (size_t)c->k);
  for (int64_t i = lo; i < hi; i++) {
    float q[3] = {c->q[i].x, c->q[i].y, c->q[i].z};
    float r2 = knn_one(c->m, q, c->k, c->radius, buf);
    for (int j = 0; j < c->k; j++) {
      c->ids[i * c->k + j] = buf[j].id;
      if (c->d2) c->d2[i * c->k + j] = buf[j].d2;
    }
    if (c->maxd2) c->maxd2[i] = r2;
  }
  free(buf);
}
int orc_knn(const orc_map* m, const pm_float3* q, int64_t nq, int32_t k, float max_radius,
            int32_t nthreads, int32_t* ids, float* d2, float* maxd2) {
  if (!m || k < 1 || k > 256) return PM_ERR_INVALID;
  knn_ctx c = {m, q, k, max_radius, ids, d2, maxd2};
  parallel_for(nq, 256, nthreads, knn_range, &c);
  return PM_OK;
}

/* shading.h:93-121 gatherPhotons; sum in (d^2, id) order. k = K_NEAREST is the
 * reference's; config 5 gathers caustics over k = 200. */
static v3 gather_ref(const orc_map* m, v3 hit, float brdf, int k);
static v3 gather_one_k(const orc_map* m, v3 hit, float brdf, int k, cand* buf) {
  if (m->ref) return gather_ref(m, hit, brdf, k);
  float q[3] = {hit.x, hit.y, hit.z};
  const float r2 = knn_one(m, q, k, K_MAX_DISTANCE, buf);
  v3 flux = V3(0.f, 0.f, 0.f);
  for (int p = 0; p < k; p++) {
    const int32_t id = buf[p].id;
    if (id < 0 || id > m->n) continue;
    const float power = m->pw[id];
    const v3 ppos = V3(m->pos[(int64_t)id * 3], m->pos[(int64_t)id * 3 + 1], m->pos[(int64_t)id * 3 + 2]);
    const v3 pcol = V3(m->col[(int64_t)id * 3], m->col[(int64_t)id * 3 + 1], m->col[(int64_t)id * 3 + 2]);
    const float dist = norm3(sub(ppos, hit));
    const float w = 1 - (dist / sqrtf(r2) * CONE_FILTER_C);
    flux = add(flux, smul(brdf * power * w, pcol));
  }
  return divf(flux, (1 - (2.f / 3.f) * (1.f / CONE_FILTER_C)) * 2 * PI_F * r2);
}
static v3 gather_one(const orc_map* m, v3 hit, float brdf, cand* buf) {
  return gather_one_k(m, hit, brdf, K_NEAREST, buf);
}
typedef struct { const orc_map* m; const pm_float3* p; const float* brdf; pm_float3* out; int k; } gather_ctx;
static void gather_range(void* vc, int64_t lo, int64_t hi) {
  gather_ctx* c = (gather_ctx*)vc;
  cand buf[256];
  for (int64_t i = lo; i < hi; i++) c->out[i] = top3(gather_one_k(c->m, fromp(c->p[i]), c->brdf[i], c->k, buf));
}
int orc_gather_k(const orc_map* m, const pm_float3* pts, const float* brdf, int64_t nq, int32_t k,
                 int32_t nthreads, pm_float3* out) {
  if (!m || k < 1 || k > 256) return PM_ERR_INVALID;
  gather_ctx c = {m, pts, brdf, out, k};
  parallel_for(nq, 256, nthreads, gather_range, &c);
  return PM_OK;
}
int orc_gather(const orc_map* m, const pm_float3* pts, const float* brdf, int64_t nq,
               int32_t nthreads, pm_float3* out) {
  return orc_gather_k(m, pts, brdf, nq, K_NEAREST, nthreads, out);
}

/* ------------------------------------------------------------------------ */
/* Alternative specifications (orc_map_set_spec): what the reference could do
 * where this build's spec had to choose, restated so that
 * their effect on the image can be measured (tests/test_spec_bounds.py). NOT
 * the product's spec and not a parity target: a bound on the unpinned choices.
 * cudaKDTree is an empty submodule in the reference; what follows restates its
 * published algorithm as the reference calls it:
 *   - tree: cukd::buildTree<Photon, Photon_traits> (ray-tracer/src/hostCode.cu:
 *     85-95), the in-place left-balanced layout of orc_kd_left_balanced, the
 *     photons reordered into tree order (the reference gathers from that array);
 *     ORC_SPEC_DOMAIN_DIM: each node's split dimension is the widest extent of
 *     its DOMAIN box -- the world bounds of all points (the buildTree output the
 *     reference passes as globalPhotonsBounds), clipped at every ancestor's split
 *     plane (left child: upper = the split coordinate, right: lower = it) --
 *     instead of the extent of the subtree's own points;
 *   - kNN (ORC_SPEC_HEAP, required): cukd::stackBased::knn with a
 *     HeapCandidateList<k> (shading.h:11-18): a pre-order walk (test the node's
 *     point, push the far child when its plane distance^2 < the cull distance,
 *     descend to the close child; pop entries not culled), candidates kept as
 *     64-bit (d^2 bits << 32 | TREE index) in a max-heap initialised to
 *     (max_radius^2, -1) (replace the root, sift down); a candidate enters when
 *     its key is below the heap's root;
 *   - gatherPhotons (shading.h:93-121) over the heap ARRAY order, ids being tree
 *     indices into the reordered photons (the `id > num_photons` test kept);
 *   - ORC_SPEC_FMA: nvcc's default contraction (-fmad=true): the squared
 *     distances as fma(z, z, fma(y, y, x * x)), the cone weight as
 *     fma(-dist / r, C, 1) and the flux sum as fma(s, colour, flux). */
#define ORC_SPEC_DOMAIN_DIM 1
#define ORC_SPEC_HEAP 2
#define ORC_SPEC_FMA 4
struct orc_refkd {
  int flags;
  int64_t n;
  float* pos; float* col; float* pw;   /* tree order */
  int8_t* dim;
};
static void refkd_destroy(struct orc_refkd* r) {
  if (!r) return;
  free(r->pos); free(r->col); free(r->pw); free(r->dim);
  free(r);
}
/* lb_build with the split dimension taken from the node's domain box */
typedef struct { lb_elem* e; int32_t* tags; int64_t t, lo, hi; float blo[3], bhi[3]; int par; } lbd_task;
static void lbd_build(lb_elem* e, int32_t* tags, int64_t t, int64_t lo, int64_t hi, const float blo_in[3],
                      const float bhi_in[3], int par);
static void* lbd_thread(void* arg) {
  lbd_task* k = (lbd_task*)arg;
  lbd_build(k->e, k->tags, k->t, k->lo, k->hi, k->blo, k->bhi, k->par);
  return NULL;
}
static void lbd_build(lb_elem* e, int32_t* tags, int64_t t, int64_t lo, int64_t hi, const float blo_in[3],
                      const float bhi_in[3], int par) {
  float blo[3] = {blo_in[0], blo_in[1], blo_in[2]}, bhi[3] = {bhi_in[0], bhi_in[1], bhi_in[2]};
  for (;;) {
    const int64_t s = hi - lo;
    if (s <= 0) return;
    int dim = 0;   /* arg_max of the box size, first on a tie */
    for (int d = 1; d < 3; d++)
      if (bhi[d] - blo[d] > bhi[dim] - blo[dim]) dim = d;
    const int64_t ls = orc_left_size(s);
    lb_select(&e[lo], s, ls, dim);
    tags[t] = (int32_t)((uint32_t)e[lo + ls].id << 2 | (uint32_t)dim);
    const float split = lb_unkey(e[lo + ls].k[dim]);
    float lhi[3] = {bhi[0], bhi[1], bhi[2]};
    lhi[dim] = split;
    if (par > 1 && s > 65536) {
      lbd_task k = {e, tags, 2 * t + 1, lo, lo + ls, {blo[0], blo[1], blo[2]}, {lhi[0], lhi[1], lhi[2]}, par / 2};
      pthread_t th;
      if (pthread_create(&th, NULL, lbd_thread, &k) == 0) {
        float rlo[3] = {blo[0], blo[1], blo[2]};
        rlo[dim] = split;
        lbd_build(e, tags, 2 * t + 2, lo + ls + 1, hi, rlo, bhi, par - par / 2);
        pthread_join(th, NULL);
        return;
      }
    }
    lbd_build(e, tags, 2 * t + 1, lo, lo + ls, blo, lhi, 1);
    blo[dim] = split;   /* right subtree: iterate */
    t = 2 * t + 2;
    lo = lo + ls + 1;
  }
}

int orc_map_set_spec(orc_map* m, int32_t flags, int32_t nthreads) {
  if (!m || (flags & ~7) || (flags && !(flags & ORC_SPEC_HEAP)) || m->n >= ((int64_t)1 << 30)) return PM_ERR_INVALID;
  refkd_destroy(m->ref);
  m->ref = NULL;
  if (!flags) return PM_OK;
  const int64_t n = m->n;
  struct orc_refkd* r = (struct orc_refkd*)calloc(1, sizeof(*r));
  r->flags = flags;
  r->n = n;
  r->pos = (float*)malloc(sizeof(float) * 3 * (size_t)(n + 1));
  r->col = (float*)malloc(sizeof(float) * 3 * (size_t)(n + 1));
  r->pw = (float*)malloc(sizeof(float) * (size_t)(n + 1));
  r->dim = (int8_t*)malloc((size_t)(n + 1));
  int32_t* tags = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
  const int par = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
  if (!(flags & ORC_SPEC_DOMAIN_DIM)) {
    orc_kd_left_balanced(m->pos, 3, n, par, tags);
  } else if (n > 0) {
    lb_elem* e = (lb_elem*)malloc(sizeof(lb_elem) * (size_t)n);
    float blo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = 0; i < n; i++) {
      for (int d = 0; d < 3; d++) {
        const float c = m->pos[i * 3 + d];
        e[i].k[d] = lb_key(c);
        blo[d] = fminf(blo[d], c);
        bhi[d] = fmaxf(bhi[d], c);
      }
      e[i].id = (int32_t)i;
    }
    lbd_build(e, tags, 0, 0, n, blo, bhi, par);
    free(e);
  }
  for (int64_t t = 0; t < n; t++) {
    const int64_t o = (uint32_t)tags[t] >> 2;
    for (int d = 0; d < 3; d++) {
      r->pos[t * 3 + d] = m->pos[o * 3 + d];
      r->col[t * 3 + d] = m->col[o * 3 + d];
    }
    r->pw[t] = m->pw[o];
    r->dim[t] = (int8_t)(tags[t] & 3);
  }
  free(tags);
  m->ref = r;
  return PM_OK;
}

static inline uint64_t hc_encode(float d2, int32_t id) {
  uint32_t u;
  memcpy(&u, &d2, 4);
  return (uint64_t)u << 32 | (uint32_t)id;
}
static inline float hc_d2(uint64_t e) {
  const uint32_t u = (uint32_t)(e >> 32);
  float f;
  memcpy(&f, &u, 4);
  return f;
}
/* HeapCandidateList<k>::push: replace the root, sift down; returns maxRadius2 */
static float hc_push(uint64_t* h, int k, float d2, int32_t id) {
  const uint64_t e = hc_encode(d2, id);
  if (e >= h[0]) return hc_d2(h[0]);
  int pos = 0;
  for (;;) {
    const int c1 = 2 * pos + 1, c2 = c1 + 1;
    int big = k;
    uint64_t bv = 0;
    if (c1 < k) { big = c1; bv = h[c1]; }
    if (c2 < k && h[c2] > bv) { big = c2; bv = h[c2]; }
    if (big == k || bv < e) { h[pos] = e; break; }
    h[pos] = bv;
    pos = big;
  }
  return hc_d2(h[0]);
}
static inline float ref_d2(const float* p, const float q[3], int fma_on) {
  const float dx = p[0] - q[0], dy = p[1] - q[1], dz = p[2] - q[2];
  if (fma_on) return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
  return dx * dx + dy * dy + dz * dz;
}
static v3 gather_ref(const orc_map* m, v3 hit, float brdf, int k) {
  const struct orc_refkd* r = m->ref;
  const int fm = (r->flags & ORC_SPEC_FMA) != 0;
  const float q[3] = {hit.x, hit.y, hit.z};
  uint64_t h[256];
  const float cut = K_MAX_DISTANCE;
  for (int i = 0; i < k; i++) h[i] = hc_encode(cut * cut, -1);
  /* cukd::stackBased::knn */
  struct { int32_t node; float d2; } stack[64];
  int sp = 0;
  float cull = hc_d2(h[0]);
  int64_t node = 0;
  const int64_t n = r->n;
  for (;;) {
    while (node < n) {
      const float* p = &r->pos[node * 3];
      cull = hc_push(h, k, ref_d2(p, q, fm), (int32_t)node);
      const int dim = r->dim[node];
      const float diff = q[dim] - p[dim];
      const int64_t l = 2 * node + 1;
      const int left_close = q[dim] < p[dim];
      const int64_t close_c = left_close ? l : l + 1, far_c = left_close ? l + 1 : l;
      const float pd2 = diff * diff;
      if (pd2 < cull && far_c < n) {
        stack[sp].node = (int32_t)far_c;
        stack[sp].d2 = pd2;
        sp++;
      }
      node = close_c;
    }
    int found = 0;
    while (sp > 0) {
      sp--;
      if (stack[sp].d2 >= cull) continue;
      node = stack[sp].node;
      found = 1;
      break;
    }
    if (!found) break;
  }
  const float r2 = cull;
  /* gatherPhotons over the heap array */
  v3 flux = V3(0.f, 0.f, 0.f);
  for (int i = 0; i < k; i++) {
    const int32_t id = (int32_t)(uint32_t)h[i];
    if (id < 0 || id > n) continue;
    const float* p = &r->pos[(int64_t)id * 3];
    const float* c = &r->col[(int64_t)id * 3];
    const float dist = sqrtf(ref_d2(p, q, fm));
    if (fm) {
      const float w = fmaf(-(dist / sqrtf(r2)), CONE_FILTER_C, 1.f);
      const float sc = brdf * r->pw[id] * w;
      flux = V3(fmaf(sc, c[0], flux.x), fmaf(sc, c[1], flux.y), fmaf(sc, c[2], flux.z));
    } else {
      const float w = 1 - (dist / sqrtf(r2) * CONE_FILTER_C);
      flux = add(flux, smul(brdf * r->pw[id] * w, V3(c[0], c[1], c[2])));
    }
  }
  return divf(flux, (1 - (2.f / 3.f) * (1.f / CONE_FILTER_C)) * 2 * PI_F * r2);
}

/* ------------------------------------------------------------------------ */
/* Render (ray-tracer/cuda/deviceCode.cu:25-231, shading.h:20-91)             */
int orc_camera_setup(pm_float3 look_from, pm_float3 look_at, pm_float3 look_up, float fovy,
                     int32_t w, int32_t h, pm_camera* out) {
  /* ray-tracer/src/hostCode.cu:100-108 (cos, not tan, kept) */
  const float aspect = (float)w / (float)h;
  const float cosf_ = cosf(fovy);
  v3 from = fromp(look_from), at = fromp(look_at), up = fromp(look_up);
  v3 d00 = normalize(sub(at, from));
  v3 du = smul(cosf_ * aspect, normalize(cross(d00, up)));
  v3 dv = smul(cosf_, normalize(cross(du, d00)));
  d00 = sub(d00, smul(0.5f, add(du, dv)));
  out->pos = top3(from); out->dir_00 = top3(d00); out->dir_du = top3(du); out->dir_dv = top3(dv);
  return PM_OK;
}

typedef struct { v3 hitpoint, normal; pm_material mat; } hitrec;
typedef struct { uint32_t rng; v3 colour; int missed; hitrec hr; } prd_t;

/* closestHit (deviceCode.cu:233-253) */
static void trace_closest(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, hitrec* hr, int* missed,
                          pm_render_stats* st) {
  float t;
  int64_t tri = closest_hit(s, o, d, tmin, tmax, &t);
  if (st) st->rays++;
  if (tri < 0) { *missed = 1; return; }
  hr->mat = s->mat[s->mesh[tri]];
  hr->hitpoint = add(o, mulf(d, t));
  const v3 n = prim_normal(s, tri);
  hr->normal = dot(d, n) < 0.f ? n : neg(n);
  hr->normal = normalize(hr->normal);
  *missed = 0;
}

/* shading.h:82-91 */
static float specular_brdf(float spec, v3 in_light, v3 out_dir, v3 n) {
  if (near_zero(sub(reflect(in_light, n), out_dir))) return spec;
  return 0;
}

typedef struct {
  const orc_scene* s; const pm_render_params* p; const pm_light* lights; int32_t nl;
  const orc_map* g; const orc_map* c;
} rctx;

/* ray_colour (deviceCode.cu:25-163) */
static v3 ray_colour(const rctx* R, v3 ro, v3 rd, prd_t* prd, cand* buf, pm_render_stats* st) {
  int missed;
  if (st) st->path_vertices++;
  trace_closest(R->s, ro, rd, EPS, INFTY_F, &prd->hr, &missed, st);
  if (missed) {
    prd->colour = fromp(R->p->sky_colour);
    prd->missed = 1;
    return prd->colour;
  }
  prd->colour = V3(0.f, 0.f, 0.f);
  prd->missed = 0;
  const v3 albedo = fromp(prd->hr.mat.albedo);
  const float diffuse_brdf = prd->hr.mat.diffuse / PI_F;
  v3 direct = V3(0.f, 0.f, 0.f);
  for (int l = 0; l < R->nl; l++) {
    const pm_light* L = &R->lights[l];
    const v3 org = prd->hr.hitpoint;
    v3 ldir = sub(fromp(L->pos), org);
    const float dist = norm3(ldir);
    ldir = normalize(ldir);
    const float ldn = dot(ldir, prd->hr.normal);
    if (ldn < 0.f) continue;
    int occ = any_hit(R->s, org, ldir, EPS, dist * (1.f - EPS));
    if (st) st->rays++;
    const float vis = occ ? 0.f : 1.f;
    const float sb = specular_brdf(prd->hr.mat.specular, ldir, rd, prd->hr.normal);
    const float pw = (float)L->power;
    const float inv = 1.f / (dist * dist);
    const float bs = diffuse_brdf + sb;
    v3 term = V3(vis * pw * ldn * inv * bs * L->rgb.x, vis * pw * ldn * inv * bs * L->rgb.y,
                 vis * pw * ldn * inv * bs * L->rgb.z);
    direct = add(direct, term);
  }
  const v3 direct_term = mulv(albedo, direct);
  if (st) st->caustic_queries++;
  const v3 caustics = gather_one_k(R->c, prd->hr.hitpoint, diffuse_brdf,
                                   R->p->caustic_k > 0 ? R->p->caustic_k : K_NEAREST, buf);
  v3 diffuse = V3(0.f, 0.f, 0.f);
  for (int s = 0; s < NUM_DIFFUSE_SAMPLES && diffuse_brdf > 0.f; s++) {
    const v3 n = normalize(prd->hr.normal);
    v3 rv, rdir;
    do {
      rv = random_unit_vector(&prd->rng);
      rdir = add(n, rv);
    } while (near_zero(rdir));
    rdir = normalize(rdir);
    hitrec dh;
    memset(&dh, 0, sizeof(dh));     /* uninitialised in the reference: zeroed */
    int dmiss;
    trace_closest(R->s, prd->hr.hitpoint, rdir, 3 * EPS, INFTY_F, &dh, &dmiss, st);
    if (dh.mat.diffuse > 0.f) {
      const float sdb = dh.mat.diffuse / PI_F;
      if (st) st->global_queries++;
      const v3 dc = gather_one(R->g, dh.hitpoint, sdb, buf);
      diffuse = add(diffuse, mulv(dc, fromp(dh.mat.albedo)));
    }
  }
  diffuse = divf(diffuse, (float)NUM_DIFFUSE_SAMPLES);
  diffuse = mulv(diffuse, albedo);
  return V3(DIFFUSE_FACTOR * diffuse.x + CAUSTICS_FACTOR * caustics.x + DIRECT_LIGHT_FACTOR * direct_term.x,
            DIFFUSE_FACTOR * diffuse.y + CAUSTICS_FACTOR * caustics.y + DIRECT_LIGHT_FACTOR * direct_term.y,
            DIFFUSE_FACTOR * diffuse.z + CAUSTICS_FACTOR * caustics.z + DIRECT_LIGHT_FACTOR * direct_term.z);
}

/* shading.h:20-55 calculate_refracted (Random by value) */
static v3 calculate_refracted(const pm_material* m, v3 rd, v3 n, uint32_t rng) {
  v3 outward, refracted = V3(0.f, 0.f, 0.f);
  float ni, R, cosine;
  if (dot(rd, n) > 0.f) {
    outward = neg(n);
    ni = m->refraction_idx;
    cosine = dot(rd, n);
    cosine = sqrtf(1.f - m->refraction_idx * m->refraction_idx * (1.f - cosine * cosine));
  } else {
    outward = n;
    ni = 1.f / m->refraction_idx;
    cosine = -dot(rd, n);
  }
  if (refract_uv(rd, outward, ni, &refracted))
    R = schlick(cosine, m->refraction_idx);
  else
    R = 1.f;
  if (orc_lcg_next(&rng) < R) return reflect(rd, n);
  return refracted;
}
/* shading.h:57-80 reflect_or_refract_ray (Random by value) */
static v3 reflect_or_refract(const pm_material* m, v3 rd, v3 n, uint32_t rng, int* absorbed, float* coef) {
  *absorbed = 0;
  const float r = orc_lcg_next(&rng);
  if (r < m->specular) { *coef = m->specular; return reflect(rd, n); }
  if (r < m->specular + m->transmission) { *coef = m->transmission; return calculate_refracted(m, rd, n, rng); }
  *coef = 0.f;
  *absorbed = 1;
  return V3(0.f, 0.f, 0.f);
}

static inline uint32_t make_rgba(v3 c) {
  /* owl make_rgba: clamp(int(f*256), 0, 255) per channel, alpha 0xff; NaN -> 0 */
  float f[3] = {c.x * 256.f, c.y * 256.f, c.z * 256.f};
  uint32_t r = 0xffu << 24;
  for (int i = 0; i < 3; i++) {
    int v;
    if (!(f[i] == f[i])) v = 0;
    else if (f[i] >= 2147483520.f) v = 255;
    else if (f[i] <= -2147483648.f) v = 0;
    else v = (int)f[i];
    if (v < 0) v = 0;
    if (v > 255) v = 255;
    r |= (uint32_t)v << (8 * i);
  }
  return r;
}

typedef struct { rctx R; int32_t row_lo, row_hi; uint32_t* rgba; float* rgb; pm_render_stats* stats;
                 pthread_mutex_t mu; } render_ctx;

/* simpleRayGen (deviceCode.cu:191-231) + tracePath (:165-189) */
static void render_rows(void* vc, int64_t lo, int64_t hi) {
  render_ctx* C = (render_ctx*)vc;
  const pm_render_params* P = C->R.p;
  cand buf[256];
  pm_render_stats st;
  memset(&st, 0, sizeof(st));
  for (int64_t yy = lo; yy < hi; yy++) {
    const int32_t py = C->row_lo + (int32_t)yy;
    for (int32_t px = 0; px < P->width; px++) {
      const int tile = (px / 16) + (py / 16) * ((P->width + 15) / 16);
      if (P->tile_count > 1 && tile % P->tile_count != P->tile_rank) continue;
      prd_t prd;
      memset(&prd, 0, sizeof(prd));   /* zero-initialised (reference: UB) */
      prd.rng = orc_lcg_init((uint32_t)px, (uint32_t)py);
      v3 fc = V3(0.f, 0.f, 0.f);
      st.pixels++;
      for (int s = 0; s < P->samples_per_pixel; s++) {
        const float ex = orc_lcg_next(&prd.rng);   /* vec2f(rnd(), rnd()): left to right */
        const float ey = orc_lcg_next(&prd.rng);
        const float su = ((float)px + ex) / (float)P->width;
        const float sv = ((float)py + ey) / (float)P->height;
        v3 ro = fromp(P->camera.pos);
        v3 rd = normalize(add(add(fromp(P->camera.dir_00), smul(su, fromp(P->camera.dir_du))),
                              smul(sv, fromp(P->camera.dir_dv))));
        v3 colour = V3(0.f, 0.f, 0.f), att = V3(1.f, 1.f, 1.f);
        for (int d = 0; d < P->max_depth; d++) {
          const v3 c = ray_colour(&C->R, ro, rd, &prd, buf, &st);
          colour = add(colour, mulv(c, att));
          int absorbed;
          float coef;
          const v3 od = reflect_or_refract(&prd.hr.mat, rd, prd.hr.normal, prd.rng, &absorbed, &coef);
          if (absorbed) break;
          att = mulv(att, smul(coef, fromp(prd.hr.mat.albedo)));
          ro = prd.hr.hitpoint;
          rd = od;
        }
        fc = add(fc, colour);
      }
      fc = mulf(fc, 1.f / (float)P->samples_per_pixel);
      const int32_t y = P->height - py;
      if (y >= P->height) continue;    /* pixelID.y == 0 writes past the buffer: dropped */
      const int64_t ofs = (int64_t)px + (int64_t)P->width * y;
      if (C->rgba) C->rgba[ofs] = make_rgba(fc);
      if (C->rgb) { C->rgb[ofs * 3] = fc.x; C->rgb[ofs * 3 + 1] = fc.y; C->rgb[ofs * 3 + 2] = fc.z; }
    }
  }
  if (C->stats) {
    pthread_mutex_lock(&C->mu);
    C->stats->pixels += st.pixels; C->stats->path_vertices += st.path_vertices;
    C->stats->caustic_queries += st.caustic_queries; C->stats->global_queries += st.global_queries;
    C->stats->rays += st.rays;
    pthread_mutex_unlock(&C->mu);
  }
}

int orc_render(const orc_scene* s, const pm_render_params* p, const pm_light* lights, int32_t nl,
               const orc_map* gmap, const orc_map* cmap, int32_t row_lo, int32_t row_hi,
               int32_t nthreads, uint32_t* rgba, float* rgb, pm_render_stats* stats) {
  if (!s || !p || !gmap || !cmap || p->width <= 0 || p->height <= 0 || p->samples_per_pixel <= 0)
    return PM_ERR_INVALID;
  if (row_hi <= row_lo) { row_lo = 0; row_hi = p->height; }
  render_ctx C;
  C.R.s = s; C.R.p = p; C.R.lights = lights; C.R.nl = nl; C.R.g = gmap; C.R.c = cmap;
  C.row_lo = row_lo; C.row_hi = row_hi; C.rgba = rgba; C.rgb = rgb; C.stats = stats;
  if (stats) memset(stats, 0, sizeof(*stats));
  pthread_mutex_init(&C.mu, NULL);
  parallel_for(row_hi - row_lo, 1, nthreads, render_rows, &C);
  pthread_mutex_destroy(&C.mu);
  return PM_OK;
}

/* -------------------------------------------------------------------------- */
/* Photon viewer (photon-viewer/src/hostCode.cu:53-75 projection with glm      */
/* 0.9.9 lookAtRH / perspectiveRH_NO / mat4 products; photonViewerRayGen,     */
/* photon-viewer/cuda/deviceCode.cu:10-38). Photons are painted in index order */
/* so the highest index wins a shared pixel (the device's atomicMax rule).     */
static float gdot(v3 a, v3 b) { const float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z; return tx + ty + tz; }
static v3 gnorm(v3 v) { const float inv = 1.0f / sqrtf(gdot(v, v)); return V3(v.x * inv, v.y * inv, v.z * inv); }
static v3 gcross(v3 x, v3 y) { return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }

void orc_viewer_matrix(const pm_viewer_params* P, float M[16]) {
  const v3 eye = fromp(P->look_from), ctr = fromp(P->look_at), up = fromp(P->look_up);
  const v3 f = gnorm(sub(ctr, eye));
  const v3 s = gnorm(gcross(f, up));
  const v3 u = gcross(s, f);
  float V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  V[0][0] = s.x; V[1][0] = s.y; V[2][0] = s.z;
  V[0][1] = u.x; V[1][1] = u.y; V[2][1] = u.z;
  V[0][2] = -f.x; V[1][2] = -f.y; V[2][2] = -f.z;
  V[3][0] = -gdot(s, eye); V[3][1] = -gdot(u, eye); V[3][2] = gdot(f, eye);
  const float aspect = (float)P->width / (float)P->height;
  const float zn = 0.1f, zf = 1000.f;
  const float th = tanf(P->fovy / 2.0f);
  float Pm[4][4] = {{0}};
  Pm[0][0] = 1.0f / (aspect * th);
  Pm[1][1] = 1.0f / th;
  Pm[2][2] = -(zf + zn) / (zf - zn);
  Pm[2][3] = -1.0f;
  Pm[3][2] = -(2.0f * zf * zn) / (zf - zn);
  for (int i = 0; i < 4; i++)
    for (int r = 0; r < 4; r++) {
      float acc = Pm[0][r] * V[i][0];
      acc = acc + Pm[1][r] * V[i][1];
      acc = acc + Pm[2][r] * V[i][2];
      acc = acc + Pm[3][r] * V[i][3];
      M[4 * i + r] = acc;
    }
}

int orc_photon_view(const orc_scene* s, const pm_photon* ph, int64_t n, const pm_viewer_params* P, uint32_t* rgba) {
  if (!s || !P || P->width <= 0 || P->height <= 0 || !rgba) return PM_ERR_INVALID;
  const int W = P->width, H = P->height;
  for (int64_t i = 0; i < (int64_t)W * H; i++) rgba[i] = 0xFF000000u;
  float M[16];
  orc_viewer_matrix(P, M);
  const v3 eye = fromp(P->look_from);
  for (int64_t i = 0; i < n; i++) {
    const pm_float3 p = ph[i].pos;
    float c[4];
    for (int r = 0; r < 4; r++) {
      const float a0 = M[0 + r] * p.x + M[4 + r] * p.y;
      const float a1 = M[8 + r] * p.z + M[12 + r];
      c[r] = a0 + a1;
    }
    if (c[2] < 0.f) continue;
    const float fx = (c[0] / c[3] + 1.f) * 0.5f * (float)W;
    const float fy = (c[1] / c[3] + 1.f) * 0.5f * (float)H;
    if (!(fx > -2147483648.f && fx < 2147483648.f) || !(fy > -2147483648.f && fy < 2147483648.f)) continue;
    const int px = (int)fx, py = H - (int)fy;
    if (px < 0 || px >= W || py < 0 || py >= H) continue;
    const v3 d = V3(p.x - eye.x, p.y - eye.y, p.z - eye.z);
    const float tmax = (float)(sqrt((double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z) - (double)1e-4f);
    if (any_hit(s, eye, normalize(d), 0.0f, tmax)) continue;
    rgba[px + (int64_t)W * py] = make_rgba(fromp(ph[i].color));
  }
  return PM_OK;
}

/* %.6f text round trip without the text (see quantize6 in pm_device.hpp). */
static float quantize6_pos(float a) {
  const double m = rint((double)a * 1e6);
  const double q = m / 1e6;
  float f = (float)q;
  const float fl = (double)f > q ? nextafterf(f, 0.0f) : f;
  const float fh = nextafterf(fl, INFINITY);
  const double mid = ((double)fl + (double)fh) * 0.5;
  if (q == mid) {
    const double r = fma(-q, 1e6, m);
    if (r > 0) f = fh;
    else if (r < 0) f = fl;
  }
  return f;
}
void orc_quantize6(const float* in, float* out, int64_t n) {
  for (int64_t i = 0; i < n; i++) out[i] = signbit(in[i]) ? -quantize6_pos(-in[i]) : quantize6_pos(in[i]);
}
