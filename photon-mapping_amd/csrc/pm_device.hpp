// pm_device.hpp — device-side arithmetic for the photon-mapping hot path (gfx950).
//
// Every function here implements the arithmetic spec of DESIGN.md §2 so that
// the HIP kernels and the CPU oracle (oracle/pm_oracle.c, an independent C
// restatement) compute bit-identical floats. Compiled with
// -ffp-contract=off (no FMA contraction) and correctly rounded f32 div/sqrt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pm.h"

namespace pmd {

constexpr float kEPS = 1e-3f;                       // common/cuda/helpers.h:8
constexpr float kPI = (float)3.141592653;            // helpers.h:9
constexpr float kINFTY = 1e10f;                      // helpers.h:7
constexpr float kPhotonTmax = 1e30f;                 // owl::Ray default tmax
constexpr int kKNearest = 50;                        // ray-tracer/cuda/shading.h:7
constexpr float kKMaxDistance = 100.0f;              // shading.h:8
constexpr float kConeFilterC = 1.1f;                 // shading.h:9
constexpr int kNumDiffuseSamples = 20;               // ray-tracer/cuda/deviceCode.cu:15
constexpr float kDirectLightFactor = 0.8f;           // deviceCode.cu:10
constexpr float kCausticsFactor = 0.08f;             // deviceCode.cu:11
constexpr float kDiffuseFactor = 0.2f;               // deviceCode.cu:12

enum { EV_MISS = 0, EV_ABSORBED = 1, EV_DIFFUSE = 2, EV_SPECULAR = 4, EV_REFRACT = 8 };

struct v3 {
  float x, y, z;
};
__host__ __device__ __forceinline__ v3 mk(float x, float y, float z) { return {x, y, z}; }
__host__ __device__ __forceinline__ v3 mk(pm_float3 p) { return {p.x, p.y, p.z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 mulf(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ v3 smul(float s, v3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ v3 mulv(v3 a, v3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ v3 divf(v3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ v3 neg(v3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v3 cross(v3 a, v3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// owl normalize(v) = v * rsqrt(dot(v,v)); spec: rsqrt := 1/sqrtf (IEEE)
__device__ __forceinline__ v3 normalize(v3 v) { return mulf(v, 1.0f / sqrtf(dot(v, v))); }
__device__ __forceinline__ float norm3(v3 v) { return sqrtf(dot(v, v)); }
__device__ __forceinline__ bool near_zero(v3 v) { return v.x < kEPS && v.y < kEPS && v.z < kEPS; }
__device__ __forceinline__ float comp(v3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// owl::LCG<16>
__device__ __forceinline__ uint32_t lcg_init(uint32_t val0, uint32_t val1) {
  uint32_t v0 = val0, v1 = val1, s0 = 0;
#pragma unroll
  for (int n = 0; n < 16; n++) {
    s0 += 0x9e3779b9u;
    v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
    v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
  }
  return v0;
}
__device__ __forceinline__ float lcg_next(uint32_t& st) {
  st = 1664525u * st + 1013904223u;
  return (float)(st & 0x00FFFFFFu) / (float)0x01000000;
}

// Deterministic acos / sincos
__device__ __forceinline__ float acos_spec(float x) {
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
__device__ __forceinline__ void sincos_spec(float x, float& s, float& c) {
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
    case 0: s = sp; c = cp; break;
    case 1: s = cp; c = -sp; break;
    case 2: s = -sp; c = -cp; break;
    default: s = -cp; c = sp; break;
  }
}

// helpers.h:27-34
__device__ __forceinline__ v3 random_point_in_unit_sphere(uint32_t& st) {
  const float u = lcg_next(st);
  const float v = lcg_next(st);
  const float theta = 2.f * kPI * u;
  const float phi = acos_spec(2.f * v - 1.f);
  float sp, cp, sth, cth;
  sincos_spec(phi, sp, cp);
  sincos_spec(theta, sth, cth);
  return {sp * cth, sp * sth, cp};
}
// helpers.h:36-43
__device__ __forceinline__ v3 random_unit_vector(uint32_t& st) {
  v3 v;
  do {
    v.x = 2.f * lcg_next(st) - 1.f;
    v.y = 2.f * lcg_next(st) - 1.f;
    v.z = 2.f * lcg_next(st) - 1.f;
  } while (dot(v, v) >= 1.f);
  return normalize(v);
}
// helpers.h:45-51
__device__ __forceinline__ v3 cosine_sample_hemisphere(v3 n, uint32_t& st) {
  return normalize(add(n, mulf(random_point_in_unit_sphere(st), (1 - kEPS))));
}
__device__ __forceinline__ v3 reflect(v3 i, v3 n) { return sub(i, mulf(n, 2.f * dot(i, n))); }
// helpers.h:57-74
__device__ __forceinline__ v3 refract_ior(v3 in, v3 n, float ior) {
  float ct = -dot(in, n);
  float mu;
  if (ct > 0.f) {
    mu = 1.f / ior;
  } else {
    mu = ior;
    ct = -ct;
  }
  const float cphi = 1.f - mu * mu * (1.f - ct * ct);
  if (cphi >= 0) return add(smul(mu, in), smul(mu * ct - sqrtf(cphi), n));
  return reflect(in, n);
}
// helpers.h:91-106
__device__ __forceinline__ bool refract_uv(v3 v, v3 n, float ni, v3& refracted) {
  const v3 uv = normalize(v);
  const float dt = dot(uv, n);
  const float disc = 1.0f - ni * ni * (1 - dt * dt);
  if (disc > 0.f) {
    refracted = sub(smul(ni, sub(uv, mulf(n, dt))), mulf(n, sqrtf(disc)));
    return true;
  }
  return false;
}
// helpers.h:108-112 (double; pow(x,5) := ((x*x)*(x*x))*x)
__device__ __forceinline__ float schlick(float cosv, float ior) {
  float r0 = (float)((1. - (double)ior) / (1. + (double)ior));
  r0 = r0 * r0;
  double x = 1. - (double)cosv;
  double x2 = x * x;
  double p5 = (x2 * x2) * x;
  return (float)((double)r0 + (1. - (double)r0) * p5);
}

// ---------------------------------------------------------------- scene
// Triangle record (48 B, 3 x float4): A.xyz|mesh, B.xyz|prim, C.xyz|global tri id.
// BVH4 node (128 B): SoA boxes of 4 children + child codes (see traverse).
struct DevScene {
  const float4* tri;       // [3*T] in leaf (Morton) order
  const float4* nodes;     // [8 * nnodes] BVH4
  const float4* mat;       // [2*nmesh]: (albedo, diffuse), (specular, transmission, ior, 0)
  int32_t ntri;
  int32_t nnodes;
};

struct Ray {
  v3 o, d, inv;
  int kx, ky, kz;
  float Sx, Sy, Sz;
};
__device__ __forceinline__ void ray_prep(Ray& r, v3 o, v3 d) {
  r.o = o;
  r.d = d;
  float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  int kz = ax > ay ? (ax > az ? 0 : 2) : (ay > az ? 1 : 2);
  int kx = kz + 1;
  if (kx == 3) kx = 0;
  int ky = kx + 1;
  if (ky == 3) ky = 0;
  const float dkz = comp(d, kz);
  if (dkz < 0.0f) {
    int t = kx;
    kx = ky;
    ky = t;
  }
  r.kx = kx;
  r.ky = ky;
  r.kz = kz;
  r.Sx = comp(d, kx) / dkz;
  r.Sy = comp(d, ky) / dkz;
  r.Sz = 1.0f / dkz;
  float cx = fabsf(d.x) < 1e-20f ? copysignf(1e-20f, d.x) : d.x;
  float cy = fabsf(d.y) < 1e-20f ? copysignf(1e-20f, d.y) : d.y;
  float cz = fabsf(d.z) < 1e-20f ? copysignf(1e-20f, d.z) : d.z;
  r.inv = {1.0f / cx, 1.0f / cy, 1.0f / cz};
}

// Watertight ray/triangle (Woop, Benthin, Wald 2013): stands in for OptiX's
// built-in triangle intersection (every optixTrace / owl::traceRay).
__device__ __forceinline__ bool wt_hit(const float4 a, const float4 b, const float4 c, const Ray& r,
                                       float& tout) {
  const float A[3] = {a.x - r.o.x, a.y - r.o.y, a.z - r.o.z};
  const float B[3] = {b.x - r.o.x, b.y - r.o.y, b.z - r.o.z};
  const float C[3] = {c.x - r.o.x, c.y - r.o.y, c.z - r.o.z};
  const float Akz = r.kz == 0 ? A[0] : (r.kz == 1 ? A[1] : A[2]);
  const float Bkz = r.kz == 0 ? B[0] : (r.kz == 1 ? B[1] : B[2]);
  const float Ckz = r.kz == 0 ? C[0] : (r.kz == 1 ? C[1] : C[2]);
  const float Akx = r.kx == 0 ? A[0] : (r.kx == 1 ? A[1] : A[2]);
  const float Bkx = r.kx == 0 ? B[0] : (r.kx == 1 ? B[1] : B[2]);
  const float Ckx = r.kx == 0 ? C[0] : (r.kx == 1 ? C[1] : C[2]);
  const float Aky = r.ky == 0 ? A[0] : (r.ky == 1 ? A[1] : A[2]);
  const float Bky = r.ky == 0 ? B[0] : (r.ky == 1 ? B[1] : B[2]);
  const float Cky = r.ky == 0 ? C[0] : (r.ky == 1 ? C[1] : C[2]);
  const float Ax = Akx - r.Sx * Akz, Ay = Aky - r.Sy * Akz;
  const float Bx = Bkx - r.Sx * Bkz, By = Bky - r.Sy * Bkz;
  const float Cx = Ckx - r.Sx * Ckz, Cy = Cky - r.Sy * Ckz;
  float U = Cx * By - Cy * Bx;
  float V = Ax * Cy - Ay * Cx;
  float W = Bx * Ay - By * Ax;
  if (U == 0.0f || V == 0.0f || W == 0.0f) {
    double CxBy = (double)Cx * (double)By, CyBx = (double)Cy * (double)Bx;
    U = (float)(CxBy - CyBx);
    double AxCy = (double)Ax * (double)Cy, AyCx = (double)Ay * (double)Cx;
    V = (float)(AxCy - AyCx);
    double BxAy = (double)Bx * (double)Ay, ByAx = (double)By * (double)Ax;
    W = (float)(BxAy - ByAx);
  }
  if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
  const float det = U + V + W;
  if (det == 0.0f) return false;
  const float Az = r.Sz * Akz, Bz = r.Sz * Bkz, Cz = r.Sz * Ckz;
  const float T = U * Az + V * Bz + W * Cz;
  tout = T / det;
  return true;
}

// slab test for one box given as (x0,x1,y0,y1,z0,z1)
__device__ __forceinline__ bool slab(float x0, float x1, float y0, float y1, float z0, float z1, const Ray& r,
                                     float tmin, float tmax, float& tn) {
  const float t0x = (x0 - r.o.x) * r.inv.x, t1x = (x1 - r.o.x) * r.inv.x;
  const float t0y = (y0 - r.o.y) * r.inv.y, t1y = (y1 - r.o.y) * r.inv.y;
  const float t0z = (z0 - r.o.z) * r.inv.z, t1z = (z1 - r.o.z) * r.inv.z;
  tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
  const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
  return tn <= tf;
}

// Slab test on (x0, x1, ...) with the origin term folded into one fma per plane:
// t = fma(x, inv, -o * inv) (noi = -o * inv, once per node). Culling only: the
// boxes are padded by 1e-5 x the scene extent and the limit by 1.00001 (see
// build_lbvh), far above the one-rounding difference to (x - o) * inv, so the
// triangles tested -- and the argmin result -- are unchanged. PM_SLAB_FMA = 0
// keeps the two-op form (A/B build knob).
#ifndef PM_SLAB_FMA
#define PM_SLAB_FMA 1
#endif
__device__ __forceinline__ bool slab_fma(float x0, float x1, float y0, float y1, float z0, float z1, const Ray& r,
                                         v3 noi, float tmin, float tmax, float& tn) {
  const float t0x = __builtin_fmaf(x0, r.inv.x, noi.x), t1x = __builtin_fmaf(x1, r.inv.x, noi.x);
  const float t0y = __builtin_fmaf(y0, r.inv.y, noi.y), t1y = __builtin_fmaf(y1, r.inv.y, noi.y);
  const float t0z = __builtin_fmaf(z0, r.inv.z, noi.z), t1z = __builtin_fmaf(z1, r.inv.z, noi.z);
  tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
  const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
  return tn <= tf;
}

// Traversal stack: the top kStackDepth entries live in LDS ([depth][blockDim],
// sized for occupancy: 16 x 4 B x 64 lanes = 4 KB per wave); deeper entries
// spill to a per-lane private (scratch) array that only deep paths touch.
// A BVH4 of depth D needs at most 3 (D - 1) entries, so scenes with D <= 22
// can never overflow; deeper ones report PM_ERR_OVERFLOW if a ray does.
#ifndef PM_STACK_DEPTH
#define PM_STACK_DEPTH 16
#endif
constexpr int kStackDepth = PM_STACK_DEPTH;

// Occupancy targets of the traversal kernels (waves per SIMD; 0 = compiler's
// choice). Build-time knobs for A/B runs.
#ifndef PM_TRACE_WAVES
#define PM_TRACE_WAVES 6   // 6: trace 75.2 -> 69.6 ms despite 80 B/lane of spills (8: no better)
#endif
#ifndef PM_PATHS_WAVES
#define PM_PATHS_WAVES 0   // fused render kernel: 5 helped (45.5 -> 42.7 ms); after the ray split the default is as good
#endif
#define PM_WAVES_ATTR(w) __attribute__((amdgpu_waves_per_eu((w) > 0 ? (w) : 1, (w) > 0 ? (w) : 10)))
// PM_NO_SPILL: LDS stack only (no private scratch in any traversal kernel);
// rays deeper than kStackDepth report PM_ERR_OVERFLOW. A/B and diagnostics.
// BVH4 (4 children per node). A BVH4 of depth D needs at most 3(D - 1) stack
// entries: 64 in total for D <= 22. (Round 3 measured, and removed in round 4,
// an 8-wide quantised BVH: bitwise on the GPU suite but slower on config 3,
// trace 33.3 -> 44.3 ms, paths 18.5 -> 26.5 ms at 6 waves/SIMD.)
// PM_BVH_Q4 (build knob, width 4): the float BVH4 is converted to 64-B nodes
// with 8-bit child boxes (bvh.hip, k_quantize4): half the bytes and 4 instead
// of 7 16-B loads per visited node, for a per-plane fma decode.
#ifndef PM_BVH_Q4
#define PM_BVH_Q4 1
#endif
constexpr bool kBvhQ4 = PM_BVH_Q4;
constexpr int kNodeF4 = kBvhQ4 ? 4 : 8;   // float4 per node
constexpr int kStackTotal = 64;
#ifdef PM_NO_SPILL
constexpr int kSpillDepth = 0;
#else
constexpr int kSpillDepth = kStackTotal - PM_STACK_DEPTH > 0 ? kStackTotal - PM_STACK_DEPTH : 1;
#endif
constexpr int32_t kBvhEmpty = INT32_MIN;

struct HitInfo {
  float t;
  int32_t slot;   // triangle slot (leaf order) or -1
  int32_t gid;    // global triangle index (tie-break key)
};

// Closest hit in (tmin, tmax): argmin (t, global triangle index). `stack`
// points at this lane's column of an LDS stack laid out [depth][blockDim].
// BVH4 node (8 x float4): lo.x[4] hi.x[4] lo.y[4] hi.y[4] lo.z[4] hi.z[4]
// codes[4] (>= 0 internal node, kBvhEmpty unused, else ~triangle slot), pad.
__device__ __forceinline__ void cas(float& ta, int& ca, float& tb, int& cb) {
  const bool sw = tb < ta;
  const float t = sw ? tb : ta;
  tb = sw ? ta : tb;
  ta = t;
  const int c = sw ? cb : ca;
  cb = sw ? ca : cb;
  ca = c;
}

template <bool ANY>
__device__ __forceinline__ bool leaf_hit(const float4 a, const float4 b, const float4 c, const Ray& r, float tmin,
                                         float tmax, int slot, HitInfo& h) {
  float t;
  if (wt_hit(a, b, c, r, t) && t > tmin && t < tmax) {
    const int gid = __float_as_int(c.w);
    if (ANY || h.slot < 0 || t < h.t || (t == h.t && gid < h.gid)) {
      h.t = t;
      h.slot = slot;
      h.gid = gid;
      return true;
    }
  }
  return false;
}

// one triangle per leaf: code ~slot (round 3's two-triangle leaves measured
// slower, trace 29.6 -> 30.3 ms, and were removed in round 4)
template <bool ANY>
__device__ __forceinline__ bool leaf_test(const DevScene& S, const Ray& r, float tmin, float tmax, int code,
                                          HitInfo& h) {
  const int slot = ~code;
  return leaf_hit<ANY>(S.tri[3 * slot + 0], S.tri[3 * slot + 1], S.tri[3 * slot + 2], r, tmin, tmax, slot, h);
}

// PM_LEAF_COMPACT (build knob): test the hit leaves in compacted rounds.
// (Issuing the triangle loads of 2 / 4 hit leaves before testing them cost
// VGPRs and measured slower, paths 22.8 -> 25.0 / 24.6 ms; removed in round 4.)
#ifndef PM_LEAF_COMPACT
#define PM_LEAF_COMPACT 1
#endif

// One traversal step: visit `node` (slab-test its 4 children, test its leaf
// children, push the internal hits near-to-far and continue with the nearest,
// or pop). Returns true when the ray is finished (stack empty, or an any-hit).
template <bool ANY>
__device__ __forceinline__ bool traverse_step4(const DevScene& S, const Ray& r, float tmin, float tmax, int* stack,
                                               int stride, int* spill, int& node, int& sp, HitInfo& h,
                                               int* overflow) {
  const float lim = (ANY || h.slot < 0) ? tmax * 1.00001f : h.t * 1.00001f;
  float t0, t1, t2, t3;
  bool b0, b1, b2, b3;
  int4 ch;
  if (kBvhQ4) {
    // 64-B node: f4[0] corner p + exponent bytes, f4[1] codes, f4[2] qlo.x qlo.y
    // qlo.z qhi.x (4 bytes each), f4[3].xy qhi.y qhi.z; plane = p + q * 2^e,
    // in ray-t space fma(q, 2^e * inv, (p - o) * inv) (conservative: the
    // decoded box contains the padded float box, as for width 8)
    const float4* qn = S.nodes + 4 * (int64_t)node;
    const float4 h0 = qn[0];
    ch = *reinterpret_cast<const int4*>(&qn[1]);
    const uint4 qa = *reinterpret_cast<const uint4*>(&qn[2]);
    const uint2 qb = *reinterpret_cast<const uint2*>(&qn[3]);
    const uint32_t eb = __float_as_uint(h0.w);
    const float ax = __uint_as_float((eb & 0xFFu) << 23) * r.inv.x;
    const float ay = __uint_as_float(((eb >> 8) & 0xFFu) << 23) * r.inv.y;
    const float az = __uint_as_float(((eb >> 16) & 0xFFu) << 23) * r.inv.z;
    const float bx = (h0.x - r.o.x) * r.inv.x, by = (h0.y - r.o.y) * r.inv.y, bz = (h0.z - r.o.z) * r.inv.z;
    float tq[4];
    bool bq[4];
    const int cd[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int sh = 8 * c;
      const float t0x = __builtin_fmaf((float)((qa.x >> sh) & 0xFFu), ax, bx);
      const float t1x = __builtin_fmaf((float)((qa.w >> sh) & 0xFFu), ax, bx);
      const float t0y = __builtin_fmaf((float)((qa.y >> sh) & 0xFFu), ay, by);
      const float t1y = __builtin_fmaf((float)((qb.x >> sh) & 0xFFu), ay, by);
      const float t0z = __builtin_fmaf((float)((qa.z >> sh) & 0xFFu), az, bz);
      const float t1z = __builtin_fmaf((float)((qb.y >> sh) & 0xFFu), az, bz);
      tq[c] = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
      const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), lim));
      bq[c] = tq[c] <= tf && cd[c] != kBvhEmpty;
    }
    t0 = tq[0], t1 = tq[1], t2 = tq[2], t3 = tq[3];
    b0 = bq[0], b1 = bq[1], b2 = bq[2], b3 = bq[3];
  } else {
  const float4* q = S.nodes + 8 * (int64_t)node;
  const float4 lx = q[0], hx = q[1], ly = q[2], hy = q[3], lz = q[4], hz = q[5];
  ch = *reinterpret_cast<const int4*>(&q[6]);
  if (PM_SLAB_FMA) {
    const v3 noi = {-r.o.x * r.inv.x, -r.o.y * r.inv.y, -r.o.z * r.inv.z};
    b0 = slab_fma(lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, r, noi, tmin, lim, t0) && ch.x != kBvhEmpty;
    b1 = slab_fma(lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, r, noi, tmin, lim, t1) && ch.y != kBvhEmpty;
    b2 = slab_fma(lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, r, noi, tmin, lim, t2) && ch.z != kBvhEmpty;
    b3 = slab_fma(lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, r, noi, tmin, lim, t3) && ch.w != kBvhEmpty;
  } else {
    b0 = slab(lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, r, tmin, lim, t0) && ch.x != kBvhEmpty;
    b1 = slab(lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, r, tmin, lim, t1) && ch.y != kBvhEmpty;
    b2 = slab(lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, r, tmin, lim, t2) && ch.z != kBvhEmpty;
    b3 = slab(lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, r, tmin, lim, t3) && ch.w != kBvhEmpty;
  }
  }
  // leaves first: a hit shrinks the limit applied to the internal children
  if (PM_LEAF_COMPACT) {
    // hit leaves compacted to the front: round k tests every lane's k-th hit
    // leaf, and the wave runs max(#hit leaves) rounds (order-free: argmin)
    const bool f0 = b0 && ch.x < 0, f1 = b1 && ch.y < 0, f2 = b2 && ch.z < 0, f3 = b3 && ch.w < 0;
    int l0 = f0 ? ch.x : (f1 ? ch.y : (f2 ? ch.z : ch.w));
    int l1 = (f0 && f1) ? ch.y : ((f0 || f1) && f2 ? ch.z : ch.w);
    int l2 = (f0 + f1 + f2 == 3) ? ch.z : ch.w;
    const int nl = f0 + f1 + f2 + f3;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (__ballot(k < nl) == 0) break;
      const int c = k == 0 ? l0 : (k == 1 ? l1 : (k == 2 ? l2 : ch.w));
      if (k < nl && leaf_test<ANY>(S, r, tmin, tmax, c, h) && ANY) return true;
    }
  } else {
    if (b0 && ch.x < 0 && leaf_test<ANY>(S, r, tmin, tmax, ch.x, h) && ANY) return true;
    if (b1 && ch.y < 0 && leaf_test<ANY>(S, r, tmin, tmax, ch.y, h) && ANY) return true;
    if (b2 && ch.z < 0 && leaf_test<ANY>(S, r, tmin, tmax, ch.z, h) && ANY) return true;
    if (b3 && ch.w < 0 && leaf_test<ANY>(S, r, tmin, tmax, ch.w, h) && ANY) return true;
  }
  const float lim2 = (ANY || h.slot < 0) ? lim : h.t * 1.00001f;
  // internal children hit within the (possibly tightened) limit, sorted
  // near-to-far: order only changes speed, the result is argmin (t, id)
  float k0 = (b0 && ch.x >= 0 && t0 <= lim2) ? t0 : INFINITY;
  float k1 = (b1 && ch.y >= 0 && t1 <= lim2) ? t1 : INFINITY;
  float k2 = (b2 && ch.z >= 0 && t2 <= lim2) ? t2 : INFINITY;
  float k3 = (b3 && ch.w >= 0 && t3 <= lim2) ? t3 : INFINITY;
  const int cnt = (k0 != INFINITY) + (k1 != INFINITY) + (k2 != INFINITY) + (k3 != INFINITY);
  int c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
  cas(k0, c0, k1, c1);
  cas(k2, c2, k3, c3);
  cas(k0, c0, k2, c2);
  cas(k1, c1, k3, c3);
  cas(k1, c1, k2, c2);
  if (cnt > 0) {
    if (sp + cnt - 1 > kStackDepth + kSpillDepth) {
      *overflow = 1;
    } else if (sp + cnt - 1 <= kStackDepth) {
      if (cnt > 3) stack[(sp++) * stride] = c3;
      if (cnt > 2) stack[(sp++) * stride] = c2;
      if (cnt > 1) stack[(sp++) * stride] = c1;
    } else if (kSpillDepth > 0) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int c = k == 0 ? c3 : (k == 1 ? c2 : c1);
        if (k >= 4 - cnt) {
          if (sp < kStackDepth) stack[sp * stride] = c;
          else spill[sp - kStackDepth] = c;
          sp++;
        }
      }
    }
    node = c0;
    return false;
  }
  if (sp == 0) return true;
  sp--;
  node = (kSpillDepth == 0 || sp < kStackDepth) ? stack[sp * stride] : spill[sp - kStackDepth];
  return false;
}

template <bool ANY>
__device__ __forceinline__ bool traverse_step(const DevScene& S, const Ray& r, float tmin, float tmax, int* stack,
                                              int stride, int* spill, int& node, int& sp, HitInfo& h,
                                              int* overflow) {
  return traverse_step4<ANY>(S, r, tmin, tmax, stack, stride, spill, node, sp, h, overflow);
}

template <bool ANY>
__device__ __forceinline__ HitInfo traverse(const DevScene& S, const Ray& r, float tmin, float tmax, int* stack,
                                            int stride, int* overflow) {
  HitInfo h{tmax, -1, -1};
  if (S.ntri <= 0) return h;
  int spill[kSpillDepth > 0 ? kSpillDepth : 1];
  int sp = 0;
  int node = 0;
  while (!traverse_step<ANY>(S, r, tmin, tmax, stack, stride, spill, node, sp, h, overflow)) {
  }
  return h;
}

// Chunked ray pool: workgroup b traces rays [b*chunk, (b+1)*chunk) of n. A lane
// whose ray is finished takes the chunk's next ray, so a wave keeps its lanes
// busy instead of idling until its slowest ray is done (one ray per lane left
// ~80 % of the VALU lanes idle in the traversal kernels). Idle lanes are
// refilled together (one LDS atomic per wave) once kPoolRefill of them wait.
// fetch(i, Ray&, tmin&, tmax&) -> false skips ray i; done(i, Ray, HitInfo)
// consumes a result. `lnext` is an LDS counter zeroed before the call (block
// barrier); every wave exits once the chunk is drained and its lanes are done.
// pool_chunk picks the chunk: up to PM_POOL_RAYS rays per lane, fewer when the
// launch would otherwise have fewer than ~16 workgroups per CU.
#ifndef PM_POOL_RAYS
#define PM_POOL_RAYS 4   // config 3 frame: 16 139.4, 8 138.4, 4 136.7, 2 136.9 ms (shorter launch tails)
#endif
__host__ __device__ inline int pool_chunk(int64_t n, int block) {
  const int64_t target = 256 * 16;   // workgroups: 256 CUs x 16
  int64_t per = (n + target * block - 1) / (target * block);
  per = per < 1 ? 1 : (per > PM_POOL_RAYS ? PM_POOL_RAYS : per);
  return (int)(per * block);
}
// Workgroups that cover ANY live count n <= np when each launch picks
// pool_chunk(n) on the device (counts that stay on the device): n / chunk(n)
// is at most 4096 while chunk(n) < PM_POOL_RAYS * block, and largest at n = np
// beyond that; never more than one workgroup per `block` rays.
inline int64_t pool_grid(int64_t np, int block) {
  const int64_t at_np = (np + pool_chunk(np, block) - 1) / pool_chunk(np, block);
  const int64_t per_ray = (np + block - 1) / block;
  const int64_t g = at_np > 4097 ? at_np : 4097;
  return g < per_ray ? g : per_ray;
}
#ifndef PM_POOL_REFILL
#define PM_POOL_REFILL 16
#endif
template <bool ANY, typename Fetch, typename Done>
__device__ __forceinline__ void traverse_pool(const DevScene& S, int* stack, int stride, int* overflow, int64_t n,
                                              int chunk, int* lnext, Fetch fetch, Done done) {
  const int64_t cbase = (int64_t)blockIdx.x * chunk;
  const int cn = (int)(n - cbase < chunk ? n - cbase : chunk);
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int spill[kSpillDepth > 0 ? kSpillDepth : 1];
  Ray r;
  float tmin = 0.f, tmax = 0.f;
  HitInfo h{0.f, -1, -1};
  int node = 0, sp = 0, cur = -1;
  bool drained = false;
  for (;;) {
    const uint64_t idle = __ballot(cur < 0);
    const int nidle = __popcll(idle);
    if (!drained && nidle >= PM_POOL_REFILL) {
      int base = 0;
      if (lane == 0) base = atomicAdd(lnext, nidle);
      base = __shfl(base, 0);
      if (base + nidle >= cn) drained = true;
      if (cur < 0) {
        const int idx = base + __popcll(idle & lt_mask);
        if (idx < cn && fetch(cbase + idx, r, tmin, tmax)) {
          cur = idx;
          h = HitInfo{tmax, -1, -1};
          node = 0;
          sp = 0;
          if (S.ntri <= 0) {   // empty scene: miss at once
            done(cbase + cur, r, h);
            cur = -1;
          }
        }
      }
    }
    if (__ballot(cur >= 0) == 0) {
      if (drained) break;
      continue;
    }
    if (cur >= 0 && traverse_step<ANY>(S, r, tmin, tmax, stack, stride, spill, node, sp, h, overflow)) {
      done(cbase + cur, r, h);
      cur = -1;
    }
  }
}

// 30-bit Morton code of a point inside the box (lo, 1 / extent): only used to
// order work for locality, never for a result.
__device__ __forceinline__ uint32_t spread3(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}
__device__ __forceinline__ uint32_t morton30(float x, float y, float z, float3 lo, float3 inv) {
  const float fx = fminf(fmaxf((x - lo.x) * inv.x * 1024.0f, 0.0f), 1023.0f);
  const float fy = fminf(fmaxf((y - lo.y) * inv.y * 1024.0f, 0.0f), 1023.0f);
  const float fz = fminf(fmaxf((z - lo.z) * inv.z * 1024.0f, 0.0f), 1023.0f);
  return (spread3((uint32_t)fx) << 2) | (spread3((uint32_t)fy) << 1) | spread3((uint32_t)fz);
}

// The %.6f text round trip of the two-process pipeline (writeAlivePhotons,
// photon-mapping/src/hostCode.cu:31-49 -> readPhotonsFromFile, ray-tracer/src/
// hostCode.cu:26-52) without the text: printf rounds the exact value to 6
// decimals (ties to even) = rint(x * 1e6), exact in double (24 + 20 bits);
// strtof returns the float nearest to m / 1e6: the double quotient rounded to
// float, except when it sits exactly between two floats, where the sign of the
// exact remainder fma(-q, 1e6, m) picks the side. Valid for |x| < 9e9.
__host__ __device__ inline float quantize6_pos(float a) {
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
__host__ __device__ inline float quantize6(float x) { return signbit(x) ? -quantize6_pos(-x) : quantize6_pos(x); }

// owl make_rgba: clamp(int(f * 256), 0, 255) per channel, alpha 0xff
// (v_cvt_i32_f32 saturates; NaN -> 0).
__device__ __forceinline__ uint32_t rgba_channel(float f) {
  const float g = f * 256.f;
  const int i = (g == g) ? (int)fminf(fmaxf(g, -2147483648.f), 2147483520.f) : 0;
  return (uint32_t)min(255, max(0, i));
}
__device__ __forceinline__ uint32_t make_rgba(v3 c) {
  return rgba_channel(c.x) | (rgba_channel(c.y) << 8) | (rgba_channel(c.z) << 16) | (0xFFu << 24);
}

// Photon emission. Point light: pointLightRayGen (photon-mapping/cuda/
// deviceCode.cu:54-72), origin = light position, direction =
// randomPointInUnitSphere. SQUARE_LIGHT (declared by the reference, world.h:
// 8-24, never emitted there; this build's definition): two draws place the
// origin uniformly on the side x side square centred at pos, spanned by
// t1 = normalize(cross(a, n)), t2 = cross(n, t1) with a = (0,1,0) if |n.x| >
// 0.9 else (1,0,0); the direction is the cosine lobe about n used by diffuse
// scattering. The oracle restates the same operations in the same order.
__device__ __forceinline__ void emit_photon(float type, v3 pos, v3 normal, float side, uint32_t& rng, v3& o,
                                            v3& d) {
  if (type == 1.0f) {
    const v3 n = normalize(normal);
    const v3 a = fabsf(n.x) > 0.9f ? v3{0.f, 1.f, 0.f} : v3{1.f, 0.f, 0.f};
    const v3 t1 = normalize(cross(a, n));
    const v3 t2 = cross(n, t1);
    const float u = lcg_next(rng);
    const float w = lcg_next(rng);
    o = add(add(pos, smul((u - 0.5f) * side, t1)), smul((w - 0.5f) * side, t2));
    d = cosine_sample_hemisphere(n, rng);
  } else {
    o = pos;
    d = random_point_in_unit_sphere(rng);
  }
}

__device__ __forceinline__ v3 tri_normal(const DevScene& S, int slot) {
  const float4 a = S.tri[3 * slot + 0];
  const float4 b = S.tri[3 * slot + 1];
  const float4 c = S.tri[3 * slot + 2];
  const v3 A = {a.x, a.y, a.z}, B = {b.x, b.y, b.z}, C = {c.x, c.y, c.z};
  return normalize(cross(sub(B, A), sub(C, A)));
}

}  // namespace pmd
