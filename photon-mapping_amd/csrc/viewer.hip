// viewer.hip — photon viewer splat (debug tool).
//
// Replaces photonViewer: loadPhotons' per-photon projection (photon-viewer/
// src/hostCode.cu:53-75) and photonViewerRayGen (photon-viewer/cuda/
// deviceCode.cu:10-38). The view-projection matrix is built on the host with
// glm 0.9.9's operation order (glm is an empty submodule in the reference, so
// this is a restatement; the oracle repeats it); the kernel projects every
// photon, casts the visibility ray from the eye (OWL Ray default tmin 0,
// tmax = norm3d(pos - eye) - 1e-4 in double) and paints make_rgba(color).
// The reference's framebuffer writes race when several photons share a pixel;
// here the highest photon index wins (atomicMax), so the image is
// deterministic.
#include <cmath>

#include "pm_internal.hpp"

namespace pmd {

constexpr int kTraceBlockViewer = 128;

namespace {

struct V3h {
  float x, y, z;
};
V3h vsub(V3h a, V3h b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
float vdot(V3h a, V3h b) {   // glm compute_dot: (x*x' + y*y') + z*z'
  const float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
  return tx + ty + tz;
}
V3h vnorm(V3h v) {           // glm normalize: v * inversesqrt(dot(v, v))
  const float inv = 1.0f / std::sqrt(vdot(v, v));
  return {v.x * inv, v.y * inv, v.z * inv};
}
V3h vcross(V3h x, V3h y) {   // glm cross
  return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}

}  // namespace

// M[col][row] = perspective(fovy, W/H, 0.1, 1000) * lookAt(eye, center, up)
void viewer_matrix(const pm_viewer_params& P, float M[4][4]) {
  const V3h eye{P.look_from.x, P.look_from.y, P.look_from.z};
  const V3h ctr{P.look_at.x, P.look_at.y, P.look_at.z};
  const V3h up{P.look_up.x, P.look_up.y, P.look_up.z};
  // lookAtRH
  const V3h f = vnorm(vsub(ctr, eye));
  const V3h s = vnorm(vcross(f, up));
  const V3h u = vcross(s, f);
  float Vm[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  Vm[0][0] = s.x; Vm[1][0] = s.y; Vm[2][0] = s.z;
  Vm[0][1] = u.x; Vm[1][1] = u.y; Vm[2][1] = u.z;
  Vm[0][2] = -f.x; Vm[1][2] = -f.y; Vm[2][2] = -f.z;
  Vm[3][0] = -vdot(s, eye); Vm[3][1] = -vdot(u, eye); Vm[3][2] = vdot(f, eye);
  // perspectiveRH_NO
  const float aspect = (float)P.width / (float)P.height;
  const float zn = 0.1f, zf = 1000.f;
  const float th = std::tan(P.fovy / 2.0f);
  float Pm[4][4] = {};
  Pm[0][0] = 1.0f / (aspect * th);
  Pm[1][1] = 1.0f / th;
  Pm[2][2] = -(zf + zn) / (zf - zn);
  Pm[2][3] = -1.0f;
  Pm[3][2] = -(2.0f * zf * zn) / (zf - zn);
  // mat4 * mat4: Result[i] = A0 * B[i][0] + A1 * B[i][1] + A2 * B[i][2] + A3 * B[i][3]
  for (int i = 0; i < 4; i++)
    for (int r = 0; r < 4; r++) {
      float acc = Pm[0][r] * Vm[i][0];
      acc = acc + Pm[1][r] * Vm[i][1];
      acc = acc + Pm[2][r] * Vm[i][2];
      acc = acc + Pm[3][r] * Vm[i][3];
      M[i][r] = acc;
    }
}

struct ViewArgs {
  float m[4][4];
  v3 eye;
  int32_t W, H;
};

__global__ __launch_bounds__(kTraceBlockViewer) void k_view(DevScene S, const pm_photon* __restrict__ ph, int64_t n,
                                                            ViewArgs V, int32_t* __restrict__ win,
                                                            int32_t* __restrict__ pix, int* overflow) {
  __shared__ int stack[kStackDepth * kTraceBlockViewer];
  const int64_t i = (int64_t)blockIdx.x * kTraceBlockViewer + threadIdx.x;
  if (i >= n) return;
  pix[i] = -1;
  const pm_float3 p = ph[i].pos;
  // mat4 * vec4 (glm): (m0 x + m1 y) + (m2 z + m3 w), w = 1
  float c[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const float a0 = V.m[0][r] * p.x + V.m[1][r] * p.y;
    const float a1 = V.m[2][r] * p.z + V.m[3][r];
    c[r] = a0 + a1;
  }
  if (c[2] < 0.f) return;
  const float fx = (c[0] / c[3] + 1.f) * 0.5f * (float)V.W;
  const float fy = (c[1] / c[3] + 1.f) * 0.5f * (float)V.H;
  // static_cast<int> of a NaN / out-of-range float is INT_MIN on the x86 host
  if (!(fx > -2147483648.f && fx < 2147483648.f) || !(fy > -2147483648.f && fy < 2147483648.f)) return;
  const int px = (int)fx, py = V.H - (int)fy;
  if (px < 0 || px >= V.W || py < 0 || py >= V.H) return;
  const v3 d = {p.x - V.eye.x, p.y - V.eye.y, p.z - V.eye.z};
  const float tmax = (float)(sqrt((double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z) - (double)1e-4f);
  Ray r;
  ray_prep(r, V.eye, normalize(d));
  const HitInfo h = traverse<true>(S, r, 0.0f, tmax, stack + threadIdx.x, kTraceBlockViewer, overflow);
  if (h.slot >= 0) return;
  const int32_t q = px + V.W * py;
  pix[i] = q;
  atomicMax(&win[q], (int32_t)i);
}

__global__ void k_view_write(const pm_photon* __restrict__ ph, int64_t n, const int32_t* __restrict__ pix,
                             const int32_t* __restrict__ win, uint32_t* __restrict__ rgba) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t q = pix[i];
  if (q < 0 || win[q] != (int32_t)i) return;
  const pm_float3 c = ph[i].color;
  rgba[q] = make_rgba(v3{c.x, c.y, c.z});
}

__global__ void k_view_clear(uint32_t* rgba, int32_t* win, int64_t np) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  rgba[i] = 0xFF000000u;   // RGBA_BLACK (photon-viewer/src/hostCode.cu:20,128-133)
  win[i] = -1;
}

hipError_t photon_view(pm_scene* sc, const pm_photon* ph, int64_t n, const pm_viewer_params& P, uint32_t* rgba,
                       hipStream_t s) {
  const int64_t np = (int64_t)P.width * P.height;
  if (np <= 0) return hipSuccess;
  DevBuf<int32_t> win(np), pix(n > 0 ? n : 1);
  if (!win.p || !pix.p) return hipErrorOutOfMemory;
  k_view_clear<<<grid_for(np, 256), 256, 0, s>>>(rgba, win.p, np);
  PM_HIP_TRY(hipGetLastError());
  if (n > 0) {
    ViewArgs V;
    viewer_matrix(P, V.m);
    V.eye = {P.look_from.x, P.look_from.y, P.look_from.z};
    V.W = P.width;
    V.H = P.height;
    k_view<<<grid_for(n, kTraceBlockViewer), kTraceBlockViewer, 0, s>>>(sc->view(), ph, n, V, win.p, pix.p,
                                                                         sc->overflow.p);
    PM_HIP_TRY(hipGetLastError());
    k_view_write<<<grid_for(n, 256), 256, 0, s>>>(ph, n, pix.p, win.p, rgba);
    PM_HIP_TRY(hipGetLastError());
  }
  return hipStreamSynchronize(s);
}

}  // namespace pmd
