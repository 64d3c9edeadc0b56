// knn.hip — exact k-nearest-photon search and radiance estimate for gfx950.
//
// Replaces cukd::stackBased::knn<HeapCandidateList<K>> (called from
// KNearestPhotons, ray-tracer/cuda/shading.h:11-18) and gatherPhotons
// (shading.h:93-121). Traversal is the stack-free left-balanced kd-tree walk
// (prev/curr with implicit parent (c+1)/2-1), so a lane needs no stack memory;
// the candidate list is K packed u64 keys (d^2 bits << 32 | original index)
// kept sorted in VGPRs (all indices compile-time after unrolling), so the
// result is ordered by (d^2, index) and the radiance sum runs in that order.
// Cut-off: only d^2 < max_radius^2 enters (HeapCandidateList(cutOff) init);
// the returned radius is the K-th d^2, or max_radius^2 when fewer were found.
#include "pm_internal.hpp"

namespace pmd {

template <int K>
__device__ __forceinline__ void list_insert(uint64_t (&list)[K], uint64_t key) {
  bool lt_next = true;   // key < list[K-1] checked by the caller
#pragma unroll
  for (int j = K - 1; j > 0; j--) {
    const uint64_t a = list[j - 1];
    const bool gt = key < a;
    list[j] = gt ? a : (lt_next ? key : list[j]);
    lt_next = gt;
  }
  list[0] = lt_next ? key : list[0];
}

template <int K>
__device__ __forceinline__ void knn_query(const float4* __restrict__ nodes, int n, v3 q, float r2,
                                          uint64_t (&list)[K]) {
  const uint64_t sentinel = ((uint64_t)__float_as_uint(r2) << 32) | 0xFFFFFFFFull;
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  if (n <= 0) return;
  float bound = r2;
  int prev = -1, curr = 0;
  for (;;) {
    const float4 nd = nodes[curr];
    const int child = 2 * curr + 1;
    const int w = __float_as_int(nd.w);
    if (prev < child) {   // arriving from the parent: visit this node
      const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
      const float d2 = dx * dx + dy * dy + dz * dz;
      if (d2 < r2) {
        const uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)(w >> 2);
        if (key < list[K - 1]) {
          list_insert<K>(list, key);
          bound = __uint_as_float((uint32_t)(list[K - 1] >> 32));
        }
      }
    }
    const int dim = w & 3;
    const float diff = (dim == 0 ? q.x : (dim == 1 ? q.y : q.z)) - (dim == 0 ? nd.x : (dim == 1 ? nd.y : nd.z));
    const int side = diff > 0.f ? 1 : 0;
    const int close_c = child + side, far_c = child + 1 - side;
    const int parent = ((curr + 1) >> 1) - 1;
    int next;
    if (prev == far_c) {
      next = parent;
    } else if (prev == close_c || close_c >= n) {
      next = (far_c < n && diff * diff <= bound) ? far_c : parent;
    } else {
      next = close_c;
    }
    if (next < 0) break;
    prev = curr;
    curr = next;
  }
}

template <int K>
__global__ __launch_bounds__(256) void k_knn(const float4* nodes, int n, const pm_float3* q, int64_t nq, int k,
                                             float r2, int32_t* ids, float* d2o, float* maxd2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  uint64_t list[K];
  const pm_float3 p = q[i];
  knn_query<K>(nodes, n, mk(p), r2, list);
  uint64_t kth = list[0];
#pragma unroll
  for (int j = 0; j < K; j++) {
    if (j < k) {
      const uint32_t id = (uint32_t)list[j];
      ids[i * k + j] = id == 0xFFFFFFFFu ? -1 : (int32_t)id;
      if (d2o) d2o[i * k + j] = __uint_as_float((uint32_t)(list[j] >> 32));
    }
    if (j == k - 1) kth = list[j];
  }
  if (maxd2) maxd2[i] = __uint_as_float((uint32_t)(kth >> 32));
}

// gatherPhotons (shading.h:93-121) for one query
__device__ __forceinline__ v3 gather_one(const float4* __restrict__ nodes, const float4* __restrict__ payload,
                                         int n, v3 hit, float brdf) {
  uint64_t list[kKNearest];
  knn_query<kKNearest>(nodes, n, hit, kKMaxDistance * kKMaxDistance, list);
  const float r2 = __uint_as_float((uint32_t)(list[kKNearest - 1] >> 32));
  v3 flux = {0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < kKNearest; p++) {
    const uint32_t id = (uint32_t)list[p];
    if (id == 0xFFFFFFFFu) continue;
    const float4 pl = payload[id];
    const float dist = sqrtf(__uint_as_float((uint32_t)(list[p] >> 32)));
    const float w = 1 - (dist / sqrtf(r2) * kConeFilterC);
    flux = add(flux, smul(brdf * pl.w * w, v3{pl.x, pl.y, pl.z}));
  }
  return divf(flux, (1 - (2.f / 3.f) * (1.f / kConeFilterC)) * 2 * kPI * r2);
}

template <int TAG>
__global__ __launch_bounds__(256) void k_gather(const float4* nodes, const float4* payload, int n,
                                                const float4* qb, int64_t nq, float4* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float4 qq = qb[i];
  const v3 f = gather_one(nodes, payload, n, v3{qq.x, qq.y, qq.z}, qq.w);
  out[i] = make_float4(f.x, f.y, f.z, 0.f);
}

__global__ void k_pack_query(const pm_float3* pts, const float* brdf, int64_t nq, float4* qb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  qb[i] = make_float4(pts[i].x, pts[i].y, pts[i].z, brdf[i]);
}
__global__ void k_unpack_out(const float4* o, int64_t nq, pm_float3* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  out[i] = {o[i].x, o[i].y, o[i].z};
}

hipError_t launch_knn(const pm_photon_map* m, const pm_float3* q, int64_t nq, int k, float radius, int32_t* ids,
                      float* d2, float* maxd2, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  const float r2 = radius * radius;
  const int n = (int)m->n;
  const int g = grid_for(nq, 256);
#define PM_KNN_CASE(KK)                                                                 \
  if (k <= KK) {                                                                        \
    k_knn<KK><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, r2, ids, d2, maxd2);           \
    return hipGetLastError();                                                           \
  }
  PM_KNN_CASE(8)
  PM_KNN_CASE(16)
  PM_KNN_CASE(32)
  PM_KNN_CASE(50)
  PM_KNN_CASE(64)
  PM_KNN_CASE(128)
#undef PM_KNN_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_gather(const pm_photon_map* m, const float4* qb, int64_t nq, float4* out, hipStream_t s,
                         int tag) {
  if (nq <= 0) return hipSuccess;
  if (tag == 1)
    k_gather<1><<<grid_for(nq, 256), 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out);
  else
    k_gather<0><<<grid_for(nq, 256), 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out);
  return hipGetLastError();
}

hipError_t launch_gather_api(const pm_photon_map* m, const pm_float3* pts, const float* brdf, int64_t nq,
                             pm_float3* out, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  DevBuf<float4> qb(nq), ob(nq);
  if (!qb.p || !ob.p) return hipErrorOutOfMemory;
  k_pack_query<<<grid_for(nq, 256), 256, 0, s>>>(pts, brdf, nq, qb.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(launch_gather(m, qb.p, nq, ob.p, s));
  k_unpack_out<<<grid_for(nq, 256), 256, 0, s>>>(ob.p, nq, out);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

}  // namespace pmd
