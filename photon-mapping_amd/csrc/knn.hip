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
#include <cstdlib>

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

// Exact kNN for one query: stack-free walk of the left-balanced kd-tree
// (prev/curr, implicit parent (c+1)/2-1) down to the bucket level; a subtree
// rooted at the bucket level is scanned linearly from its contiguous copy
// (KdBuckets), which visits a superset of the nodes the walk would visit.
template <int K>
__device__ __forceinline__ void knn_query(const float4* __restrict__ nodes, int n, const KdBuckets& bk, v3 q,
                                          float r2, uint64_t (&list)[K]) {
  const uint64_t sentinel = ((uint64_t)__float_as_uint(r2) << 32) | 0xFFFFFFFFull;
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  if (n <= 0) return;
  float bound = r2;
  int prev = -1, curr = 0;
  for (;;) {
    const int parent = ((curr + 1) >> 1) - 1;
    if (curr >= bk.first) {
      // bucket: every node of the subtree, contiguous (sentinels are +inf)
      const float4* b = bk.data + (int64_t)(curr - bk.first) * bk.slots;
      for (int s = 0; s < bk.slots; s++) {
        const float4 nd = b[s];
        const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
        const float d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < r2) {
          const uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)(__float_as_int(nd.w) >> 2);
          if (key < list[K - 1]) {
            list_insert<K>(list, key);
            bound = __uint_as_float((uint32_t)(list[K - 1] >> 32));
          }
        }
      }
      if (parent < 0) break;
      prev = curr;
      curr = parent;
      continue;
    }
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
__global__ __launch_bounds__(256) void k_knn(const float4* nodes, int n, KdBuckets bk, const pm_float3* q,
                                             int64_t nq, int k, float r2, int32_t* ids, float* d2o, float* maxd2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  uint64_t list[K];
  const pm_float3 p = q[i];
  knn_query<K>(nodes, n, bk, mk(p), r2, list);
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

// Radiance estimate from a finished candidate list: gatherPhotons
// (shading.h:93-121), neighbours summed in (d^2, index) order.
__device__ __forceinline__ v3 radiance(const uint64_t (&list)[kKNearest], const float4* __restrict__ payload,
                                       float brdf) {
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
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ nodes, const float4* __restrict__ payload,
                                                int n, KdBuckets bk, const float4* __restrict__ qb, int64_t nq,
                                                float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float4 qq = qb[i];
  uint64_t list[kKNearest];
  knn_query<kKNearest>(nodes, n, bk, v3{qq.x, qq.y, qq.z}, kKMaxDistance * kKMaxDistance, list);
  const v3 f = radiance(list, payload, qq.w);
  out[i] = make_float4(f.x, f.y, f.z, 0.f);
}

// Deferred-insert variant of the stack-free walk: a lane that finds a
// candidate parks it in a one-entry slot; the 50-wide sorted insert (the
// dominant VALU cost: it runs for the whole wave whenever any lane inserts)
// executes wave-wide only when >= kInsBatch lanes have a parked candidate or a
// lane with a parked candidate finds another one. The pruning bound is then
// at most stale-high, which keeps the search exact.
constexpr int kInsBatch = 16;

template <int TAG>
__global__ __launch_bounds__(256) void k_gather_defer(const float4* __restrict__ nodes,
                                                      const float4* __restrict__ payload, int n,
                                                      const float4* __restrict__ qb, int64_t nq,
                                                      float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < nq;
  const float r2 = kKMaxDistance * kKMaxDistance;
  const uint64_t sentinel = ((uint64_t)__float_as_uint(r2) << 32) | 0xFFFFFFFFull;
  const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const v3 q = {qq.x, qq.y, qq.z};
  uint64_t list[kKNearest];
#pragma unroll
  for (int j = 0; j < kKNearest; j++) list[j] = sentinel;
  float bound = r2;
  int prev = -1, curr = 0;
  bool walking = valid && n > 0, pend = false;
  uint64_t pkey = 0;
  for (;;) {
    bool cand = false;
    uint64_t key = 0;
    int next = -1;
    if (walking) {
      const float4 nd = nodes[curr];
      const int child = 2 * curr + 1;
      const int w = __float_as_int(nd.w);
      if (prev < child) {
        const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
        const float d2 = dx * dx + dy * dy + dz * dz;
        key = ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)(w >> 2);
        cand = d2 < r2 && key < list[kKNearest - 1];
      }
      const int dim = w & 3;
      const float diff = (dim == 0 ? q.x : (dim == 1 ? q.y : q.z)) - (dim == 0 ? nd.x : (dim == 1 ? nd.y : nd.z));
      const int side = diff > 0.f ? 1 : 0;
      const int close_c = child + side, far_c = child + 1 - side;
      const int parent = ((curr + 1) >> 1) - 1;
      if (prev == far_c) {
        next = parent;
      } else if (prev == close_c || close_c >= n) {
        next = (far_c < n && diff * diff <= bound) ? far_c : parent;
      } else {
        next = close_c;
      }
    }
    const uint64_t pm = __ballot(pend);
    const bool any_walking = __ballot(walking) != 0;
    if (pm != 0 && (!any_walking || __ballot(pend && cand) != 0 || __popcll(pm) >= kInsBatch)) {
      if (pend && pkey < list[kKNearest - 1]) {
        list_insert<kKNearest>(list, pkey);
        bound = __uint_as_float((uint32_t)(list[kKNearest - 1] >> 32));
      }
      pend = false;
    }
    if (!any_walking) break;
    if (cand) {
      pkey = key;
      pend = true;
    }
    if (walking) {
      if (next < 0) {
        walking = false;
      } else {
        prev = curr;
        curr = next;
      }
    }
  }
  if (valid) {
    const v3 f = radiance(list, payload, qq.w);
    out[i] = make_float4(f.x, f.y, f.z, 0.f);
  }
}

// Stack-based exact kNN (cukd stackBased shape): descend close-first, push the
// far child with its plane distance^2 into this lane's LDS column, pop while
// the entry is outside the lane's bound. Every node is loaded once (no parent
// re-visits as in the stack-free walk). Stack layout [depth][lane] (uint2):
// consecutive lanes hit consecutive 8-B words, so pushes/pops are conflict-free.
constexpr int kKnnStack = 32;
constexpr int kKnnBlock = 64;

template <int K>
__device__ __forceinline__ void knn_query_stack(const float4* __restrict__ nodes, int n, v3 q, float r2,
                                                uint64_t (&list)[K], uint2* st, int* overflow) {
  const uint64_t sentinel = ((uint64_t)__float_as_uint(r2) << 32) | 0xFFFFFFFFull;
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  if (n <= 0) return;
  float bound = r2;
  int sp = 0;
  int node = 0;
  for (;;) {
    while (node < n) {
      const float4 nd = nodes[node];
      const int w = __float_as_int(nd.w);
      const int dim = w & 3;
      const float diff = (dim == 0 ? q.x : (dim == 1 ? q.y : q.z)) - (dim == 0 ? nd.x : (dim == 1 ? nd.y : nd.z));
      const int child = 2 * node + 1;
      const int side = diff > 0.f ? 1 : 0;
      const int far_c = child + 1 - side;
      const float pd2 = diff * diff;
      if (far_c < n && pd2 <= bound) {
        if (sp < kKnnStack) {
          st[sp * kKnnBlock] = make_uint2((uint32_t)far_c, __float_as_uint(pd2));
          sp++;
        } else if (overflow) {
          *overflow = 1;   // unreachable: depth <= 30 for n < 2^30 (kd_build limit)
        }
      }
      const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
      const float d2 = dx * dx + dy * dy + dz * dz;
      if (d2 < r2) {
        const uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)(w >> 2);
        if (key < list[K - 1]) {
          list_insert<K>(list, key);
          bound = __uint_as_float((uint32_t)(list[K - 1] >> 32));
        }
      }
      node = child + side;
    }
    node = INT32_MAX;
    while (sp > 0) {
      sp--;
      const uint2 e = st[sp * kKnnBlock];
      if (__uint_as_float(e.y) <= bound) {
        node = (int)e.x;
        break;
      }
    }
    if (node == INT32_MAX) break;
  }
}

template <int TAG>
__global__ __launch_bounds__(kKnnBlock) void k_gather_stack(const float4* __restrict__ nodes,
                                                            const float4* __restrict__ payload, int n,
                                                            const float4* __restrict__ qb, int64_t nq,
                                                            float4* __restrict__ out, int* overflow) {
  __shared__ uint2 stack[kKnnStack * kKnnBlock];
  const int64_t i = (int64_t)blockIdx.x * kKnnBlock + threadIdx.x;
  if (i >= nq) return;
  const float4 qq = qb[i];
  uint64_t list[kKNearest];
  knn_query_stack<kKNearest>(nodes, n, v3{qq.x, qq.y, qq.z}, kKMaxDistance * kKMaxDistance, list,
                             stack + threadIdx.x, overflow);
  const v3 f = radiance(list, payload, qq.w);
  out[i] = make_float4(f.x, f.y, f.z, 0.f);
}

// Batched variant: a wave owns 64*PER consecutive (sorted) queries; lane l
// takes l, l+64, ...; a lane whose walk ends parks its list and the wave runs
// the radiance sum only when >= kBatchMin lanes are parked (or nothing else
// is running), so the wave does not wait on its slowest query and the 50-load
// sum is amortised over many lanes.
constexpr int kGatherPer = 8;
constexpr int kBatchMin = 32;

template <int TAG>
__global__ __launch_bounds__(256) void k_gather_batched(const float4* __restrict__ nodes,
                                                        const float4* __restrict__ payload, int n,
                                                        const float4* __restrict__ qb, int64_t nq,
                                                        float4* __restrict__ out) {
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float r2 = kKMaxDistance * kKMaxDistance;
  const uint64_t sentinel = ((uint64_t)__float_as_uint(r2) << 32) | 0xFFFFFFFFull;
  int64_t qi = (gtid >> 6) * 64 * kGatherPer + (gtid & 63);
  int left = kGatherPer;
  uint64_t list[kKNearest];
  v3 q = {0.f, 0.f, 0.f};
  float brdf = 0.f, bound = r2;
  int prev = -1, curr = 0;
  bool busy = false, parked = false;
  for (;;) {
    if (!busy && !parked && left > 0 && qi < nq) {
      const float4 qq = qb[qi];
      q = {qq.x, qq.y, qq.z};
      brdf = qq.w;
#pragma unroll
      for (int j = 0; j < kKNearest; j++) list[j] = sentinel;
      bound = r2;
      prev = -1;
      curr = 0;
      busy = n > 0;
      parked = n <= 0;
    }
    const uint64_t busy_m = __ballot(busy), park_m = __ballot(parked);
    if (busy_m == 0 && park_m == 0) break;
    if (park_m != 0 && (__popcll(park_m) >= kBatchMin || busy_m == 0)) {
      if (parked) {
        const v3 f = radiance(list, payload, brdf);
        out[qi] = make_float4(f.x, f.y, f.z, 0.f);
        parked = false;
        qi += 64;
        left--;
      }
      continue;
    }
    if (busy) {
      const float4 nd = nodes[curr];
      const int child = 2 * curr + 1;
      const int w = __float_as_int(nd.w);
      if (prev < child) {
        const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
        const float d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < r2) {
          const uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)(w >> 2);
          if (key < list[kKNearest - 1]) {
            list_insert<kKNearest>(list, key);
            bound = __uint_as_float((uint32_t)(list[kKNearest - 1] >> 32));
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
      if (next < 0) {
        busy = false;
        parked = true;
      } else {
        prev = curr;
        curr = next;
      }
    }
  }
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
    k_knn<KK><<<g, 256, 0, s>>>(m->nodes.p, n, m->buckets(), q, nq, k, r2, ids, d2, maxd2);           \
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
  // tuning knob (read per launch): 0 stack-free walk, 1 batched stack-free, 2 LDS-stack walk
  const char* env = std::getenv("PM_GATHER_MODE");
  const int mode = env ? std::atoi(env) : 0;
  if (mode == 3) {
    const int g = grid_for(nq, 256);
    if (tag == 1)
      k_gather_defer<1><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out);
    else
      k_gather_defer<0><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out);
    return hipGetLastError();
  }
  if (mode == 2) {
    const int g = grid_for(nq, kKnnBlock);
    if (tag == 1)
      k_gather_stack<1><<<g, kKnnBlock, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out, nullptr);
    else
      k_gather_stack<0><<<g, kKnnBlock, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out, nullptr);
    return hipGetLastError();
  }
  if (mode == 1 && m->bucket_first == INT32_MAX) {
    const int g = grid_for((nq + kGatherPer - 1) / kGatherPer, 256);
    if (tag == 1)
      k_gather_batched<1><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out);
    else
      k_gather_batched<0><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, out);
    return hipGetLastError();
  }
  const int g = grid_for(nq, 256);
  if (tag == 1)
    k_gather<1><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, m->buckets(), qb, nq, out);
  else
    k_gather<0><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, m->buckets(), qb, nq, out);
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
