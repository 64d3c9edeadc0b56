// knn.hip — exact k-nearest-photon search and radiance estimate for gfx950.
//
// Replaces cukd::stackBased::knn<HeapCandidateList<K>> (called from
// KNearestPhotons, ray-tracer/cuda/shading.h:11-18) and gatherPhotons
// (shading.h:93-121). Traversal is the stack-free left-balanced kd-tree walk
// (prev/curr with implicit parent (c+1)/2-1), so a lane needs no stack memory;
// the candidate list is K packed keys (d^2 bits << 32 | original index, held
// as doubles: see key_make) kept sorted in VGPRs (all indices compile-time
// after unrolling), so the result is ordered by (d^2, index) and the radiance
// sum runs in that order.
// Cut-off: only d^2 < max_radius^2 enters (HeapCandidateList(cutOff) init);
// the returned radius is the K-th d^2, or max_radius^2 when fewer were found.
//
// The sorted 50-wide insert is the dominant cost and runs for the whole wave
// whenever any lane inserts: it is built from v_min_f64 / v_max_f64 only
// (list_insert), and the walk tests a node's point post-order so root-path
// points meet a tight bound (knn_walk<POST = true>; variants: DESIGN.md §4.4).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pm_internal.hpp"

namespace pmd {

// Candidate keys: (d^2 bits << 32 | original id) + 2^52, held as the bits of a
// double. d^2 >= 0 so the packed integer orders candidates by (d^2, id); the
// 2^52 bias makes every key a positive NORMAL double (exponent field >= 1,
// never all-ones), whose IEEE order equals that integer order. The sorted
// insert can then use the mask-free identity
//   new[j] = max(list[j-1], min(list[j], key))
// on v_min_f64 / v_max_f64: 99 DP ops per 50-entry insert, no compares, no
// cndmasks, no VCC hazards (the u64 compare-select form issued ~400 slots).
constexpr uint64_t kKeyBias = 1ull << 52;

__device__ __forceinline__ double key_make(float d2, uint32_t id) {
  return __longlong_as_double((long long)((((uint64_t)__float_as_uint(d2) << 32) | id) + kKeyBias));
}
__device__ __forceinline__ float key_d2(double k) {
  return __uint_as_float((uint32_t)(((uint64_t)__double_as_longlong(k) - kKeyBias) >> 32));
}
__device__ __forceinline__ uint32_t key_id(double k) { return (uint32_t)__double_as_longlong(k); }

// Inline asm keeps the compiler from canonicalising each operand (an extra
// v_max_f64 x, x per op): keys are never NaN by construction.
__device__ __forceinline__ double dmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double dmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Sorted insert of a key known to be < list[K-1] (keys are unique). Each min
// is issued one entry ahead of the max that consumes it.
template <int K>
__device__ __forceinline__ void list_insert(double (&list)[K], double key) {
  double t = dmin(list[K - 1], key);
#pragma unroll
  for (int j = K - 1; j > 0; j--) {
    const double tn = dmin(list[j - 1], key);
    list[j] = dmax(list[j - 1], t);
    t = tn;
  }
  list[0] = t;
}

struct KnnCounters {
  uint32_t steps = 0, ins = 0, wave_ins = 0;
};

// Stack-free walk. Production: POST = true, QL = 8 (PM_GATHER_MODE 9); other
// instantiations are kept for A/B runs (PM_GATHER_MODE 0, 4, 5, 10).
//  POST: a node's own point is tested when the walk comes back from its close
//        child (or at once if it has none) instead of on arrival, so the
//        root-path points meet an already tight bound instead of filling the
//        list with far-away entries.
//  QP:   > 0 parks candidates in a QP-entry per-lane queue; the wave runs one
//        50-wide insert round (every lane with a queued key pops one) only
//        when some lane's queue is full or the walks are over. The pruning
//        bound ignores queued keys, i.e. it is never too tight: still exact.
//  QL:   > 0 the same with a QL-deep per-lane LIFO queue in LDS (`lq`, this
//        lane's column of a [QL][stride] array): deep batching without VGPRs.
//  lo:   only keys > lo are candidates (multi-pass k > 128: pass p collects
//        the 128 smallest keys above pass p-1's last; keys are unique).
template <int K, bool POST, int QP, bool ST, int QL = 0>
__device__ __forceinline__ void knn_walk(const float4* __restrict__ nodes, int n, v3 q, float r2, bool valid,
                                         double (&list)[K], KnnCounters* kc = nullptr, double* lq = nullptr,
                                         int lstride = 0, double lo = 0.0) {
  const double sentinel = key_make(r2, 0xFFFFFFFFu);
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  float bound = r2;
  int prev = -1, curr = 0;
  bool walking = valid && n > 0;
  double qk[QP > 0 ? QP : 1];
  int qn = 0;
  for (;;) {
    bool cand = false;
    double key = 0.0;
    if (walking) {
      const float4 nd = nodes[curr];
      const int child = 2 * curr + 1;
      const int w = __float_as_int(nd.w);
      const int dim = w & 3;
      const float diff = (dim == 0 ? q.x : (dim == 1 ? q.y : q.z)) - (dim == 0 ? nd.x : (dim == 1 ? nd.y : nd.z));
      const int side = diff > 0.f ? 1 : 0;
      const int close_c = child + side, far_c = child + 1 - side;
      const int parent = ((curr + 1) >> 1) - 1;
      const bool down = prev < child;   // arrived from the parent
      const bool test = POST ? ((down && close_c >= n) || prev == close_c) : down;
      if (test) {
        const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
        const float d2 = dx * dx + dy * dy + dz * dz;
        key = key_make(d2, (uint32_t)w >> 2);
        cand = d2 < r2 && key < list[K - 1] && key > lo;
      }
      int next;
      if (prev == far_c) {
        next = parent;
      } else if (prev == close_c || close_c >= n) {
        next = (far_c < n && diff * diff <= bound) ? far_c : parent;
      } else {
        next = close_c;
      }
      if (next < 0) {
        walking = false;
      } else {
        prev = curr;
        curr = next;
      }
      if (ST) kc->steps++;
    }
    if (QL > 0) {
      if (cand) {
        lq[qn * lstride] = key;
        qn++;
      }
      const bool any_walking = __ballot(walking) != 0;
      const bool round = __ballot(qn == QL) != 0 || !any_walking;
      double ik = __longlong_as_double(0x7FEFFFFFFFFFFFFFll);   // DBL_MAX: never inserted
      if (round && qn > 0) {
        qn--;
        ik = lq[qn * lstride];
      }
      const bool ins = ik < list[K - 1];
      if (ins) {
        list_insert<K>(list, ik);
        bound = key_d2(list[K - 1]);
      }
      if (ST) {
        kc->ins += ins;
        kc->wave_ins += round;
      }
      if (!any_walking && __ballot(qn > 0) == 0) break;
    } else if (QP == 0) {
      if (cand) {
        list_insert<K>(list, key);
        bound = key_d2(list[K - 1]);
      }
      if (ST) {
        kc->ins += cand;
        kc->wave_ins += __ballot(cand) != 0;
      }
      if (__ballot(walking) == 0) break;
    } else {
      if (cand) {
#pragma unroll
        for (int j = 0; j < QP; j++) qk[j] = j == qn ? key : qk[j];
        qn++;
      }
      // insert round (wave-uniform): every lane with a queued key pops one.
      // Same loop shape as QP == 0 (one divergent insert site, one exit at the
      // end) so the 100-VGPR list is not duplicated across the back-edge.
      const bool any_walking = __ballot(walking) != 0;
      const bool round = __ballot(qn == QP) != 0 || !any_walking;
      double ik = __longlong_as_double(0x7FEFFFFFFFFFFFFFll);   // DBL_MAX: never inserted
      if (round && qn > 0) {
        ik = qk[0];
#pragma unroll
        for (int j = 0; j + 1 < QP; j++) qk[j] = qk[j + 1];
        qn--;
      }
      const bool ins = ik < list[K - 1];
      if (ins) {
        list_insert<K>(list, ik);
        bound = key_d2(list[K - 1]);
      }
      if (ST) {
        kc->ins += ins;
        kc->wave_ins += round;
      }
      if (!any_walking && __ballot(qn > 0) == 0) break;
    }
  }
}

// The gather's walk (PM_GATHER_MODE 11): knn_walk<K, POST = true, QL> with
// fewer instructions per step, same visits and same result:
//  - the cut-off d^2 < r2 lives in the sentinel, the largest key below
//    (r2, id 0) (= (prev_float(r2), 0xFFFFFFFF)): `key < list[K-1]` alone
//    admits exactly the candidates (no f32 / lo compares per step); the
//    radius of a list that did not fill is r2 (radiance_r2);
//  - the point test and the queue write are branch-free (a non-candidate is
//    written above the queue top and overwritten later), finished lanes keep
//    re-reading their last node and their results are masked, so the step
//    runs without exec-mask branches; only the wave-uniform insert round
//    branches.
//  - cut: admit d^2 <= cut (default prev_float(r2), i.e. d^2 < r2); a seeded
//    cut-off (seed_cut) only narrows the walk, never the result.
__device__ __forceinline__ float lean_cut(float r2) { return __uint_as_float(__float_as_uint(r2) - 1u); }

//  - JUMP: finished subtrees are left without re-reading the nodes above them.
//    A per-lane bit mask records, per depth, whether the path entered that
//    depth's node as the FAR child. A node whose far child is done (or
//    skipped) is finished; so is every consecutive far-child ancestor, whose
//    far child it was. The walk jumps straight to the parent of the deepest
//    close-child ancestor-or-self (one step, one cached load), where the
//    post-order point test and the far decision run. Same visited set, same
//    point tests, fewer dependent loads.
// Walk state of one lane (knn_walk_lean).
struct LeanWalk {
  float bound;
  int prev, curr;
  uint32_t far_mask;   // JUMP: bit d set <=> the path's depth-d node is a far child
  int depth;           // JUMP: depth of curr
  bool walking;
  int qn;              // queued candidates in this lane's LDS column
  __device__ __forceinline__ void start(float b, bool valid) {
    bound = b;
    prev = -1;
    curr = 0;
    far_mask = 0;
    depth = 0;
    walking = valid;
  }
};

// One walk step of every lane (finished / idle lanes re-read their last node and
// are masked): the post-order point test queues a candidate, the walk moves on.
template <int K, bool JUMP>
__device__ __forceinline__ void lean_step(const float4* __restrict__ nodes, int n, v3 q, const double (&list)[K],
                                          LeanWalk& w, double* lq, int lstride) {
  const float4 nd = nodes[w.curr];
  const int child = 2 * w.curr + 1;
  const int wd = __float_as_int(nd.w);
  const int dim = wd & 3;
  const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
  const float diff = dim == 0 ? dx : (dim == 1 ? dy : dz);   // = q[dim] - nd[dim]
  const int side = diff > 0.f ? 1 : 0;
  const int close_c = child + side, far_c = child + 1 - side;
  const int parent = ((w.curr + 1) >> 1) - 1;
  const bool down = w.prev < child;
  const bool test = (down && close_c >= n) || w.prev == close_c;
  const float d2 = dx * dx + dy * dy + dz * dz;
  const double key = key_make(d2, (uint32_t)wd >> 2);
  const bool cand = w.walking && test && key < list[K - 1];
  int next, nprev;
  if (JUMP) {
    if (down && close_c < n) {
      next = close_c;
      nprev = w.curr;
      w.far_mask &= ~(2u << w.depth);
      w.depth++;
    } else if (far_c < n && diff * diff <= w.bound) {
      next = far_c;
      nprev = w.curr;
      w.far_mask |= 2u << w.depth;
      w.depth++;
    } else {
      // curr is finished: deepest close-child ancestor-or-self a (depth da);
      // bit 0 (the root) is always clear, so da = 0 ends the walk
      const uint32_t open = (~w.far_mask & ((2u << w.depth) - 1u)) | 1u;
      const int da = 31 - __clz(open);
      const int a = ((w.curr + 1) >> (w.depth - da)) - 1;
      next = da == 0 ? -1 : ((a + 1) >> 1) - 1;
      nprev = a;
      w.depth = da - 1;
    }
  } else {
    if (w.prev == far_c) next = parent;
    else if (w.prev == close_c || close_c >= n) next = (far_c < n && diff * diff <= w.bound) ? far_c : parent;
    else next = close_c;
    nprev = w.curr;
  }
  lq[w.qn * lstride] = key;
  w.qn += cand ? 1 : 0;
  const bool go = w.walking && next >= 0;
  w.prev = go ? nprev : w.prev;
  w.curr = go ? next : w.curr;
  w.walking = go;
}

// Wave-uniform insert round: every lane with a queued key pops one.
template <int K>
__device__ __forceinline__ void lean_round(double (&list)[K], LeanWalk& w, const double* lq, int lstride) {
  const bool pop = w.qn > 0;
  w.qn -= pop ? 1 : 0;
  const double ik = pop ? lq[w.qn * lstride] : __longlong_as_double(0x7FEFFFFFFFFFFFFFll);
  if (ik < list[K - 1]) {
    list_insert<K>(list, ik);
    w.bound = key_d2(list[K - 1]);
  }
}

__device__ __forceinline__ double lean_sentinel(float cut) {
  return __longlong_as_double((long long)((((uint64_t)__float_as_uint(cut)) << 32 | 0xFFFFFFFFull) + kKeyBias));
}

template <int K, int QL, bool JUMP = false>
__device__ __forceinline__ void knn_walk_lean(const float4* __restrict__ nodes, int n, v3 q, float cut, bool valid,
                                              double (&list)[K], double* lq, int lstride) {
  const double sentinel = lean_sentinel(cut);
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  if (n <= 0) return;   // empty map: every lane keeps the sentinel list (uniform)
  LeanWalk w;
  w.start(key_d2(sentinel), valid);
  w.qn = 0;
  for (;;) {
    lean_step<K, JUMP>(nodes, n, q, list, w, lq, lstride);
    const bool any_walking = __ballot(w.walking) != 0;
    if (__ballot(w.qn == QL) != 0 || !any_walking) {   // wave-uniform insert round
      lean_round<K>(list, w, lq, lstride);
      if (!any_walking && __ballot(w.qn > 0) == 0) break;
    }
  }
}

// radius^2 of a finished lean list: the K-th d^2, or r2 if the list did not fill
template <int K>
__device__ __forceinline__ float radiance_r2(const double (&list)[K], float r2) {
  return key_id(list[K - 1]) == 0xFFFFFFFFu ? r2 : key_d2(list[K - 1]);
}

// pm_knn: K-wide list for k <= K; k > 128 runs 128-wide passes (j0 = output
// offset of this pass, lo_in / lo_out = last key of the previous / this pass).
// QL > 0: candidates go through a QL-deep per-lane LDS queue (knn_walk), as in
// the gather; the 128-wide passes of k > 128 use it (config 5, k = 200).
template <int K, int QP, int QL = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K <= 64 ? 4 : 1))) void k_knn(
    const float4* nodes, int n, const pm_float3* q, int64_t nq, int k, int j0, float r2, int32_t* ids, float* d2o,
    float* maxd2, const double* lo_in, double* lo_out, const float* cutq = nullptr) {
  __shared__ double lq[QL > 0 ? QL * 256 : 1];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < nq;
  double list[K];
  const pm_float3 p = valid ? q[i] : pm_float3{0.f, 0.f, 0.f};
  const double lo = (valid && lo_in) ? lo_in[i] : 0.0;
  // a previous pass whose list did not fill (last key = the sentinel, id -1)
  // found every candidate: this pass has none to find, its walk is skipped
  const bool done = lo_in && key_id(lo) == 0xFFFFFFFFu;
  // cutq: a seeded (strict) cut-off per query, <= r2, that provably admits the
  // pass's keys (launch_gather_k); the reported radius stays r2
  const float rw = (valid && cutq) ? cutq[i] : r2;
  knn_walk<K, true, QP, false, QL>(nodes, n, mk(p), rw, valid && !done, list, nullptr, lq + threadIdx.x, 256, lo);
  if (!valid) return;
#pragma unroll
  for (int j = 0; j < K; j++) {
    const int jj = j0 + j;
    const bool empty = key_id(list[j]) == 0xFFFFFFFFu;
    if (jj < k) {
      ids[i * k + jj] = empty ? -1 : (int32_t)key_id(list[j]);
      if (d2o) d2o[i * k + jj] = empty ? r2 : key_d2(list[j]);
    }
    if (jj == k - 1 && maxd2) maxd2[i] = empty ? r2 : key_d2(list[j]);
  }
  if (lo_out) lo_out[i] = list[K - 1];
}

// Radiance estimate from a finished candidate list: gatherPhotons
// (shading.h:93-121), neighbours summed in (d^2, index) order.
__device__ __forceinline__ v3 radiance(const double (&list)[kKNearest], const float4* __restrict__ payload,
                                       float brdf, float r2) {
  v3 flux = {0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < kKNearest; p++) {
    const uint32_t id = key_id(list[p]);
    if (id == 0xFFFFFFFFu) continue;
    const float4 pl = payload[id];
    const float dist = sqrtf(key_d2(list[p]));
    const float w = 1 - (dist / sqrtf(r2) * kConeFilterC);
    flux = add(flux, smul(brdf * pl.w * w, v3{pl.x, pl.y, pl.z}));
  }
  return divf(flux, (1 - (2.f / 3.f) * (1.f / kConeFilterC)) * 2 * kPI * r2);
}

// TAG only separates the global-map launch into its own kernel symbol (rocprof).
// perm (optional): lane i takes query perm[i] and writes its result there, so a
// caller can walk in Morton order without permuted / unpermuted copies.
template <int TAG, bool POST, int QP, int QL = 0, bool LEAN = false, bool JUMP = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gather(
    const float4* __restrict__ nodes, const float4* __restrict__ payload, int n, const float4* __restrict__ qb,
    int64_t nq, float4* __restrict__ out, const uint32_t* __restrict__ perm) {
  __shared__ double lq[QL > 0 ? QL * 256 : 1];
  // plain block order on purpose: consecutive blocks (Morton-adjacent queries)
  // spread over the 8 XCDs keep ONE narrow window of the tree live in the
  // shared Infinity Cache; an XCD-contiguous remap measured 9 % slower.
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i0 < nq;
  const int64_t i = (valid && perm) ? (int64_t)perm[i0] : i0;
  const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  double list[kKNearest];
  const float R2 = kKMaxDistance * kKMaxDistance;
  if (LEAN) {
    knn_walk_lean<kKNearest, QL, JUMP>(nodes, n, v3{qq.x, qq.y, qq.z}, lean_cut(R2), valid, list, lq + threadIdx.x,
                                       256);
  } else {
    knn_walk<kKNearest, POST, QP, false, QL>(nodes, n, v3{qq.x, qq.y, qq.z}, R2, valid, list, nullptr,
                                             lq + threadIdx.x, 256);
  }
  if (valid) {
    const v3 f = radiance(list, payload, qq.w, LEAN ? radiance_r2(list, R2) : key_d2(list[kKNearest - 1]));
    out[i] = make_float4(f.x, f.y, f.z, 0.f);
  }
}

// Seeded cut-off (PM_GATHER_MODE 12; 13 = with the JUMP walk, default). Every kSeedStride-th query
// in walk order is a LEADER; the first k_gather_level launch runs the leaders
// with the plain cut-off and keeps (position, K-th d^2). The other queries then start from a
// cut-off that provably holds the K nearest: the leader's K points lie within
// sqrt(t') of q', hence within sqrt(t') + |q - q'| of q (triangle inequality),
// so at least K photons have d^2 <= that bound and the K smallest keys -- the
// result -- are all admitted. The bound is the smallest over the consulted
// leaders' and is inflated (1e-6 relative per step, 1e-5 on the square, 1e-30
// absolute) past the rounding of the f32 d^2 on both sides; a leader whose list
// did not fill (t' = -1) seeds nothing. The cut-off only prunes: the visited
// set shrinks, the list and the radiance are bitwise those of the plain walk.
// Leader stride and leaders consulted per follower (the enclosing pair, plus one
// more on each side): build knobs. Config 3 global gather (ms): stride 8 / 2
// leaders 50.9, 8/4 50.3, 4/2 52.2, 16/2 50.6, 16/4 49.8. A follower bound from
// the union of the enclosing leaders' neighbour sets (K-th smallest distance,
// exact by construction) was tighter but slower: 54.6 (its 1.6 KB of leader
// points per follower cost more than the walk saved). Seed tightness on config 3
// (PM_GATHER_SEEDSTATS): even the previous query in walk order gives a mean
// bound / exact K-th d^2 of 2.8 on the global map, the stride-8 pair 2.8; the
// exact-cut re-walk (mode 16) takes 34.4 ms, the floor of any seeding. Leader
// hierarchies (PM_SEED_LEVELS) measured slower: 256,16 52.7; 16,8 51.6;
// 16,4 52.0; 4096,256,16 54.5. A pooled variant (lanes refill from a per-
// workgroup chunk, as in traverse_pool) ran 2.5x slower: the 100-VGPR list plus
// the walk state leave no room for the pool's state (30 VGPRs spilled at 128).
#ifndef PM_SEED_STRIDE
#define PM_SEED_STRIDE 16
#endif
#ifndef PM_GATHER_QL
#define PM_GATHER_QL 8   // LDS insert-queue depth of the seeded gather (build knob)
#endif
#ifndef PM_SEED_LEADERS
#define PM_SEED_LEADERS 4
#endif
constexpr int kSeedStride = PM_SEED_STRIDE;

__device__ __forceinline__ double seed_bound(float4 lead, v3 q) {
  if (!(lead.w >= 0.f)) return 1e300;
  const double dx = (double)q.x - lead.x, dy = (double)q.y - lead.y, dz = (double)q.z - lead.z;
  const double c = (sqrt((double)lead.w) + sqrt(dx * dx + dy * dy + dz * dz)) * (1.0 + 1e-6);
  return c * c * (1.0 + 1e-5) + 1e-30;
}
// f32 cut-off >= bound (rounded up), capped at the plain cut-off
__device__ __forceinline__ float seed_cut(double bound, float r2) {
  const float plain = lean_cut(r2);
  if (!(bound < (double)plain)) return plain;
  float f = (float)bound;
  if ((double)f < bound) f = __uint_as_float(__float_as_uint(f) + 1u);
  return fminf(f, plain);
}

// One level of the seeded gather (modes 12 / 13). Walk ranks of this level: the
// multiples of `stride` that are not multiples of `sstride` (sstride = 0: every
// multiple, the top level, plain cut-off). Its cut-off comes from the records of
// the enclosing level (ranks that are multiples of sstride: the enclosing pair plus
// one more on each side). A level with stride >= gran (the finest leader stride)
// records (position, K-th d^2) of its queries in lead[rank / gran]. Levels
// "256,16" (PM_SEED_LEVELS): the stride-16 leaders no longer walk with the plain
// cut-off (2.6x a follower's cost per query) but are seeded by stride-256 ones.
// walk rank of the t-th query of a level (see k_gather_level)
__device__ __forceinline__ int64_t level_rank(int64_t t, int64_t stride, int64_t sstride) {
  if (sstride == 0) return t * stride;
  const int64_t m = sstride / stride;
  return ((t / (m - 1)) * m + 1 + t % (m - 1)) * stride;
}
// cut-off of rank r from the enclosing level's records
__device__ __forceinline__ float level_cut(const float4* __restrict__ lead, int64_t nq, int64_t r, int64_t sstride,
                                           int64_t gran, v3 q, float R2) {
  if (sstride <= 0) return lean_cut(R2);
  const int64_t jp = r / sstride, ls = sstride / gran, ns = (nq - 1) / sstride + 1;
  double b = seed_bound(lead[jp * ls], q);
  if (jp + 1 < ns) b = fmin(b, seed_bound(lead[(jp + 1) * ls], q));
  if (PM_SEED_LEADERS > 2) {
    if (jp >= 1) b = fmin(b, seed_bound(lead[(jp - 1) * ls], q));
    if (jp + 2 < ns) b = fmin(b, seed_bound(lead[(jp + 2) * ls], q));
  }
  if (PM_SEED_LEADERS > 4) {
    if (jp >= 2) b = fmin(b, seed_bound(lead[(jp - 2) * ls], q));
    if (jp + 3 < ns) b = fmin(b, seed_bound(lead[(jp + 3) * ls], q));
  }
  return seed_cut(b, R2);
}

template <int TAG, int QL, bool JUMP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gather_level(
    const float4* __restrict__ nodes, const float4* __restrict__ payload, int n, const float4* __restrict__ qb,
    int64_t nq, float4* __restrict__ out, const uint32_t* __restrict__ perm, float4* __restrict__ lead,
    int64_t stride, int64_t sstride, int64_t gran, int xcd) {
  __shared__ double lq[QL * 256];
  // xcd (A/B knob, off): workgroups are dealt round-robin to the 8 XCDs; remap so
  // XCD x walks the contiguous block range [x * G/8, (x+1) * G/8) (its own narrow
  // window of the tree in its L2) instead of all XCDs sharing one window (grid
  // padded to 8k). Measured on config 3: global gather 50.3 -> 60.4 ms, i.e. the
  // shared window (one copy in the Infinity Cache, fed to all 8 L2s) wins.
  const int64_t b = xcd ? (int64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : (int64_t)blockIdx.x;
  const int64_t t = b * blockDim.x + threadIdx.x;
  const int64_t r = level_rank(t, stride, sstride);
  const bool valid = r < nq;
  const int64_t i = !valid ? 0 : (perm ? (int64_t)perm[r] : r);
  const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const v3 q = {qq.x, qq.y, qq.z};
  const float R2 = kKMaxDistance * kKMaxDistance;
  const float cut = valid ? level_cut(lead, nq, r, sstride, gran, q, R2) : lean_cut(R2);
  double list[kKNearest];
  knn_walk_lean<kKNearest, QL, JUMP>(nodes, n, q, cut, valid, list, lq + threadIdx.x, 256);
  if (valid) {
    const bool full = key_id(list[kKNearest - 1]) != 0xFFFFFFFFu;
    const v3 f = radiance(list, payload, qq.w, full ? key_d2(list[kKNearest - 1]) : R2);
    out[i] = make_float4(f.x, f.y, f.z, 0.f);
    if (stride >= gran) lead[r / gran] = make_float4(qq.x, qq.y, qq.z, full ? key_d2(list[kKNearest - 1]) : -1.f);
  }
}

// Diagnostic (PM_GATHER_MODE 16): pass 1 records each query's exact K-th d^2,
// pass 2 (k_gather_exactcut) re-walks from that cut-off: the floor any seeded
// cut-off can reach.
template <int TAG, bool JUMP, bool SECOND>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gather_exactcut(
    const float4* __restrict__ nodes, const float4* __restrict__ payload, int n, const float4* __restrict__ qb,
    int64_t nq, float4* __restrict__ out, const uint32_t* __restrict__ perm, float* __restrict__ cutb) {
  __shared__ double lq[8 * 256];
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = r < nq;
  const int64_t i = !valid ? 0 : (perm ? (int64_t)perm[r] : r);
  const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float R2 = kKMaxDistance * kKMaxDistance;
  const float cut = (SECOND && valid) ? cutb[r] : lean_cut(R2);
  double list[kKNearest];
  knn_walk_lean<kKNearest, 8, JUMP>(nodes, n, v3{qq.x, qq.y, qq.z}, cut, valid, list, lq + threadIdx.x, 256);
  if (valid) {
    const v3 f = radiance(list, payload, qq.w, radiance_r2(list, R2));
    out[i] = make_float4(f.x, f.y, f.z, 0.f);
    if (!SECOND) cutb[r] = key_id(list[kKNearest - 1]) != 0xFFFFFFFFu ? key_d2(list[kKNearest - 1]) : lean_cut(R2);
  }
}

// Diagnostic (PM_GATHER_SEEDSTATS=1): how tight seeded cut-offs are. For each
// query with a full list: the bound from the query d places earlier in walk
// order (d = 1, 2, 4), and the production stride-8 two-leader bound, each
// divided by the query's exact K-th d^2; histogram of log2(ratio) in 1/4 steps.
__global__ void k_seed_stats(const float4* __restrict__ qb, int64_t nq, const uint32_t* __restrict__ perm,
                             const float* __restrict__ cutb, unsigned long long* hist) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nq || r < 8) return;
  const float4 qq = qb[perm ? perm[r] : r];
  const v3 q = {qq.x, qq.y, qq.z};
  const float ex = cutb[r];
  if (!(ex > 0.f) || ex >= 9999.f) return;
  auto bin = [&](double b) {
    const double l = log2(b / ex) * 4.0;
    return (int)fmin(fmax(l, 0.0), 31.0);
  };
  const int ds[3] = {1, 2, 4};
  for (int k = 0; k < 3; k++) {
    const int64_t o = r - ds[k];
    const float4 p = qb[perm ? perm[o] : o];
    const double b = seed_bound(make_float4(p.x, p.y, p.z, cutb[o] < 9999.f ? cutb[o] : -1.f), q);
    atomicAdd(&hist[k * 32 + bin(b)], 1ull);
  }
  if (r % kSeedStride) {
    const int64_t l0 = r - r % kSeedStride, l1 = l0 + kSeedStride;
    const float4 p0 = qb[perm ? perm[l0] : l0];
    double b = seed_bound(make_float4(p0.x, p0.y, p0.z, cutb[l0] < 9999.f ? cutb[l0] : -1.f), q);
    if (l1 < nq) {
      const float4 p1 = qb[perm ? perm[l1] : l1];
      b = fmin(b, seed_bound(make_float4(p1.x, p1.y, p1.z, cutb[l1] < 9999.f ? cutb[l1] : -1.f), q));
    }
    atomicAdd(&hist[3 * 32 + bin(b)], 1ull);
  }
}

static void seed_stats(const pm_photon_map* m, const float4* qb, int64_t nq, hipStream_t s, const uint32_t* perm) {
  DevBuf<float> cutb(nq);
  DevBuf<float4> tmp(nq);
  DevBuf<unsigned long long> hist(128);
  if (!cutb.p || !tmp.p || !hist.p || hipMemsetAsync(hist.p, 0, 128 * 8, s) != hipSuccess) return;
  const int g = grid_for(nq, 256);
  k_gather_exactcut<0, true, false><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, (int)m->n, qb, nq, tmp.p, perm,
                                                       cutb.p);
  k_seed_stats<<<g, 256, 0, s>>>(qb, nq, perm, cutb.p, hist.p);
  unsigned long long h[128] = {};
  if (hipMemcpyAsync(h, hist.p, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return;
  const char* names[4] = {"prev 1", "prev 2", "prev 4", "stride-8 leaders"};
  for (int k = 0; k < 4; k++) {
    double tot = 0, mean = 0;
    for (int b = 0; b < 32; b++) tot += (double)h[k * 32 + b];
    std::fprintf(stderr, "[seed-stats n=%lld nq=%lld] %-16s log2(bound/exact)*4 hist:", (long long)m->n,
                 (long long)nq, names[k]);
    for (int b = 0; b < 32; b++) {
      mean += (double)h[k * 32 + b] * std::exp2((b + 0.5) / 4.0);
      std::fprintf(stderr, " %.3f", tot > 0 ? h[k * 32 + b] / tot : 0.0);
    }
    std::fprintf(stderr, " | mean ratio ~%.2f\n", tot > 0 ? mean / tot : 0.0);
  }
}

// Diagnostics (PM_GATHER_STATS=1): per-lane walk steps and list insertions,
// per-wave max steps and the number of walk iterations in which ANY lane
// inserted (the wave executes the 50-wide insert that often).
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  return v;
}

template <bool POST, int QP, int QL = 0>
__global__ __launch_bounds__(256) void k_gather_stats(const float4* __restrict__ nodes, int n,
                                                      const float4* __restrict__ qb, int64_t nq,
                                                      unsigned long long* acc, const uint32_t* __restrict__ perm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  KnnCounters kc;
  const bool valid = i < nq;
  const float4 qq = valid ? qb[perm ? (int64_t)perm[i] : i] : make_float4(0.f, 0.f, 0.f, 0.f);
  double list[kKNearest];
  __shared__ double lq[QL > 0 ? QL * 256 : 1];
  knn_walk<kKNearest, POST, QP, true, QL>(nodes, n, v3{qq.x, qq.y, qq.z}, kKMaxDistance * kKMaxDistance, valid,
                                          list, &kc, lq + threadIdx.x, 256);
  const uint32_t s = wave_sum(kc.steps), in = wave_sum(kc.ins), ms = wave_max(kc.steps), wi = wave_max(kc.wave_ins);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&acc[0], (unsigned long long)s);
    atomicAdd(&acc[1], (unsigned long long)in);
    atomicAdd(&acc[2], (unsigned long long)ms);
    atomicAdd(&acc[3], (unsigned long long)wi);
    atomicAdd(&acc[4], 1ull);
  }
}

static void gather_stats(const pm_photon_map* m, const float4* qb, int64_t nq, int mode, hipStream_t s,
                         const uint32_t* perm) {
  DevBuf<unsigned long long> acc(8);
  if (!acc.p || hipMemsetAsync(acc.p, 0, 64, s) != hipSuccess) return;
  const int g = grid_for(nq, 256);
  if (mode == 4) k_gather_stats<true, 0><<<g, 256, 0, s>>>(m->nodes.p, (int)m->n, qb, nq, acc.p, perm);
  else if (mode == 5) k_gather_stats<true, 4><<<g, 256, 0, s>>>(m->nodes.p, (int)m->n, qb, nq, acc.p, perm);
  else if (mode == 0) k_gather_stats<false, 0><<<g, 256, 0, s>>>(m->nodes.p, (int)m->n, qb, nq, acc.p, perm);
  else if (mode == 10) k_gather_stats<true, 0, 16><<<g, 256, 0, s>>>(m->nodes.p, (int)m->n, qb, nq, acc.p, perm);
  else k_gather_stats<true, 0, 8><<<g, 256, 0, s>>>(m->nodes.p, (int)m->n, qb, nq, acc.p, perm);
  unsigned long long h[8] = {};
  if (hipMemcpyAsync(h, acc.p, 64, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return;
  const double q = (double)nq, w = (double)h[4];
  std::fprintf(stderr,
               "[gather-stats mode %d] n=%lld queries=%lld steps/query=%.1f inserts/query=%.1f | per wave: max steps=%.1f "
               "insert iterations=%.1f (lane-mean steps %.1f)\n",
               mode, (long long)m->n, (long long)nq, h[0] / q, h[1] / q, h[2] / w, h[3] / w, h[0] / q);
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

// Leader strides of the seeded gather, coarsest first, each a multiple of the
// next (PM_SEED_LEVELS, e.g. "256,16"; read per launch). Default: PM_SEED_STRIDE alone.
static std::vector<int64_t> seed_levels() {
  std::vector<int64_t> v;
  {
    const char* e = std::getenv("PM_SEED_LEVELS");
    if (e) {
      for (const char* p = e; *p;) {
        char* q = nullptr;
        const long long x = std::strtoll(p, &q, 10);
        if (q == p) break;
        if (x >= 2 && (v.empty() || (v.back() % x == 0 && v.back() > x))) v.push_back(x);
        p = (*q == ',') ? q + 1 : q;
      }
    }
    if (v.empty()) v.push_back(kSeedStride);
  }
  return v;
}

// cut1 / cut2 (optional): per-query strict cut-offs of the first / second pass
hipError_t launch_knn(const pm_photon_map* m, const pm_float3* q, int64_t nq, int k, float radius, int32_t* ids,
                      float* d2, float* maxd2, hipStream_t s, const float* cut1, const float* cut2) {
  if (nq <= 0) return hipSuccess;
  const float r2 = radius * radius;
  const int n = (int)m->n;
  const int g = grid_for(nq, 256);
#define PM_KNN_CASE(KK, QQ)                                                                                \
  if (k <= KK) {                                                                                           \
    k_knn<KK, QQ><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, 0, r2, ids, d2, maxd2, nullptr, nullptr, cut1); \
    return hipGetLastError();                                                                              \
  }
  PM_KNN_CASE(8, 0)
  PM_KNN_CASE(16, 0)
  PM_KNN_CASE(32, 0)
  PM_KNN_CASE(50, 0)
  PM_KNN_CASE(64, 0)
  PM_KNN_CASE(128, 0)
#undef PM_KNN_CASE
  if (k > 256) return hipErrorInvalidValue;
  // 128 < k <= 256: exact passes of W keys, each collecting the W smallest keys
  // above the previous pass's last (PM_KNN_PASS_W: 128 (2 passes, 256 VGPRs,
  // 2 waves/SIMD) or 64 (4 passes, 128 VGPRs, 4 waves/SIMD))
  const char* wenv = std::getenv("PM_KNN_PASS_W");
  const int W = (wenv && std::atoi(wenv) == 64) ? 64 : 128;
  const char* qenv = std::getenv("PM_KNN_QUEUE");   // LDS insert queue in the 128-wide passes
  const bool ql = !qenv || std::atoi(qenv) != 0;
  DevBuf<double> la(nq), lb(nq);
  if (!la.p || !lb.p) return hipErrorOutOfMemory;
  double *lin = nullptr, *lout = la.p;
  for (int j0 = 0; j0 < k; j0 += W) {
    double* lo_out = j0 + W < k ? lout : nullptr;
    const float* cut = (W == 128) ? (j0 == 0 ? cut1 : cut2) : nullptr;
    if (W == 64)
      k_knn<64, 0><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, j0, r2, ids, d2, maxd2, lin, lo_out);
    else if (ql)
      k_knn<128, 0, 8><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, j0, r2, ids, d2, maxd2, lin, lo_out, cut);
    else
      k_knn<128, 0><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, j0, r2, ids, d2, maxd2, lin, lo_out, cut);
    PM_HIP_TRY(hipGetLastError());
    lin = lout;
    lout = lout == la.p ? lb.p : la.p;
  }
  return hipStreamSynchronize(s);   // the pass bounds are freed on return
}

hipError_t launch_gather(const pm_photon_map* m, const float4* qb, int64_t nq, float4* out, hipStream_t s,
                         int tag, const uint32_t* perm) {
  if (nq <= 0) return hipSuccess;
  // A/B knob (read per launch), all variants return identical bits:
  //  13 (default) mode 12 with the JUMP walk                   49.8 ms
  //  14 mode 11 with the JUMP walk                             59.0 ms
  //  16 / 17 diagnostic: exact-cut re-walk (JUMP / plain), see k_gather_exactcut
  //  12 mode 11 behind leader-seeded cut-offs (k_gather_level)   53.5 ms
  //  11 mode 9 with the lean step (knn_walk_lean)   62.3 ms
  //   9 post-order + 8-deep LDS insert queue                  66.7 ms
  //   4 post-order, insert at once                             73.6 ms
  //   5 post-order + 4-entry VGPR queue (spills)               74.1 ms
  //  10 post-order + 16-deep LDS queue (staler bound)          69.1 ms
  //   0 pre-order, insert at once
  // (config 3 global map; depths 4 / 6: 67.3 / 66.4 ms)
  const char* env = std::getenv("PM_GATHER_MODE");
  const int mode = env ? std::atoi(env) : 13;
  if (std::getenv("PM_GATHER_STATS")) gather_stats(m, qb, nq, mode, s, perm);
  if (std::getenv("PM_GATHER_SEEDSTATS")) seed_stats(m, qb, nq, s, perm);
  const int g = grid_for(nq, 256);
  const int n = (int)m->n;
  const std::vector<int64_t> lv = seed_levels();
  const char* xenv = std::getenv("PM_GATHER_XCD");   // A/B knob: XCD-contiguous block ranges
  const int xcd = xenv ? std::atoi(xenv) : 0;
  if ((mode == 12 || mode == 13) && nq > lv.back()) {
    const int64_t gran = lv.back();
    DevBuf<float4> lead((nq + gran - 1) / gran);
    if (!lead.p) return hipErrorOutOfMemory;
    int64_t sstride = 0;
    for (size_t l = 0; l <= lv.size(); l++) {
      const int64_t stride = l < lv.size() ? lv[l] : 1;
      const int64_t nr = (nq + stride - 1) / stride - (sstride ? (nq + sstride - 1) / sstride : 0);
      {
        int gl = grid_for(nr, 256);
        if (xcd) gl = (gl + 7) / 8 * 8;
#define PM_LEVEL(T, J)                                                                                         \
  k_gather_level<T, PM_GATHER_QL, J><<<gl, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm, lead.p, stride, \
                                             sstride, gran, xcd)
        if (tag == 1 && mode == 13) PM_LEVEL(1, true);
        else if (tag == 1) PM_LEVEL(1, false);
        else if (mode == 13) PM_LEVEL(0, true);
        else PM_LEVEL(0, false);
#undef PM_LEVEL
      }
      PM_HIP_TRY(hipGetLastError());
      sstride = stride;
    }
    return hipSuccess;
  }
  if (mode == 16 || mode == 17) {
    DevBuf<float> cutb(nq);
    if (!cutb.p) return hipErrorOutOfMemory;
    if (mode == 16) {
      k_gather_exactcut<0, true, false><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm, cutb.p);
      k_gather_exactcut<1, true, true><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm, cutb.p);
    } else {
      k_gather_exactcut<0, false, false><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm, cutb.p);
      k_gather_exactcut<1, false, true><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm, cutb.p);
    }
    return hipGetLastError();
  }
#define PM_WALK(P, Q, L, LEAN, ...)                                                                                  \
  (tag == 1 ? (k_gather<1, P, Q, L, LEAN, ##__VA_ARGS__><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm)) \
            : (k_gather<0, P, Q, L, LEAN, ##__VA_ARGS__><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm)))
  switch (mode) {
    case 11: PM_WALK(true, 0, 8, true); break;
    case 14: PM_WALK(true, 0, 8, true, true); break;
    case 0: PM_WALK(false, 0, 0, false); break;
    case 4: PM_WALK(true, 0, 0, false); break;
    case 5: PM_WALK(true, 4, 0, false); break;
    case 10: PM_WALK(true, 0, 16, false); break;
    default: PM_WALK(true, 0, 8, false); break;
  }
#undef PM_WALK
  return hipGetLastError();
}

// ---- radiance estimate with k != 50 neighbours (k = 200
// caustic gather). gatherPhotons (shading.h:93-121) over the k nearest: the
// exact lists come from the pm_knn passes (k <= 128 one pass, up to 256 in
// 128-wide passes), then one kernel sums them in (d^2, index) order with
// r^2 = the k-th d^2 (max_radius^2 if fewer were found), as for k = 50.
__global__ void k_q3_from_dense(const float4* __restrict__ qb, const uint32_t* __restrict__ perm, int64_t nq,
                                pm_float3* __restrict__ q3) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float4 q = qb[perm ? (int64_t)perm[i] : i];
  q3[i] = {q.x, q.y, q.z};
}

__global__ void k_radiance_k(const float4* __restrict__ qb, const uint32_t* __restrict__ perm, int64_t nq, int k,
                             const int32_t* __restrict__ ids, const float* __restrict__ d2,
                             const float* __restrict__ maxd2, const float4* __restrict__ payload,
                             float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const int64_t r = perm ? (int64_t)perm[i] : i;
  const float brdf = qb[r].w;
  const float r2 = maxd2[i];
  v3 flux = {0.f, 0.f, 0.f};
  for (int j = 0; j < k; j++) {
    const int32_t id = ids[i * k + j];
    if (id < 0) continue;
    const float4 pl = payload[id];
    const float dist = sqrtf(d2[i * k + j]);
    const float w = 1 - (dist / sqrtf(r2) * kConeFilterC);
    flux = add(flux, smul(brdf * pl.w * w, v3{pl.x, pl.y, pl.z}));
  }
  const v3 f = divf(flux, (1 - (2.f / 3.f) * (1.f / kConeFilterC)) * 2 * kPI * r2);
  out[r] = make_float4(f.x, f.y, f.z, 0.f);
}

// Seeded cut-offs for the general-k passes (the same triangle-inequality bound
// as k_gather_level): every 16th query in walk order is a leader and runs the
// plain passes first; a query's pass-1 cut comes from the leaders' min(k, 128)-th
// d^2, its pass-2 cut from their k-th d^2 (a leader whose list did not fill
// seeds nothing). Strict cut-offs (k_knn admits d^2 < cut).
__global__ void k_q3_leaders(const pm_float3* __restrict__ q3, int64_t nl, pm_float3* __restrict__ q3l) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nl) q3l[j] = q3[j * kSeedStride];
}
__global__ void k_knn_cuts(const pm_float3* __restrict__ q3, int64_t nq, const pm_float3* __restrict__ q3l,
                           int64_t nl, int k, const int32_t* __restrict__ idsl, const float* __restrict__ d2l,
                           float* __restrict__ cut1, float* __restrict__ cut2) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nq) return;
  const v3 q = {q3[r].x, q3[r].y, q3[r].z};
  const float R2 = kKMaxDistance * kKMaxDistance;
  const int k1 = k < 128 ? k : 128;
  const int64_t jp = r / kSeedStride;
  double b1 = 1e300, b2 = 1e300;
  for (int64_t j = jp - 1; j <= jp + 2; j++) {
    if (j < 0 || j >= nl) continue;
    const float4 p = make_float4(q3l[j].x, q3l[j].y, q3l[j].z, 0.f);
    const int64_t a = j * k + (k1 - 1), c = j * k + (k - 1);
    b1 = fmin(b1, seed_bound(make_float4(p.x, p.y, p.z, idsl[a] >= 0 ? d2l[a] : -1.f), q));
    b2 = fmin(b2, seed_bound(make_float4(p.x, p.y, p.z, idsl[c] >= 0 ? d2l[c] : -1.f), q));
  }
  // seed_cut is inclusive (d^2 <= cut); the next float up makes it strict
  cut1[r] = __uint_as_float(__float_as_uint(seed_cut(b1, R2)) + 1u);
  cut2[r] = __uint_as_float(__float_as_uint(seed_cut(b2, R2)) + 1u);
}

hipError_t launch_gather_k(const pm_photon_map* m, const float4* qb, int64_t nq, float4* out, hipStream_t s,
                           int k, const uint32_t* perm) {
  if (nq <= 0) return hipSuccess;
  if (k < 1 || k > 256) return hipErrorInvalidValue;
  if (k == kKNearest) return launch_gather(m, qb, nq, out, s, 0, perm);
  DevBuf<pm_float3> q3(nq);
  DevBuf<int32_t> ids((size_t)nq * k);
  DevBuf<float> d2((size_t)nq * k), md(nq);
  if (!q3.p || !ids.p || !d2.p || !md.p) return hipErrorOutOfMemory;
  k_q3_from_dense<<<grid_for(nq, 256), 256, 0, s>>>(qb, perm, nq, q3.p);
  PM_HIP_TRY(hipGetLastError());
  // PM_KNN_SEED=1: leader-seeded cut-offs (bitwise the same). Config 5 measured
  // slower (caustic gather 195 -> 240 ms): the 128-wide passes are bound by their
  // >= 128 inserts of 255 ops each, which a tighter cut does not remove.
  const char* senv = std::getenv("PM_KNN_SEED");
  if (senv && std::atoi(senv) != 0 && nq > kSeedStride && m->n > 0) {
    const int64_t nl = (nq + kSeedStride - 1) / kSeedStride;
    DevBuf<pm_float3> q3l(nl);
    DevBuf<int32_t> idsl((size_t)nl * k);
    DevBuf<float> d2l((size_t)nl * k), mdl(nl), c1(nq), c2(nq);
    if (!q3l.p || !idsl.p || !d2l.p || !mdl.p || !c1.p || !c2.p) return hipErrorOutOfMemory;
    k_q3_leaders<<<grid_for(nl, 256), 256, 0, s>>>(q3.p, nl, q3l.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(launch_knn(m, q3l.p, nl, k, kKMaxDistance, idsl.p, d2l.p, mdl.p, s, nullptr, nullptr));
    k_knn_cuts<<<grid_for(nq, 256), 256, 0, s>>>(q3.p, nq, q3l.p, nl, k, idsl.p, d2l.p, c1.p, c2.p);
    PM_HIP_TRY(hipGetLastError());
    PM_HIP_TRY(launch_knn(m, q3.p, nq, k, kKMaxDistance, ids.p, d2.p, md.p, s, c1.p, c2.p));
    PM_HIP_TRY(hipStreamSynchronize(s));   // leader buffers are freed on return
  } else {
    PM_HIP_TRY(launch_knn(m, q3.p, nq, k, kKMaxDistance, ids.p, d2.p, md.p, s, nullptr, nullptr));
  }
  k_radiance_k<<<grid_for(nq, 256), 256, 0, s>>>(qb, perm, nq, k, ids.p, d2.p, md.p, m->payload.p, out);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);   // the lists are freed on return
}

hipError_t launch_gather_api(const pm_photon_map* m, const pm_float3* pts, const float* brdf, int64_t nq,
                             pm_float3* out, hipStream_t s, int k) {
  if (nq <= 0) return hipSuccess;
  DevBuf<float4> qb(nq), ob(nq);
  if (!qb.p || !ob.p) return hipErrorOutOfMemory;
  k_pack_query<<<grid_for(nq, 256), 256, 0, s>>>(pts, brdf, nq, qb.p);
  PM_HIP_TRY(hipGetLastError());
  PM_HIP_TRY(launch_gather_k(m, qb.p, nq, ob.p, s, k, nullptr));
  k_unpack_out<<<grid_for(nq, 256), 256, 0, s>>>(ob.p, nq, out);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

}  // namespace pmd
