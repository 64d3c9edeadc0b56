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
// points meet a tight bound (knn_walk, knn_walk_lean; variants measured: DESIGN.md §4.4).
#include <algorithm>
#include <cmath>

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

// Stack-free walk (pm_knn, and the check variant's gather). A node's own point
// is tested post-order: when the walk comes back from its close child (or at
// once if it has none), so root-path points meet an already tight bound.
//  QL:   > 0 parks candidates in a QL-deep per-lane LIFO queue in LDS (`lq`,
//        this lane's column of a [QL][stride] array); the wave runs one K-wide
//        insert round (every lane with a queued key pops one) only when some
//        lane's queue is full or the walks are over. The pruning bound ignores
//        queued keys, i.e. it is never too tight: still exact.
//  lo:   only keys > lo are candidates (multi-pass k > 128: pass p collects
//        the 128 smallest keys above pass p-1's last; keys are unique).
template <int K, int QL = 0>
__device__ __forceinline__ void knn_walk(const float4* __restrict__ nodes, int n, v3 q, float r2, bool valid,
                                         double (&list)[K], double* lq = nullptr, int lstride = 0, double lo = 0.0) {
  const double sentinel = key_make(r2, 0xFFFFFFFFu);
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  float bound = r2;
  int prev = -1, curr = 0;
  bool walking = valid && n > 0;
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
      if ((down && close_c >= n) || prev == close_c) {
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
      if (ik < list[K - 1]) {
        list_insert<K>(list, ik);
        bound = key_d2(list[K - 1]);
      }
      if (!any_walking && __ballot(qn > 0) == 0) break;
    } else {
      if (cand) {
        list_insert<K>(list, key);
        bound = key_d2(list[K - 1]);
      }
      if (__ballot(walking) == 0) break;
    }
  }
}

// The gather's walk: knn_walk<K, QL> with
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
//  - The kernel is VALU-issue bound (round 2: ~62 VALU per step x ~460 steps
//    plus ~111 per insert round x ~165 rounds per wave account for the whole
//    follower launch at 2.4 GHz), so the step is written for instruction
//    count: a lane arrives at a node either from its parent or from its close
//    child (JUMP never returns from a far child), so one `up` flag replaces
//    the previous-node index; the three transitions are computed branch-free
//    and selected; the node offset is 32-bit (saddr loads) when the map fits.
// Gather keys: (d^2 bits << 32 | node word), the node word being the kd node's
// (orig << 2 | dim) -- orig is unique, so the order is (d^2, orig) as for
// key_make -- held as a double WITHOUT the 2^52 bias: every key is a
// non-negative double (zero, denormal or normal; never -0, inf or NaN), whose
// IEEE order is the integer order because the kernels keep f64 denormals
// (float_denorm_mode_16_64 = 3). No instruction builds a key.
__device__ __forceinline__ double gkey(float d2, uint32_t word) {
  return __longlong_as_double((long long)(((uint64_t)__float_as_uint(d2) << 32) | word));
}
__device__ __forceinline__ float gkey_d2(double k) { return __uint_as_float((uint32_t)((uint64_t)__double_as_longlong(k) >> 32)); }
__device__ __forceinline__ uint32_t gkey_word(double k) { return (uint32_t)__double_as_longlong(k); }
constexpr uint32_t kNoWord = 0xFFFFFFFFu;   // sentinel's low word (never a node word: orig < 2^29)

// Walk state of one lane (knn_walk_lean). Nodes are numbered from 1 here (c1 =
// implicit index + 1: children 2 c1, 2 c1 + 1, parent c1 >> 1).
struct LeanWalk {
  float bound;
  uint32_t c1;
  uint32_t far_mask;   // bit j set <=> ancestor-or-self c1 >> j was entered as its parent's FAR child
  bool up;             // arrived at c1 from its close child: its point test is due
  bool walking;
  int qn;              // queued candidates in this lane's LDS column (slots 1..QL; slot 0 = DBL_MAX)
  // JUMP target of the current state, computed when the state is set (off the
  // node-load critical path): a = c1 >> (j1 - 1) with j1 - 1 the lowest clear
  // bit of far_mask is the deepest close-child ancestor-or-self; upnode = its
  // parent c1 >> j1 (0: a is the root, the walk is over)
  uint32_t j1, upnode;
  __device__ __forceinline__ void set_jump() {
    j1 = __builtin_ctz(~far_mask) + 1;   // far_mask has <= 30 bits: ~far_mask != 0
    upnode = c1 >> j1;
  }
  __device__ __forceinline__ void start(float b, bool valid) {
    bound = b;
    c1 = 1;
    far_mask = 0;   // the root's bit stays 0: a jump that reaches it ends the walk
    up = false;
    walking = valid;
    set_jump();
  }
};

// node c1 (1-based): a 32-bit byte offset (saddr load, -16 folded into the
// instruction) while the map has < 2^28 nodes, 64-bit addressing above
template <bool WIDE>
__device__ __forceinline__ float4 node1(const float4* __restrict__ nodes, uint32_t c1) {
  if (WIDE) return nodes[(size_t)c1 - 1];
  return *(const float4*)((const char*)nodes - 16 + (c1 << 4));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Subtree boxes: the AABB of every point in node c1's subtree, box[2 (c1 - 1)]
// = (lo, _), box[2 (c1 - 1) + 1] = (hi, _), for the nodes c1 <= nbox (the
// levels down to a chosen depth), built per gather call (build_subtree_boxes).
// The plane test alone cannot prune a subtree whose splitting planes run past q
// while all of its points are far away -- a dense caustic patch seen from a
// distant query, whose k nearest lie in a thin shell across the patch, or a
// Cornell-box wall whose photons sit in a plane the query's close-path planes
// cross -- so such walks visited nearly every photon there. A lane that
// arrives at a boxed node from its parent skips the subtree when the box's
// squared distance exceeds its bound. Exact: per dimension the box gap is
// <= |q - p| for every point p inside, and f32 subtraction, squaring and the
// (uncontracted) sum are monotone, so the box distance computed in f32 is <=
// every inside point's computed d^2; a skipped point has d^2 > bound, i.e. a
// key above the lane's tail.
__global__ void k_subtree_box(const float4* __restrict__ nodes, int64_t n, int64_t lo, int64_t hi,
                              float4* __restrict__ box) {
  const int64_t t = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // 0-based node index
  if (t >= hi) return;
  const float4 p = nodes[t];
  float4 a = make_float4(p.x, p.y, p.z, 0.f), b = a;
#pragma unroll
  for (int c = 1; c <= 2; c++) {
    const int64_t ch = 2 * t + c;
    if (ch < n) {
      const float4 cl = box[2 * ch], chh = box[2 * ch + 1];
      a = make_float4(fminf(a.x, cl.x), fminf(a.y, cl.y), fminf(a.z, cl.z), 0.f);
      b = make_float4(fmaxf(b.x, chh.x), fmaxf(b.y, chh.y), fmaxf(b.z, chh.z), 0.f);
    }
  }
  box[2 * t] = a;
  box[2 * t + 1] = b;
}
// the deepest boxed level, from its points directly: node t's subtree holds
// nodes (t + 1) 2^l - 1 + j, j < 2^l, at relative level l (contiguous per level)
__global__ void k_subtree_box_scan(const float4* __restrict__ nodes, int64_t n, int64_t lo, int64_t hi, int levels,
                                   float4* __restrict__ box) {
  const int64_t t = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hi) return;
  float4 a = make_float4(INFINITY, INFINITY, INFINITY, 0.f), b = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
  for (int l = 0; l <= levels; l++) {
    const int64_t f = ((t + 1) << l) - 1, e = std::min<int64_t>(((t + 2) << l) - 1, n);
    for (int64_t j = f; j < e; j++) {
      const float4 p = nodes[j];
      a = make_float4(fminf(a.x, p.x), fminf(a.y, p.y), fminf(a.z, p.z), 0.f);
      b = make_float4(fmaxf(b.x, p.x), fmaxf(b.y, p.y), fmaxf(b.z, p.z), 0.f);
    }
  }
  box[2 * t] = a;
  box[2 * t + 1] = b;
}

// Boxes of levels 0 .. D - skip (D = the deepest level; skip 0: every node).
// Returns the number of boxed nodes (nbox) through *nbox.
static hipError_t build_subtree_boxes(const float4* nodes, int64_t n, int skip, float4* box, int64_t* nbox,
                                      hipStream_t s) {
  *nbox = 0;
  if (n <= 0) return hipSuccess;
  int D = 0;
  while ((int64_t(2) << D) - 1 < n) D++;   // levels 0 .. D (D may be partial)
  int top = D;
  if (skip > 0) {
    top = std::max(D - skip, 0);   // a complete level (< D)
    const int64_t lo = (int64_t(1) << top) - 1, hi = (int64_t(2) << top) - 1;
    k_subtree_box_scan<<<grid_for(hi - lo, 256), 256, 0, s>>>(nodes, n, lo, hi, D - top, box);
    PM_HIP_TRY(hipGetLastError());
    top--;
  }
  for (int d = top; d >= 0; d--) {
    const int64_t lo = (int64_t(1) << d) - 1, hi = std::min<int64_t>((int64_t(2) << d) - 1, n);
    k_subtree_box<<<grid_for(hi - lo, 256), 256, 0, s>>>(nodes, n, lo, hi, box);
    PM_HIP_TRY(hipGetLastError());
  }
  *nbox = skip > 0 ? (int64_t(2) << std::max(D - skip, 0)) - 1 : n;
  return hipSuccess;
}
static int64_t boxed_nodes(int64_t n, int skip) {
  if (n <= 0) return 0;
  int D = 0;
  while ((int64_t(2) << D) - 1 < n) D++;
  return skip > 0 ? (int64_t(2) << std::max(D - skip, 0)) - 1 : n;
}

__device__ __forceinline__ float box_d2(float4 a, float4 b, v3 q) {
  const float gx = fmaxf(fmaxf(a.x - q.x, q.x - b.x), 0.f);
  const float gy = fmaxf(fmaxf(a.y - q.y, q.y - b.y), 0.f);
  const float gz = fmaxf(fmaxf(a.z - q.z, q.z - b.z), 0.f);
  return gx * gx + gy * gy + gz * gz;
}
// the boxes of node c1 (1-based, c1 <= nbox)
template <bool WIDE>
__device__ __forceinline__ const float4* box1(const float4* __restrict__ box, uint32_t c1) {
  (void)WIDE;   // 32-B records: 64-bit offsets from 2^27 nodes on
  return box + 2 * ((size_t)c1 - 1);
}
struct BoxView {
  const float4* box = nullptr;
  uint32_t nbox = 0;   // nodes 1 .. nbox carry a box
};


// One walk step of every lane (finished / idle lanes re-read their last node and
// are masked): the post-order point test queues a candidate, the walk moves on.
// Transitions (all computed, one selected):
//  - descend to the close child (arrived from the parent and it exists);
//  - else enter the far child if it exists and the plane is within the bound;
//  - else JUMP to LeanWalk::upnode (arriving from its close child), or stop
//    when that is 0.
// BOX: a lane arriving at a boxed node from its parent skips the subtree when
// its box lies beyond the bound (finished at once: the walk leaves it as after
// its far child); ba / bb hold node c1's box (stale for unboxed nodes).
template <int K, bool WIDE, bool BOX = false>
__device__ __forceinline__ void lean_step(const float4* __restrict__ nodes, uint32_t n, v3 q, double tail,
                                          LeanWalk& w, float4& nd, double* lq, int lstride, BoxView bx = {},
                                          float4* ba = nullptr, float4* bb = nullptr) {
  // software-pipelined: `nd` (node c1) was loaded by the previous step; the
  // transitions come first, so the next node's load is issued before the point
  // test, the queue write and any insert round of this step
  const uint32_t word = __float_as_uint(nd.w);
  const uint32_t dim = word & 3u;
  const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
  const float diff = dim == 0 ? dx : (dim == 1 ? dy : dz);   // = q[dim] - nd[dim]
  const bool skip = BOX && !w.up && w.c1 <= bx.nbox && box_d2(*ba, *bb, q) > w.bound;
  const uint32_t close1 = 2 * w.c1 + (diff > 0.f ? 1u : 0u), far1 = close1 ^ 1u;
  const bool closeok = close1 <= n;
  const bool test = !skip && (w.up || !closeok);
  const bool descend = !skip && !w.up && closeok;
  const bool farok = !skip && !descend && far1 <= n && diff * diff <= w.bound;
  const bool stay = descend || farok;
  const uint32_t next = descend ? close1 : (farok ? far1 : w.upnode);
  const bool go = w.walking && (stay || w.upnode != 0);
  const uint32_t c1n = go ? next : w.c1;
  const float4 ndn = node1<WIDE>(nodes, c1n);
  if (BOX && c1n <= bx.nbox) {
    const float4* bp = box1<WIDE>(bx.box, c1n);
    *ba = bp[0];
    *bb = bp[1];
  }
  const float d2 = dx * dx + dy * dy + dz * dz;
  const double key = gkey(d2, word);
  const bool cand = w.walking && test && key < tail;
  w.far_mask = stay ? (w.far_mask << 1 | (farok ? 1u : 0u)) : w.far_mask >> w.j1;
  w.up = !stay;
  lq[(w.qn + 1) * lstride] = key;
  w.qn += cand ? 1 : 0;
  w.c1 = c1n;
  w.walking = go;
  w.set_jump();
  nd = ndn;
}

// Wave-uniform insert round: every lane pops one queued key (an empty queue
// reads slot 0, DBL_MAX); list_insert leaves the list unchanged for a key above
// its last entry, so the round needs no per-lane branch.
template <int K>
__device__ __forceinline__ void lean_round(double (&list)[K], LeanWalk& w, const double* lq, int lstride) {
  const double ik = lq[w.qn * lstride];
  w.qn = w.qn > 0 ? w.qn - 1 : 0;
  list_insert<K>(list, ik);
  w.bound = gkey_d2(list[K - 1]);
}

// One phase of the walk: steps (with or without subtree-box skips) until the
// walks and queues are done (returns true) or the wave has run `limit`
// iterations (false). BUDGET > 0: at BUDGET iterations the lanes still walking
// stop and are reported through `aborted`; their lists are incomplete.
template <int K, int QL, bool WIDE, int BUDGET, bool BOX>
__device__ __forceinline__ bool lean_phase(const float4* __restrict__ nodes, uint32_t n, v3 q, double (&list)[K],
                                           double* lq, int lstride, BoxView bx, LeanWalk& w, float4& nd, float4& ba,
                                           float4& bb, int& it, int limit, bool& aborted) {
  for (;;) {
    lean_step<K, WIDE, BOX>(nodes, n, q, list[K - 1], w, nd, lq, lstride, bx, &ba, &bb);
    ++it;
    if (BUDGET > 0 && it == BUDGET) {
      aborted = w.walking;
      w.walking = false;
    }
    const bool any_walking = ballot(w.walking) != 0;
    if (ballot(w.qn == QL) != 0 || !any_walking) {   // wave-uniform insert round
      lean_round<K>(list, w, lq, lstride);
      if (!any_walking && ballot(w.qn > 0) == 0) return true;
    }
    if (it == limit) return false;
  }
}

// BOXAFTER: < 0 plane tests only; >= 0 the walk switches to subtree-box skips
// once the wave has run that many iterations (0: from the start). Box tests
// cost ~14 VALU and a 32-B load per step, which the short walks of a dense map
// do not pay back; the long ones -- a wave that wanders along planar walls or
// a thin shell of a far patch -- are cut short by them.
template <int K, int QL, bool WIDE, int BUDGET = 0, int BOXAFTER = -1>
__device__ __forceinline__ bool knn_walk_lean(const float4* __restrict__ nodes, int n, v3 q, float cut, bool valid,
                                              double (&list)[K], double* lq, int lstride, BoxView bx = {},
                                              int* it_out = nullptr) {
  const double sentinel = gkey(cut, kNoWord);
#pragma unroll
  for (int j = 0; j < K; j++) list[j] = sentinel;
  if (n <= 0) return false;   // empty map: every lane keeps the sentinel list (uniform)
  LeanWalk w;
  w.start(cut, valid);
  w.qn = 0;
  lq[0] = __longlong_as_double(0x7FEFFFFFFFFFFFFFll);   // slot 0: DBL_MAX, never inserted
  float4 nd = node1<WIDE>(nodes, 1);
  float4 ba = {}, bb = {};
  bool aborted = false;
  int it = 0;   // wave-uniform
  bool done = false;
  if (BOXAFTER != 0)
    done = lean_phase<K, QL, WIDE, BUDGET, false>(nodes, (uint32_t)n, q, list, lq, lstride, bx, w, nd, ba, bb, it,
                                                  BOXAFTER, aborted);
  if (BOXAFTER >= 0 && !done) {
    if (w.c1 <= bx.nbox) {   // the current node's box (the skip test reads it next step)
      const float4* bp = box1<WIDE>(bx.box, w.c1);
      ba = bp[0];
      bb = bp[1];
    }
    lean_phase<K, QL, WIDE, BUDGET, true>(nodes, (uint32_t)n, q, list, lq, lstride, bx, w, nd, ba, bb, it, -1,
                                          aborted);
  }
  if (it_out) *it_out = it;
  return aborted;
}

// pm_knn: K-wide list for k <= K; k > 128 runs 128-wide passes (j0 = output
// offset of this pass, lo_in / lo_out = last key of the previous / this pass).
// QL > 0: candidates go through a QL-deep per-lane LDS queue (knn_walk), as in
// the gather; the 128-wide passes of k > 128 use it (config 5, k = 200).
template <int K, int QL = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K <= 64 ? 4 : 1))) void k_knn(
    const float4* nodes, int n, const pm_float3* q, int64_t nq, int k, int j0, float r2, int32_t* ids, float* d2o,
    float* maxd2, const double* lo_in, double* lo_out) {
  __shared__ double lq[QL > 0 ? QL * 256 : 1];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < nq;
  double list[K];
  const pm_float3 p = valid ? q[i] : pm_float3{0.f, 0.f, 0.f};
  const double lo = (valid && lo_in) ? lo_in[i] : 0.0;
  // a previous pass whose list did not fill (last key = the sentinel, id -1)
  // found every candidate: this pass has none to find, its walk is skipped
  const bool done = lo_in && key_id(lo) == 0xFFFFFFFFu;
  knn_walk<K, QL>(nodes, n, mk(p), r2, valid && !done, list, lq + threadIdx.x, 256, lo);
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

// The same over a gather (gkey) list: neighbour id = node word >> 2.
__device__ __forceinline__ v3 radiance_g(const double (&list)[kKNearest], const float4* __restrict__ payload,
                                         float brdf, float r2) {
  v3 flux = {0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < kKNearest; p++) {
    const uint32_t word = gkey_word(list[p]);
    if (word == kNoWord) continue;
    const float4 pl = payload[word >> 2];
    const float dist = sqrtf(gkey_d2(list[p]));
    const float w = 1 - (dist / sqrtf(r2) * kConeFilterC);
    flux = add(flux, smul(brdf * pl.w * w, v3{pl.x, pl.y, pl.z}));
  }
  return divf(flux, (1 - (2.f / 3.f) * (1.f / kConeFilterC)) * 2 * kPI * r2);
}

// Seeded cut-offs (production). Every kSeedStride-th query in walk (Morton)
// order is a LEADER; the first k_gather_level launch runs the leaders with the
// plain cut-off and keeps (position, K-th d^2). The other queries then start
// from a cut-off that provably holds the K nearest: the leader's K points lie
// within sqrt(t') of q', hence within sqrt(t') + |q - q'| of q (triangle
// inequality), so at least K photons have d^2 <= that bound and the K smallest
// keys -- the result -- are all admitted. The bound is the smallest over the
// consulted leaders (the enclosing pair plus one more on each side) and is
// inflated (1e-6 relative per step, 1e-5 on the square, 1e-30 absolute) past
// the rounding of the f32 d^2 on both sides; a leader whose list did not fill
// (t' = -1) seeds nothing. The cut-off only prunes: the visited set shrinks,
// the list and the radiance are bitwise those of the plain walk (the check
// variant library, PM_CHECK_VARIANT, runs the plain knn_walk; tests compare).
// Config 3 global gather (ms), measured in round 1: stride 8 / 2 leaders 50.9,
// 8/4 50.3, 4/2 52.2, 16/2 50.6, 16/4 49.8; leader hierarchies, XCD-contiguous
// block ranges, pooled lanes, child-line prefetch and deeper queues measured
// slower; the exact-cut re-walk floor was 34.4 ms. Round 2,
// with the leader budget: stride 12 / 16 / 20 / 24 / 28 gave config 2
// 24.7-25.9 / 24.9-25.3 / 22.2-22.7 / 25.5-25.7 / 23.6 ms per frame and
// config 3's global gather 41.3-41.4 / 40.8-41.0 / 40.6-40.9 / 41.1-41.3 /
// 40.8 ms: 20.
#ifndef PM_SEED_STRIDE
#define PM_SEED_STRIDE 20
#endif
#ifndef PM_SEED_LEADERS
#define PM_SEED_LEADERS 4
#endif
#ifndef PM_GATHER_QL
#define PM_GATHER_QL 8
#endif
constexpr int kSeedStride = PM_SEED_STRIDE;
// Leader groups (k = 50 gather): walk ranks are dealt in blocks of G * S and the
// first G ranks of each block lead, so a leader wave's lanes come in runs of G
// neighbours that share cache lines (G = 1: every S-th rank; the wide gather
// keeps G = 1). Followers consult the two leaders before and the two after them.
// Measured (round 5, config 3's global gather): G = 1 / 4 / 8 / 16 41.4-41.5 /
// 42.9-43.0 / 43.6-43.9 / 44.5 ms; at G = 8 the leader launch 5.95 -> 5.06 ms,
// the followers 35.4 -> 38.6 ms (their seeds come from farther away): 1.
#ifndef PM_SEED_GROUP
#define PM_SEED_GROUP 1
#endif
constexpr int kSeedGroup = PM_SEED_GROUP;
template <int G>
struct Seeds {
  static constexpr int64_t GS = (int64_t)G * kSeedStride;
  static_assert(G >= 1 && kSeedStride >= 2, "a block holds G leaders and at least one follower each");
  __host__ __device__ static int64_t count(int64_t nq) { return (nq / GS) * G + (nq % GS < G ? nq % GS : G); }
  __device__ static int64_t leader_rank(int64_t l) { return (l / G) * GS + l % G; }
  __device__ static int64_t follower_rank(int64_t t) { return (t / (GS - G)) * GS + G + t % (GS - G); }
  __device__ static int64_t index(int64_t r) { return (r / GS) * G + r % GS; }   // r: a leader's rank
  __device__ static int64_t before(int64_t r) { return (r / GS) * G + G - 1; }   // r: a follower's rank
};
constexpr int kSeedLeaders = PM_SEED_LEADERS;
constexpr int kGatherQL = PM_GATHER_QL;   // LDS insert-queue depth
// Leader step budget (wave iterations; 0: none). A leader wave ends when its
// lanes are done or after this many iterations; a lane still walking then
// (on the Cornell box, depth-first walks that wander through planar walls:
// up to ~78k steps, while most leader waves need a few hundred) writes no seed
// record and is re-walked, without a budget, by the first workgroups of the
// follower launch -- beside the followers instead of
// before them. Results are unchanged (a cut-off only prunes; the retry walk
// is the leader walk). The retry workgroups come first in the launch, so the
// long walks start before (and overlap) the follower workgroups. Budget 1024 /
// 2048 / 4096 / 8192: config 2 24.8 / 24.8-25.1 / 25.5 / 26.5 ms per frame,
// config 3's global gather 41.1-41.3 / 40.7 / 40.7 / 40.7 ms.
#ifndef PM_LEADER_BUDGET
#define PM_LEADER_BUDGET 2048
#endif
constexpr int kLeaderBudget = PM_LEADER_BUDGET;
// 1: a leader cut off by the budget with a full list records its list's last
// d^2 as its seed (followers and its own retry start from it); 0: no seed
#ifndef PM_LEADER_SOFT
#define PM_LEADER_SOFT 1
#endif
constexpr bool kLeaderSoft = PM_LEADER_SOFT;
// Subtree-box skips in the k = 50 gather: 0 none, 1 leaders and retried
// leaders, 2 every walk, 3 every walk but the budgeted leaders' (whose long
// walks the retry workgroups redo with boxes; the leader launch keeps 4
// waves/SIMD); boxes down to level D - PM_GATHER_BOX_SKIP (0: all).
// Each walk switches to them after PM_BOX_AFTER wave iterations (knn_walk_lean).
// Measured (round 3, ms per frame, config 2 / config 3): none 21.4 / 108.7;
// every walk from the start 9.8 / 122.9 (config 3's global gather 41.6 ->
// 55.8 ms: -24 % iterations but ~+14 VALU and a 32-B load per step); leaders
// and retries only 15.9 / 111.0; boxes of the top levels only (skip 6) 10.5 /
// 114.6; every walk after 256 / 512 / 1024 iterations 9.05 / 9.19 / 9.15 and
// 111.7 / 108.8 / 108.5: 512 (config 2's global gather 16.3 -> 4.3 ms: the
// long Cornell walks along the box walls end, config 3's walks mostly finish
// before the switch).
// Round 3, every walk after 512 vs every walk but the leaders' (mode 3, kept):
// config 3 109.2 / 108.9 vs 107.8 / 108.4 ms (the leader launch keeps 4
// waves/SIMD instead of 3), config 2 9.01 vs 9.07 ms.
#ifndef PM_GATHER_BOX
#define PM_GATHER_BOX 3
#endif
#ifndef PM_GATHER_BOX_SKIP
#define PM_GATHER_BOX_SKIP 3
#endif
constexpr int kGatherBox = PM_GATHER_BOX;
// 1 (test variant): 64-bit node addressing for every map, so the path that
// maps of >= 2^28 nodes take runs on the small parity workloads
#ifndef PM_FORCE_WIDE
#define PM_FORCE_WIDE 0
#endif
#ifndef PM_BOX_AFTER
#define PM_BOX_AFTER 512
#endif
constexpr int kBoxAfter = PM_BOX_AFTER;

// Guessed follower cut-offs (round 6, PM_SEED_GUESS). The K-th nearest
// distance r(x) is 1-Lipschitz, so r_f <= r_L + d (d = |f - L|) holds for a
// follower f and any leader L: seed_bound. It is loose wherever the density
// varies slowly, which is almost everywhere: a follower walks with the tighter
// GUESS min(r_L + d, r_L (1 + beta) + alpha d) instead. A follower whose list
// does not fill under a guess (fewer than K photons inside it) flags its walk
// rank; k_gather_fmark lists the flags and k_gather_fretry re-walks them with
// the guaranteed (or own-subtree, if tighter) cut-off after the follower
// launch, overwriting their slots. A list that does fill holds
// the K nearest (every point inside the cut-off was visited), the same keys
// the guaranteed walk finds, so every result is bitwise the production one.
// Config 3 (profiles/r06/r06k_seed_guess_*): the misses of alpha / beta
// 0.5 / 0.1: 0.009 %, 0.25 / 0.1: 0.33 %, 0 / 0.3: 3 %, 0 / 0.2: 10 %; with
// the retries, the global gather 40.3 ms (guaranteed only) -> 37.1 (0.25 /
// 0.1), 36.8 (0.25 / 0.075), 37.1 (0.2 / 0.075, 0.25 / 0.05), 37.5 (0.3 /
// 0.025), 38.6-39.3 (0.15 / 0.05), 47.0 (0 / 0.3): a retried walk costs ~10
// follower walks (it runs nearly alone: the retries are scattered).
#ifndef PM_SEED_GUESS
#define PM_SEED_GUESS 1
#endif
#ifndef PM_SEED_GUESS_ALPHA
#define PM_SEED_GUESS_ALPHA 0.25
#endif
#ifndef PM_SEED_GUESS_BETA
#define PM_SEED_GUESS_BETA 0.075
#endif
// Follower launches of fewer walks guess nothing: the retry launch costs about
// one walk's latency (~0.7-1 ms) whatever the misses, more than the guess saves
// on a short launch (config 2, 3.7 M queries: global gather 4.2 -> 5.3 ms with
// guesses; config 3, 36 M: 40.3 -> 36.8; config 5, 45 M: 49.2 -> 46.8-47.9)
#ifndef PM_SEED_GUESS_MIN
#define PM_SEED_GUESS_MIN (1 << 23)
#endif
constexpr bool kSeedGuess = PM_SEED_GUESS;
constexpr int64_t kSeedGuessMin = PM_SEED_GUESS_MIN;
__device__ __forceinline__ double seed_sq(double c) { return c * c * (1.0 + 1e-5) + 1e-30; }
// (guaranteed, guessed) squared bounds of follower q from one leader record
__device__ __forceinline__ void seed_bounds(float4 lead, v3 q, double& guar, double& guess) {
  if (!(lead.w >= 0.f)) {
    guar = guess = 1e300;
    return;
  }
  const double dx = (double)q.x - lead.x, dy = (double)q.y - lead.y, dz = (double)q.z - lead.z;
  const double rl = sqrt((double)lead.w), dl = sqrt(dx * dx + dy * dy + dz * dz);
  const double c = rl + dl;
  guar = seed_sq(c * (1.0 + 1e-6));
  guess = seed_sq(fmin(c, rl * (1.0 + PM_SEED_GUESS_BETA) + PM_SEED_GUESS_ALPHA * dl) * (1.0 + 1e-6));
}
__device__ __forceinline__ double seed_bound(float4 lead, v3 q) {
  double g, e;
  seed_bounds(lead, q, g, e);
  return g;
}
// f32 cut-off >= bound (rounded up), capped at the plain cut-off
__device__ __forceinline__ float seed_cut(double bound, float r2) {
  const float plain = lean_cut(r2);
  if (!(bound < (double)plain)) return plain;
  float f = (float)bound;
  if ((double)f < bound) f = __uint_as_float(__float_as_uint(f) + 1u);
  return fminf(f, plain);
}

// cut-off of walk rank r (a follower) from the leaders' records: the
// guaranteed one, and in *guess (kSeedGuess) the guessed one (<= guaranteed)
template <int G>
__device__ __forceinline__ float follower_cut(const float4* __restrict__ lead, int64_t nq, int64_t r, v3 q,
                                              float R2, float* guess = nullptr) {
  const int64_t jp = Seeds<G>::before(r), ns = Seeds<G>::count(nq);
  double b, e;
  seed_bounds(lead[jp], q, b, e);
  auto more = [&](int64_t j) {
    double b1, e1;
    seed_bounds(lead[j], q, b1, e1);
    b = fmin(b, b1);
    e = fmin(e, e1);
  };
  if (jp + 1 < ns) more(jp + 1);
  if (kSeedLeaders > 2) {
    if (jp >= 1) more(jp - 1);
    if (jp + 2 < ns) more(jp + 2);
  }
  if (guess) *guess = seed_cut(e, R2);
  return seed_cut(b, R2);
}

// Leader cut-off from the leader's own kd subtree. The six complete levels
// under the depth-(D - 6) node on q's close path (D = the deepest, possibly
// partial level) hold 63 photons, so their 50th-smallest d^2 -- the 14th
// largest, kept in a descending v_med3 list -- bounds the K-th nearest d^2:
// at least 50 photons lie within it. d^2 is computed exactly as the walk does,
// so the bound admits them; it only prunes (results stay those of the plain
// walk). Without it a leader whose neighbourhood is sparse walks under the
// plain 100-unit radius until its list fills: on the Cornell box (config 2)
// some leader walks ran tens of thousands of steps and the under-filled
// leader launch (231k queries) took 16.8 ms.
constexpr int kSubtreeLevels = 6;   // 63 nodes
constexpr int kSubtreeTop = (1 << kSubtreeLevels) - 1 - (kKNearest - 1);   // 14: rank 50 of 63 from the top
template <bool WIDE>
__device__ __forceinline__ float subtree_cut(const float4* __restrict__ nodes, uint32_t n, v3 q, float plain) {
  const int D = 31 - __clz(n);   // deepest level (0-based): levels 0 .. D - 1 are complete
  const int dz = D - kSubtreeLevels;
  if (dz < 0) return plain;
  uint32_t c1 = 1;
  for (int d = 0; d < dz; d++) {   // close path
    const float4 nd = node1<WIDE>(nodes, c1);
    const uint32_t dim = __float_as_uint(nd.w) & 3u;
    const float diff = dim == 0 ? q.x - nd.x : (dim == 1 ? q.y - nd.y : q.z - nd.z);
    c1 = 2 * c1 + (diff > 0.f ? 1u : 0u);
  }
  float top[kSubtreeTop];   // descending
#pragma unroll
  for (int j = 0; j < kSubtreeTop; j++) top[j] = -1.f;
#pragma unroll
  for (int l = 0; l < kSubtreeLevels; l++) {
#pragma unroll 4
    for (uint32_t k = 0; k < (1u << l); k++) {
      const float4 nd = node1<WIDE>(nodes, (c1 << l) + k);
      const float dx = q.x - nd.x, dy = q.y - nd.y, dz2 = q.z - nd.z;
      const float d2 = dx * dx + dy * dy + dz2 * dz2;
#pragma unroll
      for (int j = kSubtreeTop - 1; j > 0; j--) top[j] = __builtin_amdgcn_fmed3f(top[j - 1], top[j], d2);
      top[0] = fmaxf(top[0], d2);
    }
  }
  return fminf(top[kSubtreeTop - 1], plain);
}

// One level of the seeded gather. LEADERS: walk ranks 0, S, 2S, ... with the
// plain cut-off, recording (position, K-th d^2) in lead[Seeds::index(r)]; followers:
// every other rank (thread t -> rank (t / (S-1)) * S + 1 + t % (S-1)), cut-off
// from the leaders. TAG only separates the global-map launches into their own
// kernel symbol (rocprof). perm: lane of walk rank r takes query perm[r] and
// writes its result there (Morton walk order without permuted copies).
// Windowed XCD swizzle of the walk order (PM_GATHER_XCD_K = k > 0): blocks are
// dealt round-robin over the 8 XCDs, so block b's XCD label is b % 8; inside
// every window of 8k consecutive blocks the k blocks that share a label take
// k consecutive 256-rank pieces of the window's walk range. The GPU still
// works on one coherent frontier of the walk order (round 6: giving each XCD
// a whole eighth of the order instead was 49.8 vs 41.0 ms), but each XCD's L2
// serves a compact eighth of it. f: the block's index among the launch's
// walk blocks, bid: its grid index (the label). The tail window keeps f.
// Config 3's global gather (ms, alternating runs, profiles/r06/r06e_*):
// k = 0 (the plain order) 41.1-41.4, 4 40.7-40.9, 8 40.2-40.5, 16 39.9-40.3,
// 32 39.9-40.2, 128 40.2-40.4; config 2's 4.27-4.38 / 4.27 / 4.17-4.26 /
// 4.24-4.34 / 4.15-4.25 / 4.51: 32.
#ifndef PM_GATHER_XCD_K
#define PM_GATHER_XCD_K 32
#endif
#ifndef PM_GATHER_XCD_KL   // the leader launch's (its blocks span 20x the walk ranks)
#define PM_GATHER_XCD_KL PM_GATHER_XCD_K
#endif
template <uint32_t K>
__device__ __forceinline__ uint32_t xcd_window_block(uint32_t f, uint32_t bid) {
  if constexpr (K == 0) {
    (void)bid;
    return f;
  } else {
    constexpr uint32_t W = 8 * K;
    const uint32_t nb = gridDim.x - (bid - f);   // the launch's walk blocks
    if (f >= nb - nb % W) return f;              // tail window: as is
    const uint32_t w0 = f - f % W;
    return w0 + (bid % 8u) * K + (f % W) / 8u;
  }
}

template <int TAG, bool LEADERS, bool WIDE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LEADERS && (kGatherBox == 1 || kGatherBox == 2) ? 3 : 4))) void k_gather_level(
    const float4* __restrict__ nodes, const float4* __restrict__ payload, int n, const float4* __restrict__ qb,
    int64_t nq, float4* __restrict__ out, const uint32_t* __restrict__ perm, float4* __restrict__ lead,
    uint32_t* __restrict__ retry, uint32_t* __restrict__ nretry, int retry_blocks, BoxView bx, int64_t t1,
    uint8_t* __restrict__ missed) {
  // lanes [0, t1): leader index (rank t S) or follower index
  // + one slot per lane: a follower walking under a guessed cut-off parks its
  // guaranteed cut-off (low word) and walk rank (high word) there, off the
  // VGPRs the walk needs (~0: not guessed)
  __shared__ double lq[(kGatherQL + 2) * 256];
  uint64_t* const park = reinterpret_cast<uint64_t*>(lq + threadIdx.x + (kGatherQL + 1) * 256);
  const bool guessing = !LEADERS && kSeedGuess && missed;
  if (guessing) *park = ~0ull;
  const float R2 = kKMaxDistance * kKMaxDistance;
  // follower launch with a leader budget: the first nretry_blocks workgroups
  // (one lane per leader) re-walk the leaders that ran out of budget, with the
  // leaders' own cut-off; the walk and the epilogue are shared
  const int64_t nrb = (!LEADERS && nretry) ? (int64_t)retry_blocks : 0;
  const uint32_t bid = blockIdx.x;
  const bool redo_lane = (int64_t)bid < nrb;
  int64_t r;
  bool valid;
  if (redo_lane) {
    const uint32_t e = bid * 256u + threadIdx.x;
    valid = e < *nretry;
    r = valid ? (int64_t)retry[e] : 0;
  } else {
    const int64_t t =
        (int64_t)xcd_window_block<LEADERS ? PM_GATHER_XCD_KL : PM_GATHER_XCD_K>(bid - (uint32_t)nrb, bid) * blockDim.x +
        threadIdx.x;
    r = LEADERS ? Seeds<kSeedGroup>::leader_rank(t) : Seeds<kSeedGroup>::follower_rank(t);
    valid = t < t1 && r < nq;
  }
  if (redo_lane && ballot(valid) == 0) return;   // wave-uniform: no retry entry for this wave
  const int64_t i = !valid ? 0 : (perm ? (int64_t)perm[r] : r);
  const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const v3 q = {qq.x, qq.y, qq.z};
  float cut = lean_cut(R2);
  if (valid) {
    if (LEADERS || redo_lane) {
      cut = subtree_cut<WIDE>(nodes, (uint32_t)n, q, cut);
      // a retried leader whose list was full when its budget ran out recorded
      // that list's last d^2: its 50 points lie within it, so it bounds the
      // 50th nearest (and admits it: only d^2 <= cut are candidates)
      if (redo_lane && kLeaderSoft) {
        const float t = lead[Seeds<kSeedGroup>::index(r)].w;
        if (t >= 0.f) cut = fminf(cut, t);
      }
    } else if (guessing) {
      float g;
      const float gc = follower_cut<kSeedGroup>(lead, nq, r, q, R2, &g);
      cut = g;
      if (g < gc) *park = (uint64_t)(uint32_t)r << 32 | __float_as_uint(gc);
    } else {
      cut = follower_cut<kSeedGroup>(lead, nq, r, q, R2);
    }
  }
  double list[kKNearest];
  bool aborted;
  int* const itp = nullptr;
  if (kGatherBox == 2 || (kGatherBox == 1 && LEADERS) || (kGatherBox == 3 && !LEADERS)) {
    aborted = knn_walk_lean<kKNearest, kGatherQL, WIDE, LEADERS ? kLeaderBudget : 0, kBoxAfter>(
        nodes, n, q, cut, valid, list, lq + threadIdx.x, 256, bx, itp);
  } else if (kGatherBox == 1 && redo_lane) {   // block-uniform: the retried leaders
    aborted = knn_walk_lean<kKNearest, kGatherQL, WIDE, 0, kBoxAfter>(nodes, n, q, cut, valid, list,
                                                                      lq + threadIdx.x, 256, bx, itp);
  } else {
    aborted = knn_walk_lean<kKNearest, kGatherQL, WIDE, LEADERS ? kLeaderBudget : 0>(nodes, n, q, cut, valid, list,
                                                                                     lq + threadIdx.x, 256, {}, itp);
  }
  if (valid && !aborted) {
    const bool full = gkey_word(list[kKNearest - 1]) != kNoWord;
    const v3 f = radiance_g(list, payload, qq.w, full ? gkey_d2(list[kKNearest - 1]) : R2);
    out[i] = make_float4(f.x, f.y, f.z, 0.f);
    // a guessed cut-off that held fewer than K photons: flagged by walk rank;
    // k_gather_fmark lists the flags in walk order, k_gather_fretry re-walks
    // them with the guaranteed cut-off and overwrites their slots
    if (guessing && !full) {
      const uint64_t pk = *park;
      if (pk != ~0ull) missed[pk >> 32] = 1;
    }
    if (LEADERS) lead[Seeds<kSeedGroup>::index(r)] = make_float4(qq.x, qq.y, qq.z, full ? gkey_d2(list[kKNearest - 1]) : -1.f);
  }
  if (LEADERS && kLeaderBudget > 0) {
    const bool redo = valid && aborted;
    // a cut-off walk's full list still bounds the 50th nearest (any 50 points
    // do): its last d^2 seeds the followers and the retry; not full: nothing
    const bool part_full = kLeaderSoft && gkey_word(list[kKNearest - 1]) != kNoWord;
    if (redo) lead[Seeds<kSeedGroup>::index(r)] = make_float4(qq.x, qq.y, qq.z, part_full ? gkey_d2(list[kKNearest - 1]) : -1.f);
    const uint64_t m = ballot(redo);
    if (m != 0) {   // wave-aggregated append to the retry list
      const int lane = threadIdx.x & 63, first = __ffsll((long long)m) - 1;
      uint32_t base = 0;
      if (lane == first) base = atomicAdd(nretry, (uint32_t)__popcll(m));
      base = __shfl(base, first);
      if (redo) retry[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint32_t)r;
    }
  }
}

// The follower retry list (kSeedGuess), in walk order: the walk ranks whose
// miss flag the follower launch set. A block takes 16,384 consecutive flags
// (64 per thread, four 16-B loads), counts them, reserves its range with ONE
// atomic and writes its ranks there in order (one atomic per wave cost 0.4 ms:
// ~10^5 misses on one address). The list fills `retry` downwards from entry
// nq - 1 (the leaders' budget retries use it upwards from 0: at most
// nl + nf = nq entries), counted in nretry[1].
constexpr int kMarkPer = 64;   // flags per thread
__global__ __launch_bounds__(256) void k_gather_fmark(const uint8_t* __restrict__ missed, int64_t nq,
                                                      uint32_t* __restrict__ retry, uint32_t* __restrict__ nretry) {
  __shared__ uint32_t wtot[4];
  __shared__ uint32_t sbase;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t r0 = (int64_t)blockIdx.x * 256 * kMarkPer; r0 < nq; r0 += (int64_t)gridDim.x * 256 * kMarkPer) {
    const int64_t rb = r0 + (int64_t)threadIdx.x * kMarkPer;
    uint4 f[kMarkPer / 16];
#pragma unroll
    for (int k = 0; k < kMarkPer / 16; k++) {
      const int64_t p = rb + 16 * k;
      if (p + 16 <= nq) {
        f[k] = *reinterpret_cast<const uint4*>(missed + p);
      } else {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int j = 0; j < 16; j++)
          if (p + j < nq) w[j >> 2] |= (uint32_t)missed[p + j] << (8 * (j & 3));
        f[k] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    uint32_t c = 0;   // flags are 0 / 1 bytes
#pragma unroll
    for (int k = 0; k < kMarkPer / 16; k++) c += __popc(f[k].x) + __popc(f[k].y) + __popc(f[k].z) + __popc(f[k].w);
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t up = __shfl_up(inc, o);
      if (lane >= o) inc += up;
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int w = 0; w < 4; w++) {
      before += w < wave ? wtot[w] : 0u;
      total += wtot[w];
    }
    if (threadIdx.x == 0 && total) sbase = atomicAdd(nretry + 1, total);
    __syncthreads();
    if (c) {
      int64_t o = (int64_t)sbase + before + inc - c;
#pragma unroll
      for (int k = 0; k < kMarkPer / 16; k++) {
        const uint32_t w4[4] = {f[k].x, f[k].y, f[k].z, f[k].w};
        for (int j = 0; j < 16; j++)
          if ((w4[j >> 2] >> (8 * (j & 3))) & 0xFFu) retry[nq - 1 - o++] = (uint32_t)(rb + 16 * k + j);
      }
    }
    __syncthreads();   // wtot / sbase reused by the next chunk
  }
}

// The follower retries (kSeedGuess): every follower whose guessed cut-off held
// fewer than K photons, re-walked with its guaranteed cut-off exactly as the
// follower launch would have (same cut-off, walk and epilogue). A fixed grid
// strides over the list, whose length only the device knows; every wave leaves
// once the block's next chunk starts past it.
template <int TAG, bool WIDE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gather_fretry(
    const float4* __restrict__ nodes, const float4* __restrict__ payload, int n, const float4* __restrict__ qb,
    int64_t nq, float4* __restrict__ out, const uint32_t* __restrict__ perm, const float4* __restrict__ lead,
    const uint32_t* __restrict__ fretry, const uint32_t* __restrict__ nfretry, BoxView bx) {
  __shared__ double lq[(kGatherQL + 1) * 256];
  const float R2 = kKMaxDistance * kKMaxDistance;
  const uint32_t cnt = *nfretry;
  for (uint32_t base = blockIdx.x * 256u; base < cnt; base += gridDim.x * 256u) {
    const uint32_t e = base + threadIdx.x;
    const bool valid = e < cnt;
    const int64_t r = valid ? (int64_t)fretry[-(int64_t)e] : 0;
    const int64_t i = !valid ? 0 : (perm ? (int64_t)perm[r] : r);
    const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const v3 q = {qq.x, qq.y, qq.z};
    // the guaranteed cut-off, or the own-subtree one where tighter (both hold
    // the K nearest: the walk's result is the same)
    float cut = lean_cut(R2);
    if (valid) cut = fminf(follower_cut<kSeedGroup>(lead, nq, r, q, R2), subtree_cut<WIDE>(nodes, (uint32_t)n, q, cut));
    double list[kKNearest];
    if (kGatherBox == 2 || kGatherBox == 3)
      knn_walk_lean<kKNearest, kGatherQL, WIDE, 0, kBoxAfter>(nodes, n, q, cut, valid, list, lq + threadIdx.x, 256,
                                                              bx, nullptr);
    else
      knn_walk_lean<kKNearest, kGatherQL, WIDE, 0>(nodes, n, q, cut, valid, list, lq + threadIdx.x, 256, {}, nullptr);
    if (valid) {
      const bool full = gkey_word(list[kKNearest - 1]) != kNoWord;
      const v3 f = radiance_g(list, payload, qq.w, full ? gkey_d2(list[kKNearest - 1]) : R2);
      out[i] = make_float4(f.x, f.y, f.z, 0.f);
    }
  }
}

// Check variant (PM_CHECK_VARIANT): the plain post-order walk with the 8-deep
// LDS queue, every query with the plain cut-off (no leaders, no JUMP, no lean
// step): independent code for the same exact lists.
template <int TAG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gather_plain(
    const float4* __restrict__ nodes, const float4* __restrict__ payload, int n, const float4* __restrict__ qb,
    int64_t nq, float4* __restrict__ out, const uint32_t* __restrict__ perm) {
  __shared__ double lq[kGatherQL * 256];
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = r < nq;
  const int64_t i = !valid ? 0 : (perm ? (int64_t)perm[r] : r);
  const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float R2 = kKMaxDistance * kKMaxDistance;
  double list[kKNearest];
  knn_walk<kKNearest, kGatherQL>(nodes, n, v3{qq.x, qq.y, qq.z}, R2, valid, list, lq + threadIdx.x, 256);
  if (valid) {
    const v3 f = radiance(list, payload, qq.w, key_d2(list[kKNearest - 1]));
    out[i] = make_float4(f.x, f.y, f.z, 0.f);
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
#define PM_KNN_CASE(KK)                                                                                 \
  if (k <= KK) {                                                                                        \
    k_knn<KK><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, 0, r2, ids, d2, maxd2, nullptr, nullptr);      \
    return hipGetLastError();                                                                           \
  }
  PM_KNN_CASE(8)
  PM_KNN_CASE(16)
  PM_KNN_CASE(32)
  PM_KNN_CASE(50)
  PM_KNN_CASE(64)
  PM_KNN_CASE(128)
#undef PM_KNN_CASE
  if (k > 256) return hipErrorInvalidValue;
  // 128 < k <= 256: exact 128-wide passes (256 VGPRs, 2 waves/SIMD; 64-wide
  // passes at 4 waves/SIMD measured slower: config 5 gather 261 vs 195 ms), each
  // collecting the 128 smallest keys above the previous pass's last
  constexpr int W = 128;
  DevBuf<double> la(nq), lb(nq);
  if (!la.p || !lb.p) return hipErrorOutOfMemory;
  double *lin = nullptr, *lout = la.p;
  for (int j0 = 0; j0 < k; j0 += W) {
    double* lo_out = j0 + W < k ? lout : nullptr;
    k_knn<W, 8><<<g, 256, 0, s>>>(m->nodes.p, n, q, nq, k, j0, r2, ids, d2, maxd2, lin, lo_out);
    PM_HIP_TRY(hipGetLastError());
    lin = lout;
    lout = lout == la.p ? lb.p : la.p;
  }
  return hipStreamSynchronize(s);   // the pass bounds are freed on return
}

hipError_t launch_gather(const pm_photon_map* m, const float4* qb, int64_t nq, float4* out, hipStream_t s,
                         int tag, const uint32_t* perm) {
  if (nq <= 0) return hipSuccess;
  const int n = (int)m->n;
#if PM_CHECK_VARIANT
  const int g = grid_for(nq, 256);
  if (tag == 1) k_gather_plain<1><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm);
  else k_gather_plain<0><<<g, 256, 0, s>>>(m->nodes.p, m->payload.p, n, qb, nq, out, perm);
  return hipGetLastError();
#else
  const int64_t nl = Seeds<kSeedGroup>::count(nq);   // leaders: walk ranks 0, S, 2S, ... (G = 1)
  DevBuf<float4> lead(nl);
  const int64_t nf = nq - nl;
  // retry lists: the leaders cut off by their budget (upwards from entry 0,
  // count nretry[0] <= nl), the followers whose guessed cut-off missed
  // (kSeedGuess; downwards from entry nq - 1, count nretry[1] <= nq - nl)
  const bool guess = kSeedGuess && nf > 0 && nf >= kSeedGuessMin;
  const bool lists = kLeaderBudget > 0 || guess;
  DevBuf<uint32_t> retry(lists ? (guess ? nq : nl) : 0), nretry(lists ? 2 : 0);
  if (!lead.p || (lists && (!retry.p || !nretry.p))) return hipErrorOutOfMemory;
  if (lists) PM_HIP_TRY(hipMemsetAsync(nretry.p, 0, 2 * sizeof(uint32_t), s));
  DevBuf<uint8_t> missed(guess ? (size_t)nq + 4 : 0);   // follower miss flags by walk rank
  if (guess) {
    if (!missed.p) return hipErrorOutOfMemory;
    PM_HIP_TRY(hipMemsetAsync(missed.p, 0, (size_t)nq + 4, s));
  }
  DevBuf<float4> box(kGatherBox ? 2 * (size_t)std::max<int64_t>(boxed_nodes(n, PM_GATHER_BOX_SKIP), 1) : 0);
  BoxView bx;
  hipEvent_t box_done = nullptr;
  if (kGatherBox) {
    if (!box.p) return hipErrorOutOfMemory;
    int64_t nbox = 0;
    // mode 3: the leader launch reads no box, so the boxes are built beside it
    // on a side stream (config 3: 43 small launches, ~0.9 ms); the follower
    // launch waits for them. The buffer goes back to s's pool when this call
    // returns; s's next use of it comes after the follower launch, which
    // waits for the build.
    hipStream_t bs = kGatherBox == 3 ? side_stream(stream_device(s), 1) : nullptr;
    hipEvent_t nodes_ready = nullptr;
    if (bs && (hipEventCreateWithFlags(&nodes_ready, hipEventDisableTiming) != hipSuccess ||
               hipEventCreateWithFlags(&box_done, hipEventDisableTiming) != hipSuccess)) {
      (void)hipGetLastError();
      if (nodes_ready) (void)hipEventDestroy(nodes_ready);
      nodes_ready = box_done = nullptr;
      bs = nullptr;
    }
    hipError_t e = hipSuccess;
    if (bs) {
      e = hipEventRecord(nodes_ready, s);
      if (e == hipSuccess) e = hipStreamWaitEvent(bs, nodes_ready, 0);
      if (e == hipSuccess) e = build_subtree_boxes(m->nodes.p, n, PM_GATHER_BOX_SKIP, box.p, &nbox, bs);
      if (e == hipSuccess) e = hipEventRecord(box_done, bs);
      (void)hipEventDestroy(nodes_ready);
      if (e != hipSuccess) {
        (void)hipStreamSynchronize(bs);   // nothing on the side stream outlives a failed call
        (void)hipEventDestroy(box_done);
        return e;
      }
    } else {
      PM_HIP_TRY(build_subtree_boxes(m->nodes.p, n, PM_GATHER_BOX_SKIP, box.p, &nbox, s));
    }
    bx.box = box.p;
    bx.nbox = (uint32_t)nbox;
  }
  // an early return still leaves s waiting for the build before the buffer
  // goes back to s's pool (the guard is destroyed before `box`)
  struct BoxWait {
    hipStream_t s;
    hipEvent_t& e;
    ~BoxWait() {
      if (e) {
        (void)hipStreamWaitEvent(s, e, 0);
        (void)hipEventDestroy(e);
      }
    }
  } box_wait{s, box_done};
  // the follower launch (and anything after it on s) waits for the boxes
  auto boxes_ready = [&]() -> hipError_t {
    if (!box_done) return hipSuccess;
    const hipError_t e = hipStreamWaitEvent(s, box_done, 0);
    (void)hipEventDestroy(box_done);
    box_done = nullptr;
    return e;
  };
  // node byte offsets fit 32 bits below 2^28 nodes (saddr loads); larger maps use 64-bit addresses
  const bool wide = PM_FORCE_WIDE || n >= (1 << 28);
  uint32_t* const rt = lists ? retry.p : nullptr;
  uint32_t* const nrt = lists ? nretry.p : nullptr;
  // one launch of k_gather_level<tag, LEADERS, wide> over lanes [0, t1)
  auto level = [&](auto leaders, int grid, int rb, int64_t t1) -> hipError_t {
    constexpr bool L = decltype(leaders)::value;
    if (grid <= 0) return hipSuccess;
    const float4 *nd = m->nodes.p, *pl = m->payload.p;
    if (tag == 1 && wide)
      k_gather_level<1, L, true><<<grid, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, rt, nrt, rb, bx, t1, missed.p);
    else if (tag == 1)
      k_gather_level<1, L, false><<<grid, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, rt, nrt, rb, bx, t1, missed.p);
    else if (wide)
      k_gather_level<0, L, true><<<grid, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, rt, nrt, rb, bx, t1, missed.p);
    else
      k_gather_level<0, L, false><<<grid, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, rt, nrt, rb, bx, t1, missed.p);
    return hipGetLastError();
  };
  // leaders (walk ranks 0, S, 2S, ...), then the followers with the retry
  // workgroups first (one lane per leader, with a leader budget)
  PM_HIP_TRY(level(std::true_type{}, grid_for(nl, 256), 0, nl));
  PM_HIP_TRY(boxes_ready());
  const int rb = kLeaderBudget > 0 ? grid_for(nl, 256) : 0;
  if (nf > 0 || kLeaderBudget > 0) PM_HIP_TRY(level(std::false_type{}, grid_for(nf, 256) + rb, rb, nf));
  if (guess) {   // the guessed cut-offs that missed, re-walked with the guaranteed ones
    k_gather_fmark<<<(int)std::min<int64_t>(grid_for(nq, 256 * kMarkPer), 2048), 256, 0, s>>>(missed.p, nq, retry.p,
                                                                                           nretry.p);
    PM_HIP_TRY(hipGetLastError());
    const int g = (int)std::min<int64_t>(grid_for(nf, 256), 1024);
    const float4 *nd = m->nodes.p, *pl = m->payload.p;
    const uint32_t *fr = retry.p + nq - 1, *nfr = nretry.p + 1;   // the list runs downwards from fr
    if (tag == 1 && wide) k_gather_fretry<1, true><<<g, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, fr, nfr, bx);
    else if (tag == 1) k_gather_fretry<1, false><<<g, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, fr, nfr, bx);
    else if (wide) k_gather_fretry<0, true><<<g, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, fr, nfr, bx);
    else k_gather_fretry<0, false><<<g, 256, 0, s>>>(nd, pl, n, qb, nq, out, perm, lead.p, fr, nfr, bx);
  }
  return hipGetLastError();
#endif
}

// ---- wide gathers (k > 64; config 5: k = 200 caustic gather): collect and sort.
// A K-wide sorted list in VGPRs stops paying above k ~ 64: every insert is a
// 2K-op min/max network run by the whole wave, a 128-wide list holds the wave
// at 2 waves/SIMD, and while a list fills under a loose cut-off nearly every
// point the walk tests is inserted (the 128-wide pm_knn passes took ~120 ms for
// config 5's 2.3 M caustic queries). Here a lane instead APPENDS each candidate
// key (d^2 < its cut-off) to its own row of CAP = 64 S keys in global memory
// (L2-resident: the rows of the waves in flight); when a row is full the wave
// sorts it cooperatively (bitonic over 64 lanes x S keys, f64 min/max on the
// gkey doubles), keeps the k smallest and tightens that lane's cut-off to the
// k-th -- each flush handles CAP - k candidates. When the walks are over, each
// row is sorted once more and its first min(cnt, k) keys are the exact k
// nearest in (d^2, index) order; the lane sums gatherPhotons (shading.h:93-121)
// over them in that order, exactly as radiance_g / k_radiance_k do.
// Cut-offs: leaders (every kSeedStride-th walk rank) start from the plain
// cut-off and record (position, k-th d^2); followers start from their leaders'
// triangle-inequality bound (follower_cut holds for any k). A cut-off only
// prunes: the kept keys are the k smallest either way.
// The grid is persistent (rows per wave in flight): a wave takes groups of 64
// consecutive walk ranks from an atomic counter until none are left.
constexpr double kDblMax = 1.7976931348623157e308;   // pad key: above every gkey
constexpr int kWideMinK = 64;                         // k > this: collect and sort

__device__ __forceinline__ void fence_wave() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Lane exchange v[lane ^ lj] without the LDS crossbar where the pattern allows:
// xor 1 / 2 are DPP quad permutes, xor 4 = half_mirror then quad reverse, xor 8
// = row_mirror then half_mirror (two DPP moves each), xor 16 a ds_swizzle; 32
// stays a ds_bpermute. (Every __shfl_xor was a ds_bpermute: 970 of them in the
// wide kernel, ~45 % of the final sorts' cost.)
// REQUIRES the whole wave active: the DPP moves use bound_ctrl = false, so a
// source lane that is inactive yields an undefined value. wave_sort / row_sort
// are called only from wave-uniform control flow; a caller under divergence
// must use __shfl_xor instead.
#ifndef PM_WIDE_DPP
#define PM_WIDE_DPP 1
#endif
__device__ __forceinline__ int lane_xor(int v, int lj) {
  if (!PM_WIDE_DPP) return __shfl_xor(v, lj);
  switch (lj) {
    case 1: return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1, 0, 3, 2]
    case 2: return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2, 3, 0, 1]
    case 4: {
      const int w = __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false);   // row_half_mirror: 7 - i in each 8
      return __builtin_amdgcn_mov_dpp(w, 0x1B, 0xF, 0xF, false);           // quad_perm [3, 2, 1, 0]
    }
    case 8: {
      const int w = __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false);   // row_mirror: 15 - i in each 16
      return __builtin_amdgcn_mov_dpp(w, 0x141, 0xF, 0xF, false);          // row_half_mirror
    }
    case 16: return __builtin_amdgcn_ds_swizzle(v, 0x1F | (16 << 10));   // bit mode, xor 16
    default: return __shfl_xor(v, lj);
  }
}
__device__ __forceinline__ double lane_xor(double v, int lj) {
  const int64_t b = __double_as_longlong(v);
  const int lo = lane_xor((int)(uint32_t)b, lj), hi = lane_xor((int)(uint32_t)(b >> 32), lj);
  return __longlong_as_double((int64_t)((uint64_t)(uint32_t)hi << 32 | (uint32_t)lo));
}

// Bitonic sort (ascending) of 64 S keys held blocked: lane L holds elements
// L S .. L S + S - 1. Strides >= S cross lanes (shuffles), smaller ones stay in
// the lane's registers.
template <int S>
__device__ __forceinline__ void wave_sort(double (&v)[S], int lane) {
  constexpr int N = 64 * S;
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int j = size >> 1; j > 0; j >>= 1) {
      if (j >= S) {
        const int lj = j / S;
        const bool keep_min = (((lane * S) & size) == 0) == ((lane & lj) == 0);
#pragma unroll
        for (int r = 0; r < S; r++) {
          const double p = lane_xor(v[r], lj);
          v[r] = keep_min ? dmin(v[r], p) : dmax(v[r], p);
        }
      } else {
#pragma unroll
        for (int r = 0; r < S; r++) {
          if (r & j) continue;
          const bool up = (((lane * S + r) & size) == 0);
          const double a = v[r], b = v[r | j];
          const double mn = dmin(a, b), mx = dmax(a, b);
          v[r] = up ? mn : mx;
          v[r | j] = up ? mx : mn;
        }
      }
    }
  }
}

// Sort the first cnt (wave-uniform, <= 64 S) keys of a row, write its smallest
// min(cnt, keep) back in order and return sorted[keep - 1] (meaningful when
// cnt >= keep).
template <int S>
__device__ __forceinline__ double row_sort(double* __restrict__ row, int cnt, int keep, int lane) {
  double v[S];
#pragma unroll
  for (int r = 0; r < S; r++) {
    const int e = lane * S + r;
    v[r] = e < cnt ? row[e] : kDblMax;
  }
  wave_sort<S>(v, lane);
  const int m = cnt < keep ? cnt : keep;
#pragma unroll
  for (int r = 0; r < S; r++)
    if (lane * S + r < m) row[lane * S + r] = v[r];
  const int kt = keep - 1, kr = kt % S;
  double t = v[0];
#pragma unroll
  for (int r = 1; r < S; r++) t = r == kr ? v[r] : t;
  return __shfl(t, (kt / S) & 63);
}

#ifndef PM_WIDE_BOX
#define PM_WIDE_BOX 1   // 0: plane test only (A/B variants)
#endif
#ifndef PM_WIDE_BOX_SKIP
#define PM_WIDE_BOX_SKIP 3   // boxes down to level D - skip (0: every node)
#endif

// One collect step of every lane: lean_step's walk and point test (with the
// subtree-box skip), the candidate appended to the lane's row instead of an
// LDS insert queue.
// PM_WIDE_STAGE: candidates are staged PM_WIDE_CHUNK at a time in an LDS
// column of the lane (`stage`, slot j at stage[j * 256]) and reach the row as
// one chunk (16-B stores) when its last key arrives: one 8-B store per
// candidate left rows partly filled in L2 (22 GB written for 7.7 GB of keys,
// config 5; staging 8: caustic gather 25.1 -> 20.6 ms).
#ifndef PM_WIDE_STAGE
#define PM_WIDE_STAGE 1
#endif
#ifndef PM_WIDE_CHUNK
#define PM_WIDE_CHUNK 8   // keys per staged chunk (8: 64 B, 16: one 128-B line)
#endif
constexpr int kChunkKeys = PM_WIDE_CHUNK;
static_assert(kChunkKeys == 8 || kChunkKeys == 16, "chunk of 8 or 16 keys");
template <bool WIDE>
__device__ __forceinline__ void collect_step(const float4* __restrict__ nodes, BoxView bx, uint32_t n, v3 q,
                                             double tail, LeanWalk& w, float4& nd, float4& ba, float4& bb,
                                             double* __restrict__ row, int& cnt, double* stage = nullptr) {
  const uint32_t word = __float_as_uint(nd.w);
  const uint32_t dim = word & 3u;
  const float dx = q.x - nd.x, dy = q.y - nd.y, dz = q.z - nd.z;
  const float diff = dim == 0 ? dx : (dim == 1 ? dy : dz);
  const bool skip = PM_WIDE_BOX && !w.up && w.c1 <= bx.nbox && box_d2(ba, bb, q) > w.bound;
  const uint32_t close1 = 2 * w.c1 + (diff > 0.f ? 1u : 0u), far1 = close1 ^ 1u;
  const bool closeok = close1 <= n;
  const bool test = !skip && (w.up || !closeok);
  const bool descend = !skip && !w.up && closeok;
  const bool farok = !skip && !descend && far1 <= n && diff * diff <= w.bound;
  const bool stay = descend || farok;
  const uint32_t next = descend ? close1 : (farok ? far1 : w.upnode);
  const bool go = w.walking && (stay || w.upnode != 0);
  const uint32_t c1n = go ? next : w.c1;
  const float4 ndn = node1<WIDE>(nodes, c1n);
  if (c1n <= bx.nbox) {
    const float4* bp = box1<WIDE>(bx.box, c1n);
    ba = bp[0];
    bb = bp[1];
  }
  const float d2 = dx * dx + dy * dy + dz * dz;
  const double key = gkey(d2, word);
  const bool cand = w.walking && test && key < tail;
  w.far_mask = stay ? (w.far_mask << 1 | (farok ? 1u : 0u)) : w.far_mask >> w.j1;
  w.up = !stay;
  if (PM_WIDE_STAGE) {
    constexpr int M = kChunkKeys - 1;
    if (cand) {
      stage[(cnt & M) * 256] = key;
      if ((cnt & M) == M) {   // the last of a chunk: [cnt - M, cnt] goes out in one piece
        double2* dst = reinterpret_cast<double2*>(row + (cnt & ~M));
#pragma unroll
        for (int j = 0; j < kChunkKeys / 2; j++)
          dst[j] = make_double2(stage[(2 * j) * 256], stage[(2 * j + 1) * 256]);
      }
    }
  } else if (cand) {
    row[cnt] = key;
  }
  cnt += cand ? 1 : 0;
  w.c1 = c1n;
  w.walking = go;
  w.set_jump();
  nd = ndn;
}


#ifndef PM_WIDE_RAD_CHUNK
#define PM_WIDE_RAD_CHUNK 8   // keys per row read in the radiance sum (1: one 8-B load per key)
#endif
// the chunked read loads key pairs (16 B) and reads whole chunks of a row
static_assert(PM_WIDE_RAD_CHUNK == 1 || (PM_WIDE_RAD_CHUNK % 2 == 0 && 64 % PM_WIDE_RAD_CHUNK == 0),
              "PM_WIDE_RAD_CHUNK: 1 or an even divisor of 64 (rows hold 64 S keys)");
// Leader step budget of the wide gather (wave iterations; 0: none): the
// leader launch is a few thousand waves on an otherwise idle GPU, so its length
// is its slowest wave's (config 5: 1,665 iterations per leader wave on
// average, 4,557 at most); lanes still walking at the budget are redone at the
// head of the follower launch, beside the followers.
#ifndef PM_WIDE_LEADER_BUDGET
#define PM_WIDE_LEADER_BUDGET 2048
#endif
constexpr int kWideLeaderBudget = PM_WIDE_LEADER_BUDGET;
// occupancy target of the wide kernels (0: the compiler's choice, 4 waves/SIMD
// at ~101 VGPRs; A/B knob)
#ifndef PM_WIDE_WAVES
#define PM_WIDE_WAVES 0
#endif
template <int TAG, bool LEADERS, bool WIDE, int S>
__global__ __launch_bounds__(256) PM_WAVES_ATTR(PM_WIDE_WAVES) void k_gather_wide(const float4* __restrict__ nodes,
                                                     const float4* __restrict__ payload, int n,
                                                     const float4* __restrict__ qb, int64_t nq,
                                                     float4* __restrict__ out, const uint32_t* __restrict__ perm,
                                                     float4* __restrict__ lead, int k, double* __restrict__ rows,
                                                     uint32_t* __restrict__ counter, int64_t nitems, BoxView bx,
                                                     uint32_t* __restrict__ retry, uint32_t* __restrict__ nretry) {
  constexpr int CAP = 64 * S;
  static_assert(CAP % kChunkKeys == 0, "rows hold whole chunks");
  static_assert(CAP % PM_WIDE_RAD_CHUNK == 0, "the radiance sum reads whole chunks of a row");
  const float R2 = kKMaxDistance * kKMaxDistance;
  const int lane = threadIdx.x & 63;
  double* const wrows = rows + ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * CAP;
  double* const row = wrows + lane * CAP;
  __shared__ double stage_lds[PM_WIDE_STAGE ? kChunkKeys * 256 : 1];
  double* const stage = stage_lds + threadIdx.x;
  // this lane's staged keys (cnt & 7 of them) into its row
  auto spill_stage = [&](int cnt) {
    constexpr int M = kChunkKeys - 1;
    if (PM_WIDE_STAGE)
      for (int j = 0; j < (cnt & M); j++) row[(cnt & ~M) + j] = stage[j * 256];
  };
  // follower launch: the leaders that ran out of budget come first (their
  // count is the leader launch's, complete before this launch starts)
  const int64_t nre = (!LEADERS && kWideLeaderBudget > 0) ? (int64_t)*nretry : 0;
  const int64_t items = nitems + nre;
  for (;;) {
    uint32_t g = 0;
    if (lane == 0) g = atomicAdd(counter, 1u);
    g = __shfl(g, 0);
    if ((int64_t)g * 64 >= items) break;   // wave-uniform: every wave reaches it
    const int64_t t0 = (int64_t)g * 64 + lane;
    const bool redo = t0 < nre;             // a retried leader
    const int64_t t = t0 - nre;
    int64_t r;
    if (redo) r = (int64_t)retry[t0];
    else r = LEADERS ? t * kSeedStride : (t / (kSeedStride - 1)) * kSeedStride + 1 + t % (kSeedStride - 1);
    const bool valid = t0 < items && r < nq;
    const int64_t i = !valid ? 0 : (perm ? (int64_t)perm[r] : r);
    const float4 qq = valid ? qb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const v3 q = {qq.x, qq.y, qq.z};
    float cut = lean_cut(R2);
    if (valid && !LEADERS) {
      if (redo) {   // its own record: the k-th d^2 of a flushed row, if it had one
        const float ts = lead[r / kSeedStride].w;
        if (ts >= 0.f) cut = fminf(cut, ts);
      } else {
        cut = follower_cut<1>(lead, nq, r, q, R2);
      }
    }
    double tail = gkey(cut, kNoWord);
    int cnt = 0;
    bool aborted = false, flushed = false;
    if (n > 0) {
      int it_b = 0;   // wave-uniform iterations (leader budget)
      LeanWalk w;
      w.start(cut, valid);
      float4 nd = node1<WIDE>(nodes, 1), ba = bx.box[0], bb = bx.box[1];
      for (;;) {
        collect_step<WIDE>(nodes, bx, (uint32_t)n, q, tail, w, nd, ba, bb, row, cnt, stage);
        if (LEADERS && kWideLeaderBudget > 0 && ++it_b == kWideLeaderBudget) {
          aborted = w.walking;   // redone at the head of the follower launch
          w.walking = false;
        }
        uint64_t full = ballot(cnt == CAP);
        const uint64_t full0 = full;
        if (full) {   // flush: keep each full row's k smallest, tighten its cut-off
          fence_wave();
          while (full) {
            const int l = __ffsll((long long)full) - 1;
            full &= full - 1;
            const double tl = row_sort<S>(wrows + l * CAP, CAP, k, lane);
            if (lane == l) {
              cnt = k;
              tail = tl;
              flushed = true;
              w.bound = gkey_d2(tl);
            }
          }
          fence_wave();
          // a full row was flushed chunk by chunk (CAP % 8 == 0); the kept k
          // keys end mid-chunk unless 8 | k: that chunk's head goes back to the
          // stage, so the next chunk write carries it
          constexpr int M = kChunkKeys - 1;
          if (PM_WIDE_STAGE && (k & M) && full0 & (1ull << lane))
            for (int j = 0; j < (k & M); j++) stage[j * 256] = row[(k & ~M) + j];
        }
        if (ballot(w.walking) == 0) break;
      }
    }
    // final sort of every row: its first min(cnt, k) keys in (d^2, index) order
    spill_stage(cnt);
    fence_wave();

    uint64_t live = ballot(cnt > 0 && !aborted);
    while (live) {
      const int l = __ffsll((long long)live) - 1;
      live &= live - 1;
      const int cl = __shfl(cnt, l);
      double* const rl = wrows + l * CAP;
      if (cl <= 64) row_sort<1>(rl, cl, k, lane);
      else if (cl <= 128) row_sort<2>(rl, cl, k, lane);
      else if (S <= 4 || cl <= 256) row_sort<(S < 4 ? S : 4)>(rl, cl, k, lane);
      else if (S <= 8 || cl <= 512) row_sort<(S < 8 ? S : 8)>(rl, cl, k, lane);
      else row_sort<S>(rl, cl, k, lane);
    }
    fence_wave();
    if (LEADERS && kWideLeaderBudget > 0) {
      // a leader cut off by the budget: a flushed row's k-th d^2 bounds its k
      // nearest (any k points do) and seeds its followers and its retry; no
      // flush yet: nothing. Its own result comes from the retry.
      if (valid && aborted) lead[r / kSeedStride] = make_float4(qq.x, qq.y, qq.z, flushed ? gkey_d2(tail) : -1.f);
      const uint64_t m = ballot(valid && aborted);
      if (m != 0) {   // wave-aggregated append to the retry list
        const int first = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane == first) base = atomicAdd(nretry, (uint32_t)__popcll(m));
        base = __shfl(base, first);
        if (valid && aborted) retry[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint32_t)r;
      }
    }
    if (valid && !aborted) {
      const int m = cnt < k ? cnt : k;
      const bool full = cnt >= k;
      const float r2 = full ? gkey_d2(row[k - 1]) : R2;
      v3 flux = {0.f, 0.f, 0.f};
#if PM_WIDE_RAD_CHUNK > 1
      // the lane's sorted row read PM_WIDE_RAD_CHUNK keys at a time (16-B loads
      // issued together: each row line is fetched once; one 8-B load per key
      // re-fetched the 64 lanes' lines, which the wave's other rows evict)
      for (int p0 = 0; p0 < m; p0 += PM_WIDE_RAD_CHUNK) {
        double key[PM_WIDE_RAD_CHUNK];
        const double2* src = reinterpret_cast<const double2*>(row + p0);
#pragma unroll
        for (int j = 0; j < PM_WIDE_RAD_CHUNK / 2; j++) {
          const double2 d = src[j];
          key[2 * j] = d.x;
          key[2 * j + 1] = d.y;
        }
#pragma unroll
        for (int j = 0; j < PM_WIDE_RAD_CHUNK; j++) {
          if (p0 + j < m) {
            const float4 pl = payload[gkey_word(key[j]) >> 2];
            const float dist = sqrtf(gkey_d2(key[j]));
            const float wgt = 1 - (dist / sqrtf(r2) * kConeFilterC);
            flux = add(flux, smul(qq.w * pl.w * wgt, v3{pl.x, pl.y, pl.z}));
          }
        }
      }
#else
      for (int p = 0; p < m; p++) {
        const double key = row[p];
        const float4 pl = payload[gkey_word(key) >> 2];
        const float dist = sqrtf(gkey_d2(key));
        const float wgt = 1 - (dist / sqrtf(r2) * kConeFilterC);
        flux = add(flux, smul(qq.w * pl.w * wgt, v3{pl.x, pl.y, pl.z}));
      }
#endif
      const v3 f = divf(flux, (1 - (2.f / 3.f) * (1.f / kConeFilterC)) * 2 * kPI * r2);
      out[i] = make_float4(f.x, f.y, f.z, 0.f);
      if (LEADERS) lead[r / kSeedStride] = make_float4(qq.x, qq.y, qq.z, full ? r2 : -1.f);
      // (a retried leader keeps its soft record: followers may be reading it)
    }
  }
}

static int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return cus;
}

template <int S>
static hipError_t launch_gather_wide_s(const pm_photon_map* m, const float4* qb, int64_t nq, float4* out,
                                       hipStream_t s, int k, const uint32_t* perm) {
  constexpr int CAP = 64 * S;
  const int n = (int)m->n;
  const int64_t nl = (nq + kSeedStride - 1) / kSeedStride, nf = nq - nl;
  const int64_t groups = (std::max(nl, nf) + 63) / 64;
  // persistent grid: the workgroups the CUs hold at once, no more than there are groups
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gather_wide<0, false, false, S>, 256, 0) !=
          hipSuccess || per_cu <= 0)
    per_cu = 4;
  const int64_t wg = std::min<int64_t>((groups + 3) / 4, (int64_t)device_cus() * per_cu);
  DevBuf<float4> lead(nl);
  DevBuf<uint32_t> ctr(3), retry(kWideLeaderBudget > 0 ? nl : 1);   // ctr[2]: retried leaders
  DevBuf<double> rows((size_t)wg * 256 * CAP);
  DevBuf<float4> box(2 * (size_t)std::max<int64_t>(boxed_nodes(n, PM_WIDE_BOX_SKIP), 1));
  if (!lead.p || !ctr.p || !rows.p || !box.p || !retry.p) return hipErrorOutOfMemory;
  PM_HIP_TRY(hipMemsetAsync(ctr.p, 0, 3 * sizeof(uint32_t), s));
  int64_t nbox = 0;
  PM_HIP_TRY(build_subtree_boxes(m->nodes.p, n, PM_WIDE_BOX_SKIP, box.p, &nbox, s));
  BoxView bx;
  bx.box = box.p;
  bx.nbox = (uint32_t)nbox;
  const bool wide = PM_FORCE_WIDE || n >= (1 << 28);
#define PM_WIDE_LAUNCH(W)                                                                                          \
  k_gather_wide<0, true, W, S><<<(int)std::min<int64_t>(wg, (nl + 255) / 256), 256, 0, s>>>(                     \
      m->nodes.p, m->payload.p, n, qb, nq, out, perm, lead.p, k, rows.p, ctr.p, nl, bx, retry.p, ctr.p + 2);      \
  PM_HIP_TRY(hipGetLastError());                                                                                 \
  if (nf > 0 || kWideLeaderBudget > 0) {                                                                          \
    k_gather_wide<0, false, W, S><<<(int)std::min<int64_t>(wg, (nf + nl + 255) / 256), 256, 0, s>>>(             \
        m->nodes.p, m->payload.p, n, qb, nq, out, perm, lead.p, k, rows.p, ctr.p + 1, nf, bx, retry.p,           \
        ctr.p + 2);                                                                                              \
    PM_HIP_TRY(hipGetLastError());                                                                               \
  }
  if (wide) {
    PM_WIDE_LAUNCH(true)
  } else {
    PM_WIDE_LAUNCH(false)
  }
#undef PM_WIDE_LAUNCH
  return hipStreamSynchronize(s);   // rows / leader records / boxes are freed on return
}

// ---- radiance estimate with k != 50 neighbours (k = 200
// caustic gather). gatherPhotons (shading.h:93-121) over the k nearest: the
// exact lists come from the pm_knn passes (k <= 128 one pass, up to 256 in
// 128-wide passes), then one kernel sums them in (d^2, index) order with
// r^2 = the k-th d^2 (max_radius^2 if fewer were found), as for k = 50.
// Production runs k > 64 through the collect-and-sort gather above; the check
// variant keeps these passes (independent code for the same lists).
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

hipError_t launch_gather_k(const pm_photon_map* m, const float4* qb, int64_t nq, float4* out, hipStream_t s,
                           int k, const uint32_t* perm) {
  if (nq <= 0) return hipSuccess;
  if (k < 1 || k > 256) return hipErrorInvalidValue;
  if (k == kKNearest) return launch_gather(m, qb, nq, out, s, 0, perm);
#if !PM_CHECK_VARIANT
  if (k > kWideMinK) {
    if (k <= 200) return launch_gather_wide_s<8>(m, qb, nq, out, s, k, perm);
    return launch_gather_wide_s<16>(m, qb, nq, out, s, k, perm);
  }
#endif
  DevBuf<pm_float3> q3(nq);
  DevBuf<int32_t> ids((size_t)nq * k);
  DevBuf<float> d2((size_t)nq * k), md(nq);
  if (!q3.p || !ids.p || !d2.p || !md.p) return hipErrorOutOfMemory;
  k_q3_from_dense<<<grid_for(nq, 256), 256, 0, s>>>(qb, perm, nq, q3.p);
  PM_HIP_TRY(hipGetLastError());
  // (leader-seeded cut-offs for these passes measured slower in round 1: config 5
  // caustic gather 195 -> 240 ms; the 128-wide passes are bound by their >= 128
  // inserts of 255 ops each, which a tighter cut does not remove)
  PM_HIP_TRY(launch_knn(m, q3.p, nq, k, kKMaxDistance, ids.p, d2.p, md.p, s));
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

