// knn_sim.c -- CPU cost model of the final-gather kNN walk (design tool, not
// product, not a test): builds the left-balanced kd-tree of a photon cloud
// (same split rules as kd_build), Morton-sorts a query cloud, and counts per
// 64-query wave:
//   A  the production per-lane walk (stack-free, post-order, JUMP, leader-
//      seeded cut-offs): node loads per lane (mean) and per wave (max lane);
//   B  a wave-uniform packet walk (one traversal per wave, a node is loaded
//      once and tested by all 64 lanes; the far child is entered when ANY
//      lane's ball crosses the plane): nodes per wave;
//   C  B with subtrees of <= BUCKET nodes tested exhaustively (one vector
//      load per bucket, every lane tests every point).
// Inserts per lane (list updates) are counted for each.
// Build: gcc -O2 -o /tmp/knn_sim tools/knn_sim.c -lm
// Run:   /tmp/knn_sim pts.f32 queries.f32 [waves_to_sample]
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define K 50
#define R2 1e4f
#define STRIDE 16
static int BUCKET = 63;
// walk rank of follower thread t (the production follower launch skips the leaders)
#define FRANK(t) (((t) / (STRIDE - 1)) * STRIDE + 1 + (t) % (STRIDE - 1))

typedef struct { float p[3]; int id, dim; } Node;
static float* P;
static Node* T;
static int N;

static int left_size(int s) {
  if (s <= 1) return 0;
  int h = 0;
  while ((1 << h) <= s) h++;
  const int half = 1 << (h - 2), full = (1 << (h - 1)) - 1, last = s - full;
  return (half - 1) + (last < half ? last : half);
}
static int cmp_dim;
static int less(int a, int b) {
  const float ca = P[3 * a + cmp_dim], cb = P[3 * b + cmp_dim];
  return ca < cb || (ca == cb && a < b);
}
static void select_k(int* v, int n, int k) {
  int lo = 0, hi = n - 1;
  while (hi > lo) {
    int pv = v[lo + (hi - lo) / 2], i = lo, j = hi;
    while (i <= j) {
      while (less(v[i], pv)) i++;
      while (less(pv, v[j])) j--;
      if (i <= j) { int t = v[i]; v[i] = v[j]; v[j] = t; i++; j--; }
    }
    if (k <= j) hi = j; else if (k >= i) lo = i; else return;
  }
}
static void build(int t, int* v, int s) {
  if (s <= 0) return;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = 0; i < s; i++)
    for (int d = 0; d < 3; d++) {
      const float c = P[3 * v[i] + d];
      if (c < mn[d]) mn[d] = c;
      if (c > mx[d]) mx[d] = c;
    }
  int dim = 0;
  if (mx[1] - mn[1] > mx[dim] - mn[dim]) dim = 1;
  if (mx[2] - mn[2] > mx[dim] - mn[dim]) dim = 2;
  const int ls = left_size(s);
  if (getenv("CLEAN") && s > 2) {
    // tie-aware: the widest dimension whose median has no equal coordinate
    // among its rank neighbours (ls - 1, ls + 1); else the widest
    int best = -1;
    for (int d = 0; d < 3; d++) {
      cmp_dim = d;
      select_k(v, s, ls);
      const float m = P[3 * v[ls] + d];
      float lo = -FLT_MAX, hi = FLT_MAX;
      for (int i = 0; i < ls; i++) lo = fmaxf(lo, P[3 * v[i] + d]);
      for (int i = ls + 1; i < s; i++) hi = fminf(hi, P[3 * v[i] + d]);
      const int clean = lo < m && m < hi;
      if (clean && (best < 0 || mx[d] - mn[d] > mx[best] - mn[best])) best = d;
    }
    if (best >= 0) dim = best;
  }
  cmp_dim = dim;
  select_k(v, s, ls);
  const int e = v[ls];
  for (int d = 0; d < 3; d++) T[t].p[d] = P[3 * e + d];
  T[t].id = e;
  T[t].dim = dim;
  build(2 * t + 1, v, ls);
  build(2 * t + 2, v + ls + 1, s - ls - 1);
}

// ---- candidate list: the K smallest (d2, id) keys, kept sorted
typedef struct { uint64_t key[K]; int n; } List;
static uint64_t mkkey(float d2, int id) {
  uint32_t b;
  memcpy(&b, &d2, 4);
  return (uint64_t)b << 32 | (uint32_t)id;
}
static float key_d2(uint64_t k) {
  const uint32_t b = (uint32_t)(k >> 32);
  float f;
  memcpy(&f, &b, 4);
  return f;
}
static void list_init(List* L) { L->n = 0; }
static int list_insert(List* L, uint64_t k) {   // returns 1 if inserted
  int n = L->n < K ? L->n : K - 1;
  if (L->n >= K && !(k < L->key[K - 1])) return 0;
  int j = n;
  while (j > 0 && L->key[j - 1] > k) { L->key[j] = L->key[j - 1]; j--; }
  L->key[j] = k;
  if (L->n < K) L->n++;
  return 1;
}
static float bound_of(const List* L, float cut) { return L->n < K ? cut : key_d2(L->key[K - 1]); }

static float dist2(const float* q, const Node* nd) {
  const float dx = q[0] - nd->p[0], dy = q[1] - nd->p[1], dz = q[2] - nd->p[2];
  return dx * dx + dy * dy + dz * dz;
}

// ---- kk nearest point ids of q (kk <= 256), sorted by (d2, id): leader lists for the Y model
static uint64_t GK[256];
static int GN, GKK;
static void gk_visit(const float* q, int t) {
  if (t >= N) return;
  const Node* nd = &T[t];
  const float diff = q[nd->dim] - nd->p[nd->dim];
  const int side = diff > 0.f;
  gk_visit(q, 2 * t + 1 + side);
  const uint64_t k = mkkey(dist2(q, nd), nd->id);
  if (GN < GKK || k < GK[GKK - 1]) {
    int j = GN < GKK ? GN++ : GKK - 1;
    while (j > 0 && GK[j - 1] > k) { GK[j] = GK[j - 1]; j--; }
    GK[j] = k;
  }
  const float b = GN < GKK ? 1e30f : key_d2(GK[GKK - 1]);
  if (diff * diff <= b) gk_visit(q, 2 * t + 2 - side);
}
static int knn_ids(const float* q, int kk, int* ids) {
  GN = 0; GKK = kk;
  gk_visit(q, 0);
  for (int i = 0; i < GN; i++) ids[i] = (int)(uint32_t)GK[i];
  return GN;
}
static int cmp_fl(const void* a, const void* b) {
  const float x = *(const float*)a, y = *(const float*)b;
  return x < y ? -1 : x > y;
}
// 50th smallest d2 from q over the distinct points of the given id sets
static float kth_of_sets(const float* q, int** sets, const int* ns, int nsets) {
  static float d[1024];
  static int seen[1024];
  int m = 0;
  for (int s = 0; s < nsets; s++)
    for (int i = 0; i < ns[s]; i++) {
      const int id = sets[s][i];
      int dup = 0;
      for (int j = 0; j < m && !dup; j++) dup = seen[j] == id;
      if (dup) continue;
      seen[m] = id;
      const float* p = &P[3 * id];
      const float dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
      d[m++] = dx * dx + dy * dy + dz * dz;
    }
  if (m < K) return 1e30f;
  qsort(d, m, sizeof(float), cmp_fl);
  return d[K - 1];
}

// ---- A: per-lane JUMP walk (lean_step), returns node loads; counts inserts
static int VERBOSE = 0;
static int BOXD = 0;   // incremental box-distance pruning (Arya-Mount) in the walk
static int walk_lane(const float* q, float cut, List* L, int* ins) {
  list_init(L);
  int prev = -1, curr = 0, depth = 0, steps = 0;
  uint32_t far_mask = 0;
  float bound = cut;
  float off[3] = {0.f, 0.f, 0.f}, rd = 0.f;
  int odep[3] = {0, 0, 0};   // BOXD 3: depth of the far entry that set off[d]
  int sdim[64];
  float soff[64];
  int sp = 0;
  for (;;) {
    const Node* nd = &T[curr];
    steps++;
    const int child = 2 * curr + 1;
    const float diff = q[nd->dim] - nd->p[nd->dim];
    const int side = diff > 0.f, close = child + side, far = child + 1 - side;
    const int down = prev < child;
    const int test = (down && close >= N) || prev == close;
    if (test) {
      const float d2 = dist2(q, nd);
      if (d2 <= cut && list_insert(L, mkkey(d2, nd->id))) {
        (*ins)++;
        bound = bound_of(L, cut);
        if (VERBOSE && (*ins <= 60 || *ins % 20 == 0)) printf("      step %d depth %d insert #%d d2 %g bound %g node (%g %g %g)\n", steps, depth, *ins, d2, bound, nd->p[0], nd->p[1], nd->p[2]);
      }
    }
    int next, nprev;
    if (down && close < N) {
      next = close; nprev = curr; far_mask &= ~(2u << depth); depth++;
    } else if (far < N && (BOXD ? rd - off[nd->dim] * off[nd->dim] + diff * diff : diff * diff) <= bound) {
      next = far; nprev = curr; far_mask |= 2u << depth; depth++;
      if (BOXD) {
        rd = rd - off[nd->dim] * off[nd->dim] + diff * diff;
        if (BOXD == 1) { sdim[sp] = nd->dim; soff[sp] = off[nd->dim]; sp++; }
        off[nd->dim] = fabsf(diff);
        odep[nd->dim] = depth;   // depth of the far child just entered
      }
    } else {
      const uint32_t open = (~far_mask & ((2u << depth) - 1u)) | 1u;
      int da = 31;
      while (!(open >> da & 1)) da--;
      const int a = ((curr + 1) >> (depth - da)) - 1;
      next = da == 0 ? -1 : ((a + 1) >> 1) - 1;
      nprev = a;
      if (BOXD == 1)
        for (int u = 0; u < depth - da; u++) {   // unwind the far entries below a's parent
          sp--;
          off[sdim[sp]] = soff[sp];
        }
      if (BOXD == 2) off[0] = off[1] = off[2] = 0.f;   // conservative: forget every offset
      if (BOXD == 3)                                    // forget the offsets set at or below a
        for (int d = 0; d < 3; d++)
          if (odep[d] >= da) off[d] = 0.f;
      if (BOXD) rd = off[0] * off[0] + off[1] * off[1] + off[2] * off[2];
      depth = da - 1;
    }
    if (next < 0) break;
    prev = nprev;
    curr = next;
  }
  return steps;
}

// ---- B / C: wave-uniform packet walk
typedef struct { const float* q[64]; float cut[64]; List L[64]; int n; long nodes, buckets, bucket_pts, ins; int lins[64]; } Packet;
static int subtree_size(int t) {   // nodes of the implicit subtree of t
  int s = 0;
  for (long lo = t, hi = t; lo < N; lo = 2 * lo + 1, hi = 2 * hi + 2) s += (int)((hi < N ? hi : N - 1) - lo + 1);
  return s;
}
static void packet_test(Packet* W, const Node* nd) {
  for (int l = 0; l < W->n; l++) {
    const float d2 = dist2(W->q[l], nd);
    if (d2 <= W->cut[l] && list_insert(&W->L[l], mkkey(d2, nd->id))) { W->ins++; W->lins[l]++; }
  }
}
static int lane_needs(Packet* W, int l, const Node* nd, int side_of_child) {
  const float diff = W->q[l][nd->dim] - nd->p[nd->dim];
  const int side = diff > 0.f;
  if (side == side_of_child) return 1;
  return diff * diff <= bound_of(&W->L[l], W->cut[l]);
}
static void packet_visit(Packet* W, int t, int bucket) {
  if (t >= N) return;
  if (bucket && subtree_size(t) <= BUCKET) {   // C: exhaustive bucket
    W->buckets++;
    for (long lo = t, hi = t; lo < N; lo = 2 * lo + 1, hi = 2 * hi + 2)
      for (long u = lo; u <= hi && u < N; u++) { packet_test(W, &T[u]); W->bucket_pts++; }
    return;
  }
  W->nodes++;
  const Node* nd = &T[t];
  int votes = 0;
  for (int l = 0; l < W->n; l++) votes += (W->q[l][nd->dim] - nd->p[nd->dim]) > 0.f;
  const int first = votes * 2 > W->n ? 1 : 0;
  int need = 0;
  for (int l = 0; l < W->n && !need; l++) need = lane_needs(W, l, nd, first);
  if (need) packet_visit(W, 2 * t + 1 + first, bucket);
  packet_test(W, nd);   // post-order (after the majority's close child)
  need = 0;
  for (int l = 0; l < W->n && !need; l++) need = lane_needs(W, l, nd, 1 - first);
  if (need) packet_visit(W, 2 * t + 2 - first, bucket);
}


// ---- D: lockstep wave model of the production loop (lean_step + LDS queue of
// QL keys). Every iteration advances every walking lane by one node; a round
// runs when some lane's queue is full or no lane walks. policy 0: each lane pops
// ONE queued key (production); policy 1: each lane merges ALL its queued keys.
// Returns iterations; *rounds = insert rounds.
static int QL = 8;
// partial insert networks: per pop-one round, the wave's lowest insertion
// position (entries below it are unchanged) rounded down to a checkpoint
// multiple of NETCP; the network then runs from there (K - start entries)
static int NETCP = 8;
static double g_net_entries = 0, g_net_rounds = 0;
typedef struct {
  const float* q; float cut, bound; List L; int prev, curr, depth, walking, qn; uint32_t far_mask; uint64_t qk[32];
} Lane;
static int wave_lockstep(const float* const* qs, const float* cuts, int policy, int* rounds, long* lane_ins) {
  Lane ln[64];
  for (int l = 0; l < 64; l++) {
    ln[l].q = qs[l]; ln[l].cut = cuts[l]; ln[l].bound = cuts[l]; list_init(&ln[l].L);
    ln[l].prev = -1; ln[l].curr = 0; ln[l].depth = 0; ln[l].walking = 1; ln[l].qn = 0; ln[l].far_mask = 0;
  }
  int it = 0;
  *rounds = 0;
  for (;;) {
    it++;
    int any_walk = 0, any_full = 0;
    for (int l = 0; l < 64; l++) {
      Lane* w = &ln[l];
      if (!w->walking) continue;
      const Node* nd = &T[w->curr];
      const int child = 2 * w->curr + 1;
      const float diff = w->q[nd->dim] - nd->p[nd->dim];
      const int side = diff > 0.f, close = child + side, far = child + 1 - side;
      const int down = w->prev < child;
      if ((down && close >= N) || w->prev == close) {
        const float d2 = dist2(w->q, nd);
        const uint64_t k = mkkey(d2, nd->id);
        const int full = w->L.n >= K;
        if (d2 <= w->cut && (!full || k < w->L.key[K - 1])) w->qk[w->qn++] = k;
      }
      int next, nprev;
      if (down && close < N) {
        next = close; nprev = w->curr; w->far_mask &= ~(2u << w->depth); w->depth++;
      } else if (far < N && diff * diff <= w->bound) {
        next = far; nprev = w->curr; w->far_mask |= 2u << w->depth; w->depth++;
      } else {
        const uint32_t open = (~w->far_mask & ((2u << w->depth) - 1u)) | 1u;
        int da = 31;
        while (!(open >> da & 1)) da--;
        const int a = ((w->curr + 1) >> (w->depth - da)) - 1;
        next = da == 0 ? -1 : ((a + 1) >> 1) - 1;
        nprev = a;
        w->depth = da - 1;
      }
      if (next < 0) w->walking = 0; else { w->prev = nprev; w->curr = next; }
    }
    for (int l = 0; l < 64; l++) { any_walk |= ln[l].walking; any_full |= ln[l].qn == QL; }
    if (any_full || !any_walk) {
      (*rounds)++;
      int left = 0;
      for (int l = 0; l < 64; l++) {
        Lane* w = &ln[l];
        if (policy == 2) {   // filtered pop: skip queued keys the list has outgrown
          while (w->qn > 0) {
            const uint64_t k = w->qk[--w->qn];
            if (list_insert(&w->L, k)) { (*lane_ins)++; break; }
          }
        } else {
          if (policy == 0 && l == 0) {   // the wave's lowest insertion position this round
            int pmin = K;
            for (int l2 = 0; l2 < 64; l2++) {
              const Lane* u = &ln[l2];
              if (u->qn <= 0) continue;
              const uint64_t k = u->qk[u->qn - 1];
              if (u->L.n >= K && !(k < u->L.key[K - 1])) continue;
              int pos = 0;
              while (pos < u->L.n && u->L.key[pos] < k) pos++;
              if (pos < pmin) pmin = pos;
            }
            if (pmin < K) { g_net_entries += K - (pmin / NETCP) * NETCP; g_net_rounds++; }
          }
          const int take = policy ? w->qn : (w->qn > 0);
          for (int t = 0; t < take; t++) {
            const uint64_t k = w->qk[--w->qn];
            if (list_insert(&w->L, k)) (*lane_ins)++;
          }
        }
        w->bound = bound_of(&w->L, w->cut);
        left |= w->qn > 0;
      }
      if (!any_walk && !left) break;
    }
  }
  return it;
}


static uint32_t part1by2(uint32_t x) {
  x &= 0x3FF;
  x = (x | (x << 16)) & 0x30000FF; x = (x | (x << 8)) & 0x300F00F;
  x = (x | (x << 4)) & 0x30C30C3; x = (x | (x << 2)) & 0x9249249;
  return x;
}
static uint64_t* MK;
static int cmp_mk(const void* a, const void* b) {
  const uint64_t x = MK[*(const int*)a], y = MK[*(const int*)b];
  return x < y ? -1 : x > y;
}
static double seed_bound(const float* lq, float lt, const float* q) {
  if (lt < 0) return 1e300;
  const double dx = (double)q[0] - lq[0], dy = (double)q[1] - lq[1], dz = (double)q[2] - lq[2];
  const double c = (sqrt((double)lt) + sqrt(dx * dx + dy * dy + dz * dz)) * (1.0 + 1e-6);
  return c * c * (1.0 + 1e-5) + 1e-30;
}

// ---- P: pooled lanes: a wave owns NPQ Morton-consecutive followers; a lane
// whose walk is over and whose queue is empty takes the next one (refill when
// >= REFILL lanes wait, or every lane waits). Rounds as in D (pop one when a
// queue is full or no lane walks). Returns iterations; *rounds.
static int pool_lockstep(const float* const* qs, const float* cuts, int nq, int refill, int* rounds) {
  Lane ln[64];
  int next = 0;
  for (int l = 0; l < 64; l++) { ln[l].walking = 0; ln[l].qn = 0; }
  int it = 0;
  *rounds = 0;
  for (;;) {
    int idle = 0;
    for (int l = 0; l < 64; l++) idle += !ln[l].walking && ln[l].qn == 0;
    if (next < nq && (idle >= refill || idle == 64)) {
      for (int l = 0; l < 64 && next < nq; l++) {
        Lane* w = &ln[l];
        if (w->walking || w->qn) continue;
        w->q = qs[next]; w->cut = cuts[next]; w->bound = cuts[next]; next++;
        list_init(&w->L); w->prev = -1; w->curr = 0; w->depth = 0; w->walking = 1; w->far_mask = 0;
      }
    }
    int any = 0;
    for (int l = 0; l < 64; l++) any |= ln[l].walking || ln[l].qn;
    if (!any && next >= nq) break;
    it++;
    for (int l = 0; l < 64; l++) {
      Lane* w = &ln[l];
      if (!w->walking) continue;
      const Node* nd = &T[w->curr];
      const int child = 2 * w->curr + 1;
      const float diff = w->q[nd->dim] - nd->p[nd->dim];
      const int side = diff > 0.f, close = child + side, far = child + 1 - side;
      const int down = w->prev < child;
      if ((down && close >= N) || w->prev == close) {
        const float d2 = dist2(w->q, nd);
        const uint64_t k = mkkey(d2, nd->id);
        if (d2 <= w->cut && (w->L.n < K || k < w->L.key[K - 1])) w->qk[w->qn++] = k;
      }
      int nx, nprev;
      if (down && close < N) { nx = close; nprev = w->curr; w->far_mask &= ~(2u << w->depth); w->depth++; }
      else if (far < N && diff * diff <= w->bound) { nx = far; nprev = w->curr; w->far_mask |= 2u << w->depth; w->depth++; }
      else {
        const uint32_t open = (~w->far_mask & ((2u << w->depth) - 1u)) | 1u;
        int da = 31;
        while (!(open >> da & 1)) da--;
        const int a = ((w->curr + 1) >> (w->depth - da)) - 1;
        nx = da == 0 ? -1 : ((a + 1) >> 1) - 1;
        nprev = a;
        w->depth = da - 1;
      }
      if (nx < 0) w->walking = 0; else { w->prev = nprev; w->curr = nx; }
    }
    int full = 0, walk = 0;
    for (int l = 0; l < 64; l++) { full |= ln[l].qn == QL; walk |= ln[l].walking; }
    // a lane whose walk is over drains its queue in the rounds the others trigger,
    // or in rounds of its own once no lane walks
    int pend = 0;
    for (int l = 0; l < 64; l++) pend += !ln[l].walking && ln[l].qn;
    if (full || !walk || pend >= refill) {
      (*rounds)++;
      for (int l = 0; l < 64; l++) {
        Lane* w = &ln[l];
        if (w->qn > 0) { list_insert(&w->L, w->qk[--w->qn]); w->bound = bound_of(&w->L, w->cut); }
      }
    }
  }
  return it;
}

// ---- F: wave max steps when the followers of each 256-query block are
// regrouped into waves by their seeded cut-off (sorted within the block).
static int cmp_f(const void* a, const void* b) {
  const float x = *(const float*)a, y = *(const float*)b;
  return x < y ? -1 : x > y;
}
// ---- G: lockstep wave with bucketed bottoms: nodes at depth >= DB are never
// walked; a walk that would enter a depth-DB node scans its whole subtree (<= 7
// nodes: levels DB..DB+2) in one iteration, testing every point. Rounds pop one
// queued key per lane when some lane holds >= QG - 7 keys (room for one scan).
// Cost model (VALU instructions): walk step WS, scan SC, round RC; a wave
// iteration costs WS if any lane walks plus SC if any lane scans.
static int DB;
static double g_cost(const float* const* qs, const float* cuts, int QG, double WS, double SC, double RC, int* iters,
                     int* rounds) {
  Lane ln[64];
  int scan_root[64];
  for (int l = 0; l < 64; l++) {
    ln[l].q = qs[l]; ln[l].cut = cuts[l]; ln[l].bound = cuts[l]; list_init(&ln[l].L);
    ln[l].prev = -1; ln[l].curr = 0; ln[l].depth = 0; ln[l].walking = 1; ln[l].qn = 0; ln[l].far_mask = 0;
    scan_root[l] = -1;
  }
  double cost = 0;
  *iters = 0; *rounds = 0;
  for (;;) {
    int any_walk = 0, any_scan = 0, any_live = 0;
    for (int l = 0; l < 64; l++) {
      Lane* w = &ln[l];
      if (!w->walking) continue;
      any_live = 1;
      if (scan_root[l] >= 0) {   // scan the bucket under scan_root, then return to its parent
        any_scan = 1;
        const int t = scan_root[l];
        for (int lev = 0; lev < 3; lev++)
          for (int j = 0; j < (1 << lev); j++) {
            const long c = (long)(t + 1) * (1 << lev) - 1 + j;
            if (c >= N) continue;
            const float d2 = dist2(w->q, &T[c]);
            const uint64_t k = mkkey(d2, T[c].id);
            if (d2 <= w->cut && (w->L.n < K || k < w->L.key[K - 1])) w->qk[w->qn++] = k;
          }
        scan_root[l] = -1;
        w->prev = t;   // back at the parent (curr), arrived from child t
        continue;
      }
      any_walk = 1;
      const Node* nd = &T[w->curr];
      const int child = 2 * w->curr + 1;
      const float diff = w->q[nd->dim] - nd->p[nd->dim];
      const int side = diff > 0.f, close = child + side, far = child + 1 - side;
      const int down = w->prev < child;
      if ((down && close >= N) || w->prev == close) {
        const float d2 = dist2(w->q, nd);
        const uint64_t k = mkkey(d2, nd->id);
        if (d2 <= w->cut && (w->L.n < K || k < w->L.key[K - 1])) w->qk[w->qn++] = k;
      }
      int next;
      if (w->prev == far) next = ((w->curr + 1) >> 1) - 1;
      else if (w->prev == close || close >= N) next = (far < N && diff * diff <= w->bound) ? far : ((w->curr + 1) >> 1) - 1;
      else next = close;
      if (next < 0) { w->walking = 0; continue; }
      if (next > w->curr && 31 - __builtin_clz((uint32_t)next + 1) >= DB) { scan_root[l] = next; continue; }
      w->prev = w->curr; w->curr = next;
    }
    if (!any_live) break;
    (*iters)++;
    cost += (any_walk ? WS : 0) + (any_scan ? SC : 0);
    int need = 0, left = 0, live = 0;
    for (int l = 0; l < 64; l++) { need |= ln[l].qn >= QG - 7; live |= ln[l].walking; }
    if (need || !live) {
      do {
        (*rounds)++;
        cost += RC;
        left = 0;
        need = 0;
        for (int l = 0; l < 64; l++) {
          Lane* w = &ln[l];
          if (w->qn > 0) { list_insert(&w->L, w->qk[--w->qn]); w->bound = bound_of(&w->L, w->cut); }
          left |= w->qn > 0;
          need |= w->qn >= QG - 7;
        }
      } while ((!live && left) || need);
    }
  }
  return cost;
}

static void regroup_model(const float* Q, const int* ord, long nq, const float* lt, long nl, int blocks) {
  double morton = 0, sorted = 0, mean = 0;
  List L;
  int dummy = 0;
  srand(777);
  for (int bk = 0; bk < blocks; bk++) {
    const long b0 = (long)((double)rand() / RAND_MAX * (nq / 256 - 2)) * 256;
    float rec[256][2];   // (cut, steps)
    for (int l = 0; l < 256; l++) {
      const long r = b0 + l;
      const float* q = &Q[3 * ord[r]];
      float cut = nextafterf(R2, 0.f);
      if (r % STRIDE) {
        const long jp = r / STRIDE;
        double b = 1e300;
        for (long j = jp - 1; j <= jp + 2; j++)
          if (j >= 0 && j < nl && lt[j] > -2.f) b = fmin(b, seed_bound(&Q[3 * ord[j * STRIDE]], lt[j], q));
        if (b < cut) cut = (float)b * (1.f + 1e-7f);
      }
      rec[l][0] = cut;
      rec[l][1] = (float)walk_lane(q, cut, &L, &dummy);
      mean += rec[l][1];
    }
    for (int w = 0; w < 4; w++) {
      float m = 0;
      for (int l = 0; l < 64; l++) m = fmaxf(m, rec[w * 64 + l][1]);
      morton += m;
    }
    qsort(rec, 256, sizeof(rec[0]), cmp_f);
    for (int w = 0; w < 4; w++) {
      float m = 0;
      for (int l = 0; l < 64; l++) m = fmaxf(m, rec[w * 64 + l][1]);
      sorted += m;
    }
  }
  printf("F followers regrouped by cut within 256-blocks: mean steps %.1f, wave max Morton %.1f -> sorted %.1f\n",
         mean / blocks / 256, morton / blocks / 4, sorted / blocks / 4);
}


static float* readf(const char* path, long* n) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(1); }
  fseek(f, 0, SEEK_END);
  *n = ftell(f) / 12;
  fseek(f, 0, SEEK_SET);
  float* a = malloc((size_t)*n * 12);
  if (fread(a, 12, (size_t)*n, f) != (size_t)*n) exit(1);
  fclose(f);
  return a;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s pts.f32 qs.f32 [waves]\n", argv[0]); return 1; }
  long np, nq;
  P = readf(argv[1], &np);
  float* Q = readf(argv[2], &nq);
  const int sample = argc > 3 ? atoi(argv[3]) : 2000;
  if (argc > 4) BUCKET = atoi(argv[4]);
  if (argc > 5) QL = atoi(argv[5]);
  if (getenv("NETCP")) NETCP = atoi(getenv("NETCP"));
  N = (int)np;
  T = malloc(sizeof(Node) * (size_t)N);
  int* v = malloc(sizeof(int) * (size_t)N);
  for (int i = 0; i < N; i++) v[i] = i;
  build(0, v, N);
  { int dm = 0; while ((2L << dm) - 1 < N) dm++; DB = dm - 2; }   // deepest level dm (0-based)
  // Morton order of the queries over their bounds (30-bit)
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (long i = 0; i < nq; i++)
    for (int d = 0; d < 3; d++) { lo[d] = fminf(lo[d], Q[3 * i + d]); hi[d] = fmaxf(hi[d], Q[3 * i + d]); }
  MK = malloc(8 * (size_t)nq);
  int* ord = malloc(sizeof(int) * (size_t)nq);
  for (long i = 0; i < nq; i++) {
    uint32_t c[3];
    for (int d = 0; d < 3; d++) {
      float u = (Q[3 * i + d] - lo[d]) / (hi[d] - lo[d]);
      c[d] = (uint32_t)fminf(fmaxf(u * 1024.f, 0.f), 1023.f);
    }
    MK[i] = ((uint64_t)(part1by2(c[0]) << 2 | part1by2(c[1]) << 1 | part1by2(c[2])) << 32) | (uint64_t)i;
    ord[i] = (int)i;
  }
  qsort(ord, (size_t)nq, sizeof(int), cmp_mk);
  const long nwaves = (nq - nq / STRIDE) / 64 - 1;
  // leader records (every STRIDE-th query in walk order, plain cut-off)
  const long nl = (nq + STRIDE - 1) / STRIDE;
  float* lt = malloc(sizeof(float) * (size_t)nl);
  List L;
  int dummy = 0;
  srand(12345);
  long* waves = malloc(sizeof(long) * (size_t)sample);
  for (int s = 0; s < sample; s++) waves[s] = (long)((double)rand() / RAND_MAX * (nwaves - 1));
  // only the leaders the sampled waves consult are walked
  char* need = calloc((size_t)nl, 1);
  const int regroup_blocks = argc > 6 ? atoi(argv[6]) : 0;
  for (int s = 0; s < sample; s++) {
    const long r0 = FRANK(waves[s] * 64);
    for (long r = r0 - 2 * STRIDE; r < r0 + 80 + 3 * STRIDE; r += STRIDE)
      if (r >= 0 && r / STRIDE < nl) need[r / STRIDE] = 1;
  }
  for (long j = 0; j < nl; j++) {
    lt[j] = -3.f;
    if (!need[j] && !regroup_blocks) continue;
    walk_lane(&Q[3 * ord[j * STRIDE]], nextafterf(R2, 0.f), &L, &dummy);
    lt[j] = L.n >= K ? key_d2(L.key[K - 1]) : -1.f;
  }
  double a_mean = 0, a_max = 0, a_ins = 0, b_nodes = 0, b_ins = 0, c_nodes = 0, c_buckets = 0, c_pts = 0, c_ins = 0;
  double e_nodes = 0, e_buckets = 0, e_pts = 0, e_ins = 0, e_max_nodes = 0, e_max_pts = 0, e_max_cost = 0;
  double pit_static = 0, prd_static = 0;
  double y_it[8] = {0}, y_rounds[8] = {0}, y_ratio[8] = {0}, y_n[8] = {0}, s_ratio = 0, s_n = 0;
  double z_it[3] = {0}, z_rd[3] = {0}, z_ratio[3] = {0}, z_n[3] = {0};
  double g_c[2] = {0}, g_it[2] = {0}, g_rd[2] = {0}, d_c[2] = {0};
  double x_it[4] = {0, 0, 0, 0}, x_rounds[4] = {0, 0, 0, 0};
  double a_plain_max = 0, b_plain = 0, c_maxins = 0, b_maxins = 0, d_it[3] = {0, 0, 0}, d_rounds[3] = {0, 0, 0}, d_ins[3] = {0, 0, 0};
  for (int s = 0; s < sample; s++) {
    const long t0 = waves[s] * 64;
    Packet W, Wp, Wc;
    float exact[64];
    memset(&W, 0, sizeof(W));
    int mx = 0, mxp = 0, ins = 0;
    for (int l = 0; l < 64; l++) {
      const long r = FRANK(t0 + l);
      const float* q = &Q[3 * ord[r]];
      float cut = nextafterf(R2, 0.f);
      if (r % STRIDE) {
        const long jp = r / STRIDE;
        double b = 1e300;
        for (long j = jp - 1; j <= jp + 2; j++)
          if (j >= 0 && j < nl) b = fmin(b, seed_bound(&Q[3 * ord[j * STRIDE]], lt[j], q));
        if (b < cut) cut = (float)b * (1.f + 1e-7f);
      }
      const int st = walk_lane(q, cut, &L, &ins);
      a_mean += st;
      if (st > mx) mx = st;
      int d2 = 0;
      const int sp = walk_lane(q, nextafterf(R2, 0.f), &L, &d2);
      if (sp > mxp) mxp = sp;
      exact[l] = L.n >= K ? key_d2(L.key[K - 1]) : nextafterf(R2, 0.f);
      W.q[l] = q;
      W.cut[l] = cut;
    }
    W.n = 64;
    {   // Y: cut from the leaders' kk-lists (50th smallest d2 over their points)
      static const int kks[4] = {50, 64, 96, 128};
      for (int v = 0; v < 8; v++) {
        const int kk = kks[v & 3], two = v >> 2;
        float yc[64];
        for (int l = 0; l < 64; l++) {
          const long r = FRANK(t0 + l);
          yc[l] = W.cut[l];
          if (r % STRIDE == 0) continue;
          const long ja = r / STRIDE, jb = ja + 1;
          static int ia[256], ib[256];
          int* sets[2] = {ia, ib};
          int ns[2];
          const float* qa = &Q[3 * ord[ja * STRIDE]];
          const float* qb = jb * STRIDE < nq ? &Q[3 * ord[jb * STRIDE]] : qa;
          const float* q = W.q[l];
          const float da = dist2(q, &(Node){{qa[0], qa[1], qa[2]}, 0, 0});
          const float db = dist2(q, &(Node){{qb[0], qb[1], qb[2]}, 0, 0});
          ns[0] = knn_ids(two || da <= db ? qa : qb, kk, ia);
          ns[1] = two ? knn_ids(qb, kk, ib) : 0;
          const float b = kth_of_sets(q, sets, ns, two ? 2 : 1) * (1.f + 1e-6f);
          if (b < yc[l]) yc[l] = b;
          y_ratio[v] += yc[l] / exact[l];
          y_n[v]++;
        }
        int rounds = 0;
        long li = 0;
        y_it[v] += wave_lockstep(W.q, yc, 0, &rounds, &li);
        y_rounds[v] += rounds;
      }
      for (int l = 0; l < 64; l++) if (FRANK(t0 + l) % STRIDE) { s_ratio += W.cut[l] / exact[l]; s_n++; }
    }
    for (int v = 0; v < 3; v++) {   // Z: cut from q's own depth-(Dmax - h) subtree (50th smallest d2 of its points)
      const int h = 5 + v;   // subtree of 2^(h+1)-1 nodes
      float zc[64];
      for (int l = 0; l < 64; l++) {
        const float* q = W.q[l];
        zc[l] = W.cut[l];
        int t = 0, dep = 0;
        while (dep < DB + 2 - h) {   // close-path descent
          const Node* nd = &T[t];
          const float diff = q[nd->dim] - nd->p[nd->dim];
          const int c = 2 * t + 1 + (diff > 0.f);
          if (c >= N) break;
          t = c; dep++;
        }
        static float d[1024];
        int m = 0;
        for (int lev = 0; lev <= h; lev++)
          for (long j = 0; j < (1L << lev); j++) {
            const long c = (long)(t + 1) * (1L << lev) - 1 + j;
            if (c < N) d[m++] = dist2(q, &T[c]);
          }
        if (getenv("ZONLY")) zc[l] = nextafterf(R2, 0.f);   // no leader bound: the subtree's alone
        if (m >= K) {
          qsort(d, m, sizeof(float), cmp_fl);
          const float b = d[K - 1] * (1.f + 1e-6f);
          if (b < zc[l]) zc[l] = b;
        }
        z_ratio[v] += zc[l] / exact[l];
        z_n[v]++;
      }
      int rounds = 0;
      long li = 0;
      z_it[v] += wave_lockstep(W.q, zc, 0, &rounds, &li);
      z_rd[v] += rounds;
    }
    for (int v = 0; v < 2; v++) {   // G: bucketed-bottom lockstep, seeded / exact cut
      float gc[64];
      for (int l = 0; l < 64; l++) gc[l] = v ? fminf(exact[l] * (1.f + 1e-6f), W.cut[l]) : W.cut[l];
      int it, rd;
      g_c[v] += g_cost(W.q, gc, 16, 50, 84, 111, &it, &rd);
      g_it[v] += it; g_rd[v] += rd;
      int it2, rd2;
      d_c[v] += wave_lockstep(W.q, gc, 0, &rd2, &(long){0}) * 60.0;
      d_c[v] += rd2 * 111.0;
    }
    for (int f = 0; f < 4; f++) {   // X: lockstep with cut = exact k-th d2 x factor
      static const float fac[4] = {1.0f, 1.15f, 1.5f, 2.0f};
      float xc[64];
      for (int l = 0; l < 64; l++) xc[l] = fminf(exact[l] * fac[f] * (1.f + 1e-6f), W.cut[l]);
      int rounds = 0;
      long li = 0;
      x_it[f] += wave_lockstep(W.q, xc, 0, &rounds, &li);
      x_rounds[f] += rounds;
    }
    for (int pol = 0; pol < 3; pol++) {
      int rounds = 0;
      long li = 0;
      d_it[pol] += wave_lockstep(W.q, W.cut, pol, &rounds, &li);
      d_rounds[pol] += rounds;
      d_ins[pol] += li;
    }
    a_max += mx;
    a_plain_max += mxp;
    a_ins += ins;
    // E: per-lane bucketed walk (each lane alone, buckets of <= BUCKET nodes)
    {
      double mn = 0, mp = 0, mc = 0;
      for (int l = 0; l < 64; l++) {
        Packet* X = malloc(sizeof(Packet));
        memset(X, 0, sizeof(Packet));
        X->n = 1;
        X->q[0] = W.q[l];
        X->cut[0] = W.cut[l];
        list_init(&X->L[0]);
        packet_visit(X, 0, 1);
        e_nodes += X->nodes;
        e_buckets += X->buckets;
        e_pts += X->bucket_pts;
        e_ins += X->ins;
        if (X->nodes > mn) mn = X->nodes;
        if (X->bucket_pts > mp) mp = X->bucket_pts;
        const double cost = 55.0 * X->nodes + 12.0 * X->bucket_pts;   // VALU model: walk step vs point test
        if (cost > mc) mc = cost;
        free(X);
      }
      e_max_nodes += mn;
      e_max_pts += mp;
      e_max_cost += mc;
    }
    Wp = W;
    for (int l = 0; l < 64; l++) { list_init(&W.L[l]); Wp.cut[l] = nextafterf(R2, 0.f); list_init(&Wp.L[l]); }
    Wc = W;
    packet_visit(&W, 0, 0);
    b_nodes += W.nodes;
    b_ins += W.ins;
    packet_visit(&Wp, 0, 0);
    b_plain += Wp.nodes;
    packet_visit(&Wc, 0, 1);
    c_nodes += Wc.nodes;
    c_buckets += Wc.buckets;
    c_pts += Wc.bucket_pts;
    c_ins += Wc.ins;
    int m = 0;
    for (int l = 0; l < 64; l++) m = Wc.lins[l] > m ? Wc.lins[l] : m;
    c_maxins += m;
    m = 0;
    for (int l = 0; l < 64; l++) m = W.lins[l] > m ? W.lins[l] : m;
    b_maxins += m;
  }
  const double S = sample;
  if (regroup_blocks) regroup_model(Q, ord, nq, lt, nl, regroup_blocks);
  printf("photons %d queries %ld waves %ld (sampled %d)\n", N, nq, nwaves, sample);
  printf("A per-lane JUMP walk, seeded: loads/lane %.1f, wave max %.1f (plain cut: wave max %.1f), inserts/lane %.1f\n",
         a_mean / S / 64, a_max / S, a_plain_max / S, a_ins / S / 64);
  printf("B packet walk, seeded: nodes/wave %.1f (plain cut %.1f), inserts/lane %.1f (max lane %.1f)\n", b_nodes / S,
         b_plain / S, b_ins / S / 64, b_maxins / S);
  printf("C packet + %d-node buckets: nodes/wave %.1f, buckets/wave %.1f (%.0f points), inserts/lane %.1f (max lane %.1f)\n",
         BUCKET, c_nodes / S, c_buckets / S, c_pts / S, c_ins / S / 64, c_maxins / S);
  printf("E per-lane bucketed walk (%d-node buckets): top nodes/lane %.1f (wave max %.1f), buckets/lane %.1f, "
         "points/lane %.1f (wave max %.1f), inserts/lane %.1f; VALU model wave max %.0f vs A %.0f\n",
         BUCKET, e_nodes / S / 64, e_max_nodes / S, e_buckets / S / 64, e_pts / S / 64, e_max_pts / S, e_ins / S / 64,
         e_max_cost / S, 55.0 * a_max / S);
  for (int pol = 0; pol < 3; pol++)
    printf("D lockstep wave (QL %d, %s rounds): iterations %.1f, rounds %.1f, inserts/lane %.1f\n", QL,
           pol == 2 ? "filtered pop-one" : pol ? "batch-merge" : "pop-one", d_it[pol] / S, d_rounds[pol] / S,
           d_ins[pol] / S / 64);
  for (int v = 0; v < 3; v++)
    printf("Z own subtree of %d nodes: cut/exact mean %.3f, iterations %.1f, rounds %.1f, VALU %.0f\n",
           (2 << (5 + v)) - 1, z_ratio[v] / z_n[v], z_it[v] / S, z_rd[v] / S, (z_it[v] * 60 + z_rd[v] * 111) / S);
  for (int v = 0; v < 2; v++)
    printf("G bucketed bottom (DB %d), %s cut: iterations %.1f, rounds %.1f, VALU %.0f vs current walk %.0f\n", DB,
           v ? "exact" : "seeded", g_it[v] / S, g_rd[v] / S, g_c[v] / S, d_c[v] / S);
  if (getenv("BOXCMP")) {   // per-lane steps, plain vs box-distance pruning, seeded followers + leaders
    double sa[4] = {0}, mx[4] = {0}, ls[4] = {0}, lw[4] = {0};
    for (int b = 0; b < 4; b++) {
      BOXD = b;
      srand(555);
      for (int s2 = 0; s2 < 200; s2++) {
        const long t0 = (long)((double)rand() / RAND_MAX * (nwaves - 2)) * 64;
        double wm = 0;
        for (int l = 0; l < 64; l++) {
          const long r = FRANK(t0 + l);
          const float* q = &Q[3 * ord[r]];
          const long jp = r / STRIDE;
          double bb = 1e300;
          for (long j = jp - 1; j <= jp + 2; j++)
            if (j >= 0 && j < nl) {
              if (lt[j] < -2.f) { BOXD = 0; walk_lane(&Q[3 * ord[j * STRIDE]], nextafterf(R2, 0.f), &L, &dummy); BOXD = b;
                                  lt[j] = L.n >= K ? key_d2(L.key[K - 1]) : -1.f; }
              bb = fmin(bb, seed_bound(&Q[3 * ord[j * STRIDE]], lt[j], q));
            }
          const float cut = bb < R2 ? (float)bb * (1.f + 1e-7f) : nextafterf(R2, 0.f);
          int ins = 0;
          const int st = walk_lane(q, cut, &L, &ins);
          sa[b] += st;
          if (st > wm) wm = st;
        }
        mx[b] += wm;
      }
      const long nw2 = nl / 64;
      for (long wv = 0; wv < nw2; wv++) {
        double wm = 0;
        for (int l = 0; l < 64; l++) {
          int ins = 0;
          const int st = walk_lane(&Q[3 * ord[(wv * 64 + l) * STRIDE]], nextafterf(R2, 0.f), &L, &ins);
          ls[b] += st;
          if (st > wm) wm = st;
        }
        if (wm > lw[b]) lw[b] = wm;
      }
      ls[b] /= nw2 * 64;
    }
    BOXD = 0;
    for (int b = 0; b < 4; b++)
      printf("BOX%d followers: mean lane steps %.1f, mean wave max %.1f; leaders: mean %.1f, worst %.0f\n", b,
             sa[b] / 200 / 64, mx[b] / 200, ls[b], lw[b]);
  }
  if (getenv("LEADALL")) {   // every leader wave with the plain cut: worst waves
    const long nw = nl / 64;
    int worst[5] = {0}; long wj[5] = {0};
    double tot = 0;
    for (long wv = 0; wv < nw; wv++) {
      static const float* lq[64];
      static float lc[64];
      for (int l = 0; l < 64; l++) { lq[l] = &Q[3 * ord[(wv * 64 + l) * STRIDE]]; lc[l] = nextafterf(R2, 0.f); }
      int rd = 0;
      const int it = wave_lockstep(lq, lc, 0, &rd, &(long){0});
      tot += it;
      for (int k = 0; k < 5; k++) if (it > worst[k]) { for (int m = 4; m > k; m--) { worst[m] = worst[m-1]; wj[m] = wj[m-1]; } worst[k] = it; wj[k] = wv; break; }
    }
    // R: close-path seed with retry: cut0 = F x max d2 of the last 6 close-path nodes;
    // a lane whose list does not fill walks again with the plain cut
    for (int fv = 0; fv < 3; fv++) {
      const float F = fv == 0 ? 4.f : (fv == 1 ? 16.f : 64.f);
      double rt = 0, rmax = 0, fails = 0;
      long rw[3] = {0};
      for (long wv = 0; wv < nw; wv++) {
        double wmax = 0;
        for (int l = 0; l < 64; l++) {
          const float* q = &Q[3 * ord[(wv * 64 + l) * STRIDE]];
          int t = 0, dep = 0;
          float last[64];
          int nl2 = 0;
          while (t < N) {
            const Node* nd = &T[t];
            last[nl2++] = dist2(q, nd);
            const float diff = q[nd->dim] - nd->p[nd->dim];
            t = 2 * t + 1 + (diff > 0.f);
            dep++;
          }
          float mx = 0.f;
          for (int i = nl2 - 6 < 0 ? 0 : nl2 - 6; i < nl2; i++) mx = fmaxf(mx, last[i]);
          const float c0 = fminf(mx * F, nextafterf(R2, 0.f));
          int ins = 0;
          double cost = dep + walk_lane(q, c0, &L, &ins);
          if (L.n < K && c0 < nextafterf(R2, 0.f)) { cost += walk_lane(q, nextafterf(R2, 0.f), &L, &ins); fails++; }
          rt += cost;
          if (cost > wmax) wmax = cost;
        }
        rmax += wmax;
        if (wmax > rw[0]) rw[0] = (long)wmax;
      }
      printf("R close-path seed x%g + retry: mean lane steps %.1f, mean wave max %.1f, worst wave %ld, lanes retried %.3f%%\n", F,
             rt / nw / 64, rmax / nw, rw[0], fails / nw / 64 * 100);
    }
    {
      double pt = 0, pmax = 0, pw = 0;
      for (long wv = 0; wv < nw; wv++) {
        double wmax = 0;
        for (int l = 0; l < 64; l++) {
          int ins = 0;
          const double c = walk_lane(&Q[3 * ord[(wv * 64 + l) * STRIDE]], nextafterf(R2, 0.f), &L, &ins);
          pt += c;
          if (c > wmax) wmax = c;
        }
        pmax += wmax;
        if (wmax > pw) pw = wmax;
      }
      printf("R plain cut: mean lane steps %.1f, mean wave max %.1f, worst wave %.0f\n", pt / nw / 64, pmax / nw, pw);
    }
    printf("LA all %ld leader waves: mean iterations %.1f, worst %d %d %d %d %d (waves %ld %ld ...)\n", nw, tot / nw,
           worst[0], worst[1], worst[2], worst[3], worst[4], wj[0], wj[1]);
    // the worst wave's lanes
    {
      const long wv = wj[0];
      for (int l = 0; l < 64; l++) {
        const float* q = &Q[3 * ord[(wv * 64 + l) * STRIDE]];
        int ins = 0;
        const int st = walk_lane(q, nextafterf(R2, 0.f), &L, &ins);
        if (st > 2000) {
          printf("  lane %d q (%g %g %g) steps %d inserts %d kth d2 %g\n", l, q[0], q[1], q[2], st, ins,
                 L.n >= K ? key_d2(L.key[K - 1]) : -1.f);
          VERBOSE = 1;
          { int ii = 0; const float vc = getenv("VCUT") ? (float)atof(getenv("VCUT")) : nextafterf(R2, 0.f);
            const int st2 = walk_lane(q, vc, &L, &ii); printf("    verbose walk with cut %g: steps %d\n", vc, st2); }
          VERBOSE = 0;
          // replay: nodes entered as FAR children, by split dim and |diff|
          static long hist[3][4];
          memset(hist, 0, sizeof hist);
          const float b = L.n >= K ? key_d2(L.key[K - 1]) : R2;
          // exact-bound recursive search counting visits
          long visits = 0;
          int stk[256], sp = 0;
          stk[sp++] = 0;
          while (sp) {
            const int t = stk[--sp];
            if (t >= N) continue;
            visits++;
            const Node* nd = &T[t];
            const float diff = q[nd->dim] - nd->p[nd->dim];
            const int close = 2 * t + 1 + (diff > 0.f), far = 2 * t + 2 - (diff > 0.f);
            if (far < N && diff * diff <= b) {
              stk[sp++] = far;
              hist[nd->dim][diff == 0.f ? 0 : (diff * diff < 1e-8f ? 1 : (diff * diff < b * 0.25f ? 2 : 3))]++;
            }
            stk[sp++] = close;
          }
          printf("    exact-bound visits %ld; far entries by dim [diff==0, tiny, <r/2, rest]: x %ld %ld %ld %ld y %ld %ld %ld %ld z %ld %ld %ld %ld\n",
                 visits, hist[0][0], hist[0][1], hist[0][2], hist[0][3], hist[1][0], hist[1][1], hist[1][2], hist[1][3],
                 hist[2][0], hist[2][1], hist[2][2], hist[2][3]);
          break;
        }
      }
    }
  }
  if (getenv("LEADZ")) {   // leader waves (64 leaders, ranks 16 apart): plain cut vs own-subtree seeds
    double it0 = 0, rd0 = 0, it1[3] = {0}, rd1[3] = {0};
    srand(99);
    const int LS = 100;
    for (int s = 0; s < LS; s++) {
      const long j0 = (long)((double)rand() / RAND_MAX * (nl - 70));
      static const float* lq[64];
      static float lc[64], zc[64];
      for (int l = 0; l < 64; l++) { lq[l] = &Q[3 * ord[(j0 + l) * STRIDE]]; lc[l] = nextafterf(R2, 0.f); }
      int rd = 0;
      it0 += wave_lockstep(lq, lc, 0, &rd, &(long){0});
      rd0 += rd;
      for (int v = 0; v < 3; v++) {
        const int h = 5 + v;
        for (int l = 0; l < 64; l++) {
          const float* q = lq[l];
          zc[l] = nextafterf(R2, 0.f);
          int t = 0, dep = 0;
          while (dep < DB + 2 - h) {
            const Node* nd = &T[t];
            const float diff = q[nd->dim] - nd->p[nd->dim];
            const int c = 2 * t + 1 + (diff > 0.f);
            if (c >= N) break;
            t = c; dep++;
          }
          static float d[1024];
          int m = 0;
          for (int lev = 0; lev <= h; lev++)
            for (long j = 0; j < (1L << lev); j++) {
              const long c = (long)(t + 1) * (1L << lev) - 1 + j;
              if (c < N) d[m++] = dist2(q, &T[c]);
            }
          if (m >= K) {
            qsort(d, m, sizeof(float), cmp_fl);
            const float b = d[K - 1] * (1.f + 1e-6f);
            if (b < zc[l]) zc[l] = b;
          }
        }
        rd = 0;
        it1[v] += wave_lockstep(lq, zc, 0, &rd, &(long){0});
        rd1[v] += rd;
      }
    }
    printf("L leader waves, plain cut: iterations %.1f, rounds %.1f\n", it0 / LS, rd0 / LS);
    for (int v = 0; v < 3; v++)
      printf("L leader waves, own-subtree (%d nodes) seed: iterations %.1f, rounds %.1f\n", (2 << (5 + v)) - 1,
             it1[v] / LS, rd1[v] / LS);
  }
  if (getenv("POOL")) {   // P: pooled lanes over 4 waves' worth of consecutive followers
    double pit[3] = {0}, prd[3] = {0};
    const int refills[3] = {1, 8, 16};
    srand(4242);
    const int PS = 100;
    for (int s = 0; s < PS; s++) {
      const long t0 = (long)((double)rand() / RAND_MAX * (nwaves - 8)) * 64;
      static const float* pq[256];
      static float pc[256];
      for (int i = 0; i < 256; i++) {
        const long r = FRANK(t0 + i);
        const float* q = &Q[3 * ord[r]];
        float cut = nextafterf(R2, 0.f);
        const long jp = r / STRIDE;
        double b = 1e300;
        for (long j = jp - 1; j <= jp + 2; j++)
          if (j >= 0 && j < nl) {
            if (lt[j] < -2.f) {   // leader not walked yet
              walk_lane(&Q[3 * ord[j * STRIDE]], nextafterf(R2, 0.f), &L, &dummy);
              lt[j] = L.n >= K ? key_d2(L.key[K - 1]) : -1.f;
            }
            b = fmin(b, seed_bound(&Q[3 * ord[j * STRIDE]], lt[j], q));
          }
        if (b < cut) cut = (float)b * (1.f + 1e-7f);
        pq[i] = q; pc[i] = cut;
      }
      for (int v = 0; v < 3; v++) {
        int rd = 0;
        pit[v] += pool_lockstep(pq, pc, 256, refills[v], &rd);
        prd[v] += rd;
      }
      // static: 4 waves of 64
      for (int w = 0; w < 4; w++) {
        int rd = 0;
        pit_static += wave_lockstep(pq + 64 * w, pc + 64 * w, 0, &rd, &(long){0});
        prd_static += rd;
      }
    }
    printf("P static 4 waves x 64: iterations %.1f, rounds %.1f per 256 queries\n", pit_static / PS, prd_static / PS);
    for (int v = 0; v < 3; v++)
      printf("P pooled 256 queries, refill at %d idle: iterations %.1f, rounds %.1f\n", refills[v], pit[v] / PS, prd[v] / PS);
  }
  if (g_net_rounds > 0)
    printf("partial networks (checkpoint %d): mean entries per round %.1f of %d (rounds with an insert %.0f)\n", NETCP,
           g_net_entries / g_net_rounds, K, g_net_rounds);
  printf("seeded (triangle) cut / exact k-th d2: mean %.3f\n", s_ratio / s_n);
  for (int v = 0; v < 8; v++)
    printf("Y %s leader list kk=%d: cut/exact mean %.3f, iterations %.1f, rounds %.1f\n", v >> 2 ? "two" : "nearest",
           (int[]){50, 64, 96, 128}[v & 3], y_ratio[v] / y_n[v], y_it[v] / S, y_rounds[v] / S);
  for (int f = 0; f < 4; f++)
    printf("X lockstep, cut = min(seeded, exact k-th d2 x %.2f): iterations %.1f, rounds %.1f\n",
           (double)(f == 0 ? 1.0f : f == 1 ? 1.15f : f == 2 ? 1.5f : 2.0f), x_it[f] / S, x_rounds[f] / S);
  return 0;
}
