// pm_internal.hpp — handle layouts and kernel-launch entry points shared by the
// translation units of libpm_hip.so (not part of the public C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/pm.h"
#include "pm_device.hpp"
#include "prims.hpp"

// Device-resident scene: triangles in BVH leaf order + BVH4 nodes + materials.
struct pm_scene {
  pmd::DevBuf<float4> tri;      // 3 per triangle
  pmd::DevBuf<float4> nodes;    // 8 per BVH4 node
  pmd::DevBuf<float4> mat;      // 2 per mesh
  pmd::DevBuf<int32_t> overflow;
  int32_t ntri = 0, nnodes = 0, nmesh = 0, depth = 0;
  int device = 0;   // the HIP device its memory lives on (the creating thread's current device)
  pm_box bounds{};
  std::vector<pm_material> host_mat;
  pmd::DevScene view() const {
    pmd::DevScene s;
    s.tri = tri.p;
    s.nodes = nodes.p;
    s.mat = mat.p;
    s.ntri = ntri;
    s.nnodes = nnodes;
    return s;
  }
};

// Photon map: left-balanced kd-tree nodes (x, y, z, bits(orig<<2 | dim)) in
// kd order + gather payload (color.xyz, power) in ORIGINAL order.
struct pm_photon_map {
  pmd::DevBuf<float4> nodes;
  pmd::DevBuf<float4> payload;
  int64_t n = 0;
  hipStream_t made_on = nullptr;   // its memory returns to this stream's allocator pool
  int device = 0;                  // the device of made_on
};

// PM_CHECK_VARIANT (build-time, tests only: lib_check/libpm_hip.so): every
// alternate path that must give bit-identical results in one library -- the
// plain kNN walk instead of the leader-seeded one, all-global kd levels instead
// of the LDS finish, the Karras LBVH instead of PLOC, a one-slot first guess
// for the render's continuation vertices (always rerun), the per-bounce
// wavefront photon trace instead of the fused paths (the Makefile's check
// target sets PM_TRACE_FUSED=0) -- plus a 4-entry LDS
// traversal stack (PM_STACK_DEPTH=4: nearly every ray spills to scratch).
// tests/test_gpu_check_variant.py compares it with the production library.
#ifndef PM_CHECK_VARIANT
#define PM_CHECK_VARIANT 0
#endif

namespace pmd {

// Largest photon map / kd-tree: node tags are int32 (original index << 2 | split
// dimension), so every original index must stay below 2^29 for the tag to stay
// non-negative (ids >= 2^29 would sign-extend when decoded).
constexpr int64_t kMaxMapPhotons = int64_t(1) << 29;

// Light for the photon tracer: pos.xyz, rgb.xyz, rgb.w = type (0 point,
// 1 square), nrm = (normal.xyz, side length).
struct LightDev {
  float4 pos;
  float4 rgb;
  float4 nrm;
};

// One photon set of a trace launch (trace.hip): photons [g_lo, g_lo + np) of the
// set's global index range (per-light offsets loff, device), its mode, and its
// deposit slots (deposit k of photon i at slots[k * np + i]) and counts.
struct PathSet {
  const int64_t* loff = nullptr;
  int64_t g_lo = 0, np = 0;
  int caustic = 0;
  pm_photon* slots = nullptr;
  uint32_t* cnt = nullptr;
};
// Both sets in one launch (B.np may be 0; see launch_trace_fused).
hipError_t launch_trace_sets(pm_scene* sc, const LightDev* d_lights, int nl, PathSet A, PathSet B, int maxd,
                             hipStream_t s);

// phase timers (pm_last_phase_us)
enum Phase { PH_TRACE = 0, PH_COMPACT = 1, PH_KDBUILD = 2, PH_PATHS = 3, PH_GATHER = 4, PH_RESOLVE = 5, PH_BVH = 6,
             PH_GATHER_GLOBAL = 7, PH_COUNT = 8 };
struct PhaseTimer {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s = nullptr;
  int phase;
  PhaseTimer(int ph, hipStream_t st);
  ~PhaseTimer();
};
void record_phase_us(int phase, double us);

hipError_t build_lbvh(pm_scene* sc, const std::vector<float4>& tri_host, hipStream_t s);

// Core left-balanced kd-tree build over elements (x, y, z, bits(orig)).
// Writes nodes[t] = (x, y, z, bits(orig << 2 | dim)).
hipError_t kd_build(const float4* d_elems, int64_t n, float4* d_nodes, hipStream_t s);

// Sharded build of one tree (kdshard.hip).
int shard_levels(int world);
bool shard_ok(int64_t n, int L);
hipError_t kd_shard_top(const float4* elems, int64_t n, int L, float4* top, std::vector<int64_t>& sizes,
                        hipStream_t s);
hipError_t kd_shard_classify(const float4* elems, int64_t n, int L, const float4* top, uint8_t* sub, hipStream_t s);
// Per-tile start of every subtree's elements (once per plan, nb = 2^L subtrees):
// boff[j * tiles + t] = elements of subtrees < j, plus those of subtree j in
// tiles < t (kShardExtTile elements per tile); sized by kd_shard_tiles.
int64_t kd_shard_tiles(int64_t n);
hipError_t kd_shard_offsets(const uint8_t* subof, int64_t n, int nb, const int64_t* expect, uint32_t* boff,
                            hipStream_t s);
hipError_t kd_shard_subtree(const float4* elems, const uint8_t* subof, const uint32_t* boff, int64_t n, int j,
                            int64_t size, int32_t* out, hipStream_t s);
hipError_t kd_shard_assemble(const float4* elems, const float4* top, int L, const int32_t* tags,
                             const std::vector<int64_t>& sizes, float4* nodes, hipStream_t s);
struct ShardSel {
  int dim[16];
  uint64_t prefix[16];   // key bits above `shift + 8` selected so far
};
// Distributed top selection (kdshard.hip): the rank's own photons with their
// global indices (a: aid + i, b: bid + i); step() issues one pass into the
// caller's int64 buffer (op 1: SUM, 2: MIN across ranks, 0: finished) after
// consuming the caller's reduction of the previous one.
struct KdTopSel {
  DevBuf<float4> elems, top;
  DevBuf<uint32_t> ob, hist;
  DevBuf<uint64_t> off, cand;
  DevBuf<unsigned long long> cnt;
  int64_t n = 0;   // local elements
  int64_t seg_total = 0;   // the gathered map's size
  int L = 0, level = 0, pending = -1;   // pending: 0 bounds, 1-2 top-byte histograms, 3-8 candidate histograms
  std::vector<int64_t> seg, rank, ncand;
  std::vector<uint64_t> ho;
  ShardSel sel{};
  hipError_t init(const pm_photon* a, int64_t na, int64_t aid, const pm_photon* b, int64_t nb, int64_t bid,
                  int64_t n_total, int levels, hipStream_t s);
  hipError_t step(int64_t* red, int64_t* count, int* op, hipStream_t s);
  hipError_t issue(int64_t* red, int64_t* count, int* op, hipStream_t s);
  hipError_t consume(const int64_t* red, hipStream_t s);
};
hipError_t kd_shard_top_fix(const float4* elems, float4* top, int L, hipStream_t s);
// One contiguous run of photon rows (pm_photon_rows segment, or a whole
// pm_photon array): n rows of `stride` floats, position at 0..2, colour at
// coff..coff+2, gather power `power`. A map's photons are a list of runs,
// concatenated in order (original index = position in the concatenation).
struct RowRun {
  const float* rows;
  int stride, coff;
  int64_t n;
  float power;
};
using RowRuns = std::vector<RowRun>;
int64_t rows_total(const RowRuns& runs);
// elements (x, y, z, original index) + payload (colour, power), one launch per run
hipError_t launch_elems_from_rows(const RowRuns& runs, float4* elems, float4* payload, hipStream_t s);
// the same and each element's subtree below the top L levels (top_path), one pass
hipError_t kd_shard_elems_classify(const RowRuns& runs, const float4* top, int L, float4* elems, float4* payload,
                                   uint8_t* sub, hipStream_t s);

// gatherPhotons over k != 50 neighbours (pm_knn passes + one summing kernel).
hipError_t launch_gather_k(const pm_photon_map* m, const float4* d_query, int64_t nq, float4* d_out, hipStream_t s,
                           int k, const uint32_t* perm);

// K = 50 gather (gatherPhotons) for a batch of queries.
// tag 0: API / caustic-map launches, 1: global-map launch (separate kernel symbol for rocprof)
hipError_t launch_gather(const pm_photon_map* m, const float4* d_query /*pos, brdf*/, int64_t nq,
                         float4* d_out, hipStream_t s, int tag = 0, const uint32_t* perm = nullptr);

}  // namespace pmd
