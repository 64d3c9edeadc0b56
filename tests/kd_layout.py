"""The kd-tree layout expected from the oracle (oracle.kd_left_balanced: the
in-place left-balanced tree of cukd::buildTree, ray-tracer/src/hostCode.cu:
94-95, as this build specifies it): the records a HIP build must produce, node
for node, so the GPU tests can compare them bit for bit. SPEC-PINNED,
CUKD-UNPINNED: the split dimension from the subtree's point extent and the
tie order by original index are this build's rules (oracle/pm_oracle.c, the
layout header); cudaKDTree itself is absent.
  - map_records: pm_photon_map_export's output for a map built from photon
    sets (loadPhotons order, ray-tracer/src/hostCode.cu:54-99: a ++ b, their
    powers); a NaN coordinate is stored as +inf (include/pm.h), dir is zero;
  - inplace_records: pm_kdtree_build's in-place reorder of kd records, the
    record of node t is input[orig(t)] with split_dim set (photon.h:36-39)."""
import numpy as np

import oracle


def _split_dim_word(tags, base_word):
    """word 10 of a pm_kd_photon: quantized_normal[3] then split_dim (high byte)"""
    return (base_word & np.uint32(0x00FFFFFF)) | ((tags & 3).astype(np.uint32) << np.uint32(24))


def map_records(parts, nthreads=8):
    """parts: [(pm_photon rows (n, 10) float32, power), ...] in map order"""
    pos = np.concatenate([np.asarray(p, np.float32)[:, 0:3] for p, _ in parts]) if parts else np.zeros((0, 3))
    pos = np.ascontiguousarray(np.where(np.isnan(pos), np.float32(np.inf), pos), np.float32)
    col = np.concatenate([np.asarray(p, np.float32)[:, 7:10] for p, _ in parts])
    pw = np.concatenate([np.full(len(p), w, np.float32) for p, w in parts])
    tags = oracle.kd_left_balanced(pos, nthreads)
    orig = (tags.view(np.uint32) >> 2).astype(np.int64)
    out = np.zeros((len(pos), 11), np.float32)
    out[:, 0:3] = pos[orig]
    out[:, 6:9] = col[orig]
    out[:, 9] = pw[orig]
    ov = out.view(np.uint32)
    ov[:, 10] = _split_dim_word(tags, np.uint32(0))
    return out, tags


def inplace_records(rec, nthreads=8):
    """rec: (n, 11) pm_kd_photon rows before pm_kdtree_build"""
    rec = np.ascontiguousarray(rec, np.float32)
    tags = oracle.kd_left_balanced(rec, nthreads)
    orig = (tags.view(np.uint32) >> 2).astype(np.int64)
    out = rec[orig].copy()
    ov = out.view(np.uint32)
    ov[:, 10] = _split_dim_word(tags, ov[:, 10])
    return out, tags


def assert_same(got, want, what=""):
    g = np.ascontiguousarray(got, np.float32).view(np.uint32)
    w = np.ascontiguousarray(want, np.float32).view(np.uint32)
    assert g.shape == w.shape, (what, g.shape, w.shape)
    bad = np.nonzero(np.any(g != w, axis=1))[0]
    assert len(bad) == 0, f"{what}: {len(bad)} of {len(g)} kd nodes differ from the oracle layout, " \
                          f"first at node {bad[0]}: got {got[bad[0]]} want {want[bad[0]]}"
