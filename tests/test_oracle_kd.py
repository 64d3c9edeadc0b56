"""The oracle's restatement of cukd::buildTree's left-balanced layout
(ray-tracer/src/hostCode.cu:94-95, traits ray-tracer/include/photon.h:23-40;
rules in DESIGN.md §4.3) checked on the CPU against a second, independent
restatement written here with numpy: a full sort of each subtree by (orderable
coordinate key, original index) instead of the oracle's quickselect, and a
brute-force left_size from the complete-tree shape. The GPU tests then compare
pm_kdtree_build / pm_photon_map_export node for node with the oracle
(tests/test_gpu_parity.py, test_gpu_workloads.py, test_gpu_fullsize.py)."""
import numpy as np
import pytest

import oracle


def _okey(c):
    c = np.where(np.isnan(c), np.float32(np.inf), c).astype(np.float32)
    c = np.where(c == 0, np.float32(0.0), c).astype(np.float32)
    u = c.view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def _unkey(k):
    k = np.uint32(k)
    u = (k & np.uint32(0x7FFFFFFF)) if (k & np.uint32(0x80000000)) else ~k
    return np.array([u], np.uint32).view(np.float32)[0]


def _left_size_shape(s):
    """left subtree size of the complete binary tree with s nodes, by counting
    the heap-order nodes 0..s-1 that lie under node 1"""
    cnt, lo, width = 0, 1, 1
    while lo < s:
        cnt += min(width, s - lo)
        lo, width = 2 * lo + 1, width * 2
    return cnt


def _numpy_layout(pos):
    n = len(pos)
    keys = np.stack([_okey(pos[:, d]) for d in range(3)], 1)
    tags = np.full(n, -1, np.int64)

    def build(t, ids):
        s = len(ids)
        if s == 0:
            return
        ext = [np.float32(_unkey(keys[ids, d].max()) - _unkey(keys[ids, d].min())) for d in range(3)]
        dim = 0
        for d in (1, 2):
            if ext[d] > ext[dim]:
                dim = d
        order = ids[np.lexsort((ids, keys[ids, dim]))]
        ls = _left_size_shape(s)
        tags[t] = (int(order[ls]) << 2) | dim
        build(2 * t + 1, order[:ls])
        build(2 * t + 2, order[ls + 1:])

    build(0, np.arange(n))
    assert (tags >= 0).all()
    return tags.astype(np.int32)


def test_left_size_matches_tree_shape():
    for s in list(range(0, 300)) + [2 ** 20 - 1, 2 ** 20, 2 ** 20 + 1, 45_400_123]:
        want = _left_size_shape(s) if s < 10 ** 6 else None
        got = oracle.left_size(s)
        if want is not None:
            assert got == want, s
        assert 0 <= got <= max(0, s - 1)
        # right subtree is never larger than the left one, nor smaller than half of it
        r = s - 1 - got if s else 0
        assert r <= got and (s < 2 or r >= (got - 1) // 2)


def _cloud(n, seed, kind):
    rng = np.random.default_rng(seed)
    p = rng.uniform(-20, 20, size=(n, 3)).astype(np.float32)
    if kind == "ties":
        p = (np.round(p / 2.5) * 2.5).astype(np.float32)
        p[rng.random(n) < 0.2, 1] = -0.0
    elif kind == "dups":
        if n:
            p[: n // 3] = p[0]
    elif kind == "special":
        m = rng.random((n, 3))
        p[m < 0.05] = np.nan
        p[(m >= 0.05) & (m < 0.1)] = np.inf
        p[(m >= 0.1) & (m < 0.15)] = -np.inf
        p[(m >= 0.15) & (m < 0.25)] = -0.0
    elif kind == "plane":
        p[:, 2] = 1.0
    elif kind == "flat":   # every extent zero: dimension 0 on the tie
        p[:] = 3.0
    return p


@pytest.mark.parametrize("kind", ["uniform", "ties", "dups", "special", "plane", "flat"])
@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 100, 1023, 1025, 3001])
def test_oracle_layout_vs_numpy(kind, n):
    pos = _cloud(n, n * 7 + len(kind), kind)
    got = oracle.kd_left_balanced(pos, nthreads=4)
    assert np.array_equal(got, _numpy_layout(pos)), (kind, n)


def test_oracle_layout_is_a_permutation_and_threads_agree():
    pos = _cloud(300_001, 3, "ties")
    a = oracle.kd_left_balanced(pos, nthreads=1)
    b = oracle.kd_left_balanced(pos, nthreads=8)
    assert np.array_equal(a, b)
    orig = a.view(np.uint32) >> 2
    assert np.array_equal(np.sort(orig), np.arange(len(pos), dtype=np.uint32))
    assert ((a & 3) <= 2).all()


def test_oracle_layout_stride_and_invariant():
    """strided records (pm_kd_photon is 11 floats) and the left-balanced
    ancestor invariant on the oracle's own output"""
    rng = np.random.default_rng(5)
    rec = np.zeros((20_000, 11), np.float32)
    rec[:, 0:3] = rng.uniform(-5, 5, size=(20_000, 3))
    tags = oracle.kd_left_balanced(rec)
    assert np.array_equal(tags, oracle.kd_left_balanced(np.ascontiguousarray(rec[:, 0:3])))
    pos = rec[(tags.view(np.uint32) >> 2).astype(np.int64), 0:3]
    dims = (tags & 3).astype(np.int64)
    n = len(pos)
    node = np.arange(n)
    cur = node.copy()
    while True:
        parent = (cur + 1) // 2 - 1
        m = parent >= 0
        node, cur, parent = node[m], cur[m], parent[m]
        if len(node) == 0:
            break
        left = cur == 2 * parent + 1
        d = dims[parent]
        assert np.all(pos[node[left], d[left]] <= pos[parent[left], d[left]])
        assert np.all(pos[node[~left], d[~left]] >= pos[parent[~left], d[~left]])
        cur = parent
