"""Known-answer tests pinning the CPU oracle (no GPU).

The reference ships no tests or golden vectors, so the
oracle is pinned by: independent re-implementations (Python big-int LCG,
numpy float32 kNN / radiance estimate), hand-computed geometry, analytic
accuracy bounds for the deterministic trig, semantics of the reference's host
arithmetic (photons per watt), and internal consistency (BVH == brute force).
"""
import ctypes as C
import math

import numpy as np
import pytest

import conftest


def py_lcg_init(v0, v1):
    """owl::LCG<16>::init restated with Python ints (independent of the C oracle)."""
    M = 0xFFFFFFFF
    s0 = 0
    for _ in range(16):
        s0 = (s0 + 0x9E3779B9) & M
        v0 = (v0 + ((((v1 << 4) & M) + 0xA341316C) ^ ((v1 + s0) & M) ^ (((v1 >> 5) + 0xC8013EA4) & M))) & M
        v0 &= M
        v1 = (v1 + ((((v0 << 4) & M) + 0xAD90777D) ^ ((v0 + s0) & M) ^ (((v0 >> 5) + 0x7E95761E) & M))) & M
    return v0


def py_lcg_draws(state, n):
    out = []
    for _ in range(n):
        state = (1664525 * state + 1013904223) & 0xFFFFFFFF
        out.append(np.float32((state & 0xFFFFFF) / 16777216.0))
    return out


@pytest.mark.parametrize("seed", [(0, 0), (1, 0), (600, 330), (4999, 0), (1919, 1079), (0xFFFFFFFF, 7)])
def test_lcg_known_answers(seed):
    import oracle
    st = oracle.lib.orc_lcg_init(*seed)
    assert st == py_lcg_init(*seed)
    s = C.c_uint32(st)
    got = [oracle.lib.orc_lcg_next(C.byref(s)) for _ in range(16)]
    exp = py_lcg_draws(st, 16)
    assert np.array_equal(np.float32(got), np.float32(exp))


def test_trig_accuracy():
    import oracle
    xs = np.linspace(-1, 1, 20001, dtype=np.float32)
    a = np.array([oracle.lib.orc_acosf(float(x)) for x in xs], np.float32)
    # A&S 4.4.46 (|eps| <= 2e-8) + float32 rounding of values up to pi (ulp 2.4e-7)
    assert np.abs(a.astype(np.float64) - np.arccos(xs.astype(np.float64))).max() < 5e-7
    ts = np.linspace(0, 2 * np.pi, 20001, dtype=np.float32)
    s = np.array([oracle.lib.orc_sinf(float(t)) for t in ts], np.float64)
    c = np.array([oracle.lib.orc_cosf(float(t)) for t in ts], np.float64)
    assert np.abs(s - np.sin(ts.astype(np.float64))).max() < 4e-7
    assert np.abs(c - np.cos(ts.astype(np.float64))).max() < 4e-7


def test_random_point_in_unit_sphere_is_unit():
    import oracle
    st = C.c_uint32(oracle.lib.orc_lcg_init(3, 0))
    out = (C.c_float * 3)()
    v = []
    for _ in range(2000):
        oracle.lib.orc_random_point_in_unit_sphere(C.byref(st), out)
        v.append(list(out))
    v = np.array(v)
    assert np.abs(np.linalg.norm(v, axis=1) - 1).max() < 2e-6
    assert np.abs(v.mean(0)).max() < 0.06       # roughly uniform on the sphere


def test_refract_cases():
    import oracle
    out = (C.c_float * 3)()
    # normal incidence passes straight through (helpers.h:57-74)
    oracle.lib.orc_refract((C.c_float * 3)(0, -1, 0), (C.c_float * 3)(0, 1, 0), 1.5, out)
    assert np.allclose(list(out), [0, -1, 0], atol=1e-7)
    # oblique entry: Snell's law with mu = 1/1.5
    d = np.array([math.sin(0.5), -math.cos(0.5), 0], np.float32)
    oracle.lib.orc_refract((C.c_float * 3)(*d), (C.c_float * 3)(0, 1, 0), 1.5, out)
    r = np.array(list(out))
    assert abs(r[0] / np.linalg.norm(r) - math.sin(0.5) / 1.5) < 1e-6
    # total internal reflection from inside falls back to reflect: exiting at
    # grazing angle with the unflipped normal (cosTheta <= 0 -> mu = ior)
    d = np.array([math.sin(1.2), math.cos(1.2), 0], np.float32)
    oracle.lib.orc_refract((C.c_float * 3)(*d), (C.c_float * 3)(0, 1, 0), 1.5, out)
    assert np.allclose(list(out), [d[0], -d[1], 0], atol=1e-6)


@pytest.mark.parametrize("powers,casted,expected", [
    ((10.0, 10.0), 10000, [5000, 5000]),        # cornell-box lights.txt, 10k
    ((10.0, 10.0), 1_000_000, [500000, 500000]),
    ((10.0, 10.0), 10, [0, 0]),                 # casted < sum P: int ppw == 0
    ((2.5, 7.5), 1000, [250, 750]),
    ((3.3, 1.1), 1000, [749, 249]),             # int(3.3 * 227) = 749: double then int truncation
    ((1000.0,), 500, [0]),
])
def test_photons_per_light(powers, casted, expected):
    import oracle
    import pm_amd
    lights = [{"pos": (0, 0, 0), "rgb": (1, 1, 1), "power": p} for p in powers]
    assert oracle.photons_per_light(lights, casted) == expected
    assert pm_amd.compute_photons_per_watt(lights, casted) == expected


def _tri_scene(tris, mats=None):
    import pm_amd
    meshes = []
    for i, t in enumerate(tris):
        meshes.append(pm_amd.MeshData(np.asarray(t, np.float32).reshape(3, 3), np.array([[0, 1, 2]], np.int32),
                                      np.asarray(mats[i] if mats else (1, 1, 1, 1, 0, 0, 0), np.float32)))
    return meshes


def _rays(o, d, tmin=1e-3, tmax=1e10):
    r = np.zeros((len(o), 8), np.float32)
    r[:, 0:3] = o
    r[:, 3] = tmin
    r[:, 4:7] = d
    r[:, 7] = tmax
    return r


def test_intersection_hand_computed():
    import oracle
    meshes = _tri_scene([[0, 0, 0, 1, 0, 0, 0, 1, 0], [0, 0, -2, 1, 0, -2, 0, 1, -2]])
    for bvh in (False, True):
        s = oracle.Scene(meshes, use_bvh=bvh)
        h = s.intersect(_rays([[0.25, 0.25, 1], [0.25, 0.25, 1], [2, 2, 1], [0.25, 0.25, 1], [0.25, 0.25, -1]],
                              [[0, 0, -1], [0, 0, 1], [0, 0, -1], [1, 0, 0], [0, 0, -1]]))
        t = h[:, 0].view(np.float32)
        assert h[0, 1] == 0 and t[0] == 1.0             # closest of two stacked triangles
        assert h[1, 1] == -1 and h[2, 1] == -1 and h[3, 1] == -1
        assert h[4, 1] == 1 and t[4] == 1.0
        # tmax excludes, tmin excludes
        h = s.intersect(_rays([[0.25, 0.25, 1]] * 2, [[0, 0, -1]] * 2, tmin=np.float32([1e-3, 1.5]),
                              tmax=np.float32([0.5, 1e10])))
        assert h[0, 1] == -1 and h[1, 1] == 1


def test_watertight_shared_edge():
    """Rays through the shared diagonal of a quad hit one of its triangles (OptiX
    triangles are watertight; the oracle restates that with Woop et al. 2013)."""
    import oracle
    quad = [[0, 0, 0, 1, 0, 0, 1, 1, 0], [0, 0, 0, 1, 1, 0, 0, 1, 0]]
    s = oracle.Scene(_tri_scene(quad), use_bvh=False)
    u = np.linspace(0.0, 1.0, 4097, dtype=np.float32)[1:-1]
    o = np.stack([u, u, np.full_like(u, 1.0)], 1)
    d = np.tile(np.float32([[0.0, 0.0, -1.0]]), (len(u), 1))
    # tilted rays too
    o2 = o + np.float32([0.3, -0.1, 0])
    d2 = np.tile(np.float32([[-0.3, 0.1, -1.0]]), (len(u), 1))
    h = s.intersect(_rays(np.concatenate([o, o2]), np.concatenate([d, d2])))
    assert np.all(h[:, 1] >= 0)
    # closest-hit tie on the shared edge resolves to the lower triangle index
    assert np.all(h[: len(u), 3] == 0)


@pytest.mark.parametrize("which", ["cornell", "sphere"])
def test_oracle_bvh_equals_bruteforce(which, request):
    import oracle
    meshes, _ = request.getfixturevalue(which)
    rng = np.random.default_rng(11)
    n = 3000 if which == "sphere" else 20000
    o = rng.uniform([-25, -5, -25], [25, 45, 25], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = _rays(o, d)
    a = oracle.Scene(meshes, use_bvh=True).intersect(r)
    b = oracle.Scene(meshes, use_bvh=False).intersect(r)
    assert np.array_equal(a, b)
    r[:, 7] = 12.0
    assert np.array_equal(oracle.Scene(meshes, use_bvh=True).occluded(r),
                          oracle.Scene(meshes, use_bvh=False).occluded(r))


def _brute_knn(pts, q, k, r):
    diff = (q[:, None, :] - pts[None, :, :]).astype(np.float32)
    d2 = (diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]) + diff[..., 2] * diff[..., 2]
    ids = np.full((len(q), k), -1, np.int32)
    dd = np.full((len(q), k), (np.float32(r) * np.float32(r)), np.float32)
    for i in range(len(q)):
        ok = np.nonzero(d2[i] < (np.float32(r) * np.float32(r)))[0]
        order = ok[np.lexsort((ok, d2[i, ok]))][:k]
        ids[i, : len(order)] = order
        dd[i, : len(order)] = d2[i, order]
    return ids, dd


def test_oracle_knn_vs_numpy_bruteforce():
    import oracle
    rng = np.random.default_rng(5)
    pts = rng.integers(-4, 5, size=(2500, 3)).astype(np.float32)     # lattice: exact ties
    ph = np.zeros((len(pts), 10), np.float32)
    ph[:, :3] = pts
    m = oracle.PhotonMap(ph, 1.0)
    q = rng.uniform(-5, 5, size=(300, 3)).astype(np.float32)
    for k, r in [(50, 100.0), (8, 1.5), (1, 0.7), (64, 2.0)]:
        ids, d2, md = m.knn(q, k, r)
        bi, bd = _brute_knn(pts, q, k, r)
        assert np.array_equal(ids, bi) and np.array_equal(d2.view(np.uint32), bd.view(np.uint32))
        assert np.array_equal(md.view(np.uint32), bd[:, -1].view(np.uint32))


def numpy_gather(pos, col, pw, q, brdf):
    """gatherPhotons (shading.h:93-121) in numpy float32, neighbours in (d^2, id) order."""
    ids, dd = _brute_knn(pos, q[None, :], 50, 100.0)
    r2 = dd[0, -1]
    flux = np.zeros(3, np.float32)
    for j in range(50):
        i = ids[0, j]
        if i < 0:
            continue
        dist = np.sqrt(dd[0, j], dtype=np.float32)
        w = np.float32(1) - (dist / np.sqrt(r2, dtype=np.float32) * np.float32(1.1))
        s = np.float32(brdf) * pw[i] * w
        flux = (flux + s * col[i]).astype(np.float32)
    den = np.float32(np.float32(1) - np.float32(np.float32(2) / np.float32(3)) * np.float32(np.float32(1) /
                                                                                              np.float32(1.1)))
    den = np.float32(np.float32(den * np.float32(2)) * np.float32(3.141592653)) * r2
    return (flux / den).astype(np.float32)


def test_oracle_gather_vs_numpy():
    import oracle
    rng = np.random.default_rng(9)
    n = 1500
    ph = np.zeros((n, 10), np.float32)
    ph[:, :3] = rng.uniform(-10, 10, size=(n, 3))
    ph[:, 7:10] = rng.uniform(0, 1, size=(n, 3))
    cph = ph[:300].copy()
    m = oracle.PhotonMap(ph, 1.0, cph, 0.5)
    allp = np.concatenate([ph, cph])
    pw = np.concatenate([np.ones(n, np.float32), np.full(300, 0.5, np.float32)])
    q = rng.uniform(-10, 10, size=(40, 3)).astype(np.float32)
    brdf = rng.uniform(0, 0.3, size=40).astype(np.float32)
    got = m.gather(q, brdf)
    for i in range(len(q)):
        exp = numpy_gather(allp[:, :3], allp[:, 7:10], pw, q[i], brdf[i])
        assert np.array_equal(got[i].view(np.uint32), exp.view(np.uint32)), i


def test_oracle_trace_invariants(cornell):
    import oracle
    meshes, lights = cornell
    s = oracle.Scene(meshes)
    g = oracle.trace(s, lights, 10000, 10, False)
    c = oracle.trace(s, lights, 10000, 10, True)
    # deposits lie on the box surfaces, colours only shrink (albedo <= 1), dir unit length
    assert np.all(np.abs(g[:, :3]) < 41) and np.all(g[:, 1] > -1)
    assert np.abs(np.linalg.norm(g[:, 3:6], axis=1) - 1).max() < 1e-5
    assert g[:, 7:10].max() <= 1.0 and c[:, 7:10].max() <= 1.0
    assert np.all(g[:, 6] == 0)                        # power never written (photon.h:9)
    # sharding: rank-order concatenation == full run
    parts = [oracle.trace(s, lights, 10000, 10, False, shard_rank=r, shard_count=4) for r in range(4)]
    assert np.array_equal(np.concatenate(parts).view(np.uint32), g.view(np.uint32))
    assert len(oracle.trace(s, lights, 10000, 1, False)) == 0


def test_oracle_render_invariants(cornell):
    import oracle
    meshes, lights = cornell
    s = oracle.Scene(meshes)
    g = oracle.trace(s, lights, 5000, 10, False)
    c = oracle.trace(s, lights, 5000, 10, True)
    gm, cm = oracle.PhotonMap(g, 1.0, c, 0.5), oracle.PhotonMap(c, 0.5)
    cam = oracle.camera_setup((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 40, 30)
    full, frgb, st = oracle.render(s, cam, 40, 30, 1, 30, (1, 1, 1), lights, gm, cm)
    assert np.all(full[0] == 0)                        # row H - 0 is out of bounds in the reference
    assert np.all((full[1:] >> 24) == 0xFF)
    assert st.pixels == 40 * 30 and st.caustic_queries <= st.path_vertices
    parts = [oracle.render(s, cam, 40, 30, 1, 30, (1, 1, 1), lights, gm, cm, tile_rank=r, tile_count=3)[0]
             for r in range(3)]
    assert np.array_equal(parts[0] | parts[1] | parts[2], full)


def test_square_light_emission():
    """SQUARE_LIGHT (this build's definition, pm_device.hpp emit_photon): origin
    uniform on the square about pos in the plane normal to n, direction in the
    hemisphere of n (cosine lobe); a point light keeps pointLightRayGen."""
    import oracle
    n = np.array([0.3, -1.0, 0.2], np.float32)
    n /= np.linalg.norm(n)
    L = dict(pos=(1.0, 10.0, -2.0), rgb=(1, 1, 1), power=50.0, normal=tuple(n), side=4.0)
    pts, dirs = [], []
    for pid in range(4000):
        o, d = oracle.emit_photon(L, pid)
        pts.append(o)
        dirs.append(d)
    pts, dirs = np.array(pts), np.array(dirs)
    rel = pts - np.array(L["pos"], np.float32)
    assert np.abs(rel @ n).max() < 1e-5                               # in the light's plane
    a = np.array([0, 1, 0] if abs(n[0]) > 0.9 else [1, 0, 0], np.float32)
    t1 = np.cross(a, n)
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(n, t1)
    u, v = rel @ t1, rel @ t2
    assert np.abs(u).max() <= 2.0 + 1e-5 and np.abs(v).max() <= 2.0 + 1e-5
    assert abs(u.mean()) < 0.1 and abs(v.mean()) < 0.1 and u.std() > 1.0   # ~uniform on [-2, 2]
    cos = dirs @ n
    assert cos.min() > 0 and abs(np.linalg.norm(dirs, axis=1) - 1).max() < 1e-5
    assert abs(cos.mean() - 2 / 3) < 0.03                             # cosine lobe: E[cos] = 2/3
    # a point light ignores normal/side: same as the reference raygen
    P = dict(pos=(1.0, 10.0, -2.0), rgb=(1, 1, 1), power=50.0)
    o, d = oracle.emit_photon(P, 7)
    assert np.array_equal(o, np.float32([1.0, 10.0, -2.0]))
    st = np.array([oracle.lib.orc_lcg_init(7, 0)], np.uint32)
    buf = (oracle.C.c_float * 3)()
    s = oracle.C.c_uint32(int(st[0]))
    oracle.lib.orc_random_point_in_unit_sphere(oracle.C.byref(s), buf)
    assert np.array_equal(d, np.array(buf[:], np.float32))


def test_viewer_projection():
    """photonViewer projection (glm perspective x lookAt, hostCode.cu:53-75):
    the oracle's float matrix agrees with a float64 evaluation of the glm
    formulas; the look-at point lands on the centre pixel, a photon behind the
    eye is dropped, an occluded one is not painted."""
    import oracle
    eye, ctr, up, fovy, W, H = (80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87, 64, 48
    P = oracle.viewer_params(eye, ctr, up, fovy, W, H)
    M = oracle.viewer_matrix(P).astype(np.float64)          # column-major: M[col][row]
    e, c, u = (np.array(v, np.float64) for v in (eye, ctr, up))
    f = (c - e) / np.linalg.norm(c - e)
    s = np.cross(f, u)
    s /= np.linalg.norm(s)
    uu = np.cross(s, f)
    V = np.eye(4)
    V[0, 0:3], V[1, 0:3], V[2, 0:3] = s, uu, -f            # rows of the view matrix
    V[0:3, 3] = -s @ e, -uu @ e, f @ e
    th = np.tan(fovy / 2)
    Pm = np.zeros((4, 4))
    Pm[0, 0], Pm[1, 1] = 1 / (W / H * th), 1 / th
    Pm[2, 2], Pm[2, 3], Pm[3, 2] = -(1000.1) / (999.9), -2 * 1000 * 0.1 / 999.9, -1
    ref = Pm @ V                                            # row-major
    assert np.allclose(M.T, ref, rtol=1e-5, atol=1e-6)
    empty = oracle.Scene([])
    ph = np.zeros((3, 10), np.float32)
    ph[0, 0:3] = ctr
    ph[0, 7:10] = (1.0, 0.5, 0.25)
    ph[1, 0:3] = (120.0, 30.0, 0.0)                         # behind the eye: clip z < 0
    ph[1, 7:10] = 1.0
    ph[2, 0:3] = (10.0, 60.0, 0.0)                          # outside the frame
    img = oracle.view_photons(empty, ph, P)
    painted = np.argwhere(img != 0xFF000000)
    assert len(painted) == 1
    y, x = painted[0]
    assert abs(x - W / 2) <= 1 and abs(y - H / 2) <= 1
    assert img[y, x] == (0xFF000000 | (64 << 16) | (128 << 8) | 255)
    import pm_amd
    wall = pm_amd.MeshData(np.float32([[40, -50, -50], [40, 50, -50], [40, 0, 50]]), np.int32([[0, 1, 2]]),
                           np.float32([1, 1, 1, 1, 0, 0, 1]))
    assert (oracle.view_photons(oracle.Scene([wall]), ph[:1], P) == 0xFF000000).all()
