"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the
same seeded inputs. Integer / index results and the arithmetic-spec floats are
compared bit for bit; the image is compared with the north-star tolerance
(L_inf <= 1e-3 per channel on the [0,1]-clamped colour) and the exact-match
fraction is asserted too."""
import numpy as np
import pytest

import conftest
import kd_layout

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import pm_amd
    if not torch.cuda.is_available() or pm_amd.device_count() == 0:
        pytest.fail("GPU tests need a visible MI355X (HIP device)")


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def random_rays(n, lo, hi, seed, tmin=1e-3, tmax=1e10):
    rng = np.random.default_rng(seed)
    o = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = o
    r[:, 3] = tmin
    r[:, 4:7] = d
    r[:, 7] = tmax
    return r


def _scene_pair(meshes, use_bvh=True):
    import oracle
    import pm_amd
    return pm_amd.Scene(meshes), oracle.Scene(meshes, use_bvh=use_bvh)


@pytest.mark.parametrize("which", ["cornell", "sphere"])
def test_intersect_bitwise(which, request):
    meshes, _ = request.getfixturevalue(which)
    gs, os_ = _scene_pair(meshes, use_bvh=(which != "cornell"))
    rays = random_rays(20000, [-25, -5, -25], [25, 45, 25], seed=1)
    # include axis-aligned and boundary-grazing rays
    rays[:500, 4:7] = np.eye(3, dtype=np.float32)[np.arange(500) % 3]
    hg = gs.intersect(torch.from_numpy(rays).cuda()).cpu().numpy()
    ho = os_.intersect(rays)
    assert np.array_equal(hg[:, 1:], ho[:, 1:]), "hit ids differ"
    assert np.array_equal(hg[:, 0], ho[:, 0]), "hit t differs (bits)"
    assert (ho[:, 1] >= 0).mean() > 0.5


def test_occluded(cornell):
    meshes, _ = cornell
    gs, os_ = _scene_pair(meshes, use_bvh=False)
    rays = random_rays(20000, [-19, 1, -19], [19, 39, 19], seed=2, tmax=15.0)
    og = gs.occluded(torch.from_numpy(rays).cuda()).cpu().numpy()
    oo = os_.occluded(rays)
    assert np.array_equal(og, oo)
    assert 0 < og.mean() < 1


def test_scene_stats(sphere):
    import pm_amd
    meshes, _ = sphere
    s = pm_amd.Scene(meshes).stats()
    assert s.num_triangles == sum(len(m.indices) for m in meshes)
    # BVH4 collapsed from a binary LBVH with T - 1 internal nodes
    assert (s.num_triangles - 1) // 3 <= s.num_nodes <= s.num_triangles - 1   # BVH4 collapsed from a binary tree
    assert 0 < s.max_depth <= 32


@pytest.mark.parametrize("which,casted", [("cornell", 10000), ("sphere", 100000)])
@pytest.mark.parametrize("caustics", [False, True])
def test_trace_bitwise(which, casted, caustics, request):
    import oracle
    import pm_amd
    meshes, lights = request.getfixturevalue(which)
    gs, os_ = _scene_pair(meshes)
    pg = pm_amd.run_point_light_ray_gen(gs, lights, casted, 10, caustics).cpu().numpy()
    po = oracle.trace(os_, lights, casted, 10, caustics)
    assert pg.shape == po.shape, (pg.shape, po.shape)
    assert np.array_equal(_bits(pg), _bits(po))
    assert len(pg) > 0


@pytest.mark.parametrize("caustics", [False, True])
def test_trace_square_light_bitwise(cornell, caustics):
    """SQUARE_LIGHT emission (this build's definition) traced bit-identically."""
    import oracle
    import pm_amd
    meshes, _ = cornell
    lights = [dict(pos=(0.0, 39.0, 0.0), rgb=(1.0, 0.9, 0.8), power=30.0, normal=(0.0, -1.0, 0.0), side=8.0),
              dict(pos=(-10.0, 20.0, 5.0), rgb=(1.0, 1.0, 1.0), power=10.0, normal=(1.0, 0.2, 0.0), side=3.0),
              dict(pos=(5.0, 30.0, -5.0), rgb=(0.5, 0.5, 1.0), power=10.0)]
    gs, os_ = _scene_pair(meshes)
    pg = pm_amd.run_point_light_ray_gen(gs, lights, 30000, 10, caustics).cpu().numpy()
    po = oracle.trace(os_, lights, 30000, 10, caustics)
    assert len(pg) > 0 and np.array_equal(_bits(pg), _bits(po))


@pytest.mark.parametrize("max_depth", [2, 3, 30])
@pytest.mark.parametrize("caustics", [False, True])
def test_trace_depth_bitwise(cornell, caustics, max_depth):
    """Path-length limits: the fused path kernel (csrc/trace.hip k_ph_paths)
    ends a path at bounce max_depth - 1 exactly as shootPhoton's loop does."""
    import oracle
    import pm_amd
    meshes, lights = cornell
    gs, os_ = _scene_pair(meshes)
    pg = pm_amd.run_point_light_ray_gen(gs, lights, 20000, max_depth, caustics).cpu().numpy()
    po = oracle.trace(os_, lights, 20000, max_depth, caustics)
    assert pg.shape == po.shape and np.array_equal(_bits(pg), _bits(po))


@pytest.mark.parametrize("casted,caustic,max_depth,shard", [
    (20000, 20000, 10, (0, 1)), (30000, 5000, 30, (1, 3)), (20000, 0, 10, (0, 1)), (0, 20000, 10, (0, 1)),
    (10000, 10000, 1, (0, 1))])
def test_trace_photon_sets_equal_two_calls(cornell, casted, caustic, max_depth, shard):
    """pm_trace_photon_sets (both sets in one k_ph_paths launch) gives each set
    exactly the photons of its own pm_trace_photons call, bitwise; with point
    and square lights (per-set light offsets differ with the counts)."""
    import pm_amd
    meshes, lights = cornell
    lights = list(lights) + [dict(pos=(0.0, 39.0, 0.0), rgb=(1.0, 0.9, 0.8), power=30.0, normal=(0.0, -1.0, 0.0),
                                  side=8.0)]
    gs = pm_amd.Scene(meshes)
    kw = dict(shard_rank=shard[0], shard_count=shard[1])
    g, c = pm_amd.run_photon_sets(gs, lights, casted, caustic, max_depth, **kw)
    window, compact = pm_amd.phase_us("trace"), pm_amd.phase_us("compact")
    g1 = pm_amd.run_point_light_ray_gen(gs, lights, casted, max_depth, False, **kw)
    c1 = pm_amd.run_point_light_ray_gen(gs, lights, caustic, max_depth, True, **kw)
    assert g.shape == g1.shape and c.shape == c1.shape
    assert np.array_equal(_bits(g.cpu().numpy()), _bits(g1.cpu().numpy()))
    assert np.array_equal(_bits(c.cpu().numpy()), _bits(c1.cpu().numpy()))
    if len(g1) + len(c1) > 0:
        assert window >= compact > 0.0


def test_trace_photon_sets_mid_size_full_grid(cornell):
    """a photon count that fills the persistent grid many times over
    (2 M + 1 M photons, max_depth 30), so the global-counter drain, the refill at
    PM_POOL_REFILL idle lanes and the event batching run at full occupancy in the
    regular suite; each set against its own call and a 1 % shard vs the oracle."""
    import oracle
    import pm_amd
    meshes, lights = cornell
    gs, os_ = _scene_pair(meshes)
    g, c = pm_amd.run_photon_sets(gs, lights, 2_000_000, 1_000_000, 30)
    g1 = pm_amd.run_point_light_ray_gen(gs, lights, 2_000_000, 30, False)
    c1 = pm_amd.run_point_light_ray_gen(gs, lights, 1_000_000, 30, True)
    assert np.array_equal(_bits(g.cpu().numpy()), _bits(g1.cpu().numpy()))
    assert np.array_equal(_bits(c.cpu().numpy()), _bits(c1.cpu().numpy()))
    for caustics, casted in ((False, 2_000_000), (True, 1_000_000)):
        pg = pm_amd.run_point_light_ray_gen(gs, lights, casted, 30, caustics, shard_rank=57, shard_count=100)
        po = oracle.trace(os_, lights, casted, 30, caustics, shard_rank=57, shard_count=100,
                          nthreads=conftest.ORACLE_THREADS)
        assert np.array_equal(_bits(pg.cpu().numpy()), _bits(po))


def test_trace_photon_sets_capacity(cornell):
    import pm_amd
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    small = torch.empty((10, 10), dtype=torch.float32, device="cuda")
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.run_photon_sets(gs, lights, 10000, 10000, 10, out=(small, None))
    assert e.value.status == pm_amd.PM_ERR_CAPACITY
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.run_photon_sets(gs, lights, 10000, 10000, 10, out=(None, small))
    assert e.value.status == pm_amd.PM_ERR_CAPACITY


def test_trace_shards_concatenate(cornell):
    import pm_amd
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    full = pm_amd.run_normal(gs, lights, 30000, 10).cpu().numpy()
    parts = [pm_amd.run_normal(gs, lights, 30000, 10, shard_rank=r, shard_count=3).cpu().numpy() for r in range(3)]
    assert np.array_equal(_bits(np.concatenate(parts)), _bits(full))


def test_trace_capacity_error(cornell):
    import pm_amd
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    small = torch.empty((10, 10), dtype=torch.float32, device="cuda")
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.run_normal(gs, lights, 10000, 10, out=small)
    assert e.value.status == pm_amd.PM_ERR_CAPACITY


def test_trace_edge_cases(cornell):
    import pm_amd
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    assert pm_amd.run_normal(gs, lights, 10, 10).shape[0] == 0          # casted < sum P -> 0 photons
    assert pm_amd.run_normal(gs, lights, 10000, 1).shape[0] == 0        # max_depth 1: no i > 0 bounce
    assert pm_amd.run_normal(gs, lights, 10000, 0).shape[0] == 0
    assert pm_amd.run_normal(gs, [], 10000, 10).shape[0] == 0


def _check_left_balanced(pos, dims):
    """every node vs all its ancestors: left subtree <= ancestor <= right subtree
    on the ancestor's split dimension (cukd left-balanced kd-tree invariant)."""
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
        ac = pos[parent, d]
        ic = pos[node, d]
        assert np.all(ic[left] <= ac[left]) and np.all(ic[~left] >= ac[~left])
        cur = parent
    return True


@pytest.mark.parametrize("n", [1, 2, 3, 7, 1000, 65537, 300000, 2_000_003])
def test_kdtree_build_left_balanced(n):
    import pm_amd
    rng = np.random.default_rng(n)
    rec = np.zeros((n, 11), np.float32)
    rec[:, 0:3] = rng.uniform(-20, 20, size=(n, 3))
    if n > 10:
        rec[: n // 10, 1] = 0.0        # a plane of ties
        rec[n // 10: n // 5, 0:3] = 5.0  # exact duplicates
    rec[:, 6:9] = rng.uniform(0, 1, size=(n, 3))
    rec[:, 9] = 1.0
    t = torch.from_numpy(rec.copy()).cuda()
    b = pm_amd.build_tree(t).cpu().numpy()
    out = t.cpu().numpy()
    dims = out[:, 10].view(np.uint32) >> 24
    assert np.all(dims <= 2)
    assert np.allclose(b[0], rec[:, :3].min(0)) and np.allclose(b[1], rec[:, :3].max(0))
    # permutation of the input records (ignoring split_dim byte)
    key = lambda a: np.lexsort(a[:, :10].view(np.uint32).T[::-1])
    o2 = out.copy()
    o2[:, 10] = 0
    assert np.array_equal(rec[key(rec)][:, :10].view(np.uint32), o2[key(o2)][:, :10].view(np.uint32))
    _check_left_balanced(out[:, :3], dims.astype(np.int64))
    # node for node against the oracle's restatement of the layout
    want, _ = kd_layout.inplace_records(rec, conftest.ORACLE_THREADS)
    kd_layout.assert_same(out, want, f"pm_kdtree_build n={n}")


def _brute_knn(pts, q, k, r):
    # same float32 evaluation order as the spec: (dx*dx + dy*dy) + dz*dz
    diff = (q[:, None, :] - pts[None, :, :]).astype(np.float32)
    d2 = (diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]).astype(np.float32) + diff[..., 2] * diff[..., 2]
    ids = np.full((len(q), k), -1, np.int32)
    dd = np.full((len(q), k), (np.float32(r) * np.float32(r)), np.float32)
    for i in range(len(q)):
        ok = np.nonzero(d2[i] < (np.float32(r) * np.float32(r)))[0]
        order = ok[np.lexsort((ok, d2[i, ok]))][:k]
        ids[i, : len(order)] = order
        dd[i, : len(order)] = d2[i, order]
    return ids, dd


def test_knn_bruteforce_with_ties():
    import pm_amd
    rng = np.random.default_rng(7)
    n = 3000
    pts = rng.integers(-5, 6, size=(n, 3)).astype(np.float32)   # lattice: many exact ties
    ph = np.zeros((n, 10), np.float32)
    ph[:, 0:3] = pts
    ph[:, 7:10] = 1.0
    m = pm_amd.PhotonMap(torch.from_numpy(ph).cuda(), 1.0)
    q = rng.uniform(-6, 6, size=(400, 3)).astype(np.float32)
    q[:50] = pts[:50]                                           # queries on photons
    for k, r in [(50, 100.0), (8, 2.5), (64, 1.0), (16, 0.0)]:
        ids, d2, md = pm_amd.knn(m, torch.from_numpy(q).cuda(), k, r)
        bi, bd = _brute_knn(pts, q, k, r)
        assert np.array_equal(ids.cpu().numpy(), bi), (k, r)
        assert np.array_equal(_bits(d2.cpu().numpy()), _bits(bd)), (k, r)
        assert np.array_equal(_bits(md.cpu().numpy()), _bits(bd[:, -1]))


def test_knn_and_gather_vs_oracle(cornell):
    import oracle
    import pm_amd
    meshes, lights = cornell
    os_ = oracle.Scene(meshes)
    g = oracle.trace(os_, lights, 20000, 10, False)
    c = oracle.trace(os_, lights, 20000, 10, True)
    gm = pm_amd.PhotonMap(torch.from_numpy(g).cuda(), 1.0, torch.from_numpy(c).cuda(), 0.5)
    om = oracle.PhotonMap(g, 1.0, c, 0.5)
    rng = np.random.default_rng(3)
    q = g[rng.integers(0, len(g), 2000), 0:3] + rng.normal(scale=0.5, size=(2000, 3)).astype(np.float32)
    q = q.astype(np.float32)
    ids, d2, md = pm_amd.knn(gm, torch.from_numpy(q).cuda(), 50, 100.0)
    oi, od, omd = om.knn(q, 50, 100.0)
    assert np.array_equal(ids.cpu().numpy(), oi)
    assert np.array_equal(_bits(d2.cpu().numpy()), _bits(od))
    assert np.array_equal(_bits(md.cpu().numpy()), _bits(omd))
    brdf = rng.uniform(0, 0.4, size=2000).astype(np.float32)
    fg = pm_amd.gather_photons(gm, torch.from_numpy(q).cuda(), torch.from_numpy(brdf).cuda()).cpu().numpy()
    fo = om.gather(q, brdf)
    assert np.array_equal(_bits(fg), _bits(fo))


@pytest.mark.parametrize("k,radius", [(1, 100.0), (64, 100.0), (128, 100.0), (129, 100.0), (200, 100.0),
                                      (256, 100.0), (200, 1.5)])
def test_knn_k_range_vs_oracle(cornell, k, radius):
    """pm_knn for every list width, incl. the two-pass path for 128 < k <= 256
    (config 5 asks for k = 200) and a radius that leaves lists partly empty."""
    import oracle
    import pm_amd
    meshes, lights = cornell
    os_ = oracle.Scene(meshes)
    g = oracle.trace(os_, lights, 10000, 10, False)
    gm = pm_amd.PhotonMap(torch.from_numpy(g).cuda(), 1.0)
    om = oracle.PhotonMap(g, 1.0)
    rng = np.random.default_rng(k)
    q = (g[rng.integers(0, len(g), 500), 0:3] + rng.normal(scale=0.5, size=(500, 3))).astype(np.float32)
    ids, d2, md = pm_amd.knn(gm, torch.from_numpy(q).cuda(), k, radius)
    oi, od, omd = om.knn(q, k, radius)
    assert np.array_equal(ids.cpu().numpy(), oi)
    assert np.array_equal(_bits(d2.cpu().numpy()), _bits(od))
    assert np.array_equal(_bits(md.cpu().numpy()), _bits(omd))
    if radius < 10:
        assert (oi == -1).any()


def test_photon_map_export(cornell):
    import oracle
    import pm_amd
    meshes, lights = cornell
    g = oracle.trace(oracle.Scene(meshes), lights, 5000, 10, False)
    m = pm_amd.PhotonMap(torch.from_numpy(g).cuda(), 1.0)
    e = m.export().cpu().numpy()
    assert len(e) == len(g)
    dims = e[:, 10].view(np.uint32) >> 24
    _check_left_balanced(e[:, :3], dims.astype(np.int64))
    assert np.all(e[:, 9] == 1.0)
    kd_layout.assert_same(e, kd_layout.map_records([(g, 1.0)])[0], "export")
    # two photon sets (loadPhotons: diffuse ++ caustic, powers 1 / 0.5)
    c = oracle.trace(oracle.Scene(meshes), lights, 5000, 10, True)
    m2 = pm_amd.PhotonMap(torch.from_numpy(g).cuda(), 1.0, torch.from_numpy(c).cuda(), 0.5)
    kd_layout.assert_same(m2.export().cpu().numpy(), kd_layout.map_records([(g, 1.0), (c, 0.5)])[0], "export a++b")


def _render_pair(meshes, lights, casted, W, H, spp, tiles=(0, 1), caustic_k=0):
    import oracle
    import pm_amd
    os_ = oracle.Scene(meshes)
    gs = pm_amd.Scene(meshes)
    gph = pm_amd.run_normal(gs, lights, casted, 10)
    cph = pm_amd.run_caustics(gs, lights, casted, 10)
    g_np, c_np = gph.cpu().numpy(), cph.cpu().numpy()
    gmap, cmap = pm_amd.load_photons(gph, cph)
    cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, W, H)
    ocam = oracle.camera_setup((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, W, H)
    assert bytes(cam) == bytes(ocam)
    rgba, rgb = pm_amd.render(gs, cam, W, H, spp, 30, (1, 1, 1), lights, gmap, cmap, tile_rank=tiles[0],
                              tile_count=tiles[1], caustic_k=caustic_k)
    om_g = oracle.PhotonMap(g_np, 1.0, c_np, 0.5)
    om_c = oracle.PhotonMap(c_np, 0.5)
    orgba, orgb, ost = oracle.render(os_, ocam, W, H, spp, 30, (1, 1, 1), lights, om_g, om_c,
                                     tile_rank=tiles[0], tile_count=tiles[1], caustic_k=caustic_k)
    return rgba.cpu().numpy().view(np.uint32), rgb.cpu().numpy(), orgba, orgb, ost


@pytest.mark.parametrize("which,casted,W,H,spp", [("cornell", 20000, 64, 48, 2), ("sphere", 20000, 48, 40, 1)])
def test_render_vs_oracle(which, casted, W, H, spp, request):
    import pm_amd
    meshes, lights = request.getfixturevalue(which)
    rgba, rgb, orgba, orgb, ost = _render_pair(meshes, lights, casted, W, H, spp)
    st = pm_amd.render_stats()
    assert (st.pixels, st.path_vertices, st.caustic_queries, st.global_queries, st.rays) == \
        (ost.pixels, ost.path_vertices, ost.caustic_queries, ost.global_queries, ost.rays)
    err = np.abs(np.clip(rgb, 0, 1) - np.clip(orgb, 0, 1)).max()
    assert err <= 1e-3, err
    exact = np.mean(_bits(rgb) == _bits(orgb))
    assert exact >= 0.999, exact
    assert np.mean(rgba != orgba) <= 0.001
    assert np.all(rgba[0] == 0)   # row 0 is never written (deviceCode.cu:224-229)


def test_render_tiles_cover_image(cornell):
    meshes, lights = cornell
    parts = []
    for r in range(3):
        rgba, rgb, orgba, orgb, _ = _render_pair(meshes, lights, 5000, 40, 36, 1, tiles=(r, 3))
        assert np.array_equal(_bits(rgb), _bits(orgb)) or np.abs(rgb - orgb).max() <= 1e-3
        parts.append(rgba)
    full, _, ofull, _, _ = _render_pair(meshes, lights, 5000, 40, 36, 1)
    merged = parts[0] | parts[1] | parts[2]
    assert np.array_equal(merged, full)


def test_render_empty_maps(cornell):
    import pm_amd
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    empty = torch.zeros((0, 10), dtype=torch.float32, device="cuda")
    gmap, cmap = pm_amd.load_photons(empty, empty)
    cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 32, 32)
    rgba, rgb = pm_amd.render(gs, cam, 32, 32, 1, 30, (1, 1, 1), lights, gmap, cmap)
    assert torch.isfinite(rgb).all()


@pytest.mark.parametrize("caustics", [False, True])
def test_photon_viewer_vs_oracle(cornell, caustics):
    """photonViewer splat (pm_photon_view) equals the oracle image bit for bit."""
    import oracle
    import pm_amd
    meshes, lights = cornell
    os_ = oracle.Scene(meshes)
    ph = oracle.trace(os_, lights, 20000, 10, caustics)
    gs = pm_amd.Scene(meshes)
    cam = ((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87)
    img = pm_amd.view_photons(gs, torch.from_numpy(ph).cuda(), *cam, 160, 120).cpu().numpy().view(np.uint32)
    ref = oracle.view_photons(os_, ph, oracle.viewer_params(*cam, 160, 120))
    assert np.array_equal(img, ref)
    assert (img != 0xFF000000).sum() > 50


def test_quantize_matches_text_roundtrip(tmp_path):
    """pm_photons_quantize (device) == write_alive_photons -> read_photons_from_file."""
    import pm_amd
    import test_host_io
    v = test_host_io._quantize_corpus()
    v = v[: len(v) // 9 * 9]
    ph = np.zeros((len(v) // 9, 10), np.float32)
    ph[:, 0:6] = v.reshape(-1, 9)[:, 0:6]
    ph[:, 7:10] = v.reshape(-1, 9)[:, 6:9]
    ph[:, 6] = np.float32(3.0)
    p = str(tmp_path / "q.txt")
    pm_amd.write_alive_photons(ph, p)
    back = pm_amd.read_photons_from_file(p)
    t = torch.from_numpy(ph.copy()).cuda()
    pm_amd.quantize_photons(t)
    assert np.array_equal(t.cpu().numpy().view(np.uint32), back.view(np.uint32))


def test_render_begin_finish_equals_render(cornell):
    """pm_render_begin + pm_render_finish (on a different stream) give exactly
    pm_render's image and stats; a job finishes once."""
    import pm_amd
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    gph = pm_amd.run_point_light_ray_gen(gs, lights, 20000, 10, False)
    cph = pm_amd.run_caustics(gs, lights, 20000, 10)
    gmap, cmap = pm_amd.load_photons(gph, cph)
    W, H = 56, 40
    cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, W, H)
    rgba, rgb = pm_amd.render(gs, cam, W, H, 2, 30, (1, 1, 1), lights, gmap, cmap)
    st = pm_amd.render_stats()
    side = torch.cuda.Stream()
    job = pm_amd.render_begin(gs, cam, W, H, 2, 30, (1, 1, 1), lights, stream=side.cuda_stream)
    rgba2, rgb2 = job.finish(gmap, cmap)
    st2 = pm_amd.render_stats()
    assert torch.equal(rgba, rgba2)
    assert np.array_equal(_bits(rgb.cpu().numpy()), _bits(rgb2.cpu().numpy()))
    assert bytes(st) == bytes(st2)
    with pytest.raises(pm_amd.PMError):
        job.finish(gmap, cmap)
    job.close()
    # the caustic gather ahead of finish (pm_render_gather_caustic, on the side
    # stream): finish then takes no caustic map, or the same one, not another
    for again in (None, cmap):
        job = pm_amd.render_begin(gs, cam, W, H, 2, 30, (1, 1, 1), lights, stream=side.cuda_stream)
        job.gather_caustic(cmap, stream=side.cuda_stream)
        with pytest.raises(pm_amd.PMError):
            job.gather_caustic(cmap)   # once per job
        with pytest.raises(pm_amd.PMError):
            job.finish(gmap, gmap)   # not the map it gathered
        rgba3, rgb3 = job.finish(gmap, again)
        assert torch.equal(rgba, rgba3)
        assert np.array_equal(_bits(rgb.cpu().numpy()), _bits(rgb3.cpu().numpy()))
        assert bytes(st) == bytes(pm_amd.render_stats())
        job.close()
    job = pm_amd.render_begin(gs, cam, W, H, 2, 30, (1, 1, 1), lights)
    with pytest.raises(pm_amd.PMError):
        job.finish(gmap, None)   # no caustic map and none gathered
    job.close()


def test_frame_driver_matches_direct_pipeline(cornell):
    """dist.frame over GpuBackend (world 1) renders exactly the image of the
    direct pm_amd calls (trace -> maps -> render), frame after frame."""
    import pm_amd
    from pm_amd import dist as pmdist
    meshes, lights = cornell
    gs = pm_amd.Scene(meshes)
    cfg = pmdist.FrameConfig(casted=40000, caustic=20000, width=64, height=48)
    g = pm_amd.run_point_light_ray_gen(gs, lights, cfg.casted, cfg.max_depth, False)
    c = pm_amd.run_point_light_ray_gen(gs, lights, cfg.caustic, cfg.max_depth, True)
    gmap, cmap = pm_amd.load_photons(g, c)
    cam = pm_amd.setup_camera(cfg.camera["look_from"], cfg.camera["look_at"], cfg.camera["look_up"],
                              cfg.camera["fovy"], cfg.width, cfg.height)
    ref, _ = pm_amd.render(gs, cam, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.sky, lights, gmap, cmap,
                           want_rgb=False)
    be = pmdist.GpuBackend(gs, lights, cfg, 0, 1)
    rgba = torch.zeros((cfg.height, cfg.width), dtype=torch.int32, device="cuda")
    for _ in range(2):
        rgba.zero_()
        out, info = pmdist.frame(be, 0, 1, None, rgba)
        assert info["n_global"] == gmap.n and info["n_caustic"] == cmap.n
        assert torch.equal(out, ref)


@pytest.mark.parametrize("jitter", [0.0, 1e-3, 0.5])
def test_seeded_gather_tight_neighbours(cornell, jitter):
    """The production gather (leader-seeded cut-offs) on queries in spatial
    order, where the leader bounds are tight: queries at photon positions
    (d^2 = 0 ties), exact duplicates and small jitters; bitwise equal to the
    oracle's exact kNN radiance estimate."""
    import oracle
    import pm_amd
    meshes, lights = cornell
    os_ = oracle.Scene(meshes)
    g = oracle.trace(os_, lights, 30000, 10, False)
    c = oracle.trace(os_, lights, 30000, 10, True)
    rng = np.random.default_rng(11)
    q = g[rng.integers(0, len(g), 6000), 0:3].astype(np.float32)
    q = np.concatenate([q, q[:500]])   # exact duplicates
    q = q + (rng.normal(scale=jitter, size=q.shape).astype(np.float32) if jitter else 0)
    q = np.ascontiguousarray(q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))].astype(np.float32))
    brdf = rng.uniform(0, 0.4, size=len(q)).astype(np.float32)
    for a, pa, b, pb in ((g, 1.0, c, 0.5), (c, 0.5, None, 0.0)):
        gm = pm_amd.PhotonMap(torch.from_numpy(a).cuda(), pa, None if b is None else torch.from_numpy(b).cuda(), pb)
        om = oracle.PhotonMap(a, pa, b, pb)
        got = pm_amd.gather_photons(gm, torch.from_numpy(q).cuda(), torch.from_numpy(brdf).cuda()).cpu().numpy()
        assert np.array_equal(_bits(got), _bits(om.gather(q, brdf)))


def _synthetic_photons(n, seed, grid=None):
    """(n, 10) pm_photon rows; `grid` snaps positions to a coarse lattice (ties,
    exact duplicates, -0.0 and +0.0 on the planes)."""
    rng = np.random.default_rng(seed)
    p = np.zeros((n, 10), np.float32)
    pos = rng.uniform(-20, 20, size=(n, 3)).astype(np.float32)
    if grid:
        pos = (np.round(pos / grid) * grid).astype(np.float32)
        pos[rng.random(n) < 0.1, 1] = -0.0
    p[:, 0:3] = pos
    p[:, 3:6] = rng.normal(size=(n, 3))
    p[:, 7:10] = rng.uniform(0, 1, size=(n, 3))
    return torch.from_numpy(p).cuda()


@pytest.mark.parametrize("world", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("data", ["cornell", "ties"])
def test_sharded_kd_build_equals_replicated(cornell, world, data):
    """SURVEY §8e build step: top levels selected on every rank, subtree j built
    by rank j % world, all-gathered (here: concatenated in rank order) and placed;
    the map's kd records equal the one-device build bit for bit, and so does a
    gather through it."""
    import pm_amd
    from pm_amd import dist as pmdist
    if data == "cornell":
        meshes, lights = cornell
        gs = pm_amd.Scene(meshes)
        g = pm_amd.run_point_light_ray_gen(gs, lights, 30000, 10, False)
        c = pm_amd.run_point_light_ray_gen(gs, lights, 30000, 10, True)
    else:
        g, c = _synthetic_photons(70001, 5, grid=2.5), _synthetic_photons(999, 6, grid=2.5)
    ref = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
    plan = pm_amd.KdShardPlan(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=world)
    L = min((world - 1).bit_length() + 1, 5)
    assert len(plan.sizes) == 2 ** L and sum(plan.sizes) == ref.n - (2 ** L - 1)
    owner, load = pmdist.shard_owners(plan.sizes, world)
    assert sorted(set(owner)) == list(range(min(world, 2 ** L)))
    bufs = [pmdist.shard_local(plan, r, world)[0] for r in range(world)]
    m = pmdist.shard_assemble(plan, torch.cat(bufs), world)
    assert m.n == ref.n
    assert torch.equal(m.export().view(torch.int32), ref.export().view(torch.int32))
    if world == 2:   # the one-device tree itself against the oracle's layout
        want, _ = kd_layout.map_records([(g.cpu().numpy(), pm_amd.PHOTON_POWER),
                                         (c.cpu().numpy(), pm_amd.CAUSTICS_PHOTON_POWER)])
        kd_layout.assert_same(ref.export().cpu().numpy(), want, f"map ({data})")
    rng = np.random.default_rng(3)
    q = torch.from_numpy(rng.uniform(-20, 20, size=(3000, 3)).astype(np.float32)).cuda()
    brdf = torch.from_numpy(rng.uniform(0, 0.4, size=3000).astype(np.float32)).cuda()
    assert torch.equal(pm_amd.gather_photons(m, q, brdf).view(torch.int32),
                       pm_amd.gather_photons(ref, q, brdf).view(torch.int32))


@pytest.mark.parametrize("world", [2, 3, 8, 16])
@pytest.mark.parametrize("data", ["cornell", "ties"])
def test_distributed_top_selection_equals_replicated(cornell, world, data):
    """the top levels selected from each rank's own photons
    (pm_kd_top_sel: every pass over 1/G of the elements, its histograms
    all-reduced; here the ranks run in one process and the reductions are done
    on the host side of the test) give the same top nodes and subtree sizes as
    the replicated selection over all photons, and the map built through them
    equals the one-device map bit for bit (NaN positions included: +inf)."""
    import pm_amd
    from pm_amd import dist as pmdist
    if data == "cornell":
        meshes, lights = cornell
        gs = pm_amd.Scene(meshes)
        g = pm_amd.run_point_light_ray_gen(gs, lights, 30000, 10, False)
        c = pm_amd.run_point_light_ray_gen(gs, lights, 30000, 10, True)
    else:
        g, c = _synthetic_photons(70001, 5, grid=2.5), _synthetic_photons(999, 6, grid=2.5)
        g[17, 1] = float("nan")   # sorts last in every pass, as in the one-device build
    ref = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
    rep = pm_amd.KdShardPlan(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=world)
    sel, _ = pmdist.simulated_top_selection(pm_amd, g, c, world)
    assert sel.steps > 1
    plan = pm_amd.KdShardPlan(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=world, sel=sel)
    assert plan.sizes == rep.sizes and len(plan.sizes) > 0
    bufs = [pmdist.shard_local(plan, r, world)[0] for r in range(world)]
    m = pmdist.shard_assemble(plan, torch.cat(bufs), world)
    assert torch.equal(m.export().view(torch.int32), ref.export().view(torch.int32))


def test_distributed_top_selection_no_split(cornell):
    """A map too small to split (or one rank) finishes at once: 0 subtrees, the
    whole tree built in the map call, equal to the one-device build."""
    import pm_amd
    from pm_amd import dist as pmdist
    g, c = _synthetic_photons(9, 1), _synthetic_photons(3, 2)
    ref = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
    for world in (1, 8):
        sel, _ = pmdist.simulated_top_selection(pm_amd, g, c, world)
        plan = pm_amd.KdShardPlan(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=world, sel=sel)
        assert plan.sizes == []
        assert torch.equal(plan.map().export().view(torch.int32), ref.export().view(torch.int32))


def test_sharded_kd_build_small_map():
    """A map too small to split (n < 2^(L+1)) is built whole by every rank."""
    from pm_amd import dist as pmdist
    assert pmdist.shard_owners([5, 9, 9, 3], 2) == ([0, 0, 1, 1], [14, 12])
    import pm_amd
    g, c = _synthetic_photons(9, 1), _synthetic_photons(3, 2)
    plan = pm_amd.KdShardPlan(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=8)
    assert plan.sizes == []
    ref = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
    assert torch.equal(plan.map().export().view(torch.int32), ref.export().view(torch.int32))


@pytest.mark.parametrize("k", [1, 8, 50, 64, 128, 129, 200, 256])
def test_gather_k_vs_oracle(cornell, k):
    """pm_gather_k (config 5: k = 200 caustic gather): the radiance estimate over
    the k nearest equals the oracle's bit for bit, incl. lists that do not fill."""
    import oracle
    import pm_amd
    meshes, lights = cornell
    os_ = oracle.Scene(meshes)
    g = oracle.trace(os_, lights, 20000, 10, False)
    c = oracle.trace(os_, lights, 20000, 10, True)
    rng = np.random.default_rng(9)
    q = np.concatenate([g[rng.integers(0, len(g), 1500), 0:3] + rng.normal(scale=0.5, size=(1500, 3)),
                        rng.uniform(-300, 300, size=(100, 3))]).astype(np.float32)   # + far queries
    brdf = rng.uniform(0, 0.4, size=len(q)).astype(np.float32)
    q = q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))]   # spatial order
    for a, pa, b, pb in ((g, 1.0, c, 0.5), (c, 0.5, None, 0.0)):
        gm = pm_amd.PhotonMap(torch.from_numpy(a).cuda(), pa, None if b is None else torch.from_numpy(b).cuda(), pb)
        om = oracle.PhotonMap(a, pa, b, pb)
        fg = pm_amd.gather_photons(gm, torch.from_numpy(q).cuda(), torch.from_numpy(brdf).cuda(), k=k).cpu().numpy()
        assert np.array_equal(_bits(fg), _bits(om.gather(q, brdf, k=k)))


def test_render_caustic_k200_vs_oracle(cornell):
    """Config 5's caustic gather (k = 200) inside pm_render matches the oracle's
    render with the same k; k = 0 and k = 50 are the reference render."""
    import pm_amd
    meshes, lights = cornell
    rgba, rgb, orgba, orgb, _ = _render_pair(meshes, lights, 20000, 48, 36, 1, caustic_k=200)
    assert np.abs(np.clip(rgb, 0, 1) - np.clip(orgb, 0, 1)).max() <= 1e-3
    assert np.mean(_bits(rgb) == _bits(orgb)) >= 0.999
    ref = _render_pair(meshes, lights, 20000, 48, 36, 1)[1]
    k50 = _render_pair(meshes, lights, 20000, 48, 36, 1, caustic_k=50)[1]
    assert np.array_equal(_bits(ref), _bits(k50))
    assert not np.array_equal(_bits(ref), _bits(rgb))   # 200 neighbours change the caustic term


def test_nan_positions_build_as_inf(cornell):
    """a NaN photon coordinate compares false both ways, so the count
    and partition passes of the kd build could classify it differently. Every
    build takes NaN as +inf (include/pm.h): the map equals the oracle's map of
    the same photons with NaN replaced by +inf, gathers and all, the sharded
    build included, and in-place pm_kdtree_build keeps a valid tree."""
    import oracle
    import pm_amd
    from pm_amd import dist as pmdist
    meshes, lights = cornell
    g = oracle.trace(oracle.Scene(meshes), lights, 20000, 10, False)
    rng = np.random.default_rng(11)
    bad = rng.choice(len(g), size=len(g) // 20, replace=False)
    gn = g.copy()
    gn[bad, rng.integers(0, 3, size=len(bad))] = np.nan
    gi = gn.copy()
    gi[:, 0:3] = np.where(np.isnan(gn[:, 0:3]), np.inf, gn[:, 0:3])
    assert not np.isnan(gi[:, 0:3]).any() and np.isinf(gi[:, 0:3]).sum() == len(bad)
    gm = pm_amd.PhotonMap(torch.from_numpy(gn).cuda(), 1.0)
    om = oracle.PhotonMap(gi, 1.0)
    q = (g[rng.integers(0, len(g), 1000), 0:3] + rng.normal(scale=0.5, size=(1000, 3))).astype(np.float32)
    ids, d2, md = pm_amd.knn(gm, torch.from_numpy(q).cuda(), 50, 100.0)
    oi, od, omd = om.knn(q, 50, 100.0)
    assert np.array_equal(ids.cpu().numpy(), oi)
    assert not np.isin(bad, ids.cpu().numpy()).any()
    brdf = rng.uniform(0, 0.4, size=1000).astype(np.float32)
    fg = pm_amd.gather_photons(gm, torch.from_numpy(q).cuda(), torch.from_numpy(brdf).cuda()).cpu().numpy()
    assert np.array_equal(_bits(fg), _bits(om.gather(q, brdf)))
    # the sharded build of the same photons: the same tree
    t = torch.from_numpy(gn).cuda()
    plan = pm_amd.KdShardPlan(t, 1.0, world=4)
    if plan.sizes:
        sm = pmdist.shard_assemble(plan, torch.cat([pmdist.shard_local(plan, r, 4)[0] for r in range(4)]), 4)
        assert torch.equal(sm.export().view(torch.int32), gm.export().view(torch.int32))
    # in place on kd records: a left-balanced tree over the +inf positions
    rec = np.zeros((len(gn), 11), np.float32)
    rec[:, 0:3] = gn[:, 0:3]
    tr = torch.from_numpy(rec).cuda()
    pm_amd.build_tree(tr, bounds=False)
    out = tr.cpu().numpy()
    pos = np.where(np.isnan(out[:, 0:3]), np.inf, out[:, 0:3])
    _check_left_balanced(pos, (out[:, 10].view(np.uint32) >> 24).astype(np.int64))
    kd_layout.assert_same(out, kd_layout.inplace_records(rec)[0], "in place, NaN as +inf")
    kd_layout.assert_same(gm.export().cpu().numpy(), kd_layout.map_records([(gn, 1.0)])[0], "map, NaN as +inf")


def test_shard_plan_from_mismatched_selection_is_refused():
    """a plan whose subtree sizes come from a distributed selection
    over OTHER photons (wrong offsets or reductions) must not extract past its
    subtree buffers: the first pm_kd_shard_build checks the counted subtree
    sizes against the plan's and returns PM_ERR_INVALID."""
    import pm_amd
    from pm_amd import dist as pmdist
    g, c = _synthetic_photons(70001, 5), _synthetic_photons(999, 6)
    sel, _ = pmdist.simulated_top_selection(pm_amd, g, c, 4)
    g2 = g.flip(0).contiguous()   # the same points under other indices
    g2[: len(g2) // 2, 0] += 7.0
    plan = pm_amd.KdShardPlan(g2, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=4, sel=sel)
    with pytest.raises(pm_amd.PMError) as e:
        pmdist.shard_local(plan, 0, 4)
    assert e.value.status == pm_amd.PM_ERR_INVALID


@pytest.mark.parametrize("world", [1, 3, 8])
def test_photon_rows_maps_equal_photon_maps(world):
    """pm_photon_rows (ABI 5): the maps and the sharded plan
    built straight from the exchange's padded (position, colour) buffer -- rank
    r's rows at [r m, r m + n_r), padding rows between -- equal those built
    from the concatenated pm_photon arrays, bit for bit (tree, payload, and the
    sharded build with and without the distributed top selection)."""
    import pm_amd
    from pm_amd import dist as pmdist
    g, c = _synthetic_photons(70001, 5, grid=2.5), _synthetic_photons(4999, 6, grid=2.5)

    def padded(t):
        parts = [t[pmdist.shard_range(t.shape[0], r, world)[0]: pmdist.shard_range(t.shape[0], r, world)[1]]
                 for r in range(world)]
        ns = [p.shape[0] for p in parts]
        m = max(ns) + 3   # extra padding rows: never read
        buf = torch.full((world * m, 6), float("nan"), device="cuda")
        for r, p in enumerate(parts):
            pmdist.pack_rows(p, buf[r * m: r * m + ns[r]])
        return pm_amd.PhotonRows.of_padded(buf, ns, m)

    gr, cr = padded(g), padded(c)
    assert gr.n == g.shape[0] and torch.equal(gr.photons()[:, [0, 1, 2, 7, 8, 9]], g[:, [0, 1, 2, 7, 8, 9]])
    ref = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
    m = pm_amd.PhotonMap(gr, pm_amd.PHOTON_POWER, cr, pm_amd.CAUSTICS_PHOTON_POWER)
    assert m.n == ref.n and torch.equal(m.export().view(torch.int32), ref.export().view(torch.int32))
    mc = pm_amd.PhotonMap(cr, pm_amd.CAUSTICS_PHOTON_POWER)
    assert torch.equal(mc.export().view(torch.int32),
                       pm_amd.PhotonMap(c, pm_amd.CAUSTICS_PHOTON_POWER).export().view(torch.int32))
    w = max(world, 2)
    for sel in (None, pmdist.simulated_top_selection(pm_amd, g, c, w)[0]):
        plan = pm_amd.KdShardPlan(gr, pm_amd.PHOTON_POWER, cr, pm_amd.CAUSTICS_PHOTON_POWER, world=w, sel=sel)
        assert plan.n == ref.n and len(plan.sizes) > 0
        sm = pmdist.shard_assemble(plan, torch.cat([pmdist.shard_local(plan, r, w)[0] for r in range(w)]), w)
        assert torch.equal(sm.export().view(torch.int32), ref.export().view(torch.int32))
    # a malformed descriptor is refused
    bad = pm_amd.PhotonRows.of_padded(gr.buf, [1], 1)
    bad.color_offset = 4   # colour would run past the 6-float row
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.PhotonMap(bad, 1.0)
    assert e.value.status == pm_amd.PM_ERR_INVALID
