"""Full-size parity of the BASELINE workloads against the CPU oracle (VERDICT r2,
missing 2-3): configs 3 and 5 at the bench's own sizes, checked on samples an
oracle finishes in seconds.
  - trace: three 1 % shards of the full photon-id range (first, middle, last:
    the same ids, seeds and deposit slots as the full launch) traced by the
    oracle and by the GPU, bitwise;
  - gather: one production frame at 1920x1080 (render_begin + finish over the
    full maps: config 3's 45.4 M-photon global map and 36 M final-gather
    queries, config 5's k = 200 caustic gather over 2.3 M queries); 50 k of the
    frame's own queries per map, sampled uniformly, must carry bit for bit the
    radiance the oracle's gatherPhotons (shading.h:93-121, over an independent
    exact kNN, shading.h:11-18) computes on maps built from the same photons.
  - kd layout: both maps' trees node for node against the oracle's
    restatement of cukd's left-balanced layout (tests/kd_layout.py);
  - image: a 48-row band at the frame centre rendered by the oracle over the
    full maps, L_inf <= 1e-3 and >= 99.9 % of pixels bitwise vs the HIP frame;
    the same band under the oracle's alternative specifications of the
    reference's unpinned behaviour (tests/test_spec_bounds.py) within 1e-3 of it.
The GPU photons the maps are built from are the ones the frame used (their
bitwise agreement with the oracle is the trace check above and, at reduced
size, test_gpu_workloads.py)."""
import numpy as np
import pytest

import conftest
import kd_layout

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
NT = conftest.ORACLE_THREADS
CAM = ((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87)
SAMPLE = 50_000
BAND = 48


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _trace_shards_vs_oracle(gs, os_, lights, casted, caustics):
    import oracle
    import pm_amd
    for rank in (0, 37, 99):
        g = pm_amd.run_point_light_ray_gen(gs, lights, casted, 10, caustics, shard_rank=rank, shard_count=100)
        o = oracle.trace(os_, lights, casted, 10, caustics, shard_rank=rank, shard_count=100, nthreads=NT)
        assert g.shape[0] == len(o), (rank, caustics)
        assert np.array_equal(_bits(g.cpu().numpy()), _bits(o)), (rank, caustics)


def _frame_vs_oracle(gs, os_, lights, g, c, caustic_k, W=1920, H=1080):
    import oracle
    import pm_amd
    gm, cm = pm_amd.load_photons(g, c)
    og, oc = g.cpu().numpy(), c.cpu().numpy()
    # the two kd-trees node for node against the oracle's left-balanced layout
    # (cukd::buildTree, ray-tracer/src/hostCode.cu:94-95; the global map is
    # built by the selection build at this size)
    for m, parts, what in ((gm, [(og, 1.0), (oc, 0.5)], "global"), (cm, [(oc, 0.5)], "caustic")):
        want, _ = kd_layout.map_records(parts, NT)
        kd_layout.assert_same(m.export().cpu().numpy(), want, what)
        del want
    cam = pm_amd.setup_camera(*CAM, W, H)
    job = pm_amd.render_begin(gs, cam, W, H, 1, 30, (1, 1, 1), lights, caustic_k=caustic_k)
    rgba, rgb = job.finish(gm, cm)
    rgb = rgb.cpu().numpy()
    st = pm_amd.render_stats()
    rng = np.random.default_rng(2024)
    checked = {}
    om = {"global": oracle.PhotonMap(og, 1.0, oc, 0.5, nthreads=NT), "caustic": oracle.PhotonMap(oc, 0.5, nthreads=NT)}
    for which, k in (("global", 50), ("caustic", caustic_k or 50)):
        q, r = job.queries(which)
        n = q.shape[0]
        assert n == (st.global_queries if which == "global" else st.caustic_queries)
        idx = torch.from_numpy(np.sort(rng.choice(n, size=min(SAMPLE, n), replace=False))).cuda()
        qs, rs = q[idx].cpu().numpy(), r[idx].cpu().numpy()
        pts = np.ascontiguousarray(qs[:, 0:3])
        want = om[which].gather(pts, np.ascontiguousarray(qs[:, 3]), nthreads=NT, k=k)
        assert np.array_equal(_bits(rs[:, 0:3]), _bits(want)), which
        assert np.count_nonzero(want) > 0.05 * want.size, which   # lit queries, not an all-zero comparison
        checked[which] = n
    job.close()
    # a BAND-row strip of the full-resolution frame at its centre, rendered by the
    # oracle over the full maps (simpleRayGen, ray-tracer/cuda/deviceCode.cu:
    # 191-231: camera paths, direct light, caustic gather, 20 final-gather rays
    # per vertex, the framebuffer row H - y written at :229-230)
    lo = H // 2 - BAND // 2
    ocam = oracle.camera_setup(*CAM, W, H)
    orgba, orgb, ost = oracle.render(os_, ocam, W, H, 1, 30, (1, 1, 1), lights, om["global"], om["caustic"],
                                     rows=(lo, lo + BAND), nthreads=NT, caustic_k=caustic_k)
    rows = slice(H - (lo + BAND) + 1, H - lo + 1)
    a, b = np.clip(rgb[rows], 0, 1), np.clip(orgb[rows], 0, 1)
    err = float(np.abs(a - b).max())
    exact = float(np.mean(np.all(_bits(rgb[rows]) == _bits(orgb[rows]), axis=-1)))
    assert ost.pixels == BAND * W
    assert err <= 1e-3, err
    assert exact >= 0.999, exact
    assert np.mean(rgba.cpu().numpy().view(np.uint32)[rows] != orgba[rows]) <= 0.001
    assert np.mean(orgb[rows]) > 0.01   # a lit band, not an all-black comparison
    checked["band_exact"] = exact
    # the same band under the alternative specifications of the reference's
    # unpinned behaviour (tests/test_spec_bounds.py): heap-order sums over
    # tree-index ids, domain-box split dimensions, nvcc contraction
    import test_spec_bounds as sb
    S = oracle.PhotonMap
    images = sb.spec_images(os_, lights, om["global"], om["caustic"], W, H,
                            (S.SPEC_HEAP, S.SPEC_HEAP | S.SPEC_DOMAIN_DIM,
                             S.SPEC_HEAP | S.SPEC_DOMAIN_DIM | S.SPEC_FMA),
                            rows=(lo, lo + BAND), caustic_k=caustic_k)
    assert np.array_equal(_bits(images[0]), _bits(orgb))   # the production spec is the band above
    bounds = sb.spec_bounds(images, rows)
    sb.report(f"config{'5' if caustic_k else '3'} band {BAND}x{W}", bounds)
    for f, (e, _) in bounds.items():
        assert e <= sb.TOL, (f, e)
    checked["spec_bounds"] = bounds
    del om
    return st, checked, gm.n, cm.n


def test_config3_full_size_vs_oracle():
    """BASELINE config 3 at the bench's size: Sponza-class scene, 10 M + 1 M
    photons, 1920x1080 spp 1, k = 50."""
    import oracle
    import pm_amd
    from pm_amd import scenes
    meshes, lights = scenes.sponza_class()
    gs, os_ = pm_amd.Scene(meshes), oracle.Scene(meshes)
    _trace_shards_vs_oracle(gs, os_, lights, 10_000_000, False)
    _trace_shards_vs_oracle(gs, os_, lights, 1_000_000, True)
    g = pm_amd.run_normal(gs, lights, 10_000_000, 10)
    c = pm_amd.run_caustics(gs, lights, 1_000_000, 10)
    st, checked, ng, nc = _frame_vs_oracle(gs, os_, lights, g, c, 0)
    assert ng > 40_000_000 and checked["global"] > 30_000_000, (ng, checked)


def test_config5_full_size_vs_oracle():
    """Config 5 at the bench's per-GPU size: square area light + glass, 10 M
    diffuse + 6.25 M caustic photons, caustic gather over k = 200."""
    import oracle
    import pm_amd
    from pm_amd import scenes
    meshes, lights = scenes.sponza_caustics()
    gs, os_ = pm_amd.Scene(meshes), oracle.Scene(meshes)
    _trace_shards_vs_oracle(gs, os_, lights, 10_000_000, False)
    _trace_shards_vs_oracle(gs, os_, lights, 6_250_000, True)
    g = pm_amd.run_normal(gs, lights, 10_000_000, 10)
    c = pm_amd.run_caustics(gs, lights, 6_250_000, 10)
    st, checked, ng, nc = _frame_vs_oracle(gs, os_, lights, g, c, 200)
    assert nc > 500_000 and checked["caustic"] > 2_000_000, (nc, checked)
