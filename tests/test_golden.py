"""Committed golden fixtures (tests/golden/golden.npz, made by make_golden.py):
the oracle must keep reproducing them (CPU), and the HIP path must match them
(GPU) without consulting the oracle at all."""
import ctypes as C
import hashlib
import os

import numpy as np
import pytest

import conftest

G = np.load(os.path.join(conftest.GOLDEN, "golden.npz"))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest().encode()


def test_oracle_reproduces_lcg_and_trig():
    import oracle
    for i, seed in enumerate([(0, 0), (1, 0), (600, 330)]):
        st = oracle.lib.orc_lcg_init(*seed)
        assert st == int(G[f"lcg_{i}_state"])
        s = C.c_uint32(st)
        d = np.float32([oracle.lib.orc_lcg_next(C.byref(s)) for _ in range(16)])
        assert np.array_equal(d.view(np.uint32), G[f"lcg_{i}_draws"].view(np.uint32))
    a = np.float32([oracle.lib.orc_acosf(float(v)) for v in G["trig_x"]])
    s = np.float32([oracle.lib.orc_sinf(float(v)) for v in G["trig_t"]])
    c = np.float32([oracle.lib.orc_cosf(float(v)) for v in G["trig_t"]])
    for got, key in ((a, "acos"), (s, "sin"), (c, "cos")):
        assert np.array_equal(got.view(np.uint32), G[key].view(np.uint32))


def _cornell_oracle():
    import oracle
    import pm_amd
    meshes, lights = pm_amd.load_scene_file(conftest.CORNELL)
    sc = oracle.Scene(meshes)
    return oracle, sc, lights


def test_oracle_reproduces_cornell_photons_knn_image():
    oracle, sc, lights = _cornell_oracle()
    g = oracle.trace(sc, lights, 10000, 10, False)
    c = oracle.trace(sc, lights, 10000, 10, True)
    assert len(g) == int(G["cornell_global_count"]) and len(c) == int(G["cornell_caustic_count"])
    assert _sha(g) == G["cornell_global_sha256"].item() and _sha(c) == G["cornell_caustic_sha256"].item()
    gm, cm = oracle.PhotonMap(g, 1.0, c, 0.5), oracle.PhotonMap(c, 0.5)
    ids, _, md = gm.knn(G["knn_queries"], 50, 100.0)
    assert np.array_equal(ids, G["knn_ids"]) and np.array_equal(md.view(np.uint32), G["knn_maxd2"].view(np.uint32))
    cam = oracle.camera_setup((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 64, 48)
    rgba, rgb, _ = oracle.render(sc, cam, 64, 48, 1, 30, (1, 1, 1), lights, gm, cm)
    assert np.array_equal(rgba, G["img_rgba"]) and np.array_equal(rgb.view(np.uint32), G["img_rgb"].view(np.uint32))


@pytest.mark.gpu
def test_hip_matches_golden():
    torch = pytest.importorskip("torch")
    import pm_amd
    meshes, lights = pm_amd.load_scene_file(conftest.CORNELL)
    s = pm_amd.Scene(meshes)
    g = pm_amd.run_normal(s, lights, 10000, 10)
    c = pm_amd.run_caustics(s, lights, 10000, 10)
    gn, cn = g.cpu().numpy(), c.cpu().numpy()
    assert _sha(gn) == G["cornell_global_sha256"].item() and _sha(cn) == G["cornell_caustic_sha256"].item()
    gm, cm = pm_amd.load_photons(g, c)
    ids, _, md = pm_amd.knn(gm, torch.from_numpy(G["knn_queries"]).cuda(), 50, 100.0)
    assert np.array_equal(ids.cpu().numpy(), G["knn_ids"])
    cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 64, 48)
    rgba, rgb = pm_amd.render(s, cam, 64, 48, 1, 30, (1, 1, 1), lights, gm, cm)
    err = np.abs(np.clip(rgb.cpu().numpy(), 0, 1) - np.clip(G["img_rgb"], 0, 1)).max()
    assert err <= 1e-3
    assert np.mean(rgba.cpu().numpy().view(np.uint32) != G["img_rgba"]) <= 0.001
