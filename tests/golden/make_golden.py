#!/usr/bin/env python3
"""Generate tests/golden/golden.npz from the CPU oracle (SURVEY §8c golden plan).

The reference publishes no golden vectors and cannot run here, so these are
ORACLE-generated regression fixtures (parity vs the reference: unpinned):
  * owl::LCG<16> states/draws for seeds (0,0), (1,0), (600,330)
  * bits of the spec's acos / sin / cos on a fixed grid
  * Cornell box (reference asset), 10k diffuse + 10k caustic photons, max_depth 10:
    counts, sha256 of the full arrays, first 1000 records of each
  * k = 50 kNN ids (original indices) for 1000 seeded queries on the global map
  * 64x48, spp 1, depth 30 render (float rgb + RGBA8) with the config.toml.example camera
Run: python tests/golden/make_golden.py   (after `make -C oracle`)
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "photon-mapping_amd")]

import oracle  # noqa: E402
import pm_amd  # noqa: E402  (host-side ingest only; no GPU)

CAM = ((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def build():
    out = {}
    for i, seed in enumerate([(0, 0), (1, 0), (600, 330)]):
        st = oracle.lib.orc_lcg_init(*seed)
        s = C.c_uint32(st)
        draws = [oracle.lib.orc_lcg_next(C.byref(s)) for _ in range(16)]
        out[f"lcg_{i}_state"] = np.uint32(st)
        out[f"lcg_{i}_draws"] = np.float32(draws)
    x = np.linspace(-1, 1, 257, dtype=np.float32)
    t = np.linspace(0, 6.2831855, 257, dtype=np.float32)
    out["trig_x"], out["trig_t"] = x, t
    out["acos"] = np.float32([oracle.lib.orc_acosf(float(v)) for v in x])
    out["sin"] = np.float32([oracle.lib.orc_sinf(float(v)) for v in t])
    out["cos"] = np.float32([oracle.lib.orc_cosf(float(v)) for v in t])
    meshes, lights = pm_amd.load_scene_file(os.path.join(HERE, "scenes", "cornell-box", "cornell-box.glb"))
    sc = oracle.Scene(meshes)
    g = oracle.trace(sc, lights, 10000, 10, False)
    c = oracle.trace(sc, lights, 10000, 10, True)
    out["cornell_global_count"], out["cornell_caustic_count"] = np.int64(len(g)), np.int64(len(c))
    out["cornell_global_sha256"] = np.bytes_(sha(g))
    out["cornell_caustic_sha256"] = np.bytes_(sha(c))
    out["cornell_global_head"], out["cornell_caustic_head"] = g[:1000], c[:1000]
    gm, cm = oracle.PhotonMap(g, 1.0, c, 0.5), oracle.PhotonMap(c, 0.5)
    rng = np.random.default_rng(2024)
    q = rng.uniform([-20, 0, -20], [20, 40, 20], size=(1000, 3)).astype(np.float32)
    ids, d2, md = gm.knn(q, 50, 100.0)
    out["knn_queries"], out["knn_ids"], out["knn_maxd2"] = q, ids, md
    cam = oracle.camera_setup(*CAM, 64, 48)
    rgba, rgb, _ = oracle.render(sc, cam, 64, 48, 1, 30, (1.0, 1.0, 1.0), lights, gm, cm)
    out["img_rgba"], out["img_rgb"] = rgba, rgb
    return out


if __name__ == "__main__":
    out = build()
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print({k: (v.shape if hasattr(v, "shape") else v) for k, v in out.items()})
