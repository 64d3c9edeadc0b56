"""GPU parity of the traversal-stack spill path.

The BVH4 traversal keeps the top PM_STACK_DEPTH stack entries in LDS and
spills deeper ones to private (scratch) memory (pm_device.hpp, traverse). At
the production depth (32) Sponza-class scenes rarely reach the spill region, so
this test loads a variant library built with PM_STACK_DEPTH=4 — nearly every
ray spills — in ONE child process, and checks closest-hit, any-hit and photon
tracing bit for bit against the CPU oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

import conftest

pytestmark = pytest.mark.gpu

PKG = os.path.join(conftest.ROOT, "photon-mapping_amd")
VARIANT = os.path.join(PKG, "lib_s4", "libpm_hip.so")

CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [{pkg!r}]
import pm_amd
assert pm_amd.LIB_PATH.endswith("lib_s4/libpm_hip.so"), pm_amd.LIB_PATH
d = np.load({inp!r})
meshes = [pm_amd.MeshData(d["v"], d["i"], d["mat"])]
sc = pm_amd.Scene(meshes)
rays = torch.from_numpy(d["rays"]).cuda()
hits = sc.intersect(rays).cpu().numpy()
occ = sc.occluded(rays).cpu().numpy()
lights = [dict(pos=(0.1, 0.2, 0.3), rgb=(1, 1, 1), power=100.0)]
ph = pm_amd.run_normal(sc, lights, 20000, 10).cpu().numpy()
np.savez({out!r}, hits=hits, occ=occ, ph=ph)
"""


def _ensure_variant():
    # incremental: rebuilds only when a source is newer than the variant
    subprocess.run(["make", "-j16", "BUILD=build_s4", "LIB=lib_s4/libpm_hip.so", "EXTRA=-DPM_STACK_DEPTH=4",
                        "variant"], cwd=PKG, check=True, timeout=900)


def _cloud(n, seed):
    """n small randomly oriented triangles filling a cube: rays cross many
    overlapping boxes, so the traversal stack grows deep."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, size=(n, 1, 3))
    v = (c + rng.normal(scale=0.6, size=(n, 3, 3))).reshape(-1, 3).astype(np.float32)
    return v, np.arange(3 * n, dtype=np.int32).reshape(n, 3)


def test_spill_path_bitwise(tmp_path):
    import oracle
    import pm_amd
    _ensure_variant()
    v, i = _cloud(30000, seed=7)
    rng = np.random.default_rng(8)
    n = 20000
    o = rng.uniform(-12, 12, size=(n, 3)).astype(np.float32)
    dr = rng.normal(size=(n, 3)).astype(np.float32)
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 3], rays[:, 4:7], rays[:, 7] = o, 1e-3, dr, 1e10
    rays[n // 2:, 7] = 3.0
    inp, out = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    mat = np.array([0.7, 0.6, 0.5, 0.6, 0.2, 0.2, 1.5], np.float32)
    np.savez(inp, v=v, i=i, rays=rays, mat=mat)
    env = dict(os.environ, PM_HIP_LIB=VARIANT)
    r = subprocess.run([sys.executable, "-c", CHILD.format(pkg=PKG, inp=inp, out=out)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    g = np.load(out)
    meshes = [pm_amd.MeshData(v, i, mat)]
    os_ = oracle.Scene(meshes)
    ho = os_.intersect(rays)
    assert np.array_equal(g["hits"].view(np.uint32), ho.view(np.uint32))
    assert np.array_equal(g["occ"], os_.occluded(rays))
    lights = [dict(pos=(0.1, 0.2, 0.3), rgb=(1, 1, 1), power=100.0)]
    po = oracle.trace(os_, lights, 20000, 10, False)
    assert len(g["ph"]) == len(po) > 0
    assert np.array_equal(g["ph"].view(np.uint32), po.view(np.uint32))
