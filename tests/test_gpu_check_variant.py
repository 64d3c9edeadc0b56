"""GPU parity of every alternate path against the production library.

lib_check/libpm_hip.so is built with PM_CHECK_VARIANT=1 and PM_STACK_DEPTH=4
(photon-mapping_amd/Makefile `check`, built by __graft_entry__.build()). It runs
the plain post-order kNN walk instead of the leader-seeded one, all-global kd
levels instead of the LDS finish, the Karras LBVH instead of PLOC, a one-slot
first guess for the render's continuation vertices (so every render reruns
k_paths), and keeps 4 traversal-stack entries in LDS (nearly every ray spills
to scratch). All of these are bit-identical by construction; the workloads of
tests/variant_workloads.py run once per library (the check variant in ONE child
process) and every output must match bit for bit. The full-size case is BASELINE
config 3: 10M + 1M photons on the Sponza-class scene, the 45.4M-photon map and
the 36M-query 1920x1080 final gather (seeded gather == plain walk at scale),
and config 5: 10M + 6.25M photons, the k = 200 caustic gather at 1920x1080.
The spill path is also checked against the CPU oracle directly."""
import os
import subprocess
import sys

import numpy as np
import pytest

import conftest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

PKG = os.path.join(conftest.ROOT, "photon-mapping_amd")
VARIANT = os.path.join(PKG, "lib_check", "libpm_hip.so")
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    assert os.path.exists(VARIANT), f"check variant not built ({VARIANT}): run __graft_entry__.build()"
    import variant_workloads
    out = str(tmp_path_factory.mktemp("variant") / "check.npz")
    env = dict(os.environ, PM_HIP_LIB=VARIANT)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "variant_workloads.py"), out, "--full"], env=env,
                       capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "lib_check/libpm_hip.so" in r.stdout, r.stdout
    prod = variant_workloads.run(full=True)
    return prod, dict(np.load(out))


KEYS = ["cloud_hits", "cloud_occ", "cloud_photons", "cornell_g", "cornell_c", "cornell_gmap", "cornell_cmap",
        "gather_g", "gather_c", "gather_e", "gather_k200", "gather_k256", "knn_ids", "knn_d2", "knn_md", "render_64_rgba", "render_64_rgb",
        "render_64_stats", "render_40_rgba", "render_40_rgb", "render_40_stats", "kd_5", "kd_1023", "kd_1024",
        "kd_70000", "kd_2000003", "kd_same_5000", "kd_wall_300001", "kd_special_70001", "sphere_g", "sphere_c", "sphere_rgb", "sphere_stats"]
FULL = ["c3_counts", "c3_g_crc", "c3_c_crc", "c3_gmap_crc", "c3_stats", "c3_rgba", "c3_rgb",
        "c5_counts", "c5_c_crc", "c5_cmap_crc", "c5_stats", "c5_rgba", "c5_rgb"]


@pytest.mark.parametrize("key", KEYS + FULL)
def test_check_variant_bitwise(runs, key):
    prod, check = runs
    a, b = prod[key], check[key]
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8)), key
    if key == "c3_stats":
        assert a[3] > 30_000_000   # the full-size final gather: > 30M global-map queries
    if key == "c3_counts":
        assert a[0] > 40_000_000   # > 40M photons in the global map
    if key == "c5_stats":
        assert a[2] > 2_000_000    # the full-size k = 200 caustic gather: > 2M queries


def test_spill_path_vs_oracle(runs):
    """The 4-entry-stack traversal (scratch spill) against the CPU oracle."""
    import oracle
    import pm_amd
    import variant_workloads as vw
    _, check = runs
    v, i = vw.cloud(30000, 7)
    rays = vw.cloud_rays(20000, 8)
    os_ = oracle.Scene([pm_amd.MeshData(v, i, vw.CLOUD_MAT)])
    assert np.array_equal(check["cloud_hits"].view(np.uint32), os_.intersect(rays).view(np.uint32))
    assert np.array_equal(check["cloud_occ"], os_.occluded(rays))
    po = oracle.trace(os_, vw.CLOUD_LIGHTS, 20000, 10, False)
    assert len(check["cloud_photons"]) == len(po) > 0
    assert np.array_equal(check["cloud_photons"].view(np.uint32), po.view(np.uint32))


def test_continuation_rerun_happened(runs):
    """The renders above had continuation vertices (so the check variant's
    one-slot guess was short and k_paths reran)."""
    prod, _ = runs
    st = prod["render_64_stats"]
    assert st[1] > st[0] * 2   # path_vertices > pixels x spp
