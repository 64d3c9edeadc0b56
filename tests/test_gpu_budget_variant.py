"""The gather's leader-budget retry path against the production library.

lib_budget/libpm_hip.so is built with PM_LEADER_BUDGET=4 (photon-mapping_amd/
Makefile `budget`, built by __graft_entry__.build()): a leader wave stops after
4 walk iterations, so nearly every leader writes no seed record and is re-walked
by the retry workgroups at the head of the follower launch (csrc/knn.hip,
k_gather_level), while the followers fall back to whatever leaders finished
(none: the plain cut-off). Production uses a budget of 2048 wave iterations,
which mostly the Cornell box's wandering leader walks reach. The variant also
switches every gather walk to subtree-box skips after one iteration
(PM_BOX_AFTER=1; production: after 512, which these small workloads rarely
reach), so the box path runs on all of them, addresses kd nodes with 64
bits (PM_FORCE_WIDE=1; production: maps of >= 2^28 nodes only), and builds
every kd-tree with the selection build (PM_KD_SEL_MIN=0; production: maps of
>= 2^22 elements, the presorted build below), and keeps only 4 traversal-stack
entries in LDS (PM_STACK_DEPTH=4: the fused photon-path kernel and the render's
ray pools spill to scratch on the deep-stack scene; the check variant, which
also has a 4-entry stack, traces photons with the per-bounce wavefront path), so its trees of these small
workloads (ties, duplicates, one repeated point, axis planes, signed zeros
and infinities) must equal production's presorted ones. The lists
and radiance must not depend on any of it: the small workloads of tests/variant_workloads.py (seeded
gathers with ties and duplicates, Cornell and sphere renders) run in one child
process with the variant and must match production bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

import conftest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

PKG = os.path.join(conftest.ROOT, "photon-mapping_amd")
VARIANT = os.path.join(PKG, "lib_budget", "libpm_hip.so")
HERE = os.path.dirname(os.path.abspath(__file__))

KEYS = ["cloud_hits", "cloud_occ", "cloud_photons", "cornell_g", "cornell_c", "gather_g", "gather_c", "gather_e", "gather_k200", "gather_k256", "render_64_rgba", "render_64_rgb", "render_64_stats", "render_40_rgba",
        "render_40_rgb", "render_40_stats", "sphere_rgb", "sphere_stats", "cornell_gmap", "cornell_cmap",
        "kd_5", "kd_1023", "kd_1024", "kd_70000", "kd_2000003", "kd_same_5000", "kd_wall_300001",
        "kd_special_70001"]


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    assert os.path.exists(VARIANT), f"budget variant not built ({VARIANT}): run __graft_entry__.build()"
    import variant_workloads
    out = str(tmp_path_factory.mktemp("budget") / "budget.npz")
    env = dict(os.environ, PM_HIP_LIB=VARIANT)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "variant_workloads.py"), out], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "lib_budget/libpm_hip.so" in r.stdout, r.stdout
    return variant_workloads.run(full=False), dict(np.load(out))


@pytest.mark.parametrize("key", KEYS)
def test_budget_variant_bitwise(runs, key):
    prod, var = runs
    a, b = prod[key], var[key]
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8)), key
