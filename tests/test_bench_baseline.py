"""bench.py's cpu_baseline leg on a tiny Cornell workload (CPU only): both map
modes run, report their sample honestly, and give a positive rate. The full-
photon mode takes the frame's photon sets (here the oracle's own trace stands
in for the GPU's, which is bitwise equal to it: tests/test_gpu_fullsize.py)."""
import types

import conftest


def _args(**kw):
    a = dict(casted=4000, caustic=2000, max_depth=10, cpu_sample_photons=1000, width=32, height=24, spp=1,
             depth=30, caustic_k=50, cpu_sample_rows=4)
    a.update(kw)
    return types.SimpleNamespace(**a)


def test_cpu_baseline_modes():
    import bench
    import oracle
    import pm_amd
    meshes, lights = pm_amd.load_scene_file(conftest.CORNELL)
    a = _args()
    sc = oracle.Scene(meshes)
    g = oracle.trace(sc, lights, a.casted, a.max_depth, False, nthreads=2)
    c = oracle.trace(sc, lights, a.caustic, a.max_depth, True, nthreads=2)
    n_full = len(g) + len(c)
    full = bench.cpu_baseline(meshes, lights, a, n_full, 2, full_photons=(g, c))
    samp = bench.cpu_baseline(meshes, lights, a, n_full, 2)
    for r in (full, samp):
        assert r["value"] > 0 and r["cores"] == 2 and r["kind"] == "port"
        assert set(r["phase_s"]) == {"trace", "build", "render"}
    assert "full maps" in full["sample"] and f"({n_full} photons" in full["sample"]
    assert "sparser" in samp["sample"]
