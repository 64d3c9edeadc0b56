#!/usr/bin/env python3
"""A/B of build variants (GPU box): one config-3 frame pipeline through the
library PM_HIP_LIB names (default: lib/), timed per phase (HIP events), plus an
order-sensitive digest of the float image so that variants can be checked for
bit-identical output. Prints one JSON line.
    PM_HIP_LIB=photon-mapping_amd/lib_x/libpm_hip.so python tools/ab_frame.py [--steps N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "photon-mapping_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--scene", default="sponza", choices=["sponza", "caustics", "cornell"])
    ap.add_argument("--casted", type=int, default=10_000_000)
    ap.add_argument("--caustic", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--caustic-k", type=int, default=0)
    a = ap.parse_args()
    import torch
    import pm_amd
    from pm_amd import scenes
    from variant_workloads import _digest
    if a.scene == "sponza":
        meshes, lights = scenes.sponza_class()
    elif a.scene == "caustics":
        meshes, lights = scenes.sponza_caustics()
    else:
        meshes, lights = pm_amd.load_scene_file(os.path.join(ROOT, "tests", "golden", "scenes", "cornell-box",
                                                             "cornell-box.glb"))
    sc = pm_amd.Scene(meshes)
    cam = pm_amd.setup_camera((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87, a.width, a.height)
    ph = {}
    dig = None
    for step in range(a.steps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = pm_amd.run_normal(sc, lights, a.casted, 10)
        tr = pm_amd.phase_us("trace") + pm_amd.phase_us("compact")
        c = pm_amd.run_caustics(sc, lights, a.caustic, 10)
        tr += pm_amd.phase_us("trace") + pm_amd.phase_us("compact")
        cm = pm_amd.PhotonMap(c, pm_amd.CAUSTICS_PHOTON_POWER)
        kd = pm_amd.phase_us("kdbuild")
        gm = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
        kd += pm_amd.phase_us("kdbuild")
        rgba, rgb = pm_amd.render(sc, cam, a.width, a.height, 1, 30, (1, 1, 1), lights, gm, cm,
                                  caustic_k=a.caustic_k)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        cur = {"wall": wall, "trace": tr / 1e3, "kdbuild": kd / 1e3}
        for k in ("paths", "gather", "gather_global", "resolve"):
            cur[k] = pm_amd.phase_us(k) / 1e3
        if step == 0:
            dig = _digest(rgb).tolist()
            continue
        for k, v in cur.items():
            ph[k] = ph.get(k, 0.0) + v / a.steps
        del g, c, gm, cm, rgba, rgb
    print(json.dumps({"lib": os.path.relpath(pm_amd.LIB_PATH, ROOT), "digest": dig,
                      "ms": {k: round(v, 3) for k, v in ph.items()}}), flush=True)


if __name__ == "__main__":
    main()
