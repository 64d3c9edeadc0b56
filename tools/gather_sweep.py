#!/usr/bin/env python3
"""One-process A/B of gather variants on the config-3 workload (trace once,
then per variant: rebuild the photon maps, render, read the global gather
kernel time). Usage: python tools/gather_sweep.py ENV=VAL[,ENV=VAL] ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "photon-mapping_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pm_amd  # noqa: E402
from pm_amd import scenes  # noqa: E402

meshes, lights = scenes.sponza_class()
sc = pm_amd.Scene(meshes)
casted = int(os.environ.get("CASTED", "10000000"))
g = pm_amd.run_normal(sc, lights, casted, 10)
c = pm_amd.run_caustics(sc, lights, casted // 10, 10)
cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 1920, 1080)
res, ref = {}, None
for rnd in range(2):
    for v in sys.argv[1:]:
        for kv in v.split(","):
            k, val = kv.split("=")
            os.environ[k] = val
        gm, cm = pm_amd.load_photons(g, c)
        rgba, rgb = pm_amd.render(sc, cam, 1920, 1080, 1, 30, (1, 1, 1), lights, gm, cm)
        img = rgb.cpu().numpy()
        if ref is None:
            ref = img
        same = bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)))
        res.setdefault(v, []).append((round(pm_amd.phase_us("gather_global") / 1e3, 2), same))
        del gm, cm
for v, r in res.items():
    print(f"{v}: gather_global ms / bitwise-equal-to-first {r}")
