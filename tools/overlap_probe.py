#!/usr/bin/env python3
"""Times one config-3 frame serially and with pm_render_begin (camera paths,
final-gather and shadow rays, direct light: map-independent) on a side stream
from a second host thread while the main thread traces and builds the maps.
Prints wall ms of both and whether the images match bit for bit."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "photon-mapping_amd")]


def main(steps=3):
    import torch
    import pm_amd
    from pm_amd import scenes
    meshes, lights = scenes.sponza_class()
    sc = pm_amd.Scene(meshes)
    W, H = 1920, 1080
    cam = pm_amd.setup_camera((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87, W, H)

    def maps():
        g = pm_amd.run_normal(sc, lights, 10_000_000, 10)
        c = pm_amd.run_caustics(sc, lights, 1_000_000, 10)
        cm = pm_amd.PhotonMap(c, 0.5)
        return pm_amd.PhotonMap(g, 1.0, c, 0.5), cm

    def serial():
        gm, cm = maps()
        return pm_amd.render(sc, cam, W, H, 1, 30, (1, 1, 1), lights, gm, cm)[1]

    def overlapped():
        side = torch.cuda.Stream()
        box = {}
        th = threading.Thread(target=lambda: box.update(
            job=pm_amd.render_begin(sc, cam, W, H, 1, 30, (1, 1, 1), lights, stream=side.cuda_stream)))
        th.start()
        gm, cm = maps()
        th.join()
        rgb = box["job"].finish(gm, cm)[1]
        box["job"].close()
        return rgb

    res = {}
    for name, fn in (("serial", serial), ("overlapped", overlapped)) * 2:
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            img = fn()
        torch.cuda.synchronize()
        res[name] = ((time.perf_counter() - t) / steps * 1e3, img.cpu().numpy())
        print(f"{name}: {res[name][0]:.2f} ms/frame", flush=True)
    print("images bitwise equal:", np.array_equal(res["serial"][1].view(np.uint32), res["overlapped"][1].view(np.uint32)))


if __name__ == "__main__":
    main()
