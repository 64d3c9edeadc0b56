#!/usr/bin/env python3
"""Concurrency probe (GPU box): pm_render_begin on a side stream from a second
host thread while the main thread traces photons and builds the kd-trees of
the same scene on the default stream. Every result is
compared bit for bit with the same calls run serially. Prints one line per
round; exit status 0 only if every round matches."""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "photon-mapping_amd")]


def main(rounds=3):
    import torch
    import pm_amd
    from pm_amd import scenes
    meshes, lights = scenes.sponza_class()
    sc = pm_amd.Scene(meshes)
    W, H = 640, 360
    cam = pm_amd.setup_camera((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87, W, H)

    def pipeline():
        g = pm_amd.run_normal(sc, lights, 2_000_000, 10)
        c = pm_amd.run_caustics(sc, lights, 200_000, 10)
        return g, c, pm_amd.PhotonMap(g, 1.0, c, 0.5), pm_amd.PhotonMap(c, 0.5)

    # serial reference
    g, c, gm, cm = pipeline()
    ref_rgba, ref_rgb = pm_amd.render(sc, cam, W, H, 1, 30, (1, 1, 1), lights, gm, cm)
    ref = [g.cpu().numpy(), c.cpu().numpy(), gm.export().cpu().numpy(), ref_rgb.cpu().numpy()]
    torch.cuda.synchronize()
    ok_all = True
    for r in range(rounds):
        side = torch.cuda.Stream()
        box = {}

        def begin():
            box["job"] = pm_amd.render_begin(sc, cam, W, H, 1, 30, (1, 1, 1), lights, stream=side.cuda_stream)

        th = threading.Thread(target=begin)
        th.start()
        g, c, gm, cm = pipeline()   # default stream, concurrently with the side stream's begin half
        th.join()
        rgba, rgb = box["job"].finish(gm, cm)
        box["job"].close()
        torch.cuda.synchronize()
        got = [g.cpu().numpy(), c.cpu().numpy(), gm.export().cpu().numpy(), rgb.cpu().numpy()]
        same = [np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(got, ref)]
        print(f"round {r}: photons {same[0]} caustic {same[1]} kd {same[2]} image {same[3]}", flush=True)
        ok_all &= all(same)
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
