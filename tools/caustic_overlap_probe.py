#!/usr/bin/env python3
"""Config-3 frame pieces timed one by one (host-synchronised), then the frame
serially and with the caustic pass (caustic trace + caustic kd build: small,
under-filled launches) on a side stream from a second host thread while the
main thread traces the global photons. Prints ms and whether the images match
bit for bit."""
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
    cap_g = pm_amd.trace_capacity(lights, 10_000_000, 10, False)
    cap_c = pm_amd.trace_capacity(lights, 1_000_000, 10, True)
    gbuf = torch.empty((cap_g, 10), dtype=torch.float32, device="cuda")
    cbuf = torch.empty((cap_c, 10), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((H, W), dtype=torch.int32, device="cuda")

    def timed(label, fn, acc):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        acc[label] = acc.get(label, 0.0) + (time.perf_counter() - t) * 1e3
        return r

    acc = {}
    for it in range(steps + 1):
        if it == 1:
            acc = {}
        g = timed("trace_global", lambda: pm_amd.run_normal(sc, lights, 10_000_000, 10, out=gbuf), acc)
        c = timed("trace_caustic", lambda: pm_amd.run_caustics(sc, lights, 1_000_000, 10, out=cbuf), acc)
        cm = timed("map_caustic", lambda: pm_amd.PhotonMap(c, 0.5), acc)
        gm = timed("map_global", lambda: pm_amd.PhotonMap(g, 1.0, c, 0.5), acc)
        timed("render", lambda: pm_amd.render(sc, cam, W, H, 1, 30, (1, 1, 1), lights, gm, cm, want_rgb=False,
                                              rgba=rgba), acc)
        del gm, cm
    print(" ".join(f"{k}={v / steps:.2f}" for k, v in acc.items()), "ms", flush=True)

    def serial():
        g = pm_amd.run_normal(sc, lights, 10_000_000, 10, out=gbuf)
        c = pm_amd.run_caustics(sc, lights, 1_000_000, 10, out=cbuf)
        cm = pm_amd.PhotonMap(c, 0.5)
        gm = pm_amd.PhotonMap(g, 1.0, c, 0.5)
        pm_amd.render(sc, cam, W, H, 1, 30, (1, 1, 1), lights, gm, cm, want_rgb=False, rgba=rgba)
        return rgba.clone()

    side = torch.cuda.Stream()

    def overlapped():
        box = {}

        def caustic_pass():
            with torch.cuda.stream(side):
                c = pm_amd.run_caustics(sc, lights, 1_000_000, 10, out=cbuf, stream=side.cuda_stream)
                box["c"] = c
                box["cm"] = pm_amd.PhotonMap(c, 0.5, stream=side.cuda_stream)
            side.synchronize()

        th = threading.Thread(target=caustic_pass)
        th.start()
        g = pm_amd.run_normal(sc, lights, 10_000_000, 10, out=gbuf)
        th.join()
        gm = pm_amd.PhotonMap(g, 1.0, box["c"], 0.5)
        pm_amd.render(sc, cam, W, H, 1, 30, (1, 1, 1), lights, gm, box["cm"], want_rgb=False, rgba=rgba)
        return rgba.clone()

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
    print("images bitwise equal:", np.array_equal(res["serial"][1], res["overlapped"][1]), flush=True)


if __name__ == "__main__":
    main()
