"""Isolated timing of config 5's caustic gather (k = 200 over the 647 k-photon
caustic map, the frame's own 2.3 M Morton-ordered caustic queries): render_begin,
then pm_render_gather_caustic timed alone with events, several frames.
PM_HIP_LIB selects a variant library (stats builds print walk statistics).
  python tools/wide_probe.py [--k 200] [--frames 4] [--caustic 6250000]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "photon-mapping_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=200)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--caustic", type=int, default=6_250_000)
    a = ap.parse_args()
    import torch
    import pm_amd
    from pm_amd import scenes
    meshes, lights = scenes.sponza_caustics()
    gs = pm_amd.Scene(meshes)
    c = pm_amd.run_caustics(gs, lights, a.caustic, 10)
    cm = pm_amd.PhotonMap(c, pm_amd.CAUSTICS_PHOTON_POWER)
    cam = pm_amd.setup_camera((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87, 1920, 1080)
    torch.cuda.synchronize()
    times = []
    for f in range(a.frames):
        job = pm_amd.render_begin(gs, cam, 1920, 1080, 1, 30, (1, 1, 1), lights, caustic_k=a.k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        job.gather_caustic(cm)
        e1.record()
        torch.cuda.synchronize()
        times.append((e0.elapsed_time(e1), (time.perf_counter() - t0) * 1e3))
        job.close()
    print(f"caustic map {cm.n} photons, k={a.k}: gather ms (events, wall) per frame: "
          + ", ".join(f"{x:.2f}/{y:.2f}" for x, y in times), flush=True)


if __name__ == "__main__":
    main()
