"""How much would a SPATIAL split of the final gather's queries buy at N > 1?
(design probe, not product.) Config 4's 8-rank global map on one GPU
(pm_amd.replay.record), then pm_gather timed on 1/8 of the frame's global-gather
queries chosen two ways:
  tiles     rank r's own queries (its round-robin 16x16 tiles, dist.frame's split);
  spatial   the r-th eighth of ALL the frame's queries in Morton order (what an
            all-to-all of queries by key range would hand rank r).
Both walk their set in Morton order (pm_gather keeps the given order)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "photon-mapping_amd"))
import torch  # noqa: E402

import pm_amd  # noqa: E402
from pm_amd import dist as pmdist, replay, scenes  # noqa: E402

W, H, G = 1920, 1080, int(os.environ.get("WORLD", "8"))
CAM = ((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87)
torch.cuda.set_device(0)
meshes, lights = scenes.sponza_class()
scene = pm_amd.Scene(meshes)
cfg = pmdist.FrameConfig(casted=10_000_000 * G, caustic=1_000_000 * G, width=W, height=H)
rec = replay.record(scene, lights, cfg, G, keep_map=False)
g, c = rec.gathered()
gm, cm = pm_amd.PhotonMap(g, 1.0, c, 0.5), pm_amd.PhotonMap(c, 0.5)
cam = pm_amd.setup_camera(*CAM, W, H)


def morton(q):
    lo, hi = q.min(0).values, q.max(0).values
    u = ((q - lo) / (hi - lo).clamp_min(1e-30) * 1023.0).clamp(0, 1023).to(torch.int64)
    def spread(v):
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        v = (v | (v << 2)) & 0x09249249
        return v
    return (spread(u[:, 0]) << 2) | (spread(u[:, 1]) << 1) | spread(u[:, 2])


def timed_gather(q):
    q = q[torch.argsort(morton(q[:, 0:3]))].contiguous()
    pts, brdf = q[:, 0:3].contiguous(), q[:, 3].contiguous()
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pm_amd.gather_photons(gm, pts, brdf)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
    return ms


job = pm_amd.render_begin(scene, cam, W, H, 1, 30, (1, 1, 1), lights)
job.finish(gm, cm, want_rgb=False)
qa, _ = job.queries("global", results=False)
qa = qa.clone()
job.close()
print(f"map {gm.n} photons, frame queries {qa.shape[0]}; full set: {timed_gather(qa):.2f} ms", flush=True)
order = torch.argsort(morton(qa[:, 0:3]))
n = qa.shape[0]
for r in range(G):
    jr = pm_amd.render_begin(scene, cam, W, H, 1, 30, (1, 1, 1), lights, tile_rank=r, tile_count=G)
    jr.finish(gm, cm, want_rgb=False)
    qt, _ = jr.queries("global", results=False)
    qt = qt.clone()
    jr.close()
    qs = qa[order[r * n // G: (r + 1) * n // G]]
    print(f"rank {r}: tiles {qt.shape[0]} queries {timed_gather(qt):.2f} ms | spatial {qs.shape[0]} queries "
          f"{timed_gather(qs):.2f} ms", flush=True)
