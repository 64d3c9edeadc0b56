"""Per-rank cost of the N-GPU frame, measured on one GPU:
weak scaling as bench.py --gpus N runs it (10 M + 1 M photons per GPU; config
5: 10 M + 6.25 M, caustic k = 200), every rank's production frame run through
pm_amd.replay (collectives replayed from a recording: the photon and tag
all-gathers become device copies, the top selection's all-reduces writes of
the recorded sums). Prints one JSON line per N with each rank's frame ms, the
slowest rank's phases, and a projection that puts back what one GPU cannot
measure: the RCCL all-gathers over xGMI at an assumed receive bandwidth.

  WORLDS="2 4 8"  CONFIG=3|5  XGMI_GBS="300 450"  (effective all-gather receive
  bandwidth per GPU, GB/s; MI355X: 7 xGMI links per GPU)  RANKS="0 2" (ranks to
  run; default all)  REPS=2 (frames per rank, the last is reported)
  FRAME_OPTS="begin_after_trace=0" (boolean FrameConfig fields, comma-separated)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "photon-mapping_amd"))
import torch  # noqa: E402

import pm_amd  # noqa: E402
from pm_amd import dist as pmdist  # noqa: E402
from pm_amd import replay  # noqa: E402
from pm_amd import scenes  # noqa: E402

CAMERA = dict(look_from=(80.0, 30.0, 0.0), look_at=(10.0, 20.0, 0.0), look_up=(0.0, 1.0, 0.0), fovy=0.87)
config = int(os.environ.get("CONFIG", "3"))
per_gpu = (10_000_000, 6_250_000 if config == 5 else 1_000_000)
caustic_k = 200 if config == 5 else 0
meshes, lights = scenes.sponza_caustics() if config == 5 else scenes.sponza_class()
torch.cuda.set_device(0)
scene = pm_amd.Scene(meshes)
bws = [float(x) for x in os.environ.get("XGMI_GBS", "300 450").split()]

for world in [int(x) for x in os.environ.get("WORLDS", "2 4 8").split()]:
    cfg = pmdist.FrameConfig(casted=per_gpu[0] * world, caustic=per_gpu[1] * world, width=1920, height=1080,
                             camera=CAMERA, caustic_k=caustic_k)
    for opt in filter(None, os.environ.get("FRAME_OPTS", "").split(",")):
        k, v = opt.split("=")
        setattr(cfg, k, v == "1")
    t0 = time.time()
    rec = replay.record(scene, lights, cfg, world, keep_map=False)
    t_rec = time.time() - t0
    emitted = sum(pm_amd.compute_photons_per_watt(lights, cfg.casted)) + \
        sum(pm_amd.compute_photons_per_watt(lights, cfg.caustic))
    ranks = []
    sel = [int(x) for x in os.environ["RANKS"].split()] if os.environ.get("RANKS") else range(world)
    for r in [r for r in sel if r < world]:
        for rep in range(int(os.environ.get("REPS", "2"))):   # the first frame of a rank pays its allocations
            _, info, ms = replay.rank_frame(rec, scene, lights, cfg, r)
        ranks.append((ms, {k: round(v / 1e3, 2) for k, v in info["us"].items()}))
        print(f"# N={world} rank {r}: {ms:.1f} ms {ranks[-1][1]}", file=sys.stderr, flush=True)
    slow = max(range(len(ranks)), key=lambda r: ranks[r][0])
    ms, ph = ranks[slow]
    slow = list(sel)[slow]
    tags_bytes = (world - 1) / world * sum(rec.plan_sizes) * 4
    proj = {}
    for bw in bws:
        t_rows = rec.exchange_bytes() / (bw * 1e9) * 1e3
        t_tags = tags_bytes / (bw * 1e9) * 1e3
        # the photon all-gather overlaps the caustic map and the top selection
        # (the replayed exchange window holds those plus the device copies)
        f = ms - ph.get("exchange", 0.0) + max(ph.get("exchange", 0.0), t_rows) + t_tags
        proj[f"{bw:g}GBs"] = {"allgather_rows_ms": round(t_rows, 2), "allgather_tags_ms": round(t_tags, 2),
                              "frame_ms": round(f, 2), "mphotons_s": round(emitted / f / 1e3, 1)}
    print(json.dumps({
        "config": config, "world": world, "emitted": emitted, "global_map": sum(rec.ns_g) + sum(rec.ns_c),
        "subtrees": len(rec.plan_sizes), "record_s": round(t_rec, 1),
        "rank_frame_ms": [round(x[0], 2) for x in ranks], "slowest_rank": slow, "slowest_phases_ms": ph,
        "replayed_mphotons_s": round(emitted / ms / 1e3, 1),
        "exchange_gb_in_per_rank": round(rec.exchange_bytes() / 1e9, 3), "projection": proj}), flush=True)
    del rec
    torch.cuda.empty_cache()
