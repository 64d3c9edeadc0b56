#!/usr/bin/env python3
"""bench.py — photon-mapping hot path on MI355X (BASELINE.json metric).

One step = one full frame of the reference pipeline on synthetic input:
  trace    runNormal + runCaustics (photon-mapping/src/hostCode.cu:112-138)
  exchange all-gather of the photon buffers over RCCL (N > 1 only)
  build    loadPhotons: global + caustic kd-trees (ray-tracer/src/hostCode.cu:54-99)
  render   owlRayGenLaunch2D(simpleRayGen) final gather (ray-tracer/src/hostCode.cu:231-237)
Workload (BASELINE config 3): Sponza-class procedural scene (pm_amd.scenes,
~267k triangles, 373 meshes; Sponza itself is not available offline),
10M diffuse + 1M caustic photons per GPU, 1920x1080, spp 1, depth 30,
k = 50, max_depth 10. value = emitted photons of the whole job / wall time of
a step (Mphotons/s traced + gathered). N > 1: photon-index sharding with a
single all-gather, sharded kd-tree build (top levels selected from every
rank's own photons, subtrees built per rank), 16x16-tile-sharded final gather,
image reduce to rank 0 ("weak": photons per GPU fixed, config 4 at N = 8).
--config 5: the caustics pass (square area light + glass, 6.25M caustic photons
per GPU = 50M at N = 8, caustic gather over k = 200); the default line is config 3.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "photon-mapping_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
CAMERA = dict(look_from=(80.0, 30.0, 0.0), look_at=(10.0, 20.0, 0.0), look_up=(0.0, 1.0, 0.0), fovy=0.87)
SKY = (1.0, 1.0, 1.0)


def knn_query_bytes(n_photons: int, k: int = 50) -> int:
    """Algorithmic bytes of one kNN radiance query: 16*ceil(log2 N) + 28*k + 24."""
    return 16 * math.ceil(math.log2(max(2, n_photons))) + 28 * k + 24


def host_cores():
    """(threads to use, os.cpu_count(), affinity-mask CPUs, cgroup CPU quota or None).
    The CPU baseline runs on every CPU this process may use: the affinity mask,
    capped by the cgroup v2 CPU quota when one is set (extra threads beyond a
    quota only time-slice)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        quota = None
    use = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    return use, nproc, aff, quota


def cpu_baseline(meshes, lights, args, n_global_full, nthreads, full_photons=None):
    """Scalar oracle (oracle/libpm_oracle.so, pthreads) on a bounded sample of the
    same workload, scaled linearly to one frame. full_photons = (diffuse,
    caustic) pm_photon arrays of the whole frame (the GPU trace's; three 1 %
    id-shards of the same full-size trace are checked bitwise against the
    oracle's in tests/test_gpu_fullsize.py, not the whole array): the maps are then built from all of
    them (timed, not scaled) and the sampled rows are rendered over maps of the
    frame's own photon density; without them, maps of the traced sample."""
    import numpy as np
    import oracle
    t0 = time.time()
    sc = oracle.Scene(meshes)
    counts_g = oracle.photons_per_light(lights, args.casted)
    counts_c = oracle.photons_per_light(lights, args.caustic)
    P = sum(counts_g) + sum(counts_c)
    frac = min(1.0, args.cpu_sample_photons / max(1, sum(counts_g)))
    sg = int(sum(counts_g) * frac)
    scn = int(sum(counts_c) * frac)
    t = time.time()
    g = oracle.trace(sc, lights, args.casted, args.max_depth, False, nthreads=nthreads, g_range=(0, sg))
    c = oracle.trace(sc, lights, args.caustic, args.max_depth, True, nthreads=nthreads, g_range=(0, scn))
    t_trace = (time.time() - t) / frac
    if full_photons is not None:
        g, c = full_photons
    t = time.time()
    gm = oracle.PhotonMap(g, 1.0, c, 0.5, nthreads=nthreads)
    cm = oracle.PhotonMap(c, 0.5, nthreads=nthreads)
    t_build_s = time.time() - t
    n_s = max(2, len(g) + len(c))
    t_build = t_build_s * (n_global_full / n_s) * (math.log2(max(2, n_global_full)) / math.log2(n_s))
    cam = oracle.camera_setup(CAMERA["look_from"], CAMERA["look_at"], CAMERA["look_up"], CAMERA["fovy"],
                              args.width, args.height)
    rows = args.cpu_sample_rows
    r0 = args.height // 2 - rows // 2
    t = time.time()
    oracle.render(sc, cam, args.width, args.height, args.spp, args.depth, SKY, lights, gm, cm,
                  rows=(r0, r0 + rows), nthreads=nthreads, caustic_k=args.caustic_k)
    t_render = (time.time() - t) * args.height / rows
    total = t_trace + t_build + t_render
    _, nproc, aff, quota = host_cores()
    return {
        "value": P / total / 1e6, "unit": "Mphotons/s", "cores": nthreads, "kind": "port",
        "nproc": nproc, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
        "sample": (f"oracle (pthreads x{nthreads}) traced {sg + scn} of {P} photons (scaled x{1 / frac:.1f}), "
                   + (f"kd-built the frame's full maps ({n_s} photons: the GPU trace's, whose 1 % id-shards "
                      f"0/37/99 tests/test_gpu_fullsize.py checks bitwise against the oracle's), rendered {rows} of {args.height} rows at {args.width} px (scaled "
                      f"x{args.height / rows:.1f}) over those full-density maps"
                      if full_photons is not None and n_s == n_global_full else
                      f"kd-built {n_s} photons (scaled N log N to {n_global_full}), rendered {rows} of "
                      f"{args.height} rows at {args.width} px (scaled x{args.height / rows:.1f}) over maps of the "
                      f"traced sample ({n_global_full / n_s:.1f}x sparser than the frame's)")
                   + f"; wall {time.time() - t0:.1f}s"),
        "ms_per_frame": total * 1e3,
        "phase_s": {"trace": t_trace, "build": t_build, "render": t_render},
    }


def source_digest():
    """sha256 over the library's sources (photon-mapping_amd/csrc, its Makefile,
    include/pm.h) and the compile flags it was built with (build_flags.txt,
    written by the Makefile beside the library in use: PM_HIP_LIB or lib/):
    the identity of the code a PMC profile was collected on. The built .so is
    not bit-reproducible across rebuilds (hipcc embeds per-build ids in the
    code objects), so a rebuild of the same sources must not drop
    roofline.traffic; an edited kernel, or a variant library built from the
    same sources with other -D flags (make check / budget, tools/
    build_variant.sh), changes this digest and does."""
    import hashlib
    h = hashlib.sha256()
    pkg = os.path.join(ROOT, "photon-mapping_amd")
    lib = os.environ.get("PM_HIP_LIB") or os.path.join(pkg, "lib", "libpm_hip.so")
    flags = os.path.join(os.path.dirname(os.path.abspath(lib)), "build_flags.txt")
    if os.path.exists(flags):
        with open(flags, "rb") as fh:
            h.update(b"flags:" + b" ".join(fh.read().split()))
    else:
        h.update(b"flags:unknown")
    files = [os.path.join(pkg, "Makefile"), os.path.join(ROOT, "include", "pm.h")]
    for d, _, fs in os.walk(os.path.join(pkg, "csrc")):
        files += [os.path.join(d, f) for f in fs if f.endswith((".hip", ".hpp", ".cpp", ".h"))]
    for f in sorted(files):
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def secondary_config2(args):
    """The Cornell-box line (config 2, north_star's second workload) measured in a
    child process (its own device buffers and scene; this process's stay
    allocated), so the default bench line carries both configurations. The
    child is a plain `bench.py --config 2` run: same clock, same contract."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--config", "2", "--steps", str(max(10, args.steps)),
           "--warmup", str(max(3, args.warmup)), "--no-cpu-baseline", "--no-secondary"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not line:
            return {"error": f"exit {r.returncode}: {r.stderr.strip()[-400:]}"}
        d = json.loads(line[-1])
    except Exception as e:   # reported, never fatal to the main line
        return {"error": repr(e)}
    keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_frame", "config", "phases_ms", "photon_maps",
            "render")
    res = {k: d[k] for k in keep if k in d}
    res["roofline_frac"] = d.get("roofline", {}).get("frac")
    res["command"] = " ".join(["python", "bench.py"] + cmd[2:])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 5],
                    help="3: Sponza-class, 10M + 1M photons per GPU (the headline line); 2: Cornell box "
                         "(the reference's cornell-box.glb), 1M + 1M photons, 512x512; 5: caustics pass, "
                         "square area light + glass, 6.25M caustic photons per GPU (50M at 8), k = 200")
    ap.add_argument("--casted", type=int, default=None, help="diffuse photons per GPU (config 2: 1M, 3/5: 10M)")
    ap.add_argument("--caustic", type=int, default=None,
                    help="caustic photons per GPU (config 2: 1M, 3: 1M, 5: 6.25M)")
    ap.add_argument("--caustic-k", type=int, default=None, help="caustic gather neighbours (config 3: 50, 5: 200)")
    ap.add_argument("--max-depth", type=int, default=10)
    ap.add_argument("--width", type=int, default=None, help="config 2: 512, 3/5: 1920")
    ap.add_argument("--height", type=int, default=None, help="config 2: 512, 3/5: 1080")
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--depth", type=int, default=30)
    ap.add_argument("--scene", default=None, choices=["sponza", "cornell"],
                    help="config 2: cornell, 3/5: sponza")
    ap.add_argument("--frame-opt", action="append", default=[], metavar="FIELD=0|1",
                    help="override a boolean pm_amd.dist.FrameConfig field (A/B runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="config 3 at N=1 also measures config 2 (the reference's Cornell box) in a child "
                         "process and reports it under 'secondary'; this turns that off")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: every CPU this process may use, see host_cores)")
    ap.add_argument("--cpu-sample-photons", type=int, default=2_000_000)
    ap.add_argument("--cpu-sample-rows", type=int, default=48)
    ap.add_argument("--cpu-sample-maps", action="store_true",
                    help="CPU baseline maps from its traced sample (sparser) instead of the frame's photons")
    args = ap.parse_args()
    c2 = args.config == 2
    if args.scene is None:
        args.scene = "cornell" if c2 else "sponza"
    if args.casted is None:
        args.casted = 1_000_000 if c2 else 10_000_000
    if args.width is None:
        args.width = 512 if c2 else 1920
    if args.height is None:
        args.height = 512 if c2 else 1080
    if args.caustic is None:
        args.caustic = 6_250_000 if args.config == 5 else 1_000_000
    if args.caustic_k is None:
        args.caustic_k = 200 if args.config == 5 else 50

    import torch
    import pm_amd
    from pm_amd import dist as pmdist
    from pm_amd import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus or (world == 1 and args.gpus == 1), f"--gpus {args.gpus} but WORLD_SIZE={world}"
    # PM_DIST_BACKEND=gloo: every rank on cuda:0 with host-staged collectives, to
    # exercise the N > 1 path on a one-GPU box (the scaling runs use RCCL)
    backend_name = os.environ.get("PM_DIST_BACKEND", "nccl")
    torch.cuda.set_device(0 if backend_name == "gloo" else local_rank)
    dist = None
    sel_group = None
    if world > 1:
        import torch.distributed as tdist
        if backend_name == "gloo":
            tdist.init_process_group("gloo")
            dist = pmdist.HostStagedDist(tdist)
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            dist = tdist
            # the distributed top selection's own communicator, made (and its
            # first collective run) here, before any frame: its all-reduces run
            # beside the photon all-gather of the default group
            sel_group = tdist.new_group()
            warm = torch.zeros(1, dtype=torch.int64, device="cuda")
            tdist.all_reduce(warm, group=sel_group)
            torch.cuda.synchronize()

    if args.scene == "sponza" and args.config == 5:
        meshes, lights = scenes.sponza_caustics()
        scene_name = "sponza-class procedural, square area light + glass spheres (pm_amd.scenes.sponza_caustics)"
    elif args.scene == "sponza":
        obj = os.environ.get("PM_SPONZA_OBJ")
        if obj and os.path.exists(obj):
            meshes, lights = pm_amd.load_scene_file(obj)
            scene_name = f"sponza.obj ({obj})"
        else:
            meshes, lights = scenes.sponza_class()
            scene_name = "sponza-class procedural (pm_amd.scenes)"
    else:
        meshes, lights = pm_amd.load_scene_file(os.path.join(ROOT, "tests", "golden", "scenes", "cornell-box",
                                                             "cornell-box.glb"))
        scene_name = "cornell-box.glb"
    ntri = sum(len(m.indices) for m in meshes)
    casted_total = args.casted * world       # weak scaling: photons per GPU fixed
    caustic_total = args.caustic * world
    scene = pm_amd.Scene(meshes)
    emitted_diffuse = sum(pm_amd.compute_photons_per_watt(lights, casted_total))
    emitted = emitted_diffuse + sum(pm_amd.compute_photons_per_watt(lights, caustic_total))
    cap_g = pm_amd.trace_capacity(lights, casted_total, args.max_depth, False, rank, world)
    cap_c = pm_amd.trace_capacity(lights, caustic_total, args.max_depth, True, rank, world)
    gbuf = torch.empty((max(1, cap_g), 10), dtype=torch.float32, device="cuda")
    cbuf = torch.empty((max(1, cap_c), 10), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((args.height, args.width), dtype=torch.int32, device="cuda")
    info = {}
    cfg = pmdist.FrameConfig(casted=casted_total, caustic=caustic_total, max_depth=args.max_depth,
                             width=args.width, height=args.height, spp=args.spp, depth=args.depth, sky=SKY,
                             camera=CAMERA, caustic_k=args.caustic_k)
    for opt in args.frame_opt:
        field, _, v = opt.partition("=")
        if not isinstance(getattr(cfg, field, None), bool) or v not in ("0", "1"):
            raise SystemExit(f"--frame-opt: {opt!r} is not FIELD=0|1 for a boolean FrameConfig field")
        setattr(cfg, field, v == "1")
    backend = pmdist.GpuBackend(scene, lights, cfg, rank, world, gbuf=gbuf, cbuf=cbuf, sel_group=sel_group)

    def step():
        _, fi = pmdist.frame(backend, rank, world, dist, rgba)
        info.update(n_global=fi["n_global"], n_caustic=fi["n_caustic"], stats=pm_amd.render_stats(), us=fi["us"])

    for _ in range(args.warmup):
        step()
        rgba.zero_()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gather_us = []
    for _ in range(args.steps):
        step()
        gather_us.append(info["us"]["gather_global"])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = emitted * args.steps / elapsed / 1e6
    st = info["stats"]
    us = info["us"]
    nq_g = int(st.global_queries)
    t_g = sum(gather_us) / len(gather_us) * 1e-6
    bpq = knn_query_bytes(info["n_global"], 50)
    achieved = bpq * nq_g / t_g / 1e9 if t_g > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_gather_global.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            import hashlib
            with open(pm_amd.LIB_PATH, "rb") as f:
                lib_sha = hashlib.sha256(f.read()).hexdigest()
            # only while the library is the one the counters were collected on
            # (the same binary, or a build of the same sources)
            if pmc.get("workload") == [args.scene, args.casted, args.caustic, args.width, args.height, args.spp] \
                    and (pmc.get("lib_sha256") == lib_sha or pmc.get("src_sha256") == source_digest()):
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    queries = int(st.global_queries + st.caustic_queries)
    out = {
        "metric": "Mphotons/s traced + kNN gathers/s; ms/frame Sponza 10M photons",
        "value": round(value, 4),
        "unit": "Mphotons/s",
        # the diffuse (global) photons alone, the ">= 100 Mphotons/s" reading
        "value_diffuse_only": round(emitted_diffuse * args.steps / elapsed / 1e6, 4),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (procedural Sponza-class scene; photons from the reference's own emission model)",
        "config": {"workload": f"config{args.config}: {scene_name}, {casted_total} diffuse + {caustic_total} "
                               f"caustic photons, {args.width}x{args.height} spp {args.spp}, depth {args.depth}, "
                               f"k 50 (caustic gather k {args.caustic_k})",
                   "triangles": ntri, "parallelism": f"photon-shard{world}+tile{world}" if world > 1 else "1 GPU"},
        "ms_per_frame": round(ms_per_step, 3),
        # SURVEY §8d metric (i): both photon sets over the trace WINDOW, the one
        # trace launch's start to the last compaction's end (events on its stream)
        "mphotons_traced_per_s": round(emitted / (us["trace"] * 1e-6) / 1e6, 3) if us["trace"] else None,
        "knn_gathers_per_s": round(queries / (us["gather"] * 1e-6), 1) if us["gather"] else None,
        "phases_ms": {k: round(v / 1e3, 3) for k, v in us.items()},
        "photon_maps": {"global": info["n_global"], "caustic": info["n_caustic"]},
        "render": {"path_vertices": int(st.path_vertices), "caustic_queries": int(st.caustic_queries),
                   "global_queries": nq_g, "rays": int(st.rays)},
        "roofline": {"bound": "hbm", "kernel": ("pmd::k_gather_level<1, LEADERS> (global-map kNN radiance estimate: one phase, a "
                                "leader launch + a follower launch; time = both, HIP events on the launch stream)"),
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "bytes_per_query": bpq, "queries_per_launch": nq_g,
                     "avg_launch_ms": round(t_g * 1e3, 3)},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.config == 3 and not args.no_secondary:
        out["secondary"] = {"config2": secondary_config2(args)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the frame's photons (traced again after the timed region, on the GPU)
        # for the baseline's maps: its render leg walks maps of the frame's density
        full = None
        if not args.cpu_sample_maps:
            gp = pm_amd.run_point_light_ray_gen(scene, lights, casted_total, args.max_depth, False, out=gbuf)
            cp = pm_amd.run_point_light_ray_gen(scene, lights, caustic_total, args.max_depth, True, out=cbuf)
            full = (gp.cpu().numpy(), cp.cpu().numpy())
        out["cpu_baseline"] = cpu_baseline(meshes, lights, args, info["n_global"],
                                           args.cpu_threads or host_cores()[0], full_photons=full)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
