"""Multi-GPU frame driver: one process per GPU, torch.distributed
over RCCL ("nccl" backend) on MI355X, gloo on CPU for tests.

  1. trace      rank r traces global photon indices [r*P/G, (r+1)*P/G) of every
                mode; seeds are the per-light launch ids, so the union is
                bit-identical to the 1-GPU trace (pm_trace_params.shard_*).
  2. exchange   ONE all-gather per photon buffer (counts first, then the padded
                buffers) of position + colour (24 of 40 B; nothing else reaches
                a map); rank-order concatenation reproduces the 1-GPU array.
  3. build      the global map's tree is split across ranks (KdShardPlan): every
                rank selects the top ceil(log2 G) + 1 levels, the subtrees below
                are dealt to ranks balanced by size (shard_owners), ONE
                all-gather of the built subtrees (4-B node tags: positions come
                from the photons already exchanged), every rank
                places them (the same tree bit for bit; the replicated build
                cost N log N of the G-times-larger map: 311 ms at 8 GPUs vs 35 ms).
                The small caustic map is built on every rank.
  4. render     16x16 image tiles dealt round robin (tile % G == r).
  5. assemble   tiles are disjoint, so an integer SUM-reduce to rank 0 merges
                the RGBA8 image exactly.
The compute backend is pluggable: `GpuBackend` (libpm_hip.so) in production;
tests plug the CPU oracle in to check the orchestration with gloo.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field


@dataclass
class FrameConfig:
    casted: int
    caustic: int
    max_depth: int = 10
    width: int = 64
    height: int = 48
    spp: int = 1
    depth: int = 30
    sky: tuple = (1.0, 1.0, 1.0)
    camera: dict = field(default_factory=lambda: dict(look_from=(80.0, 30.0, 0.0), look_at=(10.0, 20.0, 0.0),
                                                       look_up=(0.0, 1.0, 0.0), fovy=0.87))
    # apply the %.6f photon-file round trip in memory (pm_photons_quantize), so
    # the frame equals the reference's two-process pipeline
    quantize: bool = False
    # split the global map's kd-tree build across ranks (N > 1; identical tree)
    shard_build: bool = True
    # neighbours of the caustic gather (0: the reference's 50; config 5: 200)
    caustic_k: int = 0
    # run pm_render_begin (map-independent: camera paths, shadow and final-gather
    # rays, direct light, sorted queries) on a side stream from a second host
    # thread while the photons are traced and the maps built; it fills the
    # kd build's small, under-filled launches (config 3: ~0.6 ms per frame)
    overlap_render: bool = True
    # N > 1: select the sharded build's top levels from each rank's own photons
    # (pm_kd_top_sel, all-reduced passes) while the photon all-gather runs,
    # instead of from all gathered photons on every rank
    dist_top: bool = True
    # one rank: run the caustic gather on the render side thread right after
    # the caustic map (pm_render_gather_caustic), i.e. beside the global map's
    # kd build, instead of beside the global gather in finish
    early_caustic_gather: bool = False
    # the render side thread traces the caustic photons (one rank: and builds
    # their map) beside the global trace, then holds pm_render_begin until the
    # global trace is done, so the render's ray kernels run beside the exchange
    # and the kd build instead of beside the trace. Default since the fused
    # photon-path kernel (csrc/trace.hip, PM_TRACE_FUSED), which holds every wave
    # slot it can get for the whole trace: the render begin beside it stretched
    # to 33 ms (config 3: 93.8-94.3 vs 98.4-99.0 ms per frame; the wavefront
    # trace with the render begin beside it: 96.3-96.6 ms)
    begin_after_trace: bool = True
    # one rank: the caustic photons are traced, and their map built, on the main
    # thread right after the global trace (the side thread runs pm_render_begin
    # only): for a global trace short enough that the caustic work would
    # otherwise wait behind the render begin
    caustic_after_trace: bool = False
    # both photon sets in ONE persistent trace launch (pm_trace_photon_sets,
    # backends with trace_both): the caustic photons fill the diffuse paths'
    # tail instead of queueing behind the launch on a second stream, and the
    # trace phase is one stream's window (launch through the last compaction).
    # One rank: the side thread builds the caustic map after the trace, then
    # runs pm_render_begin, both beside the global map's kd build
    one_trace: bool = True


def shard_range(total: int, rank: int, world: int):
    return total * rank // world, total * (rank + 1) // world


class _Gathered:
    """An all-gather in flight (allgather_rows_start); wait() returns the rows
    concatenated in rank order (a copy), rows() the padded buffer itself as
    PhotonRows (device tensors: no copy; rank r at rows [r m, r m + n_r))."""

    def __init__(self, work, out, ns, m, world, parts=None):
        self.work, self.out, self.ns, self.m, self.world, self.parts = work, out, ns, m, world, parts

    def _done(self):
        if self.work is not None:
            self.work.wait()
            self.work = None

    def wait(self):
        import torch
        self._done()
        if self.parts is None:
            self.parts = [self.out[r * self.m: r * self.m + self.ns[r]] for r in range(self.world)]
        return torch.cat(self.parts)

    def rows(self):
        from pm_amd import PhotonRows
        self._done()
        return PhotonRows.of_padded(self.out, self.ns, self.m, color_offset=3)


def allgather_rows_start(t, world: int, dist, pack=None):
    """Variable-length all-gather of an (n_r, C) tensor: the counts are exchanged
    first (the host sizes the padded buffer), then ONE padded all-gather is
    started asynchronously on device tensors (RCCL runs it on its own stream, so
    the caller can overlap work on the current stream until wait()).
    pack(t, out): writes t's C-column rows into `out` (the padded buffer's first
    n_r rows) instead of a copy of t itself (pm_photon -> position + colour in
    one pass)."""
    import torch
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(1, max(ns))
    cols = t.shape[1] if pack is None else PACKED_COLS
    pad = torch.empty((m, cols), dtype=t.dtype, device=t.device)
    pad[t.shape[0]:].zero_()
    if pack is None:
        pad[: t.shape[0]] = t
    else:
        pack(t, pad[: t.shape[0]])
    if t.device.type == "cuda":
        out = torch.empty((world * m, cols), dtype=t.dtype, device=t.device)
        work = dist.all_gather_into_tensor(out, pad, async_op=True)
        return _Gathered(work, out, ns, m, world)
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    return _Gathered(None, None, ns, m, world, parts=[bufs[r][: ns[r]] for r in range(world)])


def allgather_rows(t, world: int, dist):
    """Variable-length all-gather of an (n_r, C) tensor, concatenated in rank order."""
    return allgather_rows_start(t, world, dist).wait()


class _PhaseClock:
    """Elapsed time of a phase: HIP events on the current stream for device work
    (collectives included: a finished RCCL call makes the current stream wait
    for it), wall clock for host tensors."""

    def __init__(self, cuda: bool):
        import torch
        self.cuda = cuda
        if cuda:
            self.a = torch.cuda.Event(enable_timing=True)
            self.b = torch.cuda.Event(enable_timing=True)
            self.a.record()
        else:
            self.t0 = time.perf_counter()

    def stop_us(self) -> float:
        if not self.cuda:
            return (time.perf_counter() - self.t0) * 1e6
        self.b.record()
        self.b.synchronize()
        return self.a.elapsed_time(self.b) * 1e3


class _HostStagedWork:
    """A host-staged collective in flight: wait() waits for gloo, then copies
    the host result into the caller's (device) tensor, once."""

    def __init__(self, work, host, out):
        self.work, self.host, self.out = work, host, out

    def is_completed(self) -> bool:
        return self.work is None or self.work.is_completed()

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.out.copy_(self.host)
            self.work = self.host = None
        return True


class HostStagedDist:
    """torch.distributed over gloo with CUDA tensors staged through host memory:
    lets several ranks share one GPU (tests, and `bench.py` with
    PM_DIST_BACKEND=gloo on a one-GPU box); production runs use RCCL directly."""

    def __init__(self, dist):
        import torch
        self.d, self.t = dist, torch
        self.ReduceOp = dist.ReduceOp

    def all_gather(self, outs, t):
        hs = [self.t.empty_like(o, device="cpu") for o in outs]
        self.d.all_gather(hs, t.cpu())
        for o, h in zip(outs, hs):
            o.copy_(h)

    def all_gather_into_tensor(self, out, t, async_op=False):
        """async_op: gloo runs the all-gather on its worker thread and the
        returned handle's wait() finishes it (then stages the result into
        `out`), so the caller's work between start and wait overlaps it, as
        with RCCL's stream (dist._maps: the caustic map and the distributed top
        selection's all-reduces run while the global photons are in flight)."""
        h = self.t.empty_like(out, device="cpu")
        pending = _HostStagedWork(self.d.all_gather_into_tensor(h, t.cpu(), async_op=True), h, out)
        if async_op:
            return pending
        pending.wait()
        return None

    def reduce(self, t, dst, op):
        h = t.cpu()
        self.d.reduce(h, dst=dst, op=op)
        if self.d.get_rank() == dst:   # only the root's buffer receives the result
            t.copy_(h)

    def all_reduce(self, t, op):
        h = t.cpu()
        self.d.all_reduce(h, op=op)
        t.copy_(h)

    def barrier(self):
        self.d.barrier()

    def destroy_process_group(self):
        self.d.destroy_process_group()


PACKED_COLS = 6   # position + colour: what a map reads of a photon


def pack_rows(t, out=None):
    """pm_photon rows (n, 10) -> (n, 6): position, colour (into `out` if given)."""
    import torch
    if out is None:
        return torch.cat([t[:, 0:3], t[:, 7:10]], dim=1).contiguous()
    torch.cat([t[:, 0:3], t[:, 7:10]], dim=1, out=out)
    return out


def unpack_rows(p):
    """(n, 6) -> pm_photon rows with direction and power zero (never read by a map)."""
    import torch
    t = torch.zeros((p.shape[0], 10), dtype=p.dtype, device=p.device)
    t[:, 0:3] = p[:, 0:3]
    t[:, 7:10] = p[:, 3:6]
    return t


def shard_owners(sizes, world: int):
    """Subtree -> rank, balanced by size (largest first to the least-loaded rank,
    ties to the lower index): deterministic, the same on every rank."""
    load, owner = [0] * world, [0] * len(sizes)
    for j in sorted(range(len(sizes)), key=lambda j: (-sizes[j], j)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[j] = r
        load[r] += sizes[j]
    return owner, load


def shard_local(plan, rank: int, world: int):
    """Rank `rank`'s subtrees (shard_owners) built back to back, in subtree order,
    into one (m_max,) int32 tag buffer, m_max = the largest rank's total
    (all-gather padding); returns (buffer, kd-build us)."""
    import torch
    pm = _pm()
    owner, load = shard_owners(plan.sizes, world)
    local = torch.empty((max(1, max(load)),), dtype=torch.int32, device="cuda")
    off, us = 0, 0.0
    for j, sz in enumerate(plan.sizes):
        if owner[j] == rank:
            plan.build(j, out=local[off: off + sz])
            us += pm.phase_us("kdbuild")
            off += sz
    return local, us


def shard_assemble(plan, everyone, world: int):
    """The map from the all-gathered tag buffers ((world * m_max,), rank order)."""
    import torch
    owner, _ = shard_owners(plan.sizes, world)
    m_max = everyone.shape[0] // world
    parts, offs = [], [0] * world
    for j, sz in enumerate(plan.sizes):
        r = owner[j]
        parts.append(everyone[r * m_max + offs[r]: r * m_max + offs[r] + sz])
        offs[r] += sz
    return plan.map(torch.cat(parts))


def top_selection(pm, g_local, c_local, g_ns, c_ns, rank: int, world: int, dist, group=None):
    """The global tree's top levels from this rank's OWN photons (pm_kd_top_sel):
    every pass reads 1/G of the elements and its small output is all-reduced
    (SUM / MIN), so it needs no exchanged photon and runs while the photon
    all-gather is in flight (on `group`, a communicator of its own, so that
    RCCL does not queue these small reductions behind the all-gather).
    g_ns / c_ns: every rank's photon counts (the exchange's). Returns
    (selection, us)."""
    ops = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN}
    g_first = sum(g_ns[:rank])
    c_first = sum(g_ns) + sum(c_ns[:rank])
    n_total = sum(g_ns) + sum(c_ns)
    clock = _PhaseClock(g_local.device.type == "cuda")
    sel = pm.KdTopSel(g_local, g_first, c_local, c_first, n_total, world)

    def reduce(buf, op):
        if group is not None:
            dist.all_reduce(buf, op=ops[op], group=group)
        else:
            dist.all_reduce(buf, op=ops[op])
    sel.run(reduce)
    return sel, clock.stop_us()


def simulated_top_selection(pm, g, c, world: int):
    """top_selection of `world` ranks run in one process on one GPU (tests,
    tools/kd_scale_probe.py): rank r holds shard_range(r) of g and of c, the
    passes run rank after rank and the reductions are done here. Returns
    (rank 0's selection, [us of each rank's passes])."""
    import torch
    ng, nc = g.shape[0], c.shape[0]
    g_ns = [shard_range(ng, r, world)[1] - shard_range(ng, r, world)[0] for r in range(world)]
    c_ns = [shard_range(nc, r, world)[1] - shard_range(nc, r, world)[0] for r in range(world)]
    sels, us = [], [0.0] * world
    for r in range(world):
        g0, g1 = shard_range(ng, r, world)
        c0, c1 = shard_range(nc, r, world)
        t0 = time.perf_counter()
        sels.append(pm.KdTopSel(g[g0:g1], g0, c[c0:c1], ng + c0, ng + nc, world))
        torch.cuda.synchronize()
        us[r] += (time.perf_counter() - t0) * 1e6
    while True:
        outs = []
        for r, s in enumerate(sels):
            t0 = time.perf_counter()
            outs.append(s.step())
            us[r] += (time.perf_counter() - t0) * 1e6
        cnt, op = outs[0]
        assert all(o == outs[0] for o in outs), outs   # every rank runs the same passes
        if op is None:
            break
        stack = torch.stack([s.buf[:cnt] for s in sels])
        red = stack.sum(0) if op == "sum" else stack.min(0).values
        for s in sels:
            s.buf[:cnt].copy_(red)
    for s in sels[1:]:
        s.close()
    return sels[0], us


def sharded_map(pm, g, c, rank: int, world: int, dist, sel=None):
    """Global map (diffuse ++ caustic) built across ranks; returns (map, kd-build us
    of this rank, the subtree all-gather included). sel: the finished
    top_selection (else every rank selects the top levels from all photons)."""
    import torch
    plan = pm.KdShardPlan(g, pm.PHOTON_POWER, c, pm.CAUSTICS_PHOTON_POWER, world=world, sel=sel)
    us = pm.phase_us("kdbuild")
    if not plan.sizes:   # too small to split: every rank builds the whole tree
        m = plan.map()
        return m, us + pm.phase_us("kdbuild")
    local, bus = shard_local(plan, rank, world)
    clock = _PhaseClock(local.device.type == "cuda")
    everyone = torch.empty((world * local.shape[0],), dtype=torch.int32, device=local.device)
    dist.all_gather_into_tensor(everyone, local)
    xus = clock.stop_us()
    m = shard_assemble(plan, everyone, world)
    us += bus + xus + pm.phase_us("kdbuild")
    plan.close()
    return m, us


def _pm():
    import pm_amd
    return pm_amd


class GpuBackend:
    """libpm_hip.so through pm_amd (device tensors on the current cuda device)."""

    def __init__(self, scene, lights, cfg: FrameConfig, rank: int, world: int, gbuf=None, cbuf=None,
                 sel_group=None):
        """sel_group: the communicator of the distributed top selection's small
        all-reduces (N > 1, cfg.dist_top). Create it right after
        init_process_group (`dist.new_group()`), outside any frame: created
        lazily, its RCCL communicator would be set up while the photon
        all-gather is in flight on the default group."""
        import pm_amd
        self.pm = pm_amd
        self.scene, self.lights, self.cfg = scene, lights, cfg
        self.gbuf, self.cbuf = gbuf, cbuf
        self._sel_group = sel_group
        self.cam = pm_amd.setup_camera(cfg.camera["look_from"], cfg.camera["look_at"], cfg.camera["look_up"],
                                       cfg.camera["fovy"], cfg.width, cfg.height)
        self.phase = {}

    def trace_both(self, rank: int, world: int):
        """(diffuse, caustic) photons of this shard in one launch; phase
        "trace" = the trace window (the launch through the last compaction)."""
        pm = self.pm
        g, c = pm.run_photon_sets(self.scene, self.lights, self.cfg.casted, self.cfg.caustic, self.cfg.max_depth,
                                  shard_rank=rank, shard_count=world, out=(self.gbuf, self.cbuf))
        self.phase["trace"] = self.phase.get("trace", 0.0) + pm.phase_us("trace")
        return g, c

    def trace(self, caustics: bool, rank: int, world: int):
        pm = self.pm
        casted = self.cfg.caustic if caustics else self.cfg.casted
        out = self.cbuf if caustics else self.gbuf
        t = pm.run_point_light_ray_gen(self.scene, self.lights, casted, self.cfg.max_depth, caustics,
                                       shard_rank=rank, shard_count=world, out=out)
        self.phase["trace"] = self.phase.get("trace", 0.0) + pm.phase_us("trace") + pm.phase_us("compact")
        return t

    def quantize(self, t):
        return self.pm.quantize_photons(t)

    def caustic_map(self, c):
        pm = self.pm
        cm = pm.PhotonMap(c, pm.CAUSTICS_PHOTON_POWER)
        self.phase["kdbuild"] = self.phase.get("kdbuild", 0.0) + pm.phase_us("kdbuild")
        return cm

    def top_selection(self, g_local, c_local, g_ns, c_ns, rank: int, world: int, dist):
        """The distributed top selection (None: not split across ranks)."""
        if world < 2 or not self.cfg.shard_build or not self.cfg.dist_top:
            return None
        group = getattr(self, "_sel_group", None)
        if group is None and hasattr(dist, "new_group") and not isinstance(dist, HostStagedDist):
            group = self._sel_group = dist.new_group()
        sel, us = top_selection(self.pm, g_local, c_local, g_ns, c_ns, rank, world, dist, group)
        self.phase["kdbuild"] = self.phase.get("kdbuild", 0.0) + us
        return sel

    def global_map(self, g, c, rank: int = 0, world: int = 1, dist=None, sel=None):
        pm = self.pm
        if world > 1 and self.cfg.shard_build:
            gm, kd = sharded_map(pm, g, c, rank, world, dist, sel=sel)
        else:
            gm = pm.PhotonMap(g, pm.PHOTON_POWER, c, pm.CAUSTICS_PHOTON_POWER)
            kd = pm.phase_us("kdbuild")
        self.phase["kdbuild"] = self.phase.get("kdbuild", 0.0) + kd
        return gm

    def start_render(self, tile_rank: int, tile_count: int, caustic_shard=None, caustic_map: bool = False,
                     caustic_from_main: bool = False):
        """pm_render_begin on a side stream from a second host thread; returns a
        handle for finish_render. The begin half synchronises its stream before
        it returns, so the job is complete once the thread has ended. With
        caustic_shard=(rank, world) the same thread then traces the caustic
        photons on that stream (take them with caustic_photons): its short,
        latency-bound bounce launches fill the GPU beside the global trace's
        tail instead of running after it. With caustic_map as well (one rank,
        no quantisation: the map is then built from these photons alone) it
        also builds the caustic map there (take it with caustic_map_of). The
        caustic gather stays in finish_render, on a side stream beside the
        global gather's leader launch: run here (pm_render_gather_caustic) it
        landed beside the kd build (config 3: kd 25.3 -> 28 ms, frame
        unchanged) and, on the Cornell box, held the global gather back.
        caustic_from_main (FrameConfig.one_trace): the main thread traces both
        sets and hands the caustic photons over with trace_done(pending, c);
        with caustic_map the thread then builds their map on its stream. With
        cfg.begin_after_trace, pm_render_begin always waits for trace_done."""
        import threading
        import torch
        pm, c = self.pm, self.cfg
        if getattr(self, "_rside", None) is None:
            self._rside = torch.cuda.Stream()
        side, box = self._rside, {"c_ready": threading.Event(), "trace_done": threading.Event()}
        device = side.device   # this rank's GPU (the caller's current device)

        def run():
            try:
                # HIP's and torch's current device are per host thread, and a new
                # thread starts on device 0: without this, rank r's side thread
                # would allocate its tensors (torch.empty(device="cuda")) on GPU 0
                # (the library itself follows the stream's device, include/pm.h)
                torch.cuda.set_device(device)
                def begin():
                    j = pm.render_begin(self.scene, self.cam, c.width, c.height, c.spp, c.depth, c.sky, self.lights,
                                        tile_rank=tile_rank, tile_count=tile_count, stream=side.cuda_stream,
                                        caustic_k=c.caustic_k)
                    box["r"] = (j, pm.phase_us("paths"))   # phase timers are per host thread
                    return j

                late = c.begin_after_trace
                if not late:
                    job = begin()
                if caustic_from_main:
                    box["trace_done"].wait()
                    if caustic_map and "c_in" in box:
                        cm = pm.PhotonMap(box["c_in"], pm.CAUSTICS_PHOTON_POWER, stream=side.cuda_stream)
                        box["cm"] = (cm, pm.phase_us("kdbuild"))
                    if late:
                        job = begin()
                elif caustic_shard is not None:
                    t = pm.run_point_light_ray_gen(self.scene, self.lights, c.caustic, c.max_depth, True,
                                                   shard_rank=caustic_shard[0], shard_count=caustic_shard[1],
                                                   out=self.cbuf, stream=side.cuda_stream)
                    box["c"] = (t, pm.phase_us("trace") + pm.phase_us("compact"))
                    box["c_ready"].set()   # the main thread goes on; the map and gather follow here
                    if caustic_map:
                        cm = pm.PhotonMap(t, pm.CAUSTICS_PHOTON_POWER, stream=side.cuda_stream)
                        box["cm"] = (cm, pm.phase_us("kdbuild"))
                    if late:
                        box["trace_done"].wait()
                        job = begin()
                    if caustic_map and c.early_caustic_gather:
                        job.gather_caustic(cm, stream=side.cuda_stream)
                elif late:
                    box["trace_done"].wait()
                    job = begin()
            except BaseException as e:   # re-raised by finish_render / join_render
                box["e"] = e
            finally:
                box["c_ready"].set()

        th = threading.Thread(target=run, name="pm-render-begin")
        th.start()
        return th, box

    def caustic_photons(self, pending):
        """The caustic photons traced by start_render(caustic_shard=...)'s thread
        (complete: the thread synchronised its stream before signalling). Does
        not wait for the thread's caustic map and gather."""
        box = pending[1]
        box["c_ready"].wait()
        if "c" not in box:
            self.join_render(pending)   # re-raises the thread's error
        t, us = box["c"]
        self.phase["trace"] = self.phase.get("trace", 0.0) + us
        return t

    def caustic_map_of(self, pending):
        """The caustic map start_render(caustic_map=True)'s thread built (waits
        for the thread)."""
        self.join_render(pending)
        cm, kd_us = pending[1]["cm"]
        self.phase["kdbuild"] = self.phase.get("kdbuild", 0.0) + kd_us
        return cm

    @staticmethod
    def trace_done(pending, caustic=None):
        """The global trace is over (begin_after_trace's thread may go on);
        caustic: the caustic photons, for start_render(caustic_from_main=True)."""
        if caustic is not None:
            pending[1]["c_in"] = caustic
        pending[1]["trace_done"].set()

    @staticmethod
    def join_render(pending):
        th, box = pending
        box["trace_done"].set()   # never leave the thread waiting
        th.join()
        if "e" in box:
            raise box["e"]
        return box["r"]

    def finish_render(self, pending, gm, cm, rgba):
        job, paths_us = self.join_render(pending)
        try:
            job.finish(gm, cm, want_rgb=False, rgba=rgba)
        finally:
            job.close()
        self.phase["paths"] = paths_us
        for k in ("gather", "gather_global", "resolve"):
            self.phase[k] = self.pm.phase_us(k)
        return rgba

    def render(self, gm, cm, tile_rank: int, tile_count: int, rgba):
        pm = self.pm
        c = self.cfg
        pm.render(self.scene, self.cam, c.width, c.height, c.spp, c.depth, c.sky, self.lights, gm, cm,
                  tile_rank=tile_rank, tile_count=tile_count, want_rgb=False, rgba=rgba, caustic_k=c.caustic_k)
        for k in ("paths", "gather", "gather_global", "resolve"):
            self.phase[k] = pm.phase_us(k)
        return rgba


def frame(backend, rank: int, world: int, dist=None, rgba=None):
    """One frame through `backend`; returns (rgba on rank 0 (merged), info).
    With cfg.overlap_render (backends that have start_render), the render's
    map-independent half runs on a side stream beside the trace and the map
    builds; the phases then add up to more than the frame. N > 1: the caustic
    photons are exchanged first (small), then the global photons' all-gather
    runs on RCCL's stream while the caustic map is built; phases_us["exchange"]
    is that window (HIP events), caustic build included."""
    backend.phase = {}
    pending = None
    one = getattr(backend.cfg, "one_trace", False) and hasattr(backend, "trace_both")
    early_caustic = side_caustic = False
    if backend.cfg.overlap_render and hasattr(backend, "start_render"):
        if one:
            early_caustic = world == 1 and not backend.cfg.quantize
            pending = backend.start_render(rank, world, caustic_map=early_caustic, caustic_from_main=True)
        else:
            side_caustic = not (world == 1 and backend.cfg.caustic_after_trace)
            early_caustic = world == 1 and not backend.cfg.quantize and side_caustic
            pending = backend.start_render(rank, world, caustic_shard=(rank, world) if side_caustic else None,
                                           caustic_map=early_caustic)
    try:
        g, c, gm, cm = _maps(backend, rank, world, dist, pending, pending is not None and early_caustic,
                             side_caustic=pending is not None and side_caustic, one_trace=one)
    except BaseException:
        if pending is not None:   # no side work outlives a failed frame
            try:
                backend.join_render(pending)[0].close()
            except BaseException:
                pass
        raise
    if world > 1 and rgba is not None:
        rgba.zero_()   # tiles are disjoint: the SUM-reduce needs zeros outside this rank's tiles
    if pending is not None:
        if cm is None:
            cm = backend.caustic_map_of(pending)
        rgba = backend.finish_render(pending, gm, cm, rgba)
    else:
        rgba = backend.render(gm, cm, rank, world, rgba)
    if world > 1:
        dist.reduce(rgba, dst=0, op=dist.ReduceOp.SUM)
    info = {"n_global": int(gm.n), "n_caustic": int(cm.n), "n_global_rows": nrows(g),
            "us": dict(backend.phase)}
    return rgba, info


def _gathered_set(x):
    """A finished photon all-gather as a map input: PhotonRows over the padded
    device buffer, or (host tensors: the CPU test backends) pm_photon rows."""
    if x.out is not None and x.world <= _pm().ROWS_MAX_SEGS:
        return x.rows()
    # host tensors, or more ranks than pm_photon_rows has segments: the rows
    # concatenated and re-expanded (a copy)
    return unpack_rows(x.wait())


def nrows(x) -> int:
    """photons in a set (tensor rows or PhotonRows)"""
    return int(x.n if hasattr(x, "segments") else x.shape[0])


def _maps(backend, rank: int, world: int, dist, pending=None, early_caustic: bool = False, side_caustic=None,
          one_trace: bool = False):
    """Trace both photon sets, exchange them (N > 1), build both maps. one_trace:
    both sets in one launch (backend.trace_both); with a render pending, its
    thread is handed the caustic photons and, with early_caustic (world 1),
    builds their map (returned as None here). Otherwise, with a render pending
    from start_render(caustic_shard=...) (side_caustic), the caustic photons
    come from its thread, and with early_caustic so does the caustic map."""
    if one_trace:
        g, c = backend.trace_both(rank, world)
        if pending is not None and hasattr(backend, "trace_done"):
            backend.trace_done(pending, c)
    else:
        if side_caustic is None:
            side_caustic = pending is not None
        g = backend.trace(False, rank, world)
        if pending is not None and hasattr(backend, "trace_done"):
            backend.trace_done(pending)
        c = backend.caustic_photons(pending) if side_caustic else backend.trace(True, rank, world)
    if backend.cfg.quantize:   # elementwise: the same before or after the exchange
        g, c = backend.quantize(g), backend.quantize(c)
    sel = None
    if world > 1:
        # only position and colour reach the maps (kd nodes + gather payload):
        # 24 of the 40 bytes of a photon cross xGMI, packed straight into the
        # padded all-gather buffer; on the device the maps read that buffer as
        # it is (PhotonRows: rank r's rows at [r m, r m + n_r)), with no
        # compaction and no re-expansion to pm_photon rows
        clock = _PhaseClock(g.device.type == "cuda")
        g_local, c_local = g, c
        cx = allgather_rows_start(c_local, world, dist, pack=pack_rows)
        c = _gathered_set(cx)
        xfer = allgather_rows_start(g_local, world, dist, pack=pack_rows)
        cm = backend.caustic_map(c)   # overlaps the global photons' transfer
        if hasattr(backend, "top_selection"):   # so does the top selection (own photons only)
            sel = backend.top_selection(g_local, c_local, xfer.ns, cx.ns, rank, world, dist)
        g = _gathered_set(xfer)
        backend.phase["exchange"] = clock.stop_us()
    else:
        backend.phase["exchange"] = 0.0
        # None: start_render's thread builds it (frame() takes it before the render)
        cm = None if early_caustic else backend.caustic_map(c)
    gm = backend.global_map(g, c, rank, world, dist, sel=sel) if sel is not None else \
        backend.global_map(g, c, rank, world, dist)
    return g, c, gm, cm
