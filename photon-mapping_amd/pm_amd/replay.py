"""G ranks of the multi-GPU frame (pm_amd.dist.frame) on ONE GPU, with the
collectives replayed: the configurations that need 8 GPUs (config 4: 80 M
photons; config 5 at 8x: 50 M caustic photons, k = 200) run here rank by
rank at their full size, through the production frame path, so their
363 M-node maps, the 64-bit-addressing gather they need (maps of >= 2^28
nodes) and the sharded kd build are exercised and timed on one device.

The reference renders on one device (photon-mapping/src/hostCode.cu:145,
owlContextCreate(nullptr, 1)); the split itself is SURVEY §8e's.

Pass 1, `record()`: from the production building blocks, every rank's
contribution to each collective that `frame()` issues and the collective's
result, in call order:
  1. all_gather of the caustic photon counts, 2. the padded all-gather of the
     caustic (position, colour) rows, 3./4. the same for the global photons;
  5. the distributed top selection's all-reduces (pm_kd_top_sel_step);
  6. the all-gather of the built subtrees' node tags.
Pass 2, `ReplayDist(rec, rank)`: the torch.distributed stand-in that rank
`rank`'s `frame()` is handed. Each collective first checks that the rank's own
contribution equals the recorded one (so the rank computed exactly what pass 1
assumed), then writes the recorded result; the image SUM-reduce (7.) keeps the
rank's image for the caller to sum. The one-device copies that stand in for
the xGMI transfers are timed inside the rank's "exchange" phase; what RCCL
would take instead is the one term this cannot measure."""
from __future__ import annotations

from dataclasses import dataclass, field

from pm_amd import dist as pmdist


class _Done:
    """A finished collective (what async_op=True returns here)."""

    def wait(self):
        return True


def _same(a, b) -> bool:
    import torch
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.dtype.is_floating_point:   # bitwise: NaN rows compare equal to themselves
        return torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))
    return torch.equal(a, b)


@dataclass
class Recording:
    world: int
    ops: list = field(default_factory=list)   # (kind, payload) in frame() call order
    ns_g: list = field(default_factory=list)
    ns_c: list = field(default_factory=list)
    rows_g: object = None                     # the padded all-gather buffers as frame() receives them
    rows_c: object = None
    m_g: int = 0
    m_c: int = 0
    plan_sizes: list = field(default_factory=list)
    sharded_map: object = None                # the map assembled from all ranks' subtrees
    sel_steps: int = 0

    def gathered(self):
        """(global, caustic) photon sets as every rank holds them after the
        exchange: PhotonRows over the padded buffers."""
        from pm_amd import PhotonRows
        return (PhotonRows.of_padded(self.rows_g, self.ns_g, self.m_g, color_offset=3),
                PhotonRows.of_padded(self.rows_c, self.ns_c, self.m_c, color_offset=3))

    def exchange_bytes(self) -> int:
        """Bytes each rank receives from the others in the two photon all-gathers."""
        return (self.world - 1) * (self.m_g + self.m_c) * pmdist.PACKED_COLS * 4


def _padded(parts, world):
    import torch
    ns = [int(p.shape[0]) for p in parts]
    m = max(1, max(ns))
    out = torch.zeros((world * m, pmdist.PACKED_COLS), dtype=torch.float32, device="cuda")
    for r, p in enumerate(parts):
        pmdist.pack_rows(p, out[r * m: r * m + ns[r]])
    return out, ns, m


def record(scene, lights, cfg: "pmdist.FrameConfig", world: int, keep_map: bool = True) -> Recording:
    """Pass 1 for `world` ranks of cfg's job (photon counts are the whole job's,
    as in FrameConfig). Needs cfg.shard_build and cfg.dist_top (the N > 1
    defaults) and no quantisation."""
    import torch
    import pm_amd as pm
    assert world >= 2 and cfg.shard_build and cfg.dist_top and not cfg.quantize
    rec = Recording(world)
    # 1-4: every rank traces its photon-id shard (dist.frame: the global photons
    # on the caller's stream, the caustic ones on the render side thread's; the
    # same launch either way)
    cap = max(pm.trace_capacity(lights, cfg.casted, cfg.max_depth, False, r, world) for r in range(world))
    buf = torch.empty((max(1, cap), 10), dtype=torch.float32, device="cuda")
    gl = [pm.run_point_light_ray_gen(scene, lights, cfg.casted, cfg.max_depth, False, shard_rank=r,
                                     shard_count=world, out=buf).clone() for r in range(world)]
    cap = max(pm.trace_capacity(lights, cfg.caustic, cfg.max_depth, True, r, world) for r in range(world))
    buf = torch.empty((max(1, cap), 10), dtype=torch.float32, device="cuda")
    cl = [pm.run_point_light_ray_gen(scene, lights, cfg.caustic, cfg.max_depth, True, shard_rank=r,
                                     shard_count=world, out=buf).clone() for r in range(world)]
    del buf
    rec.rows_c, rec.ns_c, rec.m_c = _padded(cl, world)
    rec.rows_g, rec.ns_g, rec.m_g = _padded(gl, world)
    rec.ops += [("counts", rec.ns_c), ("rows", (rec.rows_c, rec.m_c)),
                ("counts", rec.ns_g), ("rows", (rec.rows_g, rec.m_g))]
    # 5: the distributed top selection, each rank over its own photons
    ns_g, ns_c = rec.ns_g, rec.ns_c
    n_total = sum(ns_g) + sum(ns_c)
    sels = [pm.KdTopSel(gl[r], sum(ns_g[:r]), cl[r], sum(ns_g) + sum(ns_c[:r]), n_total, world)
            for r in range(world)]
    while True:
        outs = [s.step() for s in sels]
        cnt, op = outs[0]
        assert all(o == outs[0] for o in outs), outs   # every rank runs the same passes
        if op is None:
            break
        ins = [s.buf[:cnt].clone() for s in sels]
        stack = torch.stack(ins)
        red = stack.sum(0) if op == "sum" else stack.min(0).values
        for s in sels:
            s.buf[:cnt].copy_(red)
        rec.ops.append(("reduce", (op, ins, red)))
    rec.sel_steps = sels[0].steps
    for s in sels[1:]:
        s.close()
    del gl, cl
    # 6: the plan from the gathered photons, every rank's subtrees, their all-gather
    g, c = rec.gathered()
    plan = pm.KdShardPlan(g, pm.PHOTON_POWER, c, pm.CAUSTICS_PHOTON_POWER, world=world, sel=sels[0])
    rec.plan_sizes = list(plan.sizes)
    if plan.sizes:
        locals_ = [pmdist.shard_local(plan, r, world)[0] for r in range(world)]
        everyone = torch.cat(locals_)
        rec.ops.append(("tags", (locals_, everyone)))
        if keep_map:
            rec.sharded_map = pmdist.shard_assemble(plan, everyone, world)
    elif keep_map:
        rec.sharded_map = plan.map()
    plan.close()
    sels[0].close()
    return rec


class ReplayDist:
    """torch.distributed stand-in for rank `rank` of a Recording (pass 2)."""

    class ReduceOp:
        SUM, MIN, MAX = "sum", "min", "max"

    def __init__(self, rec: Recording, rank: int):
        self.rec, self.rank = rec, rank
        self._i = 0
        self.image = None

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.rec.world

    def _next(self, *kinds):
        assert self._i < len(self.rec.ops), "frame() issued more collectives than recorded"
        kind, payload = self.rec.ops[self._i]
        assert kind in kinds, f"collective {self._i}: frame() issued {kinds}, recorded {kind}"
        self._i += 1
        return kind, payload

    def done(self) -> bool:
        return self._i == len(self.rec.ops) and self.image is not None

    def all_gather(self, outs, t):   # the photon counts
        _, ns = self._next("counts")
        assert int(t.item()) == ns[self.rank], (self.rank, int(t.item()), ns)
        for o, v in zip(outs, ns):
            o.fill_(v)

    def all_gather_into_tensor(self, out, t, async_op=False, group=None):
        kind, payload = self._next("rows", "tags")
        r = self.rank
        if kind == "rows":
            full, m = payload
            assert _same(t, full[r * m: (r + 1) * m]), f"rank {r}: photon rows differ from the recording"
        else:
            locals_, full = payload
            # shard_local fills the first load[r] tags of its (m_max,) buffer
            n = pmdist.shard_owners(self.rec.plan_sizes, self.rec.world)[1][r]
            assert t.shape == locals_[r].shape and _same(t[:n], locals_[r][:n]), \
                f"rank {r}: subtree tags differ from the recording"
        assert out.shape == full.shape, (out.shape, full.shape)
        out.copy_(full)
        return _Done() if async_op else None

    def all_reduce(self, t, op=None, group=None):
        _, (opname, ins, red) = self._next("reduce")
        assert op == opname, (op, opname)
        assert _same(t, ins[self.rank]), f"rank {self.rank}: top-selection pass output differs from the recording"
        t.copy_(red)

    def reduce(self, t, dst=0, op=None, group=None):
        assert op == self.ReduceOp.SUM
        self.image = t.clone()

    def barrier(self):
        pass


def rank_frame(rec: Recording, scene, lights, cfg, rank: int, gbuf=None, cbuf=None, rgba=None):
    """Rank `rank`'s production frame (pm_amd.dist.frame through GpuBackend)
    with rec's collectives replayed: returns (its image before the reduce, frame
    info, wall ms of the frame)."""
    import time
    import torch
    world = rec.world
    dist = ReplayDist(rec, rank)
    be = pmdist.GpuBackend(scene, lights, cfg, rank, world, gbuf=gbuf, cbuf=cbuf)
    if rgba is None:
        rgba = torch.zeros((cfg.height, cfg.width), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, info = pmdist.frame(be, rank, world, dist, rgba)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    assert dist.done(), f"rank {rank}: frame() issued {dist._i} of {len(rec.ops)} recorded collectives"
    return dist.image, info, ms
