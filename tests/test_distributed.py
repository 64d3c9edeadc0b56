"""N > 1 orchestration (pm_amd.dist) with world_size 2 and 3 over gloo on CPU:
photon-index sharding + one all-gather reproduces the single-process photon
arrays bit for bit, and the tile-sharded render + SUM-reduce reproduces the
single-process image exactly. The compute backend is the CPU oracle here
(test infrastructure); on the GPU box the same driver runs GpuBackend over RCCL."""
import os
import socket

import numpy as np
import pytest

import conftest

torch = pytest.importorskip("torch")


class OracleBackend:
    def __init__(self, meshes, lights, cfg):
        import oracle
        self.o = oracle
        self.scene = oracle.Scene(meshes)
        self.lights, self.cfg = lights, cfg
        self.cam = oracle.camera_setup(cfg.camera["look_from"], cfg.camera["look_at"], cfg.camera["look_up"],
                                       cfg.camera["fovy"], cfg.width, cfg.height)
        self.phase = {}

    def trace(self, caustics, rank, world):
        casted = self.cfg.caustic if caustics else self.cfg.casted
        a = self.o.trace(self.scene, self.lights, casted, self.cfg.max_depth, caustics, shard_rank=rank,
                         shard_count=world, nthreads=2)
        return torch.from_numpy(a)

    def caustic_map(self, c):
        return self.o.PhotonMap(c.numpy(), 0.5)

    def top_selection(self, g_local, c_local, g_ns, c_ns, rank, world, dist):
        """The distributed top selection's orchestration (pm_amd.dist.top_selection:
        global offsets from the exchange's counts, SUM / MIN reductions of each
        pass) with a protocol stand-in for pm_amd.KdTopSel."""
        from pm_amd import dist as pmdist

        class FakePm:
            KdTopSel = _FakeTopSel
        sel, _ = pmdist.top_selection(FakePm, g_local, c_local, g_ns, c_ns, rank, world, dist)
        return sel

    def global_map(self, g, c, rank=0, world=1, dist=None, sel=None):
        self.last = (g.numpy().copy(), c.numpy().copy())
        if sel is not None:
            # every rank's reductions cover the gathered map exactly once, and
            # its global indices address its own rows in the gathered arrays
            n = g.shape[0] + c.shape[0]
            assert sel.total == [n, n * (n - 1) // 2, 0, -(n - 1)], (sel.total, n)
            gc = torch.cat([g, c])[:, [0, 1, 2, 7, 8, 9]]   # what the exchange carries
            for rows, first in ((sel.a, sel.a_first), (sel.b, sel.b_first)):
                assert torch.equal(gc[first: first + rows.shape[0]], rows[:, [0, 1, 2, 7, 8, 9]])
            self.sel_checked = True
        return self.o.PhotonMap(g.numpy(), 1.0, c.numpy(), 0.5)


    def render(self, gm, cm, tile_rank, tile_count, rgba):
        if rgba is not None:
            assert int(rgba.abs().sum()) == 0, "frame() hands a zeroed buffer to every rank's render"
        c = self.cfg
        img, _, _ = self.o.render(self.scene, self.cam, c.width, c.height, c.spp, c.depth, c.sky, self.lights, gm,
                                  cm, tile_rank=tile_rank, tile_count=tile_count, nthreads=2)
        return torch.from_numpy(img.view(np.int32).copy())


class _FakeTopSel:
    """Stand-in for pm_amd.KdTopSel with the same protocol (run(reduce) with
    "sum" / "min" passes over self.buf): pass 1 sums (row count, sum of global
    indices), pass 2 takes the min of (smallest index, -largest index)."""

    def __init__(self, a, a_first, b, b_first, n_total, world):
        self.a, self.a_first, self.b, self.b_first, self.n_total = a, a_first, b, b_first, n_total
        self.buf = torch.zeros(4, dtype=torch.int64)

    def run(self, reduce):
        ids = list(range(self.a_first, self.a_first + self.a.shape[0])) + \
            list(range(self.b_first, self.b_first + self.b.shape[0]))
        self.buf[0], self.buf[1] = len(ids), sum(ids)
        reduce(self.buf[:2], "sum")
        first = self.buf[:2].tolist()
        self.buf[0] = min(ids) if ids else self.n_total
        self.buf[1] = -max(ids) if ids else 0
        reduce(self.buf[:2], "min")
        self.total = first + self.buf[:2].tolist()
        return self


def _cfg():
    from pm_amd.dist import FrameConfig
    return FrameConfig(casted=6000, caustic=3000, width=40, height=30)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pm_amd
        from pm_amd import dist as pmdist
        meshes, lights = pm_amd.load_scene_file(conftest.CORNELL)
        cfg = _cfg()
        be = OracleBackend(meshes, lights, cfg)
        # a stale, non-zero frame buffer (as after a previous frame): frame() must
        # zero it before the tile render, or the SUM-reduce would add stale pixels
        stale = torch.full((cfg.height, cfg.width), 7, dtype=torch.int32)
        rgba, info = pmdist.frame(be, rank, world, dist, stale)
        assert getattr(be, "sel_checked", False)   # the distributed top selection ran (N > 1)
        g, c = be.last
        q.put((rank, rgba.numpy().copy() if rank == 0 else None, g, c, info["n_global"]))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_frame_matches_single_process(world):
    import torch.multiprocessing as mp
    import pm_amd
    from pm_amd import dist as pmdist
    meshes, lights = pm_amd.load_scene_file(conftest.CORNELL)
    be = OracleBackend(meshes, lights, _cfg())
    ref_img, ref_info = pmdist.frame(be, 0, 1, None)
    ref_g, ref_c = be.last
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, img, g, c, ng = q.get(timeout=300)
        res[r] = (img, g, c, ng)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keep = [0, 1, 2, 7, 8, 9]   # position + colour: what crosses the exchange (dist.pack_rows)
    for r in range(world):
        _, g, c, ng = res[r]
        assert np.array_equal(g[:, keep].view(np.uint32), ref_g[:, keep].view(np.uint32))   # == 1-process trace
        assert np.array_equal(c[:, keep].view(np.uint32), ref_c[:, keep].view(np.uint32))
        assert ng == ref_info["n_global"]
    assert np.array_equal(res[0][0], ref_img.numpy())                        # tile render + reduce == full image


def test_shard_ranges_partition():
    from pm_amd.dist import shard_range
    for total in (0, 1, 7, 10_000_001):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def test_shard_owners_balanced_and_deterministic():
    """Subtree -> rank dealing of the split kd build (pm_amd.dist.shard_owners):
    every subtree owned once, every rank used while subtrees last, the largest
    rank load within one subtree of the mean, and the same answer every call."""
    from pm_amd.dist import shard_owners
    rng = np.random.default_rng(0)
    for world in (2, 3, 4, 8, 16):
        for _ in range(20):
            sizes = [int(x) for x in rng.integers(1, 1000, size=2 * world)]
            owner, load = shard_owners(sizes, world)
            assert shard_owners(sizes, world) == (owner, load)
            assert sorted(set(owner)) == list(range(world))
            assert [sum(s for s, o in zip(sizes, owner) if o == r) for r in range(world)] == load
            assert max(load) <= sum(sizes) / world + max(sizes)


def test_pack_rows_round_trip():
    """The exchange moves position + colour only (pack_rows / unpack_rows)."""
    from pm_amd.dist import pack_rows, unpack_rows
    t = torch.from_numpy(np.random.default_rng(1).normal(size=(37, 10)).astype(np.float32))
    u = unpack_rows(pack_rows(t))
    keep = [0, 1, 2, 7, 8, 9]
    assert torch.equal(u[:, keep], t[:, keep]) and torch.count_nonzero(u[:, 3:7]) == 0


def _async_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pm_amd.dist import HostStagedDist
        hd = HostStagedDist(dist)
        t = torch.full((3, 2), float(rank + 1))
        out = torch.zeros((3 * world, 2))
        work = hd.all_gather_into_tensor(out, t, async_op=True)
        assert work is not None
        # collectives issued while the all-gather is pending (dist._maps: the
        # top selection's all-reduces) complete in order on every rank
        s = torch.tensor([rank + 1.0])
        hd.all_reduce(s, dist.ReduceOp.SUM)
        work.wait()
        work.wait()   # idempotent
        out2 = torch.zeros((3 * world, 2))
        assert hd.all_gather_into_tensor(out2, t) is None   # synchronous form
        q.put((rank, out.numpy().copy(), float(s.item()), torch.equal(out, out2)))
    finally:
        dist.destroy_process_group()


def test_host_staged_all_gather_is_async():
    """HostStagedDist.all_gather_into_tensor(async_op=True) returns a pending
    handle: the result lands in `out` at wait(), and
    collectives issued in between still match across ranks."""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (o, s, same)) for r, o, s, same in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.concatenate([np.full((3, 2), r + 1.0, np.float32) for r in range(world)])
    for r in range(world):
        o, s, same = res[r]
        assert np.array_equal(o, want) and s == 3.0 and same
