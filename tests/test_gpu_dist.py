"""Multi-process frame on the GPU: two ranks share cuda:0 and talk
over gloo (RCCL needs one device per rank; the 8-GPU run is the driver's), with
host staging around the collectives. Checks the whole N > 1 path on device:
photon-shard trace, packed all-gather, the kd-tree split across ranks
(KdShardPlan: top levels, balanced subtrees, subtree all-gather, placement),
tile-sharded render and the image reduce -- rank 0's image equals one process's."""
import os
import socket

import numpy as np
import pytest

import conftest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

W, H = 64, 48


def _frame(rank, world, dist):
    import pm_amd
    from pm_amd import dist as pmdist
    meshes, lights = pm_amd.load_scene_file(conftest.CORNELL)
    cfg = pmdist.FrameConfig(casted=40000, caustic=20000, width=W, height=H)
    be = pmdist.GpuBackend(pm_amd.Scene(meshes), lights, cfg, rank, world)
    rgba = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    out, info = pmdist.frame(be, rank, world, dist, rgba)
    return out.cpu().numpy().copy(), info["n_global"]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pm_amd.dist import HostStagedDist
        img, ng = _frame(rank, world, HostStagedDist(dist))
        q.put((rank, img if rank == 0 else None, ng))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_on_one_gpu_match_single_process(world):
    import pm_amd
    if pm_amd.device_count() == 0:
        pytest.skip("needs a GPU")
    torch.cuda.set_device(0)
    ref, ref_n = _frame(0, 1, None)
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, img, ng = q.get(timeout=110)
        res[r] = (img, ng)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(res[r][1] == ref_n for r in range(world))
    assert np.array_equal(res[0][0], ref)
