"""Device rule of the C-ABI (include/pm.h "devices") and the
allocator's steady state:
  - a host thread that never chose a device, driving a stream it was handed,
    gets the same image as the main thread (the library follows the stream);
  - a handle used with a stream of another GPU is refused with PM_ERR_DEVICE
    (needs two GPUs; skipped on a one-GPU box);
  - frames of begin/finish on a side stream, the caustic gather on the
    library's side stream (k = 50 and k = 200), do not grow the allocator's
    live + cached bytes after the first frame."""
import threading

import numpy as np
import pytest

import conftest

pytestmark = pytest.mark.gpu

W, H = 64, 48


@pytest.fixture(scope="module")
def setup(cornell):
    import pm_amd
    import torch
    torch.cuda.set_device(0)
    meshes, lights = cornell
    sc = pm_amd.Scene(meshes)
    g = pm_amd.run_normal(sc, lights, 20000, 10)
    c = pm_amd.run_caustics(sc, lights, 20000, 10)
    gm, cm = pm_amd.load_photons(g, c)
    cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, W, H)
    ref, _ = pm_amd.render(sc, cam, W, H, 1, 30, (1, 1, 1), lights, gm, cm, want_rgb=False)
    torch.cuda.synchronize()
    return sc, lights, gm, cm, cam, ref


def test_fresh_thread_follows_the_stream(setup):
    import pm_amd
    import torch
    sc, lights, gm, cm, cam, ref = setup
    side = torch.cuda.Stream()
    rgba = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    box = {}

    def run():   # no set_device here on purpose: the library takes the device from `side`
        try:
            job = pm_amd.render_begin(sc, cam, W, H, 1, 30, (1, 1, 1), lights, stream=side.cuda_stream)
            job.finish(gm, cm, want_rgb=False, rgba=rgba, stream=side.cuda_stream)
            job.close()
        except BaseException as e:
            box["e"] = e

    th = threading.Thread(target=run)
    th.start()
    th.join()
    assert "e" not in box, box.get("e")
    torch.cuda.synchronize()
    assert torch.equal(rgba, ref)


@pytest.mark.skipif("__import__('pm_amd').device_count() < 2", reason="needs two GPUs")
def test_handle_on_other_device_is_refused(setup):
    import pm_amd
    import torch
    sc, lights, gm, cm, cam, ref = setup
    with torch.cuda.device(1):
        s1 = torch.cuda.Stream()
        q = torch.zeros((4, 3), dtype=torch.float32, device="cuda:1")
        b = torch.ones((4,), dtype=torch.float32, device="cuda:1")
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.gather_photons(gm, q, b, stream=s1.cuda_stream)
    assert e.value.status == pm_amd.PM_ERR_DEVICE
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.render_begin(sc, cam, W, H, 1, 30, (1, 1, 1), lights, stream=s1.cuda_stream)
    assert e.value.status == pm_amd.PM_ERR_DEVICE
    # a buffer on GPU 1 passed with a stream of GPU 0
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.gather_photons(gm, q, b)
    assert e.value.status == pm_amd.PM_ERR_DEVICE


@pytest.mark.parametrize("caustic_k", [0, 200])
def test_side_stream_frames_do_not_grow_the_pool(setup, caustic_k):
    import pm_amd
    import torch
    sc, lights, gm, cm, cam, ref = setup
    side = torch.cuda.Stream()
    seen = []
    for frame in range(4):
        job = pm_amd.render_begin(sc, cam, W, H, 1, 30, (1, 1, 1), lights, stream=side.cuda_stream,
                                  caustic_k=caustic_k)
        rgba, _ = job.finish(gm, cm, want_rgb=False)
        job.close()
        torch.cuda.synchronize()
        if caustic_k == 0:
            assert torch.equal(rgba, ref)
        live, cached = pm_amd.pool_stats(0)
        seen.append(live + cached)
    assert seen[1] == seen[2] == seen[3], seen
