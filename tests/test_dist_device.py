"""N > 1 device rule: HIP's and torch's current device are
per host thread and a new thread starts on device 0, so GpuBackend.start_render's
side thread must make its rank's GPU current before it touches device memory.
CPU-only: torch.cuda is replaced by a recorder, the library by a stub, and the
test checks that the thread's first action is set_device(<the side stream's
device>) — before pm.render_begin and before the caustic trace."""
import threading

import pytest

import conftest  # noqa: F401  (sys.path)


class _FakeStream:
    def __init__(self, device):
        self.device = device
        self.cuda_stream = 0x1234


class _StubPM:
    PHOTON_POWER = 1.0
    CAUSTICS_PHOTON_POWER = 0.5

    def __init__(self, log):
        self.log = log

    def render_begin(self, *a, **kw):
        self.log.append(("render_begin", threading.current_thread().name))
        return object()

    def phase_us(self, name):
        return 0.0

    def run_point_light_ray_gen(self, *a, **kw):
        self.log.append(("trace", kw.get("stream")))
        return "photons"

    def PhotonMap(self, *a, **kw):
        self.log.append(("map", kw.get("stream")))
        return "cmap"


@pytest.mark.parametrize("after", [True, False])
@pytest.mark.parametrize("device", ["cuda:3", "cuda:7"])
def test_start_render_thread_sets_rank_device_first(monkeypatch, device, after):
    import torch
    from pm_amd import dist

    log = []
    monkeypatch.setattr(torch.cuda, "Stream", lambda *a, **kw: _FakeStream(torch.device(device)))
    monkeypatch.setattr(torch.cuda, "set_device",
                        lambda d: log.append(("set_device", str(torch.device(d)), threading.current_thread().name)))
    be = dist.GpuBackend.__new__(dist.GpuBackend)
    be.pm = _StubPM(log)
    be.scene, be.lights, be.cam, be.cbuf = object(), [], object(), None
    be.cfg = dist.FrameConfig(casted=10, caustic=10, begin_after_trace=after)
    be.phase = {}
    pending = be.start_render(3, 8, caustic_shard=(3, 8), caustic_map=True)
    be.trace_done(pending)   # what _maps does once the global trace is over
    job, _ = be.join_render(pending)
    assert job is not None
    assert log[0][0] == "set_device" and log[0][1] == device, log
    assert log[0][2] == "pm-render-begin"      # in the side thread, not the caller's
    # begin_after_trace (default): the caustic trace and map first, the render
    # begin once the global trace is done
    order = ["trace", "map", "render_begin"] if after else ["render_begin", "trace", "map"]
    assert [e[0] for e in log] == ["set_device"] + order, log
    for e in log[1:]:
        if e[0] != "render_begin":
            assert e[1] == 0x1234   # the trace and map run on the side stream
