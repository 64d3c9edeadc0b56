"""Single-rank frame orchestration (pm_amd.dist.frame) with a recording
backend: which thread traces the caustic photons and builds their map, and
when the render begin starts, for the default order (begin_after_trace: the
fused photon-path kernel holds the GPU for the whole global trace, DESIGN.md
§4.2) and the two alternatives. CPU only; no library calls."""
import threading

import pytest

import conftest  # noqa: F401  (sys.path)


class _Set:   # a photon set or map as frame() reads it (n, shape)
    n = 1
    shape = (1,)


class _RecordingBackend:
    def __init__(self, cfg):
        self.cfg = cfg
        self.phase = {}
        self.log = []
        self._lock = threading.Lock()

    def _rec(self, what):
        with self._lock:
            self.log.append((what, threading.current_thread().name))

    # main-thread steps
    def trace(self, caustics, rank, world):
        self._rec("trace_caustic" if caustics else "trace_global")
        return _Set()

    def caustic_map(self, c):
        self._rec("caustic_map")
        return _Set()

    def global_map(self, g, c, rank, world, dist):
        self._rec("global_map")
        return _Set()

    def trace_both(self, rank, world):
        self._rec("trace_both")
        return _Set(), _Set()

    # the side thread, as GpuBackend.start_render runs it
    def start_render(self, tile_rank, tile_count, caustic_shard=None, caustic_map=False, caustic_from_main=False):
        box = {"c_ready": threading.Event(), "trace_done": threading.Event()}
        late = self.cfg.begin_after_trace

        def run():
            if not late:
                self._rec("render_begin")
            if caustic_from_main:
                box["trace_done"].wait()
                if caustic_map and "c_in" in box:
                    self._rec("side_caustic_map")
                    box["cm"] = _Set()
                if late:
                    self._rec("render_begin")
            elif caustic_shard is not None:
                self._rec("side_trace_caustic")
                box["c"] = _Set()
                box["c_ready"].set()
                if caustic_map:
                    self._rec("side_caustic_map")
                    box["cm"] = _Set()
                if late:
                    box["trace_done"].wait()
                    self._rec("render_begin")
            elif late:
                box["trace_done"].wait()
                self._rec("render_begin")
            box["c_ready"].set()

        th = threading.Thread(target=run, name="side")
        th.start()
        return th, box

    def caustic_photons(self, pending):
        pending[1]["c_ready"].wait()
        return pending[1]["c"]

    def caustic_map_of(self, pending):
        self.join_render(pending)
        return pending[1]["cm"]

    @staticmethod
    def trace_done(pending, caustic=None):
        if caustic is not None:
            pending[1]["c_in"] = caustic
        pending[1]["trace_done"].set()

    @staticmethod
    def join_render(pending):
        pending[1]["trace_done"].set()
        pending[0].join()

    def finish_render(self, pending, gm, cm, rgba):
        self.join_render(pending)
        self._rec("finish")
        return rgba


@pytest.mark.parametrize("opts,main,side", [
    # default: both sets in one trace launch; the side thread builds the caustic
    # map and runs the render begin once the trace is over (beside the kd build)
    ({}, ["trace_both", "global_map", "finish"], ["side_caustic_map", "render_begin"]),
    ({"begin_after_trace": False}, ["trace_both", "global_map", "finish"], ["render_begin", "side_caustic_map"]),
    ({"one_trace": False}, ["trace_global", "global_map", "finish"],
     ["side_trace_caustic", "side_caustic_map", "render_begin"]),
    ({"one_trace": False, "begin_after_trace": False}, ["trace_global", "global_map", "finish"],
     ["render_begin", "side_trace_caustic", "side_caustic_map"]),
    ({"one_trace": False, "caustic_after_trace": True},
     ["trace_global", "trace_caustic", "caustic_map", "global_map", "finish"], ["render_begin"]),
])
def test_single_rank_frame_order(opts, main, side):
    from pm_amd import dist
    cfg = dist.FrameConfig(casted=10, caustic=10, **opts)
    be = _RecordingBackend(cfg)
    dist.frame(be, 0, 1)
    assert [w for w, t in be.log if t != "side"] == main, be.log
    assert [w for w, t in be.log if t == "side"] == side, be.log
    if cfg.begin_after_trace:
        # the render begin starts only once the global trace is over, whichever
        # thread traces the caustic photons (caustic_after_trace too)
        order = [w for w, _ in be.log]
        first = "trace_both" if cfg.one_trace else "trace_global"
        assert order.index("render_begin") > order.index(first)
