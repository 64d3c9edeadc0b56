"""Shared test setup. GPU tests are marked @pytest.mark.gpu and call the HIP
path through the C-ABI; everything else runs on CPU (oracle, host I/O, ABI
symbol checks, gloo multi-process logic)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "photon-mapping_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLDEN, "scenes")
CORNELL = os.path.join(SCENES, "cornell-box", "cornell-box.glb")
SPHERE = os.path.join(SCENES, "sphere", "sphere.glb")


def _oracle_threads():
    """Threads for the CPU oracle in tests: the CPUs this process may use, capped
    by a cgroup CPU quota (16 on a one-GPU box) and at 16."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return max(1, min(16, n))


ORACLE_THREADS = _oracle_threads()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def cornell():
    import pm_amd
    return pm_amd.load_scene_file(CORNELL)


@pytest.fixture(scope="session")
def sphere():
    import pm_amd
    return pm_amd.load_scene_file(SPHERE)
