"""pm_render_begin on a second stream from a second host thread, while the
main thread traces photons and builds the kd-trees of the same scene on the
default stream (pm.h: the begin half is map-independent and may overlap map
building). Round 1 saw a GPU memory fault in this configuration once; VERDICT
r1 asked for it to be re-tested on the current library. Runs
tools/concurrency_probe.py in a child process (bounded by a timeout, so a hang
or fault ends the test, not the suite): every round's photons, kd-tree and
image must equal the serial run's bit for bit."""
import os
import subprocess
import sys

import pytest

import conftest

pytestmark = pytest.mark.gpu


def test_render_begin_concurrent_with_trace_and_build():
    probe = os.path.join(conftest.ROOT, "tools", "concurrency_probe.py")
    r = subprocess.run([sys.executable, "-u", probe], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count("image True") == 3, r.stdout
