"""The drop-in boundary itself: libpm_hip.so loads, exports exactly the entry
points include/pm.h declares, struct layouts match, and (on a host without a
GPU) compute calls fail loudly instead of falling back to the CPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

import conftest

HEADER = os.path.join(conftest.ROOT, "include", "pm.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pm_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    import pm_amd
    decl = header_functions()
    assert len(decl) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", pm_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (pm_\w+)", out))
    missing = [f for f in decl if f not in exported]
    assert not missing, missing
    # every declared function is bound by the Python mirror, and nothing else
    assert sorted(pm_amd.exported_symbols()) == decl


def test_struct_sizes_match_header():
    import pm_amd
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "pm.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(pm_material), sizeof(pm_mesh),
         sizeof(pm_light), sizeof(pm_photon), sizeof(pm_kd_photon), sizeof(pm_ray), sizeof(pm_hit),
         sizeof(pm_trace_params), sizeof(pm_render_params), sizeof(pm_config), sizeof(pm_photon_rows),
         offsetof(pm_photon_rows, seg_count));
  return 0;
}
"""
    import tempfile
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "s.c"), "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", os.path.join(d, "s"), os.path.join(d, "s.c")],
                   check=True)
    got = list(map(int, subprocess.run([os.path.join(d, "s")], capture_output=True, text=True).stdout.split()))
    exp = [C.sizeof(t) for t in (pm_amd.Material, pm_amd.Mesh, pm_amd.Light, pm_amd.Photon, pm_amd.KdPhoton,
                                 pm_amd.Ray, pm_amd.Hit, pm_amd.TraceParams, pm_amd.RenderParams, pm_amd.Config,
                                 pm_amd.PhotonRowsStruct)] + [pm_amd.PhotonRowsStruct.seg_count.offset]
    assert got == exp
    assert got[:5] == [28, got[1], 64, 40, 44]      # reference record sizes


def test_status_strings():
    import pm_amd
    for s in range(9):
        assert pm_amd.lib.pm_status_string(s) != b"unknown status"
    # 2: pm_render_params.caustic_k; 3: PM_ERR_DEVICE, pm_device_pool_stats; 4: pm_kd_top_sel_*;
    # 5: pm_photon_rows (pm_photon_map_create_rows, pm_kd_shard_plan_create_rows / _from_sel_rows)
    assert pm_amd.lib.pm_abi_version() == 6


def test_no_cpu_fallback_without_gpu(cornell):
    import pm_amd
    if pm_amd.device_count() > 0:
        pytest.skip("a GPU is visible: covered by the -m gpu suite")
    meshes, lights = cornell
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.Scene(meshes)
    assert e.value.status == pm_amd.PM_ERR_NO_DEVICE
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.PhotonMap(None, 1.0)
    assert e.value.status == pm_amd.PM_ERR_NO_DEVICE


def test_host_helpers_without_gpu():
    import pm_amd
    cam = pm_amd.setup_camera((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 800, 600)
    import oracle
    ocam = oracle.camera_setup((80, 30, 0), (10, 20, 0), (0, 1, 0), 0.87, 800, 600)
    assert bytes(cam) == bytes(ocam)                  # setupCamera, bitwise
    lights = [{"pos": (0, 0, 0), "rgb": (1, 1, 1), "power": 10.0}] * 2
    assert pm_amd.trace_capacity(lights, 10000, 10, False) == 10000 * 9
    assert pm_amd.trace_capacity(lights, 10000, 10, True) == 10000
    assert pm_amd.trace_capacity(lights, 10001, 10, False, 1, 3) == (10000 * 2 // 3 - 10000 // 3) * 9


def test_map_size_limit_rejected_before_any_work():
    """kd node tags are int32 (original index << 2 | split dim): maps of 2^29
    photons or more are rejected with PM_ERR_INVALID, checked
    before the device is touched, so the guard is testable on any host."""
    import pm_amd
    lib = pm_amd.lib
    fake = C.c_void_p(64)   # never dereferenced: the size check comes first
    out = C.c_void_p()
    for na, nb in ((1 << 29, 0), ((1 << 29) - 7, 7), (1 << 30, 0)):
        assert lib.pm_photon_map_create(fake, na, C.c_float(1.0), fake, nb, C.c_float(0.5), C.byref(out),
                                        None) == pm_amd.PM_ERR_INVALID
        assert lib.pm_kd_shard_plan_create(fake, na, C.c_float(1.0), fake, nb, C.c_float(0.5), 8, C.byref(out),
                                           None) == pm_amd.PM_ERR_INVALID
    assert lib.pm_kdtree_build(fake, 1 << 29, None, None) == pm_amd.PM_ERR_INVALID
    if pm_amd.device_count() == 0:   # just under the limit passes the guard and stops at the device probe
        assert lib.pm_kdtree_build(fake, (1 << 29) - 1, None, None) == pm_amd.PM_ERR_NO_DEVICE
