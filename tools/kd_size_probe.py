"""kd build time per map size (PhotonMap of uniform random photons on cuda:0,
pm_last_phase kdbuild), to place PM_KD_SEL_MIN: run once per library
(PM_HIP_LIB). SIZES="4e6 8e6 12e6 16777215 24e6" REPS=3."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "photon-mapping_amd"))
import torch  # noqa: E402

import pm_amd  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(7)
out = {}
for n in [int(float(x)) for x in os.environ.get("SIZES", "4e6 8e6 12e6 16777215 24e6").split()]:
    ph = torch.zeros((n, 10), dtype=torch.float32, device="cuda")
    ph[:, 0:3] = torch.rand((n, 3), generator=g, device="cuda") * 100.0
    ms = []
    for _ in range(int(os.environ.get("REPS", "3"))):
        m = pm_amd.PhotonMap(ph, 1.0)
        torch.cuda.synchronize()
        ms.append(pm_amd.phase_us("kdbuild") / 1e3)
        m.close()
    out[n] = round(min(ms), 2)
    print(f"n {n}: kd build {ms} ms", flush=True)
    del ph
    torch.cuda.empty_cache()
print(json.dumps({"lib": os.environ.get("PM_HIP_LIB", "lib"), "kd_ms": out}))
