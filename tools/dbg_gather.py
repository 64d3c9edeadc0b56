import os, sys, subprocess, json
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
CHILD = r'''
import sys, os, numpy as np, torch
sys.path[:0] = [os.path.join(sys.argv[1], "photon-mapping_amd"), os.path.join(sys.argv[1], "oracle")]
import pm_amd, oracle
m, l = pm_amd.load_scene_file(os.path.join(sys.argv[1], "tests/golden/scenes/cornell-box/cornell-box.glb"))
os_ = oracle.Scene(m)
g = oracle.trace(os_, l, 30000, 10, False); c = oracle.trace(os_, l, 30000, 10, True)
rng = np.random.default_rng(11)
q = g[rng.integers(0, len(g), 6000), 0:3] + rng.normal(scale=0.5, size=(6000, 3)).astype(np.float32)
q = np.ascontiguousarray(q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))].astype(np.float32))
brdf = rng.uniform(0, 0.4, size=len(q)).astype(np.float32)
gm = pm_amd.PhotonMap(torch.from_numpy(g).cuda(), 1.0, torch.from_numpy(c).cuda(), 0.5)
om = oracle.PhotonMap(g, 1.0, c, 0.5)
ref = om.gather(q, brdf)
outs = [pm_amd.gather_photons(gm, torch.from_numpy(q).cuda(), torch.from_numpy(brdf).cuda()).cpu().numpy() for _ in range(3)]
for o in outs:
    bad = np.where(np.any(o.view(np.uint32) != ref.view(np.uint32), axis=1))[0]
    print(os.path.basename(os.path.dirname(pm_amd.LIB_PATH)), "mismatch", len(bad), "of", len(q), "first", bad[:10].tolist(), "maxrel", float(np.max(np.abs(o - ref) / (np.abs(ref) + 1e-12))) if len(bad) else 0, flush=True)
'''
for lib in sys.argv[1:]:
    env = dict(os.environ, PM_HIP_LIB=os.path.join(ROOT, "photon-mapping_amd", lib, "libpm_hip.so"))
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=200)
    print(r.stdout, r.stderr[-2000:] if r.returncode else "")
