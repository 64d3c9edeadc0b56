"""Workloads run once with the production libpm_hip.so and once, in a child
process, with the check variant (lib_check/libpm_hip.so, PM_CHECK_VARIANT: plain
kNN walk, all-global kd levels, Karras LBVH, forced continuation rerun, 4-entry
LDS traversal stack). Every output is a numpy array; the two runs must agree
bit for bit (tests/test_gpu_check_variant.py). Run as
    python variant_workloads.py OUT.npz [--full]
with PM_HIP_LIB selecting the library."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for _p in (HERE, os.path.join(ROOT, "photon-mapping_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

CAM = ((80.0, 30.0, 0.0), (10.0, 20.0, 0.0), (0.0, 1.0, 0.0), 0.87)


def cloud(n, seed):
    """n small randomly oriented triangles filling a cube: rays cross many
    overlapping boxes, so the traversal stack grows deep (spill path)."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, size=(n, 1, 3))
    v = (c + rng.normal(scale=0.6, size=(n, 3, 3))).reshape(-1, 3).astype(np.float32)
    return v, np.arange(3 * n, dtype=np.int32).reshape(n, 3)


def cloud_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-12, 12, size=(n, 3)).astype(np.float32)
    dr = rng.normal(size=(n, 3)).astype(np.float32)
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 3], rays[:, 4:7], rays[:, 7] = o, 1e-3, dr, 1e10
    rays[n // 2:, 7] = 3.0
    return rays


CLOUD_MAT = np.array([0.7, 0.6, 0.5, 0.6, 0.2, 0.2, 1.5], np.float32)
CLOUD_LIGHTS = [dict(pos=(0.1, 0.2, 0.3), rgb=(1, 1, 1), power=100.0)]


def kd_records(n, seed, kind="ties"):
    rng = np.random.default_rng(seed)
    rec = np.zeros((n, 11), np.float32)
    rec[:, 0:3] = rng.uniform(-20, 20, size=(n, 3))
    if kind == "ties":
        rec[: n // 7, 2] = 1.5          # ties on one axis
        rec[n // 7: n // 5, 0:3] = 5.0  # exact duplicates
    elif kind == "same":                # one repeated point
        rec[:, 0:3] = (1.0, -2.0, 3.0)
    elif kind == "wall":                # most points on axis planes (Cornell-like)
        f = rng.integers(0, 4, size=n)
        rec[f == 0, 0] = -10.0
        rec[f == 1, 1] = 0.0
        rec[f == 2, 2] = 10.0
    elif kind == "special":             # signed zeros and infinities
        rec[::5, 0] = -0.0
        rec[1::5, 1] = 0.0
        rec[2::11, 2] = np.inf
        rec[3::13, 0] = -np.inf
    rec[:, 6:9] = rng.uniform(0, 1, size=(n, 3))
    rec[:, 9] = 1.0
    return rec


def _stats(pm):
    st = pm.render_stats()
    return np.array([st.pixels, st.path_vertices, st.caustic_queries, st.global_queries, st.rays], np.int64)


def run(full: bool = False) -> dict:
    import torch
    import pm_amd
    from pm_amd import scenes
    out = {}
    # 1. traversal (closest hit, any hit, photon trace) on a deep-stack scene
    v, i = cloud(30000, 7)
    sc = pm_amd.Scene([pm_amd.MeshData(v, i, CLOUD_MAT)])
    rays = torch.from_numpy(cloud_rays(20000, 8)).cuda()
    out["cloud_hits"] = sc.intersect(rays).cpu().numpy()
    out["cloud_occ"] = sc.occluded(rays).cpu().numpy()
    out["cloud_photons"] = pm_amd.run_normal(sc, CLOUD_LIGHTS, 20000, 10).cpu().numpy()
    # 2. Cornell: trace, kd maps, gathers, renders (continuation rerun in the check variant)
    meshes, lights = pm_amd.load_scene_file(os.path.join(HERE, "golden", "scenes", "cornell-box", "cornell-box.glb"))
    gs = pm_amd.Scene(meshes)
    g = pm_amd.run_normal(gs, lights, 100000, 10)
    c = pm_amd.run_caustics(gs, lights, 100000, 10)
    out["cornell_g"], out["cornell_c"] = g.cpu().numpy(), c.cpu().numpy()
    gm, cm = pm_amd.load_photons(g, c)
    out["cornell_gmap"] = gm.export().cpu().numpy()
    out["cornell_cmap"] = cm.export().cpu().numpy()
    rng = np.random.default_rng(5)
    gn = out["cornell_g"]
    q = gn[rng.integers(0, len(gn), 20000), 0:3] + rng.normal(scale=1.0, size=(20000, 3)).astype(np.float32)
    q = np.concatenate([q, gn[:2000, 0:3], gn[:500, 0:3], rng.uniform(-300, 300, size=(200, 3))]).astype(np.float32)
    q = np.ascontiguousarray(q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))])   # spatial order: tight leader seeds
    brdf = rng.uniform(0, 0.4, size=len(q)).astype(np.float32)
    qt, bt = torch.from_numpy(q).cuda(), torch.from_numpy(brdf).cuda()
    empty = torch.zeros((0, 10), dtype=torch.float32, device="cuda")
    em, _ = pm_amd.load_photons(empty, empty)
    for name, m in (("g", gm), ("c", cm), ("e", em)):
        out[f"gather_{name}"] = pm_amd.gather_photons(m, qt, bt).cpu().numpy()
    # the collect-and-sort gather (k > 64): 8- and 16-key rows
    for k in (200, 256):
        out[f"gather_k{k}"] = pm_amd.gather_photons(gm, qt, bt, k=k).cpu().numpy()
    out["knn_ids"], out["knn_d2"], out["knn_md"] = [x.cpu().numpy() for x in pm_amd.knn(gm, qt[:5000], k=50)]
    for W, H, spp in ((64, 48, 2), (40, 30, 1)):
        cam = pm_amd.setup_camera(*CAM, W, H)
        rgba, rgb = pm_amd.render(gs, cam, W, H, spp, 30, (1, 1, 1), lights, gm, cm)
        out[f"render_{W}_rgba"], out[f"render_{W}_rgb"] = rgba.cpu().numpy(), rgb.cpu().numpy()
        out[f"render_{W}_stats"] = _stats(pm_amd)
    # 3. kd-trees (LDS finish vs all-global levels), ties and duplicates
    for n in (5, 1023, 1024, 70000, 2_000_003):
        t = torch.from_numpy(kd_records(n, 100 + n)).cuda()
        pm_amd.build_tree(t)
        out[f"kd_{n}"] = t.cpu().numpy()
    for kind, n in (("same", 5000), ("wall", 300001), ("special", 70001)):
        t = torch.from_numpy(kd_records(n, 7 + n, kind)).cuda()
        pm_amd.build_tree(t)
        out[f"kd_{kind}_{n}"] = t.cpu().numpy()
    # 4. sphere scene (glass): photons and a render
    meshes, lights = pm_amd.load_scene_file(os.path.join(HERE, "golden", "scenes", "sphere", "sphere.glb"))
    ss = pm_amd.Scene(meshes)
    g = pm_amd.run_normal(ss, lights, 200000, 10)
    c = pm_amd.run_caustics(ss, lights, 200000, 10)
    out["sphere_g"], out["sphere_c"] = g.cpu().numpy(), c.cpu().numpy()
    gm, cm = pm_amd.load_photons(g, c)
    cam = pm_amd.setup_camera(*CAM, 48, 40)
    rgba, rgb = pm_amd.render(ss, cam, 48, 40, 2, 30, (1, 1, 1), lights, gm, cm)
    out["sphere_rgb"], out["sphere_stats"] = rgb.cpu().numpy(), _stats(pm_amd)
    del gm, cm, g, c
    if full:
        # 5. BASELINE config 3 at full size: the seeded gather over the whole
        # 45.4 M-photon global map and 36 M Morton-ordered queries equals the
        # plain walk bit for bit (and so does every other alternate path)
        meshes, lights = scenes.sponza_class()
        sp = pm_amd.Scene(meshes)
        g = pm_amd.run_normal(sp, lights, 10_000_000, 10)
        c = pm_amd.run_caustics(sp, lights, 1_000_000, 10)
        out["c3_counts"] = np.array([g.shape[0], c.shape[0]], np.int64)
        out["c3_g_crc"] = _digest(g)
        out["c3_c_crc"] = _digest(c)
        gm, cm = pm_amd.load_photons(g, c)
        del g, c
        cam = pm_amd.setup_camera(*CAM, 1920, 1080)
        rgba, rgb = pm_amd.render(sp, cam, 1920, 1080, 1, 30, (1, 1, 1), lights, gm, cm)
        out["c3_rgb"], out["c3_rgba"], out["c3_stats"] = rgb.cpu().numpy(), rgba.cpu().numpy(), _stats(pm_amd)
        out["c3_gmap_crc"] = _digest(gm.export())
        del gm, cm, rgba, rgb, sp
        # 6. config 5 at the bench's per-GPU size: 10 M + 6.25 M photons, square
        # light + glass, the k = 200 caustic gather over the full caustic map
        meshes, lights = scenes.sponza_caustics()
        sp = pm_amd.Scene(meshes)
        g = pm_amd.run_normal(sp, lights, 10_000_000, 10)
        c = pm_amd.run_caustics(sp, lights, 6_250_000, 10)
        out["c5_counts"] = np.array([g.shape[0], c.shape[0]], np.int64)
        out["c5_c_crc"] = _digest(c)
        gm, cm = pm_amd.load_photons(g, c)
        del g, c
        out["c5_cmap_crc"] = _digest(cm.export())
        rgba, rgb = pm_amd.render(sp, cam, 1920, 1080, 1, 30, (1, 1, 1), lights, gm, cm, caustic_k=200)
        out["c5_rgb"], out["c5_rgba"], out["c5_stats"] = rgb.cpu().numpy(), rgba.cpu().numpy(), _stats(pm_amd)
        del gm, cm, rgba, rgb
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def _digest(t):
    """Order-sensitive 64-bit digest of a device tensor's bits (computed on the device)."""
    import torch
    w = t.contiguous().view(torch.int32).reshape(-1).to(torch.int64) & 0xFFFFFFFF
    idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64)
    a = int(((w * (idx % 1_000_003 + 1)) % 2_147_483_647).sum().item())
    b = int((w ^ (idx * 0x9E3779B1 & 0xFFFFFFFF)).sum().item())
    return np.array([w.numel(), a, b], np.int64)


if __name__ == "__main__":
    import torch  # noqa: F401  (torch's HIP runtime first: see pm_amd._load)
    import pm_amd
    print("library:", pm_amd.LIB_PATH, flush=True)
    res = run(full="--full" in sys.argv)
    np.savez(sys.argv[1], **res)
