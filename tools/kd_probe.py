"""kd build probe: trees of many shapes built by the library PM_HIP_LIB names,
written to OUT.npz, and the build time of a config-3-sized map.
    python3 tools/kd_probe.py OUT.npz [--time]
    python3 tools/kd_probe.py --compare A.npz B.npz
    python3 tools/kd_probe.py --stamps   (a -DPM_KD_DIAG_TIME library: config 3's
        photon sets traced, the global map built, k_kd_local_sel's per-phase
        clock64 stamps averaged over its workgroups)
Shapes: sizes around the local-finish threshold (1023 / 1024 / 2047 / 2048),
uniform clouds, planes of ties, exact duplicates, one repeated point, a few
distinct values, +inf coordinates and negative zeros."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "photon-mapping_amd"))


def records(n, kind, seed):
    rng = np.random.default_rng(seed)
    rec = np.zeros((n, 11), np.float32)
    rec[:, 0:3] = rng.uniform(-20, 20, size=(n, 3))
    if kind == "ties":
        rec[: n // 3, 1] = 0.0
        rec[n // 3: n // 2, 2] = 7.25
    elif kind == "dups":
        rec[n // 7: n // 2, 0:3] = 5.0
    elif kind == "same":
        rec[:, 0:3] = (1.0, -2.0, 3.0)
    elif kind == "few":
        rec[:, 0:3] = rng.integers(-3, 4, size=(n, 3)).astype(np.float32)
    elif kind == "wall":   # Cornell-like: most points on axis planes
        f = rng.integers(0, 4, size=n)
        rec[f == 0, 0] = -10.0
        rec[f == 1, 1] = 0.0
        rec[f == 2, 2] = 10.0
    elif kind == "special":
        rec[::5, 0] = -0.0
        rec[1::5, 1] = 0.0
        rec[2::11, 2] = np.inf
        rec[3::13, 0] = -np.inf
    elif kind == "narrow":   # a tiny range far from zero (deep key bits)
        rec[:, 0:3] = 1000.0 + rng.uniform(0, 1e-3, size=(n, 3)).astype(np.float32)
    rec[:, 6:9] = rng.uniform(0, 1, size=(n, 3))
    rec[:, 9] = 1.0
    return rec


CASES = [(n, "uniform") for n in (1, 2, 3, 5, 7, 64, 1000, 1023, 1024, 1025, 2047, 2048, 2049, 4097, 65537,
                                   70000, 300000, 2_000_003)]
CASES += [(n, k) for k in ("ties", "dups", "same", "few", "wall", "special", "narrow")
          for n in (1500, 5000, 70000, 1_000_001)]


def run(out, timing):
    import torch
    import pm_amd
    print("library:", pm_amd.LIB_PATH, flush=True)
    res = {}
    for i, (n, kind) in enumerate(CASES):
        t = torch.from_numpy(records(n, kind, 1000 + i)).cuda()
        pm_amd.build_tree(t)
        res[f"{kind}_{n}"] = t.cpu().numpy()
    torch.cuda.synchronize()
    print("trees:", len(res), flush=True)
    if timing:
        rng = np.random.default_rng(3)
        sizes = [int(x) for x in os.environ.get("KD_N", "45400000").split(",")]
        for n in sizes:
            ph = torch.zeros((n, 10), dtype=torch.float32, device="cuda")
            ph[:, 0:3] = torch.from_numpy(rng.uniform(-50, 50, size=(n, 3)).astype(np.float32)).cuda()
            ph[: n // 4, 1] = 0.0   # a floor
            ph[:, 6:9] = 0.5
            for rep in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                m = pm_amd.PhotonMap(ph, 1.0)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3
                if rep >= 3:
                    print(f"build {n}: {dt:.2f} ms (phase kdbuild {pm_amd.phase_us('kdbuild') / 1e3:.2f} ms)",
                          flush=True)
                if rep == 4:
                    res[f"big_crc_{n}"] = digest(m.export())
                del m
            del ph
    np.savez(out, **res)


def digest(t):
    import torch
    w = t.contiguous().view(torch.int32).reshape(-1).to(torch.int64) & 0xFFFFFFFF
    idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64)
    a = int(((w * (idx % 1_000_003 + 1)) % 2_147_483_647).sum().item())
    b = int((w ^ (idx * 0x9E3779B1 & 0xFFFFFFFF)).sum().item())
    return np.array([w.numel(), a, b], np.int64)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        if k not in B.files:
            print("missing", k)
            continue
        x, y = A[k], B[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
        if not same:
            bad += 1
            diff = np.nonzero((x.view(np.uint32) != y.view(np.uint32)).any(axis=-1))[0] if x.shape == y.shape else []
            print("DIFF", k, x.shape, y.shape, "rows", len(diff), diff[:8])
    print("compared", len(A.files), "bad", bad)
    return bad


def stamps():
    import ctypes
    import torch
    import pm_amd
    from pm_amd import scenes
    meshes, lights = scenes.sponza_class()
    scene = pm_amd.Scene(meshes)
    g, c = pm_amd.run_photon_sets(scene, lights, 10_000_000, 1_000_000, 30)
    names = ["load + extents", "block level 0", "block level 1", "block level 2", "block level 3",
             "wave sorts", "wave levels + write-out"]
    fn = pm_amd._lib.pm_diag_kd_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    for rep in range(3):
        m = pm_amd.PhotonMap(g, 1.0, c, 0.5)
        torch.cuda.synchronize()
        buf = np.zeros(65536 * 8, np.uint64)
        assert fn(buf.ctypes.data, buf.size) == 0
        st = buf.reshape(-1, 8).astype(np.int64)
        ok = (st[:, 0] > 0) & (st[:, 7] >= st[:, 0]) & np.all(st[:, 1:] > 0, axis=1)
        d = np.diff(st[ok], axis=1)
        tot = st[ok, 7] - st[ok, 0]
        print(f"rep {rep}: {ok.sum()} workgroups, kdbuild {pm_amd.phase_us('kdbuild') / 1e3:.2f} ms, "
              f"mean {tot.mean():.0f} clocks per workgroup", flush=True)
        for k, nm in enumerate(names):
            print(f"   {nm:26s} {d[:, k].mean():9.0f} clocks  {100 * d[:, k].mean() / tot.mean():5.1f} %", flush=True)
        del m


if __name__ == "__main__":
    if sys.argv[1] == "--stamps":
        sys.exit(stamps())
    if sys.argv[1] == "--compare":
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
    run(sys.argv[1], "--time" in sys.argv)
