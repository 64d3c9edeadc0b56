"""kd-build time vs map size on one GPU (what every rank pays per frame at N GPUs
under the replicated build): synthetic photons uniform in a box, N = k x 45.4M.
  KS="1 2 4 8" (map sizes), REPL=0 skips the replicated builds, SHARD=0 the
  sharded ones, ROWS=0 the exchange's old compaction + re-expansion."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "photon-mapping_amd"))
import torch
import pm_amd
torch.cuda.set_device(0)
base = 45_427_140
for k in [int(x) for x in os.environ.get("KS", "1 2 4 8").split()] if os.environ.get("REPL", "1") == "1" else []:
    n = base * k
    g = torch.rand((n, 10), device="cuda", dtype=torch.float32) * 100.0
    c = torch.empty((0, 10), device="cuda", dtype=torch.float32)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.time()
        m = pm_amd.PhotonMap(g, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER)
        torch.cuda.synchronize()
        print(f"N={n} ({k}x) kdbuild {pm_amd.phase_us('kdbuild') / 1e3:.1f} ms wall {(time.time() - t0) * 1e3:.1f} ms",
              flush=True)
        del m
    del g
    torch.cuda.empty_cache()

# sharded build (pm_amd.dist.sharded_map without the collective): per-rank
# critical path = plan (top selection) + its subtree + placement
if os.environ.get("SHARD", "1") == "1":
    from pm_amd import dist as pmdist
    for k in [int(x) for x in os.environ.get("KS", "1 2 4 8").split()]:
        world = k
        if world < 2:
            continue
        n = base * k
        g = torch.rand((n, 10), device="cuda", dtype=torch.float32) * 100.0
        c = torch.empty((0, 10), device="cuda", dtype=torch.float32)
        # the exchange's output: rank r's (position, colour) rows at [r m, r m + n_r)
        # of one padded buffer (pm_amd.dist.allgather_rows_start); ROWS=1 hands it to
        # the plan as it is (PhotonRows), ROWS=0 measures round 3's compaction +
        # re-expansion to pm_photon rows first
        ns = [pmdist.shard_range(n, r, world)[1] - pmdist.shard_range(n, r, world)[0] for r in range(world)]
        mpad = max(ns)
        gbuf = torch.zeros((world * mpad, 6), device="cuda", dtype=torch.float32)
        for r in range(world):
            a0, a1 = pmdist.shard_range(n, r, world)
            pmdist.pack_rows(g[a0:a1], gbuf[r * mpad: r * mpad + ns[r]])
        rows_mode = os.environ.get("ROWS", "1") == "1"
        for rep in range(2):
            torch.cuda.synchronize()
            tc = time.time()
            if rows_mode:
                gin = pm_amd.PhotonRows.of_padded(gbuf, ns, mpad)
            else:
                gin = pmdist.unpack_rows(torch.cat([gbuf[r * mpad: r * mpad + ns[r]] for r in range(world)]))
            torch.cuda.synchronize()
            t_copy = (time.time() - tc) * 1e3
            print(f"  post-gather copies ({'PhotonRows: none' if rows_mode else 'cat + unpack'}): {t_copy:.1f} ms",
                  flush=True)
            torch.cuda.synchronize()
            t0 = time.time()
            if os.environ.get("DIST", "1") == "1":
                # distributed top selection: each rank's passes over its own shard
                # (here rank after rank; the per-rank cost is the max), then the
                # plan from the gathered photons (elements, top fix, classify)
                sel, us = pmdist.simulated_top_selection(pm_amd, g, c, world)
                torch.cuda.synchronize()
                t1 = time.time()
                plan = pm_amd.KdShardPlan(gin, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=world,
                                          sel=sel)
                torch.cuda.synchronize()
                t_from = (time.time() - t1) * 1e3
                t_plan = max(us) / 1e3 + t_from
                print(f"  dist top selection: per-rank passes max {max(us) / 1e3:.1f} ms ({sel.steps} steps, "
                      f"{sel.steps - 1} all-reduces), plan from gathered photons {t_from:.1f} ms", flush=True)
            else:
                plan = pm_amd.KdShardPlan(gin, pm_amd.PHOTON_POWER, c, pm_amd.CAUSTICS_PHOTON_POWER, world=world)
                t_plan = pm_amd.phase_us("kdbuild") / 1e3
            bufs, t_sub = [], []
            for r in range(world):
                b, us = pmdist.shard_local(plan, r, world)
                bufs.append(b)
                t_sub.append(us / 1e3)
            everyone = torch.cat(bufs)
            m = pmdist.shard_assemble(plan, everyone, world)
            t_asm = pm_amd.phase_us("kdbuild") / 1e3
            torch.cuda.synchronize()
            print(f"N={n} world={world} plan {t_plan:.1f} ms, subtree max {max(t_sub):.1f} ms, place {t_asm:.1f} ms"
                  f" -> per-rank {t_plan + max(t_sub) + t_asm:.1f} ms (+ all-gather of {everyone.numel() * 4 / 1e9:.2f} GB)",
                  flush=True)
            del plan, bufs, everyone, m, gin
        del g, gbuf
        torch.cuda.empty_cache()
