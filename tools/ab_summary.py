"""Summarise gpu_ab.sh outputs: one line per bench log (frame and phase ms)."""
import glob, json
for f in sorted(glob.glob("gpurun_out/bench_*.log")):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "NO RESULT"); continue
    d = json.loads(lines[-1]); p = d["phases_ms"]
    print(f"{f[18:-4]:28s} frame {d['ms_per_frame']:7.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items()))
