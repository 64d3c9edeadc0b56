#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / LDS / occupancy from hipcc -save-temps device
assembly (gfx950): python3 tools/kernel_resources.py DIR [--scratch-only]
(DIR holds *-hip-amdgcn-amd-amdhsa-gfx950.s: cd DIR && hipcc <the Makefile's
HIPFLAGS> -save-temps -c photon-mapping_amd/csrc/X.hip)."""
import glob, re, sys
only = "--scratch-only" in sys.argv
for f in sorted(glob.glob(sys.argv[1] + "/*-hip-amdgcn-amd-amdhsa-gfx950.s")):
    s = open(f).read()
    for m in re.finditer(r"^(_Z\S+):.*\n", s, re.M):
        name = m.group(1)
        tail = s[m.end():]
        end = tail.find(".Lfunc_end")
        body = tail[:end]
        meta = tail[end:end + 20000]
        v = re.search(r"NumVgprs:\s+(\d+)", meta)
        sc = re.search(r"ScratchSize:\s+(\d+)", meta)
        if not v:
            continue
        lds = re.search(r"LDSByteSize:\s+(\d+)", meta)
        occ = re.search(r"Occupancy:\s+(\d+)", meta)
        nsc = body.count("scratch_")
        if only and int(sc.group(1)) == 0:
            continue
        print(f"{f.split('/')[-1].split('-')[0]:10s} vgpr {v.group(1):>3s} scratch {sc.group(1):>4s} ({nsc:3d} ops) "
              f"lds {lds.group(1) if lds else '?':>6s} occ {occ.group(1) if occ else '?':>2s}  {name[:90]}")
