"""bench.py's roofline.traffic identity: the PMC file is
accepted for the built library's binary sha or for the digest of the sources it
was built from, since hipcc builds are not bit-reproducible. CPU only."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _copy_tree(dst):
    for rel in ("photon-mapping_amd/csrc", ):
        shutil.copytree(os.path.join(ROOT, rel), os.path.join(dst, rel))
    os.makedirs(os.path.join(dst, "include"))
    shutil.copy(os.path.join(ROOT, "photon-mapping_amd", "Makefile"), os.path.join(dst, "photon-mapping_amd"))
    shutil.copy(os.path.join(ROOT, "include", "pm.h"), os.path.join(dst, "include"))
    flags = os.path.join(ROOT, "photon-mapping_amd", "lib", "build_flags.txt")
    if os.path.exists(flags):
        os.makedirs(os.path.join(dst, "photon-mapping_amd", "lib"))
        shutil.copy(flags, os.path.join(dst, "photon-mapping_amd", "lib"))


def test_source_digest_tracks_the_sources(tmp_path, monkeypatch):
    import bench
    monkeypatch.delenv("PM_HIP_LIB", raising=False)
    d0 = bench.source_digest()
    assert len(d0) == 64 and d0 == bench.source_digest()
    _copy_tree(str(tmp_path))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.source_digest() == d0            # same sources elsewhere: same identity
    knn = tmp_path / "photon-mapping_amd" / "csrc" / "knn.hip"
    knn.write_bytes(knn.read_bytes() + b"\n// edited\n")
    assert bench.source_digest() != d0            # an edited kernel drops the old counters
    (tmp_path / "photon-mapping_amd" / "csrc" / "notes.txt").write_text("x")
    d1 = bench.source_digest()
    (tmp_path / "photon-mapping_amd" / "csrc" / "notes.txt").write_text("y")
    assert bench.source_digest() == d1            # non-source files do not count


def test_source_digest_tracks_the_build_flags(tmp_path, monkeypatch):
    """a variant library (same sources, other -D flags) is not the
    library the counters were collected on"""
    import bench
    monkeypatch.delenv("PM_HIP_LIB", raising=False)
    _copy_tree(str(tmp_path))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    lib = tmp_path / "photon-mapping_amd" / "lib"
    lib.mkdir(exist_ok=True)
    (lib / "build_flags.txt").write_text("--offload-arch=gfx950 -O3\n")
    d0 = bench.source_digest()
    (lib / "build_flags.txt").write_text("--offload-arch=gfx950 -O3 -DPM_GATHER50_WIDE=2\n")
    d1 = bench.source_digest()
    assert d1 != d0
    var = tmp_path / "photon-mapping_amd" / "lib_v"
    var.mkdir()
    (var / "build_flags.txt").write_text("--offload-arch=gfx950 -O3\n")
    monkeypatch.setenv("PM_HIP_LIB", str(var / "libpm_hip.so"))
    assert bench.source_digest() == d0   # the library in use decides
