"""Host-side boundary (B1) without a GPU: config.toml, scene ingest, photon text
files, PNG output. Fixtures are the reference's own scene / config files
(tests/golden/scenes, tests/golden/config.toml.example)."""
import json
import os
import shutil
import struct

import numpy as np
import pytest

import conftest


def test_config_example():
    import pm_amd
    c = pm_amd.load_config(os.path.join(conftest.GOLDEN, "config.toml.example"))
    assert (c.look_from.x, c.look_from.y, c.look_from.z) == (80.0, 30.0, 0.0)
    assert abs(c.fovy - 0.87) < 1e-7
    assert c.photons_file == b"global_sphere_photons.txt"
    assert c.model_path == b"../assets/models/sphere/sphere.glb"
    assert (c.fb_width, c.fb_height, c.samples_per_pixel, c.depth) == (800, 600, 24, 30)
    assert (c.viewer_fb_width, c.viewer_fb_height) == (1920, 1080)
    assert c.casted_diffuse_photons == 1000          # "1_000" (config.toml.example:26)
    assert c.casted_caustics_photons == 500 and c.max_depth == 10
    assert pm_amd.config_key_present(c, "ray-tracer.sky_colour")


@pytest.mark.parametrize("body,needle", [
    ("[camera]\nfovy = 1\n", "not a floating"),                       # toml11 as_floating rejects ints
    ("[camera]\nlook_at = [1, 2, 3]\n", "floating"),
    ("[photon-mapper]\nmax_depth = 10.0\n", "not an integer"),
    ("[camera\nfovy = 1.0\n", "Parsing failed"),
    ("[data]\nmodel_path = \"x\nfoo\"\n", "Parsing failed"),
    ("[photon-mapper]\ncasted_diffuse_photons = 1__000\n", "Parsing failed"),
])
def test_config_errors(tmp_path, body, needle):
    import pm_amd
    p = tmp_path / "config.toml"
    p.write_text(body)
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.load_config(str(p))
    assert needle in str(e.value)


def test_config_missing_file(tmp_path):
    import pm_amd
    with pytest.raises(pm_amd.PMError) as e:
        pm_amd.load_config(str(tmp_path / "nope.toml"))
    assert e.value.status == pm_amd.PM_ERR_IO


def _glb_reference(path):
    """Independent numpy restatement of what assimp + extract_objects yield for
    a one-level glTF: per node T*R*S applied to POSITION, faces in index order."""
    b = open(path, "rb").read()
    jlen = struct.unpack_from("<I", b, 12)[0]
    J = json.loads(b[20:20 + jlen])
    off = 20 + jlen
    blen = struct.unpack_from("<I", b, off)[0]
    bin_ = b[off + 8: off + 8 + blen]

    def acc(i):
        a = J["accessors"][i]
        v = J["bufferViews"][a["bufferView"]]
        o = v.get("byteOffset", 0) + a.get("byteOffset", 0)
        dt = {5126: np.float32, 5125: np.uint32, 5123: np.uint16, 5121: np.uint8}[a["componentType"]]
        nc = {"SCALAR": 1, "VEC2": 2, "VEC3": 3}[a["type"]]
        return np.frombuffer(bin_, dt, a["count"] * nc, o).reshape(a["count"], nc)

    out = []
    for ni in J["scenes"][0]["nodes"]:
        n = J["nodes"][ni]
        x, y, z, w = n.get("rotation", [0, 0, 0, 1])
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        S = np.diag(n.get("scale", [1, 1, 1]))
        T = np.array(n.get("translation", [0, 0, 0]))
        for p in J["meshes"][n["mesh"]]["primitives"]:
            P = acc(p["attributes"]["POSITION"]).astype(np.float64)
            I = acc(p["indices"]).reshape(-1, 3)
            W = P @ (R @ S).T + T
            tri = W[I]                     # (T, 3, 3) world positions, face order kept
            out.append((J["materials"][p["material"]]["name"], tri))
    return out


@pytest.mark.parametrize("scene", ["cornell-box/cornell-box.glb", "sphere/sphere.glb"])
def test_glb_ingest_matches_independent_reader(scene):
    import pm_amd
    path = os.path.join(conftest.SCENES, scene)
    meshes, lights = pm_amd.load_scene_file(path)
    ref = _glb_reference(path)
    assert [m.name for m in meshes] == [r[0] for r in ref]
    for m, (_, tri) in zip(meshes, ref):
        got = m.vertices[m.indices]                       # (T, 3, 3)
        assert got.shape == tri.shape
        assert np.abs(got - tri).max() < 1e-4
        # extract_objects dedup: unique exact positions in first-occurrence order
        flat = m.vertices[m.indices].reshape(-1, 3)
        _, first = np.unique(flat, axis=0, return_index=True)
        assert len(m.vertices) == len(first)
        assert np.array_equal(m.vertices, flat[np.sort(first)])
    assert len(lights) >= 1


def test_cornell_structure(cornell):
    meshes, lights = cornell
    assert sum(len(m.indices) for m in meshes) == 58                  # SURVEY §2 assets
    assert [len(m.vertices) for m in meshes] == [4] * 5 + [8] * 4     # position dedup
    mirror = [m for m in meshes if m.name == "mirror.001"][0]
    assert mirror.material.tolist() == [1.0, 1.0, 1.0, 0.0, 1.0, 0.0, 1.0]
    assert lights == [{"pos": (5.0, 35.0, -10.0), "rgb": (1.0, 1.0, 1.0), "power": 10.0},
                      {"pos": (-5.0, 35.0, 10.0), "rgb": (1.0, 1.0, 1.0), "power": 10.0}]


def test_ingest_fallbacks(tmp_path, capfd):
    import pm_amd
    src = os.path.join(conftest.SCENES, "cornell-box")
    shutil.copy(os.path.join(src, "cornell-box.glb"), tmp_path / "box.glb")
    # missing lights.txt: the reference throws runtime_error (assetImporter.cxx:109)
    with pytest.raises(pm_amd.PMError):
        pm_amd.load_scene_file(str(tmp_path / "box.glb"))
    (tmp_path / "lights.txt").write_text("# comment\n\n1 2 3 1 1 1 5.5\n")
    # missing .mtl: every mesh gets the default white diffuse material (ior 0)
    meshes, lights = pm_amd.load_scene_file(str(tmp_path / "box.glb"))
    assert all(m.material.tolist() == [1, 1, 1, 1, 0, 0, 0] for m in meshes)
    assert lights == [{"pos": (1.0, 2.0, 3.0), "rgb": (1.0, 1.0, 1.0), "power": 5.5}]
    # partial .mtl with an invalid line: warning, other names still apply
    (tmp_path / "box.mtl").write_text("floor.001 0.1 0.2 0.3 0.5 0.5 0 1\nbroken line\n")
    meshes, _ = pm_amd.load_scene_file(str(tmp_path / "box.glb"))
    assert meshes[0].material.tolist()[:3] == pytest.approx([0.1, 0.2, 0.3])
    assert meshes[1].material.tolist() == [1, 1, 1, 1, 0, 0, 0]
    # Windows separators are accepted (the reference rewrites '/' -> '\\', §5.1-11)
    meshes2, _ = pm_amd.load_scene_file(str(tmp_path / "box.glb").replace("/", "\\"))
    assert len(meshes2) == len(meshes)
    (tmp_path / "lights.txt").write_text("1 2 three\n")
    with pytest.raises(pm_amd.PMError):
        pm_amd.load_scene_file(str(tmp_path / "box.glb"))


def test_square_light_line(tmp_path):
    """lights.txt extension of this build: 11 values = SQUARE_LIGHT (normal,
    side); 7 = point light as in the reference; anything in between is an
    invalid line (the reference's runtime_error)."""
    import pm_amd
    src = os.path.join(conftest.SCENES, "cornell-box")
    shutil.copy(os.path.join(src, "cornell-box.glb"), tmp_path / "box.glb")
    (tmp_path / "lights.txt").write_text("0 39 0 1 0.9 0.8 100 0 -1 0 5\n1 2 3 1 1 1 5.5\n")
    _, lights = pm_amd.load_scene_file(str(tmp_path / "box.glb"))
    assert lights[0] == {"pos": (0.0, 39.0, 0.0), "rgb": (1.0, pytest.approx(0.9), pytest.approx(0.8)),
                         "power": 100.0, "normal": (0.0, -1.0, 0.0), "side": 5.0}
    assert lights[1] == {"pos": (1.0, 2.0, 3.0), "rgb": (1.0, 1.0, 1.0), "power": 5.5}
    (tmp_path / "lights.txt").write_text("0 39 0 1 1 1 100 0 -1\n")
    with pytest.raises(pm_amd.PMError):
        pm_amd.load_scene_file(str(tmp_path / "box.glb"))


def test_obj_ingest(tmp_path):
    import pm_amd
    (tmp_path / "lights.txt").write_text("0 5 0 1 1 1 10\n")
    (tmp_path / "quad.obj").write_text("o Q\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nusemtl Mat\nf 1 2 3 4\n"
                                       "o T\nv 0 0 1\nv 1 0 1\nv 0 1 1\nf 5/1/1 6/2/2 -1\n")
    (tmp_path / "quad.mtl").write_text("Mat 0.5 0.5 0.5 0.9 0.1 0 1\n")
    meshes, lights = pm_amd.load_scene_file(str(tmp_path / "quad.obj"))
    assert [len(m.indices) for m in meshes] == [2, 1]
    assert [len(m.vertices) for m in meshes] == [4, 3]
    assert meshes[0].material.tolist()[:4] == pytest.approx([0.5, 0.5, 0.5, 0.9])


def test_photon_text_roundtrip(tmp_path):
    import pm_amd
    rng = np.random.default_rng(0)
    ph = np.zeros((257, 10), np.float32)
    ph[:, 0:6] = rng.uniform(-40, 40, size=(257, 6))
    ph[:, 7:10] = rng.uniform(0, 1, size=(257, 3))
    p = str(tmp_path / "photons.txt")
    pm_amd.write_alive_photons(ph, p)
    lines = open(p).read().splitlines()
    assert len(lines) == 257
    # std::fixed << setprecision(6): 9 values, pos dir color (hostCode.cu:39-45)
    exp = " ".join("%.6f" % float(v) for v in np.concatenate([ph[0, 0:6], ph[0, 7:10]]))
    assert lines[0] == exp
    back = pm_amd.read_photons_from_file(p)
    assert back.shape == ph.shape
    q = np.array([[float("%.6f" % float(v)) for v in row] for row in ph], np.float64).astype(np.float32)
    q[:, 6] = 0
    assert np.array_equal(back, q)
    assert pm_amd.read_photons_from_file(str(tmp_path / "missing.txt")).shape == (0, 10)


def test_png_writer(tmp_path):
    import pm_amd
    from PIL import Image
    rng = np.random.default_rng(1)
    rgba = rng.integers(0, 2 ** 32, size=(37, 53), dtype=np.uint64).astype(np.uint32)
    p = str(tmp_path / "o.png")
    pm_amd.write_png(p, rgba)
    im = np.array(Image.open(p))
    assert im.shape == (37, 53, 4)
    assert np.array_equal(im.reshape(37, 53 * 4).view(np.uint32).reshape(37, 53), rgba)


def _quantize_corpus():
    rng = np.random.default_rng(5)
    v = np.concatenate([
        rng.uniform(-50, 50, 200000), rng.normal(scale=1e-3, size=50000), rng.uniform(-1, 1, 50000),
        rng.uniform(-2e4, 2e4, 50000),
        # exact decimal ties at the 7th digit and their neighbours: k * 5e-7 in float
        (np.arange(-20000, 20000) * 5e-7), np.float32(np.arange(1, 4000)) / np.float32(1024),
        [0.0, -0.0, 1e-9, -1e-9, 5e-7, -5e-7, 1.5e-6, 0.0000015, 123456.789, -0.000000499, 9e8]]).astype(np.float32)
    return v


def test_quantize6_matches_text_roundtrip(tmp_path):
    """orc_quantize6 (the algorithm of pm_photons_quantize) equals the %.6f
    write + parse of writeAlivePhotons -> readPhotonsFromFile, sign of zero included."""
    import oracle
    import pm_amd
    v = _quantize_corpus()
    v = v[: len(v) // 9 * 9]
    ph = np.zeros((len(v) // 9, 10), np.float32)
    ph[:, 0:6] = v.reshape(-1, 9)[:, 0:6]
    ph[:, 7:10] = v.reshape(-1, 9)[:, 6:9]
    p = str(tmp_path / "q.txt")
    pm_amd.write_alive_photons(ph, p)
    back = pm_amd.read_photons_from_file(p)
    q = oracle.quantize6(ph)
    q[:, 6] = 0
    assert np.array_equal(back.view(np.uint32), q.view(np.uint32))


def test_binary_photon_file(tmp_path):
    import pm_amd
    rng = np.random.default_rng(6)
    ph = rng.normal(size=(1001, 10)).astype(np.float32)
    ph[:, 6] = rng.integers(0, 5, 1001).astype(np.int32).view(np.float32)
    p = str(tmp_path / "p.bin")
    pm_amd.write_photons_bin(ph, p)
    assert os.path.getsize(p) == 16 + 1001 * 40
    assert np.array_equal(pm_amd.read_photons_bin(p).view(np.uint32), ph.view(np.uint32))
    pm_amd.write_photons_bin(ph[:0], p)
    assert pm_amd.read_photons_bin(p).shape == (0, 10)
    (tmp_path / "bad.bin").write_bytes(b"NOTPHOTN" + b"\0" * 8)
    with pytest.raises(pm_amd.PMError):
        pm_amd.read_photons_bin(str(tmp_path / "bad.bin"))
