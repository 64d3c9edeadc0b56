"""Scene ingest (B1, assets::import_scene, common/src/assetImporter.cxx:16-205)
against every scene the reference ships under assets/models/ (copied as data
fixtures into tests/golden/scenes/), plus synthetic files for the cases the
shipped assets do not reach:
  - triangle / mesh / light counts of each shipped scene (58,
    15,882, 15,918, 91,226 triangles);
  - material lookup by mesh name from the custom `<stem>.mtl`
    (assetImporter.cxx:137-205), the white-diffuse default when it is missing;
  - the Wavefront-.mtl collision of one-cube/cube.obj: every
    line of the Blender .mtl fails the 8-value parse, so every mesh gets the
    default material; and the missing lights.txt throws (assetImporter.cxx:109);
  - a multi-level glTF node hierarchy, flattened BFS with transform =
    node * parent (assetImporter.cxx:33-46), which differs from the glTF
    parent * node order whenever the two do not commute;
  - a large multi-group OBJ (the PM_SPONZA_OBJ route) against a restatement of
    the importer's grouping / fan triangulation / per-mesh dedup rules;
  - malformed GLBs (cyclic nodes, negative accessor count) fail with PM_ERR_IO.
Runs on CPU (host-side ingest, no device)."""
import json
import os
import shutil
import struct

import numpy as np
import pytest

import conftest

S = conftest.SCENES
DEFAULT_MAT = [1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0]   # assetImporter.cxx:182-187


def _load(path):
    import pm_amd
    return pm_amd.load_scene_file(path)


def _mtl(path):
    """The reference's custom .mtl: `name r g b diffuse specular transmission ior`."""
    out = {}
    for line in open(path):
        if not line.strip() or line.startswith("#"):
            continue
        t = line.split()
        try:
            out[t[0]] = [float(x) for x in t[1:8]]
            assert len(out[t[0]]) == 7
        except (ValueError, AssertionError, IndexError):
            out.pop(t[0], None)
    return out


@pytest.mark.parametrize("rel,nmesh,ntri,nlight", [
    ("cornell-box/cornell-box.glb", 9, 58, 2),
    ("cornell-box/cornell-box2.glb", 9, 58, 2),
    ("sphere/sphere.glb", 6, 15882, 1),
    ("sphere/sphere2.glb", 9, 15918, 1),
    ("dragon/dragon-box.glb", 6, 91226, 1),
    ("simple-cube/cubes.glb", 2, 24, 1),
    ("simpler-cube/cube.glb", 1, 12, 1),
])
def test_reference_assets_counts_and_materials(rel, nmesh, ntri, nlight):
    path = os.path.join(S, rel)
    meshes, lights = _load(path)
    assert len(meshes) == nmesh
    assert sum(len(m.indices) for m in meshes) == ntri
    assert len(lights) == nlight
    mtl_path = os.path.splitext(path)[0] + ".mtl"
    table = _mtl(mtl_path) if os.path.exists(mtl_path) else {}
    for m in meshes:
        assert np.all(m.indices >= 0) and np.all(m.indices < len(m.vertices))
        # per-mesh exact-position dedup (assetImporter.cxx:65-73): no repeated vertex
        assert len(np.unique(m.vertices, axis=0)) == len(m.vertices)
        exp = table.get(m.name, DEFAULT_MAT)
        assert np.allclose(m.material, np.float32(exp)), (m.name, m.material, exp)
    if rel.startswith("dragon"):
        assert sorted(m.name for m in meshes) == sorted(["dragon", "floor", "roof", "left_wall", "right_wall",
                                                        "back_wall"])
        assert lights[0]["pos"] == (0.0, 30.0, 0.0) and lights[0]["power"] == 1000.0
    if rel.startswith("simple"):
        # lights.txt rgb 255 255 255 is read as given (no normalisation, assetImporter.cxx:124-126)
        assert lights[0]["rgb"] == (255.0, 255.0, 255.0)


def test_one_cube_missing_lights_throws():
    """one-cube ships no lights.txt: extract_lights throws (assetImporter.cxx:108-110)."""
    import pm_amd
    with pytest.raises(pm_amd.PMError) as e:
        _load(os.path.join(S, "one-cube", "cube.obj"))
    assert e.value.status == pm_amd.PM_ERR_IO


def test_one_cube_wavefront_mtl_collision(tmp_path):
    """cube.obj's Blender cube.mtl shares the custom .mtl's name: no line of it
    parses as `name r g b d s t ior`, so every mesh gets the default material
    (SURVEY §5.1-12)."""
    for f in ("cube.obj", "cube.mtl"):
        shutil.copy(os.path.join(S, "one-cube", f), tmp_path / f)
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 100\n")
    assert _mtl(str(tmp_path / "cube.mtl")) == {}
    meshes, lights = _load(str(tmp_path / "cube.obj"))
    nfaces = sum(1 for line in open(tmp_path / "cube.obj") if line.startswith("f "))
    assert len(meshes) == 1 and meshes[0].name == "Material.002"
    assert len(meshes[0].indices) == nfaces
    assert len(meshes[0].vertices) == 8   # every position is listed 3 times in the .obj: deduplicated per mesh
    assert np.allclose(meshes[0].material, DEFAULT_MAT)
    assert len(lights) == 1


# ---------------------------------------------------------------- synthetic glTF
def _glb(nodes, scene_nodes, positions, indices, materials=None, count_override=None):
    """Minimal glTF 2.0 binary: one mesh per (positions, indices) pair."""
    bin_ = b""
    accessors, views, meshes = [], [], []
    for i, (p, ix) in enumerate(zip(positions, indices)):
        p = np.ascontiguousarray(p, np.float32)
        ix = np.ascontiguousarray(ix, np.uint32).ravel()
        for arr, kind, ctype in ((p, "VEC3", 5126), (ix, "SCALAR", 5125)):
            views.append({"buffer": 0, "byteOffset": len(bin_), "byteLength": arr.nbytes})
            acc = {"bufferView": len(views) - 1, "componentType": ctype, "count": len(arr), "type": kind}
            if kind == "VEC3":
                acc["min"] = p.min(0).tolist()
                acc["max"] = p.max(0).tolist()
            accessors.append(acc)
            bin_ += arr.tobytes()
        if count_override is not None:
            accessors[-2]["count"] = count_override
        prim = {"attributes": {"POSITION": 2 * i}, "indices": 2 * i + 1}
        if materials:
            prim["material"] = i
        meshes.append({"primitives": [prim]})
    j = {"asset": {"version": "2.0"}, "scene": 0, "scenes": [{"nodes": scene_nodes}], "nodes": nodes,
         "meshes": meshes, "accessors": accessors, "bufferViews": views, "buffers": [{"byteLength": len(bin_)}]}
    if materials:
        j["materials"] = [{"name": n} for n in materials]
    js = json.dumps(j).encode()
    js += b" " * (-len(js) % 4)
    bin_ += b"\0" * (-len(bin_) % 4)
    total = 12 + 8 + len(js) + 8 + len(bin_)
    return (struct.pack("<III", 0x46546C67, 2, total) + struct.pack("<II", len(js), 0x4E4F534A) + js +
            struct.pack("<II", len(bin_), 0x004E4942) + bin_)


TRI = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)


def test_gltf_node_hierarchy_node_times_parent(tmp_path):
    """Two levels under the root: the reference composes node * parent
    (assetImporter.cxx:43, aiMatrix4x4 column-vector convention), i.e. the
    parent's transform is applied FIRST. Root translates by (10, 0, 0), its
    child scales by 2, the grandchild translates by (0, 5, 0): a vertex v lands
    at T_g(S_c(T_r(v))), not at the glTF T_r(S_c(T_g(v)))."""
    nodes = [{"translation": [10.0, 0.0, 0.0], "children": [1], "mesh": 0},
             {"scale": [2.0, 2.0, 2.0], "children": [2], "mesh": 1},
             {"translation": [0.0, 5.0, 0.0], "mesh": 2}]
    (tmp_path / "h.glb").write_bytes(_glb(nodes, [0], [TRI] * 3, [[0, 1, 2]] * 3, materials=["a", "b", "c"]))
    (tmp_path / "lights.txt").write_text("# x y z r g b power\n0 20 0 1 1 1 10\n")
    (tmp_path / "h.mtl").write_text("b 0.5 0.25 0.125 0.9 0.1 0.0 1.0\n")
    meshes, _ = _load(str(tmp_path / "h.glb"))
    assert [m.name for m in meshes] == ["a", "b", "c"]   # BFS order
    v = TRI.astype(np.float64)
    exp = [v + [10, 0, 0], 2 * (v + [10, 0, 0]), 2 * (v + [10, 0, 0]) + [0, 5, 0]]
    for m, e in zip(meshes, exp):
        assert np.array_equal(m.vertices, e.astype(np.float32)), (m.name, m.vertices, e)
    assert np.allclose(meshes[1].material, [0.5, 0.25, 0.125, 0.9, 0.1, 0.0, 1.0])
    assert np.allclose(meshes[0].material, DEFAULT_MAT)
    # the glTF (parent * node) order would put the grandchild elsewhere
    assert not np.array_equal(meshes[2].vertices, (2 * v + [20, 10, 0]).astype(np.float32))


def test_gltf_multiple_roots_and_dedup(tmp_path):
    """Several scene roots sit under one synthetic root (assimp glTF2), and a
    mesh's repeated positions are merged per mesh in first-occurrence order."""
    quad = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32)
    nodes = [{"mesh": 0}, {"mesh": 1, "translation": [0, 0, 3]}]
    (tmp_path / "m.glb").write_bytes(_glb(nodes, [0, 1], [quad, TRI], [np.arange(6), [0, 1, 2]]))
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n")
    meshes, _ = _load(str(tmp_path / "m.glb"))
    assert len(meshes) == 2
    assert meshes[0].vertices.tolist() == [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]]
    assert meshes[0].indices.tolist() == [[0, 1, 2], [0, 2, 3]]
    assert np.array_equal(meshes[1].vertices, TRI + np.float32([0, 0, 3]))


@pytest.mark.parametrize("bad", ["cycle", "two_parents", "negative_count", "bad_mesh"])
def test_malformed_gltf_rejected(tmp_path, bad):
    import pm_amd
    nodes = [{"mesh": 0, "children": [1]}, {"mesh": 0}]
    kw = {}
    if bad == "cycle":
        nodes[1]["children"] = [0]
    elif bad == "two_parents":
        nodes = [{"children": [1, 2]}, {"children": [2]}, {"mesh": 0}]
    elif bad == "negative_count":
        kw["count_override"] = -5
    else:
        nodes[1]["mesh"] = 0
        nodes.append({"mesh": 0})
    blob = _glb(nodes, [0], [TRI], [[0, 1, 2]], **kw)
    if bad == "bad_mesh":   # a node naming a mesh the file does not have is ignored, like a missing one
        blob = blob.replace(b'"mesh": 0}]', b'"mesh": 7}]', 1)
    (tmp_path / "x.glb").write_bytes(blob)
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n")
    if bad == "bad_mesh":
        meshes, _ = _load(str(tmp_path / "x.glb"))
        assert len(meshes) >= 1
        return
    with pytest.raises(pm_amd.PMError) as e:
        _load(str(tmp_path / "x.glb"))
    assert e.value.status == pm_amd.PM_ERR_IO


# ---------------------------------------------------------------- large multi-group OBJ
def _obj_reference_meshes(text):
    """Restatement of the OBJ rules the loader documents: a new mesh per
    (o | g | usemtl) section at its first face, faces fan-triangulated,
    negative indices relative to the end, then per-mesh position dedup."""
    V, meshes, cur, mtl = [], [], None, "DefaultMaterial"
    for line in text.splitlines():
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            V.append([np.float32(x) for x in t[1:4]])
        elif t[0] in ("o", "g"):
            cur = None
        elif t[0] == "usemtl":
            mtl, cur = t[1], None
        elif t[0] == "f":
            if cur is None:
                cur = {"name": mtl, "tris": []}
                meshes.append(cur)
            ids = []
            for tok in t[1:]:
                k = int(tok.split("/")[0])
                ids.append(k - 1 if k > 0 else len(V) + k)
            for j in range(1, len(ids) - 1):
                cur["tris"].append([V[ids[0]], V[ids[j]], V[ids[j + 1]]])
    out = []
    for m in meshes:
        verts, idx, seen = [], [], {}
        for tri in m["tris"]:
            row = []
            for p in tri:
                key = tuple(float(x) + 0.0 for x in p)   # -0.0 == +0.0, as operator==
                if key not in seen:
                    seen[key] = len(verts)
                    verts.append(p)
                row.append(seen[key])
            idx.append(row)
        out.append((m["name"], np.array(verts, np.float32).reshape(-1, 3), np.array(idx, np.int32).reshape(-1, 3)))
    return out


def test_large_multigroup_obj(tmp_path):
    rng = np.random.default_rng(4)
    lines, nv = ["# synthetic Sponza-like OBJ: many groups, materials, quads/pentagons, negative indices"], 0
    mats = [f"mat_{i}" for i in range(12)]
    for gi in range(60):
        lines.append(f"g group_{gi}" if gi % 3 else f"o object_{gi}")
        if gi % 2 == 0:
            lines.append(f"usemtl {mats[gi % len(mats)]}")
        base = nv
        pts = np.round(rng.uniform(-50, 50, size=(40, 3)), 3)
        pts[::7] = pts[1::7][: len(pts[::7])]   # repeated positions: per-mesh dedup
        for p in pts:
            lines.append("v %.3f %.3f %.3f" % tuple(p))
        nv += len(pts)
        for fi in range(25):
            n = 3 + fi % 3
            ids = rng.choice(40, size=n, replace=False) + base + 1
            toks = [str(i) if (fi + j) % 4 else str(i - nv - 1) for j, i in enumerate(ids)]   # some negative
            lines.append("f " + " ".join(f"{t}/1/1" if fi % 5 == 0 else t for t in toks))
        if gi == 30:
            lines.append("usemtl mat_3")   # a material switch inside a group starts a new mesh
            for fi in range(5):
                lines.append(f"f {base + 1} {base + 2 + fi} {base + 3 + fi}")
    text = "\n".join(lines) + "\n"
    (tmp_path / "big.obj").write_text(text)
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n0 25 5 1 0.5 0.5 20\n")
    (tmp_path / "big.mtl").write_text("".join(f"{m} {i / 12:.3f} 0.5 0.5 0.9 0.1 0.0 1.0\n" for i, m in enumerate(mats)))
    meshes, lights = _load(str(tmp_path / "big.obj"))
    ref = _obj_reference_meshes(text)
    assert len(lights) == 2
    assert len(meshes) == len(ref) > 60
    table = _mtl(str(tmp_path / "big.mtl"))
    for m, (name, v, ix) in zip(meshes, ref):
        assert m.name == name
        assert np.array_equal(m.vertices, v)
        assert np.array_equal(m.indices, ix)
        assert np.allclose(m.material, table.get(name, DEFAULT_MAT))
