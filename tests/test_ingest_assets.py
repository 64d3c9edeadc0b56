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


# ---------------------------------------------------------------- FBX
def test_fbx_cornell_matches_glb():
    """assets/models/cornell-box/cornell-box.fbx (binary FBX 7400, the reference
    reaches it through assimp, assetImporter.cxx:18-21) is the Cornell box of
    cornell-box.glb exported at 100x: the same 9 meshes in the same order, the
    same 58 triangles, each mesh's vertices within 1e-4 of the
    GLB's after the 1/100 scale, the same triangles as position triples. The
    FBX material names (floor, ..., "Right wall") are not the custom .mtl's
    (floor.001, ...), so every mesh gets the white default, as the reference's
    name lookup (assetImporter.cxx:191-204) would. Parity unpinned (assimp
    cannot run here): the GLB is the check."""
    f_meshes, f_lights = _load(os.path.join(S, "cornell-box", "cornell-box.fbx"))
    g_meshes, g_lights = _load(os.path.join(S, "cornell-box", "cornell-box.glb"))
    assert len(f_meshes) == len(g_meshes) == 9
    assert sum(len(m.indices) for m in f_meshes) == 58
    assert len(f_lights) == len(g_lights)
    assert [m.name for m in f_meshes] == ["floor", "left_wall", "back_wall", "Right wall", "roof", "pink_cube",
                                          "mirror", "glass", "white_cube"]
    for fm, gm in zip(f_meshes, g_meshes):
        assert gm.name.startswith(fm.name.lower().replace(" ", "_")), (fm.name, gm.name)
        assert fm.vertices.shape == gm.vertices.shape and fm.indices.shape == gm.indices.shape
        fv = fm.vertices.astype(np.float64) / 100.0
        gv = gm.vertices.astype(np.float64)
        d = np.sqrt(((fv[:, None, :] - gv[None, :, :]) ** 2).sum(-1))
        assert d.min(0).max() < 1e-4 and d.min(1).max() < 1e-4, fm.name
        tri = lambda v, idx: sorted(tuple(sorted(tuple(np.round(v[i], 2)) for i in t)) for t in idx)
        assert tri(fv, fm.indices) == tri(gv, gm.indices), fm.name
        assert np.allclose(fm.material, DEFAULT_MAT)


def _fbx_node(name, props=(), kids=()):
    """One FBX 7400 record (32-bit offsets) at offset 0; kids are pre-encoded
    with relative offsets fixed up by _fbx_file."""
    return (name, list(props), list(kids))


def _fbx_encode(node, offset):
    name, props, kids = node
    pb = b""
    for p in props:
        if isinstance(p, bool):
            pb += b"C" + struct.pack("<?", p)
        elif isinstance(p, int):
            pb += b"L" + struct.pack("<q", p)
        elif isinstance(p, float):
            pb += b"D" + struct.pack("<d", p)
        elif isinstance(p, str):
            s = p.encode().replace(b"::", b"\x00\x01")
            pb += b"S" + struct.pack("<I", len(s)) + s
        elif isinstance(p, tuple) and p[0] == "d":
            raw = struct.pack("<%dd" % len(p[1]), *p[1])
            pb += b"d" + struct.pack("<III", len(p[1]), 0, len(raw)) + raw
        elif isinstance(p, tuple) and p[0] == "i":
            raw = struct.pack("<%di" % len(p[1]), *p[1])
            pb += b"i" + struct.pack("<III", len(p[1]), 0, len(raw)) + raw
        else:
            raise ValueError(p)
    nm = name.encode()
    head = 12 + 1 + len(nm)
    body = b""
    pos = offset + head + len(pb)
    for k in kids:
        kb = _fbx_encode(k, pos)
        body += kb
        pos += len(kb)
    if kids:
        body += b"\x00" * 13   # nested end marker
    end = offset + head + len(pb) + len(body)
    return struct.pack("<III", end, len(props), len(pb)) + bytes([len(nm)]) + nm + pb + body


def _fbx_file(top):
    out = b"Kaydara FBX Binary  \x00\x1a\x00" + struct.pack("<I", 7400)
    for n in top:
        out += _fbx_encode(n, len(out))
    return out + b"\x00" * 13


def _p70(**vals):
    return _fbx_node("Properties70", [], [_fbx_node("P", [k, k, "", "A", *map(float, v)]) for k, v in vals.items()])


def _model(mid, name, **trs):
    return _fbx_node("Model", [mid, f"{name}::Model", "Mesh"], [_p70(**trs)])


def _geometry(gid, name, verts, polys, mat=None):
    idx = []
    for p in polys:
        idx += list(p[:-1]) + [~p[-1]]
    kids = [_fbx_node("Vertices", [("d", [float(x) for x in np.ravel(verts)])]),
            _fbx_node("PolygonVertexIndex", [("i", idx)])]
    if mat is not None:
        kids.append(_fbx_node("LayerElementMaterial", [0], [
            _fbx_node("MappingInformationType", ["ByPolygon" if len(mat) > 1 else "AllSame"]),
            _fbx_node("Materials", [("i", list(mat))])]))
    return _fbx_node("Geometry", [gid, f"{name}::Geometry", "Mesh"], kids)


def test_fbx_hierarchy_materials_and_quads(tmp_path):
    """A synthetic binary FBX: a root model translated by (10, 0, 0) with a
    child scaled by 2 (the reference composes node * parent,
    assetImporter.cxx:43: the parent's transform applies first), a rotation
    about z by 90 degrees (Euler XYZ, R = Rz Ry Rx), a two-material geometry
    split into one mesh per material in first-appearance order, a concave quad
    split at its reflex corner (assimp Triangulate) and a pentagon fan."""
    sq = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float64)
    dart = np.array([[0, 0, 0], [2, 1, 0], [0, 2, 0], [0.5, 1, 0]], np.float64)   # reflex corner at 3
    pent = np.array([[0, 0, 0], [2, 0, 0], [3, 1, 0], [1, 2, 0], [-1, 1, 0]], np.float64)
    two = np.concatenate([sq, sq + [0, 0, 1]])
    objects = _fbx_node("Objects", [], [
        _geometry(11, "g_sq", sq, [[0, 1, 2, 3]]),
        _geometry(12, "g_two", two, [[0, 1, 2], [4, 5, 6], [0, 2, 3]], mat=[1, 0, 1]),
        _geometry(13, "g_dart", dart, [[0, 1, 2, 3]]),
        _geometry(14, "g_pent", pent, [[0, 1, 2, 3, 4]]),
        _model(21, "root", **{"Lcl Translation": (10, 0, 0)}),
        _model(22, "child", **{"Lcl Scaling": (2, 2, 2)}),
        _model(23, "rot", **{"Lcl Rotation": (0, 0, 90)}),
        _model(24, "shapes"),
        _fbx_node("Material", [31, "red::Material", ""]),
        _fbx_node("Material", [32, "blue::Material", ""]),
    ])
    C = lambda a, b: _fbx_node("C", ["OO", a, b])
    conns = _fbx_node("Connections", [], [C(21, 0), C(23, 0), C(24, 0), C(22, 21), C(11, 21), C(12, 22),
                                          C(31, 22), C(32, 22), C(11, 23), C(13, 24), C(14, 24)])
    (tmp_path / "s.fbx").write_bytes(_fbx_file([_fbx_node("FBXHeaderExtension", [], [_fbx_node("FBXVersion", [7400])]),
                                                objects, conns]))
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n")
    (tmp_path / "s.mtl").write_text("blue 0.1 0.2 0.9 1.0 0.0 0.0 1.0\n")
    meshes, _ = _load(str(tmp_path / "s.fbx"))
    # BFS: root's mesh, rot's mesh, shapes' two meshes, then child's two (material 1 = blue first)
    assert [m.name for m in meshes] == ["DefaultMaterial", "DefaultMaterial", "DefaultMaterial", "DefaultMaterial",
                                        "blue", "red"]
    f32 = lambda a: np.asarray(a, np.float32)
    assert np.array_equal(meshes[0].vertices, f32(sq + [10, 0, 0]))
    assert meshes[0].indices.tolist() == [[0, 1, 2], [0, 2, 3]]
    assert np.allclose(meshes[1].vertices, f32(np.stack([-sq[:, 1], sq[:, 0], sq[:, 2]], 1)), atol=1e-6)
    # concave quad: start at the reflex corner 3 -> (3, 0, 1), (3, 1, 2)
    dv = meshes[2].vertices
    tris = [[tuple(dv[i]) for i in t] for t in meshes[2].indices]
    assert tris == [[tuple(f32(dart[3])), tuple(f32(dart[0])), tuple(f32(dart[1]))],
                    [tuple(f32(dart[3])), tuple(f32(dart[1])), tuple(f32(dart[2]))]]
    assert len(meshes[3].indices) == 3   # pentagon fan
    # child: node * parent -> scale first, then the parent's translation... applied as S(T(v))
    blue_tris = 2 * (two[[0, 1, 2, 0, 2, 3]] + [10, 0, 0])
    assert np.array_equal(np.sort(meshes[4].vertices, 0), np.sort(f32(np.unique(blue_tris, axis=0)), 0))
    assert np.allclose(meshes[4].material, [0.1, 0.2, 0.9, 1.0, 0.0, 0.0, 1.0])
    assert np.allclose(meshes[5].material, DEFAULT_MAT)
    assert np.array_equal(np.sort(meshes[5].vertices, 0), np.sort(f32(2 * (two[4:7] + [10, 0, 0])), 0))


@pytest.mark.parametrize("bad", ["magic", "truncated", "array_len", "pivot", "cycle", "two_parents", "zlib_bomb"])
def test_malformed_fbx_rejected(tmp_path, bad):
    """PM_ERR_IO, never a crash: bad magic, truncation, array lengths, pivots,
    a model hierarchy that is not a tree (a cycle, a model with two parents;
    load_glb rejects the same), a compressed array whose header asks for far
    more than zlib can expand its payload to."""
    import pm_amd
    objects = _fbx_node("Objects", [], [_geometry(11, "g", TRI.astype(np.float64), [[0, 1, 2]]),
                                        _model(21, "m", **({"RotationPivot": (1, 0, 0)} if bad == "pivot" else {})),
                                        _model(22, "k"), _model(23, "j")])
    C = lambda a, b: _fbx_node("C", ["OO", a, b])
    extra = {"cycle": [C(22, 21), C(23, 22), C(22, 23)], "two_parents": [C(22, 21), C(23, 21), C(23, 22)]}
    conns = _fbx_node("Connections", [], [C(21, 0), C(11, 21)] + extra.get(bad, []))
    blob = _fbx_file([objects, conns])
    if bad == "zlib_bomb":   # Vertices array: enc 1, 2^28 doubles claimed from its few payload bytes
        i = blob.index(b"Vertices") + len(b"Vertices") + 1
        n, enc, clen = struct.unpack("<III", blob[i:i + 12])
        blob = blob[:i] + struct.pack("<III", 1 << 28, 1, clen) + blob[i + 12:]
    if bad == "magic":
        blob = b"Kaydara FBX Ascii   " + blob[20:]
    elif bad == "truncated":
        blob = blob[: len(blob) // 2]
    elif bad == "array_len":
        i = blob.index(b"Vertices") + len(b"Vertices") + 1
        blob = blob[:i] + struct.pack("<I", 1000) + blob[i + 4:]
    (tmp_path / "x.fbx").write_bytes(blob)
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n")
    with pytest.raises(pm_amd.PMError) as e:
        _load(str(tmp_path / "x.fbx"))
    assert e.value.status == pm_amd.PM_ERR_IO


def test_fbx_repeated_parent_connection_is_one_edge(tmp_path):
    """The same child -> parent OO connection listed twice is still a tree
    (ADVICE r4): loaded as if listed once, not rejected as 'two parents'."""
    objects = _fbx_node("Objects", [], [_geometry(11, "g", TRI.astype(np.float64), [[0, 1, 2]]),
                                        _model(21, "m", **{"Lcl Translation": (5, 0, 0)}), _model(22, "k")])
    C = lambda a, b: _fbx_node("C", ["OO", a, b])
    once = [C(21, 0), C(22, 21), C(11, 22)]
    out = {}
    for name, conns in (("once", once), ("twice", once[:2] + [C(22, 21)] + once[2:])):
        (tmp_path / f"{name}.fbx").write_bytes(_fbx_file([objects, _fbx_node("Connections", [], conns)]))
        (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n")
        out[name], _ = _load(str(tmp_path / f"{name}.fbx"))
    assert len(out["twice"]) == len(out["once"]) == 1
    assert np.array_equal(out["twice"][0].vertices, out["once"][0].vertices)
    assert np.array_equal(out["once"][0].vertices, (TRI + [5, 0, 0]).astype(np.float32))


def test_fbx_short_material_record_falls_back(tmp_path):
    """A Material record without its name property: the mesh takes
    DefaultMaterial instead of reading past the record."""
    objects = _fbx_node("Objects", [], [_geometry(11, "g", TRI.astype(np.float64), [[0, 1, 2]], mat=[0]),
                                        _model(21, "m"), _fbx_node("Material", [31])])
    C = lambda a, b: _fbx_node("C", ["OO", a, b])
    conns = _fbx_node("Connections", [], [C(21, 0), C(11, 21), C(31, 21)])
    (tmp_path / "x.fbx").write_bytes(_fbx_file([objects, conns]))
    (tmp_path / "lights.txt").write_text("0 20 0 1 1 1 10\n")
    meshes, _ = _load(str(tmp_path / "x.fbx"))
    assert [m.name for m in meshes] == ["DefaultMaterial"]
    assert np.allclose(meshes[0].material, DEFAULT_MAT)
