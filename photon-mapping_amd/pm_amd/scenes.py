"""Deterministic "Sponza-class" procedural scene (bench workload, BASELINE config 3).

Sponza is neither in the reference nor in this container (no network), so the
bench uses this generator (SURVEY §7 'Hard parts', §8d config 3): a two-storey
atrium open towards +x (where the reference camera of config.toml.example
looks in from (80, 30, 0)), ~262k triangles in ~380 meshes: subdivided floor,
walls and roof slabs, two colonnades per storey, arches, balcony slabs with
railing posts, hanging curtains, and mirror / glass spheres (caustics).
Materials use the reference's custom .mtl semantics (albedo, diffuse,
specular, transmission, ior). Winding: surfaces face the atrium interior /
outward for closed solids, because the reference samples the diffuse lobe
around the unflipped geometric normal (helpers.h:45-47, 76-85).
If a real Sponza OBJ is provided (PM_SPONZA_OBJ) the bench uses it instead.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from . import MeshData

WALL = (0.75, 0.7, 0.6, 0.9, 0.1, 0.0, 1.0)
FLOOR = (0.5, 0.5, 0.5, 0.9, 0.1, 0.0, 1.0)
STONE = (0.8, 0.78, 0.72, 1.0, 0.0, 0.0, 1.0)
RED = (0.8, 0.15, 0.1, 1.0, 0.0, 0.0, 1.0)
GREEN = (0.15, 0.6, 0.2, 1.0, 0.0, 0.0, 1.0)
BLUE = (0.1, 0.2, 0.8, 1.0, 0.0, 0.0, 1.0)
METAL = (0.9, 0.9, 0.9, 0.3, 0.7, 0.0, 1.0)
MIRROR = (1.0, 1.0, 1.0, 0.0, 1.0, 0.0, 1.0)
GLASS = (1.0, 1.0, 1.0, 0.0, 0.1, 0.9, 1.5)


def _grid(nu: int, nv: int, fn) -> Tuple[np.ndarray, np.ndarray]:
    """Parametric surface on [0,1]^2 -> (verts, tris); fn(u, v) -> (..., 3)."""
    u, v = np.meshgrid(np.linspace(0, 1, nu + 1), np.linspace(0, 1, nv + 1), indexing="ij")
    P = fn(u, v).reshape(-1, 3)
    idx = np.arange((nu + 1) * (nv + 1)).reshape(nu + 1, nv + 1)
    a, b, c, d = idx[:-1, :-1], idx[1:, :-1], idx[1:, 1:], idx[:-1, 1:]
    t = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return P.astype(np.float32), t.astype(np.int32)


def _quad(o, eu, ev, nu, nv):
    o, eu, ev = (np.asarray(x, np.float64) for x in (o, eu, ev))
    return _grid(nu, nv, lambda u, v: o + u[..., None] * eu + v[..., None] * ev)


def _flip(mesh):
    v, t = mesh
    return v, t[:, ::-1].copy()


def _box(lo, hi, n=2):
    """Closed axis-aligned box with outward normals, each face n x n quads."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    dx, dy, dz = hi - lo
    faces = [
        _quad(lo, [0, dy, 0], [dx, 0, 0], n, n),                       # -z
        _quad([lo[0], lo[1], hi[2]], [dx, 0, 0], [0, dy, 0], n, n),    # +z
        _quad(lo, [0, 0, dz], [0, dy, 0], n, n),                       # -x
        _quad([hi[0], lo[1], lo[2]], [0, dy, 0], [0, 0, dz], n, n),    # +x
        _quad(lo, [dx, 0, 0], [0, 0, dz], n, n),                       # -y
        _quad([lo[0], hi[1], lo[2]], [0, 0, dz], [dx, 0, 0], n, n),    # +y
    ]
    return _merge(faces)


def _merge(parts):
    vs, ts, off = [], [], 0
    for v, t in parts:
        vs.append(v)
        ts.append(t + off)
        off += len(v)
    return np.concatenate(vs).astype(np.float32), np.concatenate(ts).astype(np.int32)


def _cylinder(base, radius, height, seg, rings, caps=True):
    bx, by, bz = base

    def f(u, v):
        th = 2 * np.pi * u
        return np.stack([bx + radius * np.cos(th), by + height * v, bz - radius * np.sin(th)], -1)

    parts = [_grid(seg, rings, f)]
    if caps:
        th = 2 * np.pi * np.arange(seg) / seg
        for y, up in ((by, False), (by + height, True)):
            ring = np.stack([bx + radius * np.cos(th), np.full(seg, y), bz - radius * np.sin(th)], -1)
            v = np.concatenate([[[bx, y, bz]], ring]).astype(np.float32)
            i = np.arange(seg)
            t = np.stack([np.zeros(seg, int), 1 + i, 1 + (i + 1) % seg], -1)
            if not up:
                t = t[:, ::-1]
            parts.append((v, t.astype(np.int32)))
    return _merge(parts)


def _sphere(center, radius, seg, rings):
    cx, cy, cz = center

    def f(u, v):
        th = 2 * np.pi * u
        ph = np.pi * v
        return np.stack([cx + radius * np.sin(ph) * np.cos(th), cy - radius * np.cos(ph),
                         cz - radius * np.sin(ph) * np.sin(th)], -1)

    return _grid(seg, rings, f)


def _arch(x0, x1, y0, z, thick, depth, seg):
    """Half-torus-like arch band between columns at x0..x1 (spanning in x), band in z."""
    cx, r = 0.5 * (x0 + x1), 0.5 * (x1 - x0)

    def under(u, v):  # underside of the arch (faces down/inward)
        th = np.pi * u
        return np.stack([cx - r * np.cos(th), y0 + r * np.sin(th), z - depth / 2 + depth * v], -1)

    def face(zz, sign):
        def f(u, v):
            th = np.pi * u
            rr = r + thick * v
            return np.stack([cx - rr * np.cos(th), y0 + rr * np.sin(th), np.full_like(u, zz)], -1)
        m = _grid(seg, 2, f)
        return m if sign > 0 else _flip(m)

    return _merge([_flip(_grid(seg, 4, under)), face(z + depth / 2, 1), face(z - depth / 2, -1)])


def _curtain(x, y_top, z, width, height, nu, nv, phase):
    def f(u, v):
        return np.stack([x + 0.6 * np.sin(6 * np.pi * u + phase) * (0.3 + v), y_top - height * v,
                         z - width / 2 + width * u], -1)
    return _grid(nu, nv, f)


def sponza_class() -> Tuple[List[MeshData], List[dict]]:
    meshes: List[MeshData] = []

    def add(mesh, mat, name):
        v, t = mesh
        meshes.append(MeshData(np.ascontiguousarray(v, np.float32), np.ascontiguousarray(t, np.int32),
                               np.asarray(mat, np.float32), name))

    X0, X1, Z0, Z1, H = -60.0, 60.0, -16.0, 16.0, 40.0
    # floor (faces up), roof (faces down), long walls (face inward), back wall (+x open)
    add(_quad([X0, 0, Z0], [0, 0, Z1 - Z0], [X1 - X0, 0, 0], 96, 48), FLOOR, "floor")
    add(_quad([X0, H, Z0], [X1 - X0, 0, 0], [0, 0, Z1 - Z0], 96, 48), WALL, "roof")
    add(_quad([X0, 0, Z0], [X1 - X0, 0, 0], [0, H, 0], 96, 40), WALL, "wall_south")
    add(_quad([X0, 0, Z1], [0, H, 0], [X1 - X0, 0, 0], 96, 40), WALL, "wall_north")
    add(_quad([X0, 0, Z0], [0, H, 0], [0, 0, Z1 - Z0], 48, 40), RED, "wall_west")
    # colonnades: 2 storeys x 2 rows x 12 columns
    xs = np.linspace(X0 + 8, X1 - 8, 12)
    for storey, (y0, hgt) in enumerate(((0.0, 17.0), (20.0, 14.0))):
        for zc in (Z0 + 6.0, Z1 - 6.0):
            for i, x in enumerate(xs):
                add(_cylinder((x, y0, zc), 1.1 if storey == 0 else 0.8, hgt, 48, 16), STONE,
                    f"column_{storey}_{int(zc)}_{i}")
                add(_box((x - 1.6, y0 + hgt - 0.6, zc - 1.6), (x + 1.6, y0 + hgt, zc + 1.6), 3), STONE,
                    f"capital_{storey}_{int(zc)}_{i}")
            for i in range(len(xs) - 1):
                add(_arch(xs[i] + 1.2, xs[i + 1] - 1.2, y0 + hgt, zc, 1.2, 2.0, 40), WALL,
                    f"arch_{storey}_{int(zc)}_{i}")
    # balcony slabs + railing posts along both sides at y = 20
    for zc, zi in ((Z0 + 6.0, Z0), (Z1 - 6.0, Z1)):
        add(_box((X0, 19.2, min(zc, zi)), (X1 - 4, 20.0, max(zc, zi)), 24), STONE, f"balcony_{int(zc)}")
        zr = zc + (1.5 if zc < 0 else -1.5)
        for i, x in enumerate(np.linspace(X0 + 2, X1 - 6, 56)):
            add(_cylinder((x, 20.0, zr), 0.12, 2.2, 12, 6), METAL, f"post_{int(zc)}_{i}")
        add(_box((X0, 22.1, zr - 0.15), (X1 - 6, 22.4, zr + 0.15), 8), METAL, f"rail_{int(zc)}")
    # curtains hanging from the balconies
    for j, x in enumerate(np.linspace(X0 + 10, X1 - 14, 10)):
        for zc, s in ((Z0 + 3.5, 1), (Z1 - 3.5, -1)):
            add(_curtain(x, 19.0, zc, 6.0, 12.0, 20, 30, 0.7 * j), (RED, GREEN, BLUE)[j % 3],
                f"curtain_{j}_{s}")
    # mirror and glass spheres on plinths (caustics)
    for k, x in enumerate(np.linspace(X0 + 14, X1 - 18, 6)):
        add(_box((x - 2.2, 0, -2.2), (x + 2.2, 3.0, 2.2), 2), STONE, f"plinth_{k}")
        add(_sphere((x, 6.0, 0.0), 3.0, 64, 32), GLASS if k % 2 == 0 else MIRROR, f"sphere_{k}")
    # vases along the floor
    for k, x in enumerate(np.linspace(X0 + 6, X1 - 10, 40)):
        for zc in (Z0 + 2.5, Z1 - 2.5):
            add(_cylinder((x, 0.0, zc), 0.7, 2.5, 24, 8), (METAL if k % 5 == 0 else GREEN),
                f"vase_{k}_{int(zc)}")
    lights = [{"pos": (-20.0, 34.0, 0.0), "rgb": (1.0, 1.0, 1.0), "power": 1000.0},
              {"pos": (25.0, 34.0, 0.0), "rgb": (1.0, 0.95, 0.9), "power": 1000.0}]
    return meshes, lights


def sponza_caustics() -> Tuple[List[MeshData], List[dict]]:
    """the same atrium (glass and mirror spheres on plinths)
    lit by one SQUARE_LIGHT (this build's area-light emission, pm.h) under the
    roof, facing down."""
    meshes, _ = sponza_class()
    lights = [{"pos": (0.0, 38.0, 0.0), "rgb": (1.0, 0.97, 0.92), "power": 2000.0,
               "normal": (0.0, -1.0, 0.0), "side": 12.0}]
    return meshes, lights


def scene_summary(meshes) -> dict:
    return {"meshes": len(meshes), "triangles": int(sum(len(m.indices) for m in meshes)),
            "vertices": int(sum(len(m.vertices) for m in meshes))}
