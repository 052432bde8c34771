"""Deterministic ray sets for pinning the oracle's intersection arithmetic to
the reference's own CPU code (oracle/ref/isect_driver.cpp: BVH::Intersect /
IntersectP, TriangleIntersect(P), BoundIntersect of /root/reference/include).

TEST INFRASTRUCTURE.  Used by tests/golden/make_isect_golden.py (which runs the
reference build and commits hashes + sampled records) and by
tests/test_isect_pin.py (which runs the oracle on the same rays).  Every array
is float32 numpy arithmetic from one seeded PCG64 stream, so both sides see
identical bits.

Ray families (n x 7 floats: origin, dir, tMax):
  camera   eye -> random image positions (normalised dir), tMax 1e7 (GLSL FLOAT_MAX)
  bounce   random points on random triangles + N*1e-4, random unit dirs, tMax 1e7
  shadow   surface points -> light-triangle points, UNnormalised dir, tMax 1-1e-4
  axis     dirs with exact zero components (the watertight test's permutation
           branch, infinite slab reciprocals), signed zeros
  plane    origins on the Cornell walls' planes with in-plane dirs (0*inf = NaN slabs)
  box      origins on random node boxes' faces / corners, random dirs
  wide     origins in a box around the scene, random dirs, random tMax in [0.05, 20]
"""
from __future__ import annotations

import numpy as np

F = np.float32
FAMILIES = ("camera", "bounce", "shadow", "axis", "plane", "box", "wide")


def _unit(rng, n):
    v = rng.standard_normal((n, 3)).astype(F)
    return (v / np.sqrt((v * v).sum(1, dtype=F))[:, None]).astype(F)


def _tri_points(rng, p, tris, n, edge_frac=0.2):
    """Random points on random triangles (barycentrics in float32); a share lie
    exactly on edges / vertices."""
    t = rng.integers(0, len(tris), n)
    ids = tris[t, :3].astype(np.int64)
    u = rng.random((n, 2)).astype(F)
    s = np.sqrt(u[:, 0]).astype(F)
    b0 = (F(1) - s).astype(F)
    b1 = (u[:, 1] * s).astype(F)
    k = rng.random(n) < edge_frac
    b1[k & (rng.random(n) < 0.5)] = F(0)
    b0[k & (rng.random(n) < 0.3)] = F(1)
    b1[b0 == F(1)] = F(0)
    b2 = (F(1) - b0 - b1).astype(F)
    pos = p[ids[:, 0]] * b0[:, None] + p[ids[:, 1]] * b1[:, None] + p[ids[:, 2]] * b2[:, None]
    return pos.astype(F), t


def _face_normals(p, tris, t):
    ids = tris[t, :3].astype(np.int64)
    e1 = (p[ids[:, 1]] - p[ids[:, 0]]).astype(F)
    e2 = (p[ids[:, 2]] - p[ids[:, 0]]).astype(F)
    n = np.cross(e1, e2).astype(F)
    ln = np.sqrt((n * n).sum(1, dtype=F)).astype(F)
    ln[ln == 0] = F(1)
    return (n / ln[:, None]).astype(F)


def make_rays(packed, camera, family: str, n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng([seed, FAMILIES.index(family)])
    p = np.ascontiguousarray(packed.vertices[:, 0:3], F)
    tris = packed.triangles
    nodes = packed.nodes
    lo = nodes[0, 0:3].astype(F)
    hi = nodes[0, 3:6].astype(F)
    out = np.zeros((n, 7), F)
    if family == "camera":
        cam = np.asarray(camera, F).reshape(4, 3)
        s = rng.random(n).astype(F)
        t = rng.random(n).astype(F)
        d = (cam[1] + s[:, None] * cam[2] + t[:, None] * cam[3] - cam[0]).astype(F)
        d = (d / np.sqrt((d * d).sum(1, dtype=F))[:, None]).astype(F)
        out[:, 0:3] = cam[0]
        out[:, 3:6] = d
        out[:, 6] = F(1e7)
    elif family == "bounce":
        pos, t = _tri_points(rng, p, tris, n)
        nn = _face_normals(p, tris, t)
        d = _unit(rng, n)
        flip = (d * nn).sum(1, dtype=F) < 0
        nn[flip] = -nn[flip]                          # offset to the side the ray leaves
        out[:, 0:3] = pos + nn * F(1e-4)
        out[:, 3:6] = d
        out[:, 6] = F(1e7)
    elif family == "shadow":
        pos, t = _tri_points(rng, p, tris, n)
        nn = _face_normals(p, tris, t)
        if len(packed.lights):
            li = packed.lights[rng.integers(0, len(packed.lights), n), 0].astype(np.int64)
        else:
            li = rng.integers(0, len(tris), n)
        tgt, _ = _tri_points(rng, p, tris[li], n, edge_frac=0.0)
        o = (pos + nn * F(1e-4)).astype(F)
        out[:, 0:3] = o
        out[:, 3:6] = (tgt - o).astype(F)             # unnormalised, ray_tracing.comp:886-889
        out[:, 6] = F(1) - F(1e-4)
    elif family == "axis":
        o = (lo + rng.random((n, 3)).astype(F) * (hi - lo)).astype(F)
        d = _unit(rng, n)
        which = rng.integers(0, 7, n)
        for k, mask in enumerate([(0,), (1,), (2,), (0, 1), (0, 2), (1, 2), ()]):
            for a in mask:
                d[which == k, a] = F(0)
        neg0 = rng.random((n, 3)) < 0.5
        d[(d == 0) & neg0] = F(-0.0)
        bad = ~np.any(d != 0, axis=1)
        d[bad, 2] = F(1)
        out[:, 0:3] = o
        out[:, 3:6] = d
        out[:, 6] = np.where(rng.random(n) < 0.5, F(1e7), (rng.random(n) * 20).astype(F))
    elif family == "plane":
        # Cornell walls: y = 0 floor, z = -2.75 front, x = +-2.75 sides, y = 5.54 ceiling
        planes = [(1, F(0)), (2, F(-2.75)), (0, F(2.75)), (0, F(-2.75)), (1, F(5.54))]
        k = rng.integers(0, len(planes), n)
        o = (lo + rng.random((n, 3)).astype(F) * (hi - lo)).astype(F)
        d = _unit(rng, n)
        for j, (ax, v) in enumerate(planes):
            o[k == j, ax] = v
            d[k == j, ax] = F(0)
        out[:, 0:3] = o
        out[:, 3:6] = d
        out[:, 6] = F(1e7)
    elif family == "box":
        ni = rng.integers(0, len(nodes), n)
        blo = nodes[ni, 0:3].astype(F)
        bhi = nodes[ni, 3:6].astype(F)
        o = (blo + rng.random((n, 3)).astype(F) * (bhi - blo)).astype(F)
        ax = rng.integers(0, 3, n)
        side = rng.random(n) < 0.5
        r = np.arange(n)
        o[r, ax] = np.where(side, blo[r, ax], bhi[r, ax])
        corner = rng.random(n) < 0.1
        o[corner] = np.where(rng.random((int(corner.sum()), 3)) < 0.5, blo[corner], bhi[corner])
        out[:, 0:3] = o
        out[:, 3:6] = _unit(rng, n)
        out[:, 6] = np.where(rng.random(n) < 0.5, F(1e7), (rng.random(n) * 5).astype(F))
    elif family == "wide":
        c = ((lo + hi) * F(0.5)).astype(F)
        ext = (hi - lo).astype(F)
        o = (c + (rng.random((n, 3)).astype(F) - F(0.5)) * ext * F(1.5)).astype(F)
        out[:, 0:3] = o
        out[:, 3:6] = _unit(rng, n)
        out[:, 6] = (F(0.05) + rng.random(n).astype(F) * F(20)).astype(F)
    else:
        raise ValueError(family)
    return out


def make_pairs(packed, n: int, seed: int, what: str):
    """(rays, idx) for the per-primitive kinds: rays aimed at triangle idx[i]
    (what='tri') or at the box of node idx[i] (what='box'); a share of them
    aimed at edges and vertices / faces and corners, a share at random."""
    rng = np.random.default_rng([seed, 100 + (what == "box")])
    p = np.ascontiguousarray(packed.vertices[:, 0:3], F)
    tris = packed.triangles
    nodes = packed.nodes
    lo = nodes[0, 0:3].astype(F)
    hi = nodes[0, 3:6].astype(F)
    c = ((lo + hi) * F(0.5)).astype(F)
    ext = (hi - lo).astype(F)
    o = (c + (rng.random((n, 3)).astype(F) - F(0.5)) * ext * F(1.2)).astype(F)
    if what == "tri":
        tgt, idx = _tri_points(rng, p, tris, n, edge_frac=0.35)
    else:
        idx = rng.integers(0, len(nodes), n)
        blo = nodes[idx, 0:3].astype(F)
        bhi = nodes[idx, 3:6].astype(F)
        tgt = (blo + rng.random((n, 3)).astype(F) * (bhi - blo)).astype(F)
        face = rng.random(n) < 0.4
        ax = rng.integers(0, 3, n)
        r = np.arange(n)
        tgt[face, ax[face]] = np.where(rng.random(int(face.sum())) < 0.5, blo[face, ax[face]], bhi[face, ax[face]])
    d = (tgt - o).astype(F)
    norm = rng.random(n) < 0.5
    ln = np.sqrt((d * d).sum(1, dtype=F)).astype(F)
    ln[ln == 0] = F(1)
    d[norm] = (d[norm] / ln[norm, None]).astype(F)
    rand = rng.random(n) < 0.2
    d[rand] = _unit(rng, int(rand.sum()))
    zero = rng.random(n) < 0.05
    d[zero, rng.integers(0, 3, int(zero.sum()))] = F(0)
    rays = np.zeros((n, 7), F)
    rays[:, 0:3] = o
    rays[:, 3:6] = d
    u = rng.random(n)
    rays[:, 6] = np.where(u < 0.5, F(1e7), np.where(u < 0.75, F(1) - F(1e-4), (rng.random(n) * 3).astype(F)))
    return rays, idx.astype(np.int32)
