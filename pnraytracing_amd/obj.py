"""Wavefront OBJ/MTL ingestion with the semantics of the reference's import path
(SURVEY 8f row 1): ``Model`` (model.hpp:20-78) calls Assimp's OBJ importer with
``aiProcess_Triangulate | aiProcess_FlipUVs | aiProcess_CalcTangentSpace`` and
keeps, per aiMesh, the vertices, the face indices and the first diffuse
texture (``texturePathToId`` dedup, ``stbi_load(path, .., 0)``).

Restated here (Assimp is not in the reference tree; parity of this module is
pinned only by the tests' hand-built files, see tests/test_obj.py):

* a new mesh starts at every ``o``/``g`` and at every ``usemtl`` that changes
  the material of a mesh that already has faces (ObjFileParser's
  needsNewMesh); meshes are emitted in file order, as ``processNode`` visits
  the objects;
* vertices are NOT shared: every face corner becomes its own vertex
  (ObjFileImporter::createVertexArray), so a mesh's vertex count is the number
  of face corners;
* polygons are triangulated as a fan (aiProcess_Triangulate); a quad whose
  corner ``k`` is concave fans from ``k``, as Assimp's quad special case does;
* ``vt`` v is flipped to 1 - v (aiProcess_FlipUVs); missing ``vt``/``vn`` give
  zero texcoords / zero normals (ModelOutput then falls back to face normals
  in the shader, :338-348);
* tangents/bitangents (CalcTangentSpace) are left zero: ray_tracing.comp never
  reads them.
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np

from .host import Mesh


@dataclasses.dataclass
class ObjMesh:
    mesh: Mesh
    object_name: str
    material_name: str
    diffuse_texture: str | None      # absolute path of map_Kd, if any


def _parse_mtl(path: str) -> dict:
    out, cur = {}, None
    if not os.path.exists(path):
        return out
    base = os.path.dirname(path)
    with open(path, "r", encoding="utf-8", errors="replace") as f:      # Blender writes UTF-8 names
        for line in f:
            t = line.split()
            if not t or t[0].startswith("#"):
                continue
            if t[0] == "newmtl":
                cur = " ".join(t[1:])
                out[cur] = None
            elif t[0] == "map_Kd" and cur is not None and len(t) > 1:
                # options (-s, -o, ...) precede the file name; the name is last
                out[cur] = os.path.join(base, t[-1])
    return out


def _quad_start(P: np.ndarray) -> int:
    """Assimp TriangulateProcess, 4-gon case: fan from the concave corner if any."""
    n = np.cross(P[1] - P[0], P[2] - P[0]) + np.cross(P[2] - P[0], P[3] - P[0])
    for k in range(4):
        a, b, c = P[(k + 3) % 4], P[k], P[(k + 1) % 4]
        if np.dot(np.cross(b - a, c - b), n) < 0:
            return k
    return 0


def load_obj(path: str) -> list[ObjMesh]:
    base = os.path.dirname(os.path.abspath(path))
    V, T, N = [], [], []
    mtl = {}
    runs: list = []                # [object, material, faces (corner tuples)]
    obj_name, mat_name = "defaultobject", ""
    new_mesh = True
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        for line in f:
            t = line.split()
            if not t or t[0].startswith("#"):
                continue
            k = t[0]
            if k == "v":
                V.append([float(x) for x in t[1:4]])
            elif k == "vt":
                T.append([float(t[1]), float(t[2]) if len(t) > 2 else 0.0])
            elif k == "vn":
                N.append([float(x) for x in t[1:4]])
            elif k in ("o", "g"):
                obj_name = " ".join(t[1:]) or "default"
                new_mesh = True
            elif k == "usemtl":
                name = " ".join(t[1:])
                if name != mat_name:
                    new_mesh = True
                mat_name = name
            elif k == "mtllib":
                for name in t[1:]:
                    mtl.update(_parse_mtl(os.path.join(base, name)))
            elif k == "f":
                corners = []
                for c in t[1:]:
                    parts = (c.split("/") + ["", ""])[:3]
                    idx = []
                    for p, n in zip(parts, (len(V), len(T), len(N))):
                        if p == "":
                            idx.append(-1)
                        else:
                            i = int(p)
                            idx.append(i - 1 if i > 0 else n + i)
                    corners.append(tuple(idx))
                if new_mesh or not runs:
                    runs.append([obj_name, mat_name, []])
                    new_mesh = False
                runs[-1][2].append(corners)
    V = np.asarray(V, np.float32).reshape(-1, 3)
    T = np.asarray(T, np.float32).reshape(-1, 2)
    N = np.asarray(N, np.float32).reshape(-1, 3)
    out = []
    for oname, mname, faces in runs:
        pos, nrm, uv, idx = [], [], [], []
        for corners in faces:
            start = len(pos)
            for (vi, ti, ni) in corners:                 # one vertex per face corner
                pos.append(V[vi])
                nrm.append(N[ni] if ni >= 0 else np.zeros(3, np.float32))
                uv.append((T[ti][0], 1.0 - T[ti][1]) if ti >= 0 else (0.0, 0.0))
            m = len(corners)
            if m < 3:
                continue                                  # points / lines carry no triangles
            s = _quad_start(np.asarray(pos[start:start + 4], np.float64)) if m == 4 else 0
            for j in range(1, m - 1):
                idx += [start + s, start + (s + j) % m, start + (s + j + 1) % m]
        mesh = Mesh(np.asarray(pos, np.float32).reshape(-1, 3), np.asarray(nrm, np.float32).reshape(-1, 3),
                    np.asarray(uv, np.float32).reshape(-1, 2), np.asarray(idx, np.int32))
        out.append(ObjMesh(mesh, oname, mname, mtl.get(mname)))
    return out


class TextureTable:
    """``texturePathToId`` + ``textures`` / ``textureInfos`` (model.hpp:62-73)."""

    def __init__(self):
        self.ids: dict = {}
        self.textures: list = []           # (pixels u8, w, h, ch) as stbi_load returns them

    def id_for(self, path: str | None) -> int:
        if not path:
            return -1
        if path in self.ids:
            return self.ids[path]
        if not os.path.exists(path):
            return -1                          # "Cannot load texture": textureId stays -1
        from .scenes import load_texture
        self.ids[path] = len(self.textures)
        self.textures.append(load_texture(path))
        return self.ids[path]


def add_obj(builder, path: str, ops, material, name: str = "", textures: TextureTable | None = None) -> int:
    """``Model(path, modelMatrix, material, name)`` for an OBJ file: every mesh
    of the file with the model's material and its own diffuse texture id."""
    meshes = load_obj(path)
    textures = textures if textures is not None else TextureTable()
    tex_ids = [textures.id_for(m.diffuse_texture) for m in meshes]
    return builder.add_model([m.mesh for m in meshes], ops, material, name, texture_ids=tex_ids)


def write_obj(path: str, meshes, material_names=None, mtllib: str | None = None) -> None:
    """Write meshes as a Wavefront OBJ that :func:`load_obj` reads back to the
    same triangles: one ``o``/``usemtl`` per mesh, positions and normals as
    ``%.9g`` (float32 round-trips exactly), texcoords stored pre-flipped
    (``vt u 1-v``) for FlipUVs, faces in index order.  u round-trips exactly;
    v comes back as float32 ``1 - (1 - v)``, within 2^-24 of v (exact for v in
    [0.5, 1] and for multiples of 2^-24), since FlipUVs on the read side cannot
    be undone bit for bit for every v.  (Scene export for tests and tools; the
    reference only reads OBJ.)"""
    with open(path, "w", encoding="utf-8") as f:
        if mtllib:
            f.write(f"mtllib {mtllib}\n")
        base = 0
        for k, m in enumerate(meshes):
            f.write(f"o mesh{k}\n")
            if material_names:
                f.write(f"usemtl {material_names[k]}\n")
            P = np.asarray(m.positions, np.float32)
            Nn = np.asarray(m.normals, np.float32) if m.normals is not None else np.zeros_like(P)
            T = np.asarray(m.texcoords, np.float32) if m.texcoords is not None else np.zeros((len(P), 2), np.float32)
            for p in P:
                f.write("v %.9g %.9g %.9g\n" % tuple(float(x) for x in p))
            for t in T:
                f.write("vt %.9g %.9g\n" % (float(t[0]), float(np.float32(1.0) - t[1])))
            for n in Nn:
                f.write("vn %.9g %.9g %.9g\n" % tuple(float(x) for x in n))
            idx = np.asarray(m.indices, np.int64).reshape(-1, 3) + base + 1
            for a, b, c in idx:
                f.write(f"f {a}/{a}/{a} {b}/{b}/{b} {c}/{c}/{c}\n")
            base += len(P)

