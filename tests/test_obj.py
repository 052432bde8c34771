"""OBJ/MTL ingestion (Assimp OBJ semantics as model.hpp uses them; SURVEY 8f
row 1).  Assimp itself is absent, so parity is pinned only by these
hand-built files: unshared per-corner vertices, fan triangulation (concave
quads fan from the concave corner), FlipUVs, negative indices, mesh splits at
o/g/usemtl, map_Kd texture dedup."""
import os

import numpy as np

from pnraytracing_amd import host as H
from pnraytracing_amd import obj

OBJ = """# test
mtllib t.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.2 0.5 0
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 1
o first
usemtl red
f 1/1/1 2/2/1 3/3/1 4/4/1
usemtl tex
f -5/1 -4/2 -2/4
o second
usemtl tex
f 1 2 3 5 4
"""
MTL = """newmtl red
Kd 1 0 0
newmtl tex
map_Kd -s 1 1 1 albedo.png
"""


def _write(tmp_path):
    (tmp_path / "t.obj").write_text(OBJ)
    (tmp_path / "t.mtl").write_text(MTL)
    from PIL import Image
    Image.fromarray(np.arange(5 * 3 * 3, dtype=np.uint8).reshape(3, 5, 3), "RGB").save(tmp_path / "albedo.png")
    return str(tmp_path / "t.obj")


def test_meshes_vertices_and_triangulation(tmp_path):
    ms = obj.load_obj(_write(tmp_path))
    assert [(m.object_name, m.material_name) for m in ms] == [("first", "red"), ("first", "tex"), ("second", "tex")]
    quad, tri, penta = (m.mesh for m in ms)
    assert len(quad.positions) == 4 and quad.indices.tolist() == [0, 1, 2, 0, 2, 3]
    assert np.allclose(quad.texcoords[:, 1], [1, 1, 0, 0])            # FlipUVs
    assert np.allclose(quad.normals, [[0, 0, 1]] * 4)
    assert len(tri.positions) == 3 and np.allclose(tri.positions[2], [0, 1, 0])   # negative indices (-2 = v4)
    assert np.allclose(tri.normals, 0)                                 # no vn on that face
    assert len(penta.positions) == 5 and penta.indices.tolist() == [0, 1, 2, 0, 2, 3, 0, 3, 4]
    assert ms[1].diffuse_texture.endswith("albedo.png") and ms[0].diffuse_texture is None


def test_concave_quad_fans_from_concave_corner(tmp_path):
    (tmp_path / "c.obj").write_text("v 0 0 0\nv 2 0 0\nv 0.5 0.5 0\nv 0 2 0\nf 1 2 3 4\n")
    m = obj.load_obj(str(tmp_path / "c.obj"))[0].mesh
    assert m.indices.tolist() == [2, 3, 0, 2, 0, 1]


def test_add_obj_texture_ids(tmp_path):
    path = _write(tmp_path)
    sb = H.SceneBuilder()
    table = obj.TextureTable()
    obj.add_obj(sb, path, [H.scale(2.0)], H.Material(), "t", table)
    obj.add_obj(sb, path, [H.translate(0, 0, -1)], H.Material(), "t2", table)
    assert len(table.textures) == 1 and table.textures[0][1:] == (5, 3, 3)
    p = sb.build()
    tex = p.triangles[:, 4].astype(int)
    assert sorted(set(tex.tolist())) == [-1, 0]
    assert len(p.triangles) == 2 * (2 + 1 + 3)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_reference_mtl_files():
    """The reference's own MTL files (model/marry/Marry.mtl, model/floor/floor.mtl,
    committed under tests/golden as data): Blender's UTF-8 material names and
    map_Kd resolved next to the MTL file (model.hpp:57-77 loads it from there)."""
    m = obj._parse_mtl(os.path.join(GOLDEN, "Marry.mtl"))
    assert list(m) == ["MC003_Kozakura_Mari", "材质"]
    assert m["MC003_Kozakura_Mari"] == os.path.join(GOLDEN, "MC003_Kozakura_Mari.png") and m["材质"] is None
    assert obj._parse_mtl(os.path.join(GOLDEN, "floor.mtl")) == {"None": None}


def test_usemtl_utf8_names_split_meshes(tmp_path):
    import shutil
    shutil.copy(os.path.join(GOLDEN, "Marry.mtl"), tmp_path / "Marry.mtl")
    text = ("mtllib Marry.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\no Mari\nusemtl MC003_Kozakura_Mari\n"
            "f 1 2 3\nusemtl 材质\nf 2 4 3\nusemtl 材质\nf 1 2 4\n")
    (tmp_path / "m.obj").write_text(text, encoding="utf-8")
    ms = obj.load_obj(str(tmp_path / "m.obj"))
    assert [(x.material_name, len(x.mesh.indices) // 3) for x in ms] == [("MC003_Kozakura_Mari", 1), ("材质", 2)]
    assert ms[0].diffuse_texture == str(tmp_path / "MC003_Kozakura_Mari.png") and ms[1].diffuse_texture is None


def _teapot_scene(via_obj_dir=None):
    """C4's geometry (teapot + floor + area light), its meshes either built
    procedurally or written to OBJ files and loaded back through load_obj."""
    sb = H.SceneBuilder()
    meshes = [H.mesh_teapot(), H.mesh_quad(27.5), H.mesh_quad(27.5)]
    if via_obj_dir is not None:
        for k, m in enumerate(meshes):
            p = os.path.join(via_obj_dir, f"m{k}.obj")
            obj.write_obj(p, [m])
            meshes[k] = [x.mesh for x in obj.load_obj(p)]
    sb.add_model(meshes[0], [H.scale(0.2)], H.Material(baseColor=(0.6, 0.7, 0.2), metallic=0.7, roughness=0.3), "teapot")
    sb.add_model(meshes[1], [H.scale(1.0)], H.Material(baseColor=(0.73, 0.73, 0.73), metallic=0.2, roughness=0.85),
                 "floor")
    sb.add_model(meshes[2], [H.translate(1.5, 3.0, 1.0), H.rotate(180.0, 0, 0, 1), H.scale(0.02)],
                 H.Material(baseColor=(0.73, 0.73, 0.73), emssive=(8.0, 8.0, 8.0)), "area_light")
    return sb.build()


def test_obj_round_trip_same_triangles_and_bvh(tmp_path):
    """Meshes written as OBJ and read back (unshared per-corner vertices, as
    Assimp builds them) give the same triangles, BVH, light list and materials
    as the procedural meshes; only the vertex array is unshared."""
    a, b = _teapot_scene(), _teapot_scene(str(tmp_path))
    for name in ("nodes", "lights", "materials"):
        x, y = getattr(a, name), getattr(b, name)
        assert x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32)), name
    ta, tb = a.triangles.reshape(-1, 6), b.triangles.reshape(-1, 6)
    va, vb = a.vertices.reshape(-1, 15), b.vertices.reshape(-1, 15)
    assert len(ta) == len(tb) and len(vb) == 3 * len(tb)
    for k in range(3):       # corner k of every triangle: same position and normal (cols 0-5)
        pa, pb = va[ta[:, k].astype(np.int64), :6], vb[tb[:, k].astype(np.int64), :6]
        assert np.array_equal(pa.view(np.uint32), pb.view(np.uint32))


def test_obj_round_trip_texcoords(tmp_path):
    """write_obj -> load_obj on a mesh with non-trivial texcoords: positions,
    normals and u exactly; v (flipped by FlipUVs on the way in and back) within
    2^-24, exactly for v in [0.5, 1]."""
    rng = np.random.default_rng(5)
    m = H.mesh_displaced_sphere(12, 8, 1.0, (0.0, 0.0, 0.0), 0.05, 7)
    uv = rng.random((len(m.positions), 2)).astype(np.float32)
    uv[:4] = [[0.0, 0.0], [1.0, 1.0], [0.1, 0.5], [0.75, 1e-9]]
    m = H.Mesh(m.positions, m.normals, uv, m.indices)
    p = str(tmp_path / "uv.obj")
    obj.write_obj(p, [m])
    back = obj.load_obj(p)[0].mesh
    idx = np.asarray(m.indices, np.int64)
    got = np.asarray(back.texcoords, np.float32)          # one vertex per face corner, in face order
    want = uv[idx]
    assert np.array_equal(got[:, 0].view(np.uint32), want[:, 0].view(np.uint32))
    assert np.max(np.abs(got[:, 1].astype(np.float64) - want[:, 1])) <= 2.0 ** -24
    hi = want[:, 1] >= 0.5
    assert np.array_equal(got[hi, 1].view(np.uint32), want[hi, 1].view(np.uint32))
    assert np.array_equal(np.asarray(back.positions, np.float32).view(np.uint32),
                          np.asarray(m.positions, np.float32)[idx].view(np.uint32))
