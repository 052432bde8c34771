"""OBJ/MTL ingestion (Assimp OBJ semantics as model.hpp uses them; SURVEY 8f
row 1).  Assimp itself is absent, so parity is pinned only by these
hand-built files: unshared per-corner vertices, fan triangulation (concave
quads fan from the concave corner), FlipUVs, negative indices, mesh splits at
o/g/usemtl, map_Kd texture dedup."""
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
