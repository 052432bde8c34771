"""Host arrays vs the reference's own code (oracle/_ref build of BVH.hpp,
bound.hpp, triangle.hpp, camera.hpp and glm), via committed fixtures.

Pins: ModelOutput restatement, binned-SAH BuildBVH (node order, partition,
leaf ranges), the light prefix list, main.cpp packing, glm matrices and
Camera::UpdateCamera -- all bit for bit."""
import hashlib
import json
import os

import numpy as np
import pytest

from pnraytracing_amd import host as H
from pnraytracing_amd import scenes as S

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIX = json.load(open(os.path.join(GOLD, "reference_fixtures.json")))


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def test_c1_arrays_bitwise_equal_reference_build():
    ref = np.load(os.path.join(GOLD, "c1_reference_arrays.npz"))
    p = S.cornell_c1().packed
    for k in ("vertices", "triangles", "nodes", "lights"):
        np.testing.assert_array_equal(bits(getattr(p, k)), bits(ref[k]), err_msg=k)
    np.testing.assert_array_equal(bits(p.materials), bits(ref["materials"]))


def test_c1_bvh_shape_matches_survey_probe():
    # 9 nodes, BVH-order materials 3 3 0 0 1 1 2 2 4 4 5 5, root axis 1 right 8
    p = S.cornell_c1().packed
    assert len(p.nodes) == 9
    assert p.triangles[:, 3].astype(int).tolist() == [3, 3, 0, 0, 1, 1, 2, 2, 4, 4, 5, 5]
    assert p.nodes[0, 6] == 1 and p.nodes[0, 7] == 8


def test_c1_model_matrices_match_glm():
    ref = np.load(os.path.join(GOLD, "c1_reference_arrays.npz"))
    ops = [[H.scale(0.1)],
           [H.translate(0, 2.75, -2.75), H.rotate(90.0, 1, 0, 0), H.scale(0.1)],
           [H.translate(2.75, 2.75, 0), H.rotate(90.0, 0, 0, 1), H.scale(0.1)],
           [H.translate(-2.75, 2.75, 0.0), H.rotate(-90.0, 0, 0, 1), H.scale(0.1)],
           [H.translate(0, 5.54, 0), H.rotate(180.0, 0, 0, 1), H.scale(0.1)],
           [H.translate(0, 5.54, 0), H.rotate(180.0, 0, 0, 1), H.scale(0.02)]]
    for i, o in enumerate(ops):
        np.testing.assert_array_equal(bits(H.model_matrix(o)), bits(ref["matrices"][i]))


BUILDERS = {"C2": S.bunny_c2, "C3": S.marry_c3, "C4": S.teapot_c4, "C5": S.synthetic_c5}


@pytest.mark.parametrize("key", ["C2", "C3", "C4", "C5"])
def test_scene_arrays_hash_equal_reference_build(key):
    """Whole arrays (sha256) and 64 sampled rows of each: C5 is the 4.19M-triangle
    build (4,228,165 nodes) of SURVEY 8c item 1."""
    fx = FIX[key]
    cfg = BUILDERS[key](env=False)
    p = cfg.packed
    for k in ("vertices", "triangles", "nodes", "lights"):
        arr = getattr(p, k)
        assert len(arr) == fx["counts"][k], k
        for i, row in fx["samples"].get(k, {}).items():
            np.testing.assert_array_equal(bits(arr[int(i)]), bits(np.array(row, np.float32)), err_msg=f"{k}[{i}]")
        assert sha(arr) == fx["sha256"][k], k
    np.testing.assert_array_equal(bits(cfg.camera), bits(np.array(fx["camera"], np.float32)))


@pytest.mark.parametrize("res", ["256x256", "512x512", "1920x1080", "3840x2160"])
def test_camera_kat(res):
    w, h = map(int, res.split("x"))
    cam = H.camera_update((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, np.float32(w) / np.float32(h))
    np.testing.assert_array_equal(bits(cam), bits(np.array(FIX["camera_kat"][res], np.float32)))


def test_camera_survey_values():
    # SURVEY.md 8c camera KATs
    c = H.camera_update((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, 1.0)
    assert np.float32(c[1, 0]) == np.float32(-0.414213568) and np.float32(c[1, 1]) == np.float32(2.38578629)
    assert np.float32(c[2, 0]) == np.float32(0.828427136) and np.float32(c[0, 1]) == np.float32(2.79999995)
    c = H.camera_update((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, np.float32(1920) / np.float32(1080))
    assert np.float32(c[1, 0]) == np.float32(-0.736379683) and np.float32(c[2, 0]) == np.float32(1.47275937)


def test_hdr_decode_and_table_match_reference_probe():
    """RGBE decode (stbi_loadf) + LoadHDRImage table vs the SURVEY 8c probe of
    the reference's own shader.hpp code (sha256 prefix/suffix, spot values)."""
    pr = FIX["hdr_1k_survey_probe"]
    rgb, tab = H.load_hdr(S.HDR_1K)
    assert rgb.shape == (512, 1024, 3)
    h1, h2 = sha(rgb), sha(tab)
    assert h1.startswith(pr["rgb_sha256_prefix"]) and h1.endswith(pr["rgb_sha256_suffix"]), h1
    assert h2.startswith(pr["table_sha256_prefix"]) and h2.endswith(pr["table_sha256_suffix"]), h2
    for key, val in pr["table_spots"].items():
        j, i = map(int, key.split(","))
        np.testing.assert_allclose(tab[j, i], val, rtol=1e-7)
    assert np.float32(tab[..., 2].max()) == np.float32(pr["table_max_pdf"])


def test_sobol_table_matches_reference_shader():
    V = json.load(open(os.path.join(GOLD, "sobol_v.json")))["V"]
    assert hashlib.sha256(np.array(V, "<u4").tobytes()).hexdigest() == FIX["sobol_v_sha256"]
    root = os.path.dirname(os.path.dirname(__file__))
    for path in ("oracle/sobol_v.inc", "pnraytracing_amd/csrc/sobol_v.inc"):
        txt = open(os.path.join(root, path)).read().split("*/", 1)[1]
        ours = [int(x.strip().rstrip("u")) for x in txt.replace("\n", " ").split(",") if x.strip()]
        assert ours == V, path


def test_host_errors_are_reported():
    sb = H.SceneBuilder()
    with pytest.raises(H.HostError):
        sb.build()                      # no triangles
    sb.add_material(H.Material())
    m = H.mesh_quad(1.0)
    bad = H.Mesh(m.positions, m.normals, m.texcoords, np.array([0, 1, 99], np.int32))
    with pytest.raises(H.HostError):
        sb.add_model(bad, [H.scale(1.0)], H.Material())
