"""Randomised scenes, GPU vs CPU oracle, bit for bit.

Every Disney parameter drawn at random per material (metallic, clearcoat,
anisotropic, sheen, subsurface, roughness down to 0 ...), triangle soups and
quads with and without vertex normals, several emissive materials (multi-
light binary search) or none at all (GetLightIndex -> -1), environment on and
off, RGB/RGBA/grey textures of odd widths on some meshes, odd image sizes and
row-band shards, depth 1..4 -- the cases the fixed C1-C5 scenes do not reach.
"""
import os

import numpy as np
import pytest

import pyoracle
from pnraytracing_amd import host as H
from pnraytracing_amd import scenes as S

pytestmark = pytest.mark.gpu


def random_scene(seed: int):
    rng = np.random.default_rng(seed)
    sb = H.SceneBuilder()
    n_lights = int(rng.integers(0, 4))
    textures = []
    n_tex = int(rng.integers(0, 3))
    for t in range(n_tex):
        w, h, ch = int(rng.integers(3, 40)), int(rng.integers(2, 30)), int(rng.choice([1, 3, 4]))
        textures.append(S.checker_texture(w, h, ch, seed=seed * 7 + t))

    def rand_material(emissive=False):
        m = H.Material(baseColor=tuple(rng.uniform(0, 1, 3)), subsurface=rng.uniform(0, 1),
                       metallic=float(rng.choice([0.0, 1.0, rng.uniform(0, 1)])), specular=rng.uniform(0, 1),
                       specularTint=rng.uniform(0, 1), roughness=float(rng.choice([0.0, 1.0, rng.uniform(0, 1)])),
                       anisotropic=rng.uniform(0, 1), sheen=rng.uniform(0, 1), sheenTint=rng.uniform(0, 1),
                       clearcoat=rng.uniform(0, 1), clearcoatGloss=rng.uniform(0, 1))
        if emissive:
            m = m.copy(emssive=tuple(rng.uniform(0.5, 30, 3)))
        return m

    # an enclosure so paths bounce: the Cornell walls with random materials
    S._cornell_walls(sb, rand_material(), floor_mat=rand_material(), light=rng.random() < 0.6)
    # triangle soups
    for k in range(int(rng.integers(1, 4))):
        n = int(rng.integers(4, 200))
        base = rng.uniform(-2, 2, (n, 1, 3)) + np.array([0, 2.5, 0])
        P = (base + rng.normal(0, 0.4, (n, 3, 3))).reshape(-1, 3).astype(np.float32)
        normals = None if rng.random() < 0.3 else rng.normal(0, 1, (3 * n, 3)).astype(np.float32)
        if normals is not None and rng.random() < 0.3:
            normals[rng.integers(0, 3 * n, 5)] = 0.0       # a zero vertex normal -> face normal (:338-348)
        uv = rng.uniform(-1, 2, (3 * n, 2)).astype(np.float32)
        mesh = H.Mesh(P, normals, uv, np.arange(3 * n, dtype=np.int32))
        tex = [int(rng.integers(-1, n_tex))] if n_tex else None
        sb.add_model(mesh, [H.rotate(float(rng.uniform(0, 360)), 0, 1, 0)], rand_material(), f"soup{k}",
                     texture_ids=tex)
    for k in range(n_lights):
        pos = rng.uniform(-2, 2, 3)
        sb.add_model(H.mesh_quad(27.5), [H.translate(pos[0], 5.0 - k * 0.7, pos[2]), H.rotate(180.0, 0, 0, 1),
                                         H.scale(float(rng.uniform(0.005, 0.03)))], rand_material(True), f"light{k}")
    W, Hh = int(rng.integers(17, 70)), int(rng.integers(9, 50))
    eye = (float(rng.uniform(-1, 1)), float(rng.uniform(1.5, 4)), float(rng.uniform(5, 8)))
    cam = H.camera_update(eye, (0, 2.6, 0), (0, 1, 0), float(rng.uniform(30, 70)), np.float32(W) / np.float32(Hh))
    rgb = tab = None
    if rng.random() < 0.6:
        rgb = H.synthetic_hdr(64, 32, seed)
        tab = H.hdr_table(rgb)
    cfg = S.SceneConfig(f"fuzz{seed}", sb.build(), cam, W, Hh, 1, max_depth=int(rng.integers(1, 5)),
                        env_rgb=rgb, env_table=tab, textures=textures)
    return cfg, rng


@pytest.fixture(scope="module")
def pt():
    from pnraytracing_amd.tracer import PathTracer
    with PathTracer(0) as t:
        yield t


# PNRT_FUZZ_SEEDS=N widens the campaign (default 24 seeds; 400 were run once),
# PNRT_FUZZ_FIRST=k starts it at seed k (a fresh range)
_FIRST = int(os.environ.get("PNRT_FUZZ_FIRST", "0"))


@pytest.mark.parametrize("seed", list(range(_FIRST, _FIRST + int(os.environ.get("PNRT_FUZZ_SEEDS", "24")))))
def test_random_scene_bitwise(pt, seed):
    from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL
    cfg, rng = random_scene(seed)
    first, n = int(rng.integers(0, 20)), int(rng.integers(1, 10))
    ref, _ = pyoracle.Oracle(cfg).render(first, n)
    for mode in (TRAVERSE_ZCULL, TRAVERSE_EXACT, TRAVERSE_ZCULL | KERNEL_V1):
        pt.load(cfg, mode)
        pt.reset_accum()
        pt.render(first, n)
        got = pt.read_accum()
        bad = np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1)
        assert not bad.any(), (f"seed {seed} mode {mode:#x}: {int(bad.sum())} of {bad.size} pixels differ "
                               f"(depth {cfg.max_depth}, {cfg.width}x{cfg.height}, env {cfg.env_rgb is not None}, "
                               f"lights {len(cfg.packed.lights)})")


@pytest.mark.parametrize("seed", [101, 102, 103])
def test_random_scene_shards(pt, seed):
    """Odd sizes and bands: the union of the shards equals the full render."""
    cfg, rng = random_scene(seed)
    band, nsh = int(rng.integers(1, 9)), int(rng.integers(2, 5))
    ref, _ = pyoracle.Oracle(cfg).render(0, 2)
    pt.load(cfg)
    pt.reset_accum()
    for sh in range(nsh):
        pt.render(0, 2, band, nsh, sh)
    got = pt.read_accum()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("copies", [130, 300])
def test_coincident_triangles_table_leaf(pt, copies):
    """`copies` identical triangles: one degenerate-centre leaf (BVH.hpp:117-120)
    too large for an inline leaf ref (> 127 triangles -> the leaf table), and
    exact t ties everywhere -- the reference's `>` rule (the later triangle wins,
    :311-312) decides which triangle's material is hit."""
    from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL
    rng = np.random.default_rng(copies)
    sb = H.SceneBuilder()
    S._cornell_walls(sb, H.Material(baseColor=(0.6, 0.6, 0.6)))
    tri = np.array([[-1.0, 0.5, -1.0], [1.5, 0.7, -0.5], [0.0, 3.0, -1.2]], np.float32)
    for k in range(3):                       # three materials share the same geometry
        P = np.tile(tri, (copies // 3, 1))
        mesh = H.Mesh(P, None, None, np.arange(len(P), dtype=np.int32))
        sb.add_model(mesh, [H.scale(1.0)], H.Material(baseColor=tuple(rng.uniform(0, 1, 3)), metallic=0.3 * k),
                     f"stack{k}")
    W, Hh = 40, 30
    cfg = S.SceneConfig("coincident", sb.build(), S._cornell_camera(W, Hh), W, Hh, 1, max_depth=3,
                        env_rgb=None, env_table=None)
    nd = cfg.packed.nodes
    leaves = nd[:, 7] == -1
    assert (nd[leaves, 9] - nd[leaves, 8]).max() > 127
    ref, _ = pyoracle.Oracle(cfg).render(0, 3)
    for mode in (TRAVERSE_ZCULL, TRAVERSE_EXACT, TRAVERSE_ZCULL | KERNEL_V1):
        pt.load(cfg, mode)
        pt.reset_accum()
        pt.render(0, 3)
        got = pt.read_accum()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), mode


def test_nonfinite_box_disables_culling(pt):
    """A BVH box with an infinite coordinate (a conservative bound: the tree stays
    a valid BVH).  z-slab culling's proof needs finite boxes, so the library
    traverses such a scene without culling; every mode still equals the oracle
    bit for bit."""
    import dataclasses
    from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL
    cfg, _ = random_scene(7)
    nd = cfg.packed.nodes.copy()
    leaf = int(np.flatnonzero(nd[:, 7] == -1)[0])
    nd[leaf, 5] = np.inf                     # the first leaf's box max z
    cfg = dataclasses.replace(cfg, packed=dataclasses.replace(cfg.packed, nodes=nd))
    ref, _ = pyoracle.Oracle(cfg).render(0, 3)
    for mode in (TRAVERSE_ZCULL, TRAVERSE_EXACT, TRAVERSE_ZCULL | KERNEL_V1):
        pt.load(cfg, mode)
        pt.reset_accum()
        pt.render(0, 3)
        got = pt.read_accum()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), mode


@pytest.mark.parametrize("seed,exp10", [(200 + k, (-30, -20, -10, 10, 20, 25)[k % 6]) for k in range(48)])
def test_random_scene_extreme_emission(pt, seed, exp10):
    """Emission scaled by 10^exp10 (every emissive material): radiance terms far
    below or above Lo's rounding, subnormal products at 1e-30 -- where the moot-ray
    test (pt_wf.h WF_SKIP_MOOT) decides most often; still bit for bit."""
    import dataclasses
    from pnraytracing_amd.tracer import TRAVERSE_ZCULL
    cfg, rng = random_scene(seed)
    mats = cfg.packed.materials.copy()
    mats[:, 0:3] = (mats[:, 0:3].astype(np.float64) * 10.0 ** exp10).astype(np.float32)
    cfg = dataclasses.replace(cfg, packed=dataclasses.replace(cfg.packed, materials=mats),
                              max_depth=4)
    first, n = int(rng.integers(0, 20)), 6
    ref, _ = pyoracle.Oracle(cfg).render(first, n)
    assert np.isfinite(ref).all()
    pt.load(cfg, TRAVERSE_ZCULL)
    pt.reset_accum()
    pt.render(first, n)
    got = pt.read_accum()
    bad = np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1)
    assert not bad.any(), f"seed {seed} x1e{exp10}: {int(bad.sum())} of {bad.size} pixels differ"
