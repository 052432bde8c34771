"""GPU BuildBVH (pnrt_bvh_build, csrc/pt_bvh.h) against the host BuildBVH
restatement (csrc/host/pnrt_host.cpp BvhBuilder, itself pinned to the
reference's include/BVH.hpp by tests/test_host_arrays.py): node arrays,
triangle order and depth must be identical bit for bit.

Inputs: the C1-C5 scenes, and adversarial bound sets built the way
ModelOutput does (model.hpp:125-128: Bound::Union of the three vertices with
glm's first-operand-on-ties min/max, centre = (pMax + pMin) * .5f) -- integer
grids (bucket / centroid ties), signed zeros (the first-occurrence rule),
coincident centres (degenerate-centre leaves), collinear and huge
coordinates, and sizes around the one-wave (64) and chunk (2048) limits.
"""
import numpy as np
import pytest

from pnraytracing_amd import host as H
from pnraytracing_amd import scenes as S

F32_MAX = np.float32(3.4028235e38)


def glm_bounds(p0, p1, p2):
    """(n, 9) Bound + boundCenter of triangles (n, 3) x 3, glm semantics."""
    mn = np.full(p0.shape, F32_MAX, np.float32)
    mx = np.full(p0.shape, -F32_MAX, np.float32)
    for p in (p0, p1, p2):
        mn = np.where(p < mn, p, mn)          # glm::min(x, y) = y < x ? y : x
        mx = np.where(mx < p, p, mx)          # glm::max(x, y) = x < y ? y : x
    c = ((mx + mn) * np.float32(0.5)).astype(np.float32)
    return np.ascontiguousarray(np.concatenate([mn, mx, c], 1), np.float32)


def adversarial(kind: str, n: int, seed: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if kind == "random":
        pts = [rng.standard_normal((n, 3)).astype(np.float32) for _ in range(3)]
        base = rng.uniform(-10, 10, (n, 3)).astype(np.float32)
        pts = [base + 0.05 * p for p in pts]
    elif kind == "grid":                  # integer coordinates: many equal centres and buckets
        base = rng.integers(-6, 7, (n, 3)).astype(np.float32)
        pts = [base + rng.integers(0, 2, (n, 3)).astype(np.float32) for _ in range(3)]
    elif kind == "signed_zero":           # -0 / +0 everywhere: the first-occurrence rule decides bits
        choice = np.array([-0.0, 0.0, 1.0, -1.0, 0.5], np.float32)
        pts = [choice[rng.integers(0, len(choice), (n, 3))] for _ in range(3)]
    elif kind == "coincident":            # identical triangles: degenerate centre bound
        t = rng.standard_normal((1, 3)).astype(np.float32)
        pts = [np.repeat(t + k, n, 0).astype(np.float32) for k in range(3)]
    elif kind == "collinear":             # all on one line, zero-area boxes
        s = rng.uniform(-5, 5, (n, 1)).astype(np.float32)
        d = np.array([[1.0, 2.0, -0.5]], np.float32)
        pts = [(s + k * np.float32(0.01)) * d for k in range(3)]
    elif kind == "clustered":             # a few hot spots + outliers
        cen = rng.standard_normal((5, 3)).astype(np.float32) * 4
        base = cen[rng.integers(0, 5, n)] + rng.standard_normal((n, 3)).astype(np.float32) * 1e-3
        base[rng.random(n) < 0.01] *= 100
        pts = [base + rng.standard_normal((n, 3)).astype(np.float32) * 1e-4 for _ in range(3)]
    elif kind == "huge":
        pts = [(rng.standard_normal((n, 3)) * 1e30).astype(np.float32) for _ in range(3)]
    else:
        raise ValueError(kind)
    return glm_bounds(*pts)


def same_build(a, b):
    (na, oa, da), (nb, ob, db) = a, b
    assert na.shape == nb.shape, (na.shape, nb.shape)
    bad = np.flatnonzero(np.any(na.view(np.uint32) != nb.view(np.uint32), axis=1))
    assert bad.size == 0, f"{bad.size} nodes differ, first {bad[0]}: {na[bad[0]]} vs {nb[bad[0]]}"
    assert np.array_equal(oa, ob), f"triangle order differs at {np.flatnonzero(oa != ob)[:5]}"
    assert da == db


# ---- CPU: the bare-bounds host build is the scene build ---------------------------------------
def _scene_builder(seed=3):
    sb = H.SceneBuilder()
    S._cornell_walls(sb, H.Material(baseColor=(0.65, 0.65, 0.65)))
    sb.add_model(H.mesh_displaced_sphere(40, 25, 0.3, (0.0, 1.0, 0.0), 0.1, seed), [H.scale(2.0)],
                 H.Material(baseColor=(0.5, 0.5, 0.5)), "ball")
    return sb


def test_cpu_bounds_build_matches_scene_build():
    sb = _scene_builder()
    tb = sb.tri_bounds()
    nodes, order, depth = H.bvh_build_cpu(tb)
    packed = sb.build()
    assert np.array_equal(nodes.view(np.uint32), packed.nodes.view(np.uint32))
    assert depth == packed.max_depth
    # installing the same build through pnrt_scene_set_bvh gives the same packed arrays
    sb2 = _scene_builder()
    n2, o2, d2 = H.bvh_build_cpu(sb2.tri_bounds())
    H._check(sb2._lib.pnrt_scene_set_bvh(sb2._s, H.N.iptr(o2), H.N.fptr(n2), len(n2), d2), "set_bvh")
    packed2 = sb2._pack()
    for a, b in zip(packed.arrays(), packed2.arrays()):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("kind", ["random", "grid", "signed_zero", "coincident", "collinear", "clustered", "huge"])
def test_cpu_adversarial_sets_build(kind):
    for n in (1, 2, 3, 65, 300):
        nodes, order, depth = H.bvh_build_cpu(adversarial(kind, n, seed=n))
        assert sorted(order.tolist()) == list(range(n))
        assert len(nodes) <= 2 * n - 1


# ---- GPU: identical to the host build -------------------------------------------------------
@pytest.fixture(scope="module")
def tracer():
    from pnraytracing_amd.tracer import PathTracer
    with PathTracer(0) as pt:
        yield pt


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["random", "grid", "signed_zero", "coincident", "collinear", "clustered", "huge"])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 63, 64, 65, 66, 129, 300, 2047, 2048, 2049, 5000, 40000])
def test_gpu_build_matches_host(tracer, kind, n):
    tb = adversarial(kind, n, seed=1000 + n)
    same_build(tracer.build_bvh(tb), H.bvh_build_cpu(tb))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["random", "grid", "signed_zero", "clustered"])
def test_gpu_build_matches_host_large(tracer, kind):
    tb = adversarial(kind, 300_000, seed=7)
    same_build(tracer.build_bvh(tb), H.bvh_build_cpu(tb))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C4"])
def test_gpu_built_scene_arrays_identical(tracer, name):
    kw = {"C1": {}, "C2": {"env": False}, "C3": {}, "C4": {}}[name]
    ref = S.CONFIGS[name](**kw).packed
    got = S.CONFIGS[name](bvh_tracer=tracer, **kw).packed
    for a, b, what in zip(ref.arrays(), got.arrays(), ("vertices", "materials", "triangles", "nodes", "lights")):
        assert a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32)), what
    assert ref.lights_sum_area == got.lights_sum_area and ref.max_depth == got.max_depth


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_build_c5_4m(tracer):
    sb = H.SceneBuilder()
    big = H.mesh_displaced_sphere(2048, 1024, S.BUNNY_RADIUS, S.BUNNY_CENTER, 0.12, 0x5EED)
    sb.add_model(big, [H.translate(0, 0, -2), H.scale(8)], H.Material(baseColor=(0.65, 0.65, 0.65)), "sphere4m")
    S._cornell_walls(sb, H.Material(baseColor=(0.65, 0.65, 0.65)))
    tb = sb.tri_bounds()
    same_build(tracer.build_bvh(tb), H.bvh_build_cpu(tb))
