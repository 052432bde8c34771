"""GPU parity: the HIP library (through its C ABI) vs the CPU oracle.

Bar: bit-exact images (the integrator output is fp32, but both sides evaluate
the same IEEE operation sequence, so any difference is a real divergence --
tolerance 0 ulp).  Large configurations are compared on a row subset that the
oracle finishes in seconds; size-independent properties (progressive-mean
order, shard union, traversal-mode equivalence) run at full size on the GPU.
"""
import numpy as np
import pytest

import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL, PathTracer, PnrtError

pytestmark = pytest.mark.gpu

_cache = {}


def cfg(name, **kw):
    key = (name, tuple(sorted(kw.items())))
    if key not in _cache:
        _cache[key] = S.CONFIGS[name](**kw)
    return _cache[key]


@pytest.fixture(scope="module")
def pt():
    t = PathTracer(0)
    yield t
    t.close()


def gpu_render(pt, c, first, n, mode=TRAVERSE_ZCULL, shard=(1, 1, 0)):
    pt.load(c, mode)
    pt.reset_accum()
    pt.render(first, n, *shard)
    return pt.read_accum()


def assert_bitwise(got, ref, what):
    g, r = got.view(np.uint32), ref.view(np.uint32)
    bad = np.argwhere(np.any(g != r, axis=-1))
    assert len(bad) == 0, f"{what}: {len(bad)} pixels differ, first {bad[:5].tolist()} " \
                          f"gpu={got[tuple(bad[0])]} oracle={ref[tuple(bad[0])]}"


# ---- PN-libm and IEEE primitives ------------------------------------------------------------
SPECIAL = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-38, 1.17549435e-38, 0.5, 1.0, -1.0, 2.0, 3.14159265,
                    1.5707964, 1e6, -1e6, 1e30, np.inf, -np.inf, np.nan], np.float32)


def _inputs(fn, rng, n=200000):
    if fn in (0, 1):
        a = rng.uniform(-20, 20, n)
    elif fn == 3:
        a = rng.uniform(-1.05, 1.05, n)
    elif fn in (4, 5):
        a = np.exp(rng.uniform(-90, 90, n))
    elif fn == 6:
        a = rng.uniform(-160, 140, n)
    elif fn in (9, 10):
        a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    else:
        a = rng.standard_normal(n) * np.exp(rng.uniform(-40, 40, n))
    b = rng.standard_normal(n) * np.exp(rng.uniform(-40, 40, n)) if fn in (2, 8) else rng.uniform(0, 1.2, n)
    with np.errstate(over="ignore"):          # (exp(+-90) leaves float32 range on purpose: inf inputs)
        a = np.concatenate([np.asarray(a, np.float32), SPECIAL, SPECIAL])
        b = np.concatenate([np.asarray(b, np.float32), SPECIAL, SPECIAL[::-1]])
    return a, b


@pytest.mark.parametrize("fn", list(range(11)))
def test_math_bitwise(pt, fn):
    rng = np.random.default_rng(100 + fn)
    a, b = _inputs(fn, rng)
    got = pt.debug_math(fn, a, b)
    ref = pyoracle.math_eval(fn, a, b)
    both_nan = np.isnan(got) & np.isnan(ref)
    diff = (got.view(np.uint32) != ref.view(np.uint32)) & ~both_nan
    assert not diff.any(), (fn, a[diff][:4], b[diff][:4], got[diff][:4], ref[diff][:4])


# ---- whole images ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", [TRAVERSE_EXACT, TRAVERSE_ZCULL, TRAVERSE_ZCULL | KERNEL_V1])
@pytest.mark.parametrize("first,n", [(0, 1), (0, 4), (7, 3), (0, 11)])
def test_c1_bitwise(pt, mode, first, n):
    c = cfg("C1")
    got = gpu_render(pt, c, first, n, mode)
    ref, st = pyoracle.Oracle(c).render(first, n)
    assert st["stack_overflow"] == 0
    assert_bitwise(got, ref, f"C1 mode={mode} frames {first}+{n}")


def test_c1_depth_variants(pt):
    for depth in (0, 1, 2):
        c = S.cornell_c1(64, 48)
        c.max_depth = depth
        got = gpu_render(pt, c, 0, 2)
        ref, _ = pyoracle.Oracle(c).render(0, 2)
        assert_bitwise(got, ref, f"C1 depth {depth}")


@pytest.mark.parametrize("mode", [TRAVERSE_ZCULL, TRAVERSE_ZCULL | KERNEL_V1])
def test_c2_small_bitwise(pt, mode):
    c = cfg("C2", width=192, height=108, spp=4)
    got = gpu_render(pt, c, 0, 4, mode)
    ref, _ = pyoracle.Oracle(c).render(0, 4)
    assert_bitwise(got, ref, "C2 192x108")


def test_c2_fullsize_rows_bitwise(pt):
    """Bench config (1920x1080, 4 spp, 1k env): every 36th row vs the oracle."""
    c = cfg("C2")
    got = gpu_render(pt, c, 0, 4)
    o = pyoracle.Oracle(c)
    ref = np.zeros_like(got)
    o.render(0, 4, rows=(5, c.height), y_step=36, accum=ref)
    rows = np.arange(5, c.height, 36)
    assert_bitwise(got[rows], ref[rows], "C2 1080p rows")
    assert np.isfinite(got).all() and (got[..., 3] == 1).all()


def test_c4_rows_bitwise(pt):
    """Teapot + area light + env: light, env and BSDF pdfs all active."""
    c = cfg("C4", width=640, height=360)
    got = gpu_render(pt, c, 2, 3)
    ref = np.zeros_like(got)
    pyoracle.Oracle(c).render(2, 3, rows=(1, c.height), y_step=9, accum=ref)
    rows = np.arange(1, c.height, 9)
    assert_bitwise(got[rows], ref[rows], "C4 rows")


def test_c3_textured_bitwise(pt):
    """Albedo textures: RGBA 2048x1024 (REPEAT, bilinear, UNORM8) and an RGB
    texture of odd width (GL_UNPACK_ALIGNMENT 4 row skew); all Disney lobes."""
    c = cfg("C3", width=192, height=108)
    got = gpu_render(pt, c, 0, 4)
    ref, st = pyoracle.Oracle(c).render(0, 4)
    assert st["albedo_bytes"] > 0
    assert_bitwise(got, ref, "C3 192x108")


def test_c3_fullsize_rows_bitwise(pt):
    c = cfg("C3")
    got = gpu_render(pt, c, 4, 4)
    ref = np.zeros_like(got)
    pyoracle.Oracle(c).render(4, 4, rows=(3, c.height), y_step=45, accum=ref)
    rows = np.arange(3, c.height, 45)
    assert_bitwise(got[rows], ref[rows], "C3 1080p rows")


def test_c5_4m_triangles_rows_bitwise(pt):
    """4.19M-triangle BVH (depth, leaf-table refs, stack spill) + 4k synthetic
    env, at a reduced resolution."""
    c = cfg("C5", width=320, height=180)
    got = gpu_render(pt, c, 0, 2)
    info = pt.device_info()
    assert info["n_triangles"] == c.n_triangles and info["n_interior"] > 1_000_000
    ref = np.zeros_like(got)
    pyoracle.Oracle(c).render(0, 2, rows=(1, c.height), y_step=6, accum=ref)
    rows = np.arange(1, c.height, 6)
    assert_bitwise(got[rows], ref[rows], "C5 rows")


# ---- size-independent properties at full size ------------------------------------------------
def test_traversal_modes_agree_fullsize(pt):
    """z-slab culling is result-neutral and both kernels compute the same
    image: every pixel of the 1080p bench image (8.3M samples)."""
    c = cfg("C2")
    a = gpu_render(pt, c, 0, 4, TRAVERSE_EXACT)
    b = gpu_render(pt, c, 0, 4, TRAVERSE_ZCULL)
    assert_bitwise(b, a, "exact vs zcull")
    other = gpu_render(pt, c, 0, 4, TRAVERSE_ZCULL | KERNEL_V1)
    assert_bitwise(other, a, "v1 kernel vs wavefront")


def test_progressive_split_calls(pt):
    c = cfg("C2", width=192, height=108, spp=4)
    pt.load(c)
    pt.reset_accum()
    pt.render(0, 4)
    a = pt.read_accum()
    pt.reset_accum()
    pt.render(0, 1)
    pt.render(1, 3)
    b = pt.read_accum()
    assert_bitwise(b, a, "render(0,1)+render(1,3) vs render(0,4)")


def test_large_frame_batches(pt):
    """An 8192x4320 frame (35.4M path slots) fits 7 frames in one batch (2^28
    slots), so a full-frame call of 9 frames renders batches of 7 + 2 frames; a
    1/16 row shard of the same call fits all nine in one batch.  Its rows must
    match."""
    c = S.bunny_c2(8192, 4320)
    pt.load(c)
    pt.reset_accum()
    pt.render(0, 9)
    full = pt.read_accum()
    pt.reset_accum()
    pt.render(0, 9, 8, 16, 0)
    part = pt.read_accum()
    rows = (np.arange(c.height) // 8) % 16 == 0
    assert_bitwise(part[rows], full[rows], "8192x4320: shard (one batch) vs full frame (batches of 7 + 2 frames)")


def test_many_frames_and_calls(pt):
    """One call of 140 frames (two frame groups: batches of <= 128 frames) and six
    calls in a row (the pipelined buffer sets rotate twice) both equal the
    oracle's 140 / 12-frame progressive means."""
    c = cfg("C2", width=80, height=48, spp=4)
    got = gpu_render(pt, c, 0, 140)
    ref, _ = pyoracle.Oracle(c).render(0, 140)
    assert_bitwise(got, ref, "render(0, 140)")
    pt.reset_accum()
    for k in range(6):
        pt.render(2 * k, 2)
    ref, _ = pyoracle.Oracle(c).render(0, 12)
    assert_bitwise(pt.read_accum(), ref, "6 x render(2k, 2)")


def test_shard_union_equals_full(pt):
    c = cfg("C2", width=200, height=100, spp=4)
    full = gpu_render(pt, c, 0, 2)
    pt.reset_accum()
    for s in range(3):
        pt.render(0, 2, 8, 3, s)
    assert_bitwise(pt.read_accum(), full, "3 shards of 8-row bands")


def test_pack_rows(pt):
    import torch
    c = cfg("C2", width=64, height=40, spp=1)
    full = gpu_render(pt, c, 0, 1)
    from pnraytracing_amd.tracer import shard_rows
    rows = shard_rows(40, 8, 3, 1)
    dst = torch.zeros((len(rows), 64, 4), dtype=torch.float32, device="cuda")
    pt.pack_rows(dst.data_ptr(), 8, 3, 1)
    pt.synchronize()
    np.testing.assert_array_equal(dst.cpu().numpy().view(np.uint32), full[rows].view(np.uint32))


def test_errors_are_reported(pt):
    t = PathTracer(0)
    with pytest.raises(PnrtError):
        t.render(0, 1)                      # nothing uploaded
    c = cfg("C1")
    t.upload_scene(c.packed)
    with pytest.raises(PnrtError):
        t.set_frame(16, 16, c.camera, 5)    # MAX_BOUNCE_DEPTH <= 4 (8 Sobol dims)
    bad = c.packed.triangles.copy()
    bad[0, 0] = 1e6
    import dataclasses
    with pytest.raises(PnrtError):
        t.upload_scene(dataclasses.replace(c.packed, triangles=bad))
    t.close()


def test_obj_ingested_scene_bitwise(pt, tmp_path):
    """SURVEY 8f row 1 on the GPU: C4's meshes written as OBJ files and read back
    through pnraytracing_amd.obj (unshared per-corner vertices, as Assimp
    builds them) render the same image as the procedural scene, and the oracle's."""
    import dataclasses
    import test_obj
    base = cfg("C4", width=192, height=108)
    c = dataclasses.replace(base, name="C4-obj", packed=test_obj._teapot_scene(str(tmp_path)))
    got = gpu_render(pt, c, 0, 4)
    ref, _ = pyoracle.Oracle(c).render(0, 4)
    assert_bitwise(got, ref, "C4 via OBJ")
    assert np.array_equal(got.view(np.uint32), gpu_render(pt, base, 0, 4).view(np.uint32))
