"""GPU build of LoadHDRImage's RandomHDR table (shader.hpp:145-203, SURVEY 8f
row 3) vs the host restatement (itself pinned to the reference's probe
hashes in test_host_arrays.py): bit-exact."""
import time

import numpy as np
import pytest

from pnraytracing_amd import host as H
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pt():
    t = PathTracer(0)
    yield t
    t.close()


def _check(pt, rgb):
    t0 = time.perf_counter()
    ref = H.hdr_table(rgb)
    t_host = time.perf_counter() - t0
    pt.upload_env_build(rgb)          # warm-up (module load)
    t0 = time.perf_counter()
    pt.upload_env_build(rgb)
    t_gpu = time.perf_counter() - t0
    got = pt.read_env_table()
    bad = np.argwhere(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1))
    assert len(bad) == 0, f"{len(bad)} texels differ, first {bad[:3].tolist()}"
    print(f"{rgb.shape[1]}x{rgb.shape[0]}: host {t_host * 1e3:.1f} ms, gpu {t_gpu * 1e3:.1f} ms")


def test_table_reference_hdr(pt):
    rgb, _ = H.load_hdr(S.HDR_1K)
    _check(pt, rgb)


def test_table_synthetic_4k(pt):
    _check(pt, H.synthetic_hdr(4096, 2048, 0x5EED))


@pytest.mark.parametrize("w,h", [(37, 13), (64, 1), (1, 50)])
def test_table_odd_sizes(pt, w, h):
    rng = np.random.default_rng(w * 100 + h)
    rgb = (rng.random((h, w, 3)) ** 4 * 50).astype(np.float32)
    _check(pt, rgb)


def test_render_with_gpu_table(pt):
    c = S.bunny_c2(96, 54)
    pt.load(c)
    pt.reset_accum()
    pt.render(0, 2)
    a = pt.read_accum()
    pt.upload_env_build(c.env_rgb)
    pt.reset_accum()
    pt.render(0, 2)
    assert np.array_equal(pt.read_accum().view(np.uint32), a.view(np.uint32))


@pytest.mark.parametrize("w,h", [(1, 1), (2, 3), (37, 13), (64, 1), (1, 50)])
def test_render_odd_env_sizes_bitwise(pt, w, h):
    """Environment lookups through the footprint records (edge clamps on every
    side, one-texel rows and columns) equal the oracle's four-tap reads."""
    import dataclasses
    import pyoracle
    rng = np.random.default_rng(7 * w + h)
    rgb = (rng.random((h, w, 3)) ** 4 * 50).astype(np.float32)
    c = dataclasses.replace(S.bunny_c2(64, 36), env_rgb=rgb, env_table=H.hdr_table(rgb))
    pt.load(c)
    pt.reset_accum()
    pt.render(0, 2)
    got = pt.read_accum()
    ref, _ = pyoracle.Oracle(c).render(0, 2)
    bad = np.argwhere(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1))
    assert len(bad) == 0, f"{w}x{h} env: {len(bad)} pixels differ, first {bad[:3].tolist()}"
