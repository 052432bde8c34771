"""Moot rays (pt_wf.h WF_SKIP_MOOT): shadow rays and last-bounce continuation
rays whose outcome cannot change the path are not traced.  Scenes that push the
test to its ends, each against the oracle bit for bit (tolerance 0 ulp):

* no emission anywhere (LDirect = 0 for every light ray, emit_max = 0: every
  last-bounce continuation ray is moot), at depths 1-4;
* the light's emission raised a millionfold by pnrt_update_materials after
  frames were rendered with it tiny -- the library's emission bound must follow
  the edit, or last-bounce rays that now hit a bright light would be skipped;
* the reverse edit (bright to dark).
The hand-picked and random float cases of the bound itself are in
tests/test_moot_bound.py (CPU)."""
import numpy as np
import pytest

import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer

pytestmark = pytest.mark.gpu

W, H = 80, 60


def _bitwise(got, ref):
    return int(np.count_nonzero(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1)))


def test_no_emission_anywhere():
    cfg = S.cornell_c1(W, H)
    cfg.packed.materials = cfg.packed.materials.copy()
    cfg.packed.materials[:, 0:3] = 0.0
    with PathTracer(0) as pt:
        for depth in (1, 2, 3, 4):
            cfg.max_depth = depth
            pt.load(cfg)
            pt.reset_accum()
            pt.render(0, 3)
            ref, _ = pyoracle.Oracle(cfg).render(0, 3)
            assert _bitwise(pt.read_accum(), ref) == 0, f"depth {depth}"


@pytest.mark.parametrize("scale", [1e6, 1e-6])
def test_emission_edit_moves_the_bound(scale):
    cfg = S.cornell_c1(W, H)
    mats = cfg.packed.materials.copy()
    light = [i for i in range(len(mats)) if mats[i, :3].max() > 0]
    assert light
    start = mats.copy()
    for li in light:                       # start from the other end of the edit
        start[li, 0:3] = mats[li, 0:3] / np.float32(scale)
    edited = start.copy()
    for li in light:
        edited[li, 0:3] = start[li, 0:3] * np.float32(scale)
    cfg.packed.materials = start
    ref = np.zeros((H, W, 4), np.float32)
    pyoracle.Oracle(cfg).render(0, 2, accum=ref)
    cfg.packed.materials = edited
    pyoracle.Oracle(cfg).render(2, 3, accum=ref)
    cfg.packed.materials = start
    with PathTracer(0) as pt:
        pt.load(cfg)
        pt.reset_accum()
        pt.render(0, 2)
        pt.synchronize()
        pt.update_materials(0, edited)
        pt.render(2, 3)
        assert _bitwise(pt.read_accum(), ref) == 0
