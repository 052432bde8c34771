"""Moot rays (pt_wf.h WF_SKIP_MOOT): shadow rays and last-bounce continuation
rays whose outcome cannot change the path are not traced.  Scenes that push the
test to its ends, each against the oracle bit for bit (tolerance 0 ulp):

* no emission anywhere (LDirect = 0 for every light ray, emit_max = 0: every
  last-bounce continuation ray is moot), at depths 1-4;
* the light's emission raised a millionfold by pnrt_update_materials after
  frames were rendered with it tiny -- the library's emission bound must follow
  the edit, or last-bounce rays that now hit a bright light would be skipped;
* the reverse edit (bright to dark);
* the environment dimmed / brightened by 10^6, then the original uploaded
  between frames (the bound includes the env's largest texel).
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


@pytest.mark.parametrize("scale", [1e6, 1e-6])
def test_env_upload_moves_the_bound(scale):
    """The emission bound follows pnrt_upload_env too: C2 (env-lit) rendered
    with its environment dimmed (or brightened) by 10^6, then the original
    environment uploaded between frames (same importance table both times)."""
    import dataclasses
    full = S.bunny_c2(96, 64, spp=4)
    other = dataclasses.replace(full, env_rgb=(full.env_rgb / np.float32(scale)).astype(np.float32))
    ref = np.zeros((64, 96, 4), np.float32)
    pyoracle.Oracle(other).render(0, 2, accum=ref)
    pyoracle.Oracle(full).render(2, 3, accum=ref)
    with PathTracer(0) as pt:
        pt.load(other)
        pt.reset_accum()
        pt.render(0, 2)
        pt.synchronize()
        pt.upload_env(full.env_rgb, full.env_table)
        pt.render(2, 3)
        assert _bitwise(pt.read_accum(), ref) == 0


_CHILD = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {oracle!r})
import numpy as np
import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer
cfg = S.bunny_c2(96, 64, spp=4)
with PathTracer(0) as pt:
    print("LIB", pt.version(), flush=True)
    pt.load(cfg)
    pt.reset_accum()
    pt.render(0, 4)
    got = pt.read_accum()
ref, _ = pyoracle.Oracle(cfg).render(0, 4)
bad = int(np.count_nonzero(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1)))
print("DIFFERING", bad, flush=True)
"""


def test_moot_rays_are_skipped_and_counted():
    """The census build (build.py DIAG_VARIANTS "stats") counts, per bounce, the
    light, env and last-bounce continuation rays its setup found moot: on C2
    (lights, env, depth 4) all three kinds occur, bounce 0 (gen: no test) has
    none, and the image still equals the oracle's."""
    import os
    import re
    import subprocess
    import sys
    from pnraytracing_amd import build
    lib = build.variant_path("stats")
    assert os.path.exists(lib), "variants/libpnrt_stats.so not built (__graft_entry__.build())"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _CHILD.format(repo=repo, oracle=os.path.join(repo, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PNRT_DEVICE_LIB=lib),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "DIAGNOSTIC" in r.stdout and "DIFFERING 0" in r.stdout, r.stdout[-1000:]
    moot = {int(m.group(1)): tuple(map(int, m.group(2, 3, 4))) for m in
            re.finditer(r"\[trace moot\] bounce (\d+) light=(\d+) env=(\d+) cont=(\d+)", r.stderr)}
    assert sorted(moot) == [0, 1, 2, 3], r.stderr[-2000:]
    assert moot[0] == (0, 0, 0)
    assert sum(v[0] for v in moot.values()) > 0 and sum(v[1] for v in moot.values()) > 0
    assert moot[3][2] > 0 and all(moot[b][2] == 0 for b in (1, 2))
