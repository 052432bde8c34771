"""GPU parity at the BASELINE configurations' FULL sizes (BASELINE.json
configs[1..4]), against the CPU oracle and through size-independent
properties.

* C2 (1920x1080, 4 spp, the bench frame): every pixel vs the oracle.
* C3 (1920x1080, textured figure + metal boards + env: albedo textures,
  every Disney lobe): every pixel vs the oracle.
* C4 (1920x1080, teapot + area light + env: all three pdfs active): every
  pixel vs the oracle.
* C5 (3840x2160, 4.19M triangles, 4k env): every pixel vs the oracle.
* C4 / C5: EXACT = ZCULL = v1 kernels on every pixel; the union of the 8
  row-band shards of the 8-GPU split (one pnrt_render call per
  shard as each rank makes it) = the single-call frame, bit for bit.
* A frame too large for two per batch (8192x4320: one frame per batch) vs
  the oracle on a row subset.
* pnrt_set_stream between pipelined calls keeps the blends in frame order.

Tolerance: 0 ulp (bit-exact) throughout.
"""
import numpy as np
import pytest

import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL, PathTracer

pytestmark = pytest.mark.gpu

_cache = {}


def cfg(name):
    if name not in _cache:
        _cache[name] = S.CONFIGS[name]()
    return _cache[name]


@pytest.fixture(scope="module")
def pt():
    t = PathTracer(0)
    yield t
    t.close()


def gpu_render(pt, c, first, n, mode=TRAVERSE_ZCULL, shard=(1, 1, 0), load=True):
    if load:
        pt.load(c, mode)
    else:
        pt.set_options(mode)
    pt.reset_accum()
    pt.render(first, n, *shard)
    return pt.read_accum()


def assert_bitwise(got, ref, what):
    g, r = got.view(np.uint32), ref.view(np.uint32)
    bad = np.argwhere(np.any(g != r, axis=-1))
    assert len(bad) == 0, f"{what}: {len(bad)} pixels differ, first {bad[:5].tolist()} " \
                          f"gpu={got[tuple(bad[0])]} oracle={ref[tuple(bad[0])]}"


def test_c2_whole_frame_bitwise(pt):
    """The bench frame itself: 1920x1080 x 4 spp (8.3M samples), every pixel."""
    c = cfg("C2")
    got = gpu_render(pt, c, 0, 4)
    ref, st = pyoracle.Oracle(c).render(0, 4)
    assert st["stack_overflow"] == 0
    assert_bitwise(got, ref, "C2 1920x1080 whole frame")


def test_c3_whole_frame_bitwise(pt):
    """C3 at its full 1920x1080 x 4 spp, every pixel: albedo textures (RGBA
    2048x1024 and an odd-width RGB one, GL unpack alignment), every Disney
    lobe, the env (it was checked on every 45th row only)."""
    c = cfg("C3")
    got = gpu_render(pt, c, 0, 4)
    ref, st = pyoracle.Oracle(c).render(0, 4)
    assert st["albedo_bytes"] > 0 and st["env_samples"] > 0 and st["stack_overflow"] == 0
    assert_bitwise(got, ref, "C3 1920x1080 whole frame")


def test_c4_whole_frame_bitwise(pt):
    """C4 at its full 1920x1080 (frames 4..7: Sobol indices past the first
    iteration), every pixel; the light, env and BSDF pdfs are all active."""
    c = cfg("C4")
    got = gpu_render(pt, c, 4, 4)
    ref, st = pyoracle.Oracle(c).render(4, 4)
    assert st["light_samples"] > 0 and st["env_samples"] > 0
    assert_bitwise(got, ref, "C4 1920x1080 whole frame")


def test_c5_whole_frame_bitwise(pt):
    """C5 at its full 3840x2160 with the 4.19M-triangle BVH and the 4k env:
    every pixel (33.2M samples) vs the oracle (it was every 16th
    row; the oracle takes ~25 s on the box's 16 CPUs)."""
    c = cfg("C5")
    got = gpu_render(pt, c, 0, 4)
    ref, st = pyoracle.Oracle(c).render(0, 4)
    assert st["stack_overflow"] == 0
    assert_bitwise(got, ref, "C5 3840x2160 whole frame")
    assert np.isfinite(got).all() and (got[..., 3] == 1).all()


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_fullsize_traversal_modes_agree(pt, name):
    """z-slab culling and the v1 one-lane-per-pixel kernel give the wavefront
    EXACT image on every pixel at full size."""
    c = cfg(name)
    a = gpu_render(pt, c, 0, 4, TRAVERSE_EXACT)
    b = gpu_render(pt, c, 0, 4, TRAVERSE_ZCULL, load=False)
    assert_bitwise(b, a, f"{name}: zcull vs exact")
    v1 = gpu_render(pt, c, 0, 4, TRAVERSE_ZCULL | KERNEL_V1, load=False)
    assert_bitwise(v1, a, f"{name}: v1 vs wavefront")


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_fullsize_eight_shards_union_equals_full(pt, name):
    """The 8-GPU split (8-row bands dealt to 8 ranks): each shard as
    its own pnrt_render call into one accumulation image equals the
    single-call frame bit for bit, so the gathered image of 8 ranks does."""
    c = cfg(name)
    full = gpu_render(pt, c, 0, 4)
    pt.reset_accum()
    for s in range(8):
        pt.render(0, 4, 8, 8, s)
    assert_bitwise(pt.read_accum(), full, f"{name}: union of 8 shards")


def test_one_frame_per_batch_vs_oracle(pt):
    """8192x4320 frames exceed two per batch, so this call renders one frame per
    batch (three batches in one call); rows vs the oracle."""
    c = S.bunny_c2(8192, 4320)
    got = gpu_render(pt, c, 0, 3)
    rows = np.arange(270, c.height, 540)
    ref = np.zeros_like(got)
    pyoracle.Oracle(c).render(0, 3, rows=(270, c.height), y_step=540, accum=ref)
    assert_bitwise(got[rows], ref[rows], "8192x4320 one frame per batch")


def test_set_stream_between_pipelined_calls(pt):
    """pnrt_set_stream while calls are in flight: the blends (progressive mean,
    frame order) continue after the old stream's, so the image equals a
    single-stream render bit for bit."""
    import torch
    c = S.bunny_c2(320, 180)
    ref = gpu_render(pt, c, 0, 8)
    s2 = torch.cuda.Stream()
    pt.reset_accum()
    pt.render(0, 2)
    pt.render(2, 2)
    pt.set_stream(s2.cuda_stream)          # no synchronisation in between
    pt.render(4, 2)
    pt.set_stream(None)                    # back to the context's own stream
    pt.render(6, 2)
    assert_bitwise(pt.read_accum(), ref, "stream switches mid-sequence")


def test_batch_beyond_2_26_paths(pt):
    """One call of 40 frames of the 1080p C4 frame is ONE batch of 83M paths --
    path entries above 2^26, the 28-bit slot and ray-id fields (pt_wf.h
    WF_SLOT_BITS) -- and equals the same 40 frames rendered as five 8-frame calls
    (batches of 16.6M paths, which the rest of the suite pins to the oracle), bit
    for bit; two of its rows are checked against the oracle as well."""
    c = cfg("C4")
    big = gpu_render(pt, c, 0, 40)
    pt.reset_accum()
    for k in range(5):
        pt.render(8 * k, 8)
    small = pt.read_accum()
    assert_bitwise(big, small, "C4 40 frames: one 83M-path batch vs 8-frame calls")
    o = pyoracle.Oracle(c)
    for y in (0, 701):
        ref, _ = o.render(0, 40, rows=(y, y + 1))
        assert_bitwise(big[y:y + 1], ref[y:y + 1], f"C4 40 frames, row {y}: one batch vs oracle")


def test_batch_bytes_cap(pt):
    """PNRT_BATCH_BYTES (read when a context first renders) caps one batch's device
    buffers: a 40-frame C4 call then runs in 14 batches of at most 3 frames
    (≈ 0.64 GB per 1080p frame) and equals the one-batch call bit for bit."""
    import os
    c = cfg("C4")
    one = gpu_render(pt, c, 0, 40)
    os.environ["PNRT_BATCH_BYTES"] = str(3 * 10**9)
    capped = PathTracer(0)
    try:
        got = gpu_render(capped, c, 0, 40)
    finally:
        capped.close()
        del os.environ["PNRT_BATCH_BYTES"]
    assert_bitwise(got, one, "C4 40 frames: 3-frame batches (PNRT_BATCH_BYTES) vs one batch")
