"""The shape the driver's bench times, against the oracle (VERDICT r3 "What's
weak" 1): C2 at its full 1920x1080, one untimed sizing call, an accumulation
reset, then back-to-back 16-frame pnrt_render calls (33.2M paths each, above
WF_STAGGER_PATHS: staggered calls on two buffer sets and worker streams, the
whole trace grid, each call starting when the previous one has reached its
drain-heavy end through the ev_stage event) -- no synchronisation between them
-- and the progressive mean over
all their frames (ray_tracing.comp:975-991) compared with the oracle on every
36th row, bit for bit.  A second case drives the same shape through the
1-frame calls of the reference's own loop (main.cpp:573-630) at 512x512.

Tolerance: 0 ulp."""
import numpy as np
import pytest

import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer

pytestmark = pytest.mark.gpu

STEP = 36


def _oracle_rows(cfg, frames, step=STEP, offset=0):
    ref = np.zeros((cfg.height, cfg.width, 4), np.float32)
    _, st = pyoracle.Oracle(cfg).render(0, frames, rows=(offset, cfg.height), y_step=step, accum=ref)
    assert st["stack_overflow"] == 0
    return ref, np.arange(offset, cfg.height, step)


def _assert_rows(got, ref, rows, what):
    g, r = got[rows].view(np.uint32), ref[rows].view(np.uint32)
    bad = np.argwhere(np.any(g != r, axis=-1))
    assert len(bad) == 0, f"{what}: {len(bad)} of {len(rows) * got.shape[1]} pixels differ, first (row, x) " \
                          f"{[int(rows[bad[0][0]]), int(bad[0][1])]}"


def test_bench_shape_c2_pipelined_16_frame_calls():
    """bench.py's default C2 run: sizing call, reset, then 16-frame calls
    staggered over two pipes (frames 0..63), rows vs the oracle."""
    cfg = S.bunny_c2()
    with PathTracer(0) as pt:
        pt.load(cfg)
        pt.render(0, 16)                 # the sizing call (every buffer set allocated)
        pt.synchronize()
        pt.reset_accum()
        for k in range(4):               # 4 back-to-back calls: both pipes twice, each waiting on ev_stage
            pt.render(16 * k, 16)
        got = pt.read_accum()
    ref, rows = _oracle_rows(cfg, 64)
    _assert_rows(got, ref, rows, "C2 1080p, four pipelined 16-frame calls")


def test_reference_loop_shape_512_one_frame_calls():
    """The reference's own dispatch shape (D2: 512x512, one 1-spp frame per
    call, main.cpp:613): 48 pipelined calls (small calls: the rotation over the
    buffer sets, primary records reused across calls), rows vs the oracle."""
    cfg = S.bunny_c2(512, 512, spp=1)
    with PathTracer(0) as pt:
        pt.load(cfg)
        for f in range(48):
            pt.render(f, 1)
        got = pt.read_accum()
    ref, rows = _oracle_rows(cfg, 48, step=8, offset=3)
    _assert_rows(got, ref, rows, "512x512 1-frame calls")
