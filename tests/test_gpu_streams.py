"""pnrt_set_stream never touches the previous stream: a caller
stream that has been destroyed before the switch away from it is safe, and the
frame-ordered blends of calls on either side of switches still equal the
oracle bit for bit.  The raw hipStream_t comes from libamdhip64 through ctypes
(no torch stream pool in between)."""
import ctypes

import numpy as np
import pytest

import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer

pytestmark = pytest.mark.gpu


def _hip():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return hip


def test_switch_away_from_destroyed_stream():
    hip = _hip()
    cfg = S.cornell_c1(96, 80)
    ref, _ = pyoracle.Oracle(cfg).render(0, 6)
    with PathTracer(0) as pt:
        pt.load(cfg)
        s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s1)) == 0 and hip.hipStreamCreate(ctypes.byref(s2)) == 0
        pt.set_stream(s1.value)
        pt.render(0, 2)                     # frames 0-1 blended on s1
        pt.set_stream(s2.value)             # s2 after s1's last op
        pt.render(2, 2)
        assert hip.hipStreamSynchronize(s2) == 0
        assert hip.hipStreamDestroy(s1) == 0     # the caller drops the old stream ...
        pt.set_stream(None)                 # ... and switches from s2 (alive) back to the context stream
        pt.render(4, 1)
        pt.set_stream(s2.value)
        assert hip.hipStreamSynchronize(s2) == 0
        assert hip.hipStreamDestroy(s2) == 0     # destroyed while current (nothing queued on it since)
        pt.set_stream(None)                 # switching away from a destroyed stream touches nothing
        pt.render(5, 1)
        got = pt.read_accum()
    bad = np.argwhere(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1))
    assert len(bad) == 0, f"{len(bad)} pixels differ"


def test_v1_kernel_then_stream_switch():
    """The v1 kernel accumulates on the context's stream directly; a stream switch
    right after it (no synchronisation) must order the next frames after it
    (every op queued on the stream records the context's last event)."""
    from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_ZCULL
    hip = _hip()
    cfg = S.cornell_c1(96, 80)
    ref, _ = pyoracle.Oracle(cfg).render(0, 6)
    with PathTracer(0) as pt:
        pt.load(cfg)
        pt.set_options(TRAVERSE_ZCULL | KERNEL_V1)
        s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s1)) == 0 and hip.hipStreamCreate(ctypes.byref(s2)) == 0
        pt.set_stream(s1.value)
        pt.render(0, 3)                     # v1: frames 0-2 blended in-kernel on s1
        pt.set_stream(s2.value)             # no synchronisation in between
        pt.render(3, 3)
        pt.set_stream(None)
        got = pt.read_accum()
        assert hip.hipStreamSynchronize(s1) == 0 and hip.hipStreamSynchronize(s2) == 0
        assert hip.hipStreamDestroy(s1) == 0 and hip.hipStreamDestroy(s2) == 0
    bad = np.argwhere(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1))
    assert len(bad) == 0, f"{len(bad)} pixels differ"
