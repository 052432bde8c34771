"""Interactive loop pieces: the camera controls against
golden states produced by the reference's own camera.hpp
(tests/golden/make_camera_golden.py), and the redraw / frameCount rule of
main.cpp:589-628 on the GPU against the CPU oracle."""
import json
import os

import numpy as np
import pytest

from pnraytracing_amd.session import CameraController, InteractiveSession

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "camera_controls.json")


def test_camera_controls_match_reference_camera_hpp():
    g = json.load(open(GOLDEN))
    inits = iter(g["init"])
    cam = None
    for (kind, a, b), want in zip(g["ops"], g["states"]):
        if kind == 0:
            v = [float.fromhex(t) if t.startswith("0x") else float(t) for t in next(inits).split()]
            cam = CameraController(v[0:3], v[3:6], v[6:9], v[9], v[10])
        elif kind == 1:
            cam.rotate(a, b)
        elif kind == 2:
            cam.translate(-a, b)            # the callback passes -dx (main.cpp:131)
        else:
            cam.zoom(a)
        exp = np.array([float.fromhex(t) for t in want], np.float32)
        got = cam.record()
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (kind, a, b, got, exp)


def test_camera_rejections():
    cam = CameraController((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, 1.0)
    assert not cam.zoom(50.0) and cam.state.fov_deg == 45.0        # fov must stay in (1, 89)
    assert cam.zoom(-2.0) and cam.state.fov_deg == 43.0
    before = cam.record()
    assert not cam.rotate(0.0, 149.9)                               # |up . nv| > 0.9995
    assert np.array_equal(before, cam.record())


@pytest.mark.gpu
def test_redraw_sequence_matches_oracle():
    """frames: still x2, drag (redraw) x2, still x3 -- the accumulation image after
    every frame equals the oracle replaying the same uniforms."""
    import pyoracle
    from pnraytracing_amd import scenes
    from pnraytracing_amd.tracer import PathTracer

    W, H = 64, 48
    cfg = scenes.bunny_c2(W, H, spp=1, nu=24, nv=12)
    cam = CameraController((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, np.float32(W) / np.float32(H))
    orc = pyoracle.Oracle(cfg)
    acc = np.zeros((H, W, 4), np.float32)
    with PathTracer(0) as pt:
        pt.load(cfg)
        sess = InteractiveSession(pt, W, H, cam)
        for step, redraw in enumerate([False, False, True, True, False, False, False]):
            if redraw:
                cam.rotate(3.0, -1.0)
            depth, _ = sess.frame(redraw)
            fc = 0 if redraw else sess.frame_count - 1
            u = cam.uniforms()
            f = orc.frame
            f.eye[:], f.lower_left[:], f.horizontal[:], f.vertical[:] = (list(map(float, r)) for r in u)
            f.max_bounce_depth = depth
            orc.render(fc, 1, accum=acc)
            got = pt.read_accum()
            bad = int(np.count_nonzero(np.any(got.view(np.uint32) != acc.view(np.uint32), axis=-1)))
            assert bad == 0, f"frame {step} (redraw={redraw}): {bad} pixels differ"
        assert sess.frame_count == 3
