"""Headless replacement of main.cpp's interactive render loop (main.cpp:573-630).

``CameraController`` is ``Camera`` (camera.hpp:4-77) with the controls the
mouse callbacks call (main.cpp:96-142), glm-exact in libpnrt_host.so.
``InteractiveSession.frame(redraw)`` is one loop iteration: when the scene or
camera is being changed (the GUI combo, a pressed mouse button or a scroll
event, main.cpp:592) the frame is rendered with MAX_BOUNCE_DEPTH 1 and
frameCount 0 -- the progressive mean then overwrites the image (a = 1/(0+1)) --
and the counter is not advanced (main.cpp:628); otherwise MAX_BOUNCE_DEPTH 4
and frameCount, then ++frameCount.  All rendering goes through libpnrt.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N


class CameraState(ctypes.Structure):
    _fields_ = [("eye", ctypes.c_float * 3), ("center", ctypes.c_float * 3), ("up", ctypes.c_float * 3),
                ("fov_deg", ctypes.c_float), ("aspect", ctypes.c_float),
                ("u", ctypes.c_float * 3), ("v", ctypes.c_float * 3), ("w", ctypes.c_float * 3),
                ("distance", ctypes.c_float),
                ("lower_left", ctypes.c_float * 3), ("horizontal", ctypes.c_float * 3),
                ("vertical", ctypes.c_float * 3)]


def _lib():
    lib = N.host_lib()
    if not getattr(lib, "_pnrt_cam_typed", False):
        P = ctypes.POINTER(CameraState)
        for name, args in (("pnrt_camera_state_init", [P, N.F, N.F, N.F, ctypes.c_float, ctypes.c_float]),
                           ("pnrt_camera_rotate", [P, ctypes.c_float, ctypes.c_float]),
                           ("pnrt_camera_translate", [P, ctypes.c_float, ctypes.c_float]),
                           ("pnrt_camera_zoom", [P, ctypes.c_float])):
            fn = getattr(lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = args
        lib._pnrt_cam_typed = True
    return lib


class CameraController:
    """``Camera`` + its interactive controls (camera.hpp:33-65)."""

    def __init__(self, eye, center, up, fov_deg: float, aspect: float):
        self.state = CameraState()
        a = [np.ascontiguousarray(v, np.float32) for v in (eye, center, up)]
        rc = _lib().pnrt_camera_state_init(ctypes.byref(self.state), *(N.fptr(x) for x in a),
                                           ctypes.c_float(fov_deg), ctypes.c_float(aspect))
        if rc < 0:
            raise ValueError("camera_state_init failed")

    def rotate(self, dx: float, dy: float) -> bool:        # left-button drag (main.cpp:127-129)
        return _lib().pnrt_camera_rotate(ctypes.byref(self.state), dx, dy) == 1

    def translate(self, dx: float, dy: float) -> bool:     # right-button drag: UpdateTranslateUV(-dx, dy)
        return _lib().pnrt_camera_translate(ctypes.byref(self.state), -dx, dy) == 1

    def zoom(self, yoffset: float) -> bool:                # scroll (main.cpp:139-142)
        return _lib().pnrt_camera_zoom(ctypes.byref(self.state), yoffset) == 1

    def uniforms(self) -> np.ndarray:
        """(4, 3): camera.eye, lowerLeftCorner, horizontal, vertical (main.cpp:606-610)."""
        s = self.state
        return np.array([list(s.eye), list(s.lower_left), list(s.horizontal), list(s.vertical)], np.float32)

    def record(self) -> np.ndarray:
        """All 31 floats of the state (eye center up fov aspect u v w distance llc hor ver)."""
        s = self.state
        return np.array([*s.eye, *s.center, *s.up, s.fov_deg, s.aspect, *s.u, *s.v, *s.w, s.distance,
                         *s.lower_left, *s.horizontal, *s.vertical], np.float32)


class InteractiveSession:
    """main.cpp:573-630 without the window: one ``frame()`` per loop iteration."""

    def __init__(self, tracer, width: int, height: int, camera: CameraController, max_bounce_depth: int = 4):
        self.pt = tracer
        self.width, self.height = width, height
        self.camera = camera
        self.max_bounce_depth = max_bounce_depth
        self.frame_count = 0

    def frame(self, redraw: bool = False, band: int = 1, n_shards: int = 1, shard: int = 0):
        if redraw:                                   # main.cpp:592-596
            depth = 1
            self.frame_count = 0
        else:                                        # main.cpp:597-601
            depth = self.max_bounce_depth
        self.pt.set_frame(self.width, self.height, self.camera.uniforms(), depth)
        self.pt.render(self.frame_count, 1, band, n_shards, shard)   # main.cpp:612-613
        if not redraw:                               # main.cpp:628
            self.frame_count += 1
        return depth, self.frame_count
