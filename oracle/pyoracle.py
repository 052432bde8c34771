"""oracle/pyoracle.py -- TEST INFRASTRUCTURE: ctypes wrapper of liboracle.so
(the CPU restatement of shaders/ray_tracing.comp in pn_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, always as the checker / CPU baseline, never as the thing measured.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
MAXTEX = 20


class Scene(ctypes.Structure):
    _fields_ = [
        ("vertices", ctypes.c_void_p), ("n_vertices", ctypes.c_int),
        ("materials", ctypes.c_void_p), ("n_materials", ctypes.c_int),
        ("triangles", ctypes.c_void_p), ("n_triangles", ctypes.c_int),
        ("nodes", ctypes.c_void_p), ("n_nodes", ctypes.c_int),
        ("lights", ctypes.c_void_p), ("n_lights", ctypes.c_int),
        ("lights_sum_area", ctypes.c_float),
        ("n_textures", ctypes.c_int),
        ("tex_data", ctypes.c_void_p * MAXTEX),
        ("tex_w", ctypes.c_int * MAXTEX), ("tex_h", ctypes.c_int * MAXTEX), ("tex_ch", ctypes.c_int * MAXTEX),
        ("has_hdr", ctypes.c_int), ("hdr_w", ctypes.c_int), ("hdr_h", ctypes.c_int),
        ("hdr_rgb", ctypes.c_void_p), ("random_hdr", ctypes.c_void_p),
    ]


class Frame(ctypes.Structure):
    _fields_ = [("eye", ctypes.c_float * 3), ("lower_left", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3),
                ("width", ctypes.c_int), ("height", ctypes.c_int), ("max_bounce_depth", ctypes.c_int)]


STAT_FIELDS = ["samples", "node_pops", "sibling_tests", "tri_tests", "tri_hits", "material_fetches",
               "light_probes", "light_samples", "env_samples", "env_lookups", "albedo_bytes", "accum_rmw",
               "traversals"]
PRIM_FIELDS = ["prim_node_pops", "prim_sibling_tests", "prim_tri_tests", "prim_tri_hits"]


class Stats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in STAT_FIELDS] + [("stack_overflow", ctypes.c_int)] + \
               [(f, ctypes.c_uint64) for f in PRIM_FIELDS]

    def as_dict(self):
        d = {f: int(getattr(self, f)) for f in STAT_FIELDS + PRIM_FIELDS}
        d["stack_overflow"] = int(self.stack_overflow)
        return d


# bytes of reference-layout records touched per access (no cache reuse)
BYTES = {"node_pops": 48, "sibling_tests": 24, "tri_tests": 60, "tri_hits": 60, "material_fetches": 72,
         "light_probes": 12, "light_samples": 96, "env_samples": 96, "env_lookups": 48, "accum_rmw": 32}


def algorithmic_bytes(stats: dict) -> int:
    return sum(stats[k] * v for k, v in BYTES.items()) + stats["albedo_bytes"]


TRAVERSAL = ("node_pops", "sibling_tests", "tri_tests")


def bounce_traversal_bytes(stats: dict) -> int:
    """Algorithmic bytes of the bounce rays' traversals (every BVHIntersect /
    BVHIntersectP except the camera ray's): node pops, sibling pre-tests and
    triangle tests of the SURVEY 8d table.  This is the work of the GPU's
    per-bounce traversal kernel; the closest hit's attribute fetch (+60 B)
    happens in its shade/setup kernels and is not included."""
    return sum((stats[k] - stats["prim_" + k]) * BYTES[k] for k in TRAVERSAL)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB)
        L.pno_render.restype = ctypes.c_int
        L.pno_render.argtypes = [ctypes.POINTER(Scene), ctypes.POINTER(Frame), ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.POINTER(Stats)]
        L.pno_math_eval.restype = None
        L.pno_math_eval.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.pno_wang_hash.restype = ctypes.c_uint32
        L.pno_wang_hash.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.pno_intersect.restype = ctypes.c_int
        L.pno_intersect.argtypes = [ctypes.POINTER(Scene), ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.pno_sobol.restype = ctypes.c_float
        L.pno_sobol.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        _lib = L
    return _lib


def gl_unpacked(pixels: np.ndarray, w: int, h: int, ch: int) -> np.ndarray:
    """The bytes glTexImage2D reads from stbi's tightly packed buffer with the
    default GL_UNPACK_ALIGNMENT 4: row j starts at j*align4(w*ch); bytes past
    the caller's buffer are taken as 0 (same rule as pnrt_upload_texture)."""
    src = np.ascontiguousarray(pixels, np.uint8).reshape(-1)
    stride = (w * ch + 3) & ~3
    out = np.zeros(stride * h, np.uint8)
    n = min(len(src), len(out))
    out[:n] = src[:n]
    return out


class Oracle:
    """Holds a scene (reference-layout arrays) for repeated CPU renders."""

    def __init__(self, cfg):
        self.cfg = cfg
        p = cfg.packed
        self._keep = []

        def ptr(a, dt=np.float32):
            if a is None or len(a) == 0:
                return None
            a = np.ascontiguousarray(a, dt)
            self._keep.append(a)
            return a.ctypes.data

        s = Scene()
        s.vertices, s.n_vertices = ptr(p.vertices), len(p.vertices)
        s.materials, s.n_materials = ptr(p.materials), len(p.materials)
        s.triangles, s.n_triangles = ptr(p.triangles), len(p.triangles)
        s.nodes, s.n_nodes = ptr(p.nodes), len(p.nodes)
        s.lights, s.n_lights = ptr(p.lights), len(p.lights)
        s.lights_sum_area = p.lights_sum_area
        s.n_textures = len(cfg.textures)
        for i, (px, w, h, ch) in enumerate(cfg.textures):
            s.tex_data[i] = ptr(gl_unpacked(px, w, h, ch), np.uint8)
            s.tex_w[i], s.tex_h[i], s.tex_ch[i] = w, h, ch
        if cfg.env_rgb is not None:
            s.has_hdr = 1
            s.hdr_h, s.hdr_w = cfg.env_rgb.shape[:2]
            s.hdr_rgb = ptr(cfg.env_rgb)
            s.random_hdr = ptr(cfg.env_table)
        self.scene = s
        f = Frame()
        cam = np.asarray(cfg.camera, np.float32).reshape(4, 3)
        f.eye[:], f.lower_left[:], f.horizontal[:], f.vertical[:] = (list(map(float, r)) for r in cam)
        f.width, f.height, f.max_bounce_depth = cfg.width, cfg.height, cfg.max_depth
        self.frame = f

    def render(self, first_frame: int, n_frames: int, rows=None, accum: np.ndarray | None = None,
               threads: int = 0, y_step: int = 1):
        """Render rows [y0, y1) (step y_step) of frames first..first+n-1 into accum
        (H, W, 4) float32; returns (accum, stats dict)."""
        W, Hh = self.cfg.width, self.cfg.height
        if accum is None:
            accum = np.zeros((Hh, W, 4), np.float32)
        y0, y1 = (0, Hh) if rows is None else rows
        st = Stats()
        rc = lib().pno_render(ctypes.byref(self.scene), ctypes.byref(self.frame), first_frame, n_frames,
                              y0, y1, y_step, accum.ctypes.data, threads, ctypes.byref(st))
        if rc != 0:
            raise RuntimeError(f"pno_render failed ({rc})")
        return accum, st.as_dict()

    def intersect(self, rays: np.ndarray, kind: int, sem: int, idx: np.ndarray | None = None,
                  threads: int = 0) -> np.ndarray:
        """The oracle's intersection routines on caller rays (pn_oracle.h
        pno_intersect): rays (n, 7) float32 = origin, dir, tMax; kind 0 closest
        hit, 1 any hit, 2/3 triangle idx[i], 4 box of node idx[i]; sem 0 = the
        GLSL's rules, 1 = the reference CPU headers' rules.  Returns (n, 13) u32."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 7)
        n = len(rays)
        out = np.zeros((n, 13), np.uint32)
        ip = None
        if idx is not None:
            idx = np.ascontiguousarray(idx, np.int32)
            assert len(idx) == n
            ip = idx.ctypes.data
        rc = lib().pno_intersect(ctypes.byref(self.scene), rays.ctypes.data, n, kind, sem, ip, out.ctypes.data,
                                 threads)
        if rc != 0:
            raise RuntimeError(f"pno_intersect failed ({rc})")
        return out


def math_eval(fn: int, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
    a = np.ascontiguousarray(a, np.float32)
    out = np.empty_like(a)
    bb = None if b is None else np.ascontiguousarray(b, np.float32)
    lib().pno_math_eval(fn, a.ctypes.data, None if bb is None else bb.ctypes.data, out.ctypes.data, len(a))
    return out
