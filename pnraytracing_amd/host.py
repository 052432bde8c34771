"""Host-side scene assembly over ``libpnrt_host.so`` (C ABI: ``include/pnrt_host.h``).

Mirrors the reference's host pipeline, producing the SAME flattened arrays
``main.cpp`` uploads:

=====================================  ==========================================
reference                              here
=====================================  ==========================================
``Material`` (PnRT.hpp:66-81)          :class:`Material`
``Model(path, M, material, name)``    :meth:`SceneBuilder.add_model`
``ModelOutput`` (model.hpp:101-135)    native ``pnrt_scene_add_mesh``
``BVH`` ctor / ``BuildBVH``            :meth:`SceneBuilder.build` (native)
light list (main.cpp:374-383)          :meth:`SceneBuilder.build` (native)
packing loops (main.cpp:409-524)       :class:`PackedScene`
``Camera::UpdateCamera``               :func:`camera_update`
``LoadHDRImage`` (shader.hpp:126-225)  :func:`load_hdr` / :func:`hdr_table`
=====================================  ==========================================
"""
from __future__ import annotations

import ctypes
import time
import dataclasses
from typing import Sequence

import numpy as np

from . import _native as N


class HostError(RuntimeError):
    pass


def _check(rc: int, what: str):
    if rc < 0:
        raise HostError(f"{what} failed ({rc}): {N.host_lib().pnrt_host_last_error().decode()}")
    return rc


@dataclasses.dataclass
class Material:
    """``Material`` with the reference defaults (PnRT.hpp:66-81)."""
    emssive: Sequence[float] = (0.0, 0.0, 0.0)
    baseColor: Sequence[float] = (0.8, 0.8, 0.8)
    subsurface: float = 0.0
    metallic: float = 0.0
    specular: float = 0.0
    specularTint: float = 0.0
    roughness: float = 0.5
    anisotropic: float = 0.0
    sheen: float = 0.0
    sheenTint: float = 0.0
    clearcoat: float = 0.0
    clearcoatGloss: float = 0.0
    IOR: float = 1.0
    transmission: float = 0.0

    def pack(self) -> np.ndarray:
        """18 floats in main.cpp:438-456 order (double literals -> float as glm does)."""
        return np.array([*self.emssive, *self.baseColor, self.subsurface, self.metallic,
                         self.specular, self.specularTint, self.roughness, self.anisotropic,
                         self.sheen, self.sheenTint, self.clearcoat, self.clearcoatGloss,
                         self.IOR, self.transmission], dtype=np.float32)

    def copy(self, **kw) -> "Material":
        return dataclasses.replace(self, **kw)


@dataclasses.dataclass
class Mesh:
    """One Assimp mesh in model space (model.hpp:131-178): unshared vertices."""
    positions: np.ndarray            # (nv, 3) float32
    normals: np.ndarray | None       # (nv, 3) float32
    texcoords: np.ndarray | None     # (nv, 2) float32
    indices: np.ndarray              # (nt*3,) int32

    @property
    def n_triangles(self) -> int:
        return len(self.indices) // 3


def translate(x, y, z):
    return (0, 0.0, (float(x), float(y), float(z)))


def rotate(deg, ax, ay, az):
    return (1, float(deg), (float(ax), float(ay), float(az)))


def scale(x, y=None, z=None):
    y = x if y is None else y
    z = x if z is None else z
    return (2, 0.0, (float(x), float(y), float(z)))


def model_matrix(ops) -> np.ndarray:
    """glm::translate(mat4(1),..) * glm::rotate(mat4(1),..) * glm::scale(mat4(1),..)
    evaluated with glm's float operation order (column-major 16 floats)."""
    arr = (N.Xform * len(ops))()
    for i, (k, a, v) in enumerate(ops):
        arr[i].kind = k
        arr[i].angle_deg = a
        arr[i].v[:] = v
    out = np.zeros(16, np.float32)
    _check(N.host_lib().pnrt_model_matrix(arr, len(ops), N.fptr(out)), "pnrt_model_matrix")
    return out


def camera_update(eye, center, up, fov: float, aspect: float) -> np.ndarray:
    """Camera::UpdateCamera (camera.hpp:11-31) -> (eye, llc, horizontal, vertical)."""
    f = lambda v: np.asarray(v, np.float32)  # noqa: E731
    e, c, u = f(eye), f(center), f(up)
    out = np.zeros(12, np.float32)
    _check(N.host_lib().pnrt_camera_update(N.fptr(e), N.fptr(c), N.fptr(u), float(np.float32(fov)),
                                           float(np.float32(aspect)), N.fptr(out)), "camera_update")
    return out.reshape(4, 3)


def decode_rgbe(data: bytes) -> np.ndarray:
    """stbi_loadf on a Radiance .hdr (3 channels, row 0 = first scanline)."""
    buf = np.frombuffer(data, np.uint8).copy()
    w, h = ctypes.c_int(), ctypes.c_int()
    lib = N.host_lib()
    _check(lib.pnrt_hdr_decode_rgbe(N.u8ptr(buf), len(buf), ctypes.byref(w), ctypes.byref(h), None), "rgbe header")
    out = np.zeros((h.value, w.value, 3), np.float32)
    _check(lib.pnrt_hdr_decode_rgbe(N.u8ptr(buf), len(buf), ctypes.byref(w), ctypes.byref(h), N.fptr(out)), "rgbe decode")
    return out


def hdr_table(rgb: np.ndarray) -> np.ndarray:
    """LoadHDRImage's RandomHDR inverse-CDF table (shader.hpp:145-203)."""
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    out = np.zeros((h, w, 3), np.float32)
    _check(N.host_lib().pnrt_hdr_build_table(N.fptr(rgb), w, h, N.fptr(out)), "hdr_table")
    return out


def load_hdr(path: str) -> tuple[np.ndarray, np.ndarray]:
    with open(path, "rb") as f:
        rgb = decode_rgbe(f.read())
    return rgb, hdr_table(rgb)


def synthetic_hdr(w: int, h: int, seed: int = 0x5EED) -> np.ndarray:
    out = np.zeros((h, w, 3), np.float32)
    _check(N.host_lib().pnrt_hdr_synthetic(w, h, seed, N.fptr(out)), "hdr_synthetic")
    return out


def _mesh_from(fn, *args) -> Mesh:
    nv, nt = ctypes.c_int(), ctypes.c_int()
    _check(fn(*args, None, None, None, None, ctypes.byref(nv), ctypes.byref(nt)), fn.__name__)
    P = np.zeros((nv.value, 3), np.float32)
    Nn = np.zeros((nv.value, 3), np.float32)
    T = np.zeros((nv.value, 2), np.float32)
    idx = np.zeros(nt.value * 3, np.int32)
    _check(fn(*args, N.fptr(P), N.fptr(Nn), N.fptr(T), N.iptr(idx), ctypes.byref(nv), ctypes.byref(nt)), fn.__name__)
    return Mesh(P, Nn, T, idx)


def mesh_quad(half: float = 27.5) -> Mesh:
    """floor.obj stand-in: 2-triangle quad in XZ (|x|,|z| <= half), normal +Y."""
    return _mesh_from(N.host_lib().pnrt_mesh_quad, ctypes.c_float(half))


def mesh_displaced_sphere(nu: int, nv: int, radius: float, center, amp: float, seed: int) -> Mesh:
    c = np.asarray(center, np.float32)
    return _mesh_from(N.host_lib().pnrt_mesh_displaced_sphere, nu, nv, ctypes.c_float(radius),
                      N.fptr(c), ctypes.c_float(amp), ctypes.c_uint32(seed))


def mesh_teapot() -> Mesh:
    return _mesh_from(N.host_lib().pnrt_mesh_teapot)


def bvh_build_cpu(tri_bounds: np.ndarray):
    """Host BuildBVH (BVH.hpp:92-173) over bare (n, 9) bounds: (nodes, order, max_depth),
    the same contract as :meth:`pnraytracing_amd.tracer.PathTracer.build_bvh`."""
    tb = np.ascontiguousarray(tri_bounds, np.float32).reshape(-1, 9)
    n = len(tb)
    cap = max(2 * n - 1, 1)
    nodes = np.empty((cap, 12), np.float32)
    order = np.empty(n, np.int32)
    nn, md = ctypes.c_int(), ctypes.c_int()
    _check(N.host_lib().pnrt_bvh_build_cpu(N.fptr(tb), n, N.fptr(nodes), cap, ctypes.byref(nn), N.iptr(order),
                                           ctypes.byref(md)), "bvh_build_cpu")
    return nodes[:nn.value].copy(), order, md.value


@dataclasses.dataclass
class PackedScene:
    """The five arrays main.cpp uploads (texture units 0-4) + uniforms."""
    vertices: np.ndarray     # (nv, 15)
    materials: np.ndarray    # (nm, 18)
    triangles: np.ndarray    # (nt, 6)
    nodes: np.ndarray        # (nn, 12)
    lights: np.ndarray       # (nl, 3)
    lights_sum_area: float
    max_depth: int
    # BuildBVH's input (per-triangle Bound + boundCenter, (n, 9)) and how long the
    # build took (seconds; host pnrt_scene_build or GPU pnrt_bvh_build incl. PCIe)
    tri_bounds: np.ndarray | None = None
    bvh_seconds: float = 0.0
    bvh_by: str = "host"

    def arrays(self):
        return self.vertices, self.materials, self.triangles, self.nodes, self.lights


class SceneBuilder:
    """Model list -> ModelOutput -> BuildBVH -> light list -> packed arrays."""

    def __init__(self):
        self._lib = N.host_lib()
        self._s = self._lib.pnrt_scene_create()
        self.models: list[tuple[str, int]] = []

    def __del__(self):
        if getattr(self, "_s", None):
            self._lib.pnrt_scene_destroy(self._s)
            self._s = None

    def add_material(self, m: Material) -> int:
        return _check(self._lib.pnrt_scene_add_material(self._s, N.fptr(m.pack())), "add_material")

    def add_model(self, meshes: Mesh | Sequence[Mesh], ops, material: Material, name: str = "",
                  texture_ids: Sequence[int] | None = None) -> int:
        """``Model(path, modelMatrix, material, name)``: registers the material
        (model.hpp:112-113) and appends every mesh (ModelOutput)."""
        if isinstance(meshes, Mesh):
            meshes = [meshes]
        mat_id = self.add_material(material)
        M = model_matrix(ops)
        for k, mesh in enumerate(meshes):
            tex = -1 if texture_ids is None else int(texture_ids[k])
            P = np.ascontiguousarray(mesh.positions, np.float32)
            Nn = None if mesh.normals is None else np.ascontiguousarray(mesh.normals, np.float32)
            T = None if mesh.texcoords is None else np.ascontiguousarray(mesh.texcoords, np.float32)
            idx = np.ascontiguousarray(mesh.indices, np.int32)
            _check(self._lib.pnrt_scene_add_mesh(self._s, mat_id, tex, N.fptr(M), N.fptr(P), N.fptr(Nn),
                                                 None, None, N.fptr(T), len(P), N.iptr(idx), len(idx)),
                   f"add_mesh({name})")
        self.models.append((name, mat_id))
        return mat_id

    def tri_bounds(self) -> np.ndarray:
        """(n, 9) per-triangle Bound + boundCenter in the current order (BuildBVH's input)."""
        info = N.SceneInfo()
        _check(self._lib.pnrt_scene_get_info(self._s, ctypes.byref(info)), "get_info")
        out = np.zeros((info.n_triangles, 9), np.float32)
        _check(self._lib.pnrt_scene_tri_bounds(self._s, N.fptr(out)), "tri_bounds")
        return out

    def build(self, bvh_tracer=None) -> PackedScene:
        """BuildBVH + light list + packing.  With ``bvh_tracer`` (a
        :class:`pnraytracing_amd.tracer.PathTracer`) the BVH is built on its GPU
        (pnrt_bvh_build) -- the same arrays as the host build, bit for bit."""
        tb = self.tri_bounds()
        t = time.perf_counter()
        if bvh_tracer is None:
            _check(self._lib.pnrt_scene_build(self._s), "scene_build")
        else:
            nodes, order, depth = bvh_tracer.build_bvh(tb)
            _check(self._lib.pnrt_scene_set_bvh(self._s, N.iptr(order), N.fptr(nodes), len(nodes), depth),
                   "scene_set_bvh")
        dt = time.perf_counter() - t
        return dataclasses.replace(self._pack(), tri_bounds=tb, bvh_seconds=dt,
                                   bvh_by="host" if bvh_tracer is None else "gpu")

    def _pack(self) -> PackedScene:
        info = N.SceneInfo()
        _check(self._lib.pnrt_scene_get_info(self._s, ctypes.byref(info)), "get_info")
        V = np.zeros((info.n_vertices, 15), np.float32)
        M = np.zeros((info.n_materials, 18), np.float32)
        T = np.zeros((info.n_triangles, 6), np.float32)
        Nd = np.zeros((info.n_nodes, 12), np.float32)
        L = np.zeros((info.n_lights, 3), np.float32)
        _check(self._lib.pnrt_scene_pack(self._s, N.fptr(V), N.fptr(M), N.fptr(T), N.fptr(Nd),
                                         N.fptr(L) if info.n_lights else None), "scene_pack")
        return PackedScene(V, M, T, Nd, L, float(info.lights_sum_area), int(info.max_depth))
