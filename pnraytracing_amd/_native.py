"""Loading of the in-tree native libraries (ctypes; no torch types cross the ABI).

* ``libpnrt.so``      -- HIP device library, C ABI in ``include/pnrt.h``
* ``libpnrt_host.so`` -- host scene library, C ABI in ``include/pnrt_host.h``

Both are built in-tree by :mod:`pnraytracing_amd.build` (``__graft_entry__.build()``).
There is no fallback: if a library is missing or fails to load, the error is
raised to the caller (the product path never substitutes a CPU implementation).
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
DEVICE_LIB = os.environ.get("PNRT_DEVICE_LIB") or os.path.join(PKG_DIR, "libpnrt.so")
HOST_LIB = os.path.join(PKG_DIR, "libpnrt_host.so")

_cache: dict[str, ctypes.CDLL] = {}


class NativeLibraryError(RuntimeError):
    pass


def _load(path: str) -> ctypes.CDLL:
    lib = _cache.get(path)
    if lib is not None:
        return lib
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"{os.path.basename(path)} is not built ({path}); run "
            "`python -c 'import __graft_entry__ as g; g.build()'` first")
    try:
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - surfaced verbatim
        raise NativeLibraryError(f"failed to load {path}: {e}") from e
    _cache[path] = lib
    return lib


def host_lib() -> ctypes.CDLL:
    lib = _load(HOST_LIB)
    if not getattr(lib, "_pnrt_typed", False):
        _type_host(lib)
        lib._pnrt_typed = True
    return lib


def device_lib() -> ctypes.CDLL:
    lib = _load(DEVICE_LIB)
    if not getattr(lib, "_pnrt_typed", False):
        _type_device(lib)
        lib._pnrt_typed = True
    return lib


P = ctypes.c_void_p
F = ctypes.POINTER(ctypes.c_float)
I32 = ctypes.POINTER(ctypes.c_int32)
U8 = ctypes.POINTER(ctypes.c_uint8)
INT = ctypes.c_int
PINT = ctypes.POINTER(ctypes.c_int)


class Xform(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("angle_deg", ctypes.c_float), ("v", ctypes.c_float * 3)]


class SceneInfo(ctypes.Structure):
    _fields_ = [("n_vertices", ctypes.c_int), ("n_materials", ctypes.c_int),
                ("n_triangles", ctypes.c_int), ("n_nodes", ctypes.c_int),
                ("n_lights", ctypes.c_int), ("lights_sum_area", ctypes.c_float),
                ("max_depth", ctypes.c_int)]


class Camera(ctypes.Structure):
    """``pnrt_camera`` (camera.hpp:28-30 uniforms)."""
    _fields_ = [("eye", ctypes.c_float * 3), ("lower_left", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3)]


class DeviceInfo(ctypes.Structure):
    _fields_ = [("n_interior", ctypes.c_int), ("n_triangles", ctypes.c_int),
                ("max_depth", ctypes.c_int), ("device_bytes", ctypes.c_int64),
                ("root_is_leaf", ctypes.c_int), ("stack_limit", ctypes.c_int)]


K_CLASSES = ("primary", "gen", "setup", "trace", "shade", "blend", "v1")   # PNRT_K_* order


class Profile(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double * len(K_CLASSES)), ("launches", ctypes.c_int64 * len(K_CLASSES))]


def _sig(lib, name, res, *args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = list(args)


def _type_host(lib):
    _sig(lib, "pnrt_host_last_error", ctypes.c_char_p)
    _sig(lib, "pnrt_model_matrix", INT, ctypes.POINTER(Xform), INT, F)
    _sig(lib, "pnrt_scene_create", P)
    _sig(lib, "pnrt_scene_destroy", None, P)
    _sig(lib, "pnrt_scene_add_material", INT, P, F)
    _sig(lib, "pnrt_scene_add_mesh", INT, P, INT, INT, F, F, F, F, F, F, INT, I32, INT)
    _sig(lib, "pnrt_scene_build", INT, P)
    _sig(lib, "pnrt_scene_get_info", INT, P, ctypes.POINTER(SceneInfo))
    _sig(lib, "pnrt_scene_pack", INT, P, F, F, F, F, F)
    _sig(lib, "pnrt_scene_tri_bounds", INT, P, F)
    _sig(lib, "pnrt_scene_set_bvh", INT, P, I32, F, INT, INT)
    _sig(lib, "pnrt_bvh_build_cpu", INT, F, INT, F, INT, PINT, I32, PINT)
    _sig(lib, "pnrt_camera_update", INT, F, F, F, ctypes.c_float, ctypes.c_float, F)
    _sig(lib, "pnrt_hdr_decode_rgbe", INT, U8, ctypes.c_int64, PINT, PINT, F)
    _sig(lib, "pnrt_hdr_build_table", INT, F, INT, INT, F)
    _sig(lib, "pnrt_mesh_quad", INT, ctypes.c_float, F, F, F, I32, PINT, PINT)
    _sig(lib, "pnrt_mesh_displaced_sphere", INT, INT, INT, ctypes.c_float, F, ctypes.c_float,
         ctypes.c_uint32, F, F, F, I32, PINT, PINT)
    _sig(lib, "pnrt_mesh_teapot", INT, F, F, F, I32, PINT, PINT)
    _sig(lib, "pnrt_hdr_synthetic", INT, INT, INT, ctypes.c_uint32, F)


def _type_device(lib):
    _sig(lib, "pnrt_version", ctypes.c_char_p)
    _sig(lib, "pnrt_create", INT, INT, ctypes.POINTER(P))
    _sig(lib, "pnrt_destroy", None, P)
    _sig(lib, "pnrt_last_error", ctypes.c_char_p, P)
    _sig(lib, "pnrt_set_stream", INT, P, P)
    _sig(lib, "pnrt_upload_scene", INT, P, F, INT, F, INT, F, INT, F, INT, F, INT, ctypes.c_float)
    _sig(lib, "pnrt_upload_texture", INT, P, INT, U8, INT, INT, INT)
    _sig(lib, "pnrt_update_materials", INT, P, INT, INT, F)
    _sig(lib, "pnrt_upload_env", INT, P, F, F, INT, INT)
    _sig(lib, "pnrt_set_frame", INT, P, INT, INT, ctypes.POINTER(Camera), INT)
    _sig(lib, "pnrt_set_options", INT, P, INT)
    _sig(lib, "pnrt_render", INT, P, ctypes.c_uint32, ctypes.c_uint32, INT, INT, INT)
    _sig(lib, "pnrt_reset_accum", INT, P)
    _sig(lib, "pnrt_read_accum", INT, P, F)
    _sig(lib, "pnrt_accum_device_ptr", P, P)
    _sig(lib, "pnrt_pack_rows", INT, P, P, INT, INT, INT)
    _sig(lib, "pnrt_unpack_rows", INT, P, P, P, INT, INT, INT)
    _sig(lib, "pnrt_synchronize", INT, P)
    _sig(lib, "pnrt_get_device_info", INT, P, ctypes.POINTER(DeviceInfo))
    _sig(lib, "pnrt_debug_math", INT, P, INT, F, F, F, INT)
    _sig(lib, "pnrt_profile_enable", INT, P, INT)
    _sig(lib, "pnrt_profile_select", INT, P, INT)
    _sig(lib, "pnrt_get_stream", P, P)
    _sig(lib, "pnrt_upload_env_build", INT, P, F, INT, INT)
    _sig(lib, "pnrt_read_env_table", INT, P, F)
    _sig(lib, "pnrt_profile_read", INT, P, ctypes.POINTER(Profile))
    _sig(lib, "pnrt_bvh_build", INT, P, F, INT, F, INT, PINT, I32, PINT)


def fptr(a) -> ctypes.POINTER(ctypes.c_float):
    """float32 numpy array -> float* (None -> NULL)."""
    if a is None:
        return None
    assert a.dtype.name == "float32" and a.flags["C_CONTIGUOUS"], "need contiguous float32"
    return a.ctypes.data_as(F)


def iptr(a):
    if a is None:
        return None
    assert a.dtype.name == "int32" and a.flags["C_CONTIGUOUS"], "need contiguous int32"
    return a.ctypes.data_as(I32)


def u8ptr(a):
    if a is None:
        return None
    assert a.dtype.name == "uint8" and a.flags["C_CONTIGUOUS"], "need contiguous uint8"
    return a.ctypes.data_as(U8)
