"""``PathTracer``: the host-side operator over ``libpnrt.so`` (include/pnrt.h).

It is the headless replacement of the GL part of main.cpp: upload the packed
arrays (main.cpp:409-524), set the per-frame uniforms (main.cpp:606-611),
dispatch frames (main.cpp:613) and read the progressive accumulation image.
All compute runs in the HIP library; if it is missing this module raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from .host import PackedScene

TRAVERSE_EXACT = 0
TRAVERSE_ZCULL = 1
KERNEL_V1 = 0x100      # | with a traverse mode: one-lane-per-pixel A/B baseline kernel
SERIAL = 0x200         # | measurement: one call in flight, full trace grid (exclusive kernel times)


class PnrtError(RuntimeError):
    pass


class PathTracer:
    def __init__(self, device: int = 0):
        self._lib = N.device_lib()
        ctx = ctypes.c_void_p()
        rc = self._lib.pnrt_create(device, ctypes.byref(ctx))
        if rc != 0:
            raise PnrtError(f"pnrt_create(device={device}) failed ({rc}): no usable HIP device")
        self._ctx = ctx
        self.width = self.height = 0

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.pnrt_destroy(self._ctx)
            self._ctx = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _ck(self, rc, what):
        if rc != 0:
            raise PnrtError(f"{what} failed ({rc}): {self._lib.pnrt_last_error(self._ctx).decode()}")

    # ---- uploads ---------------------------------------------------------------------
    def upload_scene(self, p: PackedScene):
        V, M, T, Nd, L = (np.ascontiguousarray(a, np.float32) for a in p.arrays())
        self._ck(self._lib.pnrt_upload_scene(self._ctx, N.fptr(V), len(V), N.fptr(M), len(M), N.fptr(T), len(T),
                                             N.fptr(Nd), len(Nd), N.fptr(L) if len(L) else None, len(L),
                                             ctypes.c_float(p.lights_sum_area)), "pnrt_upload_scene")

    def update_materials(self, first: int, records: np.ndarray):
        """Overwrite materials first.. with (n, 18) records in place (pnrt_update_materials:
        the material panel's glTexSubImage1D edit, ImGuiLayer.hpp:73-83)."""
        rec = np.ascontiguousarray(records, np.float32).reshape(-1, 18)
        self._ck(self._lib.pnrt_update_materials(self._ctx, first, len(rec), N.fptr(rec)), "pnrt_update_materials")

    def upload_texture(self, slot: int, pixels: np.ndarray, width: int, height: int, channels: int):
        px = np.ascontiguousarray(pixels, np.uint8).reshape(-1)
        self._ck(self._lib.pnrt_upload_texture(self._ctx, slot, N.u8ptr(px), width, height, channels),
                 "pnrt_upload_texture")

    def upload_env(self, rgb: np.ndarray | None, table: np.ndarray | None):
        if rgb is None:
            self._ck(self._lib.pnrt_upload_env(self._ctx, None, None, 0, 0), "pnrt_upload_env")
            return
        rgb = np.ascontiguousarray(rgb, np.float32)
        table = np.ascontiguousarray(table, np.float32)
        h, w = rgb.shape[:2]
        self._ck(self._lib.pnrt_upload_env(self._ctx, N.fptr(rgb), N.fptr(table), w, h), "pnrt_upload_env")

    def upload_env_build(self, rgb: np.ndarray):
        """Environment with its RandomHDR table built on the GPU (pt_env.h)."""
        rgb = np.ascontiguousarray(rgb, np.float32)
        h, w = rgb.shape[:2]
        self._ck(self._lib.pnrt_upload_env_build(self._ctx, N.fptr(rgb), w, h), "pnrt_upload_env_build")
        self._env_shape = (h, w)

    def read_env_table(self) -> np.ndarray:
        h, w = self._env_shape
        out = np.empty((h, w, 3), np.float32)
        self._ck(self._lib.pnrt_read_env_table(self._ctx, N.fptr(out)), "pnrt_read_env_table")
        return out

    def build_bvh(self, tri_bounds: np.ndarray):
        """GPU BuildBVH (pnrt_bvh_build): (nodes (nn, 12) float32, order (n,) int32, max_depth)
        from per-triangle Bound + boundCenter (n, 9) -- the host build's result, bit for bit."""
        tb = np.ascontiguousarray(tri_bounds, np.float32).reshape(-1, 9)
        n = len(tb)
        cap = max(2 * n - 1, 1)
        nodes = np.empty((cap, 12), np.float32)
        order = np.empty(n, np.int32)
        nn, md = ctypes.c_int(), ctypes.c_int()
        self._ck(self._lib.pnrt_bvh_build(self._ctx, N.fptr(tb), n, N.fptr(nodes), cap, ctypes.byref(nn), N.iptr(order),
                                          ctypes.byref(md)), "pnrt_bvh_build")
        return nodes[:nn.value].copy(), order, md.value

    def set_frame(self, width: int, height: int, camera: np.ndarray, max_depth: int = 4):
        cam = N.Camera()
        c = np.asarray(camera, np.float32).reshape(4, 3)
        cam.eye[:], cam.lower_left[:], cam.horizontal[:], cam.vertical[:] = (list(map(float, r)) for r in c)
        self._ck(self._lib.pnrt_set_frame(self._ctx, width, height, ctypes.byref(cam), max_depth), "pnrt_set_frame")
        self.width, self.height = width, height

    def set_options(self, traverse_mode: int):
        self._ck(self._lib.pnrt_set_options(self._ctx, traverse_mode), "pnrt_set_options")

    def stream_handle(self) -> int:
        """The context's own hipStream_t (for torch.cuda.ExternalStream)."""
        return int(self._lib.pnrt_get_stream(self._ctx) or 0)

    def set_stream(self, stream_handle: int | None):
        self._ck(self._lib.pnrt_set_stream(self._ctx, ctypes.c_void_p(stream_handle or 0)), "pnrt_set_stream")

    def load(self, cfg, traverse_mode: int = TRAVERSE_ZCULL):
        """Upload a :class:`pnraytracing_amd.scenes.SceneConfig`."""
        self.upload_scene(cfg.packed)
        for slot, (px, w, h, ch) in enumerate(cfg.textures):
            self.upload_texture(slot, px, w, h, ch)
        self.upload_env(cfg.env_rgb, cfg.env_table)
        self.set_frame(cfg.width, cfg.height, cfg.camera, cfg.max_depth)
        self.set_options(traverse_mode)

    # ---- frames ----------------------------------------------------------------------
    def render(self, first_frame: int, n_frames: int, band: int = 1, n_shards: int = 1, shard: int = 0):
        self._ck(self._lib.pnrt_render(self._ctx, first_frame, n_frames, band, n_shards, shard), "pnrt_render")

    def reset_accum(self):
        self._ck(self._lib.pnrt_reset_accum(self._ctx), "pnrt_reset_accum")

    def synchronize(self):
        self._ck(self._lib.pnrt_synchronize(self._ctx), "pnrt_synchronize")

    def read_accum(self) -> np.ndarray:
        out = np.empty((self.height, self.width, 4), np.float32)
        self._ck(self._lib.pnrt_read_accum(self._ctx, N.fptr(out)), "pnrt_read_accum")
        return out

    def accum_ptr(self) -> int:
        return int(self._lib.pnrt_accum_device_ptr(self._ctx) or 0)

    def pack_rows(self, dst_ptr: int, band: int, n_shards: int, shard: int):
        self._ck(self._lib.pnrt_pack_rows(self._ctx, ctypes.c_void_p(dst_ptr), band, n_shards, shard), "pnrt_pack_rows")

    def unpack_rows(self, src_ptr: int, dst_ptr: int, band: int, n_shards: int, shard: int):
        """Shard `shard`'s packed rows (device buffer) into their rows of a device image
        (height x width x 4 floats), on the context stream (pnrt_unpack_rows)."""
        self._ck(self._lib.pnrt_unpack_rows(self._ctx, ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr), band,
                                            n_shards, shard), "pnrt_unpack_rows")

    def device_info(self) -> dict:
        info = N.DeviceInfo()
        self._ck(self._lib.pnrt_get_device_info(self._ctx, ctypes.byref(info)), "pnrt_get_device_info")
        return {f: getattr(info, f) for f, _ in info._fields_}

    def profile_enable(self, on: bool = True):
        """Bracket every kernel launch with HIP events on the launch stream (resets totals)."""
        self._ck(self._lib.pnrt_profile_enable(self._ctx, int(bool(on))), "pnrt_profile_enable")

    def profile_select(self, classes=None):
        """Kernel classes to time (names of K_CLASSES; None = all)."""
        mask = -1 if classes is None else sum(1 << N.K_CLASSES.index(k) for k in classes)
        self._ck(self._lib.pnrt_profile_select(self._ctx, mask), "pnrt_profile_select")

    def profile_read(self) -> dict:
        """{kernel class: (total ms, launches)} since profile_enable (synchronises)."""
        p = N.Profile()
        self._ck(self._lib.pnrt_profile_read(self._ctx, ctypes.byref(p)), "pnrt_profile_read")
        return {k: (p.ms[i], int(p.launches[i])) for i, k in enumerate(N.K_CLASSES)}

    def version(self) -> str:
        """pnrt_version(): library version + sha256 of the device sources it was built from."""
        return self._lib.pnrt_version().decode()

    def debug_math(self, fn: int, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
        a = np.ascontiguousarray(a, np.float32)
        b = None if b is None else np.ascontiguousarray(b, np.float32)
        out = np.empty_like(a)
        self._ck(self._lib.pnrt_debug_math(self._ctx, fn, N.fptr(a), N.fptr(b), N.fptr(out), len(a)), "pnrt_debug_math")
        return out


def shard_rows(height: int, band: int, n_shards: int, shard: int) -> np.ndarray:
    """Rows y with (y // band) % n_shards == shard, increasing (pnrt_pack_rows order)."""
    y = np.arange(height)
    return y[(y // band) % n_shards == shard]
