"""Benchmark / parity scene configurations C1-C5 (BASELINE.json ``configs``,
SURVEY.md 8d), assembled the way main.cpp's scene functions do it.

The reference's meshes (``Bunny.obj``, ``floor.obj``, ``teapot.obj``,
``marry.obj``) are git-ignored and absent, so each is replaced by a
deterministic procedural stand-in of the same role and size class; the
Cornell box transforms, materials and cameras are the reference's own
(main.cpp:198-247, :329-347).

Every builder takes ``bvh_tracer``: a PathTracer whose GPU builds the BVH
(pnrt_bvh_build) instead of the host library -- the same arrays either way.
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np

from . import host as H

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
HDR_1K = os.path.join(ASSETS, "vignaioli_night_1k.hdr")
MARI_PNG = os.path.join(ASSETS, "MC003_Kozakura_Mari.png")

# bun_zipper bounding box centre / extent (~0.155 units): the stand-in sphere
# occupies the same region before main.cpp's translate(0,0,-2)*scale(8).
BUNNY_CENTER = (-0.0168, 0.1101, -0.0015)
BUNNY_RADIUS = 0.075


@dataclasses.dataclass
class SceneConfig:
    name: str
    packed: H.PackedScene
    camera: np.ndarray                 # (4,3): eye, lowerLeftCorner, horizontal, vertical
    width: int
    height: int
    spp: int
    max_depth: int = 4
    env_rgb: np.ndarray | None = None  # (h, w, 3)
    env_table: np.ndarray | None = None
    textures: list = dataclasses.field(default_factory=list)   # (pixels u8, w, h, ch)
    description: str = ""

    @property
    def n_triangles(self) -> int:
        return len(self.packed.triangles)


def _cornell_walls(sb: H.SceneBuilder, m: H.Material, floor_mat: H.Material | None = None, light: bool = True):
    """CornellBox() walls (main.cpp:204-237): floor.obj x6 with the reference transforms."""
    q = H.mesh_quad(27.5)
    fm = floor_mat or m
    sb.add_model(q, [H.scale(0.1)], fm, "floor")
    sb.add_model(q, [H.translate(0, 2.75, -2.75), H.rotate(90.0, 1, 0, 0), H.scale(0.1)], m, "front_wall")
    m = m.copy(baseColor=(0.12, 0.45, 0.15))
    sb.add_model(q, [H.translate(2.75, 2.75, 0), H.rotate(90.0, 0, 0, 1), H.scale(0.1)], m, "right_wall")
    m = m.copy(baseColor=(0.65, 0.05, 0.05))
    sb.add_model(q, [H.translate(-2.75, 2.75, 0.0), H.rotate(-90.0, 0, 0, 1), H.scale(0.1)], m, "left_wall")
    m = m.copy(baseColor=(0.73, 0.73, 0.73))
    sb.add_model(q, [H.translate(0, 5.54, 0), H.rotate(180.0, 0, 0, 1), H.scale(0.1)], m, "ceiling")
    if not light:
        return
    m = m.copy(emssive=(60.0, 60.0, 60.0))
    sb.add_model(q, [H.translate(0, 5.54, 0), H.rotate(180.0, 0, 0, 1), H.scale(0.02)], m, "ceiling_light")


def _cornell_camera(w, h):
    # main.cpp:199-202
    return H.camera_update((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, np.float32(w) / np.float32(h))


def _env_1k():
    return H.load_hdr(HDR_1K)


def cornell_c1(width=256, height=256, spp=1, bvh_tracer=None) -> SceneConfig:
    """C1: Cornell box, 12 triangles, no environment (CPU-oracle config)."""
    sb = H.SceneBuilder()
    _cornell_walls(sb, H.Material(baseColor=(0.65, 0.65, 0.65)))
    return SceneConfig("C1-cornell", sb.build(bvh_tracer), _cornell_camera(width, height), width, height, spp,
                       description="Cornell box (12 tris), 256x256, 1 spp, depth 4, no env")


def bunny_c2(width=1920, height=1080, spp=4, nu=264, nv=132, env=True, bvh_tracer=None) -> SceneConfig:
    """C2: Cornell box + ~70k-triangle bunny stand-in + vignaioli_night_1k env."""
    sb = H.SceneBuilder()
    m = H.Material(baseColor=(0.65, 0.65, 0.65))
    bunny = H.mesh_displaced_sphere(nu, nv, BUNNY_RADIUS, BUNNY_CENTER, 0.12, 0x5EED)
    sb.add_model(bunny, [H.translate(0, 0, -2), H.scale(8)], m, "bunny")   # main.cpp:207-208
    _cornell_walls(sb, m)
    rgb = tab = None
    if env:
        rgb, tab = _env_1k()
    return SceneConfig("C2-bunny", sb.build(bvh_tracer), _cornell_camera(width, height), width, height, spp,
                       env_rgb=rgb, env_table=tab,
                       description=f"Cornell + bunny stand-in ({nu * nv * 2} tris) + 1k HDR env, "
                                   f"{width}x{height}, {spp} spp")


def load_texture(path: str):
    """stbi_load(path, &w, &h, &n, 0) as model.hpp:66-73 calls it: 8-bit rows
    top-first, no vertical flip, the file's own channel count."""
    from PIL import Image
    im = Image.open(path)
    if im.mode not in ("L", "RGB", "RGBA"):
        im = im.convert("RGBA")
    px = np.asarray(im, np.uint8)
    ch = 1 if px.ndim == 2 else px.shape[2]
    return (np.ascontiguousarray(px).reshape(-1), im.width, im.height, ch)


def checker_texture(w: int, h: int, ch: int = 3, seed: int = 7):
    """Deterministic 8-bit test texture (odd widths exercise GL_UNPACK_ALIGNMENT 4)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = ((x // 8 + y // 8) % 2) * 160 + 40
    px = np.stack([(base + rng.integers(0, 50, (h, w))) % 256 for _ in range(ch)], -1).astype(np.uint8)
    return (px.reshape(-1), w, h, ch)


def marry_c3(width=1920, height=1080, spp=4, nu=176, nv=144, env=True, bvh_tracer=None) -> SceneConfig:
    """C3: CornellBox() with its commented-out "marry" model (main.cpp:209) -- a
    UV-mapped ~50k-triangle figure stand-in textured with MC003_Kozakura_Mari.png
    (RGBA 2048x1024, texture unit 5) -- plus SceneFlat()'s metal boards
    (main.cpp:254-292, Disney metallic/roughness varied) carrying an RGB texture
    of odd width, and the 1k env.  Every Disney lobe is non-zero somewhere."""
    sb = H.SceneBuilder()
    m = H.Material(baseColor=(0.65, 0.65, 0.65))
    figure = H.mesh_displaced_sphere(nu, nv, 1.0, (0.0, 0.0, 0.0), 0.05, 0xA11CE)
    fm = H.Material(baseColor=(0.8, 0.8, 0.8), subsurface=0.3, specular=0.5, specularTint=0.2, roughness=0.45,
                    anisotropic=0.3, sheen=0.4, sheenTint=0.5, clearcoat=0.6, clearcoatGloss=0.8)
    sb.add_model(figure, [H.translate(0.1, 1.55, -0.5), H.scale(0.75, 1.5, 0.6)], fm, "marry", texture_ids=[0])
    _cornell_walls(sb, m)
    board = H.mesh_quad(27.5)
    for k, (met, rough, z) in enumerate([(0.95, 0.02, -2.2), (0.80, 0.15, -1.4), (0.60, 0.35, -0.6)]):
        bm = H.Material(baseColor=(0.83, 0.83, 0.83), metallic=met, roughness=rough)
        sb.add_model(board, [H.translate(-1.6 + 1.6 * k, 0.6, z), H.rotate(50.0 - 15.0 * k, 1, 0, 0),
                             H.scale(0.012, 1.0, 0.004)], bm, f"board{k + 1}", texture_ids=[1])
    rgb, tab = _env_1k() if env else (None, None)
    tex = [load_texture(MARI_PNG), checker_texture(333, 97, 3)]
    return SceneConfig("C3-marry", sb.build(bvh_tracer), _cornell_camera(width, height), width, height, spp,
                       env_rgb=rgb, env_table=tab, textures=tex,
                       description=f"Cornell + textured figure stand-in ({nu * nv * 2} tris, Mari 2048x1024 RGBA) "
                                   f"+ metal boards (RGB 333x97) + 1k env")


def teapot_c4(width=1920, height=1080, spp=4, env=True, bvh_tracer=None) -> SceneConfig:
    """C4: teapot() scene (main.cpp:329-347) + an emissive quad and the 1k env,
    so the light, environment and BSDF pdfs are all active."""
    sb = H.SceneBuilder()
    m = H.Material(baseColor=(0.6, 0.7, 0.2), metallic=0.7, roughness=0.3)
    sb.add_model(H.mesh_teapot(), [H.scale(0.2)], m, "teapot")
    m = H.Material(baseColor=(0.73, 0.73, 0.73), metallic=0.2, roughness=0.85)
    sb.add_model(H.mesh_quad(27.5), [H.scale(1.0)], m, "floor")
    light = H.Material(baseColor=(0.73, 0.73, 0.73), emssive=(8.0, 8.0, 8.0))
    sb.add_model(H.mesh_quad(27.5), [H.translate(1.5, 3.0, 1.0), H.rotate(180.0, 0, 0, 1), H.scale(0.02)],
                 light, "area_light")
    rgb, tab = _env_1k() if env else (None, None)
    cam = H.camera_update((0, 5, 5), (0, 0, 0), (0, 1, 0), 45.0, np.float32(width) / np.float32(height))
    return SceneConfig("C4-teapot", sb.build(bvh_tracer), cam, width, height, spp, env_rgb=rgb, env_table=tab,
                       description="teapot stand-in + floor + area light + 1k env")


def synthetic_c5(width=3840, height=2160, spp=4, nu=2048, nv=1024, env_w=4096, env_h=2048, env=True,
                 bvh_tracer=None) -> SceneConfig:
    """C5: 4,194,304-triangle displaced sphere in the Cornell box, 4k synthetic env."""
    sb = H.SceneBuilder()
    m = H.Material(baseColor=(0.65, 0.65, 0.65))
    big = H.mesh_displaced_sphere(nu, nv, BUNNY_RADIUS, BUNNY_CENTER, 0.12, 0x5EED)
    sb.add_model(big, [H.translate(0, 0, -2), H.scale(8)], m, "sphere4m")
    _cornell_walls(sb, m)
    rgb = tab = None
    if env:
        rgb = H.synthetic_hdr(env_w, env_h, 0x5EED)
        tab = H.hdr_table(rgb)
    return SceneConfig("C5-synthetic4m", sb.build(bvh_tracer), _cornell_camera(width, height), width, height, spp,
                       env_rgb=rgb, env_table=tab,
                       description=f"{nu * nv * 2}-tri displaced sphere + {env_w}x{env_h} synthetic env")


CONFIGS = {"C1": cornell_c1, "C2": bunny_c2, "C3": marry_c3, "C4": teapot_c4, "C5": synthetic_c5}


def export_pnd1(cfg: SceneConfig, path: str) -> None:
    """Write a scene as the "PND1" file a compiled C caller of the drop-in reads
    (tests/abi/c_abi_dloop.cpp): the five main.cpp-layout arrays, the frame and
    camera, the environment and its RandomHDR table, the textures."""
    p = cfg.packed
    V, M, T, N, L = (np.ascontiguousarray(a, np.float32) for a in p.arrays())
    env = cfg.env_rgb is not None
    eh, ew = (cfg.env_rgb.shape[:2] if env else (0, 0))
    with open(path, "wb") as f:
        f.write(b"PND1")
        f.write(np.array([len(V), len(M), len(T), len(N), len(L)], np.int32).tobytes())
        f.write(np.array([p.lights_sum_area], np.float32).tobytes())
        f.write(np.array([cfg.width, cfg.height, cfg.max_depth, ew, eh, len(cfg.textures)], np.int32).tobytes())
        f.write(np.ascontiguousarray(cfg.camera, np.float32).reshape(12).tobytes())
        for a in (V, M, T, N, L):
            f.write(a.tobytes())
        if env:
            f.write(np.ascontiguousarray(cfg.env_rgb, np.float32).tobytes())
            f.write(np.ascontiguousarray(cfg.env_table, np.float32).tobytes())
        for px, w, h, ch in cfg.textures:
            f.write(np.array([w, h, ch], np.int32).tobytes())
            f.write(np.ascontiguousarray(px, np.uint8).reshape(-1).tobytes())
