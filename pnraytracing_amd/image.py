"""Output of the accumulation image.

The reference displays ``output_image`` by sampling it on a full-screen quad
(render.vert / render.frag: ``fragColor = texture(output_image, texCoord)``,
no tone mapping, no gamma) into the default 8-bit framebuffer.  ``to_display``
reproduces that: rows flipped (GL row 0 is the bottom), clamp to [0, 1],
UNORM8 conversion ``round(c * 255)`` (GL spec 2.3.5).  PFM keeps the float
image losslessly (PFM rows are stored bottom-first, like GL's).
"""
from __future__ import annotations

import numpy as np


def to_display(accum: np.ndarray) -> np.ndarray:
    """(H, W, 4) float accumulation image -> (H, W, 3) uint8, top row first."""
    rgb = np.clip(np.asarray(accum, np.float32)[::-1, :, :3], 0.0, 1.0)
    return np.floor(rgb * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


def write_png(path: str, accum: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(to_display(accum), "RGB").save(path)


def write_pfm(path: str, accum: np.ndarray) -> None:
    """Little-endian RGB PFM, bottom row first (lossless float32)."""
    a = np.ascontiguousarray(np.asarray(accum, np.float32)[:, :, :3], "<f4")
    h, w = a.shape[:2]
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode("ascii"))
        f.write(a.tobytes())


def read_pfm(path: str) -> np.ndarray:
    """(H, W, 3) float32, row 0 = bottom (as written by write_pfm)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"PF":
            raise ValueError("not an RGB PFM file")
        w, h = (int(v) for v in f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3).astype(np.float32)
