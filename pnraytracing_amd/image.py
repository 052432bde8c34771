"""Output of the accumulation image.

The reference displays ``output_image`` by sampling it on a full-screen quad
(render.vert / render.frag: ``fragColor = texture(output_image, texCoord)``,
no tone mapping, no gamma) into the default 8-bit framebuffer.  ``to_display``
reproduces that: rows flipped (GL row 0 is the bottom), clamp to [0, 1],
UNORM8 conversion ``round(c * 255)`` (GL spec 2.3.5).  PFM and OpenEXR keep
the float image losslessly (PFM rows are stored bottom-first, like GL's; EXR
top-first, as its increasing-y line order says).
"""
from __future__ import annotations

import struct

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


def _attr(name: str, typ: str, data: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def write_exr(path: str, accum: np.ndarray) -> None:
    """OpenEXR 2.0, single-part scanline image, no compression, 32-bit float
    R, G, B, A (the accumulation image as stored, lossless), top row first.
    Written from the format's published layout (magic, version, attribute
    header, scanline offset table, one scanline per chunk); no library needed."""
    a = np.asarray(accum, np.float32)
    h, w = a.shape[:2]
    ch = a.shape[2] if a.ndim == 3 else 1
    names = ["R", "G", "B", "A"][:ch] if ch in (3, 4) else ["Y"]
    order = sorted(range(len(names)), key=lambda k: names[k])    # channels are stored in name order
    chlist = b"".join(names[k].encode() + b"\0" + struct.pack("<iB3xii", 2, 0, 1, 1) for k in order) + b"\0"
    box = struct.pack("<4i", 0, 0, w - 1, h - 1)
    header = (b"\x76\x2f\x31\x01" + struct.pack("<i", 2) +
              _attr("channels", "chlist", chlist) + _attr("compression", "compression", b"\0") +
              _attr("dataWindow", "box2i", box) + _attr("displayWindow", "box2i", box) +
              _attr("lineOrder", "lineOrder", b"\0") + _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)) +
              _attr("screenWindowCenter", "v2f", struct.pack("<2f", 0.0, 0.0)) +
              _attr("screenWindowWidth", "float", struct.pack("<f", 1.0)) + b"\0")
    top = a[::-1].reshape(h, w, len(names))                     # GL row 0 is the bottom
    line_bytes = w * 4 * len(names)
    first = len(header) + 8 * h
    offsets = struct.pack(f"<{h}Q", *(first + y * (8 + line_bytes) for y in range(h)))
    with open(path, "wb") as f:
        f.write(header)
        f.write(offsets)
        for y in range(h):
            f.write(struct.pack("<ii", y, line_bytes))
            for k in order:
                f.write(np.ascontiguousarray(top[y, :, k], "<f4").tobytes())


def read_exr(path: str) -> np.ndarray:
    """The images write_exr writes (uncompressed scanline float): (H, W, C) float32,
    row 0 = bottom, channels R, G, B[, A]."""
    b = open(path, "rb").read()
    if b[:4] != b"\x76\x2f\x31\x01":
        raise ValueError("not an OpenEXR file")
    pos, attrs = 8, {}
    while b[pos] != 0:
        n = b.index(b"\0", pos)
        t = b.index(b"\0", n + 1)
        size = struct.unpack_from("<i", b, t + 1)[0]
        attrs[b[pos:n].decode()] = (b[n + 1:t].decode(), b[t + 5:t + 5 + size])
        pos = t + 5 + size
    pos += 1
    if attrs["compression"][1] != b"\0":
        raise ValueError("compressed EXR not supported")
    cl, names, q = attrs["channels"][1], [], 0
    while cl[q] != 0:
        e = cl.index(b"\0", q)
        names.append(cl[q:e].decode())
        if struct.unpack_from("<i", cl, e + 1)[0] != 2:
            raise ValueError("only 32-bit float channels")
        q = e + 1 + 16
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    offs = struct.unpack_from(f"<{h}Q", b, pos)
    img = np.zeros((h, w, len(names)), np.float32)
    for o in offs:
        y, size = struct.unpack_from("<ii", b, o)
        line = np.frombuffer(b, "<f4", size // 4, o + 8).reshape(len(names), w)
        img[y - y0] = line.T
    want = [c for c in ("R", "G", "B", "A", "Y") if c in names]
    return img[::-1][:, :, [names.index(c) for c in want]]
