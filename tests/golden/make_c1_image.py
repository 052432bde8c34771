"""Generate tests/golden/c1_oracle_image.npz: the CPU oracle's C1 image (Cornell
box, 256x256, depth 4, frames 0..3 progressively blended) -- the expected
output of the compiled C-ABI caller (tests/abi/c_abi_render.cpp,
tests/test_gpu_c_abi.py).  tests/test_oracle_kat.py re-renders it on the CPU
to keep the fixture tied to the current oracle.

Usage:  python tests/golden/make_c1_image.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import pyoracle  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402

W, H, FRAMES = 256, 256, 4


def render():
    cfg = S.cornell_c1(W, H)
    img, _ = pyoracle.Oracle(cfg).render(0, FRAMES)
    return img


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "c1_oracle_image.npz"), image=render(), frames=FRAMES)
    print("wrote c1_oracle_image.npz")
