"""Child process of tests/test_gpu_coop.py: renders the cooperative-finish cases
on the library PNRT_DEVICE_LIB names and compares every image with the oracle
bit for bit.  Prints one "case <name> mode <m>: ok" line per case and exits
non-zero on the first difference.  (A diagnostic WF_DIAG_COOP library prints
its per-launch hand-over counts on stderr; the parent sums them.)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), HERE]

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from pnraytracing_amd import host as H  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402
from pnraytracing_amd.tracer import TRAVERSE_EXACT, TRAVERSE_ZCULL, PathTracer  # noqa: E402


def coincident_inline(copies: int = 100, W: int = 40, Hh: int = 30) -> S.SceneConfig:
    """`copies` identical triangles in the Cornell box: one degenerate-centre leaf
    (BVH.hpp:117-120) of 65..127 triangles -- still an inline (packed) leaf ref --
    with exact t ties, so a closest-hit cooperative finish that reaches it collects
    more than 64 candidates and gives the ray back (-2)."""
    rng = np.random.default_rng(copies)
    sb = H.SceneBuilder()
    S._cornell_walls(sb, H.Material(baseColor=(0.6, 0.6, 0.6)))
    tri = np.array([[-1.0, 0.5, -1.0], [1.5, 0.7, -0.5], [0.0, 3.0, -1.2]], np.float32)
    P = np.tile(tri, (copies, 1))
    mesh = H.Mesh(P, None, None, np.arange(len(P), dtype=np.int32))
    sb.add_model(mesh, [H.scale(1.0)], H.Material(baseColor=tuple(rng.uniform(0, 1, 3)), metallic=0.3), "stack")
    cfg = S.SceneConfig(f"coincident{copies}", sb.build(), S._cornell_camera(W, Hh), W, Hh, 1, max_depth=3)
    nd = cfg.packed.nodes
    leaves = nd[:, 7] == -1
    big = int((nd[leaves, 9] - nd[leaves, 8]).max())
    assert 64 < big <= 127, big
    return cfg


def ceiling_light_ties(W: int = 96, Hh: int = 64) -> S.SceneConfig:
    """C1 seen from below the ceiling: the ceiling quad and the ceiling light lie
    in one plane (main.cpp:229-237, both at y = 5.54), so camera and bounce rays
    meet both at the same t -- the reference's `>` rule (:311-312) picks the
    later triangle."""
    c1 = S.cornell_c1(W, Hh)
    cam = H.camera_update((0.3, 3.2, 1.5), (0.0, 5.54, 0.0), (0, 0, -1), 60.0, np.float32(W) / np.float32(Hh))
    c1.camera = cam
    c1.name = "C1-ceiling-ties"
    return c1


def cases(which: str):
    out = []
    if which in ("all", "fixed"):
        out += [("C1", S.cornell_c1(), 0, 2), ("C2-320x180", S.bunny_c2(320, 180), 0, 2),
                ("C4-320x180", S.teapot_c4(320, 180), 0, 2), ("ceiling-ties", ceiling_light_ties(), 0, 3),
                ("coincident-100", coincident_inline(100), 0, 3), ("coincident-65", coincident_inline(65), 0, 3)]
    if which in ("all", "fuzz"):
        from test_gpu_fuzz import random_scene
        for seed in range(int(os.environ.get("PNRT_COOP_SEEDS", "24"))):
            cfg, rng = random_scene(seed)
            out.append((f"fuzz{seed}", cfg, int(rng.integers(0, 20)), int(rng.integers(1, 10))))
    return out


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    sync_frames = "--sync-frames" in sys.argv      # one frame per call, synchronised: lone calls (closest coop)
    pt = PathTracer(0)
    print("library:", pt.version(), flush=True)
    for name, cfg, first, n in cases(which):
        ref, st = pyoracle.Oracle(cfg).render(first, n)
        assert st["stack_overflow"] == 0
        for mode in (TRAVERSE_ZCULL, TRAVERSE_EXACT):
            pt.load(cfg, mode)
            pt.reset_accum()
            if sync_frames:
                for f in range(first, first + n):
                    pt.render(f, 1)
                    pt.synchronize()
            else:
                pt.render(first, n)
            got = pt.read_accum()
            bad = np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1)
            if bad.any():
                y, x = np.argwhere(bad)[0]
                print(f"case {name} mode {mode}: {int(bad.sum())} of {bad.size} pixels differ, first (row {y}, x {x})",
                      flush=True)
                sys.exit(5)
            print(f"case {name} mode {mode}: ok", flush=True)
    pt.close()
    print("COOP-WORKER-DONE", flush=True)


if __name__ == "__main__":
    main()
