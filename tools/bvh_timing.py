"""Host vs GPU BuildBVH wall time (incl. transfers) on the C2 and C5 triangle sets;
checks the two builds are identical.  python tools/bvh_timing.py"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import host as H  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402
from pnraytracing_amd.tracer import PathTracer  # noqa: E402


def bounds(nu, nv):
    sb = H.SceneBuilder()
    m = H.Material(baseColor=(0.65, 0.65, 0.65))
    sb.add_model(H.mesh_displaced_sphere(nu, nv, S.BUNNY_RADIUS, S.BUNNY_CENTER, 0.12, 0x5EED),
                 [H.translate(0, 0, -2), H.scale(8)], m, "mesh")
    S._cornell_walls(sb, m)
    return sb.tri_bounds()


with PathTracer(0) as pt:
    pt.build_bvh(bounds(16, 8))                     # warm-up (module load)
    for name, nu, nv in (("C2", 264, 132), ("C5", 2048, 1024)):
        tb = bounds(nu, nv)
        t = time.perf_counter(); cpu = H.bvh_build_cpu(tb); tc = time.perf_counter() - t
        t = time.perf_counter(); gpu = pt.build_bvh(tb); tg = time.perf_counter() - t
        same = (np.array_equal(cpu[0].view(np.uint32), gpu[0].view(np.uint32)) and np.array_equal(cpu[1], gpu[1])
                and cpu[2] == gpu[2])
        print(f"{name}: {len(tb)} tris -> {len(cpu[0])} nodes, depth {cpu[2]}: host {tc * 1e3:.1f} ms, "
              f"GPU {tg * 1e3:.1f} ms (incl. PCIe), identical={same}", flush=True)
