"""Rank 0's share of an N-way row-band split rendered alone (for profiling):
    python tools/shard_sim_one.py N [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes  # noqa: E402
from pnraytracing_amd.tracer import PathTracer, shard_rows  # noqa: E402

n = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
cfg = scenes.bunny_c2()
with PathTracer(0) as pt:
    pt.load(cfg)
    rows = len(shard_rows(cfg.height, 8, n, 0))
    for k in range(3):
        pt.render(4 * k, 4, 8, n, 0)
    pt.synchronize()
    t = time.perf_counter()
    cpu = 0.0
    for k in range(steps):
        c0 = time.perf_counter()
        pt.render(4 * (3 + k), 4, 8, n, 0)
        cpu += time.perf_counter() - c0
    pt.synchronize()
    dt = (time.perf_counter() - t) / steps
    print(f"N={n}: {dt * 1e3:.3f} ms/step ({rows * cfg.width * 4 / dt / 1e6:.1f} Msamples/s per rank), "
          f"host time in pnrt_render {cpu / steps * 1e3:.3f} ms/step", flush=True)
