"""Per-rank throughput of the N-GPU row-band split, measured on one GPU: render only
shard 0 of N (what rank 0 does at N GPUs, without the gather) and report the implied
whole-node rate N x per-rank.  python tools/shard_sim.py [steps] [frames per call | auto]
(auto: bench.py's call size for the share, iters_per_call x 4 frames)"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes  # noqa: E402
from pnraytracing_amd.tracer import PathTracer, shard_rows  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
arg = sys.argv[2] if len(sys.argv) > 2 else "4"         # frames per pnrt_render call (4 = one 4-spp step)
cfg = scenes.bunny_c2()


def frames_per_call(rows):
    if arg != "auto":
        return int(arg)
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return 4 * bench.iters_per_call(type("A", (), {"iters_per_call": 0})(), rows * cfg.width)


with PathTracer(0) as pt:
    pt.load(cfg)
    for n in (1, 2, 4, 8):
        rows = len(shard_rows(cfg.height, 8, n, 0))
        fpc = frames_per_call(rows)
        for k in range(4):                  # every buffer set allocated before timing
            pt.render(fpc * k, fpc, 8, n, 0)
        pt.synchronize()
        t = time.perf_counter()
        for k in range(steps):
            pt.render(fpc * (4 + k), fpc, 8, n, 0)
        pt.synchronize()
        dt = (time.perf_counter() - t) / steps
        per_rank = rows * cfg.width * fpc / dt / 1e6
        print(f"N={n}: rank-0 rows {rows}, {fpc} frames per call, {dt * 1e3 / fpc * 4:.3f} ms per 4 frames, {per_rank:.1f} Msamples/s per rank, "
              f"implied node {per_rank * n:.1f} (efficiency vs N=1 in the last column)", flush=True)
