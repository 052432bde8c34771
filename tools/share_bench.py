"""Rank 0's share of an N-GPU C2 bench run, timed the way bench.py times it:
one untimed sizing call, a reset, the warm-up calls, a synchronise, then the K
timed steps as calls of `ipc` 4-spp iterations (the last one cut) and a
synchronise -- without the gather.  Measures what the calls' size does to a
rank's rate inside the driver's 20-step region (iters_per_call).

    python tools/share_bench.py N ipc [steps] [warmup]      (on the GPU box)
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes  # noqa: E402
from pnraytracing_amd.tracer import PathTracer, shard_rows  # noqa: E402

n, ipc = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 5
SPP = 4
cfg = scenes.bunny_c2()
rows = len(shard_rows(cfg.height, 8, n, 0))


def calls(pt, lo, hi):
    for k in range(lo, hi, ipc):
        m = min(ipc, hi - k)
        pt.render(SPP * k, SPP * m, 8, n, 0)


with PathTracer(0) as pt:
    pt.load(cfg)
    pt.render(0, SPP * ipc, 8, n, 0)        # sizing call
    pt.synchronize()
    pt.reset_accum()
    calls(pt, 0, warm)
    pt.synchronize()
    t = time.perf_counter()
    calls(pt, warm, warm + steps)
    pt.synchronize()
    dt = (time.perf_counter() - t) / steps
    per_rank = rows * cfg.width * SPP / dt / 1e6
    print(f"N={n} ipc={ipc}: rank-0 rows {rows}, {dt * 1e3:.3f} ms/step, {per_rank:.1f} Msamples/s per rank", flush=True)
