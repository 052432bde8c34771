"""Exclusive per-kernel times (PNRT_SERIAL: one call in flight, full trace grid) of
rank 0's share of an N-way row-band split, against 1/N of the whole frame's:
which kernels lose efficiency on small shares.
    python tools/shard_kernels.py [steps] [frames per call]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes  # noqa: E402
from pnraytracing_amd.tracer import SERIAL, TRAVERSE_ZCULL, PathTracer  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
fpc = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cfg = scenes.bunny_c2()
with PathTracer(0) as pt:
    pt.load(cfg)
    pt.set_options(TRAVERSE_ZCULL | SERIAL)
    base = None
    for n in (1, 2, 4, 8):
        for k in range(2):
            pt.render(fpc * k, fpc, 8, n, 0)
        pt.synchronize()
        pt.profile_select(None)
        pt.profile_enable(True)
        for k in range(steps):
            pt.render(fpc * (2 + k), fpc, 8, n, 0)
        prof = pt.profile_read()
        pt.profile_enable(False)
        per_call = {k: ms / steps for k, (ms, c) in prof.items() if c}
        tot = sum(per_call.values())
        if base is None:
            base = per_call
        rel = " ".join(f"{k}={v:.3f}({v * n / base[k]:.2f}x)" for k, v in per_call.items())
        print(f"N={n}: per call ms (x = vs 1/N of N=1): {rel}  sum={tot:.3f} ({tot * n / sum(base.values()):.2f}x)",
              flush=True)
