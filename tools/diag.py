"""GPU diagnostic: per-depth / per-kernel-variant diff counts vs the oracle."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer, KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL

pt = PathTracer(0)
for name, mk in [("C1", lambda: S.cornell_c1(64, 48)), ("C2", lambda: S.bunny_c2(96, 54))]:
    for depth in (0, 1, 2, 4):
        c = mk(); c.max_depth = depth
        ref, _ = pyoracle.Oracle(c).render(0, 1)
        out = []
        for label, opt in [("v3", TRAVERSE_EXACT), ("v3z", TRAVERSE_ZCULL), ("v1", TRAVERSE_EXACT | KERNEL_V1)]:
            pt.load(c, opt); pt.reset_accum(); pt.render(0, 1)
            got = pt.read_accum()
            bad = np.any(got.view(np.uint32) != ref.view(np.uint32), axis=-1)
            out.append(f"{label}:{int(bad.sum())}")
            if label == "v3" and bad.any():
                j, i = np.argwhere(bad)[0]
                out.append(f"(first {j},{i} gpu={got[j,i,:3]} ref={ref[j,i,:3]} mean gpu/ref={got[...,:3].mean():.4f}/{ref[...,:3].mean():.4f})")
        print(name, "depth", depth, " ".join(out), flush=True)
