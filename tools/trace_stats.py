"""Run one C2 step with a WF_STATS build (PNRT_DEVICE_LIB) and print the census."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes as S
from pnraytracing_amd.tracer import PathTracer
pt = PathTracer(0)
pt.load(S.bunny_c2())
pt.render(0, 4)
pt.synchronize()
