"""CPU model of the trace step's traversal state machine and of the cooperative
finishes (tools/trace_emu.py), in binary32 with the reference's watertight test
and `>` tie rule (ray_tracing.comp:269-312) and its whole-line slab test
(:213-228): the packed pending-range word (REF_LEAF | count << 24 | first) and
the wide first / count pair drive identical traversals -- same hits, same step
counts -- with the invariant the step relies on (pending triangles => cur ==
REF_NONE) at every step; the any-hit and closest-hit finishes from random
hand-over points give the sequential traversal's result, on a scene whose rays
meet exact t ties (coincident triangle stacks, the coplanar ceiling light) and an
inline leaf of more than 64 candidates (the -2 restart)."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traversal_and_cooperative_finishes_model():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "trace_emu.py"), "150"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    for scene in ("C2", "ties"):
        assert f"[{scene}] rays 150 mismatches 0" in out
        m = re.search(rf"\[{scene}\] coop rays (\d+) mismatches (\d+)", out)
        assert m and int(m.group(1)) > 0 and m.group(2) == "0", out
        m = re.search(rf"\[{scene}\] coop closest rays (\d+) mismatches (\d+) restarts (\d+) ties (\d+)", out)
        assert m and int(m.group(1)) > 0 and m.group(2) == "0", out
        if scene == "ties":
            # ties present (a later triangle won an equal t), and the >64-candidate leaf restarted
            assert int(m.group(4)) > 0 and int(m.group(3)) > 0, out
    assert "total mismatches 0" in out
