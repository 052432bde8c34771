"""CPU model of the trace step's traversal state machine (tools/trace_emu.py):
the packed pending-range word (REF_LEAF | count << 24 | first) and the wide
first / count pair drive identical traversals -- same hits, same step counts --
and the invariant the step relies on (pending triangles => cur == REF_NONE:
the fourth-quarter fetch of a triangle lane lies out of range) holds at every
step.  A model of the control flow in float64, not of the device bits."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_packed_and_wide_ranges_agree():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "trace_emu.py"), "150"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rays 150 mismatches 0" in r.stdout
    # the wave-cooperative finish of any-hit rays (pt_wf.h wf_coop_anyhit) gives the
    # sequential traversal's occlusion from any hand-over point
    assert "coop rays" in r.stdout and "coop rays 0 " not in r.stdout and " mismatches 0 iterations" in r.stdout
    # ... and of closest-hit rays (wf_coop_closest: DFS-order keys, the candidates folded in key order)
    assert "coop closest rays" in r.stdout and "coop closest rays 0 " not in r.stdout
    assert [ln for ln in r.stdout.splitlines() if ln.startswith("coop closest")][0].split()[5] == "0"
