"""The cooperative drain finishes (pt_wf.h wf_coop_anyhit / wf_coop_closest)
forced onto every ray, against the oracle bit for bit (VERDICT r4 "Next" 2).

In the product library the finishes run only where a drained wave is down to
its last ray (closest-hit ones only in calls with nothing else in flight), so
no scene chooses which rays reach them.  Two diagnostic libraries
(build.py DIAG_VARIANTS, pt_diag.h WF_DIAG_COOP) hand EVERY ray -- light and
env shadow rays (any-hit) and continuation rays (closest-hit), in every
launch -- to the finish after a hash-chosen 0..24 lane steps, with every
fetch / store / frontier index bounds-checked:

* ``coop``       the product limits: the finish completes nearly every ray --
                 up to eight due rays of a wave on one shared frontier
                 (wf_coop_multi, the lone calls' drain finish), a lone any-hit
                 ray on its own (wf_coop_anyhit, the pipelined launches');
* ``coopsmall``  the limits shrunk (one-entry depth-first regime above 8
                 frontier entries, at most 2 candidates, keys 12 levels deep):
                 closest-hit rays routinely come back as -2 and are traced
                 again from the root by their own lane (WF_RID_NOCOOP).

Cases: C1, C2 and C4 at 320x180, the Cornell ceiling / ceiling-light plane
(main.cpp:229-237: exact t ties, the `>` rule of ray_tracing.comp:311-312),
inline leaves of 65 and 100 coincident triangles (more than 64 closest-hit
candidates: the -2 path in the product library too), and 24 fuzz seeds --
each in the culling and the exact traversal mode.  The hand-over and
restart counts the libraries print must be non-zero where stated.
Tolerance: 0 ulp."""
import os
import re
import subprocess
import sys

import pytest

from pnraytracing_amd import build

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(lib, which, *extra, timeout=400):
    env = dict(os.environ)
    if lib:
        env["PNRT_DEVICE_LIB"] = lib
    r = subprocess.run([sys.executable, os.path.join(HERE, "coop_worker.py"), which, *extra], env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0 and "COOP-WORKER-DONE" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    tot = [0, 0, 0, 0, 0]
    for m in re.finditer(r"\[coop\] bounce \d+ n=\d+ anyhit=(\d+) closest=(\d+) restarts=(\d+) multi=(\d+) deep=(\d+)",
                         r.stderr):
        for k in range(5):
            tot[k] += int(m.group(k + 1))
    return r.stdout, tot


@pytest.mark.parametrize("variant", ["coop", "coopsmall"])
def test_forced_cooperative_finish_fixed_scenes(variant):
    lib = build.variant_path(variant)
    assert os.path.exists(lib), f"variants/libpnrt_{variant}.so not built (__graft_entry__.build())"
    out, (anyhit, closest, restarts, multi, deep) = _run(lib, "fixed")
    assert "DIAGNOSTIC BUILD" in out
    print(f"{variant}: rays handed over any-hit {anyhit}, closest-hit {closest}, restarts {restarts}, "
          f"finishes of 2-8 rays together {multi}, rays with spilled stack entries {deep}")
    assert anyhit > 1000 and closest > 1000 and multi > 100 and deep > 0
    assert restarts > (1000 if variant == "coopsmall" else 0)   # (coop: the 65 / 100-triangle leaves)


@pytest.mark.parametrize("variant", ["coop", "coopsmall"])
def test_forced_cooperative_finish_fuzz(variant):
    lib = build.variant_path(variant)
    out, (anyhit, closest, restarts, multi, deep) = _run(lib, "fuzz")
    print(f"{variant} fuzz: rays handed over any-hit {anyhit}, closest-hit {closest}, restarts {restarts}, "
          f"finishes of 2-8 rays together {multi}, rays with spilled stack entries {deep}")
    assert anyhit > 0 and closest > 0
    if variant == "coopsmall":
        assert restarts > 0


def test_product_library_lone_frames_coincident_leaves():
    """The product library on the same fixed cases, one synchronised frame per
    call (lone calls: the closest-hit finish is live, and a drained wave's last
    ray in the 100-triangle leaf returns -2)."""
    out, _ = _run(None, "fixed", "--sync-frames")
    assert "DIAGNOSTIC" not in out
