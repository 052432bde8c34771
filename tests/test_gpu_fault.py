"""A trace launch that leaves queued rays untraced must fail loudly, never
return a silently wrong image (the reference traces every ray,
ray_tracing.comp:429-494).

The diagnostic library variants/libpnrt_guard1.so (build.py DIAG_VARIANTS:
-DWF_DIAG_GUARD=1) lets the trace kernel's block-queue claim give up after one
attempt, so blocks quit with published segments unclaimed and queue items never
dequeued.  Loaded in a child process (PNRT_DEVICE_LIB), every completion point
must return PNRT_E_TRACE (-6) with a message, pnrt_reset_accum clears the fault,
and the next render faults again.  The product library runs the same sequence
without a fault (and every parity test would raise on one)."""
import os
import subprocess
import sys

import pytest

from pnraytracing_amd import build

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, {repo!r})
from pnraytracing_amd import scenes
from pnraytracing_amd.tracer import PathTracer, PnrtError

expect_fault = {expect!r}
cfg = scenes.cornell_c1(128, 96)          # 12k paths: 48 queue segments per ray kind
pt = PathTracer(0)
print("library:", pt.version())
pt.load(cfg)

def fails(fn, what):
    try:
        fn()
    except PnrtError as e:
        msg = str(e)
        assert "(-6)" in msg and "trace fault" in msg, msg
        print(what, "->", msg)
        return True
    print(what, "-> ok")
    return False

pt.render(0, 2)
assert fails(pt.synchronize, "synchronize") == expect_fault
assert fails(pt.read_accum, "read_accum") == expect_fault
assert fails(lambda: pt.render(2, 1), "render") == expect_fault
assert fails(lambda: pt.pack_rows(pt.accum_ptr(), 8, 1, 0), "pack_rows") == expect_fault
pt.reset_accum()                          # a new accumulation clears the fault
pt.synchronize()
pt.render(0, 1)
assert fails(pt.synchronize, "synchronize after reset + render") == expect_fault
pt.close()
print("FAULT-CHECK-DONE")
"""


def _run(lib, expect):
    env = dict(os.environ)
    if lib:
        env["PNRT_DEVICE_LIB"] = lib
    r = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO, expect=expect)], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0 and "FAULT-CHECK-DONE" in r.stdout, r.stdout + r.stderr
    return r.stdout


def test_forced_guard_expiry_is_reported():
    lib = build.variant_path("guard1")
    assert os.path.exists(lib), "variants/libpnrt_guard1.so not built (__graft_entry__.build())"
    out = _run(lib, True)
    assert "DIAGNOSTIC BUILD" in out
    assert "never dequeued" in out or "fewer rays" in out or "bounded wait" in out


def test_product_library_reports_no_fault():
    out = _run(None, False)
    assert "DIAGNOSTIC" not in out
