"""The C-ABI libraries load and export every symbol their headers declare
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

import pytest

from pnraytracing_amd import _native as N

INC = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include")


def declared(header):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pnrt_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("header,path", [("pnrt.h", N.DEVICE_LIB), ("pnrt_host.h", N.HOST_LIB)])
def test_library_exports_declared_symbols(header, path):
    lib = ctypes.CDLL(path)
    names = declared(header)
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_device_library_typed_and_versioned():
    """pnrt_version() carries the sha256 of the device sources it was built from
    (build.py stamps it): a stale prebuilt libpnrt.so beside newer sources --
    e.g. one shipped to the GPU box -- fails here instead of testing old code."""
    from pnraytracing_amd import build
    lib = N.device_lib()
    v = lib.pnrt_version().decode()
    assert "gfx950" in v
    assert v.endswith("src " + build.device_source_hash()), (v, build.device_source_hash())


def test_device_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pnraytracing_amd.tracer import PathTracer, PnrtError
    with pytest.raises(PnrtError):
        PathTracer(0)


def test_diag_variant_is_marked_diagnostic():
    """The fault-injection library the GPU fault test loads (build.DIAG_VARIANTS)
    exists, exports the same ABI and can never pass for the product library."""
    from pnraytracing_amd import build
    path = build.variant_path("guard1")
    if not os.path.exists(path):
        pytest.skip("diagnostic variant not built (no hipcc)")
    lib = ctypes.CDLL(path)
    missing = [n for n in declared("pnrt.h") if not hasattr(lib, n)]
    assert not missing, missing
    lib.pnrt_version.restype = ctypes.c_char_p
    assert "DIAGNOSTIC BUILD" in lib.pnrt_version().decode()
