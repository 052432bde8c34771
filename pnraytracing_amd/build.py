"""In-tree build of the native libraries (no JIT cache, nothing installed).

    libpnrt_host.so  g++   csrc/host/pnrt_host.cpp          (host scene library)
    libpnrt.so       hipcc csrc/pnrt_device.hip, gfx950     (device library)
    oracle/liboracle.so    gcc (TEST-ONLY parity oracle; see oracle/)
    oracle/_ref/ref_driver g++ on /root/reference headers (only where present)

Floating point: every library is built with -ffp-contract=off and without
fast-math so the HIP kernel, the host library and the oracle evaluate the
same IEEE binary32 operation sequences (bit-exact parity).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(REPO, "include")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PNRT_OFFLOAD_ARCH", "gfx950")

DEVICE_SRCS = ["pnrt_device.hip"]
DEVICE_DEPS = ["pnrt_device.hip", "pt_diag.h", "pt_common.h", "pt_kernel.h", "pt_shade.h", "pt_path.h", "pt_passes.h", "pt_wf.h",
               "pt_env.h", "pt_bvh.h", "pn_math.h", "sobol_v.inc"]


def _run(cmd, cwd=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=cwd)


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_host(force=False):
    out = os.path.join(PKG, "libpnrt_host.so")
    src = os.path.join(CSRC, "host", "pnrt_host.cpp")
    if force or _stale(out, [src, os.path.join(INC, "pnrt_host.h")]):
        _run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
              "-Wall", "-I", INC, src, "-o", out])
    return out


def device_source_hash() -> str:
    """sha256 (16 hex) of the device library's sources, stamped into
    pnrt_version() so a stale prebuilt libpnrt.so is detectable."""
    h = hashlib.sha256()
    for d in [os.path.join(CSRC, d) for d in DEVICE_DEPS] + [os.path.join(INC, "pnrt.h")]:
        h.update(os.path.basename(d).encode())
        h.update(open(d, "rb").read())
    return h.hexdigest()[:16]


def build_device(force=False, extra=()):
    out = os.path.join(PKG, "libpnrt.so")
    deps = [os.path.join(CSRC, d) for d in DEVICE_DEPS] + [os.path.join(INC, "pnrt.h")]
    if force or extra or _stale(out, deps):
        cmd = [HIPCC, f"--offload-arch={ARCH}", os.environ.get("PNRT_OPT", "-O3"), "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-fno-fast-math", "-fno-gpu-rdc",
               # no SLP packing into v_pk_*_f32: the register pairs it needs cost the
               # trace kernel a wave per SIMD and the setup kernels one
               "-fno-slp-vectorize", f'-DPNRT_SRC_HASH="{device_source_hash()}"', "-I", INC,
               *extra, *[os.path.join(CSRC, s) for s in DEVICE_SRCS], "-o", out]
        _run(cmd)
    return out


# Diagnostic device libraries the GPU tests load in a child process (PNRT_DEVICE_LIB):
# never the product library (pnrt_version() says DIAGNOSTIC BUILD).
#   guard1  the trace kernel's block-queue claim gives up after one attempt, so
#           queued rays go untraced: pnrt_* must report PNRT_E_TRACE
#   bounds  every fetch / store index of the integrator kernels checked against its
#           array (pt_diag.h WF_DIAG_BOUNDS): a violation is reported as PNRT_E_TRACE
#   coop    every ray handed to the cooperative finish after a hash-chosen 0..24 lane
#           steps (pt_diag.h WF_DIAG_COOP), with the bounds checks: same images
#   coopsmall  the same with the finishes' limits shrunk (WF_DIAG_COOP_SMALL), so the
#           closest-hit restart (-2) and the one-entry depth-first regime run routinely
DIAG_VARIANTS = {"guard1": ["-DPNRT_DIAG_BUILD", "-DWF_DIAG_GUARD=1"],
                 "bounds": ["-DPNRT_DIAG_BUILD", "-DWF_DIAG_BOUNDS=1"],
                 "coop": ["-DPNRT_DIAG_BUILD", "-DWF_DIAG_COOP=24", "-DWF_DIAG_BOUNDS=1"],
                 "coopsmall": ["-DPNRT_DIAG_BUILD", "-DWF_DIAG_COOP=24", "-DWF_DIAG_COOP_SMALL=1", "-DWF_DIAG_BOUNDS=1"],
                 # the trace census (tools/census.py; moot-ray counts, tests/test_gpu_moot.py)
                 "stats": ["-DPNRT_DIAG_BUILD", "-DWF_PIPES=1", "-DWF_STATS=1"]}


def variant_path(name: str) -> str:
    return os.path.join(PKG, "variants", f"libpnrt_{name}.so")


def build_diag_variants(force=False):
    deps = [os.path.join(CSRC, d) for d in DEVICE_DEPS] + [os.path.join(INC, "pnrt.h")]
    os.makedirs(os.path.join(PKG, "variants"), exist_ok=True)
    for name, flags in DIAG_VARIANTS.items():
        out = variant_path(name)
        if force or _stale(out, deps):
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                  "-fno-fast-math", "-fno-gpu-rdc", "-fno-slp-vectorize", f'-DPNRT_SRC_HASH="{device_source_hash()}"',
                  "-I", INC, *flags, *[os.path.join(CSRC, s) for s in DEVICE_SRCS], "-o", out])


def build_abi_caller(force=False):
    """tests/abi/c_abi_render: a compiled C++ caller of include/pnrt.h +
    include/pnrt_host.h linked against the two libraries (TEST-ONLY; exercises
    the drop-in boundary without Python, tests/test_gpu_c_abi.py)."""
    src = os.path.join(REPO, "tests", "abi", "c_abi_render.cpp")
    out = os.path.join(REPO, "tests", "abi", "c_abi_render")
    deps = [src, os.path.join(INC, "pnrt.h"), os.path.join(INC, "pnrt_host.h"),
            os.path.join(PKG, "libpnrt.so"), os.path.join(PKG, "libpnrt_host.so")]
    if not os.path.exists(src) or not all(os.path.exists(d) for d in deps):
        return None
    if force or _stale(out, deps):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-I", INC, src, "-o", out, "-L", PKG, "-lpnrt", "-lpnrt_host",
              "-Wl,-rpath,$ORIGIN/../../pnraytracing_amd", "-Wl,-rpath-link,/opt/rocm/lib"])
    # the reference's render loop (one pnrt_render per frame) through the C ABI alone, for parity and timing
    dsrc = os.path.join(REPO, "tests", "abi", "c_abi_dloop.cpp")
    dout = os.path.join(REPO, "tests", "abi", "c_abi_dloop")
    if os.path.exists(dsrc) and (force or _stale(dout, deps[1:2] + deps[3:4] + [dsrc])):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-I", INC, dsrc, "-o", dout, "-L", PKG, "-lpnrt",
              "-Wl,-rpath,$ORIGIN/../../pnraytracing_amd", "-Wl,-rpath-link,/opt/rocm/lib"])
    # the multi-GPU caller: one process, one RCCL communicator per device (ncclCommInitAll + ncclGather)
    msrc = os.path.join(REPO, "tests", "abi", "c_abi_multigpu.cpp")
    mout = os.path.join(REPO, "tests", "abi", "c_abi_multigpu")
    if os.path.exists(msrc) and (force or _stale(mout, deps[1:] + [msrc])):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I", "/opt/rocm/include", msrc,
              "-o", mout, "-L", PKG, "-L", "/opt/rocm/lib", "-lpnrt", "-lpnrt_host", "-lamdhip64", "-lrccl",
              "-Wl,-rpath,$ORIGIN/../../pnraytracing_amd", "-Wl,-rpath,/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"])
    return out


def build_oracle(force=False):
    odir = os.path.join(REPO, "oracle")
    _run(["make", "-s", "-C", odir] + (["-B"] if force else []))
    ref = os.environ.get("PNRT_REFERENCE", "/root/reference")
    if os.path.isdir(os.path.join(ref, "include")):
        _run(["make", "-s", "-C", os.path.join(odir, "ref"), f"REF={ref}"] + (["-B"] if force else []))


def build_all(force=False):
    build_host(force)
    build_device(force)
    build_diag_variants(force)
    build_abi_caller(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
