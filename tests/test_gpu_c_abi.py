"""The drop-in boundary exercised by a COMPILED C++ caller (no Python, no
ctypes): tests/abi/c_abi_render.cpp includes include/pnrt.h + pnrt_host.h,
links libpnrt.so + libpnrt_host.so and runs INTEGRATION.md section 1's
sequence (create, upload_scene, camera_update, set_frame, one pnrt_render per
frame as main.cpp:587-628 dispatches, read_accum).  Its input arrays are the
ones the reference's own headers build for C1 (tests/golden/
c1_reference_arrays.npz, oracle/_ref/ref_driver); its output must equal the
committed oracle image bit for bit."""
import os
import struct
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
EXE = os.path.join(HERE, "abi", "c_abi_render")

pytestmark = pytest.mark.gpu


def write_scene(path):
    ref = np.load(os.path.join(GOLD, "c1_reference_arrays.npz"))
    arrays = [ref["vertices"], ref["materials"], ref["triangles"], ref["nodes"], ref["lights"]]
    sum_area = float(ref["lights"][-1, 1]) if len(ref["lights"]) else 0.0     # main.cpp:392
    with open(path, "wb") as f:
        f.write(b"PNC1" + struct.pack("<5i", *[len(a) for a in arrays]) + struct.pack("<f", sum_area))
        for a in arrays:
            f.write(np.ascontiguousarray(a, "<f4").tobytes())


def test_compiled_caller_renders_c1_bit_exact(tmp_path):
    assert os.path.exists(EXE), "tests/abi/c_abi_render not built (python -c 'import __graft_entry__ as g; g.build()')"
    gold = np.load(os.path.join(GOLD, "c1_oracle_image.npz"))
    H, W = gold["image"].shape[:2]
    scene, out = str(tmp_path / "c1.bin"), str(tmp_path / "out.bin")
    write_scene(scene)
    r = subprocess.run([EXE, scene, out, str(W), str(H), str(int(gold["frames"]))], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "expected error:" in r.stdout                       # errors are codes + messages, not exit()
    img = np.fromfile(out, np.float32).reshape(H, W, 4)
    bad = np.argwhere(np.any(img.view(np.uint32) != gold["image"].view(np.uint32), axis=-1))
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}"


MEXE = os.path.join(HERE, "abi", "c_abi_multigpu")


@pytest.mark.parametrize("n_shards", [3, 8])
def test_compiled_multigpu_caller_gathers_bit_exact(tmp_path, n_shards):
    """SURVEY 8e's process model in C++: one process,
    ncclCommInitAll over the visible devices, one pnrt context per row-band
    shard, pnrt_pack_rows + ncclGather to device 0.  The gathered image equals
    the single-context render (checked inside the program) and the committed
    oracle image, bit for bit.  On a one-GPU box the shards share the device."""
    assert os.path.exists(MEXE), "tests/abi/c_abi_multigpu not built (python -c 'import __graft_entry__ as g; g.build()')"
    gold = np.load(os.path.join(GOLD, "c1_oracle_image.npz"))
    H, W = gold["image"].shape[:2]
    scene, out = str(tmp_path / "c1.bin"), str(tmp_path / "out.bin")
    write_scene(scene)
    r = subprocess.run([MEXE, scene, out, str(W), str(H), str(int(gold["frames"])), str(n_shards)], capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-identical to the single-context render" in r.stdout, r.stdout
    img = np.fromfile(out, np.float32).reshape(H, W, 4)
    bad = np.argwhere(np.any(img.view(np.uint32) != gold["image"].view(np.uint32), axis=-1))
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}"


DEXE = os.path.join(HERE, "abi", "c_abi_dloop")


@pytest.mark.parametrize("config", ["C2", "C3"])
def test_compiled_reference_loop_bit_exact(tmp_path, config):
    """tests/abi/c_abi_dloop: the reference's render loop (one pnrt_render per
    frame, pnrt_synchronize after each, main.cpp:587-628) from a PND1 scene file
    (scenes.export_pnd1: arrays, env + RandomHDR table, textures, camera) through
    the C ABI alone -- the program tools/dloop.py times.  Its image equals the
    oracle's bit for bit (C2's bunny + env, C3's textures, at 96x64)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    import pyoracle
    from pnraytracing_amd import scenes as S
    assert os.path.exists(DEXE), "tests/abi/c_abi_dloop not built (python -c 'import __graft_entry__ as g; g.build()')"
    cfg = {"C2": S.bunny_c2, "C3": S.marry_c3}[config](width=96, height=64, spp=1)
    scene, out = str(tmp_path / "s.bin"), str(tmp_path / "out.bin")
    S.export_pnd1(cfg, scene)
    for mode in ("sync", "pipe"):
        r = subprocess.run([DEXE, scene, "5", "3", mode, out], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "ms_per_frame" in r.stdout, r.stdout + r.stderr
        img = np.fromfile(out, np.float32).reshape(cfg.height, cfg.width, 4)
        ref, _ = pyoracle.Oracle(cfg).render(0, 8)
        bad = np.argwhere(np.any(img.view(np.uint32) != ref.view(np.uint32), axis=-1))
        assert len(bad) == 0, f"{config} {mode}: {len(bad)} pixels differ, first {bad[:4].tolist()}"
