#!/usr/bin/env python3
"""The reference's own loop (main.cpp:573-630: one 1-spp frame per dispatch) timed
through the C ABI alone: exports the D2 / D3 scene (C2 / C3 at 512x512,
PnRT.hpp:41-42) as a PND1 file and runs tests/abi/c_abi_dloop -- pnrt_render(k, 1)
per frame, synchronised (pnrt_synchronize) after every frame, then pipelined --
with no Python in the timed loop.  Prints one JSON line per config.

    python tools/dloop.py [D2 D3] [--frames 240 --warmup 16]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes as S  # noqa: E402

EXE = os.path.join(REPO, "tests", "abi", "c_abi_dloop")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["D2", "D3"])
    ap.add_argument("--frames", type=int, default=240)
    ap.add_argument("--warmup", type=int, default=16)
    a = ap.parse_args()
    for c in a.configs:
        cfg = {"D2": S.bunny_c2, "D3": S.marry_c3}[c](width=512, height=512, spp=1)
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "scene.bin")
            S.export_pnd1(cfg, p)
            out = {"config": c, "workload": f"{cfg.name}@512: one pnrt_render per frame through the C ABI (no Python)",
                   "frames": a.frames}
            for mode in ("sync", "pipe"):
                r = subprocess.run([EXE, p, str(a.frames), str(a.warmup), mode], capture_output=True, text=True,
                                   timeout=300)
                if r.returncode != 0:
                    sys.exit(f"{c} {mode}: rc {r.returncode}: {r.stderr[-2000:]}")
                ms = float(r.stdout.split("ms_per_frame")[1].split()[0])
                out[f"ms_per_frame_{mode}"] = ms
                out[f"host_render_us_{mode}"] = float(r.stdout.split("host_render_us")[1].split()[0])
                out[f"host_sync_us_{mode}"] = float(r.stdout.split("host_sync_us")[1].split()[0])
                out[f"msamples_per_s_{mode}"] = round(512 * 512 / ms / 1e3, 2)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
