"""Driver of the trace-step cost model (tools/step_model/step_model.cpp, VERDICT r5
"Next" 1): writes the C2 scene the bench renders (reference-layout BVH, triangle
positions, light triangles, camera) as raw float32 files, builds the model with g++
and runs it.  CPU only; nothing here is on the product path.

    python tools/step_model/step_model.py [tile_step] [VALU_unified VALU_node VALU_tri VALU_quad]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes as S  # noqa: E402


def main():
    cfg = {"C2": S.bunny_c2, "C3": S.marry_c3, "C4": S.teapot_c4}[os.environ.get("CONFIG", "C2")]()
    p = cfg.packed
    d = tempfile.mkdtemp(prefix="step_model_")
    tri = p.triangles[:, :3].astype(np.int64)
    pos = p.vertices[:, :3].astype(np.float32)
    p.nodes.astype(np.float32).tofile(os.path.join(d, "nodes.bin"))
    pos[tri].reshape(-1, 9).astype(np.float32).tofile(os.path.join(d, "tripos.bin"))
    p.lights[:, 0].astype(np.float32).tofile(os.path.join(d, "lights.bin"))
    np.asarray(cfg.camera, np.float32).reshape(-1).tofile(os.path.join(d, "camera.bin"))
    exe = os.path.join(d, "step_model")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", os.path.join(HERE, "step_model.cpp"), "-o", exe],
                   check=True)
    subprocess.run([exe, d, *sys.argv[1:]], check=True)


if __name__ == "__main__":
    main()
