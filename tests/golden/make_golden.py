"""Generate the committed golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists; the GPU box only reads the outputs).

Sources of truth, all from the reference itself:
  * oracle/_ref/ref_driver -- the reference's own BVH.hpp / bound.hpp /
    triangle.hpp / camera.hpp / glm compiled by oracle/ref/Makefile; fed the
    same model-space meshes, materials and transforms as our scenes.
  * shaders/ray_tracing.comp -- the Sobol direction table V[8*32] (:508-510),
    parsed as data.
  * SURVEY.md 8c -- probe values recorded from the reference's LoadHDRImage
    (sha256 prefixes/suffixes and spot entries of the RGB and RandomHDR blobs).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from pnraytracing_amd import host as H  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402

REF = os.environ.get("PNRT_REFERENCE", "/root/reference")
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")


class Recorder(H.SceneBuilder):
    """SceneBuilder that also records the model list for the reference driver."""

    def __init__(self):
        super().__init__()
        self.mats, self.meshes = [], []

    def add_model(self, meshes, ops, material, name="", texture_ids=None):
        if isinstance(meshes, H.Mesh):
            meshes = [meshes]
        mid = len(self.mats)
        self.mats.append(material.pack())
        for k, m in enumerate(meshes):
            tex = -1 if texture_ids is None else int(texture_ids[k])
            self.meshes.append((mid, tex, ops, m))
        return super().add_model(meshes, ops, material, name, texture_ids)


def driver_input(rec: Recorder, cam_args) -> bytes:
    out = [b"PNRF", struct.pack("<i", len(rec.mats)), np.concatenate(rec.mats).astype("<f4").tobytes(),
           struct.pack("<i", len(rec.meshes))]
    for mid, tex, ops, m in rec.meshes:
        out.append(struct.pack("<iii", mid, tex, len(ops)))
        for k, a, v in ops:
            out.append(struct.pack("<if3f", k, a, *v))
        nv = len(m.positions)
        out.append(struct.pack("<i", nv))
        out.append(np.ascontiguousarray(m.positions, "<f4").tobytes())
        out.append(np.ascontiguousarray(m.normals, "<f4").tobytes())
        out.append(np.ascontiguousarray(m.texcoords, "<f4").tobytes())
        out.append(struct.pack("<i", len(m.indices)))
        out.append(np.ascontiguousarray(m.indices, "<i4").tobytes())
    eye, center, up, fov, aspect = cam_args
    out.append(np.array([*eye, *center, *up, fov, aspect], "<f4").tobytes())
    return b"".join(out)


def run_driver(blob: bytes) -> dict:
    res = subprocess.run([DRIVER], input=blob, capture_output=True, check=True)
    b = res.stdout
    off = 0

    def take(n, width):
        nonlocal off
        a = np.frombuffer(b, "<f4", n * width, off).reshape(n, width).copy()
        off += 4 * n * width
        return a

    def cnt():
        nonlocal off
        (v,) = struct.unpack_from("<i", b, off)
        off += 4
        return v

    out = {"vertices": take(cnt(), 15), "triangles": take(cnt(), 6), "nodes": take(cnt(), 12),
           "lights": take(cnt(), 3), "camera": take(1, 12).reshape(4, 3)}
    out["matrices"] = take(cnt(), 16)
    return out


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def build_recorded(fn, **kw):
    """Run a scenes.* builder with a recording SceneBuilder."""
    rec_holder = {}
    orig = H.SceneBuilder

    class R(Recorder):
        def __init__(self):
            super().__init__()
            rec_holder["r"] = self

    S.H.SceneBuilder = R
    try:
        cfg = fn(**kw)
    finally:
        S.H.SceneBuilder = orig
    return cfg, rec_holder["r"]


ASPECT_1080 = float(np.float32(1920) / np.float32(1080))
ASPECT_2160 = float(np.float32(3840) / np.float32(2160))
CORNELL_CAM = ((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0)
# (fixture key, scenes.* builder, camera args as main.cpp passes them, builder kwargs)
SCENES = [("C2", S.bunny_c2, CORNELL_CAM + (ASPECT_1080,), {"env": False}),
          ("C3", S.marry_c3, CORNELL_CAM + (ASPECT_1080,), {"env": False}),
          ("C4", S.teapot_c4, ((0, 5, 5), (0, 0, 0), (0, 1, 0), 45.0, ASPECT_1080), {"env": False}),
          ("C5", S.synthetic_c5, CORNELL_CAM + (ASPECT_2160,), {"env": False})]


def main():
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle", "ref"), f"REF={REF}"], check=True)
    fixtures = {}

    # ---- C1: full arrays from the reference build -----------------------------------------
    cam1 = ((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, 1.0)
    cfg1, rec1 = build_recorded(S.cornell_c1)
    ref1 = run_driver(driver_input(rec1, cam1))
    np.savez_compressed(os.path.join(HERE, "c1_reference_arrays.npz"), **ref1,
                        materials=np.stack(rec1.mats))
    print("C1:", {k: v.shape for k, v in ref1.items()})

    # ---- C2-C5: hashes + samples of the reference-built arrays ------------------------------
    for key, fn, cam, kw in SCENES:
        cfg, rec = build_recorded(fn, **kw)
        ref = run_driver(driver_input(rec, cam))
        rng = np.random.default_rng(7)
        samp = {k: sorted(rng.choice(len(ref[k]), min(64, len(ref[k])), replace=False).tolist())
                for k in ("vertices", "triangles", "nodes")}
        fixtures[key] = {
            "counts": {k: int(len(ref[k])) for k in ("vertices", "triangles", "nodes", "lights")},
            "sha256": {k: sha(ref[k]) for k in ("vertices", "triangles", "nodes", "lights", "camera", "matrices")},
            "samples": {k: {str(i): ref[k][i].tolist() for i in idx} for k, idx in samp.items()},
            "camera": ref["camera"].tolist(),
        }
        print(key, fixtures[key]["counts"])

    # ---- camera KATs at the bench resolutions --------------------------------------------------
    cams = {}
    for w, h in [(256, 256), (512, 512), (1920, 1080), (3840, 2160)]:
        aspect = float(np.float32(w) / np.float32(h))
        rec = Recorder()
        rec.add_model(H.mesh_quad(1.0), [H.scale(1.0)], H.Material(emssive=(1, 1, 1)))
        rec.build()
        ref = run_driver(driver_input(rec, ((0, 2.8, 7), (0, 2.8, 0), (0, 1, 0), 45.0, aspect)))
        cams[f"{w}x{h}"] = ref["camera"].tolist()
    fixtures["camera_kat"] = cams

    # ---- Sobol table (data of ray_tracing.comp:508-510) -----------------------------------------
    src = open(os.path.join(REF, "shaders", "ray_tracing.comp"), encoding="latin-1").read()
    m = re.search(r"const uint V\[8\*32\] = \{(.*?)\};", src, re.S)
    V = [int(x.strip().rstrip("u")) for x in m.group(1).split(",") if x.strip()]
    fixtures["sobol_v_sha256"] = hashlib.sha256(np.array(V, "<u4").tobytes()).hexdigest()
    json.dump({"V": V}, open(os.path.join(HERE, "sobol_v.json"), "w"))

    # ---- LoadHDRImage probe values recorded in SURVEY.md 8c -------------------------------------
    fixtures["hdr_1k_survey_probe"] = {
        "rgb_sha256_prefix": "4256464593adfc7f", "rgb_sha256_suffix": "4755",
        "table_sha256_prefix": "08113da799d3489a", "table_sha256_suffix": "4d1e",
        "table_spots": {"0,0": [0.0, 0.0, 4.9968367e-09], "256,512": [0.41503906, 0.44921875, 0.02314819],
                        "511,1023": [0.98144531, 0.99414062, 4.7016865e-08]},
        "table_max_pdf": 0.059689388,
    }
    json.dump(fixtures, open(os.path.join(HERE, "reference_fixtures.json"), "w"), indent=1)
    print("wrote", os.path.join(HERE, "reference_fixtures.json"))


if __name__ == "__main__":
    main()
