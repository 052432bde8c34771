"""The oracle's intersection arithmetic pinned to the reference's OWN CPU code.

tests/golden/isect_fixtures.json holds what /root/reference/include's
BVH::Intersect / IntersectP (BVH.hpp:21-85), TriangleIntersect(P)
(triangle.hpp:15-181) and BoundIntersect (bound.hpp:31-47), compiled here by
oracle/ref/Makefile (oracle/_ref/isect_driver), return for seeded rays over the
reference-built BVHs of C1, C2, C4 and C5 (tests/golden/make_isect_golden.py):
about 3.4M ray queries per 200k-ray scene.

The CPU headers and the GLSL differ in three documented rules (SURVEY 8a
a9/a10): ties (`>=` vs `>`), slab clipping to [0, tMax] with std::max/min
(the GLSL tests the whole line with NaN-dropping min/max), and
glm::normalize (v * 1/sqrt) vs v / sqrt.  The oracle carries each rule as a
switch of its pinning hook (pno_intersect `sem`), everything else -- the
watertight shear, edge functions, determinant, barycentrics, interpolated /
face normals, hit position, uv, traversal order and stack discipline -- is
the one code path pno_render runs.  With all three switched to the CPU
headers' rules the oracle must reproduce the reference bit for bit; with the
normalisation rule alone switched back, every word but the normal must still
match and the normal must be within 1 ulp.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import isect_rays as IR  # noqa: E402
import pyoracle  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402

GOLD = os.path.join(HERE, "golden")
FIX = json.load(open(os.path.join(GOLD, "isect_fixtures.json")))
SAMPLES = np.load(os.path.join(GOLD, "isect_samples.npz"))
BUILD = {"C1": lambda: S.cornell_c1(), "C2": lambda: S.bunny_c2(env=False),
         "C4": lambda: S.teapot_c4(env=False), "C5": lambda: S.synthetic_c5(env=False)}
SEM_GLSL, SEM_CPU_NO_NORM, SEM_CPU = 0, 3, 7
NORMAL = [4, 5, 6]
OTHER = [c for c in range(13) if c not in NORMAL]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def cases(key, cfg):
    seed = FIX["seed"]
    ent = FIX["scenes"][key]
    n_rays = ent["camera/0"]["n"]
    for fam in IR.FAMILIES:
        rays = IR.make_rays(cfg.packed, cfg.camera, fam, n_rays, seed)
        for kind in (0, 1):
            yield f"{fam}/{kind}", kind, rays, None
    for what, kinds in (("tri", (2, 3)), ("box", (4,))):
        rays, idx = IR.make_pairs(cfg.packed, ent[f"{what}/{kinds[0]}"]["n"], seed, what)
        for kind in kinds:
            yield f"{what}/{kind}", kind, rays, idx


def ulp_diff(a_bits, b_bits):
    a = a_bits.astype(np.int64)
    b = b_bits.astype(np.int64)
    a = np.where(a >= 2**31, 2**31 - a, a)
    b = np.where(b >= 2**31, 2**31 - b, b)
    return np.abs(a - b)


@pytest.mark.parametrize("key", ["C1", "C2", "C4", "C5"])
def test_oracle_intersections_match_reference_cpu_code(key):
    cfg = BUILD[key]()
    o = pyoracle.Oracle(cfg)
    ent = FIX["scenes"][key]
    report = []
    for name, kind, rays, idx in cases(key, cfg):
        fx = ent[name]
        assert sha(rays) == fx["rays_sha256"], f"{key} {name}: ray generator drifted"
        if idx is not None:
            assert sha(idx.astype("<i4")) == fx["idx_sha256"], f"{key} {name}: index generator drifted"
        got = o.intersect(rays, kind, SEM_CPU, idx)
        if sha(got) != fx["out_sha256"]:
            ref = SAMPLES[f"{key}/{name}"]
            bad = np.nonzero(np.any(got[:len(ref)] != ref, axis=1))[0]
            detail = f"first differing sampled ray {bad[0]}: oracle {got[bad[0]].tolist()} ref {ref[bad[0]].tolist()}" \
                if len(bad) else "differences lie outside the sampled records"
            pytest.fail(f"{key} {name}: oracle (CPU-header rules) != reference build; {detail}")
        assert int(got[:, 0].sum()) == fx["hits"]
        # the normalisation rule alone: every other word identical, normals within 1 ulp
        mixed = o.intersect(rays, kind, SEM_CPU_NO_NORM, idx)
        np.testing.assert_array_equal(mixed[:, OTHER], got[:, OTHER], err_msg=f"{key} {name}")
        if kind in (0, 2):
            hit = got[:, 0] == 1
            assert ulp_diff(mixed[hit][:, NORMAL], got[hit][:, NORMAL]).max(initial=0) <= 1, f"{key} {name}"
        # the GLSL rules (as rendered): differences are the documented ones; report them
        glsl = o.intersect(rays, kind, SEM_GLSL, idx)
        cols = [0] if kind == 4 else OTHER           # sem 0 box queries return the flag only
        report.append(f"{name}:{int(np.any(glsl[:, cols] != got[:, cols], axis=1).sum())}")
    print(f"{key}: rays whose GLSL-rule result differs from the CPU headers' (ties / slab clipping / NaN slabs):",
          " ".join(report))

