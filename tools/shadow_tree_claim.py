#!/usr/bin/env python3
"""Is occlusion independent of the tree?  

The reference tests a triangle for a shadow ray only when every box on the
triangle's ancestor chain passes the whole-line float slab test
(BoundIntersect, ray_tracing.comp:213-228, inside BVHIntersectP :464-494).  A
different tree over the same triangles returns the same occlusion bit only if
that box test never rejects an ancestor of a triangle TriangleIntersectP
(:360-427) accepts.  This counts, over seeded shadow-like ray families, the
(ray, triangle) pairs with

    TriangleIntersectP(ray, tri) accepted   AND   some ancestor box rejected

using the oracle's own routines (pno_intersect kinds 3 and 4, GLSL rules).
Brute force over triangles: C1 and C4 all pairs; C2 only the pairs whose
triangle AABB, widened by 1e-3 of the scene extent, meets the ray in float64
(the watertight test cannot accept a triangle outside its own box by more
than rounding).  A non-zero count refutes the claim by example.

    python tools/shadow_tree_claim.py [OUT.json]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import isect_rays as IR  # noqa: E402
import pyoracle  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402

FAMILIES = ("shadow", "plane", "box", "axis", "bounce")


def ancestor_chains(nodes: np.ndarray, n_tris: int):
    """Per triangle (BVH order) the reference node ids from the root to its leaf
    (pre-order layout: left child = i + 1, right child = node[7], leaf node[7] == -1
    with triangle range [node[8], node[9]))."""
    chains = [None] * n_tris
    st = [(0, (0,))]
    while st:
        i, path = st.pop()
        n = nodes[i]
        if int(n[7]) == -1:
            for t in range(int(n[8]), int(n[9])):
                chains[t] = path
            continue
        st.append((i + 1, path + (i + 1,)))
        st.append((int(n[7]), path + (int(n[7]),)))
    return chains


def candidates(rays, lo, hi, eps):
    """(ray, tri) pairs whose widened triangle AABB meets the ray's segment in float64."""
    o = rays[:, None, 0:3].astype(np.float64)
    d = rays[:, None, 3:6].astype(np.float64)
    tmax = rays[:, 6].astype(np.float64)[:, None]
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1 = (lo[None] - eps - o) * inv
        t2 = (hi[None] + eps - o) * inv
    tn = np.nanmax(np.minimum(t1, t2), axis=2)
    tf = np.nanmin(np.maximum(t1, t2), axis=2)
    # zero direction components: inside the slab or never
    inside = (o >= lo[None] - eps) & (o <= hi[None] + eps)
    ok = np.all(np.where(d == 0, inside, True), axis=2)
    tn = np.where(np.isnan(tn), -np.inf, tn)
    tf = np.where(np.isnan(tf), np.inf, tf)
    hit = ok & (tf >= np.maximum(tn, -1e-3)) & (tn <= tmax * 1.001 + 1e-3)
    r, t = np.nonzero(hit)
    return r, t


def count(cfg, n_rays, seed, brute_force):
    o = pyoracle.Oracle(cfg)
    p = cfg.packed
    nodes = p.nodes
    verts = p.vertices[:, 0:3].astype(np.float64)
    ids = p.triangles[:, 0:3].astype(np.int64)
    tri = verts[ids]                                    # (n, 3, 3)
    lo, hi = tri.min(1), tri.max(1)
    ext = float(np.max(nodes[0, 3:6] - nodes[0, 0:3]))
    chains = ancestor_chains(nodes, len(p.triangles))
    res = {}
    for fam in FAMILIES:
        rays = IR.make_rays(p, cfg.camera, fam, n_rays, seed)
        if fam not in ("shadow",):                     # shadow-ray ranges (light rays: 1 - 1e-4)
            rays[:, 6] = np.where(np.arange(n_rays) % 2 == 0, np.float32(1e7), rays[:, 6])
        if brute_force:
            r = np.repeat(np.arange(n_rays), len(p.triangles))
            t = np.tile(np.arange(len(p.triangles)), n_rays)
        else:
            rs, ts = [], []
            for k in range(0, n_rays, 64):
                a, b = candidates(rays[k:k + 64], lo, hi, 1e-3 * ext)
                rs.append(a + k); ts.append(b)
            r, t = np.concatenate(rs), np.concatenate(ts)
        acc_pairs = 0
        bad = []
        for k in range(0, len(r), 1 << 20):
            rr, tt = r[k:k + (1 << 20)], t[k:k + (1 << 20)]
            out = o.intersect(rays[rr], 3, 0, tt.astype(np.int32))
            acc = out[:, 0] != 0
            acc_pairs += int(acc.sum())
            for ri, ti in zip(rr[acc], tt[acc]):
                ch = np.asarray(chains[ti], np.int32)
                bx = o.intersect(np.repeat(rays[ri:ri + 1], len(ch), 0), 4, 0, ch)
                if not np.all(bx[:, 0] != 0):
                    fail = ch[bx[:, 0] == 0]
                    bad.append({"ray": rays[ri].tolist(), "triangle": int(ti), "failing_nodes": fail.tolist()[:4]})
        res[fam] = {"rays": n_rays, "pairs_tested": int(len(r)), "accepted_pairs": acc_pairs,
                    "accepted_with_a_rejected_ancestor": len(bad), "examples": bad[:3]}
        print(f"  {cfg.name} {fam}: {len(r)} pairs, {acc_pairs} accepted, {len(bad)} with a rejected ancestor box",
              flush=True)
    return res


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    result = {"what": __doc__.split("\n\n")[1].strip(), "scenes": {}}
    for key, cfg, n, bf in (("C1", S.cornell_c1(), 20000, True), ("C4", S.teapot_c4(env=False), 1500, False),
                            ("C2", S.bunny_c2(env=False), 1500, False)):
        result["scenes"][key] = count(cfg, n, 20261017, bf)
    tot = sum(f["accepted_with_a_rejected_ancestor"] for s in result["scenes"].values() for f in s.values())
    result["total_accepted_with_a_rejected_ancestor"] = tot
    print("total:", tot)
    if out:
        json.dump(result, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
