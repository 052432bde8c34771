"""SAH-cost estimate for DESIGN section 10 item 1 (a second tree for shadow rays).

Occlusion (BVHIntersectP, ray_tracing.comp:465-494) does not depend on the
traversal order, so shadow rays could walk any tree over the same triangles.
This script prices that lever before anyone builds it: the expected traversal
cost (surface-area heuristic, one unit per interior-node visit and per triangle
test -- the trace kernel's lane step) of the reference tree (BuildBVH,
BVH.hpp:92-173, as packed by main.cpp:488-501) against trees built here with
more buckets, all three axes and a cost-based leaf rule.

    python tools/shadow_tree_sah.py [C2|C3|C4|C5]

CPU only; no GPU, no oracle.  The cost is a proxy (uniform random lines through
the root box, no early exit for any-hit), not a measured lane-step count.
Result on C2: reference tree 10.81, every variant here
12.04-12.06.
"""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from pnraytracing_amd import scenes  # noqa: E402


def area(lo, hi):
    d = np.maximum(hi - lo, 0.0)
    return 2.0 * (d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2] + d[..., 2] * d[..., 0])


def reference_cost(nodes):
    """SAH cost of the packed reference tree: rows pMin(3) pMax(3) axis rightChild start end."""
    lo, hi = nodes[:, 0:3].astype(np.float64), nodes[:, 3:6].astype(np.float64)
    sa = area(lo, hi) / area(lo[0], hi[0])
    leaf = nodes[:, 6] < 0
    ntri = nodes[:, 9] - nodes[:, 8]
    return float(sa[~leaf].sum() + (sa[leaf] * ntri[leaf]).sum()), int(leaf.sum()), float(ntri[leaf].mean())


def build_cost(tlo, thi, cen, buckets, max_leaf):
    """Binned SAH over all three axes; a range becomes a leaf when testing its
    triangles costs no more than the best split (trav 1, triangle 1).  Returns
    (cost, leaves, mean leaf size)."""
    root_sa = area(tlo.min(0), thi.max(0))
    cost, leaves, leaf_tris = 0.0, 0, 0
    stack = [np.arange(len(tlo))]
    while stack:
        idx = stack.pop()
        lo, hi = tlo[idx].min(0), thi[idx].max(0)
        sa = area(lo, hi) / root_sa
        n = len(idx)
        best = (np.inf, None)
        if n > 1:
            c = cen[idx]
            clo, chi = c.min(0), c.max(0)
            for d in range(3):
                ext = chi[d] - clo[d]
                if ext <= 0:
                    continue
                b = np.minimum(((c[:, d] - clo[d]) / ext * buckets).astype(np.int64), buckets - 1)
                cnt = np.bincount(b, minlength=buckets)
                blo = np.full((buckets, 3), np.inf)
                bhi = np.full((buckets, 3), -np.inf)
                np.minimum.at(blo, b, tlo[idx])
                np.maximum.at(bhi, b, thi[idx])
                llo, lhi = np.minimum.accumulate(blo, 0), np.maximum.accumulate(bhi, 0)
                rlo, rhi = np.minimum.accumulate(blo[::-1], 0)[::-1], np.maximum.accumulate(bhi[::-1], 0)[::-1]
                cl, cr = np.cumsum(cnt), np.cumsum(cnt[::-1])[::-1]
                with np.errstate(invalid="ignore"):
                    s = 1.0 + (area(llo[:-1], lhi[:-1]) * cl[:-1] + area(rlo[1:], rhi[1:]) * cr[1:]) / area(lo, hi)
                s[(cl[:-1] == 0) | (cr[1:] == 0)] = np.inf
                m = int(np.argmin(s))
                if s[m] < best[0]:
                    best = (float(s[m]), (d, b <= m))
        if best[1] is None or (n <= max_leaf and n <= best[0]):
            cost += sa * n
            leaves += 1
            leaf_tris += n
            continue
        cost += sa
        d, left = best[1]
        stack.append(idx[left])
        stack.append(idx[~left])
    return cost, leaves, leaf_tris / max(leaves, 1)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    fn = {"C2": scenes.bunny_c2, "C3": scenes.marry_c3, "C4": scenes.teapot_c4, "C5": scenes.synthetic_c5}[name]
    cfg = fn()
    p = cfg.packed
    tb = p.tri_bounds.astype(np.float64)
    tlo, thi, cen = tb[:, 0:3], tb[:, 3:6], tb[:, 6:9]
    rc, rl, rm = reference_cost(p.nodes)
    print(f"{name}: {len(tb)} triangles")
    print(f"  reference tree (12 buckets, longest centre axis): SAH cost {rc:.2f}, {rl} leaves, {rm:.2f} tris/leaf")
    for buckets, max_leaf in ((12, 255), (32, 255), (32, 4)):
        t = time.time()
        c, nl, ml = build_cost(tlo, thi, cen, buckets, max_leaf)
        print(f"  all axes, {buckets} buckets, leaf <= {max_leaf}: SAH cost {c:.2f} ({c / rc:.3f} of reference), "
              f"{nl} leaves, {ml:.2f} tris/leaf ({time.time() - t:.0f} s)")


if __name__ == "__main__":
    main()
