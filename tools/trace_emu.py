"""CPU model of the trace step's traversal state machine (pt_wf.h wf_step) and of
the wave-cooperative finishes (wf_coop_anyhit / wf_coop_closest), one lane /
one wave, in IEEE binary32 arithmetic: the reference's watertight triangle test
with its `>` tie rule (ray_tracing.comp:254-318 / :360-424 -- equal t is
accepted, so the later triangle wins) and its whole-line slab test (:213-228),
evaluated on numpy float32 scalars in the GLSL operation order (no fused
multiply-adds).  Exact traversal mode (no z-slab culling).

* the pending triangle range in both representations (wide first / count,
  packed leaf word): the hits and step counts must agree and the invariant
  "pending triangles => cur == REF_NONE" must hold at every step;
* the any-hit finish from a random hand-over point: the occlusion boolean of the
  sequential traversal;
* the closest-hit finish: DFS-order keys, candidates at the relaxed bound
  E (1 + 1e-4) in float32, the device's limits -- a frontier of (STK + 1) * 32
  entries, keys 47 levels deep, at most 64 candidates (else -2: the ray is
  traced again from its start) -- and the exact fold in key order: the
  sequential traversal's hit.

Two scenes: the C2 bunny stand-in at low resolution, and a tie scene -- the
Cornell walls with the coplanar ceiling light (main.cpp:229-237), a stack of
12 coincident triangles and one of 100 (an inline leaf of more than 64
candidates) -- with rays aimed at the ties.  "ties" counts the closest-hit rays
whose sequential traversal accepted an equal t again (a later triangle winning
a tie).

    python tools/trace_emu.py [n_rays]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pnraytracing_amd import host as H  # noqa: E402
from pnraytracing_amd import scenes as S  # noqa: E402

LEAF, NONE = 0x80000000, 0xFFFFFFFF
f32 = np.float32
ONE = f32(1.0)
FLOAT_MAX = f32(3.402823466e38)


def fmin_(a, b):          # GLSL min with the oracle's NaN rule (pn_oracle.c fmin_)
    return b if (b < a or a != a) else a


def fmax_(a, b):
    return b if (b > a or a != a) else a


class Scene:
    def __init__(self, cfg):
        self.N = cfg.packed.nodes
        self.V = cfg.packed.vertices
        self.T = cfg.packed.triangles
        N = self.N
        order = []
        if int(N[0, 7]) != -1:
            order.append(0)
        q = 0
        while q < len(order):                    # device numbering: BFS over interior nodes
            i = order[q]
            q += 1
            rc = int(N[i, 7])
            if int(N[i + 1, 7]) != -1:
                order.append(i + 1)
            if int(N[rc, 7]) != -1:
                order.append(rc)
        self.order = order
        self.dn = {i: k for k, i in enumerate(order)}
        self.pts = [[tuple(f32(x) for x in self.V[int(j), :3]) for j in self.T[t, :3]] for t in range(len(self.T))]
        self.maxleaf = max(int(n[9]) - int(n[8]) for n in N if int(n[7]) == -1)

    def childref(self, ci, packed):
        n = self.N[ci]
        if int(n[7]) != -1:
            return self.dn[ci]
        s0, cnt = int(n[8]), int(n[9]) - int(n[8])
        if cnt <= 0:
            return LEAF
        if packed:
            return LEAF | (cnt << 24) | s0
        assert cnt <= 127 and s0 < (1 << 23)
        return LEAF | (s0 << 7) | cnt

    def node_rec(self, k, packed):
        i = self.order[k]
        rc = int(self.N[i, 7])
        return self.N[i + 1, :6], self.N[rc, :6], self.childref(i + 1, packed), self.childref(rc, packed), int(self.N[i, 6])


def tri_hit(sc, o, d, t, tmax):
    """The watertight test in float32 (pn_oracle.c tri_test, ray_tracing.comp:269-312)
    against tmax with the `>` rule; the hit distance ts * (1 / det), or None."""
    p = sc.pts[t]
    P = [[p[k][i] - o[i] for i in range(3)] for k in range(3)]
    rd = list(d)
    if rd[2] == 0:
        a = 0 if abs(rd[0]) > abs(rd[1]) else 1
        for k in range(3):
            P[k][a], P[k][2] = P[k][2], P[k][a]
        rd[a], rd[2] = rd[2], rd[a]
    invDz = ONE / rd[2]
    for k in range(3):
        P[k][0] = P[k][0] - (P[k][2] * rd[0]) * invDz
        P[k][1] = P[k][1] - (P[k][2] * rd[1]) * invDz
        P[k][2] = P[k][2] * invDz
    e0 = P[1][0] * P[2][1] - P[1][1] * P[2][0]
    e1 = P[2][0] * P[0][1] - P[2][1] * P[0][0]
    e2 = P[0][0] * P[1][1] - P[0][1] * P[1][0]
    if (e0 < 0 or e1 < 0 or e2 < 0) and (e0 > 0 or e1 > 0 or e2 > 0):
        return None
    det = (e0 + e1) + e2
    if det == 0:
        return None
    ts = (e0 * P[0][2] + e1 * P[1][2]) + e2 * P[2][2]
    if det > 0 and (ts <= 0 or ts > tmax * det):
        return None
    if det < 0 and (ts >= 0 or ts < tmax * det):
        return None
    return ts * (ONE / det)


def box_hit(o, inv, b):
    """BoundIntersect (:213-228): the whole-line slab test in float32."""
    f = [(f32(b[3 + i]) - o[i]) * inv[i] for i in range(3)]
    n = [(f32(b[i]) - o[i]) * inv[i] for i in range(3)]
    tmx = [fmax_(f[i], n[i]) for i in range(3)]
    tmn = [fmin_(f[i], n[i]) for i in range(3)]
    return fmin_(tmx[0], fmin_(tmx[1], tmx[2])) >= fmax_(tmn[0], fmax_(tmn[1], tmn[2]))


def trace(sc, o, d, any_hit, packed, stop_after=None):
    """The lane's sequential step loop.  Returns (hit, steps, states, ties) or, with
    stop_after, the state handed over: (None, steps, (cur, lt, stack), tMax, hit)."""
    inv = [ONE / d[i] for i in range(3)]
    tmax = FLOAT_MAX                 # (env shadow and continuation rays: tMax = FLOAT_MAX)
    root = sc.childref(0, packed) if int(sc.N[0, 7]) == -1 else 0
    cur, lt, lc, hit, ties = NONE, 0, 0, -1, 0
    if box_hit(o, inv, sc.N[0, :6]):
        if root & LEAF:
            if packed:
                lt = root
            else:
                lt, lc = (root >> 7) & 0x7fffff, root & 0x7f
        else:
            cur = root
    stack, steps, states = [], 0, []
    while True:
        if stop_after is not None and steps == stop_after:      # hand the state over (packed only)
            return None, steps, (cur, lt, list(stack)), tmax, (-1 if hit == -1 else (hit & 0xffffff))
        steps += 1
        assert steps < 200000, "runaway"
        assert len(stack) < 64, "stack overflow"
        is_tri = (lt >= (LEAF | (1 << 24))) if packed else lc > 0
        is_node = cur != NONE
        assert not (is_tri and is_node), "invariant: pending triangles with a node"
        states.append((cur, (lt & 0xffffff, (lt >> 24) & 0x7f) if packed and lt >= LEAF else (lt, lc) if not packed
                       else (0, 0)))
        done = False
        if is_tri:
            ti = (lt & 0xffffff) if packed else lt
            th = tri_hit(sc, o, d, ti, tmax)
            if th is not None:
                if hit != -1 and th == tmax:
                    ties += 1
                hit = lt
                if any_hit:
                    done = True
                else:
                    tmax = th
            if packed:
                lt = (lt + (1 - (1 << 24))) & 0xffffffff
            else:
                lt += 1
                lc -= 1
        if is_node:
            bl, br, rl, rr, ax = sc.node_rec(cur, packed)
            hl, hr = box_hit(o, inv, bl), box_hit(o, inv, br)
            rf = d[ax] < 0
            far = rl if rf else rr
            if hl and hr:
                stack.append(far)
            go = rr if (hr and ((not hl) or rf)) else (rl if hl else NONE)
            go_leaf = go != NONE and (go & LEAF)
            if go_leaf:
                if packed:
                    lt = go
                else:
                    lt, lc = (go >> 7) & 0x7fffff, go & 0x7f
            cur = NONE if go_leaf else go
        has = (lt >= (LEAF | (1 << 24))) if packed else lc > 0
        idle = (not done) and (not has) and cur == NONE
        if idle and not stack:
            done = True
        if idle and stack:
            e = stack.pop()
            if e & LEAF:
                if packed:
                    lt = e
                else:
                    lt, lc = (e >> 7) & 0x7fffff, e & 0x7f
            else:
                cur = e
        if done:
            idx = -1 if hit == -1 else ((hit & 0xffffff) if packed else hit)
            return idx, steps, states, ties


def coop(sc, o, d, state, tmax, stk=8):
    """wf_coop_anyhit: the wave's 64 lanes finish an any-hit ray from its state
    (node to visit, pending leaf word, stack): frontier entries taken 64 at a time
    from the top (one at a time above CAP - 128), a node adds the children whose
    boxes pass, a leaf word tests its first triangle and adds the rest.  Returns
    (occluded, iterations, max frontier size)."""
    inv = [ONE / d[i] for i in range(3)]
    cur, lt, stack = state
    cap = (stk + 1) * 64
    fr = list(stack) + ([cur] if cur != NONE else []) + ([lt] if lt >= (LEAF | (1 << 24)) else [])
    it, peak = 0, len(fr)
    while fr:
        it += 1
        k = 1 if len(fr) > cap - 128 else min(len(fr), 64)
        take, fr = fr[len(fr) - k:], fr[:len(fr) - k]
        new = []
        for f in reversed(take):                 # lane i takes entry size - 1 - i
            if f >= (LEAF | (1 << 24)):
                if tri_hit(sc, o, d, f & 0xffffff, tmax) is not None:
                    return True, it, peak
                rest = (f + (1 - (1 << 24))) & 0xffffffff
                if rest >= (LEAF | (1 << 24)):
                    new.append(rest)
            elif not (f & LEAF):
                bl, br, rl, rr, ax = sc.node_rec(f, True)
                if box_hit(o, inv, bl) and rl != LEAF:
                    new.append(rl)
                if box_hit(o, inv, br) and rr != LEAF:
                    new.append(rr)
        fr += new
        peak = max(peak, len(fr))
        assert len(fr) <= cap, "frontier overflow"
    return False, it, peak


def coop_closest(sc, o, d, state, tmax0, hit0, stk=8, maxcand=64, keytop=55):
    """wf_coop_closest: a closest-hit ray finished by the wave.  Phase 1 walks the
    frontier in any order (64 entries at a time), each entry carrying its DFS-order
    key (rank of the hand-over entry: pending range 0, node 1, stack top 2 ...;
    then one bit per level below it -- near 0, far 1 -- ended by a sentinel bit;
    the triangle's place in its leaf in the low 8 bits); a triangle accepted at the
    relaxed bound E * 1.0001f (float32) is a candidate, E the least hit distance
    found.  Phase 2 folds the candidates in key order from (tmax0, hit0) with the
    exact test.  Returns (hit, iterations) or (None, iterations) for a restart (-2:
    capacity, key depth, more than maxcand candidates)."""
    inv = [ONE / d[i] for i in range(3)]
    cur, lt, stack = state
    cap = (stk + 1) * 32
    top = 1 << keytop
    fr = [(e, ((2 + len(stack) - 1 - k) << 56) | top) for k, e in enumerate(stack)]
    if cur != NONE:
        fr.append((cur, (1 << 56) | top))
    if lt >= (LEAF | (1 << 24)):
        fr.append((lt, top))
    E, cands, it = tmax0, [], 0
    while fr:
        it += 1
        k = 1 if len(fr) + len(cands) > cap - 128 else min(len(fr), 64)
        take, fr = fr[len(fr) - k:], fr[:len(fr) - k]
        new, er = [], E * f32(1.0001)
        ths = []
        for f, key in reversed(take):
            if f >= (LEAF | (1 << 24)):
                th = tri_hit(sc, o, d, f & 0xffffff, er)
                if th is not None:
                    if not (abs(th) < f32(3.0e38)):
                        return None, it                  # a non-finite distance ends the cooperation
                    cands.append((key, f & 0xffffff))
                    ths.append(th)
                rest = (f + (1 - (1 << 24))) & 0xffffffff
                if rest >= (LEAF | (1 << 24)):
                    new.append((rest, key + 1))
            elif not (f & LEAF):
                pk = key & ~0xff
                sent = pk & -pk
                if sent <= (1 << 8):
                    return None, it                      # deeper than the key holds: restart
                bl, br, rl, rr, ax = sc.node_rec(f, True)
                rf = d[ax] < 0
                kl = key - sent + (sent >> 1) if not rf else key + (sent >> 1)     # left child's key
                kr = key + (sent >> 1) if not rf else key - sent + (sent >> 1)
                if box_hit(o, inv, bl) and rl != LEAF:
                    new.append((rl, kl))
                if box_hit(o, inv, br) and rr != LEAF:
                    new.append((rr, kr))
        for th in ths:                                   # E after the iteration (the wave's minimum)
            E = fmin_(E, th)
        fr += new
        if len(fr) + len(cands) > cap:
            return None, it
    if len(cands) > maxcand:
        return None, it
    # phase 2: the exact fold in DFS order
    tm, hit = tmax0, hit0
    for key, tri in sorted(cands):
        th = tri_hit(sc, o, d, tri, tm)
        if th is not None:
            tm, hit = th, tri
    return hit, it


def tie_scene():
    """The Cornell walls with the coplanar ceiling light, a stack of 12 coincident
    triangles and one of 100 (inline leaves; the second has more than 64)."""
    sb = H.SceneBuilder()
    S._cornell_walls(sb, H.Material(baseColor=(0.6, 0.6, 0.6)))
    for n, off in ((12, 0.0), (100, 1.7)):
        tri = np.array([[-1.0 + off, 0.5, -1.0], [1.5 + off, 0.7, -0.5], [0.0 + off, 3.0, -1.2]], np.float32)
        P = np.tile(tri, (n, 1))
        sb.add_model(H.Mesh(P, None, None, np.arange(len(P), dtype=np.int32)), [H.scale(1.0)],
                     H.Material(baseColor=(0.3, 0.5, 0.7)), f"stack{n}")
    return S.SceneConfig("ties", sb.build(), S._cornell_camera(32, 32), 32, 32, 1)


def rays(sc, rng, n, aim):
    lo, hi = sc.N[0, :3].astype(np.float64), sc.N[0, 3:6].astype(np.float64)
    for _ in range(n):
        o = lo + (hi - lo) * rng.uniform(0.02, 0.98, 3)
        if aim is not None and rng.random() < 0.8:
            tgt = aim[int(rng.integers(0, len(aim)))]
            w = rng.dirichlet([1, 1, 1])
            d = w @ tgt - o
        else:
            d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        if rng.random() < 0.05:
            d[int(rng.integers(0, 3))] = 0.0             # axis-aligned: the permuted test (d.z == 0)
        yield tuple(f32(x) for x in o), tuple(f32(x) for x in d)


def run(name, sc, NR, rng, aim=None):
    print(f"[{name}] nodes {len(sc.N)} interior {len(sc.order)} tris {len(sc.T)} max leaf {sc.maxleaf}")
    mism = 0
    for r, (o, d) in enumerate(rays(sc, rng, NR, aim)):
        any_hit = r % 3 == 0
        a = trace(sc, o, d, any_hit, False)
        b = trace(sc, o, d, any_hit, True)
        if a[0] != b[0] or a[1] != b[1]:
            mism += 1
            if mism < 5:
                print("mismatch", r, a[:2], b[:2])
    print(f"[{name}] rays {NR} mismatches {mism}")
    # any-hit finish from a random hand-over point: the boolean must agree
    cm, its, seq, peak = 0, [], [], 0
    for r, (o, d) in enumerate(rays(sc, rng, NR, aim)):
        full = trace(sc, o, d, True, True)
        stop = int(rng.integers(0, max(1, full[1])))
        st = trace(sc, o, d, True, True, stop_after=stop)
        if st[0] is not None:                        # finished before the hand-over
            continue
        occ, n, pk = coop(sc, o, d, st[2], st[3])
        its.append(n)
        seq.append(full[1] - stop)
        peak = max(peak, pk)
        if occ != (full[0] != -1):
            cm += 1
            if cm < 5:
                print("coop mismatch", r, occ, full[:2], stop)
    print(f"[{name}] coop rays {len(its)} mismatches {cm} iterations mean {np.mean(its):.1f} vs sequential steps "
          f"{np.mean(seq):.1f}, max frontier {peak}")
    # closest-hit finish: same hand-over points, hit and tMax carried over
    hm, its2, rs, ties = 0, [], 0, 0
    for r, (o, d) in enumerate(rays(sc, rng, NR, aim)):
        full = trace(sc, o, d, False, True)
        ties += full[3] > 0
        stop = int(rng.integers(0, max(1, full[1])))
        st = trace(sc, o, d, False, True, stop_after=stop)
        if st[0] is not None:
            continue
        h, n = coop_closest(sc, o, d, st[2], st[3], st[4])
        if h is None:
            rs += 1
            continue
        its2.append(n)
        if h != full[0]:
            hm += 1
            if hm < 5:
                print("coop closest mismatch", r, h, full[:2], stop)
    print(f"[{name}] coop closest rays {len(its2)} mismatches {hm} restarts {rs} ties {ties} iterations mean "
          f"{np.mean(its2) if its2 else 0:.1f}")
    return mism + cm + hm


def main():
    NR = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    rng = np.random.default_rng(1)
    with np.errstate(all="ignore"):
        bad = run("C2", Scene(S.bunny_c2(64, 48, nu=66, nv=33)), NR, rng)
        ts = Scene(tie_scene())
        aim = [np.array([[-1.0 + off, 0.5, -1.0], [1.5 + off, 0.7, -0.5], [0.0 + off, 3.0, -1.2]]) for off in (0.0, 1.7)]
        aim.append(np.array([[-0.55, 5.54, -0.55], [0.55, 5.54, -0.55], [0.0, 5.54, 0.55]]))   # the ceiling light's plane
        bad += run("ties", ts, NR, rng, aim)
    print(f"total mismatches {bad}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
