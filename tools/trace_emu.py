"""CPU model of the trace step's traversal state machine (pt_wf.h wf_step), one
lane, in both pending-range representations side by side (wide first / count,
packed leaf word): the hits and step counts must agree, the invariant "pending
triangles => cur == REF_NONE" must hold at every step, stacks stay bounded.
Float64 intersection tests (a model of the control flow, not of the bits).

    python tools/trace_emu.py [n_rays]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pnraytracing_amd import scenes as S

LEAF, NONE = 0x80000000, 0xFFFFFFFF
cfg = S.bunny_c2(64, 48, nu=66, nv=33)
N = cfg.packed.nodes
V = cfg.packed.vertices
T = cfg.packed.triangles
nn = len(N)
fint = lambda x: int(x)
# device numbering: BFS over interior nodes
order = []
if fint(N[0, 7]) != -1: order.append(0)
q = 0
while q < len(order):
    i = order[q]; q += 1
    rc = fint(N[i, 7])
    if fint(N[i + 1, 7]) != -1: order.append(i + 1)
    if fint(N[rc, 7]) != -1: order.append(rc)
dn = {i: k for k, i in enumerate(order)}
nt = len(T)
def childref(ci, packed):
    n = N[ci]
    if fint(n[7]) != -1: return dn[ci]
    s0, cnt = fint(n[8]), fint(n[9]) - fint(n[8])
    if cnt <= 0: return LEAF
    if packed: return LEAF | (cnt << 24) | s0
    assert cnt <= 127 and s0 < (1 << 23)
    return LEAF | (s0 << 7) | cnt
def node_rec(k, packed):
    i = order[k]; rc = fint(N[i, 7])
    return N[i + 1, :6], N[rc, :6], childref(i + 1, packed), childref(rc, packed), fint(N[i, 6])
print("nodes", nn, "interior", len(order), "tris", nt, "max leaf", max(fint(n[9]) - fint(n[8]) for n in N if fint(n[7]) == -1))

def tri_pts(t):
    idx = T[t, :3].astype(int)
    return [V[j, :3].astype(np.float64) for j in idx]

def tri_hit(o, d, t, tmax):
    p0, p1, p2 = tri_pts(t)
    e1, e2 = p1 - p0, p2 - p0
    h = np.cross(d, e2); a = e1 @ h
    if abs(a) < 1e-12: return None
    f = 1 / a; s = o - p0; u = f * (s @ h)
    if u < 0 or u > 1: return None
    qv = np.cross(s, e1); v = f * (d @ qv)
    if v < 0 or u + v > 1: return None
    tt = f * (e2 @ qv)
    return tt if 1e-6 < tt < tmax else None

def box_hit(o, inv, b):
    t1 = (b[:3] - o) * inv; t2 = (b[3:] - o) * inv
    return np.max(np.minimum(t1, t2)) <= np.min(np.maximum(t1, t2))

def trace(o, d, any_hit, packed, stop_after=None):
    inv = 1.0 / d
    tmax = 1e30
    root = childref(0, packed) if fint(N[0, 7]) == -1 else 0
    cur, lt, lc, hit = NONE, 0, 0, -1
    if box_hit(o, inv, N[0, :6]):
        if root & LEAF:
            if packed: lt = root
            else: lt, lc = (root >> 7) & 0x7fffff, root & 0x7f
        else: cur = root
    stack, steps, trace_states = [], 0, []
    while True:
        if stop_after is not None and steps == stop_after:      # hand the state over (packed only)
            return None, steps, (cur, lt, list(stack)), tmax, (-1 if hit == -1 else (hit & 0xffffff))
        steps += 1
        assert steps < 100000, "runaway"
        assert len(stack) < 64, "stack overflow"
        is_tri = (lt >= (LEAF | (1 << 24))) if packed else lc > 0
        is_node = cur != NONE
        assert not (is_tri and is_node), "invariant: pending triangles with a node"
        trace_states.append((cur, (lt & 0xffffff, (lt >> 24) & 0x7f) if packed and lt >= LEAF else (lt, lc) if not packed else (0, 0)))
        done = False
        if is_tri:
            ti = (lt & 0xffffff) if packed else lt
            th = tri_hit(o, d, ti, tmax)
            if th is not None:
                hit = lt
                if any_hit: done = True
                else: tmax = th
            if packed: lt = (lt + (1 - (1 << 24))) & 0xffffffff
            else: lt += 1; lc -= 1
        if is_node:
            bl, br, rl, rr, ax = node_rec(cur, packed)
            hl, hr = box_hit(o, inv, bl), box_hit(o, inv, br)
            rf = d[ax] < 0
            far = rl if rf else rr
            if hl and hr: stack.append(far)
            go = rr if (hr and ((not hl) or rf)) else (rl if hl else NONE)
            go_leaf = go != NONE and (go & LEAF)
            if go_leaf:
                if packed: lt = go
                else: lt, lc = (go >> 7) & 0x7fffff, go & 0x7f
            cur = NONE if go_leaf else go
        has = (lt >= (LEAF | (1 << 24))) if packed else lc > 0
        idle = (not done) and (not has) and cur == NONE
        if idle and not stack: done = True
        if idle and stack:
            e = stack.pop()
            if e & LEAF:
                if packed: lt = e
                else: lt, lc = (e >> 7) & 0x7fffff, e & 0x7f
            else: cur = e
        if done:
            idx = -1 if hit == -1 else ((hit & 0xffffff) if packed else hit)
            return idx, steps, trace_states

def coop(o, d, state, stk=8):
    """pt_wf.h wf_coop_anyhit: the wave's 64 lanes finish an any-hit ray from its
    state (node to visit, pending leaf word, stack): frontier entries taken 64 at a
    time from the top (one at a time above CAP - 128), a node adds the children
    whose boxes pass, a leaf word tests its first triangle and adds the rest.
    Returns (occluded, iterations, max frontier size)."""
    inv = 1.0 / d
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
                if tri_hit(o, d, f & 0xffffff, 1e30) is not None:
                    return True, it, peak
                rest = (f + (1 - (1 << 24))) & 0xffffffff
                if rest >= (LEAF | (1 << 24)):
                    new.append(rest)
            elif not (f & LEAF):
                bl, br, rl, rr, ax = node_rec(f, True)
                if box_hit(o, inv, bl) and rl != LEAF: new.append(rl)
                if box_hit(o, inv, br) and rr != LEAF: new.append(rr)
        fr += new
        peak = max(peak, len(fr))
        assert len(fr) <= cap, "frontier overflow"
    return False, it, peak


def coop_closest(o, d, state, tmax0, hit0, stk=8, delta=1e-4):
    """pt_wf.h wf_coop_closest: a closest-hit ray finished by the wave.  Phase 1
    walks the frontier in any order (64 entries at a time), each entry carrying
    its DFS-order key (rank of the hand-over entry: pending range 0, node 1, stack
    top 2 ...; then one bit per level below it -- near 0, far 1 -- ended by a
    sentinel bit; the triangle's place in its leaf in the low 8 bits); a triangle
    accepted at the relaxed bound E (1 + delta) is a candidate, E the least hit
    distance found.  Phase 2 folds the candidates in key order from (tmax0, hit0)
    with the exact test: the reference's sequential result.  Returns
    (hit, iterations) or (None, iterations) for a restart."""
    inv = 1.0 / d
    cur, lt, stack = state
    cap = (stk + 1) * 32
    top = 1 << 55
    fr = [(e, ((2 + len(stack) - 1 - k) << 56) | top) for k, e in enumerate(stack)]
    if cur != NONE: fr.append((cur, (1 << 56) | top))
    if lt >= (LEAF | (1 << 24)): fr.append((lt, top))
    E, cands, it = tmax0, [], 0
    while fr:
        it += 1
        k = 1 if len(fr) + len(cands) > cap - 128 else min(len(fr), 64)
        take, fr = fr[len(fr) - k:], fr[:len(fr) - k]
        new, er = [], E * (1 + delta)
        for f, key in reversed(take):
            if f >= (LEAF | (1 << 24)):
                th = tri_hit(o, d, f & 0xffffff, er)
                if th is not None:
                    cands.append((key, f & 0xffffff))
                    E = min(E, th)
                rest = (f + (1 - (1 << 24))) & 0xffffffff
                if rest >= (LEAF | (1 << 24)): new.append((rest, key + 1))
            elif not (f & LEAF):
                sent = (key & ~0xff) & -(key & ~0xff)
                if sent <= (1 << 8):
                    return None, it                      # deeper than the key holds: restart
                bl, br, rl, rr, ax = node_rec(f, True)
                rf = d[ax] < 0
                kl = key - sent + (sent >> 1) if not rf else key + (sent >> 1)     # left child's key
                kr = key + (sent >> 1) if not rf else key - sent + (sent >> 1)
                if box_hit(o, inv, bl) and rl != LEAF: new.append((rl, kl))
                if box_hit(o, inv, br) and rr != LEAF: new.append((rr, kr))
        fr += new
        if len(fr) + len(cands) > cap:
            return None, it
    # phase 2: the exact fold in DFS order
    tm, hit = tmax0, hit0
    for key, tri in sorted(cands):
        th = tri_hit(o, d, tri, tm)
        if th is not None:
            tm, hit = th, tri
    return hit, it


rng = np.random.default_rng(1)
lo, hi = N[0, :3].astype(np.float64), N[0, 3:6].astype(np.float64)
mism = 0
NR = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
for r in range(NR):
    o = lo + (hi - lo) * rng.uniform(0, 1, 3)
    d = rng.normal(size=3); d /= np.linalg.norm(d)
    any_hit = r % 3 == 0
    a = trace(o, d, any_hit, False)
    b = trace(o, d, any_hit, True)
    if a[0] != b[0] or a[1] != b[1]:
        mism += 1
        if mism < 5: print("mismatch", r, a[:2], b[:2])
print(f"rays {NR} mismatches {mism}")
# the cooperative finish of any-hit rays: hand over after a random number of
# sequential steps, finish with the frontier model; the boolean must agree
cm, its, seq, peak = 0, [], [], 0
for r in range(NR):
    o = lo + (hi - lo) * rng.uniform(0, 1, 3)
    d = rng.normal(size=3); d /= np.linalg.norm(d)
    full = trace(o, d, True, True)
    stop = int(rng.integers(0, max(1, full[1])))
    st = trace(o, d, True, True, stop_after=stop)
    if st[0] is not None:                        # finished before the hand-over
        continue
    occ, n, pk = coop(o, d, st[2])
    its.append(n); seq.append(full[1] - stop); peak = max(peak, pk)
    if occ != (full[0] != -1):
        cm += 1
        if cm < 5: print("coop mismatch", r, occ, full[:2], stop)
print(f"coop rays {len(its)} mismatches {cm} iterations mean {np.mean(its):.1f} vs sequential steps "
      f"{np.mean(seq):.1f}, max frontier {peak}")
# the cooperative finish of closest-hit rays: same hand-over points, hit and tMax
# carried over, the keyed fold must give the sequential traversal's hit
hm, its2, seq2, rs = 0, [], [], 0
for r in range(NR):
    o = lo + (hi - lo) * rng.uniform(0, 1, 3)
    d = rng.normal(size=3); d /= np.linalg.norm(d)
    full = trace(o, d, False, True)
    stop = int(rng.integers(0, max(1, full[1])))
    st = trace(o, d, False, True, stop_after=stop)
    if st[0] is not None:
        continue
    h, n = coop_closest(o, d, st[2], st[3], st[4])
    if h is None:
        rs += 1
        continue
    its2.append(n); seq2.append(full[1] - stop)
    if h != full[0]:
        hm += 1
        if hm < 5: print("coop closest mismatch", r, h, full[:2], stop)
print(f"coop closest rays {len(its2)} mismatches {hm} restarts {rs} iterations mean {np.mean(its2):.1f} vs "
      f"sequential steps {np.mean(seq2):.1f}")
sys.exit(1 if (mism or cm or hm) else 0)
