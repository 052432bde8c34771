// pnraytracing_amd/csrc/pt_kernel.h -- the gfx950 radiance integrator.
//
// One lane per pixel; each lane runs all frames of a pnrt_render() call for its
// pixel and blends them in order (ray_tracing.comp:988-991), so the RGBA32F
// accumulation image is read once and written once per call instead of once
// per frame.  The primary ray has no jitter (:980), so its closest hit is
// traced once per call and reused by every frame.
//
// Bit-exactness rules (vs the CPU oracle, oracle/pn_oracle.c):
//   * every float expression keeps the GLSL operation order; build with
//     -ffp-contract=off (no FMA), IEEE division and sqrt, denormals kept;
//   * BVH children are visited in the reference order (near child by the
//     sign of dir[axis] first, :447-457) and a leaf's triangles in index
//     order, so closest-hit ties resolve exactly as in BVHIntersect (:429-461);
//   * RNG draws happen in the reference order (:880, :884, :561, :757, :643).
#pragma once
#include "pt_common.h"

// ---- ray with per-ray precomputation ------------------------------------------------
struct RayP {
    f3 o, d;
    f3 inv;           // 1/dir (BoundIntersect :214); inv[kz] is the triangle test's invDz
    int perm;         // bits 0-1: kz of the axis permutation (:269-282; 2 = identity),
                      // bit 2: z-slab culling is provably result-neutral for this ray,
                      // bits 4-6: d.x < 0, d.y < 0, d.z < 0 (the near-child rule :448
                      // against a node's one-hot axis 16 << axis: one AND)
    PN_DEV int kz() const { return perm & 3; }
    PN_DEV int kx() const { return (perm & 3) == 0 ? 2 : 0; }   // kz = 0: x <-> z swapped
    PN_DEV int ky() const { return (perm & 3) == 1 ? 2 : 1; }   // kz = 1: y <-> z swapped
    PN_DEV bool cull_ok() const { return (perm & 4) != 0; }
};

PN_DEV RayP make_ray(f3 o, f3 d, int mode) {
    RayP r;
    r.o = o; r.d = d;
    r.inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    int kz = 2;
    if (d.z == 0.0f) kz = (pnm_fabs(d.x) > pnm_fabs(d.y)) ? 0 : 1;
    float dz = comp(d, kz);
    // z-slab culling needs finite rays and a non-tiny z so no sheared
    // coordinate can overflow into NaN edge functions (Culling).
    bool fin = pnm_fabs(o.x) < 1e6f && pnm_fabs(o.y) < 1e6f && pnm_fabs(o.z) < 1e6f &&
               pnm_fabs(d.x) < 1e6f && pnm_fabs(d.y) < 1e6f && pnm_fabs(d.z) < 1e6f;
    bool cull = (mode != 0) && fin && pnm_fabs(dz) >= 1e-12f;
    r.perm = kz | (cull ? 4 : 0) | (d.x < 0.0f ? 16 : 0) | (d.y < 0.0f ? 32 : 0) | (d.z < 0.0f ? 64 : 0);
    return r;
}

// BoundIntersect (:213-228) on one box, plus the box's z-slab interval in the
// triangle test's frame (zlo, zhi) for culling.
PN_DEV bool box_test(const RayP& r, float mnx, float mny, float mnz, float mxx, float mxy,
                     float mxz, float& zlo, float& zhi) {
    float fx = (mxx - r.o.x) * r.inv.x, fy = (mxy - r.o.y) * r.inv.y, fz = (mxz - r.o.z) * r.inv.z;
    float nx = (mnx - r.o.x) * r.inv.x, ny = (mny - r.o.y) * r.inv.y, nz = (mnz - r.o.z) * r.inv.z;
    float tmaxx = fmax_(fx, nx), tmaxy = fmax_(fy, ny), tmaxz = fmax_(fz, nz);
    float tminx = fmin_(fx, nx), tminy = fmin_(fy, ny), tminz = fmin_(fz, nz);
    float t1 = fmin_(tmaxx, fmin_(tmaxy, tmaxz));
    float t0 = fmax_(tminx, fmax_(tminy, tminz));
    const int kz = r.kz();
    float zf = kz == 2 ? fz : (kz == 0 ? fx : fy);
    float zn = kz == 2 ? nz : (kz == 0 ? nx : ny);
    zlo = zn < zf ? zn : zf;   // NaN -> comparisons below fail -> never culled
    zhi = zn < zf ? zf : zn;
    return t1 >= t0;
}

// Culling predicate: every triangle inside a box with this z-slab is rejected by
// the watertight test at the current tMax (proof in DESIGN.md, "Culling").
PN_DEV bool zcull(const RayP& r, float zlo, float zhi, float tmax_c) {
    return r.cull_ok() && (zhi <= 0.0f || (zlo > tmax_c && zlo > 1e-20f));
}

// Watertight triangle test front half (:254-318 / :360-424).  IDENT: the
// caller guarantees the permutation is the identity (kz = 2, i.e. rd.z != 0),
// which skips the component selects; the arithmetic is the same.
template <bool IDENT = false>
PN_DEV bool tri_test(const RayP& r, const float4& t0, const float4& t1, const float4& t2,
                     float tMax, float& e0o, float& e1o, float& e2o, float& deto, float& tso) {
    f3 p0 = mk3(t0.x, t0.y, t0.z), p1 = mk3(t0.w, t1.x, t1.y), p2 = mk3(t1.z, t1.w, t2.x);
    f3 P0 = sub(p0, r.o), P1 = sub(p1, r.o), P2 = sub(p2, r.o);
    const int kx = IDENT ? 0 : r.kx(), ky = IDENT ? 1 : r.ky(), kz = IDENT ? 2 : r.kz();
    float P0x = comp(P0, kx), P0y = comp(P0, ky), P0z = comp(P0, kz);
    float P1x = comp(P1, kx), P1y = comp(P1, ky), P1z = comp(P1, kz);
    float P2x = comp(P2, kx), P2y = comp(P2, ky), P2z = comp(P2, kz);
    // Sx = dir[kx]/dir[kz], written as the reference's (P.z * dir[kx]) * invDz
    const float sx = comp(r.d, kx), sy = comp(r.d, ky), invDz = comp(r.inv, kz);
    P0x = P0x - (P0z * sx) * invDz; P0y = P0y - (P0z * sy) * invDz; P0z = P0z * invDz;
    P1x = P1x - (P1z * sx) * invDz; P1y = P1y - (P1z * sy) * invDz; P1z = P1z * invDz;
    P2x = P2x - (P2z * sx) * invDz; P2y = P2y - (P2z * sy) * invDz; P2z = P2z * invDz;
    float e0 = P1x * P2y - P1y * P2x;
    float e1 = P2x * P0y - P2y * P0x;
    float e2 = P0x * P1y - P0y * P1x;
    // the reference's early-outs (:300-318) as one branch-free predicate: the
    // arithmetic has no side effects, so evaluating it for rejected triangles
    // changes nothing, and every comparison keeps its NaN semantics
    const float det = (e0 + e1) + e2;
    const float tScaled = (e0 * P0z + e1 * P1z) + e2 * P2z;
    const float tmd = tMax * det;
    const bool mixed = ((e0 < 0) | (e1 < 0) | (e2 < 0)) & ((e0 > 0) | (e1 > 0) | (e2 > 0));
    const bool rejPos = (det > 0) & ((tScaled <= 0) | (tScaled > tmd));
    const bool rejNeg = (det < 0) & ((tScaled >= 0) | (tScaled < tmd));
    e0o = e0; e1o = e1; e2o = e2; deto = det; tso = tScaled;
    return !(mixed | (det == 0) | rejPos | rejNeg);
}

PN_DEV void decode_leaf(const DevScene& s, uint32_t ref, int& start, int& cnt) {
    if (!s.has_leaf_table) {            // packed encoding (pt_common.h)
        // (an opaque mask: see pt_wf.h wf_tri_index -- a plain one was dropped
        // ahead of a 64-bit address multiply)
        asm("v_and_b32 %0, 0xffffff, %1" : "=v"(start) : "v"(ref));
        cnt = (int)((ref >> 24) & 0x7fu);
    } else if (ref & REF_TABLE) {
        int2 e = s.leaf_table[PT_CHECK(s.fault, ref & 0x3fffffffu, s.n_leaf_table, PT_SITE_LEAF_TABLE)];
        start = e.x; cnt = e.y;
    } else {
        start = (int)((ref >> 7) & 0x7fffffu);
        cnt = (int)(ref & 0x7fu);
    }
}

// BVHIntersect (ANY = false, returns the last accepted triangle) and
// BVHIntersectP (ANY = true): reference visit order, private stack of far
// children (used by the one-ray-per-lane kernels: primary pass and v1).
template <bool ANY>
PN_DEV bool traverse(const DevScene& s, const RayP& r, float& tMax, int& hitTri) {
    float zlo, zhi;
    if (!box_test(r, s.root_min[0], s.root_min[1], s.root_min[2], s.root_max[0], s.root_max[1],
                  s.root_max[2], zlo, zhi))
        return false;
    uint32_t stackRef[PT_STACK];
    float stackZ[PT_STACK];
    int sp = 0;
    uint32_t cur = s.root_ref;
    bool hit = false;
    const float cullScale = 1.000001f;
    for (;;) {
        if (!(cur & REF_LEAF)) {
            const float4* n = s.nodes + 4 * (size_t)cur;
            float4 a = n[0], b = n[1], c = n[2];
            uint4 m = *reinterpret_cast<const uint4*>(n + 3);
            float tmc = tMax * cullScale;
            float zloL, zhiL, zloR, zhiR;
            bool hL = box_test(r, a.x, a.y, a.z, a.w, b.x, b.y, zloL, zhiL);
            bool hR = box_test(r, b.z, b.w, c.x, c.y, c.z, c.w, zloR, zhiR);
            if (hL && zcull(r, zloL, zhiL, tmc)) hL = false;
            if (hR && zcull(r, zloR, zhiR, tmc)) hR = false;
            bool rightFirst = comp(r.d, (int)m.w) < 0;       // :448
            uint32_t nearRef = rightFirst ? m.y : m.x, farRef = rightFirst ? m.x : m.y;
            bool hNear = rightFirst ? hR : hL, hFar = rightFirst ? hL : hR;
            float zFar = rightFirst ? zloL : zloR;
            if (hNear) {
                if (hFar) { stackRef[sp] = farRef; stackZ[sp] = zFar; ++sp; }
                cur = nearRef;
                continue;
            }
            if (hFar) { cur = farRef; continue; }
        } else {
            int start, cnt;
            decode_leaf(s, cur, start, cnt);
            for (int i = start; i < start + cnt; ++i) {
                const float4* t = s.tris + 3 * (size_t)i;
                float e0, e1, e2, det, ts;
                if (tri_test(r, t[0], t[1], t[2], tMax, e0, e1, e2, det, ts)) {
                    if (ANY) return true;
                    tMax = ts * (1.0f / det);
                    hitTri = i;
                    hit = true;
                }
            }
        }
        // pop (far children re-checked against the tMax found meanwhile)
        for (;;) {
            if (sp == 0) return hit;
            --sp;
            cur = stackRef[sp];
            if (!(r.cull_ok() && stackZ[sp] > tMax * cullScale && stackZ[sp] > 1e-20f)) break;
        }
    }
}
