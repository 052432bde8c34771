// pnraytracing_amd/csrc/pt_passes.h -- per-call passes shared by the
// integrators: the primary-hit pass (the primary ray has no jitter,
// ray_tracing.comp:980, so its closest hit is traced once per pnrt_render call
// and reused by every frame) and the frame-ordered progressive-mean blend
// (ray_tracing.comp:988-991).
#pragma once
#include "pt_path.h"

PN_DEV f3 camera_dir(const FrameParams& fp, int px, int py) {
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    float sx = (float)px / (float)fp.width, sy = (float)py / (float)fp.height;
    return normalize(sub(add(add(mk3(fp.llc[0], fp.llc[1], fp.llc[2]), smul(sx, mk3(fp.hor[0], fp.hor[1], fp.hor[2]))),
                             smul(sy, mk3(fp.ver[0], fp.ver[1], fp.ver[2]))),
                         eye));
}

// ---- primary hits (once per call) ------------------------------------------------------------
#ifndef PT_PRIM_STK
#define PT_PRIM_STK 8        // primary pass: stack entries per lane in LDS (deeper ones in private memory)
#endif
// BVHIntersect (:429-461) for the primary pass: traverse<false>'s visit order and
// culling, its far-child stack in LDS (entry k of lane tl at lds[k * 256 + tl]).
PN_DEV bool traverse_closest_lds(const DevScene& s, const RayP& r, float& tMax, int& hitTri, uint2* lds, int tl) {
    float zlo, zhi;
    if (!box_test(r, s.root_min[0], s.root_min[1], s.root_min[2], s.root_max[0], s.root_max[1],
                  s.root_max[2], zlo, zhi))
        return false;
    uint2 spill[PT_STACK];
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
                if (hFar) {
                    const uint2 e = make_uint2(farRef, __float_as_uint(zFar));
                    if (sp < PT_PRIM_STK) lds[sp * 256 + tl] = e; else spill[sp - PT_PRIM_STK] = e;
                    ++sp;
                }
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
            const uint2 e = sp < PT_PRIM_STK ? lds[sp * 256 + tl] : spill[sp - PT_PRIM_STK];
            cur = e.x;
            const float z = __uint_as_float(e.y);
            if (!(r.cull_ok() && z > tMax * cullScale && z > 1e-20f)) break;
        }
    }
}

// record: q0 = (P.xyz, bits(mat)), q1 = (N.xyz, u), q2 = (v, base.xyz); mat = -1 on a miss
// (base = emissive of the hit material, or the env colour of the primary direction).
__global__ void __launch_bounds__(256) pt_primary_kernel(DevScene s, FrameParams fp, float4* rec) {
    __shared__ uint2 lds[(PT_PRIM_STK > 0 ? PT_PRIM_STK : 1) * 256];
    // 256 pixels of a row per workgroup (16x16-pixel tiles measured slower)
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)fp.rows * fp.width) return;
    const int lr = (int)(i / fp.width), px = (int)(i - (size_t)lr * fp.width);
    int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    f3 dir = camera_dir(fp, px, py);
    RayP r = make_ray(eye, dir, fp.mode);
    float tmax = PT_FLOAT_MAX;
    int hitTri = -1;
    float4 q0, q1, q2;
    if (PT_PRIM_STK > 0 ? traverse_closest_lds(s, r, tmax, hitTri, lds, threadIdx.x) : traverse<false>(s, r, tmax, hitTri)) {
        Hit h = make_hit(s, r, hitTri);
        f3 em = get_emissive(s, h.mat);
        q0 = make_float4(h.P.x, h.P.y, h.P.z, __int_as_float(h.mat));
        q1 = make_float4(h.N.x, h.N.y, h.N.z, h.u);
        q2 = make_float4(h.v, em.x, em.y, em.z);
        q0.w = __int_as_float((h.mat & 0x00ffffff) | ((h.tex + 1) << 24));   // mat < 2^24, tex in [-1,254]
    } else {
        f3 c = env_color(s, dir);
        q0 = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        q1 = make_float4(0.f, 0.f, 0.f, 0.f);
        q2 = make_float4(0.f, c.x, c.y, c.z);
    }
    rec[3 * i] = q0;
    rec[3 * i + 1] = q1;
    rec[3 * i + 2] = q2;
}

// Frame-ordered progressive mean (ray_tracing.comp:988-991) of one chunk.
__global__ void pt_blend_kernel(FrameParams fp, const float4* colors, float4* accum, int chunk_frames,
                                uint32_t first_frame) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= fp.rows * fp.width) return;
    int lr = i / fp.width, px = i - lr * fp.width;
    int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    size_t pix = (size_t)py * fp.width + px;
    float4 acc = accum[pix];
    for (int k = 0; k < chunk_frames; ++k) {
        float4 c = colors[((size_t)k * fp.rows + lr) * fp.width + px];
        float a = 1.0f / (float)(first_frame + (uint32_t)k + 1u);
        acc.x = mixf(acc.x, c.x, a);
        acc.y = mixf(acc.y, c.y, a);
        acc.z = mixf(acc.z, c.z, a);
        acc.w = 1.0f;
    }
    accum[pix] = acc;
}
