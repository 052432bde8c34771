// pnraytracing_amd/csrc/pt_wave.h -- v2 integrator: persistent state-machine
// megakernel for gfx950.
//
// Work unit = one sample (pixel, frame).  A persistent wave keeps 64 lanes busy:
// lanes that finish a path refill from a wave-local pool of consecutive samples
// (one global atomic per 1024 samples).  Every lane runs a small state machine
//   START -> SETUP(bounce) -> trace light shadow -> trace env shadow
//         -> MIS -> trace continuation -> SETUP(bounce+1) | FINISH
// and ALL rays of the wave (closest-hit and any-hit, any bounce) share ONE
// traversal loop, so a lane never waits for its neighbours' ray type.  The BRDF
// values a bounce needs after its shadow rays are evaluated speculatively in
// SETUP (same float ops, same bits), so no material state is live during
// traversal.  The traversal stack lives in LDS (16 entries/lane, deeper entries
// spill to a per-lane global slab).
//
// The primary hit of each pixel is traced once per pnrt_render call by
// pt_primary_kernel; per-sample colours are blended into the accumulation image
// in frame order by pt_blend_kernel (ray_tracing.comp:988-991).
#pragma once
#include "pt_path.h"

#define PTW_LDS_STACK 16
#define PTW_OVF_STACK 48                  // global spill entries per lane
#define PTW_CHUNK 1024u                   // samples per global dequeue
#define PTW_BLOCK 256

struct WaveArgs {
    const float4* primary;     // 3 float4 per shard pixel
    float4* colors;            // [frame][row][x]
    float4* accum;
    uint2* ovf;                // spill stack, PTW_OVF_STACK per persistent lane
    unsigned int* counter;     // global sample dequeue counter
    uint32_t total_samples;
    int tiles_x;               // 8x8 pixel tiles per row of tiles
    int chunk_frames;          // frames in this launch
    uint32_t first_frame;      // frame of chunk slot 0
};

// sample index -> (pixel x, local row, frame slot): 8x8-pixel tiles, frame-major
// inside a tile, so the 64 samples a wave takes together are one tile x frame.
PN_DEV void sample_coords(const WaveArgs& wa, uint32_t s, int& x, int& lr, int& k) {
    uint32_t per_tile = 64u * (uint32_t)wa.chunk_frames;
    uint32_t tile = s / per_tile, rem = s - tile * per_tile;
    k = (int)(rem >> 6);
    int p = (int)(rem & 63u);
    int ty = (int)(tile / (uint32_t)wa.tiles_x), tx = (int)(tile - (uint32_t)ty * wa.tiles_x);
    x = tx * 8 + (p & 7);
    lr = ty * 8 + (p >> 3);
}

PN_DEV f3 camera_dir(const FrameParams& fp, int px, int py) {
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    float sx = (float)px / (float)fp.width, sy = (float)py / (float)fp.height;
    return normalize(sub(add(add(mk3(fp.llc[0], fp.llc[1], fp.llc[2]), smul(sx, mk3(fp.hor[0], fp.hor[1], fp.hor[2]))),
                             smul(sy, mk3(fp.ver[0], fp.ver[1], fp.ver[2]))),
                         eye));
}

// ---- lane state --------------------------------------------------------------------------
enum : int { ST_IDLE = 0, ST_START, ST_SETUP, ST_TRACE, ST_DONE_TRACE, ST_FINISH };
enum : int { RK_LIGHT = 0, RK_ENV = 1, RK_CONT = 2 };

struct Trav {
    RayP r;
    float tMax;
    int hitTri;
    uint32_t cur;          // REF_NONE = pop next
    int lt, lc;            // leaf triangle cursor / remaining
    int sp;                // stack depth
    bool any, hit;
};

PN_DEV void trav_start(const DevScene& s, Trav& t, f3 o, f3 d, float tmax, bool any, int mode) {
    t.r = make_ray(o, d, mode);
    t.tMax = tmax;
    t.hitTri = -1;
    t.any = any;
    t.hit = false;
    t.sp = 0;
    t.lc = 0;
    float zlo, zhi;
    if (box_test(t.r, s.root_min[0], s.root_min[1], s.root_min[2], s.root_max[0], s.root_max[1], s.root_max[2],
                 zlo, zhi)) {
        t.cur = s.root_ref;
        if (t.cur & REF_LEAF) { decode_leaf(s, t.cur, t.lt, t.lc); t.cur = REF_NONE; }
    } else {
        t.cur = REF_NONE;
    }
}

PN_DEV void stk_push(uint2* lds, uint2* ovf, int lane, int& sp, uint32_t ref, float z) {
    uint2 e = make_uint2(ref, __float_as_uint(z));
    if (sp < PTW_LDS_STACK) lds[sp * PTW_BLOCK + lane] = e;
    else ovf[sp - PTW_LDS_STACK] = e;
    ++sp;
}
PN_DEV uint2 stk_pop(const uint2* lds, const uint2* ovf, int lane, int& sp) {
    --sp;
    return sp < PTW_LDS_STACK ? lds[sp * PTW_BLOCK + lane] : ovf[sp - PTW_LDS_STACK];
}

// One traversal iteration: a triangle test, an interior-node step, or a pop.
// Returns true when the ray has finished (t.hit holds the result).
PN_DEV bool trav_step(const DevScene& s, Trav& t, uint2* lds, uint2* ovf, int lane) {
    if (t.lc > 0) {
        const float4* tp = s.tris + 3 * (size_t)t.lt;
        float e0, e1, e2, det, ts;
        if (tri_test(t.r, tp[0], tp[1], tp[2], t.tMax, e0, e1, e2, det, ts)) {
            t.hit = true;
            if (t.any) return true;
            t.tMax = ts * (1.0f / det);
            t.hitTri = t.lt;
        }
        ++t.lt;
        --t.lc;
        return false;
    }
    if (t.cur == REF_NONE) {
        const float tmc = t.tMax * 1.000001f;
        for (;;) {
            if (t.sp == 0) return true;
            uint2 e = stk_pop(lds, ovf, lane, t.sp);
            float z = __uint_as_float(e.y);
            if (t.r.cull_ok && z > tmc && z > 1e-20f) continue;
            if (e.x & REF_LEAF) decode_leaf(s, e.x, t.lt, t.lc);
            else t.cur = e.x;
            return false;
        }
    }
    const float4* n = s.nodes + 4 * (size_t)t.cur;
    float4 a = n[0], b = n[1], c = n[2];
    uint4 m = *reinterpret_cast<const uint4*>(n + 3);
    const float tmc = t.tMax * 1.000001f;
    float zloL, zhiL, zloR, zhiR;
    bool hL = box_test(t.r, a.x, a.y, a.z, a.w, b.x, b.y, zloL, zhiL);
    bool hR = box_test(t.r, b.z, b.w, c.x, c.y, c.z, c.w, zloR, zhiR);
    if (hL && zcull(t.r, zloL, zhiL, tmc)) hL = false;
    if (hR && zcull(t.r, zloR, zhiR, tmc)) hR = false;
    bool rightFirst = comp(t.r.d, (int)m.z) < 0;          // ray_tracing.comp:448
    uint32_t nearRef = rightFirst ? m.y : m.x, farRef = rightFirst ? m.x : m.y;
    bool hNear = rightFirst ? hR : hL, hFar = rightFirst ? hL : hR;
    float zFar = rightFirst ? zloL : zloR;
    uint32_t go;
    if (hNear) {
        if (hFar) stk_push(lds, ovf, lane, t.sp, farRef, zFar);
        go = nearRef;
    } else if (hFar) {
        go = farRef;
    } else {
        t.cur = REF_NONE;
        return false;
    }
    if (go & REF_LEAF) { decode_leaf(s, go, t.lt, t.lc); t.cur = REF_NONE; }
    else t.cur = go;
    return false;
}

// ---- primary hits (once per call) ------------------------------------------------------------
// record: q0 = (P.xyz, bits(mat)), q1 = (N.xyz, u), q2 = (v, base.xyz); mat = -1 on a miss
// (base = emissive of the hit material, or the env colour of the primary direction)
__global__ void __launch_bounds__(256) pt_primary_kernel(DevScene s, FrameParams fp, float4* rec) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= fp.rows * fp.width) return;
    int lr = i / fp.width, px = i - lr * fp.width;
    int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    f3 dir = camera_dir(fp, px, py);
    RayP r = make_ray(eye, dir, fp.mode);
    float tmax = PT_FLOAT_MAX;
    int hitTri = -1;
    float4 q0, q1, q2;
    if (traverse<false>(s, r, tmax, hitTri)) {
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
    rec[3 * (size_t)i] = q0;
    rec[3 * (size_t)i + 1] = q1;
    rec[3 * (size_t)i + 2] = q2;
}

// ---- the megakernel ---------------------------------------------------------------------------
__global__ void __launch_bounds__(PTW_BLOCK) pt_wave_kernel(DevScene s, FrameParams fp, WaveArgs wa) {
    __shared__ uint2 lds_stack[PTW_LDS_STACK * PTW_BLOCK];
    const int lane_blk = threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint2* ovf = wa.ovf + ((size_t)blockIdx.x * PTW_BLOCK + lane_blk) * PTW_OVF_STACK;
    const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    // wave-local work pool
    uint32_t pool_next = 0, pool_end = 0;
    bool exhausted = false;

    // lane state
    int state = ST_IDLE;
    uint32_t sample = 0;
    int px = 0, py = 0, lrow = 0, slot = 0, bounce = 0;
    uint32_t frame = 0, seed = 0;
    f3 Lo, cw, V, P, N, base;
    float hu = 0.f, hv = 0.f;
    int hmat = -1, htex = -1;
    float cpu = 0.f, cpv = 0.f;
    // bounce candidates (speculatively evaluated in SETUP)
    f3 LD, LE, dBRDF, L, lightDir, enL;
    float pl = 0.f, pe = 0.f, NdotL = 0.f, dPDF = 0.f;
    bool wantLight = false, wantEnv = false;
    int rkind = RK_CONT;
    Trav t;
    t.hit = false; t.sp = 0; t.lc = 0; t.cur = REF_NONE;
    Lo = cw = V = P = N = base = LD = LE = dBRDF = L = lightDir = enL = mk3(0.f, 0.f, 0.f);

    for (;;) {
        // ---------------- refill idle lanes from the wave pool -----------------
        uint64_t idle = __ballot(state == ST_IDLE);
        if (idle != 0 && !exhausted) {
            int n_idle = __popcll(idle);
            if (pool_next >= pool_end) {
                uint32_t base_s = 0;
                if (lane == 0) base_s = atomicAdd(wa.counter, PTW_CHUNK);
                base_s = __shfl(base_s, 0);
                if (base_s >= wa.total_samples) {
                    exhausted = true;
                } else {
                    pool_next = base_s;
                    pool_end = min(base_s + PTW_CHUNK, wa.total_samples);
                }
            }
            if (!exhausted) {
                if (state == ST_IDLE) {
                    uint32_t s_idx = pool_next + (uint32_t)__popcll(idle & lanemask_lt);
                    if (s_idx < pool_end) { sample = s_idx; state = ST_START; }
                }
                pool_next = min(pool_next + (uint32_t)n_idle, pool_end);
            }
        }
        if (exhausted && __ballot(state != ST_IDLE) == 0) break;

        // ---------------- shading: run each lane to its next ray --------------
        while (state != ST_IDLE && state != ST_TRACE) {
            if (state == ST_START) {
                int x, lr, k;
                sample_coords(wa, sample, x, lr, k);
                if (x >= fp.width || lr >= fp.rows) { state = ST_IDLE; continue; }
                px = x; slot = k; lrow = lr;
                py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
                frame = wa.first_frame + (uint32_t)k;
                const float4* rec = wa.primary + 3 * ((size_t)lr * fp.width + x);
                float4 q0 = rec[0], q1 = rec[1], q2 = rec[2];
                base = mk3(q2.y, q2.z, q2.w);
                int mt = __float_as_int(q0.w);
                Lo = mk3(0.f, 0.f, 0.f);
                hmat = mt == -1 ? -1 : (mt & 0x00ffffff);       // -1: primary miss
                if (mt == -1 || fp.max_depth == 0) { state = ST_FINISH; continue; }
                htex = (int)((uint32_t)mt >> 24) - 1;
                P = mk3(q0.x, q0.y, q0.z);
                N = mk3(q1.x, q1.y, q1.z);
                hu = q1.w; hv = q2.x;
                V = neg(camera_dir(fp, px, py));
                cw = mk3(1.f, 1.f, 1.f);
                seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + frame * 26699u) | 1u;
                uint32_t pseed = ((uint32_t)(px * fp.width) * 1973u + (uint32_t)(py * fp.height) * 9277u +
                                  (uint32_t)(114514 / 1919) * 26699u) | 1u;
                cpu = rand01(pseed); cpv = rand01(pseed);
                bounce = 0;
                state = ST_SETUP;
            } else if (state == ST_SETUP) {
                // ---- PathTracing bounce setup (:866-934), all RNG in reference order
                Material m = get_material(s, hmat);
                if (htex != -1) m.baseColor = sample_albedo(s, htex, hu, hv);
                f3 T, B;
                if (N.z > 0.9999995f) T = mk3(1.f, 0.f, 0.f);
                else T = normalize(cross(N, mk3(0.f, 0.f, 1.f)));
                B = cross(N, T);
                BrdfCtx bc = brdf_prepare(V, N, T, B, m);

                LD = mk3(0.f, 0.f, 0.f); pl = 0.f; wantLight = false;
                int triIndex = light_index(s, rand01(seed));
                if (triIndex != -1) {
                    float u0 = rand01(seed), u1 = rand01(seed);
                    int4 id = s.tri_idx[triIndex];
                    float4 va0 = s.verts[2 * (size_t)id.x], vb0 = s.verts[2 * (size_t)id.x + 1];
                    float4 va1 = s.verts[2 * (size_t)id.y], vb1 = s.verts[2 * (size_t)id.y + 1];
                    float4 va2 = s.verts[2 * (size_t)id.z], vb2 = s.verts[2 * (size_t)id.z + 1];
                    float su0 = sqrtf(u0);
                    float bx = 1.0f - su0, by = u1 * su0, bz = (1.0f - bx) - by;
                    f3 p0 = mk3(va0.x, va0.y, va0.z), p1 = mk3(va1.x, va1.y, va1.z), p2 = mk3(va2.x, va2.y, va2.z);
                    f3 n0 = mk3(va0.w, vb0.x, vb0.y), n1 = mk3(va1.w, vb1.x, vb1.y), n2 = mk3(va2.w, vb2.x, vb2.y);
                    f3 lp = add(add(muls(p0, bx), muls(p1, by)), muls(p2, bz));
                    f3 ln;
                    if (iszero3(n0) || iszero3(n1) || iszero3(n2)) ln = normalize(cross(sub(p1, p0), sub(p2, p0)));
                    else ln = add(add(muls(n0, bx), muls(n1, by)), muls(n2, bz));
                    ln = normalize(ln);
                    int lmat = __float_as_int(s.tris[3 * (size_t)triIndex + 2].y);
                    lightDir = sub(lp, P);
                    // speculative: the values used only if the shadow ray is unoccluded
                    float dis2 = (lightDir.x * lightDir.x + lightDir.y * lightDir.y) + lightDir.z * lightDir.z;
                    f3 lightL = normalize(lightDir);
                    pl = dis2 / (pnm_fabs(dot(ln, neg(lightL))) * s.lights_sum_area);
                    f3 li = get_emissive(s, lmat);
                    f3 lightBRDF = disney(bc, lightL);
                    LD = divs(muls(mul(lightBRDF, li), pnm_fabs(dot(N, lightL))), pl);
                    wantLight = true;
                }
                LE = mk3(0.f, 0.f, 0.f); pe = 0.f; wantEnv = false;
                if (s.has_hdr) {
                    float r1 = rand01(seed), r2 = rand01(seed);
                    f3 enLi = sample_env(s, r1, r2, enL, pe);
                    if (dot(enL, N) > 0) {
                        f3 dB = disney(bc, enL);
                        LE = divs(muls(mul(dB, enLi), dot(enL, N)), pe);
                        wantEnv = true;
                    }
                }
                // BRDF sample (:928-934)
                const uint32_t g = (frame + 1u) ^ ((frame + 1u) >> 1);
                float su = sobol_dev(2u * (uint32_t)bounce, g), sv = sobol_dev(2u * (uint32_t)bounce + 1u, g);
                su += cpu; if (su > 1) su -= 1; if (su < 0) su += 1;
                sv += cpv; if (sv > 1) sv -= 1; if (sv < 0) sv += 1;
                float rDiffuse = 1.0f - m.metallic;
                float rClearcoat = 0.25f * m.clearcoat;
                float invSum = 1.0f / ((rDiffuse + 1.0f) + rClearcoat);
                float pDiffuse = rDiffuse * invSum, pSpecular = 1.0f * invSum, pClearcoat = rClearcoat * invSum;
                float rl = rand01(seed);
                float alphaGTR1 = bc.alphaDr;
                float alphaGTR2 = fmax_(0.001f, sqr(m.roughness));
                if (rl <= pDiffuse) {
                    float theta = rand01(seed), rr = rand01(seed);
                    float sth, cth;
                    pnm_sincos(theta, sth, cth);
                    float x = rr * sth, y = rr * cth;
                    float z = sqrtf((1.0f - sqr(x)) - sqr(y));
                    L = tangent_to_world(T, B, N, mk3(x, y, z));
                } else {
                    float phiH = (2.0f * PT_PI) * su;
                    float cosThetaH;
                    if (rl <= pDiffuse + pSpecular)
                        cosThetaH = sqrtf((1.0f - sv) / (1.0f + ((alphaGTR2 * alphaGTR2) - 1.0f) * sv));
                    else {
                        float a2 = alphaGTR1 * alphaGTR1;
                        cosThetaH = sqrtf((1.0f - pnm_pow(a2, 1.0f - sv)) / (1.0f - a2));
                    }
                    float sinThetaH = fmax_(0.0f, 1.0f - sqr(cosThetaH));
                    float sinPhiH = pnm_sin(phiH), cosPhiH = 1.0f - sqr(sinPhiH);
                    f3 h = tangent_to_world(T, B, N, mk3(sinThetaH * cosPhiH, sinThetaH * sinPhiH, cosThetaH));
                    L = sub(smul(2.0f * dot(V, h), h), V);
                }
                f3 H = normalize(add(L, V));
                float LdotH = dot(L, H), NdotH = dot(N, H), NdotLs = dot(N, L);
                float pdfDiffuse = NdotLs * PT_INVPI;
                float pdfSpecular = (gtr2(NdotH, alphaGTR2) * NdotH) / (4.0f * LdotH);
                float pdfClearcoat = (gtr1(NdotH, alphaGTR1) * NdotH) / (4.0f * LdotH);
                dPDF = (pDiffuse * pdfDiffuse + pSpecular * pdfSpecular) + pClearcoat * pdfClearcoat;
                dBRDF = disney(bc, L);
                NdotL = pnm_fabs(dot(N, L));
                state = ST_DONE_TRACE;      // falls into the ray issue logic below
                rkind = -1;
            } else if (state == ST_DONE_TRACE) {
                // consume the finished ray (rkind), then issue the next one
                if (rkind == RK_LIGHT) {
                    if (t.hit) { LD = mk3(0.f, 0.f, 0.f); pl = 0.f; }       // occluded (:890)
                } else if (rkind == RK_ENV) {
                    if (t.hit) LE = mk3(0.f, 0.f, 0.f);                      // occluded (:922)
                } else if (rkind == RK_CONT) {
                    if (!t.hit) {
                        if (s.has_hdr) {
                            f3 enLi = env_color(s, normalize(L));
                            Lo = add(Lo, divs(muls(mul(mul(cw, enLi), dBRDF), NdotL), dPDF));
                        }
                        state = ST_FINISH;
                        continue;
                    }
                    Hit h = make_hit(s, t.r, t.hitTri);
                    f3 em = get_emissive(s, h.mat);
                    Lo = add(Lo, divs(muls(mul(mul(cw, em), dBRDF), NdotL), dPDF));
                    cw = mul(cw, divs(muls(dBRDF, NdotL), dPDF));
                    V = neg(L);
                    P = h.P; N = h.N; hu = h.u; hv = h.v; hmat = h.mat; htex = h.tex;
                    ++bounce;
                    state = (bounce < fp.max_depth) ? ST_SETUP : ST_FINISH;
                    continue;
                }
                if (wantLight) {
                    wantLight = false;
                    rkind = RK_LIGHT;
                    trav_start(s, t, add(P, muls(N, 0.0001f)), lightDir, 1.0f - PT_SHADOW_EPS, true, fp.mode);
                    state = ST_TRACE;
                } else if (wantEnv) {
                    wantEnv = false;
                    rkind = RK_ENV;
                    trav_start(s, t, P, enL, PT_FLOAT_MAX, true, fp.mode);
                    state = ST_TRACE;
                } else {
                    // "MIS" (:936-938), then the continuation ray (:950-956)
                    float invPDFSum = 1.0f / ((pe + pl) + dPDF);
                    f3 mis = add(muls(LE, pe), muls(LD, pl));
                    Lo = add(Lo, muls(mul(cw, mis), invPDFSum));
                    rkind = RK_CONT;
                    trav_start(s, t, add(P, muls(N, 0.0001f)), L, PT_FLOAT_MAX, false, fp.mode);
                    state = ST_TRACE;
                }
            } else {   // ST_FINISH
                f3 color = (hmat == -1) ? base : add(base, Lo);
                color = mk3(clampf(color.x, 0.f, 1.f), clampf(color.y, 0.f, 1.f), clampf(color.z, 0.f, 1.f));
                wa.colors[((size_t)slot * fp.rows + lrow) * fp.width + px] = make_float4(color.x, color.y, color.z, 0.f);
                state = ST_IDLE;
            }
        }

        // ---------------- traversal: one shared loop for every ray -------------
        uint64_t tracing = __ballot(state == ST_TRACE);
        if (tracing == 0) continue;
        int thr = __popcll(tracing) / 3;
        for (;;) {
            if (state == ST_TRACE) {
                if (trav_step(s, t, lds_stack, ovf, lane_blk)) state = ST_DONE_TRACE;
            }
            if (__popcll(__ballot(state == ST_TRACE)) <= thr) break;
        }
    }
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
