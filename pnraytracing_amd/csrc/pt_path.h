// pnraytracing_amd/csrc/pt_path.h -- path-tracing pieces shared by the
// kernels (hit record, light selection, Sobol, shard rows) and the v1
// one-lane-per-pixel integrator kept for A/B comparison (PNRT_KERNEL_V1).
#pragma once
#include "pt_shade.h"

// ---- Sobol (ray_tracing.comp:508-537) ----------------------------------------------
static const uint32_t kSobolV[256] = {
#include "sobol_v.inc"
};
__constant__ uint32_t c_sobolV[256];

PN_DEV float sobol_dev(uint32_t d, uint32_t i) {
    uint32_t result = 0, offset = d * 32u;
    for (uint32_t j = 0; i != 0; i >>= 1, j++)
        if ((i & 1u) != 0) result ^= c_sobolV[(j + offset) & 255u];
    return (float)result * (1.0f / (float)0xFFFFFFFFu);
}
// sobol_dev(d, i) and sobol_dev(d + 1, i) in one pass over the set bits of i only
// (the same XOR of the same table words: the same bits)
PN_DEV void sobol_pair(uint32_t d, uint32_t i, float& a, float& b) {
    uint32_t ra = 0, rb = 0;
    const uint32_t oa = d * 32u, ob = oa + 32u;
    while (i != 0) {
        const uint32_t j = (uint32_t)__builtin_ctz(i);
        i &= i - 1u;
        ra ^= c_sobolV[(j + oa) & 255u];
        rb ^= c_sobolV[(j + ob) & 255u];
    }
    a = (float)ra * (1.0f / (float)0xFFFFFFFFu);
    b = (float)rb * (1.0f / (float)0xFFFFFFFFu);
}

// ---- per-lane path state --------------------------------------------------------------
struct Hit {      // Interaction (:60-67) of an accepted triangle
    f3 P, N;
    float u, v;
    int mat, tex;
};

// Shading data of the accepted triangle (TriangleIntersect :320-355), recomputed
// from its index: the edge functions do not depend on tMax, so they equal the
// values computed when the triangle was accepted.
// The accepted triangle's records: its 48-B test record (positions, material,
// texture) and its attribute record (the vertices' normals and uvs, i.e. the
// values of vertices[tri_idx[tri]], gathered at upload) -- one fetch level.
struct HitFetch {
    float4 t0, t1, t2, a0, a1, a2, a3;
};
PN_DEV HitFetch hit_fetch(const DevScene& s, int tri) {
    tri = (int)PT_CHECK(s.fault, tri, s.n_tris, PT_SITE_HIT_ATTR);
    HitFetch f;
    const float4* t = s.tris + 3 * (size_t)tri;
    f.t0 = t[0]; f.t1 = t[1]; f.t2 = t[2];
    const float4* ta = s.tri_attr + 4 * (size_t)tri;
    f.a0 = ta[0]; f.a1 = ta[1]; f.a2 = ta[2]; f.a3 = ta[3];
    return f;
}
// Shading data of the accepted triangle (TriangleIntersect :320-355), recomputed
// from its records: the edge functions do not depend on tMax, so they equal the
// values computed when the triangle was accepted.
PN_DEV Hit hit_resolve(const RayP& r, const HitFetch& f) {
    const float4 t0 = f.t0, t1 = f.t1, t2 = f.t2, a0 = f.a0, a1 = f.a1, a2 = f.a2, a3 = f.a3;
    float e0, e1, e2, det, ts;
    tri_test(r, t0, t1, t2, 3.402823466e38f, e0, e1, e2, det, ts);
    float invDet = 1.0f / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    f3 p0 = mk3(t0.x, t0.y, t0.z), p1 = mk3(t0.w, t1.x, t1.y), p2 = mk3(t1.z, t1.w, t2.x);
    f3 n0 = mk3(a0.x, a0.y, a0.z), n1 = mk3(a0.w, a1.x, a1.y), n2 = mk3(a1.z, a1.w, a2.x);
    Hit h;
    h.u = (a2.y * b0 + a2.w * b1) + a3.y * b2;
    h.v = (a2.z * b0 + a3.x * b1) + a3.z * b2;
    f3 nHit;
    if (iszero3(n0) || iszero3(n1) || iszero3(n2)) nHit = normalize(cross(sub(p1, p0), sub(p2, p0)));
    else nHit = add(add(muls(n0, b0), muls(n1, b1)), muls(n2, b2));
    if (dot(nHit, r.d) > 0) nHit = neg(nHit);
    h.N = normalize(nHit);
    h.P = add(add(smul(b0, p0), smul(b1, p1)), smul(b2, p2));
    h.mat = __float_as_int(t2.y);
    h.tex = __float_as_int(t2.z);
    return h;
}
PN_DEV Hit make_hit(const DevScene& s, const RayP& r, int tri) { return hit_resolve(r, hit_fetch(s, tri)); }

// GetLightIndex (:237-251)
PN_DEV int light_index(const DevScene& s, float u) {
    if (s.n_lights == 0) return -1;
    int L = 0, R = s.n_lights - 1, ans = -1;
    float randomArea = u * s.lights_sum_area;
    while (L <= R) {
        int mid = (L + R) >> 1;
        if (s.lights[mid].y >= randomArea) { ans = mid; R = mid - 1; }
        else L = mid + 1;
    }
    if (ans < 0) return 0;            // unreachable for u <= 1 (texelFetch(-1) = 0)
    return (int)s.lights[ans].x;
}

// One sample of PathTracing (:861-972) for a primary hit.
PN_DEV f3 path_trace(const DevScene& s, const FrameParams& fp, Hit isect, f3 V, uint32_t& seed,
                     uint32_t frame, float cpu, float cpv) {
    f3 Lo = mk3(0.f, 0.f, 0.f);
    f3 cw = mk3(1.f, 1.f, 1.f);
    const uint32_t g = (frame + 1u) ^ ((frame + 1u) >> 1);       // grayCode(frameCount+1)
    for (int bounce = 0; bounce < fp.max_depth; ++bounce) {
        f3 P = isect.P, N = isect.N;
        Material m = get_material(s, isect.mat);
        if (isect.tex != -1) m.baseColor = sample_albedo(s, isect.tex, isect.u, isect.v);
        f3 T, B;
        if (N.z > 0.9999995f) T = mk3(1.f, 0.f, 0.f);
        else T = normalize(cross(N, mk3(0.f, 0.f, 1.f)));
        B = cross(N, T);
        BrdfCtx bc = brdf_prepare(V, N, T, B, m);

        // ---- direct light (:878-909)
        f3 LDirect = mk3(0.f, 0.f, 0.f);
        float lightPDF = 0.0f;
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
            f3 dir = sub(lp, P);
            RayP r = make_ray(add(P, muls(N, 0.0001f)), dir, fp.mode);
            float tmax = 1.0f - PT_SHADOW_EPS;
            int dummy;
            if (!traverse<true>(s, r, tmax, dummy)) {
                float dis2 = (dir.x * dir.x + dir.y * dir.y) + dir.z * dir.z;
                f3 lightL = normalize(dir);
                lightPDF = dis2 / (pnm_fabs(dot(ln, neg(lightL))) * s.lights_sum_area);
                f3 li = get_emissive(s, lmat);
                f3 lightBRDF = disney(bc, lightL);
                LDirect = divs(muls(mul(lightBRDF, li), pnm_fabs(dot(N, lightL))), lightPDF);
            }
        }

        // ---- environment (:911-926)
        f3 LEnvironment = mk3(0.f, 0.f, 0.f);
        float enPDF = 0.0f;
        if (s.has_hdr) {
            float r1 = rand01(seed), r2 = rand01(seed);
            f3 enL;
            f3 enLi = sample_env(s, r1, r2, enL, enPDF);
            if (dot(enL, N) > 0) {
                RayP r = make_ray(P, enL, fp.mode);
                float tmax = PT_FLOAT_MAX;
                int dummy;
                if (!traverse<true>(s, r, tmax, dummy)) {
                    f3 dB = disney(bc, enL);
                    LEnvironment = divs(muls(mul(dB, enLi), dot(enL, N)), enPDF);
                }
            }
        }

        // ---- BRDF sample (:928-934)
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
        f3 L;
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
            if (rl <= pDiffuse + pSpecular) {
                cosThetaH = sqrtf((1.0f - sv) / (1.0f + ((alphaGTR2 * alphaGTR2) - 1.0f) * sv));
            } else {
                float a2 = alphaGTR1 * alphaGTR1;
                cosThetaH = sqrtf((1.0f - pnm_pow(a2, 1.0f - sv)) / (1.0f - a2));
            }
            float sinThetaH = fmax_(0.0f, 1.0f - sqr(cosThetaH));
            float sinPhiH = pnm_sin(phiH), cosPhiH = 1.0f - sqr(sinPhiH);
            f3 h = mk3(sinThetaH * cosPhiH, sinThetaH * sinPhiH, cosThetaH);
            h = tangent_to_world(T, B, N, h);
            L = sub(smul(2.0f * dot(V, h), h), V);
        }
        f3 H = normalize(add(L, V));
        float LdotH = dot(L, H), NdotH = dot(N, H), NdotLs = dot(N, L);
        float pdfDiffuse = NdotLs * PT_INVPI;
        float pdfSpecular = (gtr2(NdotH, alphaGTR2) * NdotH) / (4.0f * LdotH);
        float pdfClearcoat = (gtr1(NdotH, alphaGTR1) * NdotH) / (4.0f * LdotH);
        float dPDF = (pDiffuse * pdfDiffuse + pSpecular * pdfSpecular) + pClearcoat * pdfClearcoat;
        f3 dBRDF = disney(bc, L);
        float NdotL = pnm_fabs(dot(N, L));

        // ---- "MIS" (:936-938)
        float invPDFSum = 1.0f / ((enPDF + lightPDF) + dPDF);
        f3 mis = add(muls(LEnvironment, enPDF), muls(LDirect, lightPDF));
        Lo = add(Lo, muls(mul(cw, mis), invPDFSum));

        // ---- continuation (:950-969)
        RayP r = make_ray(add(P, muls(N, 0.0001f)), L, fp.mode);
        float tmax = PT_FLOAT_MAX;
        int hitTri = -1;
        if (!traverse<false>(s, r, tmax, hitTri)) {
            if (s.has_hdr) {
                f3 enL = normalize(L);
                f3 enLi = env_color(s, enL);
                Lo = add(Lo, divs(muls(mul(mul(cw, enLi), dBRDF), NdotL), dPDF));
            }
            return Lo;
        }
        isect = make_hit(s, r, hitTri);
        f3 em = get_emissive(s, isect.mat);
        Lo = add(Lo, divs(muls(mul(mul(cw, em), dBRDF), NdotL), dPDF));
        cw = mul(cw, divs(muls(dBRDF, NdotL), dPDF));
        V = neg(L);
    }
    return Lo;
}

// Local row index -> image row for the shard (rows y with (y / band) % n == shard).
PN_DEV int shard_row(int r, int band, int n_shards, int shard) {
    int blk = r / band;
    return (blk * n_shards + shard) * band + (r - blk * band);
}

// main (:975-992), all frames of the call for one pixel.  Grid: 16x16-pixel
// blocks (4 waves of 8x8 pixels) over the shard's rows.
__global__ void __launch_bounds__(256) pt_render_kernel(DevScene s, FrameParams fp, float4* accum) {
    const int lane = threadIdx.x;
    const int wave = lane >> 6, l = lane & 63;
    const int lx = (wave & 1) * 8 + (l & 7), ly = (wave >> 1) * 8 + (l >> 3);
    const int px = blockIdx.x * 16 + lx;
    const int lr = blockIdx.y * 16 + ly;
    if (px >= fp.width || lr >= fp.rows) return;
    const int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    if (py >= fp.height) return;

    const size_t pix = (size_t)py * fp.width + px;
    float4 acc = accum[pix];

    // CranleyPattersonRotation shift (:539-546): constant per pixel
    uint32_t pseed = ((uint32_t)(px * fp.width) * 1973u + (uint32_t)(py * fp.height) * 9277u +
                      (uint32_t)(114514 / 1919) * 26699u) | 1u;
    float cpu = rand01(pseed), cpv = rand01(pseed);

    // CameraGetRay (:205-211) and the primary closest hit, shared by all frames
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    float sx = (float)px / (float)fp.width, sy = (float)py / (float)fp.height;
    f3 dir = normalize(sub(add(add(mk3(fp.llc[0], fp.llc[1], fp.llc[2]), smul(sx, mk3(fp.hor[0], fp.hor[1], fp.hor[2]))),
                               smul(sy, mk3(fp.ver[0], fp.ver[1], fp.ver[2]))), eye));
    RayP r0 = make_ray(eye, dir, fp.mode);
    float tmax = PT_FLOAT_MAX;
    int hitTri = -1;
    bool hit0 = traverse<false>(s, r0, tmax, hitTri);
    Hit h0;
    f3 base;                      // emissive of the primary hit, or the env colour on a miss
    if (hit0) { h0 = make_hit(s, r0, hitTri); base = get_emissive(s, h0.mat); }
    else base = env_color(s, dir);

    for (uint32_t k = 0; k < fp.n_frames; ++k) {
        const uint32_t frame = fp.first_frame + k;
        uint32_t seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + frame * 26699u) | 1u;
        f3 color = base;
        if (hit0) color = add(base, path_trace(s, fp, h0, neg(dir), seed, frame, cpu, cpv));
        color = mk3(clampf(color.x, 0.f, 1.f), clampf(color.y, 0.f, 1.f), clampf(color.z, 0.f, 1.f));
        float a = 1.0f / (float)(frame + 1u);
        acc.x = mixf(acc.x, color.x, a);
        acc.y = mixf(acc.y, color.y, a);
        acc.z = mixf(acc.z, color.z, a);
        acc.w = 1.0f;
    }
    accum[pix] = acc;
}

