// pnraytracing_amd/csrc/pnrt_device.hip -- libpnrt.so: C ABI (include/pnrt.h),
// scene re-layout and the gfx950 radiance-integrator kernel that replaces
// PnRayTracing's shaders/ray_tracing.comp.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math
//        -fPIC -shared  (pnraytracing_amd/build.py)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pnrt.h"
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

// ---- per-lane path state --------------------------------------------------------------
struct Hit {      // Interaction (:60-67) of an accepted triangle
    f3 P, N;
    float u, v;
    int mat, tex;
};

// Shading data of the accepted triangle (TriangleIntersect :320-355), recomputed
// from its index: the edge functions do not depend on tMax, so they equal the
// values computed when the triangle was accepted.
PN_DEV Hit make_hit(const DevScene& s, const RayP& r, int tri) {
    const float4* t = s.tris + 3 * (size_t)tri;
    float4 t0 = t[0], t1 = t[1], t2 = t[2];
    float e0, e1, e2, det, ts;
    tri_test(r, t0, t1, t2, 3.402823466e38f, e0, e1, e2, det, ts);
    float invDet = 1.0f / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    int4 id = s.tri_idx[tri];
    float4 va0 = s.verts[2 * (size_t)id.x], vb0 = s.verts[2 * (size_t)id.x + 1];
    float4 va1 = s.verts[2 * (size_t)id.y], vb1 = s.verts[2 * (size_t)id.y + 1];
    float4 va2 = s.verts[2 * (size_t)id.z], vb2 = s.verts[2 * (size_t)id.z + 1];
    f3 p0 = mk3(t0.x, t0.y, t0.z), p1 = mk3(t0.w, t1.x, t1.y), p2 = mk3(t1.z, t1.w, t2.x);
    f3 n0 = mk3(va0.w, vb0.x, vb0.y), n1 = mk3(va1.w, vb1.x, vb1.y), n2 = mk3(va2.w, vb2.x, vb2.y);
    Hit h;
    h.u = (vb0.z * b0 + vb1.z * b1) + vb2.z * b2;
    h.v = (vb0.w * b0 + vb1.w * b1) + vb2.w * b2;
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

__global__ void pt_pack_rows_kernel(const float4* accum, float4* dst, int width, int rows, int band,
                                    int n_shards, int shard) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t total = (size_t)rows * width;
    if (i >= total) return;
    int r = (int)(i / width), x = (int)(i - (size_t)r * width);
    int y = shard_row(r, band, n_shards, shard);
    dst[i] = accum[(size_t)y * width + x];
}

__global__ void pt_math_kernel(int fn, const float* a, const float* b, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i], r;
    uint32_t u;
    switch (fn) {
    case 0: r = pnm_sin(x); break;
    case 1: r = pnm_cos(x); break;
    case 2: r = pnm_atan2(x, y); break;
    case 3: r = pnm_asin(x); break;
    case 4: r = pnm_log(x); break;
    case 5: r = pnm_pow(x, y); break;
    case 6: r = pnm_exp2(x); break;
    case 7: r = sqrtf(x); break;
    case 8: r = x / y; break;
    case 9: u = __float_as_uint(x); r = (float)u; break;
    case 10: u = __float_as_uint(x); wang_hash(u); r = __uint_as_float(u); break;
    default: r = pnm_nan(); break;
    }
    out[i] = r;
}

// =====================================================================================
// host side
// =====================================================================================
struct pnrt_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // scene
    std::vector<void*> scene_allocs;
    DevScene scene{};
    bool has_scene = false;
    int max_depth = 0, n_interior = 0, root_is_leaf = 0;
    int64_t scene_bytes = 0;
    // env + textures
    void* hdr = nullptr;
    void* rnd = nullptr;
    void* tex[PT_MAX_TEXTURES] = {};
    int tex_w[PT_MAX_TEXTURES] = {}, tex_h[PT_MAX_TEXTURES] = {};
    float* unorm8 = nullptr;
    // frame
    int width = 0, height = 0, max_bounce = 4;
    pnrt_camera cam{};
    bool has_frame = false;
    float4* accum = nullptr;
    int mode = PNRT_TRAVERSE_ZCULL;
};

static int set_err(pnrt_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}
#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return set_err(ctx, PNRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

static void free_scene(pnrt_ctx* c) {
    for (void* p : c->scene_allocs) (void)hipFree(p);
    c->scene_allocs.clear();
    c->has_scene = false;
}

template <class T>
static int upload(pnrt_ctx* c, const std::vector<T>& v, const T** out) {
    void* p = nullptr;
    size_t bytes = v.size() * sizeof(T);
    if (bytes == 0) { *out = nullptr; return 0; }
    HIPCHK(c, hipMalloc(&p, bytes));
    c->scene_allocs.push_back(p);
    HIPCHK(c, hipMemcpy(p, v.data(), bytes, hipMemcpyHostToDevice));
    c->scene_bytes += (int64_t)bytes;
    *out = static_cast<const T*>(p);
    return 0;
}

static inline int fint(float f) { return (int)f; }   // GLSL int(float)

extern "C" {

const char* pnrt_version(void) { return "pnrt-mi355x 0.1 (gfx950)"; }

int pnrt_create(int device, pnrt_ctx** out) {
    if (!out) return PNRT_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PNRT_E_HIP;
    pnrt_ctx* c = new pnrt_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return PNRT_E_HIP;
    }
    c->stream = c->own_stream;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_sobolV), kSobolV, sizeof kSobolV) != hipSuccess) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PNRT_E_HIP;
    }
    float lut[256];
    for (int i = 0; i < 256; ++i) lut[i] = (float)i / 255.0f;   // GL UNORM8 -> float
    if (hipMalloc(&c->unorm8, sizeof lut) != hipSuccess ||
        hipMemcpy(c->unorm8, lut, sizeof lut, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PNRT_E_HIP;
    }
    *out = c;
    return PNRT_OK;
}

void pnrt_destroy(pnrt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    free_scene(c);
    (void)hipFree(c->hdr); (void)hipFree(c->rnd);
    for (void* t : c->tex) (void)hipFree(t);
    (void)hipFree(c->unorm8);
    (void)hipFree(c->accum);
    (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* pnrt_last_error(pnrt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pnrt_set_stream(pnrt_ctx* c, void* s) {
    if (!c) return PNRT_E_ARG;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
    return PNRT_OK;
}

int pnrt_set_options(pnrt_ctx* c, int mode) {
    if (!c) return PNRT_E_ARG;
    if (mode != PNRT_TRAVERSE_EXACT && mode != PNRT_TRAVERSE_ZCULL) return set_err(c, PNRT_E_ARG, "unknown traverse mode");
    c->mode = mode;
    return PNRT_OK;
}

int pnrt_upload_scene(pnrt_ctx* c, const float* V, int nv, const float* M, int nm, const float* T, int nt,
                      const float* N, int nn, const float* Lt, int nl, float lsum) {
    if (!c) return PNRT_E_ARG;
    if (!V || !M || !T || !N || nv <= 0 || nm <= 0 || nt <= 0 || nn <= 0 || nl < 0 || (nl > 0 && !Lt))
        return set_err(c, PNRT_E_ARG, "upload_scene: missing or empty arrays");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    free_scene(c);
    c->scene_bytes = 0;

    // triangles: positions gathered in BVH order, ids validated
    std::vector<float4> tris((size_t)nt * 3);
    std::vector<int4> tidx(nt);
    for (int i = 0; i < nt; ++i) {
        const float* t = T + 6 * (size_t)i;
        int id[3] = {fint(t[0]), fint(t[1]), fint(t[2])};
        for (int k = 0; k < 3; ++k)
            if (id[k] < 0 || id[k] >= nv) return set_err(c, PNRT_E_SCENE, "triangle " + std::to_string(i) + " has an out-of-range vertex index");
        int mat = fint(t[3]), tex = fint(t[4]);
        if (mat < 0 || mat >= nm) return set_err(c, PNRT_E_SCENE, "triangle " + std::to_string(i) + " has an out-of-range material id");
        const float* p0 = V + 15 * (size_t)id[0];
        const float* p1 = V + 15 * (size_t)id[1];
        const float* p2 = V + 15 * (size_t)id[2];
        float4 a, b, d;
        a.x = p0[0]; a.y = p0[1]; a.z = p0[2]; a.w = p1[0];
        b.x = p1[1]; b.y = p1[2]; b.z = p2[0]; b.w = p2[1];
        int mb, tb; std::memcpy(&mb, &mat, 4); std::memcpy(&tb, &tex, 4);
        d.x = p2[2];
        std::memcpy(&d.y, &mat, 4); std::memcpy(&d.z, &tex, 4); d.w = 0.f;
        (void)mb; (void)tb;
        tris[3 * (size_t)i] = a; tris[3 * (size_t)i + 1] = b; tris[3 * (size_t)i + 2] = d;
        tidx[i] = make_int4(id[0], id[1], id[2], 0);
    }
    std::vector<float4> verts((size_t)nv * 2);
    for (int i = 0; i < nv; ++i) {
        const float* v = V + 15 * (size_t)i;
        verts[2 * (size_t)i] = make_float4(v[0], v[1], v[2], v[3]);
        verts[2 * (size_t)i + 1] = make_float4(v[4], v[5], v[12], v[13]);
    }
    // BVH: validate the reference tree (pre-order, left = id + 1) from the root,
    // number interior nodes, and store child boxes in the parent.
    std::vector<int> dn(nn, -1), depth(nn, 0), order;
    std::vector<int> st{0};
    std::vector<char> seen(nn, 0);
    int maxd = 0;
    while (!st.empty()) {
        int i = st.back(); st.pop_back();
        if (i < 0 || i >= nn || seen[i]) return set_err(c, PNRT_E_SCENE, "BVH node array is not a tree");
        seen[i] = 1;
        const float* n = N + 12 * (size_t)i;
        int rc = fint(n[7]), s0 = fint(n[8]), e0 = fint(n[9]);
        if (rc == -1) {
            if (s0 < 0 || e0 > nt || s0 > e0) return set_err(c, PNRT_E_SCENE, "BVH leaf with bad triangle range");
            continue;
        }
        int ax = fint(n[6]);
        if (ax < 0 || ax > 2 || i + 1 >= nn || rc <= 0 || rc >= nn) return set_err(c, PNRT_E_SCENE, "BVH interior node with bad axis/children");
        dn[i] = (int)order.size();
        order.push_back(i);
        depth[i + 1] = depth[rc] = depth[i] + 1;
        if (depth[i] + 1 > maxd) maxd = depth[i] + 1;
        st.push_back(rc);
        st.push_back(i + 1);
    }
    if (maxd >= PT_STACK - 1)
        return set_err(c, PNRT_E_SCENE, "BVH depth " + std::to_string(maxd) + " exceeds the kernel stack");
    auto childref = [&](int ci, int& ref, int& cnt) {
        const float* n = N + 12 * (size_t)ci;
        if (fint(n[7]) == -1) {
            int s0 = fint(n[8]), e0 = fint(n[9]);
            cnt = e0 - s0;
            ref = cnt > 0 ? s0 : -1;
        } else { ref = dn[ci]; cnt = 0; }
    };
    std::vector<float4> nodes(order.size() * 4);
    for (size_t k = 0; k < order.size(); ++k) {
        int i = order[k];
        const float* n = N + 12 * (size_t)i;
        int rc = fint(n[7]);
        const float* L = N + 12 * (size_t)(i + 1);
        const float* R = N + 12 * (size_t)rc;
        int rl, cl, rr, cr;
        childref(i + 1, rl, cl);
        childref(rc, rr, cr);
        nodes[4 * k + 0] = make_float4(L[0], L[1], L[2], L[3]);
        nodes[4 * k + 1] = make_float4(L[4], L[5], R[0], R[1]);
        nodes[4 * k + 2] = make_float4(R[2], R[3], R[4], R[5]);
        int meta[4] = {rl, rr, (int)((uint32_t)cl | ((uint32_t)fint(n[6]) << 30)), cr};
        std::memcpy(&nodes[4 * k + 3], meta, 16);
    }
    std::vector<float2> lights(nl);
    for (int i = 0; i < nl; ++i) {
        lights[i] = make_float2(Lt[3 * (size_t)i], Lt[3 * (size_t)i + 1]);
        int li = fint(Lt[3 * (size_t)i]);
        if (li < 0 || li >= nt) return set_err(c, PNRT_E_SCENE, "light references an out-of-range triangle");
    }
    std::vector<float> mats(M, M + 18 * (size_t)nm);

    DevScene& s = c->scene;
    int rc;
    if ((rc = upload(c, nodes, &s.nodes)) || (rc = upload(c, tris, &s.tris)) || (rc = upload(c, tidx, &s.tri_idx)) ||
        (rc = upload(c, verts, &s.verts)) || (rc = upload(c, mats, &s.materials)) || (rc = upload(c, lights, &s.lights)))
        return rc;
    s.n_nodes = (int)order.size(); s.n_tris = nt; s.n_verts = nv; s.n_materials = nm; s.n_lights = nl;
    s.lights_sum_area = lsum;
    const float* root = N;
    for (int k = 0; k < 3; ++k) { s.root_min[k] = root[k]; s.root_max[k] = root[3 + k]; }
    childref(0, s.root_ref, s.root_cnt);
    c->root_is_leaf = fint(root[7]) == -1;
    c->n_interior = (int)order.size();
    c->max_depth = maxd;
    c->has_scene = true;
    return PNRT_OK;
}

int pnrt_upload_texture(pnrt_ctx* c, int slot, const uint8_t* px, int w, int h, int ch) {
    if (!c) return PNRT_E_ARG;
    if (slot < 0 || slot >= PT_MAX_TEXTURES || !px || w <= 0 || h <= 0 || ch < 1 || ch > 4)
        return set_err(c, PNRT_E_ARG, "upload_texture: bad arguments");
    HIPCHK(c, hipSetDevice(c->device));
    // glTexImage2D with the default GL_UNPACK_ALIGNMENT 4 (main.cpp:545): row j
    // starts at j * align4(w * ch) in the caller's tightly packed buffer; bytes
    // past the buffer read as 0.  GL_RED -> (r, 0, 0).
    size_t stride = ((size_t)w * ch + 3) & ~(size_t)3, avail = (size_t)w * h * ch;
    std::vector<uint32_t> texels((size_t)w * h);
    for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i) {
            uint32_t rgb[3] = {0, 0, 0};
            for (int k = 0; k < (ch >= 3 ? 3 : ch); ++k) {
                size_t o = (size_t)j * stride + (size_t)i * ch + k;
                rgb[k] = o < avail ? px[o] : 0;
            }
            texels[(size_t)j * w + i] = rgb[0] | (rgb[1] << 8) | (rgb[2] << 16);
        }
    (void)hipFree(c->tex[slot]);
    c->tex[slot] = nullptr;
    HIPCHK(c, hipMalloc(&c->tex[slot], texels.size() * 4));
    HIPCHK(c, hipMemcpy(c->tex[slot], texels.data(), texels.size() * 4, hipMemcpyHostToDevice));
    c->tex_w[slot] = w; c->tex_h[slot] = h;
    return PNRT_OK;
}

int pnrt_upload_env(pnrt_ctx* c, const float* rgb, const float* rnd, int w, int h) {
    if (!c) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)hipFree(c->hdr); (void)hipFree(c->rnd);
    c->hdr = c->rnd = nullptr;
    c->scene.has_hdr = 0;
    if (!rgb) return PNRT_OK;
    if (!rnd || w <= 0 || h <= 0) return set_err(c, PNRT_E_ARG, "upload_env: bad arguments");
    std::vector<float4> a((size_t)w * h), b((size_t)w * h);
    for (size_t i = 0; i < a.size(); ++i) {
        a[i] = make_float4(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 0.f);
        b[i] = make_float4(rnd[3 * i], rnd[3 * i + 1], rnd[3 * i + 2], 0.f);
    }
    HIPCHK(c, hipMalloc(&c->hdr, a.size() * 16));
    HIPCHK(c, hipMalloc(&c->rnd, b.size() * 16));
    HIPCHK(c, hipMemcpy(c->hdr, a.data(), a.size() * 16, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->rnd, b.data(), b.size() * 16, hipMemcpyHostToDevice));
    c->scene.has_hdr = 1;
    c->scene.hdr_w = w; c->scene.hdr_h = h;
    return PNRT_OK;
}

int pnrt_set_frame(pnrt_ctx* c, int w, int h, const pnrt_camera* cam, int depth) {
    if (!c) return PNRT_E_ARG;
    if (w <= 0 || h <= 0 || !cam || depth < 0 || depth > 4)
        return set_err(c, PNRT_E_ARG, "set_frame: bad arguments (MAX_BOUNCE_DEPTH must be 0..4: 8 Sobol dims)");
    HIPCHK(c, hipSetDevice(c->device));
    if (w != c->width || h != c->height || !c->accum) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->accum);
        c->accum = nullptr;
        HIPCHK(c, hipMalloc(&c->accum, (size_t)w * h * 16));
        HIPCHK(c, hipMemsetAsync(c->accum, 0, (size_t)w * h * 16, c->stream));
        c->width = w; c->height = h;
    }
    c->cam = *cam;
    c->max_bounce = depth;
    c->has_frame = true;
    return PNRT_OK;
}

static int shard_rows(int h, int band, int n, int shard) {
    int rows = 0;
    for (int y0 = shard * band; y0 < h; y0 += band * n) rows += (h - y0 < band) ? h - y0 : band;
    return rows;
}

int pnrt_render(pnrt_ctx* c, uint32_t first, uint32_t nf, int band, int nsh, int shard) {
    if (!c) return PNRT_E_ARG;
    if (!c->has_scene || !c->has_frame) return set_err(c, PNRT_E_STATE, "render: upload_scene and set_frame first");
    if (band < 1 || nsh < 1 || shard < 0 || shard >= nsh) return set_err(c, PNRT_E_ARG, "render: bad shard selector");
    if (nf == 0) return PNRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    FrameParams fp;
    std::memcpy(fp.eye, c->cam.eye, 12); std::memcpy(fp.llc, c->cam.lower_left, 12);
    std::memcpy(fp.hor, c->cam.horizontal, 12); std::memcpy(fp.ver, c->cam.vertical, 12);
    fp.width = c->width; fp.height = c->height; fp.max_depth = c->max_bounce;
    fp.first_frame = first; fp.n_frames = nf;
    fp.band = band; fp.n_shards = nsh; fp.shard = shard;
    fp.rows = shard_rows(c->height, band, nsh, shard);
    fp.mode = c->mode;
    if (fp.rows == 0) return PNRT_OK;
    DevScene s = c->scene;
    s.hdr = static_cast<const float4*>(c->hdr);
    s.rnd = static_cast<const float4*>(c->rnd);
    s.n_tex = PT_MAX_TEXTURES;
    for (int i = 0; i < PT_MAX_TEXTURES; ++i) {
        s.tex[i] = static_cast<const uint32_t*>(c->tex[i]);
        s.tex_w[i] = c->tex_w[i]; s.tex_h[i] = c->tex_h[i];
    }
    s.unorm8 = c->unorm8;
    dim3 grid((c->width + 15) / 16, (fp.rows + 15) / 16);
    hipLaunchKernelGGL(pt_render_kernel, grid, dim3(256), 0, c->stream, s, fp, c->accum);
    HIPCHK(c, hipGetLastError());
    return PNRT_OK;
}

int pnrt_reset_accum(pnrt_ctx* c) {
    if (!c) return PNRT_E_ARG;
    if (!c->accum) return PNRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(c->accum, 0, (size_t)c->width * c->height * 16, c->stream));
    return PNRT_OK;
}

int pnrt_read_accum(pnrt_ctx* c, float* out) {
    if (!c || !out) return PNRT_E_ARG;
    if (!c->accum) return set_err(c, PNRT_E_STATE, "read_accum: no frame");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(out, c->accum, (size_t)c->width * c->height * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PNRT_OK;
}

void* pnrt_accum_device_ptr(pnrt_ctx* c) { return c ? c->accum : nullptr; }

int pnrt_pack_rows(pnrt_ctx* c, void* dst, int band, int nsh, int shard) {
    if (!c || !dst) return PNRT_E_ARG;
    if (!c->accum) return set_err(c, PNRT_E_STATE, "pack_rows: no frame");
    if (band < 1 || nsh < 1 || shard < 0 || shard >= nsh) return set_err(c, PNRT_E_ARG, "pack_rows: bad shard selector");
    HIPCHK(c, hipSetDevice(c->device));
    int rows = shard_rows(c->height, band, nsh, shard);
    size_t total = (size_t)rows * c->width;
    if (total == 0) return PNRT_OK;
    hipLaunchKernelGGL(pt_pack_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c->stream,
                       c->accum, static_cast<float4*>(dst), c->width, rows, band, nsh, shard);
    HIPCHK(c, hipGetLastError());
    return PNRT_OK;
}

int pnrt_synchronize(pnrt_ctx* c) {
    if (!c) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PNRT_OK;
}

int pnrt_get_device_info(pnrt_ctx* c, pnrt_device_info* info) {
    if (!c || !info) return PNRT_E_ARG;
    info->n_interior = c->n_interior;
    info->n_triangles = c->scene.n_tris;
    info->max_depth = c->max_depth;
    info->device_bytes = c->scene_bytes;
    info->root_is_leaf = c->root_is_leaf;
    info->stack_limit = PT_STACK;
    return PNRT_OK;
}

int pnrt_debug_math(pnrt_ctx* c, int fn, const float* a, const float* b, float* out, int n) {
    if (!c || !a || !out || n <= 0) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    float *da, *db, *dout;
    size_t bytes = (size_t)n * 4;
    HIPCHK(c, hipMalloc(&da, bytes));
    HIPCHK(c, hipMalloc(&db, bytes));
    HIPCHK(c, hipMalloc(&dout, bytes));
    HIPCHK(c, hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    if (b) HIPCHK(c, hipMemcpy(db, b, bytes, hipMemcpyHostToDevice));
    else HIPCHK(c, hipMemset(db, 0, bytes));
    hipLaunchKernelGGL(pt_math_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, fn, da, db, dout, n);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
    return PNRT_OK;
}

}  // extern "C"
