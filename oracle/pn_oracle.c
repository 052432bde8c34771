/*
 * oracle/pn_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of
 * shaders/ray_tracing.comp (PnRayTracing).  See pn_oracle.h for the pinning
 * status ("integrator parity unpinned by the reference itself").
 *
 * Every function restates the GLSL it cites, in the GLSL's own evaluation
 * order (left-to-right binary ops, no contraction, IEEE binary32, correctly
 * rounded / and sqrt).  Where GLSL leaves a result undefined the choice made
 * here is written next to it; the HIP kernel makes the same choices.
 *
 * Deliberately literal: reference-layout records fetched per access,
 * a 128-entry traversal stack, no tMax box culling -- this is the algorithm
 * the reference runs, not a fast one.
 *
 * Build: gcc -O2 -std=c11 -fopenmp -ffp-contract=off -fno-fast-math
 *        -fno-math-errno -fPIC -shared  (oracle/Makefile)
 */
#include "pn_oracle.h"
#include "pn_libm.h"
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- constants (ray_tracing.comp:5-9) ------------------------------------ */
#define FLOAT_MAX 10000000.0f
#define PI 3.1415926535897f
#define InvPI 0.318309886183f
#define ShadowEpsilon 0.0001f

/* ---- GLSL vector semantics ------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } f2;
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return V3(s * a.x, s * a.y, s * a.z); }
static inline v3 divs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
/* dot = x0*y0 + x1*y1 + x2*y2, left to right */
static inline float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* GLSL 4.50 8.5: cross(x,y) = (x1*y2 - y1*x2, x2*y0 - y2*x0, x0*y1 - y0*x1) */
static inline v3 cross(v3 a, v3 b) {
    return V3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline float length(v3 a) { return sqrtf(dot(a, a)); }
/* normalize(x) = x / length(x) (GLSL 4.50 8.5) */
static inline v3 normalize(v3 a) { return divs(a, length(a)); }
/* glm::normalize (glm 0.9.9.8 func_geometric.inl:88, inversesqrt = 1/sqrt):
 * only for the CPU-header semantics of pno_intersect */
static v3 glm_normalize(v3 a) { return muls(a, 1.0f / sqrtf(dot(a, a))); }
/* min/max: GLSL undefined for NaN; here NaN-dropping (IEEE minNum/maxNum),
 * first operand on ties. */
static inline float fmin_(float a, float b) { return (b < a || a != a) ? b : a; }
static inline float fmax_(float a, float b) { return (b > a || a != a) ? b : a; }
static inline float clampf(float x, float lo, float hi) { return fmin_(fmax_(x, lo), hi); }
/* mix(x,y,a) = x*(1-a) + y*a (GLSL 4.50 8.3) */
static inline float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
static inline v3 mixv(v3 x, v3 y, float a) {
    return V3(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a));
}
static inline float sqr(float x) { return x * x; }                      /* :626 */
static inline int iszero3(v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
static inline float comp(v3 a, int i) { return i == 0 ? a.x : i == 1 ? a.y : a.z; }

/* ---- records (ray_tracing.comp:11-74) ------------------------------------ */
typedef struct { v3 position, normal, tangent, bitangent; f2 texcoord; } Vertex;
typedef struct {
    v3 emssive, baseColor;
    float subsurface, metallic, specular, specularTint, roughness, anisotropic;
    float sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission;
} Material;
typedef struct { v3 pMin, pMax; } Bound;
typedef struct { int indices[3]; int materialId, textureId; float area; } Triangle;
typedef struct { Bound bound; int axis, rightChild, startIndex, endIndex; } BVHNode;
typedef struct { v3 origin, dir; float tMax; } Ray;
typedef struct { int index; float prefixArea; } Light;
typedef struct { v3 position, normal; f2 texcoord; int materialId, textureId; float time; } Interaction;

typedef struct {
    const pno_scene* s;
    const pno_frame* f;
    /* invocation state (ray_tracing.comp:99-100, 497) */
    int px, py;
    uint32_t frameCount;
    uint32_t seed;
    int bounce;
    pno_stats* st;
    /* 0: the GLSL's rules (what pno_render uses).  Otherwise a mask of the
     * reference CPU headers' rules, for pinning against them (pno_intersect):
     * SEM_TIE   triangle.hpp:75-76 rejects tScaled >= tMax*det (ties keep the
     *           FIRST triangle; the GLSL keeps the last),
     * SEM_BOX   bound.hpp:31-47 clips the slab to [0, tMax] with std::max/min,
     * SEM_NORM  glm::normalize = v * (1/sqrt(dot(v,v))) (glm func_geometric.inl:88). */
    int sem;
} Ctx;
#define SEM_TIE 1
#define SEM_BOX 2
#define SEM_NORM 4

/* texelFetch on an RGB32F buffer texture: out-of-range -> 0 (robust access). */
static inline v3 texel(const float* buf, int n_texels, int i) {
    if (i < 0 || i >= n_texels) return V3(0.0f, 0.0f, 0.0f);
    return V3(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]);
}

/* GetVertex / GetVertexPosition / GetVertexNormal  (:102-120) */
static Vertex GetVertex(const Ctx* c, int i) {
    int off = i * 5, n = c->s->n_vertices * 5;
    Vertex v;
    v.position = texel(c->s->vertices, n, off + 0);
    v.normal = texel(c->s->vertices, n, off + 1);
    v.tangent = texel(c->s->vertices, n, off + 2);
    v.bitangent = texel(c->s->vertices, n, off + 3);
    v3 t = texel(c->s->vertices, n, off + 4);
    v.texcoord.x = t.x; v.texcoord.y = t.y;
    return v;
}
static v3 GetVertexPosition(const Ctx* c, int i) { return texel(c->s->vertices, c->s->n_vertices * 5, i * 5); }
static v3 GetVertexNormal(const Ctx* c, int i) { return texel(c->s->vertices, c->s->n_vertices * 5, i * 5 + 1); }

/* GetMaterial (:122-144).  Reference bug kept: clearcoatGloss/IOR/transmission
 * are assigned from param3, not param4 (:139-142). */
static Material GetMaterial(Ctx* c, int i) {
    int off = i * 6, n = c->s->n_materials * 6;
    const float* b = c->s->materials;
    Material m;
    c->st->material_fetches++;
    m.emssive = texel(b, n, off + 0);
    m.baseColor = texel(b, n, off + 1);
    v3 p1 = texel(b, n, off + 2);
    m.subsurface = p1.x; m.metallic = p1.y; m.specular = p1.z;
    v3 p2 = texel(b, n, off + 3);
    m.specularTint = p2.x; m.roughness = p2.y; m.anisotropic = p2.z;
    v3 p3 = texel(b, n, off + 4);
    m.sheen = p3.x; m.sheenTint = p3.y; m.clearcoat = p3.z;
    (void)texel(b, n, off + 5);               /* param4: fetched, unused */
    m.clearcoatGloss = p3.x; m.IOR = p3.y; m.transmission = p3.z;
    return m;
}

/* GetTriangle (:146-155): ints are int(float) (truncation). */
static Triangle GetTriangle(const Ctx* c, int i) {
    int off = i * 2, n = c->s->n_triangles * 2;
    Triangle t;
    v3 a = texel(c->s->triangles, n, off + 0);
    v3 p = texel(c->s->triangles, n, off + 1);
    t.indices[0] = (int)a.x; t.indices[1] = (int)a.y; t.indices[2] = (int)a.z;
    t.materialId = (int)p.x; t.textureId = (int)p.y; t.area = p.z;
    return t;
}

/* GetBVHNode (:157-169) */
static BVHNode GetBVHNode(const Ctx* c, int i) {
    int off = i * 4, n = c->s->n_nodes * 4;
    BVHNode node;
    node.bound.pMin = texel(c->s->nodes, n, off + 0);
    node.bound.pMax = texel(c->s->nodes, n, off + 1);
    v3 p1 = texel(c->s->nodes, n, off + 2);
    node.axis = (int)p1.x; node.rightChild = (int)p1.y; node.startIndex = (int)p1.z;
    v3 p2 = texel(c->s->nodes, n, off + 3);
    node.endIndex = (int)p2.x;
    return node;
}

/* GetLight (:171-178) */
static Light GetLight(Ctx* c, int i) {
    Light l;
    v3 p = texel(c->s->lights, c->s->n_lights, i);
    c->st->light_probes++;
    l.index = (int)p.x; l.prefixArea = p.y;
    return l;
}

/* ---- texture sampling ----------------------------------------------------- */
/* GL 4.5 core spec 8.14.2, LINEAR filter, level 0:
 *   u' = s*W - 0.5, i0 = floor(u'), a = frac(u') = u' - floor(u'), i1 = i0+1,
 *   wrapped (CLAMP_TO_EDGE: clamp to [0,W-1]; REPEAT: mod W);
 *   tau = (1-a)(1-b) T00 + a(1-b) T10 + (1-a)b T01 + ab T11, summed left to right.
 * Integer conversion of floor(): clamped in float first so it is defined for
 * any input; NaN coordinates give index 0 and NaN weights. */
static inline int wrap_clamp(float fl, int n) {
    if (fl != fl) return 0;
    fl = fmin_(fmax_(fl, -1.0f), (float)n);
    int i = (int)fl;
    return i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
}
static inline int wrap_repeat(float fl, int n) {
    if (fl != fl) return 0;
    float q = floorf(fl / (float)n);
    float m = fl - (float)n * q;
    m = fmin_(fmax_(m, 0.0f), (float)n);
    int i = (int)m;
    if (i >= n) i -= n;
    if (i < 0) i += n;
    return i;
}

/* texture(sampler2D RGB32F, CLAMP_TO_EDGE, LINEAR) -- HDRImage / RandomHDR */
static v3 sample_rgb32f_clamp(const float* img, int w, int h, f2 uv) {
    float fu = uv.x * (float)w - 0.5f, fv = uv.y * (float)h - 0.5f;
    float flu = floorf(fu), flv = floorf(fv);
    float a = fu - flu, b = fv - flv;
    int i0 = wrap_clamp(flu, w), i1 = wrap_clamp(flu + 1.0f, w);
    int j0 = wrap_clamp(flv, h), j1 = wrap_clamp(flv + 1.0f, h);
    const float* t00 = img + 3 * ((size_t)j0 * w + i0);
    const float* t10 = img + 3 * ((size_t)j0 * w + i1);
    const float* t01 = img + 3 * ((size_t)j1 * w + i0);
    const float* t11 = img + 3 * ((size_t)j1 * w + i1);
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    v3 r;
    r.x = ((w00 * t00[0] + w10 * t10[0]) + w01 * t01[0]) + w11 * t11[0];
    r.y = ((w00 * t00[1] + w10 * t10[1]) + w01 * t01[1]) + w11 * t11[1];
    r.z = ((w00 * t00[2] + w10 * t10[2]) + w01 * t01[2]) + w11 * t11[2];
    return r;
}

/* UNORM8 -> float: c / 255 (GL 2.3.5.1), correctly rounded division. */
static inline float unorm8(uint8_t c) { return (float)c / 255.0f; }
static v3 fetch_u8(const Ctx* c, int t, int i, int j) {
    const pno_scene* s = c->s;
    int ch = s->tex_ch[t];
    size_t stride = (size_t)((s->tex_w[t] * ch + 3) & ~3);
    const uint8_t* p = s->tex_data[t] + (size_t)j * stride + (size_t)i * ch;
    if (ch == 1) return V3(unorm8(p[0]), 0.0f, 0.0f);       /* GL_RED: (r,0,0) */
    if (ch == 2) return V3(unorm8(p[0]), unorm8(p[1]), 0.0f);
    return V3(unorm8(p[0]), unorm8(p[1]), unorm8(p[2]));
}
/* texture(textures[t], uv).rgb (:871): REPEAT, LINEAR (compute shaders have
 * implicit LOD 0, so LINEAR_MIPMAP_LINEAR samples level 0).  Unbound unit -> 0. */
static v3 sample_albedo(Ctx* c, int t, f2 uv) {
    const pno_scene* s = c->s;
    if (t < 0 || t >= s->n_textures || !s->tex_data[t]) return V3(0.0f, 0.0f, 0.0f);
    int w = s->tex_w[t], h = s->tex_h[t];
    float fu = uv.x * (float)w - 0.5f, fv = uv.y * (float)h - 0.5f;
    float flu = floorf(fu), flv = floorf(fv);
    float a = fu - flu, b = fv - flv;
    int i0 = wrap_repeat(flu, w), i1 = wrap_repeat(flu + 1.0f, w);
    int j0 = wrap_repeat(flv, h), j1 = wrap_repeat(flv + 1.0f, h);
    v3 t00 = fetch_u8(c, t, i0, j0), t10 = fetch_u8(c, t, i1, j0);
    v3 t01 = fetch_u8(c, t, i0, j1), t11 = fetch_u8(c, t, i1, j1);
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    c->st->albedo_bytes += 4u * (uint64_t)s->tex_ch[t];
    v3 r;
    r.x = ((w00 * t00.x + w10 * t10.x) + w01 * t01.x) + w11 * t11.x;
    r.y = ((w00 * t00.y + w10 * t10.y) + w01 * t01.y) + w11 * t11.y;
    r.z = ((w00 * t00.z + w10 * t10.z) + w01 * t01.z) + w11 * t11.z;
    return r;
}

/* toSphericalCoord (:181-188): invAtan = (0.1591, 0.3183) as written. */
static f2 toSphericalCoord(v3 v) {
    f2 uv;
    uv.x = pnl_atan2(v.z, v.x);
    uv.y = pnl_asin(v.y);
    uv.x = uv.x * 0.1591f; uv.y = uv.y * 0.3183f;
    uv.x = uv.x + 0.5f;    uv.y = uv.y + 0.5f;
    uv.y = 1.0f - uv.y;
    return uv;
}
/* GetHDRImageColor (:190-193).  HasHDRImage==0 -> unit 29 unbound -> black. */
static v3 GetHDRImageColor(Ctx* c, v3 v) {
    if (!c->s->has_hdr) return V3(0.0f, 0.0f, 0.0f);
    c->st->env_lookups++;
    return sample_rgb32f_clamp(c->s->hdr_rgb, c->s->hdr_w, c->s->hdr_h, toSphericalCoord(v));
}

/* ---- camera (:205-211): row 0 = bottom, no pixel jitter ------------------- */
static Ray CameraGetRay(const Ctx* c, float s, float t) {
    const pno_frame* f = c->f;
    v3 eye = V3(f->eye[0], f->eye[1], f->eye[2]);
    v3 llc = V3(f->lower_left[0], f->lower_left[1], f->lower_left[2]);
    v3 hor = V3(f->horizontal[0], f->horizontal[1], f->horizontal[2]);
    v3 ver = V3(f->vertical[0], f->vertical[1], f->vertical[2]);
    Ray r;
    r.origin = eye;
    r.dir = normalize(sub(add(add(llc, smul(s, hor)), smul(t, ver)), eye));
    r.tMax = FLOAT_MAX;
    return r;
}

/* ---- BoundIntersect (:213-228): whole-line slab test, no tMax, no t>=0 ---- */
static int BoundIntersect(Bound b, Ray r) {
    v3 invdir = V3(1.0f / r.dir.x, 1.0f / r.dir.y, 1.0f / r.dir.z);
    v3 f = mul(sub(b.pMax, r.origin), invdir);
    v3 n = mul(sub(b.pMin, r.origin), invdir);
    v3 tmax = V3(fmax_(f.x, n.x), fmax_(f.y, n.y), fmax_(f.z, n.z));
    v3 tmin = V3(fmin_(f.x, n.x), fmin_(f.y, n.y), fmin_(f.z, n.z));
    float t1 = fmin_(tmax.x, fmin_(tmax.y, tmax.z));
    float t0 = fmax_(tmin.x, fmax_(tmin.y, tmin.z));
    return t1 >= t0;
}

/* bound.hpp:31-47 BoundIntersect of the reference's CPU headers: slab clipped
 * to [0, tMax], std::swap / std::max / std::min (NaN operands drop out of
 * max/min because `a < b` is false).  Only for pno_intersect's pinning mode. */
static int BoundIntersectCPU(Bound b, Ray r, float* h0, float* h1) {
    float t0 = 0.0f, t1 = r.tMax;
    for (int i = 0; i < 3; ++i) {
        float invDir = 1.0f / comp(r.dir, i);
        float tNear = (comp(b.pMin, i) - comp(r.origin, i)) * invDir;
        float tFar = (comp(b.pMax, i) - comp(r.origin, i)) * invDir;
        if (tNear > tFar) { float t = tNear; tNear = tFar; tFar = t; }
        t0 = (t0 < tNear) ? tNear : t0;       /* std::max(t0, tNear) */
        t1 = (tFar < t1) ? tFar : t1;         /* std::min(t1, tFar)  */
        if (t0 > t1) return 0;
    }
    if (h0) *h0 = t0;
    if (h1) *h1 = t1;
    return 1;
}
static int box_hit(const Ctx* c, Bound b, const Ray* r) {
    return (c->sem & SEM_BOX) ? BoundIntersectCPU(b, *r, 0, 0) : BoundIntersect(b, *r);
}

/* ---- GetLightIndex (:237-251) ------------------------------------------- */
static int GetLightIndex(Ctx* c, float u) {
    int lightsSize = c->s->n_lights;
    if (lightsSize == 0) return -1;
    int L = 0, R = lightsSize - 1, ans = -1;
    float randomArea = u * c->s->lights_sum_area;
    while (L <= R) {
        int mid = (L + R) >> 1;
        if (GetLight(c, mid).prefixArea >= randomArea) { ans = mid; R = mid - 1; }
        else L = mid + 1;
    }
    return GetLight(c, ans).index;
}

static inline void swapf(float* a, float* b) { float t = *a; *a = *b; *b = t; }

/* Shared front half of TriangleIntersect / TriangleIntersectP (:254-318,
 * :360-424): PBRT-v3 watertight test, NOT Moller-Trumbore.  Returns 1 and
 * e0,e1,e2,det,tScaled when accepted against ray.tMax with the GLSL's `>`
 * (equal t is ACCEPTED, so ties go to the later triangle). */
static int tri_test(v3 p0, v3 p1, v3 p2, const Ray* ray, int sem,
                    float* e0o, float* e1o, float* e2o, float* deto, float* tso) {
    v3 P0 = sub(p0, ray->origin), P1 = sub(p1, ray->origin), P2 = sub(p2, ray->origin);
    v3 rd = ray->dir;
    if (rd.z == 0.0f) {
        if (pnl_fabs(rd.x) > pnl_fabs(rd.y)) {
            swapf(&P0.x, &P0.z); swapf(&P1.x, &P1.z); swapf(&P2.x, &P2.z); swapf(&rd.x, &rd.z);
        } else {
            swapf(&P0.y, &P0.z); swapf(&P1.y, &P1.z); swapf(&P2.y, &P2.z); swapf(&rd.y, &rd.z);
        }
    }
    float invDz = 1.0f / rd.z;
    P0.x = P0.x - (P0.z * rd.x) * invDz; P0.y = P0.y - (P0.z * rd.y) * invDz; P0.z = P0.z * invDz;
    P1.x = P1.x - (P1.z * rd.x) * invDz; P1.y = P1.y - (P1.z * rd.y) * invDz; P1.z = P1.z * invDz;
    P2.x = P2.x - (P2.z * rd.x) * invDz; P2.y = P2.y - (P2.z * rd.y) * invDz; P2.z = P2.z * invDz;
    float e0 = P1.x * P2.y - P1.y * P2.x;
    float e1 = P2.x * P0.y - P2.y * P0.x;
    float e2 = P0.x * P1.y - P0.y * P1.x;
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return 0; /* :300 (+dup :305) */
    float det = (e0 + e1) + e2;
    if (det == 0) return 0;
    float tScaled = (e0 * P0.z + e1 * P1.z) + e2 * P2.z;
    if (!(sem & SEM_TIE)) {
        if (det > 0 && (tScaled <= 0 || tScaled > ray->tMax * det)) return 0;
        if (det < 0 && (tScaled >= 0 || tScaled < ray->tMax * det)) return 0;
    } else {                                  /* triangle.hpp:75-76 */
        if (det > 0 && (tScaled <= 0 || tScaled >= ray->tMax * det)) return 0;
        if (det < 0 && (tScaled >= 0 || tScaled <= ray->tMax * det)) return 0;
    }
    *e0o = e0; *e1o = e1; *e2o = e2; *deto = det; *tso = tScaled;
    return 1;
}

/* TriangleIntersect (:254-357).  `out Interaction isect` is written only on
 * acceptance (the caller keeps the last accepted hit). */
static int TriangleIntersect(Ctx* c, Triangle tri, Ray* ray, Interaction* isect) {
    Vertex v0 = GetVertex(c, tri.indices[0]);
    Vertex v1 = GetVertex(c, tri.indices[1]);
    Vertex v2 = GetVertex(c, tri.indices[2]);
    v3 p0 = v0.position, p1 = v1.position, p2 = v2.position;
    float e0, e1, e2, det, tScaled;
    c->st->tri_tests++;
    if (!tri_test(p0, p1, p2, ray, c->sem, &e0, &e1, &e2, &det, &tScaled)) return 0;
    c->st->tri_hits++;
    float invDet = 1.0f / det;
    float t = tScaled * invDet;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    f2 uvHit;
    uvHit.x = (v0.texcoord.x * b0 + v1.texcoord.x * b1) + v2.texcoord.x * b2;
    uvHit.y = (v0.texcoord.y * b0 + v1.texcoord.y * b1) + v2.texcoord.y * b2;
    v3 nHit;
    v3 (*nrm)(v3) = (c->sem & SEM_NORM) ? glm_normalize : normalize;
    if (iszero3(v0.normal) || iszero3(v1.normal) || iszero3(v2.normal))
        nHit = nrm(cross(sub(p1, p0), sub(p2, p0)));
    else
        nHit = add(add(muls(v0.normal, b0), muls(v1.normal, b1)), muls(v2.normal, b2));
    if (dot(nHit, ray->dir) > 0) nHit = neg(nHit);
    nHit = nrm(nHit);
    isect->position = add(add(smul(b0, p0), smul(b1, p1)), smul(b2, p2));
    isect->normal = nHit;
    isect->texcoord = uvHit;
    isect->textureId = tri.textureId;
    isect->materialId = tri.materialId;
    isect->time = t;
    ray->tMax = t;
    return 1;
}

/* TriangleIntersectP (:360-427) */
static int TriangleIntersectP(Ctx* c, Triangle tri, const Ray* ray) {
    v3 p0 = GetVertexPosition(c, tri.indices[0]);
    v3 p1 = GetVertexPosition(c, tri.indices[1]);
    v3 p2 = GetVertexPosition(c, tri.indices[2]);
    float e0, e1, e2, det, tScaled;
    c->st->tri_tests++;
    return tri_test(p0, p1, p2, ray, c->sem, &e0, &e1, &e2, &det, &tScaled);
}

/* BVHIntersect (:429-461) / BVHIntersectP (:464-494).  128-entry stack; the
 * unconditionally pushed child is box-tested at pop, the other at push. */
#define STACK_SIZE 128
static int BVHIntersect(Ctx* c, Ray* r, Interaction* isect) {
    int nodeStack[STACK_SIZE], top = 0;
    nodeStack[top++] = 0;
    int hit = 0;
    c->st->traversals++;
    while (top > 0) {
        int curId = nodeStack[--top];
        BVHNode node = GetBVHNode(c, curId);
        c->st->node_pops++;
        if (!box_hit(c, node.bound, r)) continue;
        if (node.rightChild == -1) {
            for (int i = node.startIndex; i < node.endIndex; ++i)
                if (TriangleIntersect(c, GetTriangle(c, i), r, isect)) hit = 1;
        } else {
            if (top + 2 > STACK_SIZE) { c->st->stack_overflow = 1; return hit; }
            c->st->sibling_tests++;
            if (comp(r->dir, node.axis) < 0) {
                nodeStack[top++] = curId + 1;
                BVHNode rc = GetBVHNode(c, node.rightChild);
                if (box_hit(c, rc.bound, r)) nodeStack[top++] = node.rightChild;
            } else {
                nodeStack[top++] = node.rightChild;
                BVHNode lc = GetBVHNode(c, curId + 1);
                if (box_hit(c, lc.bound, r)) nodeStack[top++] = curId + 1;
            }
        }
    }
    return hit;
}

static int BVHIntersectP(Ctx* c, const Ray* r) {
    int nodeStack[STACK_SIZE], top = 0;
    nodeStack[top++] = 0;
    c->st->traversals++;
    while (top > 0) {
        int curId = nodeStack[--top];
        BVHNode node = GetBVHNode(c, curId);
        c->st->node_pops++;
        if (!box_hit(c, node.bound, r)) continue;
        if (node.rightChild == -1) {
            for (int i = node.startIndex; i < node.endIndex; ++i)
                if (TriangleIntersectP(c, GetTriangle(c, i), r)) return 1;
        } else {
            if (top + 2 > STACK_SIZE) { c->st->stack_overflow = 1; return 0; }
            c->st->sibling_tests++;
            if (comp(r->dir, node.axis) < 0) {
                nodeStack[top++] = curId + 1;
                BVHNode rc = GetBVHNode(c, node.rightChild);
                if (box_hit(c, rc.bound, r)) nodeStack[top++] = node.rightChild;
            } else {
                nodeStack[top++] = node.rightChild;
                BVHNode lc = GetBVHNode(c, curId + 1);
                if (box_hit(c, lc.bound, r)) nodeStack[top++] = curId + 1;
            }
        }
    }
    return 0;
}

/* ---- pinning hook: the intersection routines on caller rays ------------- */
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static void put_isect(uint32_t* o, int hit, const Interaction* is, float tmax_after) {
    memset(o, 0, 13 * sizeof(uint32_t));
    o[0] = (uint32_t)hit;
    if (hit && is) {
        o[1] = fbits(is->position.x); o[2] = fbits(is->position.y); o[3] = fbits(is->position.z);
        o[4] = fbits(is->normal.x); o[5] = fbits(is->normal.y); o[6] = fbits(is->normal.z);
        o[7] = fbits(is->texcoord.x); o[8] = fbits(is->texcoord.y);
        o[9] = (uint32_t)is->textureId; o[10] = (uint32_t)is->materialId; o[11] = fbits(is->time);
    }
    o[12] = fbits(tmax_after);
}

int pno_intersect(const pno_scene* scene, const float* rays, int n, int kind, int sem,
                  const int* idx, uint32_t* out, int threads) {
    if (!scene || !rays || !out || n < 0 || kind < 0 || kind > 4) return -1;
    if ((kind >= 2) && !idx) return -1;
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#else
    int nt = 1; (void)threads;
#endif
    int overflow = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256) num_threads(nt) reduction(|:overflow)
#endif
    for (int i = 0; i < n; ++i) {
        pno_stats st;
        memset(&st, 0, sizeof st);
        Ctx c;
        memset(&c, 0, sizeof c);
        c.s = scene; c.st = &st; c.sem = sem;
        const float* q = rays + 7 * (size_t)i;
        Ray r;
        r.origin = V3(q[0], q[1], q[2]); r.dir = V3(q[3], q[4], q[5]); r.tMax = q[6];
        Interaction is;
        memset(&is, 0, sizeof is);
        uint32_t* o = out + 13 * (size_t)i;
        int hit = 0;
        switch (kind) {
        case 0: hit = BVHIntersect(&c, &r, &is); put_isect(o, hit, &is, r.tMax); break;
        case 1: hit = BVHIntersectP(&c, &r); put_isect(o, hit, 0, r.tMax); break;
        case 2: hit = TriangleIntersect(&c, GetTriangle(&c, idx[i]), &r, &is); put_isect(o, hit, &is, r.tMax); break;
        case 3: hit = TriangleIntersectP(&c, GetTriangle(&c, idx[i]), &r); put_isect(o, hit, 0, r.tMax); break;
        default: {
            Bound b = GetBVHNode(&c, idx[i]).bound;
            float h0 = 0.0f, h1 = 0.0f;
            const int cpu = (sem & SEM_BOX) != 0;
            hit = cpu ? BoundIntersectCPU(b, r, &h0, &h1) : BoundIntersect(b, r);
            memset(o, 0, 13 * sizeof(uint32_t));
            o[0] = (uint32_t)hit;
            if (hit && cpu) { o[1] = fbits(h0); o[2] = fbits(h1); }
        }
        }
        overflow |= st.stack_overflow;
    }
    return overflow ? -6 : 0;
}

/* ---- RNG (:499-557) ------------------------------------------------------- */
uint32_t pno_wang_hash(uint32_t* seed) {
    uint32_t s = *seed;
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    *seed = s;
    return s;
}

/* Sobol direction numbers V[8*32] (:508-510): 8 dims x 32 bits. */
static const uint32_t SOBOL_V[256] = {
#include "sobol_v.inc"
};

static inline uint32_t grayCode(uint32_t i) { return i ^ (i >> 1); }    /* :513 */
/* sobol (:518-526): float(result) * (1.0f/float(0xFFFFFFFFu)); float(0xFFFFFFFF)
 * rounds to 2^32, so the scale is exactly 2^-32. */
float pno_sobol(uint32_t d, uint32_t i) {
    uint32_t result = 0, offset = d * 32u;
    for (uint32_t j = 0; i != 0; i >>= 1, j++)
        if ((i & 1u) != 0) result ^= SOBOL_V[(j + offset) & 255u];
    return (float)result * (1.0f / (float)0xFFFFFFFFu);
}
/* Rand0To1 (:528-530): float(u32) / 4294967296.0 (may round up to 1.0). */
static inline float Rand0To1(Ctx* c) { return (float)pno_wang_hash(&c->seed) / 4294967296.0f; }
static f2 sobolVec2(uint32_t i, uint32_t b) {                              /* :533 */
    f2 r; r.x = pno_sobol(b * 2u, grayCode(i)); r.y = pno_sobol(b * 2u + 1u, grayCode(i));
    return r;
}
/* CranleyPattersonRotation (:539-557): seed uses x*SCREEN_WIDTH, y*SCREEN_HEIGHT
 * and 114514/1919 == 59 (integer division). */
static f2 CranleyPattersonRotation(const Ctx* c, f2 p) {
    uint32_t pseed = ((uint32_t)(c->px * c->f->width) * 1973u +
                      (uint32_t)(c->py * c->f->height) * 9277u +
                      (uint32_t)(114514 / 1919) * 26699u) | 1u;
    float u = (float)pno_wang_hash(&pseed) / 4294967296.0f;
    float v = (float)pno_wang_hash(&pseed) / 4294967296.0f;
    p.x += u; if (p.x > 1) p.x -= 1; if (p.x < 0) p.x += 1;
    p.y += v; if (p.y > 1) p.y -= 1; if (p.y < 0) p.y += 1;
    return p;
}

/* ---- environment importance sampling (:560-576) --------------------------- */
static v3 SampleHDRImage(Ctx* c, v3* L, float* pdf) {
    float r1 = Rand0To1(c), r2 = Rand0To1(c);
    const pno_scene* s = c->s;
    f2 uv = {r1, r2};
    c->st->env_samples++;
    v3 param = sample_rgb32f_clamp(s->random_hdr, s->hdr_w, s->hdr_h, uv);
    param.y = 1.0f - param.y;
    float phi = (2.0f * PI) * (param.x - 0.5f);
    float theta = PI * (param.y - 0.5f);
    float ct = pnl_cos(theta);
    *L = V3(ct * pnl_cos(phi), pnl_sin(theta), ct * pnl_sin(phi));
    *pdf = param.z;
    float sinTheta = fmax_(1e-10f, pnl_sin(theta));
    float convert = (float)(s->hdr_w * s->hdr_h / 2) / (((2.0f * PI) * PI) * sinTheta);
    *pdf = *pdf * convert;
    f2 xy = {param.x, param.y};
    return sample_rgb32f_clamp(s->hdr_rgb, s->hdr_w, s->hdr_h, xy);
}

/* TriangleSample (:598-624) */
static Interaction TriangleSample(const Ctx* c, Triangle tri, f2 u) {
    float su0 = sqrtf(u.x);
    f2 b = {1.0f - su0, u.y * su0};
    v3 p0 = GetVertexPosition(c, tri.indices[0]);
    v3 p1 = GetVertexPosition(c, tri.indices[1]);
    v3 p2 = GetVertexPosition(c, tri.indices[2]);
    v3 n0 = GetVertexNormal(c, tri.indices[0]);
    v3 n1 = GetVertexNormal(c, tri.indices[1]);
    v3 n2 = GetVertexNormal(c, tri.indices[2]);
    Interaction res;
    float b2 = (1.0f - b.x) - b.y;
    res.position = add(add(muls(p0, b.x), muls(p1, b.y)), muls(p2, b2));
    if (iszero3(n0) || iszero3(n1) || iszero3(n2))
        res.normal = normalize(cross(sub(p1, p0), sub(p2, p0)));
    else
        res.normal = add(add(muls(n0, b.x), muls(n1, b.y)), muls(n2, b2));
    res.normal = normalize(res.normal);
    res.texcoord = b;
    res.textureId = tri.textureId;
    res.materialId = tri.materialId;
    res.time = 0.0f;
    return res;
}

/* BuildTangentSpace / TangentToWorld (:629-639) */
static void BuildTangentSpace(v3 n, v3* t, v3* b) {
    if (n.z > 0.9999995f) *t = V3(1.0f, 0.0f, 0.0f);
    else *t = normalize(cross(n, V3(0.0f, 0.0f, 1.0f)));
    *b = cross(n, *t);
}
static v3 TangentToWorld(v3 t, v3 b, v3 n, v3 v) {
    return add(add(smul(v.x, t), smul(v.y, b)), smul(v.z, n));
}
/* SampleCosineHemisphere (:642-647): non-standard (theta = rand radians). */
static v3 SampleCosineHemisphere(Ctx* c, v3 n, v3 t, v3 b) {
    float theta = Rand0To1(c), r = Rand0To1(c);
    float x = r * pnl_sin(theta), y = r * pnl_cos(theta);
    float z = sqrtf((1.0f - sqr(x)) - sqr(y));
    return TangentToWorld(t, b, n, V3(x, y, z));
}

/* ---- Disney BRDF pieces (:649-680) --------------------------------------- */
static float SchlickFresnel(float u) {
    float m = clampf(1.0f - u, 0.0f, 1.0f);
    float m2 = m * m;
    return (m2 * m2) * m;
}
static float GTR1(float NdotH, float a) {
    if (a >= 1) return 1.0f / PI;
    float a2 = a * a;
    float t = 1.0f + ((a2 - 1.0f) * NdotH) * NdotH;
    return (a2 - 1.0f) / ((PI * pnl_log(a2)) * t);
}
static float GTR2(float NdotH, float a) {
    float a2 = a * a;
    float t = 1.0f + ((a2 - 1.0f) * NdotH) * NdotH;
    return a2 / ((PI * t) * t);
}
static float GTR2_aniso(float NdotH, float HdotX, float HdotY, float ax, float ay) {
    return 1.0f / (((PI * ax) * ay) * sqr((sqr(HdotX / ax) + sqr(HdotY / ay)) + NdotH * NdotH));
}
static float smithG_GGX(float NdotV, float alphaG) {
    float a = alphaG * alphaG;
    float b = NdotV * NdotV;
    return 1.0f / (NdotV + sqrtf((a + b) - a * b));
}
static float smithG_GGX_aniso(float NdotV, float VdotX, float VdotY, float ax, float ay) {
    return 1.0f / (NdotV + sqrtf((sqr(VdotX * ax) + sqr(VdotY * ay)) + sqr(NdotV)));
}

/* SampleGTR2 (:687-695): quirks kept -- sinThetaH = max(0, 1 - cos^2) (no
 * sqrt), cosPhiH = 1 - sin^2. */
static v3 SampleGTR2(v3 n, v3 t, v3 b, v3 v, float r1, float r2, float alpha) {
    float phiH = (2.0f * PI) * r1;
    float cosThetaH = sqrtf((1.0f - r2) / (1.0f + ((alpha * alpha) - 1.0f) * r2));
    float sinThetaH = fmax_(0.0f, 1.0f - sqr(cosThetaH));
    float sinPhiH = pnl_sin(phiH), cosPhiH = 1.0f - sqr(sinPhiH);
    v3 h = V3(sinThetaH * cosPhiH, sinThetaH * sinPhiH, cosThetaH);
    h = TangentToWorld(t, b, n, h);
    return sub(smul(2.0f * dot(v, h), h), v);
}
/* SampleGTR1 (:698-707) */
static v3 SampleGTR1(v3 n, v3 t, v3 b, v3 v, float r1, float r2, float alpha) {
    float phiH = (2.0f * PI) * r1;
    float a2 = alpha * alpha;
    float cosThetaH = sqrtf((1.0f - pnl_pow(a2, 1.0f - r2)) / (1.0f - a2));
    float sinThetaH = fmax_(0.0f, 1.0f - sqr(cosThetaH));
    float sinPhiH = pnl_sin(phiH), cosPhiH = 1.0f - sqr(sinPhiH);
    v3 h = V3(sinThetaH * cosPhiH, sinThetaH * sinPhiH, cosThetaH);
    h = TangentToWorld(t, b, n, h);
    return sub(smul(2.0f * dot(v, h), h), v);
}

/* SampleDisneyBRDF (:742-786): lobe draw r, then SampleCosineHemisphere's two
 * draws only on the diffuse lobe; Sobol (r1,r2) feed GTR2/GTR1. */
static v3 SampleDisneyBRDF(Ctx* c, v3 V, v3 N, v3 T, v3 B, const Material* m,
                           float r1, float r2, float* pdf) {
    float rDiffuse = 1.0f - m->metallic;
    float rSpecular = 1.0f;
    float rClearcoat = 0.25f * m->clearcoat;
    float invSum = 1.0f / ((rDiffuse + rSpecular) + rClearcoat);
    float pDiffuse = rDiffuse * invSum, pSpecular = rSpecular * invSum, pClearcoat = rClearcoat * invSum;
    float r = Rand0To1(c);
    float alphaGTR1 = mixf(0.1f, 0.001f, m->clearcoatGloss);
    float alphaGTR2 = fmax_(0.001f, sqr(m->roughness));
    v3 L;
    if (r <= pDiffuse) L = SampleCosineHemisphere(c, N, T, B);
    else if (r <= pDiffuse + pSpecular) L = SampleGTR2(N, T, B, V, r1, r2, alphaGTR2);
    else L = SampleGTR1(N, T, B, V, r1, r2, alphaGTR1);
    v3 H = normalize(add(L, V));
    float LdotH = dot(L, H), NdotH = dot(N, H), NdotL = dot(N, L);
    float pdfDiffuse = NdotL * InvPI;
    float pdfSpecular = (GTR2(NdotH, alphaGTR2) * NdotH) / (4.0f * LdotH);
    float pdfClearcoat = (GTR1(NdotH, alphaGTR1) * NdotH) / (4.0f * LdotH);
    *pdf = (pDiffuse * pdfDiffuse + pSpecular * pdfSpecular) + pClearcoat * pdfClearcoat;
    return L;
}

/* DisneyBRDF (:788-849), X = T, Y = B. */
static v3 DisneyBRDF(v3 V, v3 N, v3 L, v3 X, v3 Y, const Material* m) {
    float NdotL = dot(N, L), NdotV = dot(N, V);
    if (NdotL < 0 || NdotV < 0) return V3(0.0f, 0.0f, 0.0f);
    v3 H = normalize(add(L, V));
    float NdotH = dot(N, H), LdotH = dot(L, H);
    v3 Cdlin = m->baseColor;
    float Cdlum = (0.3f * Cdlin.x + 0.6f * Cdlin.y) + 0.1f * Cdlin.z;
    v3 Ctint = (Cdlum > 0) ? divs(Cdlin, Cdlum) : V3(1.0f, 1.0f, 1.0f);
    v3 Cspec = smul(m->specular, mixv(V3(1.0f, 1.0f, 1.0f), Ctint, m->specularTint));
    v3 Cspec0 = mixv(smul(0.08f, Cspec), Cdlin, m->metallic);
    v3 Csheen = mixv(V3(1.0f, 1.0f, 1.0f), Ctint, m->sheenTint);
    float Fd90 = 0.5f + ((2.0f * LdotH) * LdotH) * m->roughness;
    float FL = SchlickFresnel(NdotL), FV = SchlickFresnel(NdotV);
    float Fd = mixf(1.0f, Fd90, FL) * mixf(1.0f, Fd90, FV);
    float Fss90 = (LdotH * LdotH) * m->roughness;
    float Fss = mixf(1.0f, Fss90, FL) * mixf(1.0f, Fss90, FV);
    float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
    float aspect = sqrtf(1.0f - m->anisotropic * 0.9f);
    float ax = fmax_(0.001f, sqr(m->roughness) / aspect);
    float ay = fmax_(0.001f, sqr(m->roughness) * aspect);
    float Ds = GTR2_aniso(NdotH, dot(H, X), dot(H, Y), ax, ay);
    float FH = SchlickFresnel(LdotH);
    v3 Fs = mixv(Cspec0, V3(1.0f, 1.0f, 1.0f), FH);
    float Gs = smithG_GGX_aniso(NdotL, dot(L, X), dot(L, Y), ax, ay);
    Gs = Gs * smithG_GGX_aniso(NdotV, dot(V, X), dot(V, Y), ax, ay);
    float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m->clearcoatGloss));
    float Fr = mixf(0.04f, 1.0f, FH);
    float Gr = smithG_GGX(NdotL, 0.25f) * smithG_GGX(NdotV, 0.25f);
    v3 Fsheen = smul(FH * m->sheen, Csheen);
    v3 diffuse = add(smul((1.0f / PI) * mixf(Fd, ss, m->subsurface), Cdlin), Fsheen);
    v3 specular = muls(smul(Gs, Fs), Ds);
    float cc = (((0.25f * Gr) * Fr) * Dr) * m->clearcoat;
    v3 clearcoat = V3(cc, cc, cc);
    return add(add(muls(diffuse, 1.0f - m->metallic), specular), clearcoat);
}

/* ---- PathTracing (:861-972) ---------------------------------------------- */
static v3 PathTracing(Ctx* c, Interaction isect, v3 V) {
    const pno_scene* s = c->s;
    v3 Lo = V3(0.0f, 0.0f, 0.0f);
    v3 cw = V3(1.0f, 1.0f, 1.0f);
    for (c->bounce = 0; c->bounce < c->f->max_bounce_depth; ++c->bounce) {
        v3 P = isect.position, N = isect.normal;
        Material material = GetMaterial(c, isect.materialId);
        if (isect.textureId != -1)
            material.baseColor = sample_albedo(c, isect.textureId, isect.texcoord);
        v3 T, B;
        BuildTangentSpace(N, &T, &B);

        /* direct light (:878-909) */
        v3 LDirect = V3(0.0f, 0.0f, 0.0f);
        float lightPDF = 0.0f;
        int triIndex = GetLightIndex(c, Rand0To1(c));
        if (triIndex != -1) {
            Triangle tri = GetTriangle(c, triIndex);
            f2 u; u.x = Rand0To1(c); u.y = Rand0To1(c);     /* left to right */
            c->st->light_samples++;
            Interaction triangleIsect = TriangleSample(c, tri, u);
            Ray r;
            r.dir = sub(triangleIsect.position, P);
            r.tMax = 1.0f - ShadowEpsilon;
            r.origin = add(P, muls(N, 0.0001f));
            if (!BVHIntersectP(c, &r)) {
                float dis2 = (r.dir.x * r.dir.x + r.dir.y * r.dir.y) + r.dir.z * r.dir.z;
                v3 lightL = normalize(r.dir);
                lightPDF = dis2 / (pnl_fabs(dot(triangleIsect.normal, neg(lightL))) * s->lights_sum_area);
                v3 li = GetMaterial(c, triangleIsect.materialId).emssive;
                v3 lightBRDF = DisneyBRDF(V, N, lightL, T, B, &material);
                LDirect = divs(muls(mul(lightBRDF, li), pnl_fabs(dot(N, lightL))), lightPDF);
            }
        }

        /* environment (:911-926) */
        v3 LEnvironment = V3(0.0f, 0.0f, 0.0f);
        float enPDF = 0.0f;
        if (s->has_hdr) {
            v3 enL;
            v3 enLi = SampleHDRImage(c, &enL, &enPDF);
            Ray enR; enR.origin = P; enR.dir = enL; enR.tMax = FLOAT_MAX;
            if (dot(enL, N) > 0 && !BVHIntersectP(c, &enR)) {
                v3 dBRDF = DisneyBRDF(V, N, enL, T, B, &material);
                LEnvironment = divs(muls(mul(dBRDF, enLi), dot(enL, N)), enPDF);
            }
        }

        /* BRDF sample (:928-934) */
        f2 uv = sobolVec2(c->frameCount + 1u, (uint32_t)c->bounce);
        uv = CranleyPattersonRotation(c, uv);
        float dPDF;
        v3 L = SampleDisneyBRDF(c, V, N, T, B, &material, uv.x, uv.y, &dPDF);
        v3 dBRDF = DisneyBRDF(V, N, L, T, B, &material);
        float NdotL = pnl_fabs(dot(N, L));

        /* "MIS" (:936-938) */
        float invPDFSum = 1.0f / ((enPDF + lightPDF) + dPDF);
        v3 mis = add(muls(LEnvironment, enPDF), muls(LDirect, lightPDF));
        Lo = add(Lo, muls(mul(cw, mis), invPDFSum));

        /* continuation (:950-969) */
        Ray ray;
        ray.origin = add(P, muls(N, 0.0001f));
        ray.dir = L;
        ray.tMax = FLOAT_MAX;
        if (!BVHIntersect(c, &ray, &isect)) {
            if (s->has_hdr) {
                v3 enL = normalize(ray.dir);
                v3 enLi = GetHDRImageColor(c, enL);
                Lo = add(Lo, divs(muls(mul(mul(cw, enLi), dBRDF), NdotL), dPDF));
            }
            return Lo;
        }
        v3 em = GetMaterial(c, isect.materialId).emssive;
        Lo = add(Lo, divs(muls(mul(mul(cw, em), dBRDF), NdotL), dPDF));
        cw = mul(cw, divs(muls(dBRDF, NdotL), dPDF));
        V = neg(ray.dir);
    }
    return Lo;
}

/* ---- main (:975-992) ------------------------------------------------------ */
static void shade_pixel(Ctx* c, float* px4) {
    c->seed = ((uint32_t)c->px * 1973u + (uint32_t)c->py * 9277u + c->frameCount * 26699u) | 1u;
    Ray ray = CameraGetRay(c, (float)c->px / (float)c->f->width, (float)c->py / (float)c->f->height);
    Interaction isect;
    memset(&isect, 0, sizeof isect);
    v3 color;
    const uint64_t np0 = c->st->node_pops, ns0 = c->st->sibling_tests, nt0 = c->st->tri_tests, nh0 = c->st->tri_hits;
    const int prim_hit = BVHIntersect(c, &ray, &isect);
    c->st->prim_node_pops += c->st->node_pops - np0;
    c->st->prim_sibling_tests += c->st->sibling_tests - ns0;
    c->st->prim_tri_tests += c->st->tri_tests - nt0;
    c->st->prim_tri_hits += c->st->tri_hits - nh0;
    if (!prim_hit) {
        color = GetHDRImageColor(c, ray.dir);
    } else {
        v3 em = GetMaterial(c, isect.materialId).emssive;
        color = add(em, PathTracing(c, isect, neg(ray.dir)));
    }
    color = V3(clampf(color.x, 0.0f, 1.0f), clampf(color.y, 0.0f, 1.0f), clampf(color.z, 0.0f, 1.0f));
    float a = 1.0f / (float)(c->frameCount + 1u);
    px4[0] = mixf(px4[0], color.x, a);
    px4[1] = mixf(px4[1], color.y, a);
    px4[2] = mixf(px4[2], color.z, a);
    px4[3] = 1.0f;
    c->st->accum_rmw++;
}

static void stats_add(pno_stats* d, const pno_stats* s) {
    d->samples += s->samples; d->node_pops += s->node_pops; d->sibling_tests += s->sibling_tests;
    d->tri_tests += s->tri_tests; d->tri_hits += s->tri_hits; d->material_fetches += s->material_fetches;
    d->light_probes += s->light_probes; d->light_samples += s->light_samples;
    d->env_samples += s->env_samples; d->env_lookups += s->env_lookups;
    d->albedo_bytes += s->albedo_bytes; d->accum_rmw += s->accum_rmw; d->traversals += s->traversals;
    if (s->stack_overflow) d->stack_overflow = 1;
    d->prim_node_pops += s->prim_node_pops; d->prim_sibling_tests += s->prim_sibling_tests;
    d->prim_tri_tests += s->prim_tri_tests; d->prim_tri_hits += s->prim_tri_hits;
}

int pno_render(const pno_scene* scene, const pno_frame* frame,
               uint32_t first_frame, uint32_t n_frames,
               int y_begin, int y_end, int y_step,
               float* accum, int threads, pno_stats* stats) {
    if (!scene || !frame || !accum || y_step <= 0) return -1;
    if (frame->width <= 0 || frame->height <= 0) return -2;
    if (frame->max_bounce_depth < 0 || frame->max_bounce_depth > 4) return -3;
    if (scene->n_nodes <= 0) return -4;
    if (y_begin < 0) y_begin = 0;
    if (y_end > frame->height) y_end = frame->height;
    int nrows = y_begin < y_end ? (y_end - y_begin + y_step - 1) / y_step : 0;
    pno_stats total;
    memset(&total, 0, sizeof total);
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#else
    int nt = 1; (void)threads;
#endif
    pno_stats* per = (pno_stats*)calloc((size_t)nt, sizeof(pno_stats));
    if (!per) return -5;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
    for (int ri = 0; ri < nrows; ++ri) {
#ifdef _OPENMP
        int tid = omp_get_thread_num();
#else
        int tid = 0;
#endif
        Ctx c;
        c.s = scene; c.f = frame; c.st = &per[tid]; c.py = y_begin + ri * y_step; c.sem = 0;
        for (int x = 0; x < frame->width; ++x) {
            c.px = x;
            float* p = accum + 4 * ((size_t)c.py * frame->width + x);
            for (uint32_t k = 0; k < n_frames; ++k) {
                c.frameCount = first_frame + k;
                shade_pixel(&c, p);
                per[tid].samples++;
            }
        }
    }
    for (int t = 0; t < nt; ++t) stats_add(&total, &per[t]);
    free(per);
    if (stats) stats_add(stats, &total);
    return total.stack_overflow ? -6 : 0;
}

/* ---- math parity helper --------------------------------------------------- */
void pno_math_eval(int fn, const float* a, const float* b, float* out, int n) {
    for (int i = 0; i < n; ++i) {
        float x = a[i], y = b ? b[i] : 0.0f, r = 0.0f;
        uint32_t u;
        switch (fn) {
        case 0: r = pnl_sin(x); break;
        case 1: r = pnl_cos(x); break;
        case 2: r = pnl_atan2(x, y); break;
        case 3: r = pnl_asin(x); break;
        case 4: r = pnl_log(x); break;
        case 5: r = pnl_pow(x, y); break;
        case 6: r = pnl_exp2(x); break;
        case 7: r = sqrtf(x); break;
        case 8: r = x / y; break;
        case 9: u = pnl_f2bits(x); r = (float)u; break;
        case 10: u = pnl_f2bits(x); pno_wang_hash(&u); r = pnl_bits2f(u); break;
        default: r = pnl_nan(); break;
        }
        out[i] = r;
    }
}
