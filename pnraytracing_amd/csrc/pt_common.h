// pnraytracing_amd/csrc/pt_common.h -- device-side GLSL semantics and scene
// layout shared by the integrator kernels (pnrt_device.hip).
//
// Every helper here reproduces one GLSL 4.50 built-in or one fetch of
// shaders/ray_tracing.comp with the exact IEEE binary32 operation order the
// shader writes (left-to-right binary operators, no contraction), so the
// kernel's output is bit-identical to the CPU parity oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pn_math.h"
#include "pt_diag.h"

// ---- constants (ray_tracing.comp:5-9) ---------------------------------------------
#define PT_FLOAT_MAX 10000000.0f
#define PT_PI 3.1415926535897f
#define PT_INVPI 0.318309886183f
#define PT_SHADOW_EPS 0.0001f

#define PT_MAX_TEXTURES 20
#define PT_LIGHT_SCAN 8      // light lists up to this long are scanned with all probes at once
#define PT_STACK 64          // pending far children per lane (host checks depth)

// ---- device scene layout (built from the reference arrays at upload) ----------------
// Interior node = the reference node's two children's boxes + child refs, 64 B:
//   n0 = (L.min.x, L.min.y, L.min.z, L.max.x)
//   n1 = (L.max.y, L.max.z, R.min.x, R.min.y)
//   n2 = (R.min.z, R.max.x, R.max.y, R.max.z)
//   n3 = (refL, refR, 16 << axis, axis)            (uints; the one-hot axis meets RayP::perm's sign bits)
// child ref (32 bits): interior = node index; REF_LEAF alone = an empty leaf.
// A leaf's triangle range [first, first + count) has one of two encodings, per
// scene (DevScene::has_leaf_table):
//   packed (every leaf's count <= 127, fewer than 2^24 - 1 triangles):
//     REF_LEAF | count << 24 | first -- the trace step keeps this word as its
//     pending range (pt_wf.h wf_has_tri);
//   wide (otherwise): REF_LEAF | [29:7] first | [6:0] count, or REF_LEAF |
//     REF_TABLE | index into leaf_table (int2 first, count) when that does not fit.
// Boxes are the reference floats bit for bit.
// Triangle (BVH order), 48 B: t0 = (p0.xyz, p1.x), t1 = (p1.yz, p2.xy),
//   t2 = (p2.z, matId, texId, -) ; tri_idx = (i0, i1, i2, -)
// Vertex 32 B: v0 = (pos.xyz, n.x), v1 = (n.yz, u, v)
#define REF_LEAF 0x80000000u
#define REF_TABLE 0x40000000u
#define REF_NONE 0xFFFFFFFFu

struct DevScene {
    const float4* nodes;
    const int2* leaf_table;
    const float4* tris;
    const int4* tri_idx;
    const float4* verts;
    const float* materials;     // 18 f / material (reference layout)
    const float2* lights;       // (index as float, prefixArea) as uploaded, zero-padded to >= 8 entries
    const float4* tri_attr;     // 4 float4 / triangle (BVH order): n0 n1 n2 uv0 uv1 uv2 of its vertices
    uint32_t geo_tri_off;       // nodes and tris share one allocation (nodes first): byte offset of tris,
    uint32_t geo_bytes;         // and its size (< 4 GiB - 64: 32-bit buffer offsets in the trace kernel,
                                // whose offsets >= 0xffffffc0 fall outside the range and read zeros)
    const float4* zero4;        // one float4 (0, 0, 0, 0): the load target of lanes that need no data
    const float4* light_rec;    // 7 float4 / light entry (+1 for triangle 0): its triangle's vertex
                                // records va0 vb0 va1 vb1 va2 vb2 and (emission, 0)
    int n_nodes, n_tris, n_verts, n_materials, n_lights;
    float lights_sum_area;
    float root_min[3], root_max[3];
    uint32_t root_ref;
    int has_leaf_table;         // the wide leaf encoding (REF_TABLE refs may exist); 0: packed (pt_common.h)
    int light_scan;             // <= PT_LIGHT_SCAN lights with non-decreasing prefix areas
    float lscan[PT_LIGHT_SCAN]; // their prefix areas, passed by value: scalar (kernel-argument) loads
    int has_hdr, hdr_w, hdr_h;
    float emit_max;             // bound on every |emission| and |env texel| component (NaN: unknown), WF_SKIP_MOOT
    const float4* hdr;          // RGB + pad
    const float4* rnd;          // RandomHDR + pad
    // the same two images as bilinear footprints: record (qj, qi), qi in [0, w],
    // qj in [0, h], holds the 2x2 texels a lookup with left column qi - 1 and
    // bottom row qj - 1 (clamped to the edge) reads -- one 64-B block per lookup
    const float4* hdr_q;
    const float4* rnd_q;
    int n_tex;
    const uint32_t* tex[PT_MAX_TEXTURES];   // RGBA8 texels
    int tex_w[PT_MAX_TEXTURES], tex_h[PT_MAX_TEXTURES];
    const float* unorm8;        // 256-entry c/255 table
    int n_leaf_table;           // entries of leaf_table (>= 1)
    uint32_t* fault;            // the context's fault words (WF_DIAG_BOUNDS builds report through them)
    int diag_force;             // WF_DIAG_BOUNDS builds: PNRT_DIAG_FORCE_OOB (one forced out-of-range fetch)
};

struct FrameParams {
    float eye[3], llc[3], hor[3], ver[3];
    int width, height, max_depth;
    uint32_t first_frame, n_frames;
    int band, n_shards, shard;
    int rows;                   // rows owned by this shard
    int mode;                   // PNRT_TRAVERSE_*
};

// ---- GLSL vector semantics --------------------------------------------------------
struct f3 { float x, y, z; };
PN_DEV f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
PN_DEV f3 add(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
PN_DEV f3 sub(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
PN_DEV f3 mul(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
PN_DEV f3 muls(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
PN_DEV f3 smul(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
PN_DEV f3 divs(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
PN_DEV f3 neg(f3 a) { return mk3(-a.x, -a.y, -a.z); }
PN_DEV float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
PN_DEV f3 cross(f3 a, f3 b) {
    return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
PN_DEV f3 normalize(f3 a) { return divs(a, sqrtf(dot(a, a))); }
// min/max: NaN-dropping, first operand on ties (same choice as the oracle)
PN_DEV float fmin_(float a, float b) { return (b < a || a != a) ? b : a; }
PN_DEV float fmax_(float a, float b) { return (b > a || a != a) ? b : a; }
PN_DEV float clampf(float x, float lo, float hi) { return fmin_(fmax_(x, lo), hi); }
PN_DEV float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
PN_DEV f3 mixv(f3 x, f3 y, float a) { return mk3(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a)); }
PN_DEV float sqr(float x) { return x * x; }
PN_DEV bool iszero3(f3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
PN_DEV float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// ---- RNG (ray_tracing.comp:499-557) --------------------------------------------------
PN_DEV uint32_t wang_hash(uint32_t& seed) {
    uint32_t s = seed;
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    seed = s;
    return s;
}
PN_DEV float rand01(uint32_t& seed) { return (float)wang_hash(seed) / 4294967296.0f; }
