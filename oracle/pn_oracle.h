/*
 * oracle/pn_oracle.h -- TEST INFRASTRUCTURE.  CPU restatement of the radiance
 * integrator in PnRayTracing's shaders/ray_tracing.comp (the GLSL reference),
 * used ONLY as the parity checker (tests/, __graft_entry__.smoke()) and as
 * bench.py's cpu_baseline ("kind": "port").  The product path never loads it.
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   - RNG (wang_hash), Sobol, camera, host arrays: pinned by known answers
 *     computed from the reference's own sources (SURVEY 8c KATs, oracle/_ref).
 *   - Ray/triangle, slab and BVH traversal arithmetic: PINNED bit for bit to
 *     the reference's own CPU code (triangle.hpp, bound.hpp, BVH.hpp compiled
 *     here, oracle/ref/isect_driver.cpp) on ~3.4M seeded ray queries per
 *     scene over C1/C2/C4/C5, with the three documented rule differences
 *     (ties, slab clipping, glm::normalize) switched by pno_intersect's `sem`
 *     (tests/test_isect_pin.py).
 *   - The shading half (Disney BRDF, sampling, MIS, env lookups): unpinned by
 *     the reference itself (the GLSL cannot execute in this container -- no
 *     GL 4.5 context / no glslang -- and the reference has no CPU version of
 *     it and no golden images or tests).  Its faithfulness rests on
 *     line-by-line restatement of ray_tracing.comp, with every function
 *     citing the lines it follows.
 *
 * Inputs are the reference's own flattened float arrays exactly as main.cpp
 * packs them (main.cpp:409-524): vertex 15 f, material 18 f, triangle 6 f,
 * BVH node 12 f, light 3 f; integers stored as floats.
 */
#ifndef PN_ORACLE_H
#define PN_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PNO_MAX_TEXTURES 20

typedef struct {
    const float* vertices;   int n_vertices;    /* 15 floats / vertex  */
    const float* materials;  int n_materials;   /* 18 floats / material */
    const float* triangles;  int n_triangles;   /* 6 floats / triangle */
    const float* nodes;      int n_nodes;       /* 12 floats / node    */
    const float* lights;     int n_lights;      /* 3 floats / light    */
    float lights_sum_area;
    /* albedo textures (units 5..24): GL-unpacked rows, row stride
     * = align4(w*channels) bytes (GL_UNPACK_ALIGNMENT 4, main.cpp:545) */
    int n_textures;
    const uint8_t* tex_data[PNO_MAX_TEXTURES];
    int tex_w[PNO_MAX_TEXTURES], tex_h[PNO_MAX_TEXTURES], tex_ch[PNO_MAX_TEXTURES];
    /* environment (units 29/30, shader.hpp:126-225) */
    int has_hdr, hdr_w, hdr_h;
    const float* hdr_rgb;     /* w*h*3, row 0 = first row of the file */
    const float* random_hdr;  /* w*h*3 inverse-CDF table              */
} pno_scene;

typedef struct {
    float eye[3], lower_left[3], horizontal[3], vertical[3]; /* camera.hpp:28-30 */
    int width, height;          /* SCREEN_WIDTH / SCREEN_HEIGHT uniforms */
    int max_bounce_depth;       /* MAX_BOUNCE_DEPTH uniform (1..4)       */
} pno_frame;

/* Algorithmic-byte counters, summed over all samples. */
typedef struct {
    uint64_t samples;
    uint64_t node_pops, sibling_tests, tri_tests, tri_hits;
    uint64_t material_fetches, light_probes, light_samples, env_samples;
    uint64_t env_lookups, albedo_bytes, accum_rmw;
    uint64_t traversals;
    int stack_overflow;          /* set if any traversal needed > 128 entries */
    /* the camera-ray share of node_pops / sibling_tests / tri_tests / tri_hits
     * (the GPU traces the un-jittered camera ray once per pixel per call, the
     * bounce rays in its per-bounce traversal kernel) */
    uint64_t prim_node_pops, prim_sibling_tests, prim_tri_tests, prim_tri_hits;
} pno_stats;

/* Render frames [first_frame, first_frame + n_frames) for the rows
 * y = y_begin, y_begin + y_step, ... < y_end of a width*height RGBA32F
 * accumulation image (row 0 = bottom, as imagePos.y), blending each frame
 * with the progressive mean of ray_tracing.comp:988-991.  `threads` = OpenMP
 * threads (<=0: all).  Returns 0, or <0 on invalid input. */
int pno_render(const pno_scene* scene, const pno_frame* frame,
               uint32_t first_frame, uint32_t n_frames,
               int y_begin, int y_end, int y_step,
               float* accum, int threads, pno_stats* stats);

/* Evaluate one PN-libm / IEEE primitive over n inputs (math parity test).
 * fn: 0 sin, 1 cos, 2 atan2(a,b), 3 asin, 4 log, 5 pow(a,b), 6 exp2,
 *     7 sqrt, 8 a/b, 9 float(uint32 bits of a), 10 wang_hash(bits of a) */
void pno_math_eval(int fn, const float* a, const float* b, float* out, int n);

/* Pinning hook (tests only): the oracle's intersection routines on caller
 * rays, n x 7 floats (origin, dir, tMax).  kind 0: closest hit over the BVH
 * (BVHIntersect, :429-461), 1: any hit (BVHIntersectP, :464-494), 2: one
 * triangle idx[i] (TriangleIntersect, :254-357), 3: TriangleIntersectP
 * (:360-427), 4: the box of node idx[i] (BoundIntersect, :213-228).
 * sem 0: the GLSL's rules (as rendered); otherwise a mask of the reference
 * CPU headers' rules: 1 triangle.hpp:75-76 `>=` ties, 2 bound.hpp:31-47
 * [0,tMax] slab clipping with std::max/min, 4 glm::normalize; sem 7 makes the
 * shared arithmetic comparable bit for bit with the reference compiled here
 * (oracle/ref/isect_driver.cpp).
 * out: n x 13 words: hit, position[3], normal[3], texcoord[2], textureId,
 * materialId, time (floats as bits; zeros when no hit), ray tMax after; for
 * kind 4 with sem & 2: hit, t0, t1.  Returns 0, -1 bad args, -6 stack overflow. */
int pno_intersect(const pno_scene* scene, const float* rays, int n, int kind, int sem,
                  const int* idx, uint32_t* out, int threads);

/* Known-answer helpers. */
uint32_t pno_wang_hash(uint32_t* seed);
float pno_sobol(uint32_t d, uint32_t i);

#ifdef __cplusplus
}
#endif
#endif
