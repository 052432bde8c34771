/*
 * include/pnrt.h -- C ABI of libpnrt.so, the MI355X (gfx950) path-tracing
 * library that replaces PnRayTracing's OpenGL compute-shader hot path
 * (shaders/ray_tracing.comp, dispatched from main.cpp:613).
 *
 * Each entry point replaces one piece of the GL binding contract main.cpp
 * fills today (the reference interface is cited per function).  Inputs are the
 * SAME host-built float arrays main.cpp uploads (integers stored as floats);
 * the library copies caller memory during upload* and never keeps pointers to
 * it.  No torch or HIP types appear in the signatures: streams are passed as
 * opaque pointers (a hipStream_t, or NULL for the context's own stream).
 *
 * Threading: a context belongs to one HIP device and is not thread-safe; use
 * one context per device (one process per GPU in the multi-GPU driver).
 * Errors: every int-returning call returns 0 on success or a negative PNRT_E*
 * code, with a message in pnrt_last_error(ctx).  Nothing calls exit().
 */
#ifndef PNRT_H
#define PNRT_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PNRT_OK 0
#define PNRT_E_ARG (-1)       /* invalid argument                      */
#define PNRT_E_HIP (-2)       /* HIP runtime error                     */
#define PNRT_E_STATE (-3)     /* call out of order (e.g. render before upload) */
#define PNRT_E_SCENE (-4)     /* scene arrays inconsistent / unsupported */
#define PNRT_E_NOMEM (-5)
#define PNRT_E_TRACE (-6)     /* a trace launch may have left queued rays untraced (a bounded */
                              /* wait of its ray queue ran out, or a ray count check failed): */
                              /* the accumulation image is invalid.  Returned by pnrt_render,  */
                              /* pnrt_synchronize, pnrt_read_accum and pnrt_pack_rows once the */
                              /* faulting work has completed (pnrt_synchronize / read_accum    */
                              /* always see it); sticky until pnrt_reset_accum.                */

typedef struct pnrt_ctx pnrt_ctx;

/* camera.hpp:28-30 / the camera.* uniforms set at main.cpp:606-610 */
typedef struct {
    float eye[3], lower_left[3], horizontal[3], vertical[3];
} pnrt_camera;

typedef struct {
    int n_interior;      /* interior BVH nodes in the device layout          */
    int n_triangles;
    int max_depth;       /* deepest reference node (root = 0)                */
    int64_t device_bytes;/* scene bytes resident in HBM                      */
    int root_is_leaf;
    int stack_limit;     /* traversal stack entries available per lane       */
} pnrt_device_info;

/* Options (pnrt_set_options): a traversal mode, optionally | a kernel variant. */
#define PNRT_TRAVERSE_EXACT 0   /* the reference's box visits (no tMax culling)      */
#define PNRT_TRAVERSE_ZCULL 1   /* + provably result-neutral z-slab culling (default) */
#define PNRT_KERNEL_V1 0x100    /* A/B baseline: one lane per pixel, frames in-lane        */
#define PNRT_SERIAL 0x200       /* measurement: one pnrt_render call in flight and a full- */
                                /* occupancy trace grid, so a kernel's launch duration is  */
                                /* its exclusive time (same images; slower end to end)     */
                                /* default: wavefront (setup / trace / shade per bounce)   */

/* "pnrt-mi355x <version> (gfx950) src <sha256[:16] of the device sources>" */
const char* pnrt_version(void);

/* Replaces WindowInit's GL context (main.cpp:64-94): bind HIP device. */
int pnrt_create(int device, pnrt_ctx** out);
void pnrt_destroy(pnrt_ctx* ctx);
const char* pnrt_last_error(pnrt_ctx* ctx);
/* Launch work on `hip_stream` (a hipStream_t; NULL = the context's stream).
 * The new stream is ordered after the last operation the context queued on the
 * previous one (an event the context records with every such operation), so
 * frame-ordered blends never overtake each other; the previous stream itself
 * is not touched again and may already be destroyed. */
int pnrt_set_stream(pnrt_ctx* ctx, void* hip_stream);
/* The context's own stream (created with it, before its worker streams): a caller
 * that wraps it (e.g. torch.cuda.ExternalStream) adds no stream of its own. */
void* pnrt_get_stream(pnrt_ctx* ctx);

/* Replaces the five TBO/texture uploads main.cpp:409-524 (texture units 0-4)
 * and the lightsSize/lightsSumArea uniforms (main.cpp:391-392):
 *   vertices  15 f each (main.cpp:412-428)     materials 18 f (main.cpp:438-456)
 *   triangles  6 f each (main.cpp:470-477)     bvh_nodes 12 f (main.cpp:488-501)
 *   lights     3 f each (main.cpp:513-517)     (lights may be NULL when n_lights = 0)
 * The arrays are validated and re-laid out for gfx950. */
int pnrt_upload_scene(pnrt_ctx* ctx,
                      const float* vertices, int n_vertices,
                      const float* materials, int n_materials,
                      const float* triangles, int n_triangles,
                      const float* bvh_nodes, int n_nodes,
                      const float* lights, int n_lights, float lights_sum_area);

/* Replaces the material panel's in-place edit of the material texture
 * (include/ImGuiLayer.hpp:73-83: glTexSubImage1D on unit 1 when a slider
 * moves, followed by main.cpp:592-596's redraw): overwrite materials
 * first .. first + count - 1 with count records of 18 floats in the
 * main.cpp:438-456 layout, without re-uploading or re-laying out the scene.
 * Calls already issued render with the old records (the call waits for them);
 * later calls see the new ones.  The caller resets the accumulation as the
 * reference's redraw does (pnrt_reset_accum). */
int pnrt_update_materials(pnrt_ctx* ctx, int first, int count, const float* materials18);

/* Replaces the albedo texture uploads (main.cpp:527-554, units 5..24):
 * tightly packed 8-bit rows as stbi_load returns them; GL's default
 * UNPACK_ALIGNMENT of 4 is applied as glTexImage2D would. slot 0..19. */
int pnrt_upload_texture(pnrt_ctx* ctx, int slot, const uint8_t* pixels, int width, int height,
                        int channels);

/* Replaces LoadHDRImage's two glTexImage2D calls (shader.hpp:136-214, units
 * 29/30) and the HDRImageWidth/Height/HasHDRImage uniforms.  hdr_rgb == NULL
 * clears the environment (HasHDRImage = 0). */
int pnrt_upload_env(pnrt_ctx* ctx, const float* hdr_rgb, const float* random_hdr_rgb, int width,
                    int height);

/* LoadHDRImage (shader.hpp:126-225) with its RandomHDR table built on the
 * GPU instead of on the host: the same table, bit for bit, as the
 * host restatement pnrt_hdr_build_table (every float sum in the reference's
 * order).  hdr_rgb: width*height*3 floats as stbi_loadf returns them. */
int pnrt_upload_env_build(pnrt_ctx* ctx, const float* hdr_rgb, int width, int height);
/* Copy the bound RandomHDR table (width*height*3 floats) to the host. */
int pnrt_read_env_table(pnrt_ctx* ctx, float* random_hdr_out);

/* Replaces the per-frame uniforms SCREEN_WIDTH/HEIGHT (main.cpp:389-390),
 * camera.* (main.cpp:606-610) and MAX_BOUNCE_DEPTH (main.cpp:593,599).
 * (Re)allocates a zeroed width*height RGBA32F accumulation image when the
 * size changes. */
int pnrt_set_frame(pnrt_ctx* ctx, int width, int height, const pnrt_camera* camera,
                   int max_bounce_depth);

int pnrt_set_options(pnrt_ctx* ctx, int options);

/* Replaces glDispatchCompute (main.cpp:613) called once per frame for frames
 * first_frame .. first_frame + n_frames - 1 (frameCount uniform), blended in
 * order into the accumulation image with the progressive mean of
 * ray_tracing.comp:988-991.  Shard selector (multi-GPU row bands): only rows
 * y with (y / band_rows) % n_shards == shard are rendered; full image =
 * (band_rows >= 1, n_shards = 1, shard = 0).  Asynchronous on the stream.
 * The frames run in batches of up to 128 frames and 2^28 paths (~310 B of
 * device memory per path; the environment variable PNRT_BATCH_BYTES, read at a
 * context's first render, caps one batch's bytes -- the batching changes no
 * pixel). */
int pnrt_render(pnrt_ctx* ctx, uint32_t first_frame, uint32_t n_frames, int band_rows,
                int n_shards, int shard);

/* Redraw semantics (main.cpp:592-596): zero the accumulation image.  Waits
 * for the calls in flight first, and clears a PNRT_E_TRACE fault. */
int pnrt_reset_accum(pnrt_ctx* ctx);
/* Synchronise and copy the width*height*4 floats (row 0 = bottom) to host. */
int pnrt_read_accum(pnrt_ctx* ctx, float* rgba_out);
/* Device pointer of the accumulation image (for collectives / zero-copy use). */
void* pnrt_accum_device_ptr(pnrt_ctx* ctx);
/* Copy this shard's rows, in increasing y, into a contiguous device buffer
 * (rows_of_shard * width * 4 floats), on the context stream. */
int pnrt_pack_rows(pnrt_ctx* ctx, void* dst_device, int band_rows, int n_shards, int shard);
/* The inverse, on the receiving rank of the gather: shard `shard`'s packed rows
 * (as pnrt_pack_rows wrote them on that rank) into their rows of a
 * width*height*4-float device image (row 0 = bottom), on the context stream --
 * the gathered frame assembled by the library's own kernel (the main.cpp
 * display reads one image, main.cpp:613-628). */
int pnrt_unpack_rows(pnrt_ctx* ctx, const void* src_device, void* image_device, int band_rows, int n_shards,
                     int shard);
int pnrt_synchronize(pnrt_ctx* ctx);
int pnrt_get_device_info(pnrt_ctx* ctx, pnrt_device_info* info);

/* Per-kernel timing (not in the reference, which has no GPU timers): while
 * enabled, every launch of a kernel class is bracketed by HIP events recorded on
 * the launch stream; pnrt_profile_read synchronises and returns the summed
 * event durations (ms) and launch counts.  Enabling (or disabling) resets. */
#define PNRT_K_PRIMARY 0   /* primary hits, one trace per pixel per render call */
#define PNRT_K_GEN 1       /* path state for the call's frames                  */
#define PNRT_K_SETUP 2     /* per bounce: sampling + speculative BSDF, shadow rays */
#define PNRT_K_TRACE 3     /* per bounce: persistent BVH traversal of all rays  */
#define PNRT_K_SHADE 4     /* per bounce: MIS + continuation                    */
#define PNRT_K_BLEND 5     /* progressive mean into the accumulation image      */
#define PNRT_K_V1 6        /* PNRT_KERNEL_V1 single-kernel path                 */
#define PNRT_K_COUNT 7
typedef struct {
    double ms[PNRT_K_COUNT];
    int64_t launches[PNRT_K_COUNT];
} pnrt_profile;
int pnrt_profile_enable(pnrt_ctx* ctx, int on);
int pnrt_profile_read(pnrt_ctx* ctx, pnrt_profile* out);
/* Kernel classes bracketed while profiling is enabled: bit k = PNRT_K_k (default
 * all).  Timing only the dominant class keeps the event records off the other
 * launches (each record is a queue packet between kernels). */
int pnrt_profile_select(pnrt_ctx* ctx, int class_mask);

/* GPU BuildBVH: the reference's binned-SAH build
 * (include/BVH.hpp:92-173, called from the BVH ctor :16-19 via main.cpp's
 * scene setup) run on the device, returning the SAME node array (pre-order,
 * main.cpp:488-501 layout, 12 floats per node) and the SAME triangle order as
 * the host build, bit for bit.  Input per triangle, in the current order: its
 * Bound and boundCenter (triangle.hpp:11-12) as 9 floats pMin.xyz pMax.xyz
 * centre.xyz.  Output: order_out[i] = input index of the triangle at BVH
 * position i; nodes_out needs room for 2 * n_triangles - 1 nodes.  Stateless
 * with respect to the scene (the caller packs and uploads as usual).  Bounds
 * must be finite; synchronous. */
int pnrt_bvh_build(pnrt_ctx* ctx, const float* tri_bounds9, int n_triangles, float* nodes_out,
                   int node_capacity, int* n_nodes_out, int32_t* order_out, int* max_depth_out);

/* Test hook: evaluate one PN-libm / IEEE primitive on the device (same fn
 * codes as the oracle's pno_math_eval); host in/out arrays of n floats. */
int pnrt_debug_math(pnrt_ctx* ctx, int fn, const float* a, const float* b, float* out, int n);

#ifdef __cplusplus
}
#endif
#endif
