/*
 * include/pnrt_host.h -- C ABI of libpnrt_host.so, the host-side scene
 * library.  It rebuilds, bit for bit, the flattened arrays PnRayTracing's
 * main.cpp uploads to its compute shader (main.cpp:409-524), so the device
 * library (include/pnrt.h) receives exactly what the reference would:
 *
 *   reference interface replaced             here
 *   ----------------------------------------  ------------------------------
 *   Model ctor + ModelOutput (model.hpp:22-135) pnrt_scene_add_material/_mesh
 *   BVH::BuildBVH (BVH.hpp:92-173)             pnrt_scene_build (or libpnrt.so
 *                                              pnrt_bvh_build + pnrt_scene_set_bvh)
 *   light prefix list (main.cpp:374-383)       pnrt_scene_build
 *   packing loops (main.cpp:409-524)           pnrt_scene_pack
 *   Camera::UpdateCamera (camera.hpp:11-31)    pnrt_camera_update, pnrt_camera_state_init
 *   Camera::UpdateRotate/TranslateUV/Fov       pnrt_camera_rotate/_translate/_zoom
 *     (camera.hpp:33-65, main.cpp:118-142)
 *   glm::translate/rotate/scale (main.cpp:207-237)  pnrt_model_matrix
 *   stbi_loadf RGBE (stb_image.h:6839-6990)    pnrt_hdr_decode_rgbe
 *   LoadHDRImage CDF table (shader.hpp:145-203) pnrt_hdr_build_table
 *
 * Assimp OBJ import is not reproduced (no asset files, no Linux library):
 * meshes arrive as model-space arrays (pnrt_scene_add_mesh) or from the
 * deterministic procedural generators below (bunny/teapot/marry stand-ins).
 *
 * All functions return 0 on success and a negative code on error; the
 * message is available from pnrt_host_last_error().
 */
#ifndef PNRT_HOST_H
#define PNRT_HOST_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PNRT_VERTEX_SIZE 15   /* PnRT.hpp:45 */
#define PNRT_MATERIAL_SIZE 18 /* PnRT.hpp:46 */
#define PNRT_TRIANGLE_SIZE 6  /* PnRT.hpp:47 */
#define PNRT_BVHNODE_SIZE 12  /* PnRT.hpp:48 */
#define PNRT_LIGHT_SIZE 3     /* PnRT.hpp:49 */

typedef struct pnrt_scene pnrt_scene;

/* one factor of a glm model matrix: kind 0 = translate(v), 1 = rotate(angle_deg
 * about axis v), 2 = scale(v); factors multiply left to right from identity,
 * exactly as glm::translate(mat4(1),..) * glm::rotate(mat4(1),..) * ... */
typedef struct { int kind; float angle_deg; float v[3]; } pnrt_xform;

const char* pnrt_host_last_error(void);

int pnrt_model_matrix(const pnrt_xform* ops, int n_ops, float out_col_major[16]);

pnrt_scene* pnrt_scene_create(void);
void pnrt_scene_destroy(pnrt_scene* s);
/* Material record in main.cpp:438-456 order (18 floats).  Returns its id. */
int pnrt_scene_add_material(pnrt_scene* s, const float material18[18]);
/* One Assimp mesh of one Model (model.hpp:131-178 output): model-space
 * vertices (positions/normals/tangents/bitangents 3 f each, texcoords 2 f;
 * NULL -> zeros), triangle index list, the model's matrix and ids.  Appended
 * with ModelOutput semantics (model.hpp:101-135). */
int pnrt_scene_add_mesh(pnrt_scene* s, int material_id, int texture_id,
                        const float model_matrix[16],
                        const float* positions, const float* normals,
                        const float* tangents, const float* bitangents,
                        const float* texcoords, int n_vertices,
                        const int32_t* indices, int n_indices);
/* BuildBVH over all triangles + emissive light list. */
int pnrt_scene_build(pnrt_scene* s);
/* GPU BuildBVH support (libpnrt.so pnrt_bvh_build): the builder's input,
 * Bound + boundCenter of every triangle in the current order (9 floats:
 * pMin.xyz pMax.xyz centre.xyz), and installing its output (triangle order,
 * main.cpp-layout nodes) in place of pnrt_scene_build's; the light list is
 * rebuilt in the new order as pnrt_scene_build does. */
int pnrt_scene_tri_bounds(const pnrt_scene* s, float* out9);
int pnrt_scene_set_bvh(pnrt_scene* s, const int32_t* order, const float* bvh_nodes12, int n_nodes,
                       int max_depth);
/* The host BuildBVH over bare bounds, with pnrt_bvh_build's signature (no
 * context): the CPU counterpart the GPU build is checked against. */
int pnrt_bvh_build_cpu(const float* tri_bounds9, int n_triangles, float* nodes_out, int node_capacity,
                       int* n_nodes_out, int32_t* order_out, int* max_depth_out);
typedef struct {
    int n_vertices, n_materials, n_triangles, n_nodes, n_lights;
    float lights_sum_area;
    int max_depth;           /* deepest node (root = 0) */
} pnrt_scene_info;
int pnrt_scene_get_info(const pnrt_scene* s, pnrt_scene_info* info);
/* Write the main.cpp-layout arrays (any pointer may be NULL). */
int pnrt_scene_pack(const pnrt_scene* s, float* vertices, float* materials,
                    float* triangles, float* bvh_nodes, float* lights);

/* camera.hpp:11-31 -> eye, lowerLeftCorner, horizontal, vertical */
int pnrt_camera_update(const float eye[3], const float center[3], const float up[3],
                       float fov_deg, float aspect, float out12[12]);

/* Camera state (camera.hpp:4-77) and the interactive controls that
 * main.cpp's mouse callbacks call (main.cpp:118-142): left drag ->
 * UpdateRotate(dx, dy), right drag -> UpdateTranslateUV(-dx, dy), scroll ->
 * UpdateFov(yoffset).  eye/lower_left/horizontal/vertical feed pnrt_set_frame.
 * rotate/zoom return 1 if applied, 0 if the reference rejects the move
 * (rotation within 0.9995 of the up axis; fov outside (1, 89)). */
typedef struct {
    float eye[3], center[3], up[3];
    float fov_deg, aspect;
    float u[3], v[3], w[3];
    float distance;
    float lower_left[3], horizontal[3], vertical[3];
} pnrt_camera_state;
int pnrt_camera_state_init(pnrt_camera_state* c, const float eye[3], const float center[3], const float up[3],
                           float fov_deg, float aspect);
int pnrt_camera_rotate(pnrt_camera_state* c, float phi, float theta);
int pnrt_camera_translate(pnrt_camera_state* c, float dx, float dy);
int pnrt_camera_zoom(pnrt_camera_state* c, float delta);

/* Radiance RGBE decode with stbi_loadf semantics (3 channels, row 0 = first
 * scanline).  out_rgb may be NULL to query w/h; caller allocates w*h*3. */
int pnrt_hdr_decode_rgbe(const uint8_t* bytes, int64_t n_bytes, int* w, int* h, float* out_rgb);
/* LoadHDRImage's luminance CDF + inverse lookup table (RandomHDR). */
int pnrt_hdr_build_table(const float* rgb, int w, int h, float* out_random_hdr);

/* ---- deterministic procedural stand-ins (model space, unshared vertices) --
 * Output arrays sized by the *_count functions: positions/normals 3*nv,
 * texcoords 2*nv, indices 3*nt.  Pass NULL outputs to get counts only. */
/* floor.obj stand-in: quad in XZ at y=0, |x|,|z| <= half, normal +Y. */
int pnrt_mesh_quad(float half, float* positions, float* normals, float* texcoords,
                   int32_t* indices, int* nv, int* nt);
/* displaced UV sphere: nu x nv quads (2 tris each), radius r at center c,
 * radial value-noise displacement of relative amplitude amp, seed. */
int pnrt_mesh_displaced_sphere(int nu, int nvv, float radius, const float center[3],
                               float amp, uint32_t seed,
                               float* positions, float* normals, float* texcoords,
                               int32_t* indices, int* nv, int* nt);
/* teapot-class lathe body + spout + handle (~6.1k tris). */
int pnrt_mesh_teapot(float* positions, float* normals, float* texcoords,
                     int32_t* indices, int* nv, int* nt);
/* synthetic HDR environment (sky gradient + sun lobe + seeded noise). */
int pnrt_hdr_synthetic(int w, int h, uint32_t seed, float* out_rgb);

#ifdef __cplusplus
}
#endif
#endif
