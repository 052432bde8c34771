// oracle/ref/isect_driver.cpp -- TEST INFRASTRUCTURE (golden-vector generator).
//
// Runs the reference's OWN CPU intersection code, compiled here from
// /root/reference/include by oracle/ref/Makefile, on caller rays:
//   kind 0  BVH::Intersect        (BVH.hpp:21-54)   closest hit
//   kind 1  BVH::IntersectP       (BVH.hpp:57-85)   any hit
//   kind 2  TriangleIntersect     (triangle.hpp:15-118) one triangle per ray
//   kind 3  TriangleIntersectP    (triangle.hpp:121-181)
//   kind 4  BoundIntersect        (bound.hpp:31-47)  one node box per ray
// over the BVH the reference's BuildBVH (BVH.hpp:92-173) makes of the scene.
// Its outputs pin the oracle's ray/triangle, slab and traversal arithmetic
// (oracle/pn_oracle.c pno_intersect with the CPU headers' rules).
//
// stdin: scene (scene_in.hpp format), then "RAYS", int32 kind, int32 n,
// n x 7 floats (origin, dir, tMax), and for kind >= 2 n int32 indices.
// stdout: n x 13 u32 words (hit, position, normal, texcoord, textureId,
// materialId, time -- zeros when no hit -- then the ray's tMax after the
// call); kind 4: hit, t0, t1.
#include "scene_in.hpp"

static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main() {
    SceneIn S;
    if (read_scene(S) != 0) return 2;
    BVH bvh(S.verts, S.tris);
    char magic[4];
    rd(magic, 4);
    if (memcmp(magic, "RAYS", 4) != 0) { fprintf(stderr, "bad ray magic\n"); return 2; }
    const int32_t kind = rd1<int32_t>(), n = rd1<int32_t>();
    std::vector<float> q((size_t)n * 7);
    rd(q.data(), q.size() * 4);
    std::vector<int32_t> idx;
    if (kind >= 2) { idx.resize(n); rd(idx.data(), (size_t)n * 4); }
    std::vector<uint32_t> out((size_t)n * 13, 0u);
    for (int i = 0; i < n; ++i) {
        const float* r7 = &q[(size_t)i * 7];
        Ray ray;
        ray.origin = glm::vec3(r7[0], r7[1], r7[2]);
        ray.dir = glm::vec3(r7[3], r7[4], r7[5]);
        ray.tMax = r7[6];
        Interaction is;
        bool hit = false, full = false;
        uint32_t* o = &out[(size_t)i * 13];
        switch (kind) {
        case 0: hit = bvh.Intersect(ray, &is); full = true; break;
        case 1: hit = bvh.IntersectP(ray); break;
        case 2: hit = TriangleIntersect(bvh.triangles[idx[i]], ray, bvh.vertices, &is); full = true; break;
        case 3: hit = TriangleIntersectP(bvh.triangles[idx[i]], ray, bvh.vertices); break;
        case 4: {
            float t0 = 0.f, t1 = 0.f;
            hit = BoundIntersect(bvh.bvh[idx[i]].bound, ray, &t0, &t1);
            o[0] = hit;
            if (hit) { o[1] = fb(t0); o[2] = fb(t1); }
            continue;
        }
        default: fprintf(stderr, "bad kind\n"); return 2;
        }
        o[0] = hit;
        if (hit && full) {
            o[1] = fb(is.position.x); o[2] = fb(is.position.y); o[3] = fb(is.position.z);
            o[4] = fb(is.normal.x); o[5] = fb(is.normal.y); o[6] = fb(is.normal.z);
            o[7] = fb(is.texcoord.x); o[8] = fb(is.texcoord.y);
            o[9] = (uint32_t)is.textureId; o[10] = (uint32_t)is.materialId; o[11] = fb(is.time);
        }
        o[12] = fb(ray.tMax);
    }
    wr(out.data(), out.size() * 4);
    return 0;
}
