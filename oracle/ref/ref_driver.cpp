// oracle/ref/ref_driver.cpp -- TEST INFRASTRUCTURE (golden-vector generator).
//
// Compiled ONLY in this container, against the reference's own headers where
// they lie (/root/reference/include: BVH.hpp, bound.hpp, triangle.hpp,
// camera.hpp, PnRT.hpp, vendored glm 0.9.9.8), by oracle/ref/Makefile into
// oracle/_ref/ref_driver.  Never built or run on the GPU box; its outputs are
// committed as fixtures under tests/golden/.
//
// It drives the reference's real code:
//   - glm::translate/rotate/scale, glm::inverse/transpose  (main.cpp:207-237, model.hpp:104)
//   - Bound::Union, Triangle records                       (bound.hpp, triangle.hpp)
//   - BVH::BVH -> BuildBVH (binned SAH, std::partition)     (BVH.hpp:16-19, 92-173)
//   - Camera::UpdateCamera                                  (camera.hpp:11-31)
// The per-vertex world transform and triangle record set-up mirror
// ModelOutput (model.hpp:101-135) with glm calls, because Model's only
// constructor needs Assimp (Windows .lib only).  The light list and packing
// mirror main.cpp:374-383 and main.cpp:409-524.
//
// stdin: a scene description written by tests/golden/make_golden.py;
// stdout: packed arrays.  One BVH per process (BuildBVH's static nodeId).
#include "scene_in.hpp"

int main() {
    SceneIn S;
    if (read_scene(S) != 0) return 2;
    std::vector<float>& matbuf = S.matbuf;
    std::vector<float>& matrices = S.matrices;
    const float* cam_in = S.cam_in;
    const int32_t nmesh = S.nmesh;

    BVH bvh(S.verts, S.tris);

    // main.cpp:374-383
    std::vector<Light> ls;
    for (int i = 0; i < (int)bvh.triangles.size(); ++i) {
        const Triangle& t = bvh.triangles[i];
        const float* e = &matbuf[(size_t)t.materialId * 18];
        if (glm::vec3(e[0], e[1], e[2]) != glm::vec3(0)) {
            ls.push_back({i, t.area});
            if (ls.size() > 1) ls[ls.size() - 1].prefixArea += ls[ls.size() - 2].prefixArea;
        }
    }

    Camera cam;
    cam.UpdateCamera(glm::vec3(cam_in[0], cam_in[1], cam_in[2]), glm::vec3(cam_in[3], cam_in[4], cam_in[5]),
                     glm::vec3(cam_in[6], cam_in[7], cam_in[8]), cam_in[9], cam_in[10]);

    // main.cpp:409-524 packing
    wr1<int32_t>((int32_t)bvh.vertices.size());
    for (const Vertex& v : bvh.vertices) {
        float f[15] = {v.position[0], v.position[1], v.position[2], v.normal[0], v.normal[1], v.normal[2],
                       v.tangent[0], v.tangent[1], v.tangent[2], v.bitangent[0], v.bitangent[1], v.bitangent[2],
                       v.texcoord[0], v.texcoord[1], 0.f};
        wr(f, sizeof f);
    }
    wr1<int32_t>((int32_t)bvh.triangles.size());
    for (const Triangle& t : bvh.triangles) {
        float f[6] = {(float)t.indices[0], (float)t.indices[1], (float)t.indices[2],
                      (float)t.materialId, (float)t.textureId, t.area};
        wr(f, sizeof f);
    }
    wr1<int32_t>((int32_t)bvh.bvh.size());
    for (const BVHNode& n : bvh.bvh) {
        float f[12] = {n.bound.pMin[0], n.bound.pMin[1], n.bound.pMin[2], n.bound.pMax[0], n.bound.pMax[1],
                       n.bound.pMax[2], (float)n.axis, (float)n.rightChild, (float)n.startIndex,
                       (float)n.endIndex, 0.f, 0.f};
        wr(f, sizeof f);
    }
    wr1<int32_t>((int32_t)ls.size());
    for (const Light& l : ls) { float f[3] = {(float)l.index, l.prefixArea, 0.f}; wr(f, sizeof f); }
    float camo[12] = {cam.eye.x, cam.eye.y, cam.eye.z, cam.lowerLeftCorner.x, cam.lowerLeftCorner.y,
                      cam.lowerLeftCorner.z, cam.horizontal.x, cam.horizontal.y, cam.horizontal.z,
                      cam.vertical.x, cam.vertical.y, cam.vertical.z};
    wr(camo, sizeof camo);
    wr1<int32_t>(nmesh);
    wr(matrices.data(), matrices.size() * 4);
    return 0;
}
