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
#include "model.hpp"
#include "BVH.hpp"
#include "camera.hpp"

#include <cstdint>
#include <cstdio>
#include <vector>

static void rd(void* p, size_t n) {
    if (fread(p, 1, n, stdin) != n) { fprintf(stderr, "short read\n"); exit(2); }
}
template <class T> static T rd1() { T v; rd(&v, sizeof v); return v; }
static void wr(const void* p, size_t n) { fwrite(p, 1, n, stdout); }
template <class T> static void wr1(T v) { wr(&v, sizeof v); }

int main() {
    char magic[4];
    rd(magic, 4);
    if (memcmp(magic, "PNRF", 4) != 0) { fprintf(stderr, "bad magic\n"); return 2; }

    // materials (18 floats each, main.cpp:438-456 order)
    int32_t nm = rd1<int32_t>();
    std::vector<float> matbuf((size_t)nm * 18);
    rd(matbuf.data(), matbuf.size() * 4);

    std::vector<Vertex> verts;
    std::vector<Triangle> tris;
    int32_t nmesh = rd1<int32_t>();
    std::vector<float> matrices;
    for (int k = 0; k < nmesh; ++k) {
        int32_t matId = rd1<int32_t>(), texId = rd1<int32_t>(), nops = rd1<int32_t>();
        glm::mat4 M(1.f);
        for (int o = 0; o < nops; ++o) {
            int32_t kind = rd1<int32_t>();
            float ang = rd1<float>();
            float v[3]; rd(v, 12);
            glm::mat4 f;
            if (kind == 0) f = glm::translate(glm::mat4(1), glm::vec3(v[0], v[1], v[2]));
            else if (kind == 1) f = glm::rotate(glm::mat4(1), glm::radians(ang), glm::vec3(v[0], v[1], v[2]));
            else f = glm::scale(glm::mat4(1), glm::vec3(v[0], v[1], v[2]));
            M = (o == 0) ? f : M * f;
        }
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) matrices.push_back(M[i][j]);
        int32_t nv = rd1<int32_t>();
        std::vector<float> P((size_t)nv * 3), N((size_t)nv * 3), UV((size_t)nv * 2);
        rd(P.data(), P.size() * 4); rd(N.data(), N.size() * 4); rd(UV.data(), UV.size() * 4);
        int32_t ni = rd1<int32_t>();
        std::vector<int32_t> I(ni);
        rd(I.data(), (size_t)ni * 4);

        // model.hpp:104-122 (vertex transform), :123-133 (triangle records)
        glm::mat4 normalMatrix = glm::transpose(glm::inverse(M));
        int base = (int)verts.size();
        for (int i = 0; i < nv; ++i) {
            glm::vec3 p(P[3 * i], P[3 * i + 1], P[3 * i + 2]);
            glm::vec3 n(N[3 * i], N[3 * i + 1], N[3 * i + 2]);
            glm::vec3 zero(0.f);
            Vertex w;
            w.position = glm::vec3(M * glm::vec4(p, 1.0));
            w.normal = glm::vec3(normalMatrix * glm::vec4(n, 1.0));
            w.tangent = glm::vec3(M * glm::vec4(zero, 1.0));
            w.bitangent = glm::vec3(M * glm::vec4(zero, 1.0));
            w.texcoord = glm::vec2(UV[2 * i], UV[2 * i + 1]);
            verts.push_back(w);
        }
        for (int i = 0; i < ni; i += 3) {
            Triangle t;
            for (int c = 0; c < 3; ++c) t.indices[c] = I[i + c] + base;
            t.materialId = matId;
            t.textureId = texId;
            const glm::vec3& p0 = verts[t.indices[0]].position;
            const glm::vec3& p1 = verts[t.indices[1]].position;
            const glm::vec3& p2 = verts[t.indices[2]].position;
            t.area = glm::length(glm::cross(p1 - p0, p2 - p0)) * 0.5;
            for (int c = 0; c < 3; ++c) t.bound.Union(verts[t.indices[c]].position);
            t.boundCenter = (t.bound.pMax + t.bound.pMin) * .5f;
            tris.push_back(t);
        }
    }
    float cam_in[11];
    rd(cam_in, sizeof cam_in);

    BVH bvh(verts, tris);

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
