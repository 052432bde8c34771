// oracle/ref/scene_in.hpp -- TEST INFRASTRUCTURE shared by the reference-header
// drivers (ref_driver.cpp, isect_driver.cpp): reads the scene description that
// tests/golden/make_golden.py writes and builds the reference's own Vertex /
// Triangle records from it (model.hpp:101-135 restated with glm calls, since
// Model's only constructor needs Assimp).  Built only in this container.
#pragma once
#include "model.hpp"
#include "BVH.hpp"
#include "camera.hpp"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

static void rd(void* p, size_t n) {
    if (fread(p, 1, n, stdin) != n) { fprintf(stderr, "short read\n"); exit(2); }
}
template <class T> static T rd1() { T v; rd(&v, sizeof v); return v; }
static void wr(const void* p, size_t n) { fwrite(p, 1, n, stdout); }
template <class T> static void wr1(T v) { wr(&v, sizeof v); }

struct SceneIn {
    std::vector<float> matbuf;
    std::vector<Vertex> verts;
    std::vector<Triangle> tris;
    std::vector<float> matrices;
    float cam_in[11];
    int32_t nmesh = 0;
};

static int read_scene(SceneIn& S) {
    std::vector<float>& matbuf = S.matbuf;
    std::vector<Vertex>& verts = S.verts;
    std::vector<Triangle>& tris = S.tris;
    std::vector<float>& matrices = S.matrices;
    float* cam_in = S.cam_in;
    char magic[4];
    rd(magic, 4);
    if (memcmp(magic, "PNRF", 4) != 0) { fprintf(stderr, "bad magic\n"); return -1; }

    // materials (18 floats each, main.cpp:438-456 order)
    int32_t nm = rd1<int32_t>();
    matbuf.resize((size_t)nm * 18);
    rd(matbuf.data(), matbuf.size() * 4);

    const int32_t nmesh = S.nmesh = rd1<int32_t>();
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
    rd(cam_in, sizeof S.cam_in);

    return 0;
}
