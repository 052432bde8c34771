// pnraytracing_amd/csrc/host/pnrt_host.cpp -- libpnrt_host.so
//
// Host-side scene library: rebuilds PnRayTracing's flattened upload arrays
// bit for bit (checked against the reference's own headers compiled by
// oracle/ref, see tests/test_host_arrays.py).  Float semantics follow the
// reference's C++ exactly: glm 0.9.9.8 operation order, float temporaries
// where the reference has float, double where it promotes to double.
// Build with g++ -O2 -ffp-contract=off (no FMA contraction, SSE2 float math).
#include "pnrt_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }

// ---- glm-equivalent float vector / matrix -----------------------------------
struct vec3 {
    float x = 0.f, y = 0.f, z = 0.f;
    vec3() = default;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(vec3 a, vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline vec3 operator*(vec3 v, float s) { return {v.x * s, v.y * s, v.z * s}; }
inline vec3 operator*(float s, vec3 v) { return {s * v.x, s * v.y, s * v.z}; }
inline bool operator==(vec3 a, vec3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
// glm compute_dot<vec3>: tmp = a*b; (tmp.x + tmp.y) + tmp.z
inline float dot(vec3 a, vec3 b) { vec3 t = a * b; return t.x + t.y + t.z; }
// glm compute_cross (func_geometric.inl)
inline vec3 cross(vec3 x, vec3 y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline float length(vec3 v) { return std::sqrt(dot(v, v)); }
// glm normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1 / sqrt
inline vec3 normalize(vec3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
// glm::min/max on genType: (y < x) ? y : x / (x < y) ? y : x
inline float gmin(float x, float y) { return (y < x) ? y : x; }
inline float gmax(float x, float y) { return (x < y) ? y : x; }
inline vec3 vmin(vec3 a, vec3 b) { return {gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)}; }
inline vec3 vmax(vec3 a, vec3 b) { return {gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)}; }

struct vec4 {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    float& operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
};
inline vec4 V4(float a, float b, float c, float d) { vec4 r; r.v[0] = a; r.v[1] = b; r.v[2] = c; r.v[3] = d; return r; }
inline vec4 operator+(const vec4& a, const vec4& b) { return V4(a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]); }
inline vec4 operator-(const vec4& a, const vec4& b) { return V4(a[0] - b[0], a[1] - b[1], a[2] - b[2], a[3] - b[3]); }
inline vec4 operator*(const vec4& a, const vec4& b) { return V4(a[0] * b[0], a[1] * b[1], a[2] * b[2], a[3] * b[3]); }
inline vec4 operator*(const vec4& a, float s) { return V4(a[0] * s, a[1] * s, a[2] * s, a[3] * s); }

struct mat4 {  // column major, c[col][row]
    vec4 c[4];
    static mat4 identity() { mat4 m; for (int i = 0; i < 4; ++i) m.c[i][i] = 1.f; return m; }
};
// glm type_mat4x4.inl operator*(mat4, mat4): Result[i] = A0*B[i][0] + A1*B[i][1] + A2*B[i][2] + A3*B[i][3]
inline mat4 operator*(const mat4& a, const mat4& b) {
    mat4 r;
    for (int i = 0; i < 4; ++i)
        r.c[i] = ((a.c[0] * b.c[i][0] + a.c[1] * b.c[i][1]) + a.c[2] * b.c[i][2]) + a.c[3] * b.c[i][3];
    return r;
}
// glm operator*(mat4, vec4): (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
inline vec4 operator*(const mat4& m, const vec4& v) {
    vec4 add0 = m.c[0] * v[0] + m.c[1] * v[1];
    vec4 add1 = m.c[2] * v[2] + m.c[3] * v[3];
    return add0 + add1;
}
inline mat4 transpose(const mat4& m) {
    mat4 r;
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) r.c[i][j] = m.c[j][i];
    return r;
}
// glm compute_inverse<4,4> (func_matrix.inl), same expression order
mat4 inverse(const mat4& M) {
    auto m = [&](int i, int j) { return M.c[i][j]; };
    float Coef00 = m(2,2) * m(3,3) - m(3,2) * m(2,3);
    float Coef02 = m(1,2) * m(3,3) - m(3,2) * m(1,3);
    float Coef03 = m(1,2) * m(2,3) - m(2,2) * m(1,3);
    float Coef04 = m(2,1) * m(3,3) - m(3,1) * m(2,3);
    float Coef06 = m(1,1) * m(3,3) - m(3,1) * m(1,3);
    float Coef07 = m(1,1) * m(2,3) - m(2,1) * m(1,3);
    float Coef08 = m(2,1) * m(3,2) - m(3,1) * m(2,2);
    float Coef10 = m(1,1) * m(3,2) - m(3,1) * m(1,2);
    float Coef11 = m(1,1) * m(2,2) - m(2,1) * m(1,2);
    float Coef12 = m(2,0) * m(3,3) - m(3,0) * m(2,3);
    float Coef14 = m(1,0) * m(3,3) - m(3,0) * m(1,3);
    float Coef15 = m(1,0) * m(2,3) - m(2,0) * m(1,3);
    float Coef16 = m(2,0) * m(3,2) - m(3,0) * m(2,2);
    float Coef18 = m(1,0) * m(3,2) - m(3,0) * m(1,2);
    float Coef19 = m(1,0) * m(2,2) - m(2,0) * m(1,2);
    float Coef20 = m(2,0) * m(3,1) - m(3,0) * m(2,1);
    float Coef22 = m(1,0) * m(3,1) - m(3,0) * m(1,1);
    float Coef23 = m(1,0) * m(2,1) - m(2,0) * m(1,1);
    vec4 Fac0 = V4(Coef00, Coef00, Coef02, Coef03);
    vec4 Fac1 = V4(Coef04, Coef04, Coef06, Coef07);
    vec4 Fac2 = V4(Coef08, Coef08, Coef10, Coef11);
    vec4 Fac3 = V4(Coef12, Coef12, Coef14, Coef15);
    vec4 Fac4 = V4(Coef16, Coef16, Coef18, Coef19);
    vec4 Fac5 = V4(Coef20, Coef20, Coef22, Coef23);
    vec4 Vec0 = V4(m(1,0), m(0,0), m(0,0), m(0,0));
    vec4 Vec1 = V4(m(1,1), m(0,1), m(0,1), m(0,1));
    vec4 Vec2 = V4(m(1,2), m(0,2), m(0,2), m(0,2));
    vec4 Vec3 = V4(m(1,3), m(0,3), m(0,3), m(0,3));
    vec4 Inv0 = (Vec1 * Fac0 - Vec2 * Fac1) + Vec3 * Fac2;
    vec4 Inv1 = (Vec0 * Fac0 - Vec2 * Fac3) + Vec3 * Fac4;
    vec4 Inv2 = (Vec0 * Fac1 - Vec1 * Fac3) + Vec3 * Fac5;
    vec4 Inv3 = (Vec0 * Fac2 - Vec1 * Fac4) + Vec2 * Fac5;
    vec4 SignA = V4(+1.f, -1.f, +1.f, -1.f);
    vec4 SignB = V4(-1.f, +1.f, -1.f, +1.f);
    mat4 Inv;
    Inv.c[0] = Inv0 * SignA; Inv.c[1] = Inv1 * SignB; Inv.c[2] = Inv2 * SignA; Inv.c[3] = Inv3 * SignB;
    vec4 Row0 = V4(Inv.c[0][0], Inv.c[1][0], Inv.c[2][0], Inv.c[3][0]);
    vec4 Dot0 = M.c[0] * Row0;
    float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
    float One = 1.0f / Dot1;
    mat4 r;
    for (int i = 0; i < 4; ++i) r.c[i] = Inv.c[i] * One;
    return r;
}
// glm::translate(m, v): Result[3] = m0*v0 + m1*v1 + m2*v2 + m3
mat4 translate(const mat4& m, vec3 v) {
    mat4 r = m;
    r.c[3] = ((m.c[0] * v[0] + m.c[1] * v[1]) + m.c[2] * v[2]) + m.c[3];
    return r;
}
// glm::rotate(m, angle, axis) (ext/matrix_transform.inl)
mat4 rotate(const mat4& m, float angle, vec3 v) {
    const float a = angle;
    const float c = std::cos(a);
    const float s = std::sin(a);
    vec3 axis = normalize(v);
    vec3 temp = (1.0f - c) * axis;
    float R[3][3];
    R[0][0] = c + temp[0] * axis[0];
    R[0][1] = temp[0] * axis[1] + s * axis[2];
    R[0][2] = temp[0] * axis[2] - s * axis[1];
    R[1][0] = temp[1] * axis[0] - s * axis[2];
    R[1][1] = c + temp[1] * axis[1];
    R[1][2] = temp[1] * axis[2] + s * axis[0];
    R[2][0] = temp[2] * axis[0] + s * axis[1];
    R[2][1] = temp[2] * axis[1] - s * axis[0];
    R[2][2] = c + temp[2] * axis[2];
    mat4 r;
    for (int i = 0; i < 3; ++i)
        r.c[i] = (m.c[0] * R[i][0] + m.c[1] * R[i][1]) + m.c[2] * R[i][2];
    r.c[3] = m.c[3];
    return r;
}
mat4 scale(const mat4& m, vec3 v) {
    mat4 r;
    r.c[0] = m.c[0] * v[0]; r.c[1] = m.c[1] * v[1]; r.c[2] = m.c[2] * v[2]; r.c[3] = m.c[3];
    return r;
}
// glm::radians: degrees * genType(0.01745329251994329576923690768489)
inline float radians(float d) { return d * static_cast<float>(0.01745329251994329576923690768489); }

const float FLT_MAXV = std::numeric_limits<float>::max();
const float FLT_LOWEST = std::numeric_limits<float>::lowest();

// ---- Bound (bound.hpp:4-28) ----------------------------------------------------
struct Bound {
    vec3 pMin{FLT_MAXV, FLT_MAXV, FLT_MAXV}, pMax{FLT_LOWEST, FLT_LOWEST, FLT_LOWEST};
    void Union(const Bound& b) { pMin = vmin(pMin, b.pMin); pMax = vmax(pMax, b.pMax); }
    void Union(vec3 p) { pMin = vmin(pMin, p); pMax = vmax(pMax, p); }
    vec3 Diagonal() const { return pMax - pMin; }
    float SurfaceArea() const {
        vec3 d = Diagonal();
        return (d.x * d.y + d.x * d.z + d.y * d.z) * 2.f;
    }
};

// ---- records (PnRT.hpp:52-81, triangle.hpp:5-13, BVH.hpp:6-12) ---------------------
struct Vertex { vec3 position, normal, tangent, bitangent; float uv[2] = {0.f, 0.f}; };
struct Tri {
    int indices[3] = {-1, -1, -1};
    int materialId = 0, textureId = -1;
    float area = 0.f;
    Bound bound;
    vec3 boundCenter{0.f, 0.f, 0.f};
};
struct Node { Bound bound; int axis, rightChild, startIndex, endIndex; };

// ---- BuildBVH (BVH.hpp:92-173), restated; node ids are pre-order ---------------
class BvhBuilder {
public:
    BvhBuilder(std::vector<Tri>& tris) : t_(tris) {}
    std::vector<Node> nodes;
    int maxDepth = 0;
    void build() { nextId_ = -1; if (!t_.empty()) build(0, (int)t_.size(), 0); }

private:
    static constexpr int BUCKETSIZE = 12;
    static constexpr int maxTrianglesInLeaf = 255;   // BVH.hpp:175
    static constexpr float trav = 1.f;               // BVH.hpp:176
    std::vector<Tri>& t_;
    int nextId_ = -1;   // the reference's function-static nodeId, per build

    int build(int L, int R, int depth) {
        int id = ++nextId_;
        if (depth > maxDepth) maxDepth = depth;
        Bound bound;
        for (int i = L; i < R; ++i) bound.Union(t_[i].bound);
        int n = R - L;
        if (n <= 2) { nodes.push_back({bound, -1, -1, L, R}); return id; }
        Bound cb;
        for (int i = L; i < R; ++i) cb.Union(t_[i].boundCenter);
        vec3 diag = cb.Diagonal();
        int d;
        if (diag.x >= diag.y && diag.x >= diag.z) d = 0;
        else if (diag.y >= diag.x && diag.y >= diag.z) d = 1;
        else d = 2;
        if (cb.pMax[d] == cb.pMin[d]) { nodes.push_back({bound, -1, -1, L, R}); return id; }
        struct Bucket { int n = 0; Bound b; } buc[BUCKETSIZE];
        const float lo = cb.pMin[d], ext = diag[d];
        auto bucketOf = [&](const Tri& t) {
            int pos = (int)(((t.boundCenter[d] - lo) / ext) * BUCKETSIZE);
            if (pos == BUCKETSIZE) pos = BUCKETSIZE - 1;
            return pos;
        };
        for (int i = L; i < R; ++i) {
            int pos = bucketOf(t_[i]);
            buc[pos].n++;
            buc[pos].b.Union(t_[i].bound);
        }
        float minCost = FLT_MAXV;
        int midBuc = 0;
        for (int m = 0; m < BUCKETSIZE - 1; ++m) {
            Bound b0, b1;
            int c0 = 0, c1 = 0;
            for (int i = 0; i <= m; ++i) { c0 += buc[i].n; b0.Union(buc[i].b); }
            for (int i = m + 1; i < BUCKETSIZE; ++i) { c1 += buc[i].n; b1.Union(buc[i].b); }
            float cost = trav + (b0.SurfaceArea() * c0 + b1.SurfaceArea() * c1) / bound.SurfaceArea();
            if (cost < minCost) { minCost = cost; midBuc = m; }
        }
        int mid = (int)(std::partition(t_.begin() + L, t_.begin() + R,
                                       [&](const Tri& t) { return bucketOf(t) <= midBuc; }) - t_.begin());
        float leafCost = (float)n;
        if ((n <= maxTrianglesInLeaf && leafCost <= minCost) || mid == L) {
            nodes.push_back({bound, -1, -1, L, R});
            return id;
        }
        nodes.push_back({bound, d, 0, L, R});
        build(L, mid, depth + 1);
        int rc = build(mid, R, depth + 1);
        nodes[id].rightChild = rc;
        return id;
    }
};

}  // namespace

// ---- scene ---------------------------------------------------------------------
struct pnrt_scene {
    std::vector<Vertex> vertices;
    std::vector<Tri> triangles;
    std::vector<std::vector<float>> materials;  // 18 floats each
    std::vector<Node> nodes;
    std::vector<std::pair<int, float>> lights;
    int maxDepth = 0;
    bool built = false;
};

extern "C" {

const char* pnrt_host_last_error(void) { return g_err.c_str(); }

int pnrt_model_matrix(const pnrt_xform* ops, int n_ops, float out[16]) {
    if (!ops || n_ops <= 0 || !out) return fail(-1, "pnrt_model_matrix: no factors");
    mat4 M;
    for (int k = 0; k < n_ops; ++k) {
        vec3 v(ops[k].v[0], ops[k].v[1], ops[k].v[2]);
        mat4 f;
        switch (ops[k].kind) {
        case 0: f = translate(mat4::identity(), v); break;
        case 1: f = rotate(mat4::identity(), radians(ops[k].angle_deg), v); break;
        case 2: f = scale(mat4::identity(), v); break;
        default: return fail(-2, "pnrt_model_matrix: bad factor kind");
        }
        M = (k == 0) ? f : M * f;
    }
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) out[4 * i + j] = M.c[i][j];
    return 0;
}

pnrt_scene* pnrt_scene_create(void) { return new pnrt_scene(); }
void pnrt_scene_destroy(pnrt_scene* s) { delete s; }

int pnrt_scene_add_material(pnrt_scene* s, const float m[18]) {
    if (!s || !m) return fail(-1, "add_material: null");
    s->materials.emplace_back(m, m + 18);
    s->built = false;
    return (int)s->materials.size() - 1;
}

// ModelOutput (model.hpp:101-135): vertices to world space (normal through
// transpose(inverse(M)) with w = 1, tangents with w = 1 as the reference does),
// triangles with area = |e1 x e2| * 0.5 (double), bound and bound centre.
int pnrt_scene_add_mesh(pnrt_scene* s, int material_id, int texture_id, const float mm[16],
                        const float* pos, const float* nrm, const float* tan, const float* bit,
                        const float* uv, int nv, const int32_t* idx, int ni) {
    if (!s || !mm || !pos || !idx || nv < 0 || ni < 0 || ni % 3) return fail(-1, "add_mesh: bad arguments");
    for (int i = 0; i < ni; ++i)
        if (idx[i] < 0 || idx[i] >= nv) return fail(-2, "add_mesh: index out of range");
    if ((int64_t)s->vertices.size() + nv >= (1 << 24))
        return fail(-3, "add_mesh: > 2^24 vertices cannot be stored as exact floats");
    mat4 M;
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) M.c[i][j] = mm[4 * i + j];
    mat4 N = transpose(inverse(M));
    const int base = (int)s->vertices.size();
    auto get3 = [](const float* a, int i) { return a ? vec3(a[3 * i], a[3 * i + 1], a[3 * i + 2]) : vec3(0.f, 0.f, 0.f); };
    for (int i = 0; i < nv; ++i) {
        Vertex v;
        vec3 p = get3(pos, i), n = get3(nrm, i), t = get3(tan, i), b = get3(bit, i);
        vec4 r;
        r = M * V4(p.x, p.y, p.z, 1.0f); v.position = vec3(r[0], r[1], r[2]);
        r = N * V4(n.x, n.y, n.z, 1.0f); v.normal = vec3(r[0], r[1], r[2]);
        r = M * V4(t.x, t.y, t.z, 1.0f); v.tangent = vec3(r[0], r[1], r[2]);
        r = M * V4(b.x, b.y, b.z, 1.0f); v.bitangent = vec3(r[0], r[1], r[2]);
        if (uv) { v.uv[0] = uv[2 * i]; v.uv[1] = uv[2 * i + 1]; }
        s->vertices.push_back(v);
    }
    for (int i = 0; i < ni; i += 3) {
        Tri t;
        t.indices[0] = idx[i] + base; t.indices[1] = idx[i + 1] + base; t.indices[2] = idx[i + 2] + base;
        t.materialId = material_id;
        t.textureId = texture_id;
        const vec3 p0 = s->vertices[t.indices[0]].position;
        const vec3 p1 = s->vertices[t.indices[1]].position;
        const vec3 p2 = s->vertices[t.indices[2]].position;
        t.area = (float)((double)length(cross(p1 - p0, p2 - p0)) * 0.5);
        t.bound.Union(p0); t.bound.Union(p1); t.bound.Union(p2);
        t.boundCenter = (t.bound.pMax + t.bound.pMin) * .5f;
        s->triangles.push_back(t);
    }
    s->built = false;
    return 0;
}

// main.cpp:374-383: emissive triangles in BVH order, float prefix of areas
static void build_lights(pnrt_scene* s) {
    s->lights.clear();
    for (int i = 0; i < (int)s->triangles.size(); ++i) {
        const Tri& t = s->triangles[i];
        const std::vector<float>& m = s->materials[t.materialId];
        if (!(m[0] == 0.f && m[1] == 0.f && m[2] == 0.f)) {
            s->lights.push_back({i, t.area});
            size_t n = s->lights.size();
            if (n > 1) s->lights[n - 1].second += s->lights[n - 2].second;
        }
    }
}

static int check_buildable(pnrt_scene* s, const char* who) {
    if (!s) return fail(-1, std::string(who) + ": null");
    if (s->triangles.empty()) return fail(-2, std::string(who) + ": scene has no triangles");
    for (const Tri& t : s->triangles)
        if (t.materialId < 0 || t.materialId >= (int)s->materials.size())
            return fail(-3, std::string(who) + ": triangle references an unknown material");
    return 0;
}

int pnrt_scene_build(pnrt_scene* s) {
    if (int rc = check_buildable(s, "build")) return rc;
    BvhBuilder b(s->triangles);
    b.build();
    s->nodes = std::move(b.nodes);
    s->maxDepth = b.maxDepth;
    build_lights(s);
    s->built = true;
    return 0;
}

int pnrt_scene_tri_bounds(const pnrt_scene* s, float* out) {
    if (!s || !out) return fail(-1, "tri_bounds: null");
    size_t k = 0;
    for (const Tri& t : s->triangles) {
        out[k++] = t.bound.pMin.x; out[k++] = t.bound.pMin.y; out[k++] = t.bound.pMin.z;
        out[k++] = t.bound.pMax.x; out[k++] = t.bound.pMax.y; out[k++] = t.bound.pMax.z;
        out[k++] = t.boundCenter.x; out[k++] = t.boundCenter.y; out[k++] = t.boundCenter.z;
    }
    return 0;
}

int pnrt_bvh_build_cpu(const float* tb, int n, float* nodes_out, int cap, int* n_nodes_out, int32_t* order_out,
                       int* max_depth_out) {
    if (!tb || n <= 0 || !nodes_out || !n_nodes_out || !order_out) return fail(-1, "bvh_build_cpu: bad arguments");
    std::vector<Tri> t(n);
    for (int i = 0; i < n; ++i) {
        const float* q = tb + 9 * (size_t)i;
        t[i].bound.pMin = vec3(q[0], q[1], q[2]);
        t[i].bound.pMax = vec3(q[3], q[4], q[5]);
        t[i].boundCenter = vec3(q[6], q[7], q[8]);
        t[i].indices[0] = i;                  // carries the input index through std::partition
    }
    BvhBuilder b(t);
    b.build();
    if ((int)b.nodes.size() > cap) return fail(-2, "bvh_build_cpu: node capacity exceeded");
    for (size_t i = 0; i < b.nodes.size(); ++i) {
        const Node& d = b.nodes[i];
        float* q = nodes_out + 12 * i;
        q[0] = d.bound.pMin.x; q[1] = d.bound.pMin.y; q[2] = d.bound.pMin.z;
        q[3] = d.bound.pMax.x; q[4] = d.bound.pMax.y; q[5] = d.bound.pMax.z;
        q[6] = (float)d.axis; q[7] = (float)d.rightChild; q[8] = (float)d.startIndex; q[9] = (float)d.endIndex;
        q[10] = 0.f; q[11] = 0.f;
    }
    for (int i = 0; i < n; ++i) order_out[i] = t[i].indices[0];
    *n_nodes_out = (int)b.nodes.size();
    if (max_depth_out) *max_depth_out = b.maxDepth;
    return 0;
}

int pnrt_scene_set_bvh(pnrt_scene* s, const int32_t* order, const float* nb, int n_nodes, int max_depth) {
    if (int rc = check_buildable(s, "set_bvh")) return rc;
    const int n = (int)s->triangles.size();
    if (!order || !nb || n_nodes <= 0 || n_nodes > 2 * n - 1) return fail(-4, "set_bvh: bad arguments");
    std::vector<char> seen(n, 0);
    for (int i = 0; i < n; ++i) {
        if (order[i] < 0 || order[i] >= n || seen[order[i]]) return fail(-5, "set_bvh: order is not a permutation");
        seen[order[i]] = 1;
    }
    std::vector<Tri> t(n);
    for (int i = 0; i < n; ++i) t[i] = s->triangles[order[i]];
    std::vector<Node> nodes(n_nodes);
    for (int i = 0; i < n_nodes; ++i) {
        const float* q = nb + 12 * (size_t)i;
        Node& d = nodes[i];
        d.bound.pMin = vec3(q[0], q[1], q[2]);
        d.bound.pMax = vec3(q[3], q[4], q[5]);
        d.axis = (int)q[6]; d.rightChild = (int)q[7]; d.startIndex = (int)q[8]; d.endIndex = (int)q[9];
        if (d.startIndex < 0 || d.endIndex > n || d.startIndex > d.endIndex || d.rightChild >= n_nodes)
            return fail(-6, "set_bvh: node " + std::to_string(i) + " is inconsistent");
    }
    s->triangles.swap(t);
    s->nodes.swap(nodes);
    s->maxDepth = max_depth;
    build_lights(s);
    s->built = true;
    return 0;
}

int pnrt_scene_get_info(const pnrt_scene* s, pnrt_scene_info* info) {
    if (!s || !info) return fail(-1, "get_info: null");
    info->n_vertices = (int)s->vertices.size();
    info->n_materials = (int)s->materials.size();
    info->n_triangles = (int)s->triangles.size();
    info->n_nodes = (int)s->nodes.size();
    info->n_lights = (int)s->lights.size();
    info->lights_sum_area = s->lights.empty() ? 0.f : s->lights.back().second;   // main.cpp:392
    info->max_depth = s->maxDepth;
    return 0;
}

// main.cpp:409-524 packing loops
int pnrt_scene_pack(const pnrt_scene* s, float* vb, float* mb, float* tb, float* nb, float* lb) {
    if (!s) return fail(-1, "pack: null");
    if (!s->built) return fail(-2, "pack: call pnrt_scene_build first");
    if (vb) {
        size_t k = 0;
        for (const Vertex& v : s->vertices) {
            vb[k++] = v.position.x; vb[k++] = v.position.y; vb[k++] = v.position.z;
            vb[k++] = v.normal.x; vb[k++] = v.normal.y; vb[k++] = v.normal.z;
            vb[k++] = v.tangent.x; vb[k++] = v.tangent.y; vb[k++] = v.tangent.z;
            vb[k++] = v.bitangent.x; vb[k++] = v.bitangent.y; vb[k++] = v.bitangent.z;
            vb[k++] = v.uv[0]; vb[k++] = v.uv[1]; vb[k++] = 0.f;
        }
    }
    if (mb) {
        size_t k = 0;
        for (const auto& m : s->materials) for (float f : m) mb[k++] = f;
    }
    if (tb) {
        size_t k = 0;
        for (const Tri& t : s->triangles) {
            tb[k++] = (float)t.indices[0]; tb[k++] = (float)t.indices[1]; tb[k++] = (float)t.indices[2];
            tb[k++] = (float)t.materialId; tb[k++] = (float)t.textureId; tb[k++] = t.area;
        }
    }
    if (nb) {
        size_t k = 0;
        for (const Node& n : s->nodes) {
            nb[k++] = n.bound.pMin.x; nb[k++] = n.bound.pMin.y; nb[k++] = n.bound.pMin.z;
            nb[k++] = n.bound.pMax.x; nb[k++] = n.bound.pMax.y; nb[k++] = n.bound.pMax.z;
            nb[k++] = (float)n.axis; nb[k++] = (float)n.rightChild;
            nb[k++] = (float)n.startIndex; nb[k++] = (float)n.endIndex;
            nb[k++] = 0.f; nb[k++] = 0.f;
        }
    }
    if (lb) {
        size_t k = 0;
        for (const auto& l : s->lights) { lb[k++] = (float)l.first; lb[k++] = l.second; lb[k++] = 0.f; }
    }
    return 0;
}

// Camera::UpdateCamera (camera.hpp:11-31)
int pnrt_camera_update(const float e[3], const float c[3], const float up_[3], float fov,
                       float aspect, float out[12]) {
    if (!e || !c || !up_ || !out) return fail(-1, "camera: null");
    vec3 eye(e[0], e[1], e[2]), center(c[0], c[1], c[2]), up(up_[0], up_[1], up_[2]);
    float theta = radians(fov);
    float halfHeight = (float)std::tan((double)theta * 0.5);
    float halfWidth = aspect * halfHeight;
    vec3 w = normalize(eye - center);
    vec3 u = normalize(cross(up, w));
    vec3 v = cross(w, u);
    vec3 llc = ((eye - halfWidth * u) - halfHeight * v) - w;
    vec3 hor = (2 * halfWidth) * u;
    vec3 ver = (2 * halfHeight) * v;
    const vec3 o[4] = {eye, llc, hor, ver};
    for (int i = 0; i < 4; ++i) { out[3 * i] = o[i].x; out[3 * i + 1] = o[i].y; out[3 * i + 2] = o[i].z; }
    return 0;
}

// ---- Camera (camera.hpp:4-77): state + the interactive controls main.cpp's
// mouse callbacks drive (main.cpp:118-142): left drag UpdateRotate, right drag
// UpdateTranslateUV, scroll UpdateFov.  glm-exact float arithmetic.
static void cam_update(pnrt_camera_state* c, vec3 eye, vec3 center, vec3 up, float fov, float aspect) {
    auto put = [](float* d, vec3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; };
    put(c->eye, eye); put(c->center, center); put(c->up, up);
    c->fov_deg = fov;
    c->aspect = aspect;
    const float theta = radians(fov);
    const float halfHeight = (float)std::tan((double)theta * 0.5);   // glm::tan(theta * 0.5): double
    const float halfWidth = aspect * halfHeight;
    c->distance = length(eye - center);                               // glm::distance
    const vec3 w = normalize(eye - center);
    const vec3 u = normalize(cross(up, w));
    const vec3 v = cross(w, u);
    put(c->w, w); put(c->u, u); put(c->v, v);
    put(c->lower_left, ((eye - halfWidth * u) - halfHeight * v) - w);
    put(c->horizontal, (2 * halfWidth) * u);
    put(c->vertical, (2 * halfHeight) * v);
}
static vec3 v3(const float* a) { return vec3(a[0], a[1], a[2]); }

extern "C" int pnrt_camera_state_init(pnrt_camera_state* c, const float eye[3], const float center[3],
                                      const float up[3], float fov, float aspect) {
    if (!c || !eye || !center || !up) return fail(-1, "camera_state_init: null");
    cam_update(c, v3(eye), v3(center), v3(up), fov, aspect);
    return 0;
}

extern "C" int pnrt_camera_rotate(pnrt_camera_state* c, float phi, float theta) {
    if (!c) return fail(-1, "camera_rotate: null");
    phi *= 0.6;                          // float *= double (camera.hpp:34-35)
    theta *= 0.6;
    phi = radians(phi);
    theta = radians(theta);
    vec3 nv(std::cos(phi) * std::cos(theta), std::sin(phi) * std::cos(theta), std::sin(theta));
    nv = (v3(c->w) * nv.x + v3(c->u) * nv.y) + v3(c->v) * nv.z;
    if (std::abs(dot(v3(c->up), nv)) > 0.9995f) return 0;    // rejected: too close to the up axis
    const vec3 eye = v3(c->center) + nv * c->distance;
    cam_update(c, eye, v3(c->center), v3(c->up), c->fov_deg, c->aspect);
    return 1;
}

extern "C" int pnrt_camera_translate(pnrt_camera_state* c, float dx, float dy) {
    if (!c) return fail(-1, "camera_translate: null");
    dx *= 0.05;                          // camera.hpp:47-48
    dy *= 0.05;
    const vec3 u = v3(c->u), v = v3(c->v);
    const vec3 eye = v3(c->eye) + (dx * u + dy * v);
    const vec3 center = v3(c->center) + (dx * u + dy * v);
    cam_update(c, eye, center, v3(c->up), c->fov_deg, c->aspect);
    return 1;
}

extern "C" int pnrt_camera_zoom(pnrt_camera_state* c, float delta) {
    if (!c) return fail(-1, "camera_zoom: null");
    const float nFov = c->fov_deg + delta;   // camera.hpp:57-63
    if (!(nFov < 89.f && nFov > 1.f)) return 0;
    cam_update(c, v3(c->eye), v3(c->center), v3(c->up), nFov, c->aspect);
    return 1;
}

// ---- Radiance RGBE (stbi_loadf semantics, stb_image.h v2.27 HDR loader) ----------
int pnrt_hdr_decode_rgbe(const uint8_t* bytes, int64_t n, int* pw, int* ph, float* out) {
    if (!bytes || !pw || !ph) return fail(-1, "rgbe: null");
    int64_t p = 0;
    auto eof = [&]() { return p >= n; };
    auto get8 = [&]() -> int { return p < n ? bytes[p++] : 0; };
    auto line = [&]() {
        std::string s;
        int ch = get8();
        while (!eof() && ch != '\n') {
            s.push_back((char)ch);
            if (s.size() == 1023) { while (!eof() && get8() != '\n') {} break; }
            ch = get8();
        }
        return s;
    };
    std::string t = line();
    if (t != "#?RADIANCE" && t != "#?RGBE") return fail(-2, "rgbe: not an HDR image");
    bool valid = false;
    for (;;) {
        t = line();
        if (t.empty()) break;
        if (t == "FORMAT=32-bit_rle_rgbe") valid = true;
    }
    if (!valid) return fail(-3, "rgbe: unsupported format");
    t = line();
    if (t.compare(0, 3, "-Y ") != 0) return fail(-4, "rgbe: unsupported data layout");
    const char* q = t.c_str() + 3;
    char* endp;
    int height = (int)strtol(q, &endp, 10);
    while (*endp == ' ') ++endp;
    if (strncmp(endp, "+X ", 3) != 0) return fail(-4, "rgbe: unsupported data layout");
    int width = (int)strtol(endp + 3, nullptr, 10);
    if (width <= 0 || height <= 0 || width > (1 << 24) || height > (1 << 24)) return fail(-5, "rgbe: bad size");
    *pw = width; *ph = height;
    if (!out) return 0;
    auto convert = [](float* o, const uint8_t* rgbe) {
        if (rgbe[3] != 0) {
            float f1 = (float)std::ldexp(1.0f, rgbe[3] - (int)(128 + 8));
            o[0] = rgbe[0] * f1; o[1] = rgbe[1] * f1; o[2] = rgbe[2] * f1;
        } else {
            o[0] = o[1] = o[2] = 0.f;
        }
    };
    auto flat = [&](int64_t start) {
        for (int64_t k = start; k < (int64_t)width * height; ++k) {
            uint8_t rgbe[4] = {(uint8_t)get8(), (uint8_t)get8(), (uint8_t)get8(), (uint8_t)get8()};
            convert(out + 3 * k, rgbe);
        }
    };
    if (width < 8 || width >= 32768) { flat(0); return 0; }
    std::vector<uint8_t> scan((size_t)width * 4);
    for (int j = 0; j < height; ++j) {
        int c1 = get8(), c2 = get8(), len = get8();
        if (c1 != 2 || c2 != 2 || (len & 0x80)) {
            // not RLE: stb decodes THIS pixel as pixel 0 and restarts flat at pixel 1
            uint8_t rgbe[4] = {(uint8_t)c1, (uint8_t)c2, (uint8_t)len, (uint8_t)get8()};
            convert(out, rgbe);
            flat(1);
            return 0;
        }
        len <<= 8;
        len |= get8();
        if (len != width) return fail(-6, "rgbe: invalid decoded scanline length");
        for (int k = 0; k < 4; ++k) {
            int i = 0, nleft;
            while ((nleft = width - i) > 0) {
                int count = get8();
                if (count > 128) {
                    int value = get8();
                    count -= 128;
                    if (count > nleft) return fail(-7, "rgbe: bad RLE data");
                    for (int z = 0; z < count; ++z) scan[(size_t)(i++) * 4 + k] = (uint8_t)value;
                } else {
                    if (count > nleft) return fail(-7, "rgbe: bad RLE data");
                    for (int z = 0; z < count; ++z) scan[(size_t)(i++) * 4 + k] = (uint8_t)get8();
                }
            }
        }
        for (int i = 0; i < width; ++i) convert(out + 3 * ((size_t)j * width + i), &scan[(size_t)i * 4]);
    }
    return 0;
}

// LoadHDRImage (shader.hpp:145-203): float/double mix exactly as written.
int pnrt_hdr_build_table(const float* img, int width, int height, float* rh) {
    if (!img || !rh || width <= 0 || height <= 0) return fail(-1, "hdr_table: bad arguments");
    std::vector<std::vector<float>> pdf(width, std::vector<float>(height));
    float pdfSum = 0.0f;
    for (int x = 0; x < width; ++x)
        for (int y = 0; y < height; ++y) {
            size_t pos = (size_t)y * width + x;
            float lumen = (float)(((double)img[pos * 3 + 0] * 0.2 + (double)img[pos * 3 + 1] * 0.7) +
                                  (double)img[pos * 3 + 2] * 0.1);
            pdf[x][y] = lumen;
            pdfSum += lumen;
        }
    std::vector<float> cdfX(width), pdfX(width, 0.0f);
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) {
            pdf[x][y] /= pdfSum;
            pdfX[x] += pdf[x][y];
        }
    cdfX[0] = pdfX[0];
    for (int x = 1; x < width; ++x) cdfX[x] = cdfX[x - 1] + pdfX[x];
    std::vector<std::vector<float>> cdfY(width, std::vector<float>(height));
    for (int x = 0; x < width; ++x)
        for (int y = 0; y < height; ++y)
            cdfY[x][y] = (float)((y > 0 ? (double)cdfY[x][y - 1] : 0.0) + (double)(pdf[x][y] / pdfX[x]));
    for (int i = 0; i < width; ++i)
        for (int j = 0; j < height; ++j) {
            int x = (int)(std::lower_bound(cdfX.begin(), cdfX.end(), (float)i / width) - cdfX.begin());
            if (x >= width) x = width - 1;
            if (x < 0) x = 0;
            int y = (int)(std::lower_bound(cdfY[x].begin(), cdfY[x].end(), (float)j / height) - cdfY[x].begin());
            if (y >= height) y = height - 1;
            if (y < 0) y = 0;
            size_t pos = 3 * ((size_t)j * width + i);
            rh[pos + 0] = (float)x / width;
            rh[pos + 1] = (float)y / height;
            rh[pos + 2] = pdf[x][y];
        }
    return 0;
}

}  // extern "C"

// ---- procedural stand-ins -----------------------------------------------------------
namespace {
inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
inline double lattice(int i, int j, int k, uint32_t seed) {
    uint32_t h = hash32((uint32_t)i * 73856093U ^ hash32((uint32_t)j * 19349663U ^ hash32((uint32_t)k * 83492791U ^ seed)));
    return (double)(h & 0xffffff) / (double)0xffffff * 2.0 - 1.0;
}
double value_noise(double x, double y, double z, uint32_t seed) {
    int ix = (int)std::floor(x), iy = (int)std::floor(y), iz = (int)std::floor(z);
    double fx = x - ix, fy = y - iy, fz = z - iz;
    auto s = [](double t) { return t * t * (3.0 - 2.0 * t); };
    double ux = s(fx), uy = s(fy), uz = s(fz);
    double r = 0.0;
    for (int c = 0; c < 8; ++c) {
        int dx = c & 1, dy = (c >> 1) & 1, dz = (c >> 2) & 1;
        double w = (dx ? ux : 1 - ux) * (dy ? uy : 1 - uy) * (dz ? uz : 1 - uz);
        r += w * lattice(ix + dx, iy + dy, iz + dz, seed);
    }
    return r;
}
struct MeshOut {
    float *pos, *nrm, *uv; int32_t* idx;
    int nv = 0, nt = 0;
    void vert(double px, double py, double pz, double nx, double ny, double nz, double u, double v) {
        if (pos) { pos[3 * nv] = (float)px; pos[3 * nv + 1] = (float)py; pos[3 * nv + 2] = (float)pz; }
        if (nrm) { nrm[3 * nv] = (float)nx; nrm[3 * nv + 1] = (float)ny; nrm[3 * nv + 2] = (float)nz; }
        if (uv) { uv[2 * nv] = (float)u; uv[2 * nv + 1] = (float)v; }
        ++nv;
    }
    void tri() { if (idx) { idx[3 * nt] = nv - 3; idx[3 * nt + 1] = nv - 2; idx[3 * nt + 2] = nv - 1; } ++nt; }
};
// Parametric surface f(u,v) -> (p, n) tessellated into nu x nv quads, two
// triangles per quad, unshared vertices (as Assimp's OBJ import yields).
template <class F>
void grid(MeshOut& m, int nu, int nv, F f) {
    for (int j = 0; j < nv; ++j)
        for (int i = 0; i < nu; ++i) {
            double P[4][3], N[4][3], U[4][2];
            const int ci[4] = {i, i + 1, i + 1, i}, cj[4] = {j, j, j + 1, j + 1};
            for (int c = 0; c < 4; ++c) {
                double u = (double)ci[c] / nu, v = (double)cj[c] / nv;
                f(u, v, P[c], N[c]);
                U[c][0] = u; U[c][1] = v;
            }
            const int tri_c[2][3] = {{0, 2, 1}, {0, 3, 2}};
            for (int t = 0; t < 2; ++t) {
                for (int k = 0; k < 3; ++k) {
                    int c = tri_c[t][k];
                    m.vert(P[c][0], P[c][1], P[c][2], N[c][0], N[c][1], N[c][2], U[c][0], U[c][1]);
                }
                m.tri();
            }
        }
}
}  // namespace

extern "C" {

int pnrt_mesh_quad(float half, float* pos, float* nrm, float* uv, int32_t* idx, int* nv, int* nt) {
    MeshOut m{pos, nrm, uv, idx};
    const double h = half;
    const double c[4][3] = {{-h, 0, h}, {h, 0, h}, {h, 0, -h}, {-h, 0, -h}};
    const double t[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
    const int tris[2][3] = {{0, 1, 2}, {0, 2, 3}};
    for (auto& tr : tris) {
        for (int k : tr) m.vert(c[k][0], c[k][1], c[k][2], 0, 1, 0, t[k][0], t[k][1]);
        m.tri();
    }
    if (nv) *nv = m.nv;
    if (nt) *nt = m.nt;
    return 0;
}

int pnrt_mesh_displaced_sphere(int nu, int nvv, float radius, const float center[3], float amp,
                               uint32_t seed, float* pos, float* nrm, float* uv, int32_t* idx,
                               int* nv, int* nt) {
    if (nu < 3 || nvv < 2 || !center) return fail(-1, "sphere: bad arguments");
    MeshOut m{pos, nrm, uv, idx};
    const double PI_D = 3.14159265358979323846;
    grid(m, nu, nvv, [&](double u, double v, double* P, double* N) {
        double phi = 2.0 * PI_D * u, th = PI_D * v;
        double dx = std::sin(th) * std::cos(phi), dy = std::cos(th), dz = std::sin(th) * std::sin(phi);
        double n = value_noise(4.0 * dx + 10.0, 4.0 * dy + 10.0, 4.0 * dz + 10.0, seed) +
                   0.5 * value_noise(9.0 * dx + 20.0, 9.0 * dy + 20.0, 9.0 * dz + 20.0, seed ^ 0x9e3779b9U);
        double r = radius * (1.0 + amp * n);
        P[0] = center[0] + r * dx; P[1] = center[1] + r * dy; P[2] = center[2] + r * dz;
        N[0] = dx; N[1] = dy; N[2] = dz;
    });
    if (nv) *nv = m.nv;
    if (nt) *nt = m.nt;
    return 0;
}

// Teapot-class stand-in (the Utah teapot OBJ is absent): lathe body with lid
// and knob, a tapered spout tube and a torus-section handle; ~6.1k triangles.
int pnrt_mesh_teapot(float* pos, float* nrm, float* uv, int32_t* idx, int* nv, int* nt) {
    MeshOut m{pos, nrm, uv, idx};
    const double PI_D = 3.14159265358979323846;
    // body profile r(t), y(t), t in [0,1]: bottom -> belly -> shoulder -> lid -> knob
    auto prof = [&](double t, double& r, double& y) {
        const double py[] = {0.0, 0.15, 0.55, 1.0, 1.35, 1.5, 1.58, 1.62, 1.78, 1.9, 1.95};
        const double pr[] = {0.0, 1.15, 1.45, 1.4, 1.1, 0.9, 0.75, 0.15, 0.12, 0.22, 0.0};
        double s = t * 10.0; int k = (int)s; if (k > 9) k = 9; double f = s - k;
        r = pr[k] + (pr[k + 1] - pr[k]) * f; y = py[k] + (py[k + 1] - py[k]) * f;
    };
    grid(m, 64, 32, [&](double u, double v, double* P, double* N) {
        double r, y, r2, y2; prof(v, r, y); prof(v < 1.0 ? v + 1e-3 : v - 1e-3, r2, y2);
        double a = 2.0 * PI_D * u, ca = std::cos(a), sa = std::sin(a);
        double dr = (v < 1.0 ? r2 - r : r - r2), dy = (v < 1.0 ? y2 - y : y - y2);
        double nx = dy, ny = -dr, l = std::sqrt(nx * nx + ny * ny); if (l == 0) { nx = 0; ny = 1; l = 1; }
        P[0] = r * ca; P[1] = y; P[2] = r * sa;
        N[0] = nx / l * ca; N[1] = ny / l; N[2] = nx / l * sa;
    });
    // spout: tube along a quadratic curve from the belly outwards/upwards
    grid(m, 24, 16, [&](double u, double v, double* P, double* N) {
        double cx = 1.3 + 1.0 * v, cy = 0.6 + 0.9 * v * v, rad = 0.28 - 0.16 * v;
        double tx = 1.0, ty = 1.8 * v, tl = std::sqrt(tx * tx + ty * ty); tx /= tl; ty /= tl;
        double a = 2.0 * PI_D * u, ca = std::cos(a), sa = std::sin(a);
        double nx = -ty * ca, ny = tx * ca, nz = sa;
        P[0] = cx + rad * nx; P[1] = cy + rad * ny; P[2] = rad * nz;
        N[0] = nx; N[1] = ny; N[2] = nz;
    });
    // handle: torus section on the -x side
    grid(m, 32, 12, [&](double u, double v, double* P, double* N) {
        double big = 0.55, small = 0.09;
        double a = PI_D * (0.5 + u) , b = 2.0 * PI_D * v;
        double cx = -1.35 + big * std::cos(a) * 0.8, cy = 0.85 + big * std::sin(a);
        double ox = std::cos(a) * std::cos(b), oy = std::sin(a) * std::cos(b), oz = std::sin(b);
        P[0] = cx + small * ox; P[1] = cy + small * oy; P[2] = small * oz;
        N[0] = ox; N[1] = oy; N[2] = oz;
    });
    if (nv) *nv = m.nv;
    if (nt) *nt = m.nt;
    return 0;
}

int pnrt_hdr_synthetic(int w, int h, uint32_t seed, float* out) {
    if (w <= 0 || h <= 0 || !out) return fail(-1, "hdr_synthetic: bad arguments");
    const double PI_D = 3.14159265358979323846;
    const double sun[3] = {0.42, 0.62, -0.66};
    for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i) {
            double u = (i + 0.5) / w, v = (j + 0.5) / h;
            double phi = 2.0 * PI_D * (u - 0.5), th = PI_D * (0.5 - v);   // row 0 = sky top
            double d[3] = {std::cos(th) * std::cos(phi), std::sin(th), std::cos(th) * std::sin(phi)};
            double up = d[1] > 0 ? d[1] : 0.0;
            double nz = 0.15 * value_noise(8.0 * u * 4 + 3.0, 8.0 * v * 2 + 5.0, 0.5, seed);
            double sky[3] = {0.25 + 0.5 * up, 0.35 + 0.55 * up, 0.6 + 0.7 * up};
            if (d[1] < 0) { sky[0] = 0.18; sky[1] = 0.16; sky[2] = 0.14; }
            double cs = d[0] * sun[0] + d[1] * sun[1] + d[2] * sun[2];
            double lobe = cs > 0.995 ? 2000.0 * (cs - 0.995) / 0.005 : 0.0;
            for (int c = 0; c < 3; ++c)
                out[3 * ((size_t)j * w + i) + c] = (float)(sky[c] * (1.0 + nz) + lobe * (c == 2 ? 0.8 : 1.0));
        }
    return 0;
}

}  // extern "C"
