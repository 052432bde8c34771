// tools/step_model/step_model.cpp -- cost model of the trace kernel's step loop
// (VERDICT r5 "Next" 1): which wave-level step organisation would cut the
// trace launch, priced from per-ray step sequences of a real scene.
//
// Input (written by tools/step_model.py from the C2 scene the bench renders):
// the reference-layout BVH (BVH.hpp:92-173; node = 12 floats: min 0-2, max 3-5,
// axis 6, right child 7 (-1 leaf), triangle range 8-9), triangle vertex
// positions (9 floats per triangle, BVH order), the light triangles and the
// camera.  Paths are sampled the way the bench's paths are laid out (8x8-pixel
// tiles, frame-major; cosine continuation, a light shadow ray to a point on a
// light, an env shadow ray above the surface), bounce by bounce to depth 4.
//
// Per ray the traversal is the device's (pt_wf.h wf_step): near child by the sign
// of dir[axis] (ray_tracing.comp:448), far child pushed with its z-slab lower end,
// z-slab culling against tMax, leaf triangles one per step in order, closest-hit
// tMax shrinking, any-hit rays stop at the first accepted triangle.  The model
// records each ray's sequence of step kinds (N: node visit, T: triangle test),
// and the same ray under a grandchild ("4-wide of the same binary tree")
// traversal (G: one step visiting a node's four grandchildren).
//
// Wave simulation (64 lanes, the kernel's refill rule: refill idle lanes, then step
// until at most WF_REFILL_PCT % of the refilled busy count remain): for each
// organisation the wave iterations by kind and the lanes they serve; priced with
// the VALU per iteration kind (static census of the compiled loops, given on the
// command line) and an iteration-latency share calibrated on the measured
// unified kernel (VALU issue 0.65 of the launch, profiles/r05/s23/pmc_valu.txt).
//
//   step_model <dir> [tiles_step]     (dir: the .bin files of step_model.py)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

struct V3 { float x, y, z; };
static inline V3 v3(float a, float b, float c) { return {a, b, c}; }
static inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline V3 norm(V3 a) { float l = std::sqrt(dot(a, a)); return {a.x / l, a.y / l, a.z / l}; }
static inline float c3(V3 a, int k) { return k == 0 ? a.x : k == 1 ? a.y : a.z; }

static std::vector<float> load(const std::string& f) {
    FILE* fp = fopen(f.c_str(), "rb");
    if (!fp) { fprintf(stderr, "cannot open %s\n", f.c_str()); exit(1); }
    fseek(fp, 0, SEEK_END);
    long n = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    std::vector<float> v(n / 4);
    if (fread(v.data(), 4, v.size(), fp) != v.size()) exit(1);
    fclose(fp);
    return v;
}

struct Scene {
    std::vector<float> N, T;     // nodes (12 f), triangle positions (9 f)
    std::vector<float> L;        // light triangle indices
    std::vector<float> cam;      // eye, lowerLeft, horizontal, vertical
    int nn = 0, nt = 0;
    bool leaf(int i) const { return N[12 * i + 7] < 0; }
    int right(int i) const { return (int)N[12 * i + 7]; }
    const float* box(int i) const { return &N[12 * i]; }
    int axis(int i) const { return (int)N[12 * i + 6]; }
    int t0(int i) const { return (int)N[12 * i + 8]; }
    int t1(int i) const { return (int)N[12 * i + 9]; }
};

struct Ray {
    V3 o, d, inv;
    int kz;
    float tmax;
    bool any;
    bool flip;        // far child first (an any-hit ray's visit order is free): the product flips env rays
};
static int g_flipmode = 2;        // FLIP: 0 no any-hit ray flipped, 1 every any-hit ray, 2 env rays (the product)
static int g_anyord = 0;          // ANYORD: any-hit rays by a fixed per-node order -- 1 larger child first, 2 smaller
static Ray mkray(V3 o, V3 d, float tmax, bool any, bool env = false) {
    Ray r{o, d, v3(1.f / d.x, 1.f / d.y, 1.f / d.z), 2, tmax, any,
          any && (g_flipmode == 1 || (g_flipmode == 2 && env))};
    if (d.z == 0.f) r.kz = std::fabs(d.x) > std::fabs(d.y) ? 0 : 1;
    return r;
}
// BoundIntersect (:213-228) + the z-slab of the triangle test's frame (pt_wf.h box_slabs)
static bool box(const Ray& r, const float* b, float& zlo, float& zhi) {
    float f[3], n[3];
    for (int k = 0; k < 3; ++k) {
        f[k] = (b[3 + k] - c3(r.o, k)) * c3(r.inv, k);
        n[k] = (b[k] - c3(r.o, k)) * c3(r.inv, k);
    }
    float t1 = std::fmin(std::fmax(f[0], n[0]), std::fmin(std::fmax(f[1], n[1]), std::fmax(f[2], n[2])));
    float t0 = std::fmax(std::fmin(f[0], n[0]), std::fmax(std::fmin(f[1], n[1]), std::fmin(f[2], n[2])));
    zlo = std::fmin(n[r.kz], f[r.kz]);
    zhi = std::fmax(n[r.kz], f[r.kz]);
    return t1 >= t0 && !(zhi <= 0.f);
}
static bool culled(float zlo, float tmax) {
    const float tmc = tmax * 1.000001f;
    return zlo > (tmc <= 1e-20f ? 1e-20f : tmc);
}
// watertight test (:254-357), the hit distance or -1
static float tri(const Scene& s, const Ray& r, int t, float tmax) {
    const float* p = &s.T[9 * t];
    V3 P[3];
    for (int k = 0; k < 3; ++k) P[k] = sub(v3(p[3 * k], p[3 * k + 1], p[3 * k + 2]), r.o);
    int kx = 0, ky = 1, kz = r.kz;
    if (kz == 0) kx = 2;
    if (kz == 1) ky = 2;
    float sx = c3(r.d, kx), sy = c3(r.d, ky), iz = c3(r.inv, kz);
    float X[3], Y[3], Z[3];
    for (int k = 0; k < 3; ++k) {
        float pz = c3(P[k], kz);
        X[k] = c3(P[k], kx) - (pz * sx) * iz;
        Y[k] = c3(P[k], ky) - (pz * sy) * iz;
        Z[k] = pz * iz;
    }
    float e0 = X[1] * Y[2] - Y[1] * X[2], e1 = X[2] * Y[0] - Y[2] * X[0], e2 = X[0] * Y[1] - Y[0] * X[1];
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return -1.f;
    float det = (e0 + e1) + e2;
    if (det == 0) return -1.f;
    float ts = (e0 * Z[0] + e1 * Z[1]) + e2 * Z[2];
    if (det > 0 && (ts <= 0 || ts > tmax * det)) return -1.f;
    if (det < 0 && (ts >= 0 || ts < tmax * det)) return -1.f;
    return ts * (1.f / det);
}

struct Entry { int node; float z; };   // node index (interior or leaf), z-slab lower end

// per (ray kind, bounce) census of the device traversal (the C3-vs-C2 record)
struct Census {
    double rays = 0, nodes = 0, tris = 0, leaves = 0, leaf_tris = 0, accepted = 0, depth_sum = 0;
    double depth_hist[6] = {0, 0, 0, 0, 0, 0};    // node visits by depth: 0-3, 4-7, ..., 20+
};
static std::vector<int> g_depth;

// The device traversal (binary, one node or one triangle per step): returns the hit
// triangle (-1), the step kinds ('N' / 'T'), the hit distance; the census when given
static int trace_bin(const Scene& s, Ray r, std::string* seq, float* thit, Census* cs = nullptr) {
    float zlo, zhi;
    if (seq) seq->clear();
    if (cs) cs->rays += 1;
    auto enter_leaf = [&](int n) { if (cs) { cs->leaves += 1; cs->leaf_tris += s.t1(n) - s.t0(n); } };
    if (!box(r, s.box(0), zlo, zhi)) return -1;
    std::vector<Entry> st;
    int cur = 0, hit = -1;
    int lt = 0, lc = 0;
    if (s.leaf(0)) { lt = s.t0(0); lc = s.t1(0) - lt; cur = -1; enter_leaf(0); }
    for (;;) {
        if (lc > 0) {
            if (seq) seq->push_back('T');
            if (cs) cs->tris += 1;
            float t = tri(s, r, lt, r.tmax);
            if (t >= 0) {
                hit = lt;
                if (cs) cs->accepted += 1;
                if (r.any) return hit;
                r.tmax = t;
            }
            ++lt; --lc;
        } else if (cur >= 0) {
            if (seq) seq->push_back('N');
            if (cs) { cs->nodes += 1; cs->depth_sum += g_depth[cur]; cs->depth_hist[std::min(5, g_depth[cur] / 4)] += 1; }
            int L = cur + 1, R = s.right(cur);
            float zl, zr, h;
            bool hl = box(r, s.box(L), zl, h) && !culled(zl, r.tmax);
            bool hr = box(r, s.box(R), zr, h) && !culled(zr, r.tmax);
            bool rf = (c3(r.d, s.axis(cur)) < 0) != r.flip;
            if (r.any && g_anyord) {     // a fixed per-node preference: the child of larger (1) / smaller (2) surface area
                auto sa = [&](int c) { const float* b = s.box(c); float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
                                       return dx * dy + dy * dz + dz * dx; };
                rf = (sa(R) > sa(L)) == (g_anyord == 1);
            }
            int nearc = rf ? R : L, farc = rf ? L : R;
            bool hn = rf ? hr : hl, hf = rf ? hl : hr;
            float zf = rf ? zl : zr;
            cur = -1;
            int go = -1;
            if (hn) { if (hf) st.push_back({farc, zf}); go = nearc; }
            else if (hf) go = farc;
            if (go >= 0) {
                if (s.leaf(go)) { lt = s.t0(go); lc = s.t1(go) - lt; enter_leaf(go); }
                else cur = go;
            }
        }
        if (lc <= 0 && cur < 0) {
            for (;;) {
                if (st.empty()) { if (thit) *thit = r.tmax; return hit; }
                Entry e = st.back();
                st.pop_back();
                if (culled(e.z, r.tmax)) continue;
                if (s.leaf(e.node)) { lt = s.t0(e.node); lc = s.t1(e.node) - lt; enter_leaf(e.node); }
                else cur = e.node;
                break;
            }
        }
    }
}

// The grandchild traversal of the same tree: a step at interior node n whose
// children are interior tests the (up to four) grandchildren's boxes directly and
// orders them as the reference would reach them (near child's near / far, then
// the far child's); a leaf child is taken as it is.  Same triangles, same order.
// Returns the step sequence ('G' node steps, 'T' triangle steps).
static void trace_quad(const Scene& s, Ray r, std::string& seq) {
    seq.clear();
    float zlo, zhi;
    if (!box(r, s.box(0), zlo, zhi)) return;
    std::vector<Entry> st;
    int cur = s.leaf(0) ? -1 : 0, lt = 0, lc = 0;
    if (s.leaf(0)) { lt = s.t0(0); lc = s.t1(0) - lt; }
    for (;;) {
        if (lc > 0) {
            seq.push_back('T');
            float t = tri(s, r, lt, r.tmax);
            if (t >= 0) { if (r.any) return; r.tmax = t; }
            ++lt; --lc;
        } else if (cur >= 0) {
            seq.push_back('G');
            // the children in the reference's order, each expanded once more if interior
            std::vector<Entry> order;   // visit order (first = next)
            int L = cur + 1, R = s.right(cur);
            bool rf = (c3(r.d, s.axis(cur)) < 0) != r.flip;
            int cs[2] = {rf ? R : L, rf ? L : R};
            for (int c : cs) {
                float zc, h;
                if (s.leaf(c)) {
                    if (box(r, s.box(c), zc, h) && !culled(zc, r.tmax)) order.push_back({c, zc});
                    continue;
                }
                int cl = c + 1, cr = s.right(c);
                bool crf = (c3(r.d, s.axis(c)) < 0) != r.flip;
                int gs[2] = {crf ? cr : cl, crf ? cl : cr};
                for (int g : gs) {
                    float zg;
                    if (box(r, s.box(g), zg, h) && !culled(zg, r.tmax)) order.push_back({g, zg});
                }
            }
            cur = -1;
            for (int k = (int)order.size() - 1; k >= 1; --k) st.push_back(order[k]);
            if (!order.empty()) {
                int go = order[0].node;
                if (s.leaf(go)) { lt = s.t0(go); lc = s.t1(go) - lt; }
                else cur = go;
            }
        }
        if (lc <= 0 && cur < 0) {
            for (;;) {
                if (st.empty()) return;
                Entry e = st.back();
                st.pop_back();
                if (culled(e.z, r.tmax)) continue;
                if (s.leaf(e.node)) { lt = s.t0(e.node); lc = s.t1(e.node) - lt; }
                else cur = e.node;
                break;
            }
        }
    }
}

// ---- wave simulation -------------------------------------------------------------------------------
struct WaveStats {
    double iters = 0, lane_steps = 0, it_kind[4] = {0, 0, 0, 0};   // U / N-only / T-only / G
    double lanes_kind[4] = {0, 0, 0, 0};
};
enum Policy { UNIFIED, PHASED_MAJ, PHASED_K, SKIP_SPARSE, QUAD_UNIFIED };

// Each lane consumes its ray's symbols.  UNIFIED: every busy lane advances one symbol
// per iteration.  PHASED_*: an iteration is node-only or triangle-only; only lanes whose
// next symbol is that kind advance.  SKIP_SPARSE: unified, but node-only when at most k
// lanes are at a triangle and triangle-only when at most k are at a node (the others
// wait).  QUAD_UNIFIED: unified over the 'G' / 'T' sequences.
static WaveStats simulate(const std::vector<std::string>& rays, Policy pol, int k, int refill_pct) {
    WaveStats ws;
    size_t next = 0;
    const int W = 64;
    std::vector<const std::string*> lane(W, nullptr);
    std::vector<size_t> pos(W, 0);
    bool tri_phase = false;
    for (;;) {
        // refill
        for (int l = 0; l < W && next < rays.size(); ++l)
            if (!lane[l]) {
                while (next < rays.size() && rays[next].empty()) ++next;      // a ray rejected at the root
                if (next < rays.size()) { lane[l] = &rays[next++]; pos[l] = 0; }
            }
        int busy = 0;
        for (int l = 0; l < W; ++l) busy += lane[l] != nullptr;
        if (!busy) break;
        const int thr = next < rays.size() ? busy * refill_pct / 100 : 0;
        for (;;) {
            int nN = 0, nT = 0;
            for (int l = 0; l < W; ++l)
                if (lane[l]) { char c = (*lane[l])[pos[l]]; if (c == 'T') ++nT; else ++nN; }
            int kind;     // 0 unified, 1 node-only, 2 tri-only, 3 quad unified
            switch (pol) {
            case UNIFIED: kind = 0; break;
            case QUAD_UNIFIED: kind = 3; break;
            case PHASED_MAJ: kind = nT >= nN ? 2 : 1; break;
            case PHASED_K:   // hysteresis: node phase until >= k lanes wait at triangles (or no node lane
                             // is left), triangle phase until fewer than 8 remain (or no node lane waits)
                if (tri_phase) tri_phase = nT >= 8 || (nN == 0 && nT > 0);
                else tri_phase = nT >= k || nN == 0;
                kind = tri_phase ? 2 : 1;
                break;
            default:        // SKIP_SPARSE
                kind = (nT <= k && nN > 0) ? 1 : (nN <= k && nT > 0) ? 2 : 0;
            }
            int served = 0;
            for (int l = 0; l < W; ++l) {
                if (!lane[l]) continue;
                char c = (*lane[l])[pos[l]];
                bool adv = kind == 0 || kind == 3 || (kind == 1 && c != 'T') || (kind == 2 && c == 'T');
                if (!adv) continue;
                ++served;
                if (++pos[l] == lane[l]->size()) lane[l] = nullptr;
            }
            ws.iters += 1;
            ws.it_kind[kind] += 1;
            ws.lanes_kind[kind] += served;
            ws.lane_steps += served;
            int b = 0;
            for (int l = 0; l < W; ++l) b += lane[l] != nullptr;
            if (b <= thr || b == 0) break;
        }
    }
    return ws;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: step_model <dir> [tile_step] [VALU U N T G]\n"); return 2; }
    std::string dir = argv[1];
    const int tstep = argc > 2 ? atoi(argv[2]) : 6;
    // VALU per iteration kind (static census of the executed path; defaults: the round-5
    // identity step loop 128, and the estimates for the split halves and the 4-wide step)
    double VU = argc > 3 ? atof(argv[3]) : 128, VN = argc > 4 ? atof(argv[4]) : 85, VT = argc > 5 ? atof(argv[5]) : 85,
           VG = argc > 6 ? atof(argv[6]) : 208;
    Scene s;
    s.N = load(dir + "/nodes.bin");
    s.T = load(dir + "/tripos.bin");
    s.L = load(dir + "/lights.bin");
    s.cam = load(dir + "/camera.bin");
    s.nn = (int)s.N.size() / 12;
    s.nt = (int)s.T.size() / 9;
    const int Wd = 1920, Hd = 1080, frames = 4, depth = 4;
    V3 eye = v3(s.cam[0], s.cam[1], s.cam[2]), ll = v3(s.cam[3], s.cam[4], s.cam[5]);
    V3 hor = v3(s.cam[6], s.cam[7], s.cam[8]), ver = v3(s.cam[9], s.cam[10], s.cam[11]);
    std::mt19937 rng(7);
    if (getenv("FLIP")) g_flipmode = atoi(getenv("FLIP"));
    g_anyord = getenv("ANYORD") ? atoi(getenv("ANYORD")) : 0;
    // node depths (left child = i + 1, right child = node[7]) for the census
    g_depth.assign(s.nn, 0);
    for (int i = 0; i < s.nn; ++i)
        if (!s.leaf(i)) { g_depth[i + 1] = g_depth[i] + 1; g_depth[s.right(i)] = g_depth[i] + 1; }
    Census cen[3][4];     // [cont, env, light][bounce]
    std::uniform_real_distribution<float> U(0.f, 1.f);
    auto face_n = [&](int t) {
        const float* p = &s.T[9 * t];
        V3 a = v3(p[0], p[1], p[2]), b = v3(p[3], p[4], p[5]), c = v3(p[6], p[7], p[8]);
        return norm(cross(sub(b, a), sub(c, a)));
    };
    // paths of every tile_step-th 8x8 tile, frame-major inside a tile (the device's path order)
    struct Path { V3 o, dir; bool live; };
    std::vector<Path> paths;
    for (int ty = 0; ty < Hd / 8; ty += tstep)
        for (int tx = 0; tx < Wd / 8; tx += tstep)
            for (int f = 0; f < frames; ++f)
                for (int p = 0; p < 64; ++p) {
                    int x = tx * 8 + (p & 7), y = ty * 8 + (p >> 3);
                    V3 d = norm(sub(add(add(ll, mul(hor, (x + 0.5f) / Wd)), mul(ver, (y + 0.5f) / Hd)), eye));
                    paths.push_back({eye, d, true});
                }
    printf("paths %zu (every %d-th 8x8 tile of %dx%d, %d frames), nodes %d, triangles %d\n", paths.size(), tstep, Wd, Hd,
           frames, s.nn, s.nt);
    double sumN = 0, sumT = 0, sumG = 0, sumTq = 0, nrays = 0;
    const int KS[] = {0, 2, 4, 6, 8, 12, 16};
    const int NP = 4 + (int)(sizeof(KS) / sizeof(KS[0]));
    std::vector<std::string> pname = {"unified (product)", "phased majority", "phased hysteresis k=32",
                                      "grandchild 4-wide, unified"};
    for (int k : KS) pname.push_back("unified, skip sparse k=" + std::to_string(k));
    std::vector<WaveStats> all(NP);
    // primary hits (traced once per call: not part of the trace launches)
    for (int b = 0; b < depth; ++b) {
        std::vector<std::string> qc, qe, ql, qcq, qeq, qlq;
        std::vector<Path> nextp(paths.size());
        for (size_t i = 0; i < paths.size(); ++i) {
            Path& P = paths[i];
            nextp[i].live = false;
            if (!P.live) continue;
            float th;
            Ray pr = mkray(P.o, P.dir, 3.402823466e38f, false);
            int h = trace_bin(s, pr, nullptr, &th);
            if (h < 0) continue;
            V3 X = add(P.o, mul(P.dir, th));
            V3 n = face_n(h);
            if (dot(n, P.dir) > 0) n = mul(n, -1.f);
            V3 oo = add(X, mul(n, 1e-4f));
            // continuation: cosine-weighted about n
            V3 t = std::fabs(n.z) > 0.9999995f ? v3(1, 0, 0) : norm(cross(n, v3(0, 0, 1)));
            V3 bb = cross(n, t);
            float r1 = U(rng), r2 = U(rng), ph = 6.2831853f * r1, sr = std::sqrt(r2);
            V3 dc = norm(add(add(mul(t, sr * std::cos(ph)), mul(bb, sr * std::sin(ph))), mul(n, std::sqrt(1 - r2))));
            std::string sq;
            trace_bin(s, mkray(oo, dc, 3.402823466e38f, false), &sq, nullptr, &cen[0][b]);
            qc.push_back(sq);
            std::string sq4;
            trace_quad(s, mkray(oo, dc, 3.402823466e38f, false), sq4);
            qcq.push_back(sq4);
            nextp[i] = {oo, dc, true};
            // light: a point on a light triangle, unnormalised direction, tMax = 1 - eps
            if (!s.L.empty()) {
                int lt = (int)s.L[(size_t)(U(rng) * s.L.size()) % s.L.size()];
                const float* p = &s.T[9 * lt];
                float a = std::sqrt(U(rng)), c = U(rng);
                V3 q = add(add(mul(v3(p[0], p[1], p[2]), 1 - a), mul(v3(p[3], p[4], p[5]), a * (1 - c))),
                           mul(v3(p[6], p[7], p[8]), a * c));
                V3 dl = sub(q, oo);
                trace_bin(s, mkray(oo, dl, 1.f - 1e-4f, true), &sq, nullptr, &cen[2][b]);
                ql.push_back(sq);
                trace_quad(s, mkray(oo, dl, 1.f - 1e-4f, true), sq4);
                qlq.push_back(sq4);
            }
            // env: a random direction above the surface (about 18 % of C2's paths)
            if (U(rng) < 0.18f) {
                V3 de = norm(v3(U(rng) * 2 - 1, U(rng) * 2 - 1, U(rng) * 2 - 1));
                if (dot(de, n) < 0) de = mul(de, -1.f);
                trace_bin(s, mkray(X, de, 3.402823466e38f, true, true), &sq, nullptr, &cen[1][b]);
                qe.push_back(sq);
                trace_quad(s, mkray(X, de, 3.402823466e38f, true, true), sq4);
                qeq.push_back(sq4);
            }
        }
        if (getenv("PER_KIND")) {
            auto mean = [](const std::vector<std::string>& v, char c) {
                double n = 0; for (auto& x : v) for (char y : x) n += (c == 'T') == (y == 'T'); return v.empty() ? 0 : n / v.size(); };
            printf("  per kind: cont N %.2f T %.2f | env N %.2f T %.2f | light N %.2f T %.2f\n", mean(qc, 'N'), mean(qc, 'T'),
                   mean(qe, 'N'), mean(qe, 'T'), mean(ql, 'N'), mean(ql, 'T'));
        }
        paths = nextp;
        // the launch's queue: continuation, env, light (WF_KIND_ORDER)
        std::vector<std::string> q, qq;
        for (auto* v : {&qc, &qe, &ql}) q.insert(q.end(), v->begin(), v->end());
        for (auto* v : {&qcq, &qeq, &qlq}) qq.insert(qq.end(), v->begin(), v->end());
        double n = 0, t = 0, g = 0, tq = 0;
        for (auto& x : q) for (char c : x) (c == 'T' ? t : n) += 1;
        for (auto& x : qq) for (char c : x) (c == 'T' ? tq : g) += 1;
        sumN += n; sumT += t; sumG += g; sumTq += tq; nrays += q.size();
        printf("bounce %d: rays %zu (cont %zu env %zu light %zu), node steps %.2f / ray, tri steps %.2f / ray; "
               "grandchild steps %.2f / ray\n", b, q.size(), qc.size(), qe.size(), ql.size(), n / q.size(), t / q.size(),
               g / q.size());
        for (int p = 0; p < NP; ++p) {
            WaveStats w = p == 3 ? simulate(qq, QUAD_UNIFIED, 0, 40)
                                 : simulate(q, p == 0 ? UNIFIED : p == 1 ? PHASED_MAJ : p == 2 ? PHASED_K : SKIP_SPARSE,
                                            p == 2 ? 32 : p >= 4 ? KS[p - 4] : 0, 40);
            for (int k = 0; k < 4; ++k) { all[p].it_kind[k] += w.it_kind[k]; all[p].lanes_kind[k] += w.lanes_kind[k]; }
            all[p].iters += w.iters;
            all[p].lane_steps += w.lane_steps;
        }
    }
    printf("\nall bounces: %.0f rays, %.2f node + %.2f triangle steps per ray (%.1f %% nodes); grandchild: %.2f + %.2f\n",
           nrays, sumN / nrays, sumT / nrays, 100 * sumN / (sumN + sumT), sumG / nrays, sumTq / nrays);
    // pricing: the unified kernel's launch = 0.65 VALU issue + 0.35 the rest, the rest taken
    // as per-iteration latency (one dependent fetch round per wave iteration)
    const double valu_share = 0.65;
    const double baseV = all[0].it_kind[0] * VU, baseI = all[0].iters;
    printf("\n%-30s %10s %8s %8s %8s %10s %9s %9s\n", "organisation", "iters/ray", "lanes/it", "N-it %", "T-it %",
           "VALU/ray", "VALU rel", "time rel");
    for (int p = 0; p < NP; ++p) {
        const WaveStats& w = all[p];
        double V = w.it_kind[0] * VU + w.it_kind[1] * VN + w.it_kind[2] * VT + w.it_kind[3] * VG;
        double rel = valu_share * V / baseV + (1 - valu_share) * w.iters / baseI;
        printf("%-30s %10.3f %8.1f %8.1f %8.1f %10.1f %9.3f %9.3f\n", pname[p].c_str(), w.iters / nrays, w.lane_steps / w.iters,
               100 * w.it_kind[1] / w.iters, 100 * w.it_kind[2] / w.iters, V / nrays, V / baseV, rel);
    }
    printf("\nVALU per iteration kind: unified %.0f, node-only %.0f, triangle-only %.0f, grandchild unified %.0f\n", VU, VN,
           VT, VG);
    // the census: per ray kind and bounce -- node visits and triangle tests per ray, leaves
    // entered and their mean size, triangle tests per accepted triangle (closest hit: every
    // acceptance that shrank tMax; any hit: the occluding one), node-visit depth histogram
    const char* kn[3] = {"cont", "env", "light"};
    printf("\ncensus (flip mode %d): kind bounce | rays | nodes/ray tris/ray | leaves/ray mean-leaf-size | tris/accept | "
           "mean depth | node visits by depth 0-3 4-7 8-11 12-15 16-19 20+ (%%)\n", g_flipmode);
    for (int k = 0; k < 3; ++k)
        for (int b = 0; b < depth; ++b) {
            const Census& c = cen[k][b];
            if (!c.rays) continue;
            printf("  %-5s %d | %7.0f | %5.2f %5.2f | %5.2f %5.2f | %6.2f | %5.1f |", kn[k], b, c.rays, c.nodes / c.rays,
                   c.tris / c.rays, c.leaves / c.rays, c.leaves ? c.leaf_tris / c.leaves : 0, c.accepted ? c.tris / c.accepted : 0,
                   c.nodes ? c.depth_sum / c.nodes : 0);
            for (int d = 0; d < 6; ++d) printf(" %4.1f", c.nodes ? 100 * c.depth_hist[d] / c.nodes : 0);
            printf("\n");
        }
    return 0;
}
