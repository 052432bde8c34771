// tests/abi/c_abi_dloop.cpp -- the reference's render loop (main.cpp:573-630: one
// glDispatchCompute per frame, frameCount++) driven through the C ABI alone, no
// Python: pnrt_render(frameCount, 1) per frame, either synchronised after every
// frame (pnrt_synchronize: the loop that displays each frame) or pipelined (one
// wait at the end).  TEST INFRASTRUCTURE and a measurement tool: built in-tree by
// pnraytracing_amd/build.py, checked against the oracle by tests/test_gpu_c_abi.py,
// timed by tools/dloop.py.
//
// usage: c_abi_dloop <scene.bin> <frames> <warmup> <sync|pipe> [out.bin]
// scene.bin ("PND1", written by tools/dloop.py export_scene): int32 n_vertices,
// n_materials, n_triangles, n_nodes, n_lights; float lights_sum_area; int32 width,
// height, max_depth, env_w, env_h, n_textures; float camera[12]; the five
// main.cpp-layout float arrays; env rgb + RandomHDR table (env_h x env_w x 3 floats
// each) if env_w > 0; per texture int32 w, h, ch and w * h * ch bytes.
// Prints one line: frames, mode, ms per frame (std::chrono around the timed frames).
#include "pnrt.h"

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "usage: %s scene.bin frames warmup sync|pipe [out.bin]\n", argv[0]); return 2; }
    const int frames = atoi(argv[2]), warmup = atoi(argv[3]);
    const bool sync = strcmp(argv[4], "sync") == 0;
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    char magic[4];
    int32_t n[5], fr[6];
    float sum_area = 0.f, cam12[12];
    if (!rd(f, magic, 4) || memcmp(magic, "PND1", 4) || !rd(f, n, sizeof n) || !rd(f, &sum_area, 4) ||
        !rd(f, fr, sizeof fr) || !rd(f, cam12, sizeof cam12)) {
        fprintf(stderr, "bad scene file\n");
        return 2;
    }
    const int W = fr[0], H = fr[1], depth = fr[2], ew = fr[3], eh = fr[4], ntex = fr[5];
    const int width[5] = {15, 18, 6, 12, 3};
    std::vector<float> a[5];
    for (int k = 0; k < 5; ++k) {
        a[k].resize((size_t)n[k] * width[k]);
        if (!rd(f, a[k].data(), a[k].size() * 4)) { fprintf(stderr, "short scene file\n"); return 2; }
    }
    std::vector<float> env, table;
    if (ew > 0) {
        env.resize((size_t)ew * eh * 3);
        table.resize(env.size());
        if (!rd(f, env.data(), env.size() * 4) || !rd(f, table.data(), table.size() * 4)) { fprintf(stderr, "short env\n"); return 2; }
    }
    pnrt_ctx* rt = nullptr;
    if (pnrt_create(0, &rt) != PNRT_OK) { fprintf(stderr, "pnrt_create failed: no MI355X\n"); return 3; }
    int rc = pnrt_upload_scene(rt, a[0].data(), n[0], a[1].data(), n[1], a[2].data(), n[2], a[3].data(), n[3],
                               n[4] ? a[4].data() : nullptr, n[4], sum_area);
    for (int t = 0; rc == PNRT_OK && t < ntex; ++t) {
        int32_t th[3];
        if (!rd(f, th, sizeof th)) { fprintf(stderr, "short texture\n"); return 2; }
        std::vector<uint8_t> px((size_t)th[0] * th[1] * th[2]);
        if (!rd(f, px.data(), px.size())) { fprintf(stderr, "short texture\n"); return 2; }
        rc = pnrt_upload_texture(rt, t, px.data(), th[0], th[1], th[2]);
    }
    fclose(f);
    if (rc == PNRT_OK) rc = pnrt_upload_env(rt, ew ? env.data() : nullptr, ew ? table.data() : nullptr, ew, eh);
    pnrt_camera cam;
    memcpy(cam.eye, cam12, 12);
    memcpy(cam.lower_left, cam12 + 3, 12);
    memcpy(cam.horizontal, cam12 + 6, 12);
    memcpy(cam.vertical, cam12 + 9, 12);
    if (rc == PNRT_OK) rc = pnrt_set_frame(rt, W, H, &cam, depth);
    if (rc != PNRT_OK) { fprintf(stderr, "setup: %s\n", pnrt_last_error(rt)); return 5; }

    // main.cpp:587-628: one dispatch per frame, frameCount++; warm-up frames first
    double t_render = 0.0, t_sync = 0.0;     // host time inside pnrt_render / pnrt_synchronize (timed frames)
    bool timed = false;
    auto frame = [&](uint32_t k) -> int {
        const auto a = std::chrono::steady_clock::now();
        int r = pnrt_render(rt, k, 1, 1, 1, 0);
        const auto m = std::chrono::steady_clock::now();
        if (r == PNRT_OK && sync) r = pnrt_synchronize(rt);
        const auto z = std::chrono::steady_clock::now();
        if (timed) {
            t_render += std::chrono::duration<double, std::micro>(m - a).count();
            t_sync += std::chrono::duration<double, std::micro>(z - m).count();
        }
        return r;
    };
    for (int k = 0; k < warmup && rc == PNRT_OK; ++k) rc = frame((uint32_t)k);
    if (rc == PNRT_OK) rc = pnrt_synchronize(rt);
    timed = true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = warmup; k < warmup + frames && rc == PNRT_OK; ++k) rc = frame((uint32_t)k);
    if (rc == PNRT_OK) rc = pnrt_synchronize(rt);
    const auto t1 = std::chrono::steady_clock::now();
    if (rc != PNRT_OK) { fprintf(stderr, "render: %s\n", pnrt_last_error(rt)); return 8; }
    const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    printf("frames %d mode %s ms_per_frame %.4f width %d height %d host_render_us %.1f host_sync_us %.1f\n", frames,
           sync ? "sync" : "pipe", ms / frames, W, H, t_render / frames, t_sync / frames);
    if (argc > 5) {
        std::vector<float> rgba((size_t)W * H * 4);
        if ((rc = pnrt_read_accum(rt, rgba.data()))) { fprintf(stderr, "read_accum: %s\n", pnrt_last_error(rt)); return 9; }
        FILE* o = fopen(argv[5], "wb");
        if (!o || fwrite(rgba.data(), 4, rgba.size(), o) != rgba.size()) { perror(argv[5]); return 10; }
        fclose(o);
    }
    pnrt_destroy(rt);
    return 0;
}
