// tests/abi/c_abi_render.cpp -- a compiled C++ caller of the drop-in boundary
// (TEST INFRASTRUCTURE; built in-tree by pnraytracing_amd/build.py, run by
// tests/test_gpu_c_abi.py).  It includes only include/pnrt.h and
// include/pnrt_host.h, links libpnrt.so + libpnrt_host.so, and performs the
// INTEGRATION.md section 1 sequence that replaces main.cpp's GL hot path:
//   pnrt_create                       (WindowInit's GL context, main.cpp:64-94)
//   pnrt_upload_scene                 (glBufferData/glTexBuffer x5, main.cpp:409-524)
//   pnrt_camera_update                (Camera::UpdateCamera, camera.hpp:11-31)
//   pnrt_set_frame                    (SCREEN_*, camera.*, MAX_BOUNCE_DEPTH, main.cpp:606-611)
//   pnrt_render(frameCount, 1, ...)   (glDispatchCompute + barrier, main.cpp:613-615), per frame
//   pnrt_read_accum                   (the output image, main.cpp:556-559)
//
// usage: c_abi_render <scene.bin> <out.bin> <width> <height> <frames>
// scene.bin: "PNC1", int32 n_vertices, n_materials, n_triangles, n_nodes,
// n_lights, float lights_sum_area, then the five main.cpp-layout float arrays.
#include "pnrt.h"
#include "pnrt_host.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
    if (argc != 6) { fprintf(stderr, "usage: %s scene.bin out.bin width height frames\n", argv[0]); return 2; }
    const int W = atoi(argv[3]), H = atoi(argv[4]), frames = atoi(argv[5]);
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    char magic[4];
    int32_t n[5];
    float sum_area = 0.f;
    if (!rd(f, magic, 4) || memcmp(magic, "PNC1", 4) || !rd(f, n, sizeof n) || !rd(f, &sum_area, 4)) {
        fprintf(stderr, "bad scene file\n");
        return 2;
    }
    const int width[5] = {15, 18, 6, 12, 3};
    std::vector<float> a[5];
    for (int k = 0; k < 5; ++k) {
        a[k].resize((size_t)n[k] * width[k]);
        if (!rd(f, a[k].data(), a[k].size() * 4)) { fprintf(stderr, "short scene file\n"); return 2; }
    }
    fclose(f);

    printf("%s\n", pnrt_version());
    pnrt_ctx* rt = nullptr;
    if (pnrt_create(0, &rt) != PNRT_OK) { fprintf(stderr, "pnrt_create failed: no MI355X\n"); return 3; }

    // an error is a return code + message, never exit(): render before any upload
    if (pnrt_render(rt, 0, 1, 1, 1, 0) == PNRT_OK) { fprintf(stderr, "render without a scene succeeded\n"); return 4; }
    printf("expected error: %s\n", pnrt_last_error(rt));

    int rc = pnrt_upload_scene(rt, a[0].data(), n[0], a[1].data(), n[1], a[2].data(), n[2], a[3].data(), n[3],
                               n[4] ? a[4].data() : nullptr, n[4], sum_area);
    if (rc) { fprintf(stderr, "upload_scene: %s\n", pnrt_last_error(rt)); return 5; }
    if ((rc = pnrt_upload_env(rt, nullptr, nullptr, 0, 0))) {           // HasHDRImage = 0 (C1)
        fprintf(stderr, "upload_env: %s\n", pnrt_last_error(rt));
        return 5;
    }

    // main.cpp:199-202 camera, Camera::UpdateCamera through the host library
    const float eye[3] = {0.f, 2.8f, 7.f}, center[3] = {0.f, 2.8f, 0.f}, up[3] = {0.f, 1.f, 0.f};
    float c12[12];
    if (pnrt_camera_update(eye, center, up, 45.f, (float)W / (float)H, c12)) { fprintf(stderr, "camera\n"); return 6; }
    pnrt_camera cam;
    memcpy(cam.eye, c12, 12);
    memcpy(cam.lower_left, c12 + 3, 12);
    memcpy(cam.horizontal, c12 + 6, 12);
    memcpy(cam.vertical, c12 + 9, 12);
    if ((rc = pnrt_set_frame(rt, W, H, &cam, 4))) { fprintf(stderr, "set_frame: %s\n", pnrt_last_error(rt)); return 7; }

    // the render loop, one frame per "dispatch" as main.cpp:587-628 does it
    for (uint32_t frameCount = 0; frameCount < (uint32_t)frames; ++frameCount)
        if ((rc = pnrt_render(rt, frameCount, 1, 1, 1, 0))) {
            fprintf(stderr, "render: %s\n", pnrt_last_error(rt));
            return 8;
        }
    std::vector<float> rgba((size_t)W * H * 4);
    if ((rc = pnrt_read_accum(rt, rgba.data()))) { fprintf(stderr, "read_accum: %s\n", pnrt_last_error(rt)); return 9; }
    pnrt_destroy(rt);

    FILE* o = fopen(argv[2], "wb");
    if (!o || fwrite(rgba.data(), 4, rgba.size(), o) != rgba.size()) { perror(argv[2]); return 10; }
    fclose(o);
    printf("rendered %dx%d x %d frames through the C ABI\n", W, H, frames);
    return 0;
}
