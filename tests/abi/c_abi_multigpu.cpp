// tests/abi/c_abi_multigpu.cpp -- a compiled C++ multi-GPU caller of the drop-in
// boundary (TEST INFRASTRUCTURE and the reference integration for INTEGRATION.md
// section 4; built in-tree by pnraytracing_amd/build.py, run by
// tests/test_gpu_c_abi.py).  SURVEY 8e's process model: ONE process drives every
// visible device, no torch, no Python:
//
//   ncclCommInitAll(comms, ndev, {0..ndev-1})          one RCCL communicator per device
//   per shard r of N (device r % ndev, its own pnrt context on that device's stream):
//     pnrt_upload_scene / pnrt_set_frame               the same arrays on every device
//     pnrt_render(ctx, f, n, 8, N, r)                  rows y with (y / 8) % N == r
//     pnrt_pack_rows(ctx, send + slot, 8, N, r)        contiguous rows, padded to max_rows
//   ncclGroupStart; ncclGather(send_d -> recv on device 0) per device; ncclGroupEnd
//   pnrt_unpack_rows(ctx[0], recv + slot of shard r, image, 8, N, r)   every shard's rows into one image
//   device 0: rows scattered back into image order
//
// and checks the gathered image against one single-context render of the whole
// frame, bit for bit.  With fewer devices than shards (the one-GPU test box)
// several shard contexts share a device and its stream; the collective is the
// same call.
//
// usage: c_abi_multigpu <scene.bin> <out.bin> <width> <height> <frames> <n_shards>
// scene.bin: the c_abi_render format ("PNC1", counts, lights_sum_area, arrays).
#include "pnrt.h"
#include "pnrt_host.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(what, expr)                                                                           \
    do {                                                                                         \
        if ((expr) != 0) { fprintf(stderr, "%s failed\n", what); return 20; }                   \
    } while (0)
#define HIPCK(expr)                                                                              \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #expr, hipGetErrorString(e_)); return 21; } \
    } while (0)
#define NCCLCK(expr)                                                                             \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) { fprintf(stderr, "%s: %s\n", #expr, ncclGetErrorString(r_)); return 22; } \
    } while (0)

static const int BAND = 8;

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }
static int shard_rows(int h, int n, int r) {
    int rows = 0;
    for (int y0 = r * BAND; y0 < h; y0 += BAND * n) rows += (h - y0 < BAND) ? h - y0 : BAND;
    return rows;
}

struct Scene {
    int32_t n[5];
    float sum_area;
    std::vector<float> a[5];
};

static int setup(pnrt_ctx* rt, const Scene& s, int W, int H) {
    int rc = pnrt_upload_scene(rt, s.a[0].data(), s.n[0], s.a[1].data(), s.n[1], s.a[2].data(), s.n[2], s.a[3].data(),
                               s.n[3], s.n[4] ? s.a[4].data() : nullptr, s.n[4], s.sum_area);
    if (rc == PNRT_OK) rc = pnrt_upload_env(rt, nullptr, nullptr, 0, 0);
    const float eye[3] = {0.f, 2.8f, 7.f}, center[3] = {0.f, 2.8f, 0.f}, up[3] = {0.f, 1.f, 0.f};   // main.cpp:199-202
    float c12[12];
    if (rc == PNRT_OK && pnrt_camera_update(eye, center, up, 45.f, (float)W / (float)H, c12)) return -100;
    pnrt_camera cam;
    memcpy(cam.eye, c12, 12); memcpy(cam.lower_left, c12 + 3, 12);
    memcpy(cam.horizontal, c12 + 6, 12); memcpy(cam.vertical, c12 + 9, 12);
    if (rc == PNRT_OK) rc = pnrt_set_frame(rt, W, H, &cam, 4);
    if (rc) fprintf(stderr, "setup: %s\n", pnrt_last_error(rt));
    return rc;
}

int main(int argc, char** argv) {
    if (argc != 7) { fprintf(stderr, "usage: %s scene.bin out.bin width height frames n_shards\n", argv[0]); return 2; }
    const int W = atoi(argv[3]), H = atoi(argv[4]), frames = atoi(argv[5]), N = atoi(argv[6]);
    if (W <= 0 || H <= 0 || frames <= 0 || N <= 0) return 2;
    Scene s;
    FILE* f = fopen(argv[1], "rb");
    char magic[4];
    if (!f || !rd(f, magic, 4) || memcmp(magic, "PNC1", 4) || !rd(f, s.n, sizeof s.n) || !rd(f, &s.sum_area, 4)) {
        fprintf(stderr, "bad scene file\n");
        return 2;
    }
    const int width[5] = {15, 18, 6, 12, 3};
    for (int k = 0; k < 5; ++k) {
        s.a[k].resize((size_t)s.n[k] * width[k]);
        if (!rd(f, s.a[k].data(), s.a[k].size() * 4)) { fprintf(stderr, "short scene file\n"); return 2; }
    }
    fclose(f);

    int ndev = 0;
    HIPCK(hipGetDeviceCount(&ndev));
    if (ndev <= 0) { fprintf(stderr, "no device\n"); return 3; }
    if (ndev > N) ndev = N;                       // one device per shard at most
    printf("%s\n%d shard(s) over %d device(s)\n", pnrt_version(), N, ndev);

    // one RCCL communicator per device, one stream per device shared by its shard contexts
    std::vector<int> devs(ndev);
    for (int d = 0; d < ndev; ++d) devs[d] = d;
    std::vector<ncclComm_t> comms(ndev);
    NCCLCK(ncclCommInitAll(comms.data(), ndev, devs.data()));
    std::vector<hipStream_t> stream(ndev);
    for (int d = 0; d < ndev; ++d) { HIPCK(hipSetDevice(d)); HIPCK(hipStreamCreateWithFlags(&stream[d], hipStreamNonBlocking)); }

    // shard r lives on device r % ndev, at slot r / ndev of that device's send buffer
    int max_rows = 0;
    for (int r = 0; r < N; ++r) max_rows = shard_rows(H, N, r) > max_rows ? shard_rows(H, N, r) : max_rows;
    const int per_dev = (N + ndev - 1) / ndev;                    // slots per device (the last may be padding)
    const size_t slot = (size_t)max_rows * W * 4;                 // floats per shard slot
    std::vector<pnrt_ctx*> ctx(N, nullptr);
    std::vector<float*> send(ndev, nullptr);
    float* recv = nullptr;
    for (int d = 0; d < ndev; ++d) {
        HIPCK(hipSetDevice(d));
        HIPCK(hipMalloc(&send[d], slot * per_dev * sizeof(float)));
        HIPCK(hipMemsetAsync(send[d], 0, slot * per_dev * sizeof(float), stream[d]));
    }
    HIPCK(hipSetDevice(0));
    HIPCK(hipMalloc(&recv, slot * per_dev * ndev * sizeof(float)));
    for (int r = 0; r < N; ++r) {
        const int d = r % ndev;
        if (pnrt_create(d, &ctx[r]) != PNRT_OK) { fprintf(stderr, "pnrt_create(%d) failed\n", d); return 4; }
        CK("set_stream", pnrt_set_stream(ctx[r], stream[d]));    // blends, packs and the gather in one order
        if (setup(ctx[r], s, W, H)) return 5;
    }
    // render: batches of <= 16 frames per call (one batch each), every shard
    for (int f0 = 0; f0 < frames; f0 += 16) {
        const int nf = frames - f0 < 16 ? frames - f0 : 16;
        for (int r = 0; r < N; ++r)
            if (pnrt_render(ctx[r], (uint32_t)f0, (uint32_t)nf, BAND, N, r)) {
                fprintf(stderr, "render shard %d: %s\n", r, pnrt_last_error(ctx[r]));
                return 6;
            }
    }
    for (int r = 0; r < N; ++r)
        if (pnrt_pack_rows(ctx[r], send[r % ndev] + slot * (r / ndev), BAND, N, r)) {
            fprintf(stderr, "pack_rows shard %d: %s\n", r, pnrt_last_error(ctx[r]));
            return 7;
        }
    // one gather of every device's slots to device 0 (rank order = device order)
    NCCLCK(ncclGroupStart());
    for (int d = 0; d < ndev; ++d)
        NCCLCK(ncclGather(send[d], d == 0 ? recv : nullptr, slot * per_dev, ncclFloat, 0, comms[d], stream[d]));
    NCCLCK(ncclGroupEnd());
    for (int d = 0; d < ndev; ++d) { HIPCK(hipSetDevice(d)); HIPCK(hipStreamSynchronize(stream[d])); }
    for (int r = 0; r < N; ++r)
        if (pnrt_synchronize(ctx[r])) { fprintf(stderr, "shard %d: %s\n", r, pnrt_last_error(ctx[r])); return 8; }

    // device 0: de-interleave (recv = device-major, slot-minor: shard r at d * per_dev + r / ndev)
    // into a device image with the library's pnrt_unpack_rows, on shard 0's context (device 0)
    std::vector<float> img((size_t)W * H * 4, 0.f);
    HIPCK(hipSetDevice(0));
    float* dimg = nullptr;
    HIPCK(hipMalloc(&dimg, img.size() * sizeof(float)));
    HIPCK(hipMemset(dimg, 0, img.size() * sizeof(float)));
    for (int r = 0; r < N; ++r)
        CK("unpack_rows", pnrt_unpack_rows(ctx[0], recv + slot * ((size_t)(r % ndev) * per_dev + r / ndev), dimg, BAND,
                                           N, r));
    CK("synchronize (unpack)", pnrt_synchronize(ctx[0]));
    HIPCK(hipMemcpy(img.data(), dimg, img.size() * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(dimg);

    // the single-context render of the whole frame
    pnrt_ctx* one = nullptr;
    if (pnrt_create(0, &one) != PNRT_OK || setup(one, s, W, H)) return 9;
    for (int f0 = 0; f0 < frames; f0 += 16)
        CK("render (single)", pnrt_render(one, (uint32_t)f0, (uint32_t)(frames - f0 < 16 ? frames - f0 : 16), 1, 1, 0));
    std::vector<float> ref((size_t)W * H * 4);
    CK("read_accum (single)", pnrt_read_accum(one, ref.data()));
    size_t bad = 0;
    for (size_t i = 0; i < ref.size(); ++i) bad += memcmp(&ref[i], &img[i], 4) != 0;

    FILE* o = fopen(argv[2], "wb");
    if (!o || fwrite(img.data(), 4, img.size(), o) != img.size()) { perror(argv[2]); return 10; }
    fclose(o);
    pnrt_destroy(one);
    for (pnrt_ctx* c : ctx) pnrt_destroy(c);
    for (int d = 0; d < ndev; ++d) {
        (void)hipSetDevice(d);
        (void)hipFree(send[d]);
        (void)hipStreamDestroy(stream[d]);
        ncclCommDestroy(comms[d]);
    }
    (void)hipSetDevice(0);
    (void)hipFree(recv);
    if (bad) { fprintf(stderr, "%zu floats differ from the single-context render\n", bad); return 11; }
    printf("gathered %dx%d x %d frames from %d shards over %d device(s): bit-identical to the single-context render\n",
           W, H, frames, N, ndev);
    return 0;
}
