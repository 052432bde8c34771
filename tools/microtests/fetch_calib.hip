// Calibration of rocprofv3's FETCH_SIZE for the trace kernel's access shape
// (VERDICT r2, item 3c).  MI355X_MICROARCH.md calibrates FETCH_SIZE = 1/2 of the
// bytes for wide coalesced streaming reads only; the trace kernel gathers 64-B
// node records (one half of a 128-B line) and 48-B triangle records at random.
//
// A 1 GiB table (4x the 256 MiB Infinity Cache, filled first) is read once per
// kernel with a KNOWN byte count, one dispatch per pattern:
//   0 stream    16 B per lane, coalesced: every byte of the table once
//   1 gather64  every 64-B record once, in a scattered (odd-multiplier) order:
//               both halves of each 128-B line, at unrelated times
//   2 half64    one 64-B record per 128-B line (the even ones), scattered:
//               the bytes used are half the lines touched
//   3 line128   every 128-B line once (eight 16-B loads per lane), scattered
// The loads of a lane are independent (no chain): each kernel is bandwidth-bound,
// so its time tells bytes moved as well as the counters do.  tools/fetch_calib.py
// runs it under rocprofv3 --pmc (FETCH_SIZE; TCC_EA0_RDREQ) and writes the ratio
// known bytes / FETCH_SIZE bytes per pattern to profiles/r03/fetch_calibration.json.
//   hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
//   ./fetch_calib [log2_table_bytes=30]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u4 ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
}

// item i of n (a power of two) -> a scattered item: odd multiplier mod n is a bijection
__device__ __forceinline__ uint32_t scatter(uint32_t i, uint32_t n) { return (i * 0x9E3779B1u + 0x7F4A7C15u) & (n - 1u); }

template <int MODE>
__global__ void __launch_bounds__(256) calib(const void* tab, uint32_t bytes, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, (int)bytes, 0x00020000);
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    uint32_t acc = 0;
    if (MODE == 0) {
        for (uint32_t o = tid * 16u; o < bytes; o += nth * 16u) { const u4 v = ld16(rs, o); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    } else if (MODE == 1) {
        const uint32_t n = bytes / 64u;
        for (uint32_t i = tid; i < n; i += nth) {
            const uint32_t o = scatter(i, n) * 64u;
            const u4 a = ld16(rs, o), b = ld16(rs, o + 16u), c = ld16(rs, o + 32u), d = ld16(rs, o + 48u);
            acc ^= a.x ^ b.y ^ c.z ^ d.w;
        }
    } else if (MODE == 2) {
        const uint32_t n = bytes / 128u;
        for (uint32_t i = tid; i < n; i += nth) {
            const uint32_t o = scatter(i, n) * 128u;
            const u4 a = ld16(rs, o), b = ld16(rs, o + 16u), c = ld16(rs, o + 32u), d = ld16(rs, o + 48u);
            acc ^= a.x ^ b.y ^ c.z ^ d.w;
        }
    } else {
        const uint32_t n = bytes / 128u;
        for (uint32_t i = tid; i < n; i += nth) {
            const uint32_t o = scatter(i, n) * 128u;
#pragma unroll
            for (int k = 0; k < 8; ++k) { const u4 v = ld16(rs, o + 16u * k); acc ^= v.x ^ v.w; }
        }
    }
    if (acc == 0x12345678u) out[tid] = acc;     // keeps the loads; practically never stores
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;                  // 1 GiB: 4x the Infinity Cache
    if (lg < 20 || lg > 30) { printf("log2 bytes in [20, 30]\n"); return 2; }
    const uint32_t cover = 1u << lg;                                 // a power of two: the scatter is a bijection
    void* tab = nullptr;
    uint32_t* out = nullptr;
    CHK(hipMalloc(&tab, cover));
    CHK(hipMalloc(&out, 64u << 20));
    CHK(hipMemset(tab, 0x5a, cover));
    CHK(hipDeviceSynchronize());
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const dim3 grid(cus * 16), blk(256);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    const char* names[4] = {"stream", "gather64", "half64", "line128"};
    for (int m = 0; m < 4; ++m) {
        const double known = m == 2 ? cover / 2.0 : (double)cover;   // bytes the loads return
        CHK(hipEventRecord(a));
        switch (m) {
        case 0: hipLaunchKernelGGL(calib<0>, grid, blk, 0, 0, tab, cover, out); break;
        case 1: hipLaunchKernelGGL(calib<1>, grid, blk, 0, 0, tab, cover, out); break;
        case 2: hipLaunchKernelGGL(calib<2>, grid, blk, 0, 0, tab, cover, out); break;
        default: hipLaunchKernelGGL(calib<3>, grid, blk, 0, 0, tab, cover, out); break;
        }
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0.f;
        CHK(hipEventElapsedTime(&ms, a, b));
        printf("{\"pattern\": \"%s\", \"dispatch\": %d, \"known_bytes\": %.0f, \"lines_touched_bytes\": %u, "
               "\"ms\": %.4f, \"known_GBps\": %.1f}\n", names[m], m, known, cover, ms, known / (ms * 1e-3) / 1e9);
    }
    CHK(hipFree(tab)); CHK(hipFree(out));
    return 0;
}
