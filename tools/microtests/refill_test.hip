// Micro-test of the persistent-wave refill pattern used by pt_wf_trace.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
template <bool SYNC>
__global__ void __launch_bounds__(256) refill_kernel(unsigned n, const int* steps, int* count, int* out) {
    const int tl = threadIdx.x, lane = tl & 63;
    const unsigned n_waves = gridDim.x * 4;
    const unsigned wave_id = blockIdx.x * 4 + (tl >> 6);
    const unsigned per = (n + n_waves - 1) / n_waves;
    unsigned next = min(wave_id * per, n);
    const unsigned end = min(next + per, n);
    const unsigned long long lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int busy = 0, left = 0;
    unsigned rid = 0;
    for (;;) {
        for (;;) {
            const unsigned long long idle = __ballot(busy == 0);
            if (idle == 0 || next >= end) break;
            const unsigned myid = next + (unsigned)__popcll(idle & lt_mask);
            next = min(next + (unsigned)__popcll(idle), end);
            if (busy == 0 && myid < end && (myid % 7) != 3) { rid = myid; left = steps[myid]; busy = 1; }
        }
        const unsigned long long bm = __ballot(busy != 0);
        if (bm == 0) break;
        const int thr = SYNC ? 0 : __popcll(bm) / 2;
        for (;;) {
            if (busy) {
                if (--left <= 0) { atomicAdd(&count[rid], 1); out[rid] = (int)rid; busy = 0; }
            }
            if (__popcll(__ballot(busy != 0)) <= thr) break;
        }
    }
}
int main() {
    const unsigned n = 1000000;
    std::vector<int> steps(n);
    for (unsigned i = 0; i < n; ++i) steps[i] = 1 + (int)((i * 2654435761u) >> 27);
    int *ds, *dc, *dout;
    hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&dout, n * 4);
    hipMemcpy(ds, steps.data(), n * 4, hipMemcpyHostToDevice);
    for (int sync = 0; sync < 2; ++sync) {
        hipMemset(dc, 0, n * 4); hipMemset(dout, 0xff, n * 4);
        if (sync) hipLaunchKernelGGL(refill_kernel<true>, dim3(2048), dim3(256), 0, 0, n, ds, dc, dout);
        else hipLaunchKernelGGL(refill_kernel<false>, dim3(2048), dim3(256), 0, 0, n, ds, dc, dout);
        hipError_t e = hipDeviceSynchronize();
        std::vector<int> c(n), o(n);
        hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
        hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
        long bad = 0, miss = 0, dup = 0;
        for (unsigned i = 0; i < n; ++i) {
            int want = (i % 7) != 3;
            if (c[i] != want) { bad++; if (c[i] == 0) miss++; else dup++; }
        }
        printf("sync=%d err=%s wrong=%ld missing=%ld duplicated=%ld\n", sync, hipGetErrorString(e), bad, miss, dup);
    }
    return 0;
}
