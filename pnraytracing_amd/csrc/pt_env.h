// pnraytracing_amd/csrc/pt_env.h -- LoadHDRImage's importance-sampling table
// (shader.hpp:145-203) built on the GPU, bit-identical to the host restatement
// (csrc/host/pnrt_host.cpp pnrt_hdr_build_table).
//
// Every floating-point sum keeps the reference's order, so the parallelism is
// only where the reference's loops are independent:
//   lumen        per pixel, double arithmetic rounded to float (:152)
//   pdfSum       ONE chain over x-major order (:148-155): a single wave walks
//                the x-major copy 64 values at a time and folds them in lane
//                order through v_readlane -- serial by definition
//   pdfMarginX   per column x, over y in order (:161-166)
//   cdfMarginX   one chain over x (:167-170)
//   cdfYCondX    per column x, over y, in double then rounded (:172-179)
//   table        per texel: two lower_bounds (:184-200)
#pragma once
#include "pt_common.h"

// lumY[y * w + x] (row-major, coalesced for the per-column passes) and
// lumX[x * h + y] (x-major, the order of the pdfSum chain).
__global__ void __launch_bounds__(256) env_lumen_kernel(const float4* hdr, float* lumY, float* lumX, int w, int h) {
    const size_t pos = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= (size_t)w * h) return;
    const int y = (int)(pos / (size_t)w), x = (int)(pos - (size_t)y * w);
    const float4 c = hdr[pos];
    const float l = (float)(((double)c.x * 0.2 + (double)c.y * 0.7) + (double)c.z * 0.1);
    lumY[pos] = l;
    lumX[(size_t)x * h + y] = l;
}

// pdfSum: the reference's float accumulation, in its order, by one wave.
__global__ void __launch_bounds__(64) env_sum_kernel(const float* lumX, size_t n, float* out) {
    const int lane = threadIdx.x;
    float acc = 0.0f;                       // identical on every lane (readlane is uniform)
    for (size_t base = 0; base < n; base += 64) {
        const float v = base + lane < n ? lumX[base + lane] : 0.0f;
        const int vi = __float_as_int(v);
        if (base + 64 <= n) {
#pragma unroll
            for (int k = 0; k < 64; ++k) acc = acc + __int_as_float(__builtin_amdgcn_readlane(vi, k));
        } else {
            for (int k = 0; (size_t)k < n - base; ++k) acc = acc + __int_as_float(__builtin_amdgcn_readlane(vi, k));
        }
    }
    if (lane == 0) *out = acc;
}

// pdf /= pdfSum and pdfMarginX[x] += pdf, per column, y in order.
__global__ void __launch_bounds__(256) env_margin_kernel(float* pdfY, const float* sum, float* marginX, int w, int h) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= w) return;
    const float s = *sum;
    float m = 0.0f;
    for (int y = 0; y < h; ++y) {
        const size_t pos = (size_t)y * w + x;
        const float p = pdfY[pos] / s;
        pdfY[pos] = p;
        m = m + p;
    }
    marginX[x] = m;
}

// cdfMarginX: one chain over x.
__global__ void env_cdfx_kernel(const float* marginX, float* cdfX, int w) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    float c = marginX[0];
    cdfX[0] = c;
    for (int x = 1; x < w; ++x) { c = c + marginX[x]; cdfX[x] = c; }
}

// cdfYConditionX[x][y] = (y > 0 ? cdf[y-1] : 0.0) + pdf[x][y] / pdfMarginX[x]: the
// conditional operator's double type makes the add double, rounded to float.
__global__ void __launch_bounds__(256) env_cdfy_kernel(const float* pdfY, const float* marginX, float* cdfY, int w, int h) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= w) return;
    const float m = marginX[x];
    float c = 0.0f;
    for (int y = 0; y < h; ++y) {
        const size_t pos = (size_t)y * w + x;
        c = (float)((y > 0 ? (double)c : 0.0) + (double)(pdfY[pos] / m));
        cdfY[pos] = c;
    }
}

// std::lower_bound: first index in [0, n) whose value is not less than v (n if none).
PN_DEV int lower_bound_strided(const float* a, int n, size_t stride, float v) {
    int lo = 0, cnt = n;
    while (cnt > 0) {
        const int step = cnt / 2, mid = lo + step;
        if (a[(size_t)mid * stride] < v) { lo = mid + 1; cnt -= step + 1; }
        else cnt = step;
    }
    return lo;
}

// RandomHDR texel (i, j) -> (x / w, y / h, pdf[x][y]) (:184-200).
__global__ void __launch_bounds__(256) env_table_kernel(const float* cdfX, const float* cdfY, const float* pdfY,
                                                        float4* table, int w, int h) {
    const size_t pos = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= (size_t)w * h) return;
    const int j = (int)(pos / (size_t)w), i = (int)(pos - (size_t)j * w);
    int x = lower_bound_strided(cdfX, w, 1, (float)i / (float)w);
    if (x >= w) x = w - 1;
    if (x < 0) x = 0;
    int y = lower_bound_strided(cdfY + x, h, (size_t)w, (float)j / (float)h);
    if (y >= h) y = h - 1;
    if (y < 0) y = 0;
    table[pos] = make_float4((float)x / (float)w, (float)y / (float)h, pdfY[(size_t)y * w + x], 0.0f);
}
