// Microbenchmark: dependent 64-B record gathers, the trace kernel's fetch shape.
//
// Mode 0 ("lane"): each lane fetches its own 64-B record with four 16-B buffer
//   loads (four instructions, each touching one line per lane).
// Mode 1 ("quad"): the four lanes of a quad fetch one record per instruction
//   (lane 4q+c loads quarter c of the record of lane 4q+k in instruction k), so
//   each instruction touches one line per quad; a 4x4 in-quad transpose (two
//   DPP butterfly stages, one v_cndmask with a DPP operand per dword) hands
//   every lane its own 64 B.
// The next record index depends on the loaded bytes (a chain, like traversal);
// PAD dependent VALU ops per step emulate the step's arithmetic.
//   hipcc --offload-arch=gfx950 -O3 gather_test.hip -o gather_test
//   ./gather_test <nrec> <hot_recs> <hot_pct> <pad> <iters>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u4 ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
}
template <int PERM>
__device__ __forceinline__ uint32_t qp(uint32_t v) {   // quad_perm DPP move
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, PERM, 0xf, 0xf, true);
}
#define QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))
// One butterfly stage of the in-quad transpose on one dword of four blocks:
// o[k] = (lane in the mask of k) ? in[k] : in[k ^ x] of the quad partner lane ^ x,
// as v_cndmask with a DPP operand (executed by every lane: a DPP read from a lane
// the compiler had predicated off would return 0).  s_nop 1 covers the
// VALU-write -> DPP-read hazard of the previous stage's results.
#define STAGE(NAME, PERM)                                                                                   \
    __device__ __forceinline__ void NAME(uint32_t i0, uint32_t i1, uint32_t i2, uint32_t i3, uint64_t mkeep02, \
                                         uint64_t mkeep13, uint32_t& o0, uint32_t& o1, uint32_t& o2, uint32_t& o3) { \
        asm("s_mov_b64 vcc, %8\n\ts_nop 1\n\t"                                                           \
            "v_cndmask_b32_dpp %0, %5, %4, vcc quad_perm:" PERM " row_mask:0xf bank_mask:0xf\n\t"          \
            "v_cndmask_b32_dpp %2, %7, %6, vcc quad_perm:" PERM " row_mask:0xf bank_mask:0xf\n\t"          \
            "s_mov_b64 vcc, %9\n\t"                                                                        \
            "v_cndmask_b32_dpp %1, %4, %5, vcc quad_perm:" PERM " row_mask:0xf bank_mask:0xf\n\t"          \
            "v_cndmask_b32_dpp %3, %6, %7, vcc quad_perm:" PERM " row_mask:0xf bank_mask:0xf"               \
            : "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3)                                                   \
            : "v"(i0), "v"(i1), "v"(i2), "v"(i3), "s"(mkeep02), "s"(mkeep13)                               \
            : "vcc");                                                                                       \
    }
#define M_EVEN 0x5555555555555555ull
#define M_ODD 0xAAAAAAAAAAAAAAAAull
#define M_LO2 0x3333333333333333ull
#define M_HI2 0xCCCCCCCCCCCCCCCCull
// stage x1 pairs blocks (0,1), (2,3): i0, i1, i2, i3 = blocks 0, 1, 2, 3
STAGE(stage_x1, "[1,0,3,2]")
// stage x2 pairs blocks (0,2), (1,3): called with (b0, b2, b1, b3)
STAGE(stage_x2, "[2,3,0,1]")
// 4x4 in-quad transpose of 16-B blocks: a[k] = quarter (lane & 3) of the record of
// quad lane k  ->  w[4 b + j] = dword j of quarter b of this lane's record
__device__ __forceinline__ void quad_transpose(const uint32_t (&a)[4][4], uint32_t* w) {
    uint32_t b1[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)   // B1[l][b] = ((l^b)&1) ? A[l^1][b^1] : A[l][b]
        stage_x1(a[0][j], a[1][j], a[2][j], a[3][j], M_EVEN, M_ODD, b1[0][j], b1[1][j], b1[2][j], b1[3][j]);
#pragma unroll
    for (int j = 0; j < 4; ++j)   // B2[l][b] = ((l^b)&2) ? B1[l^2][b^2] : B1[l][b]
        stage_x2(b1[0][j], b1[2][j], b1[1][j], b1[3][j], M_LO2, M_HI2, w[0 * 4 + j], w[2 * 4 + j], w[1 * 4 + j],
                 w[3 * 4 + j]);
}

__device__ __forceinline__ uint32_t next_index(const uint32_t* w, uint32_t nrec, uint32_t hot, uint32_t hot_pct,
                                               uint32_t lanesalt) {
    uint32_t h = lanesalt;
#pragma unroll
    for (int k = 0; k < 16; ++k) h = (h ^ w[k]) * 0x9E3779B1u;
    h ^= h >> 15;
    return ((h & 127u) * 100u < hot_pct * 128u) ? (h >> 7) % hot : (h >> 7) % nrec;
}

template <int MODE, int PAD>
__global__ void __launch_bounds__(256, 8) gather_kernel(const uint32_t* table, uint32_t nrec, uint32_t hot,
                                                        uint32_t hot_pct, int iters, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)table, (short)0, (int)(nrec * 64u), 0x00020000);
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, c = lane & 3u;
    __shared__ __attribute__((aligned(16))) uint32_t stage[MODE == 3 ? 4 * 1024 : 4];
    uint32_t r = (gid * 2654435761u) % nrec;
    uint32_t acc = 0;
    float f = (float)(gid & 7);
    for (int it = 0; it < iters; ++it) {
        uint32_t w[16];
        if constexpr (MODE == 0) {
            const uint32_t off = r * 64u;
            const u4 a = ld16(rs, off), b = ld16(rs, off + 16u), cc = ld16(rs, off + 32u), d = ld16(rs, off + 48u);
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
            w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
            w[8] = cc.x; w[9] = cc.y; w[10] = cc.z; w[11] = cc.w;
            w[12] = d.x; w[13] = d.y; w[14] = d.z; w[15] = d.w;
        } else if constexpr (MODE == 3) {
            // quad fetch through LDS: in instruction k the lanes of quad q DMA the four
            // quarters of quad lane k's record into this wave's 4-KB stage (lane L of
            // instruction k lands at k * 1 KB + 16 L: lane 4q + c carries quarter
            // (c - k) & 3, so the reads below are bank-conflict free); then every lane
            // reads its own 64 B with four ds_read_b128
            uint32_t* st = stage + (threadIdx.x >> 6) * 1024u;
            const uint32_t kk = c;   // this lane is quad lane k = c for its own record
            const uint32_t o0 = qp<QP(0, 0, 0, 0)>(r) * 64u, o1 = qp<QP(1, 1, 1, 1)>(r) * 64u,
                           o2 = qp<QP(2, 2, 2, 2)>(r) * 64u, o3 = qp<QP(3, 3, 3, 3)>(r) * 64u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(st + 0 * 256), 16,
                                                     o0 + 16u * ((c - 0u) & 3u), 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(st + 1 * 256), 16,
                                                     o1 + 16u * ((c - 1u) & 3u), 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(st + 2 * 256), 16,
                                                     o2 + 16u * ((c - 2u) & 3u), 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(st + 3 * 256), 16,
                                                     o3 + 16u * ((c - 3u) & 3u), 0, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t q4 = (lane >> 2) * 4u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u4 v = *reinterpret_cast<const u4*>(st + kk * 256u + (q4 + ((j + kk) & 3u)) * 4u);
                w[4 * j + 0] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
            }
        } else if constexpr (MODE == 2) {   // quad loads, no transpose (load side only; wrong words)
            const uint32_t r0 = qp<QP(0, 0, 0, 0)>(r), r1 = qp<QP(1, 1, 1, 1)>(r), r2 = qp<QP(2, 2, 2, 2)>(r),
                           r3 = qp<QP(3, 3, 3, 3)>(r);
            const u4 A0 = ld16(rs, r0 * 64u + c * 16u), A1 = ld16(rs, r1 * 64u + c * 16u),
                     A2 = ld16(rs, r2 * 64u + c * 16u), A3 = ld16(rs, r3 * 64u + c * 16u);
            w[0] = A0.x; w[1] = A0.y; w[2] = A0.z; w[3] = A0.w;
            w[4] = A1.x; w[5] = A1.y; w[6] = A1.z; w[7] = A1.w;
            w[8] = A2.x; w[9] = A2.y; w[10] = A2.z; w[11] = A2.w;
            w[12] = A3.x; w[13] = A3.y; w[14] = A3.z; w[15] = A3.w;
        } else {
            // instruction k: this lane loads quarter c of the record of lane 4q + k
            const uint32_t r0 = qp<QP(0, 0, 0, 0)>(r), r1 = qp<QP(1, 1, 1, 1)>(r), r2 = qp<QP(2, 2, 2, 2)>(r),
                           r3 = qp<QP(3, 3, 3, 3)>(r);
            const u4 A0 = ld16(rs, r0 * 64u + c * 16u), A1 = ld16(rs, r1 * 64u + c * 16u),
                     A2 = ld16(rs, r2 * 64u + c * 16u), A3 = ld16(rs, r3 * 64u + c * 16u);
            // A[l][b] = quarter l of record b; want B[l][b] = A[b][l] (lane l = own record, block b = quarter)
            uint32_t a[4][4] = {{A0.x, A0.y, A0.z, A0.w}, {A1.x, A1.y, A1.z, A1.w},
                                {A2.x, A2.y, A2.z, A2.w}, {A3.x, A3.y, A3.z, A3.w}};
            quad_transpose(a, w);
        }
#pragma unroll
        for (int q = 0; q < PAD; ++q) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(f));
        acc += w[0] + w[15];
        r = next_index(w, nrec, hot, hot_pct, __float_as_uint(f) & 1u);
    }
    if (acc == 0x12345678u) out[gid] = r;
    out[gid] = acc ^ r;
}

// host check of the transpose: every lane sees its own record's 16 words
__global__ void check_kernel(const uint32_t* table, uint32_t nrec, uint32_t* bad) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)table, (short)0, (int)(nrec * 64u), 0x00020000);
    const uint32_t lane = threadIdx.x & 63u, c = lane & 3u;
    const uint32_t r = (threadIdx.x * 7919u + 13u) % nrec;
    const uint32_t r0 = qp<QP(0, 0, 0, 0)>(r), r1 = qp<QP(1, 1, 1, 1)>(r), r2 = qp<QP(2, 2, 2, 2)>(r),
                   r3 = qp<QP(3, 3, 3, 3)>(r);
    const u4 A0 = ld16(rs, r0 * 64u + c * 16u), A1 = ld16(rs, r1 * 64u + c * 16u), A2 = ld16(rs, r2 * 64u + c * 16u),
             A3 = ld16(rs, r3 * 64u + c * 16u);
    uint32_t a[4][4] = {{A0.x, A0.y, A0.z, A0.w}, {A1.x, A1.y, A1.z, A1.w}, {A2.x, A2.y, A2.z, A2.w}, {A3.x, A3.y, A3.z, A3.w}};
    uint32_t w[16];
    quad_transpose(a, w);
    for (int k = 0; k < 16; ++k)
        if (w[k] != table[r * 16u + k]) atomicAdd(bad, 1u);
}

template <int MODE, int PAD>
static double run(const uint32_t* d_tab, uint32_t nrec, uint32_t hot, uint32_t hot_pct, int iters, uint32_t* d_out,
                  int blocks) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    gather_kernel<MODE, PAD><<<blocks, 256>>>(d_tab, nrec, hot, hot_pct, iters / 4, d_out);   // warm
    CHK(hipEventRecord(e0));
    gather_kernel<MODE, PAD><<<blocks, 256>>>(d_tab, nrec, hot, hot_pct, iters, d_out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    return (double)blocks * 256.0 * iters / (ms * 1e-3) / 1e9;   // G lane-steps / s
}

int main(int argc, char** argv) {
    const uint32_t nrec = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536;
    const uint32_t hot = argc > 2 ? (uint32_t)atoi(argv[2]) : 512;
    const uint32_t hot_pct = argc > 3 ? (uint32_t)atoi(argv[3]) : 90;
    const int iters = argc > 5 ? atoi(argv[5]) : 2000;
    std::vector<uint32_t> h((size_t)nrec * 16);
    uint32_t s = 12345;
    for (auto& v : h) { s = s * 1664525u + 1013904223u; v = s; }
    uint32_t *d_tab, *d_out, *d_bad;
    CHK(hipMalloc(&d_tab, h.size() * 4));
    CHK(hipMemcpy(d_tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const int blocks = 256 * 8;   // 8 waves per SIMD on 256 CUs
    CHK(hipMalloc(&d_out, (size_t)blocks * 256 * 4));
    CHK(hipMalloc(&d_bad, 4));
    CHK(hipMemset(d_bad, 0, 4));
    check_kernel<<<1, 256>>>(d_tab, nrec, d_bad);
    uint32_t bad = 0;
    CHK(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
    printf("transpose check: %s\n", bad ? "FAIL" : "ok");
    if (bad) return 1;
    {   // the LDS-staged quad fetch walks the same chains as the per-lane fetch
        const size_t n = (size_t)blocks * 256;
        std::vector<uint32_t> o0(n), o3(n);
        gather_kernel<0, 0><<<blocks, 256>>>(d_tab, nrec, hot, hot_pct, 50, d_out);
        CHK(hipMemcpy(o0.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        gather_kernel<3, 0><<<blocks, 256>>>(d_tab, nrec, hot, hot_pct, 50, d_out);
        CHK(hipMemcpy(o3.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        printf("lds-quad chain check: %s\n", o0 == o3 ? "ok" : "FAIL");
        if (o0 != o3) return 1;
    }
    printf("nrec %u (%.1f MB) hot %u (%.1f KB) %u%%\n", nrec, nrec * 64.0 / 1e6, hot, hot * 64.0 / 1e3, hot_pct);
#define ROW(P) printf("pad %3d: lane %.2f quad %.2f quad-noT %.2f quad-lds %.2f Glanesteps/s\n", P, \
        run<0, P>(d_tab, nrec, hot, hot_pct, iters, d_out, blocks), run<1, P>(d_tab, nrec, hot, hot_pct, iters, d_out, blocks), \
        run<2, P>(d_tab, nrec, hot, hot_pct, iters, d_out, blocks), run<3, P>(d_tab, nrec, hot, hot_pct, iters, d_out, blocks))
    ROW(0); ROW(40); ROW(80); ROW(120);
    return 0;
}
