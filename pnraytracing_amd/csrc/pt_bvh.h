// pnraytracing_amd/csrc/pt_bvh.h -- BuildBVH (include/BVH.hpp:92-173) on the GPU,
// emitting the reference's node array (pre-order, left child = id + 1) and
// triangle order bit for bit.
//
// The reference recursion touches disjoint triangle ranges per node, so every
// node of one tree level can be built at once.  What makes the result
// identical rather than merely equivalent:
//   * node bound (stored, :98-100): glm::min/max keep the FIRST operand on
//     ties, so a component's bits (the sign of a zero) are those of the first
//     triangle, in the range's current order, that attains the extreme.
//     Reduced as 64-bit keys: (ordered value, -0 == +0) << 32 | position.
//   * centre bound / bucket bounds: only their VALUES reach the bucket index
//     and the cost (a zero's sign changes neither), so plain min/max.
//   * axis (:110-114), bucket index (:131-133, :159-161), cost loop
//     (:139-154), leaf rule (:163-168): the same binary32 expressions,
//     compiled with -ffp-contract=off.
//   * std::partition (:157; libstdc++ __partition for bidirectional
//     iterators): with mid = L + count(pred), the k-th predicate-false
//     element of [L, mid) is swapped with the k-th predicate-true element of
//     [mid, R) counted from the back.  Computed from prefix counts, then
//     applied as disjoint swaps.  It runs before the leaf test, as in the
//     reference, so leaves that had a split candidate are reordered too.
//   * node ids: the tree is built level by level under temporary ids; the
//     pre-order numbering (left child = id + 1, right child = id + 1 +
//     size(left subtree), the static nodeId counter of :94-95) is assigned
//     once all subtree sizes are known.
// Ranges of at most 64 triangles are finished by ONE wave each (lane = slot
// of the range, the subtree walked depth-first in the reference's order);
// larger ranges go through chunked multi-workgroup passes, one level per round.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BVH_BUCKETS 12          // BVH.hpp:128 BUCKETSIZE
#define BVH_LEAF_MAX 255        // BVH.hpp:175 maxTrianglesInLeaf
#define BVH_SMALL 64            // ranges of <= this many triangles: one wave each
#define BVH_CHUNK 2048          // elements per workgroup in the large-range passes
#define BVH_PT (BVH_CHUNK / 256)

struct BvhSeg {                 // a large range at the current level
    int L, R, depth, tmp;       // tmp = temporary id of its node record
    int chunk0, pad[3];         // first chunk of the range in this level's chunk list
};
struct BvhChunk { int seg, start, end, pad; };
struct BvhAcc {                 // per large range, reset every level
    unsigned long long kmin[3], kmax[3];            // node bound keys (first occurrence)
    unsigned int cmin[3], cmax[3];                  // centre bound (ordered keys)
    unsigned int bcnt[BVH_BUCKETS];
    unsigned int bmin[BVH_BUCKETS][3], bmax[BVH_BUCKETS][3];
    float bound[6];
    int state;                  // 0 split candidate, 1 leaf without partition
    int d; float lo, ext;
    int cnt, K, leaf, pad;
};
struct BvhTop {                 // node record of a large range (temporary id)
    float b[6];
    int axis, L, R, depth;
    int left, right;            // >= 0: temporary id of a large child; < 0: -(small index + 1)
};
struct BvhSmall { int L, R, depth, base, count, pad[3]; };   // base/count: its local node records
struct BvhLocal { float b[6]; int axis, L, R, right; };      // right: local id, -1 for leaves
struct BvhCtr { int nseg, nch, ntop, nsmall, small_nodes, max_depth, pad[2]; };

// ---- ordered keys -----------------------------------------------------------------------
__device__ __forceinline__ unsigned int bvh_ord(float f) {        // float order -> unsigned order
    const unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float bvh_unord(unsigned int k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ unsigned int bvh_ordc(float f) {       // -0 and +0 tie
    return bvh_ord(f == 0.0f ? 0.0f : f);
}

// triangle bound / centre component j of original triangle o
// (A = pMin.xyz, centre.x; B = pMax.xyz, centre.y; C = centre.z)
__device__ __forceinline__ float bvh_bmin(const float4* A, int o, int j) {
    const float4 a = A[o];
    return j == 0 ? a.x : (j == 1 ? a.y : a.z);
}
__device__ __forceinline__ float bvh_bmax(const float4* B, int o, int j) {
    const float4 b = B[o];
    return j == 0 ? b.x : (j == 1 ? b.y : b.z);
}

// BVH.hpp:131-133 / :159-161
__device__ __forceinline__ int bvh_bucket(float c, float lo, float ext) {
    int pos = (int)(((c - lo) / ext) * (float)BVH_BUCKETS);
    if (pos == BVH_BUCKETS) pos = BVH_BUCKETS - 1;
    return pos;
}

// Bound::SurfaceArea (bound.hpp:22-25) of (pMin, pMax)
__device__ __forceinline__ float bvh_sa(const float* mn, const float* mx) {
    const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
    return (dx * dy + dx * dz + dy * dz) * 2.f;
}

// The split choice of BVH.hpp:139-154 from bucket counts and bucket bounds
// (empty bucket = the Bucket default bound; min/max over values).
__device__ __forceinline__ void bvh_best_split(const unsigned int* cnt, const float* bmn /*[12][3]*/,
                                               const float* bmx, float saNode, float& minCost, int& midBuc) {
    const float FMAX = 3.402823466e+38f, FLOW = -3.402823466e+38f;
    minCost = FMAX;
    midBuc = 0;
    for (int m = 0; m < BVH_BUCKETS - 1; ++m) {
        float b0n[3] = {FMAX, FMAX, FMAX}, b0x[3] = {FLOW, FLOW, FLOW};
        float b1n[3] = {FMAX, FMAX, FMAX}, b1x[3] = {FLOW, FLOW, FLOW};
        int c0 = 0, c1 = 0;
        for (int i = 0; i < BVH_BUCKETS; ++i) {
            float* tn = i <= m ? b0n : b1n;
            float* tx = i <= m ? b0x : b1x;
            if (i <= m) c0 += (int)cnt[i]; else c1 += (int)cnt[i];
            if (cnt[i] == 0) continue;
            for (int j = 0; j < 3; ++j) {
                const float vn = bmn[3 * i + j], vx = bmx[3 * i + j];
                tn[j] = vn < tn[j] ? vn : tn[j];
                tx[j] = tx[j] < vx ? vx : tx[j];
            }
        }
        const float cost = 1.f + (bvh_sa(b0n, b0x) * (float)c0 + bvh_sa(b1n, b1x) * (float)c1) / saNode;
        if (cost < minCost) { minCost = cost; midBuc = m; }
    }
}

template <typename T>
__device__ __forceinline__ T bvh_wmin(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { const T u = __shfl_xor(v, o); v = u < v ? u : v; }
    return v;
}
template <typename T>
__device__ __forceinline__ T bvh_wmax(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { const T u = __shfl_xor(v, o); v = u > v ? u : v; }
    return v;
}

// =====================================================================================
// large ranges: one level per round
// =====================================================================================
__global__ void bvh_init_kernel(BvhAcc* acc, int nseg) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    BvhAcc& a = acc[s];
    for (int j = 0; j < 3; ++j) {
        a.kmin[j] = ~0ull; a.kmax[j] = 0ull; a.cmin[j] = ~0u; a.cmax[j] = 0u;
    }
    for (int i = 0; i < BVH_BUCKETS; ++i) {
        a.bcnt[i] = 0u;
        for (int j = 0; j < 3; ++j) { a.bmin[i][j] = ~0u; a.bmax[i][j] = 0u; }
    }
    a.state = 0; a.K = 0; a.cnt = 0; a.leaf = 0;
}

// node bound (first-occurrence keys) + centre bound, per chunk
__global__ void __launch_bounds__(256) bvh_bounds_kernel(const BvhChunk* ch, BvhAcc* acc, const int* order,
                                                         const float4* A, const float4* B, const float* C) {
    const BvhChunk c = ch[blockIdx.x];
    unsigned long long kmn[3] = {~0ull, ~0ull, ~0ull}, kmx[3] = {0ull, 0ull, 0ull};
    unsigned int cmn[3] = {~0u, ~0u, ~0u}, cmx[3] = {0u, 0u, 0u};
    for (int p = c.start + (int)threadIdx.x; p < c.end; p += 256) {
        const int o = order[p];
        const float4 a = A[o], b = B[o];
        const float mn[3] = {a.x, a.y, a.z}, mx[3] = {b.x, b.y, b.z}, ce[3] = {a.w, b.w, C[o]};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const unsigned long long k0 = ((unsigned long long)bvh_ordc(mn[j]) << 32) | (unsigned int)p;
            const unsigned long long k1 = ((unsigned long long)bvh_ordc(mx[j]) << 32) | (0xffffffffu - (unsigned int)p);
            kmn[j] = k0 < kmn[j] ? k0 : kmn[j];
            kmx[j] = k1 > kmx[j] ? k1 : kmx[j];
            const unsigned int q = bvh_ord(ce[j]);
            cmn[j] = q < cmn[j] ? q : cmn[j];
            cmx[j] = q > cmx[j] ? q : cmx[j];
        }
    }
    __shared__ unsigned long long s_k[4][6];
    __shared__ unsigned int s_c[4][6];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        kmn[j] = bvh_wmin(kmn[j]); kmx[j] = bvh_wmax(kmx[j]);
        cmn[j] = bvh_wmin(cmn[j]); cmx[j] = bvh_wmax(cmx[j]);
    }
    if (lane == 0)
        for (int j = 0; j < 3; ++j) {
            s_k[w][j] = kmn[j]; s_k[w][3 + j] = kmx[j]; s_c[w][j] = cmn[j]; s_c[w][3 + j] = cmx[j];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int j = threadIdx.x;
        unsigned long long k = s_k[0][j];
        unsigned int q = s_c[0][j];
        for (int v = 1; v < 4; ++v) {
            k = j < 3 ? (s_k[v][j] < k ? s_k[v][j] : k) : (s_k[v][j] > k ? s_k[v][j] : k);
            q = j < 3 ? (s_c[v][j] < q ? s_c[v][j] : q) : (s_c[v][j] > q ? s_c[v][j] : q);
        }
        BvhAcc& a = acc[c.seg];
        if (j < 3) { atomicMin(&a.kmin[j], k); atomicMin(&a.cmin[j], q); }
        else { atomicMax(&a.kmax[j - 3], k); atomicMax(&a.cmax[j - 3], q); }
    }
}

// node bound bits, split axis, degenerate-centre leaf (BVH.hpp:97-121), per range
__global__ void bvh_axis_kernel(const BvhSeg* segs, BvhAcc* acc, int nseg, const int* order, const float4* A,
                                const float4* B) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    BvhAcc& a = acc[s];
    for (int j = 0; j < 3; ++j) {
        const unsigned int pn = (unsigned int)(a.kmin[j] & 0xffffffffull);
        const unsigned int px = 0xffffffffu - (unsigned int)(a.kmax[j] & 0xffffffffull);
        a.bound[j] = bvh_bmin(A, order[pn], j);
        a.bound[3 + j] = bvh_bmax(B, order[px], j);
    }
    float cn[3], cx[3], dg[3];
    for (int j = 0; j < 3; ++j) { cn[j] = bvh_unord(a.cmin[j]); cx[j] = bvh_unord(a.cmax[j]); dg[j] = cx[j] - cn[j]; }
    int d;
    if (dg[0] >= dg[1] && dg[0] >= dg[2]) d = 0;
    else if (dg[1] >= dg[0] && dg[1] >= dg[2]) d = 1;
    else d = 2;
    a.d = d;
    a.lo = cn[d];
    a.ext = dg[d];
    if (cx[d] == cn[d]) { a.state = 1; a.leaf = 1; }
    (void)segs;
}

// bucket counts and bounds (BVH.hpp:127-137), per chunk
__global__ void __launch_bounds__(256) bvh_bucket_kernel(const BvhChunk* ch, BvhAcc* acc, const int* order,
                                                         const float4* A, const float4* B, const float* C) {
    const BvhChunk c = ch[blockIdx.x];
    BvhAcc& a = acc[c.seg];
    if (a.state) return;
    __shared__ unsigned int s_n[BVH_BUCKETS], s_mn[BVH_BUCKETS * 3], s_mx[BVH_BUCKETS * 3];
    if (threadIdx.x < BVH_BUCKETS) s_n[threadIdx.x] = 0u;
    if (threadIdx.x < BVH_BUCKETS * 3) { s_mn[threadIdx.x] = ~0u; s_mx[threadIdx.x] = 0u; }
    __syncthreads();
    const int d = a.d;
    const float lo = a.lo, ext = a.ext;
    for (int p = c.start + (int)threadIdx.x; p < c.end; p += 256) {
        const int o = order[p];
        const float4 ta = A[o], tb = B[o];
        const float ce = d == 0 ? ta.w : (d == 1 ? tb.w : C[o]);
        const int pos = bvh_bucket(ce, lo, ext);
        atomicAdd(&s_n[pos], 1u);
        atomicMin(&s_mn[3 * pos], bvh_ord(ta.x)); atomicMin(&s_mn[3 * pos + 1], bvh_ord(ta.y));
        atomicMin(&s_mn[3 * pos + 2], bvh_ord(ta.z));
        atomicMax(&s_mx[3 * pos], bvh_ord(tb.x)); atomicMax(&s_mx[3 * pos + 1], bvh_ord(tb.y));
        atomicMax(&s_mx[3 * pos + 2], bvh_ord(tb.z));
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < BVH_BUCKETS) {
        if (s_n[t]) atomicAdd(&a.bcnt[t], s_n[t]);
    } else if (t < BVH_BUCKETS * 4) {
        const int q = t - BVH_BUCKETS, i = q / 3, j = q - 3 * (q / 3);
        if (s_n[i]) atomicMin(&a.bmin[i][j], s_mn[q]);
    } else if (t < BVH_BUCKETS * 7) {
        const int q = t - BVH_BUCKETS * 4, i = q / 3, j = q - 3 * (q / 3);
        if (s_n[i]) atomicMax(&a.bmax[i][j], s_mx[q]);
    }
}

// cost loop, partition count, leaf rule (BVH.hpp:139-168), per range
__global__ void bvh_split_kernel(const BvhSeg* segs, BvhAcc* acc, int nseg) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    BvhAcc& a = acc[s];
    if (a.state) return;
    float bmn[BVH_BUCKETS * 3], bmx[BVH_BUCKETS * 3];
    for (int i = 0; i < BVH_BUCKETS; ++i)
        for (int j = 0; j < 3; ++j) { bmn[3 * i + j] = bvh_unord(a.bmin[i][j]); bmx[3 * i + j] = bvh_unord(a.bmax[i][j]); }
    float minCost;
    int midBuc;
    bvh_best_split(a.bcnt, bmn, bmx, bvh_sa(a.bound, a.bound + 3), minCost, midBuc);
    int cnt = 0;
    for (int i = 0; i <= midBuc; ++i) cnt += (int)a.bcnt[i];
    const int n = segs[s].R - segs[s].L;
    a.cnt = cnt;
    a.leaf = ((n <= BVH_LEAF_MAX && (float)n <= minCost) || cnt == 0) ? 1 : 0;
    // the partition predicate needs midBuc: bucket index <= midBuc
    a.state = 0;
    a.pad = midBuc;
}

__device__ __forceinline__ bool bvh_pred(const BvhAcc& a, const float4* A, const float4* B, const float* C, int o) {
    const float ce = a.d == 0 ? A[o].w : (a.d == 1 ? B[o].w : C[o]);
    return bvh_bucket(ce, a.lo, a.ext) <= a.pad;
}

// block-wide exclusive sum of one int per thread (256 threads)
__device__ __forceinline__ int bvh_block_excl(int v, int& total) {
    __shared__ int s_w[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(x, o);
        if (lane >= o) x += u;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    int before = 0;
    for (int k = 0; k < w; ++k) before += s_w[k];
    total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return before + x - v;
}

// predicate-true count per chunk
__global__ void __launch_bounds__(256) bvh_count_kernel(const BvhChunk* ch, const BvhAcc* acc, const int* order,
                                                        const float4* A, const float4* B, const float* C,
                                                        int* chunk_true) {
    const BvhChunk c = ch[blockIdx.x];
    const BvhAcc& a = acc[c.seg];
    int k = 0;
    if (!a.state)
        for (int p = c.start + (int)threadIdx.x; p < c.end; p += 256) k += bvh_pred(a, A, B, C, order[p]) ? 1 : 0;
    int total;
    (void)bvh_block_excl(k, total);
    if (threadIdx.x == 0) chunk_true[blockIdx.x] = total;
}

// exclusive scan of the chunk counts over the level's chunk list (one workgroup)
__global__ void __launch_bounds__(1024) bvh_scan_kernel(const int* in, int* out, int n) {
    __shared__ int s[1024];
    const int per = (n + 1023) / 1024;
    const int b = threadIdx.x * per, e = min(b + per, n);
    int sum = 0;
    for (int i = b; i < e; ++i) sum += in[i];
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    int run = s[threadIdx.x] - sum;
    for (int i = b; i < e; ++i) { out[i] = run; run += in[i]; }
}

// positions of the elements std::partition swaps: Fpos[L + k] = k-th false of
// [L, mid), Tpos[L + k] = k-th true of [mid, R) from the back; K per range
__global__ void __launch_bounds__(256) bvh_lists_kernel(const BvhChunk* ch, const BvhSeg* segs, BvhAcc* acc,
                                                        const int* order, const float4* A, const float4* B,
                                                        const float* C, const int* excl, int* Fpos, int* Tpos) {
    const BvhChunk c = ch[blockIdx.x];
    BvhAcc& a = acc[c.seg];
    if (a.state) return;                           // uniform per workgroup
    const BvhSeg sg = segs[c.seg];
    const int base = c.start + (int)threadIdx.x * BVH_PT;
    bool pr[BVH_PT];
    int local = 0;
#pragma unroll
    for (int k = 0; k < BVH_PT; ++k) {
        const int p = base + k;
        pr[k] = p < c.end ? bvh_pred(a, A, B, C, order[p]) : false;
        local += pr[k] ? 1 : 0;
    }
    int total;
    int T = bvh_block_excl(local, total) + (excl[blockIdx.x] - excl[sg.chunk0]);   // trues in [L, base)
    const int mid = sg.L + a.cnt;
#pragma unroll
    for (int k = 0; k < BVH_PT; ++k) {
        const int p = base + k;
        if (p >= c.end) break;
        if (p < mid && !pr[k]) Fpos[sg.L + (p - sg.L) - T] = p;
        if (p >= mid && pr[k]) Tpos[sg.L + a.cnt - T - 1] = p;
        if (p == mid - 1) a.K = (mid - sg.L) - (T + (pr[k] ? 1 : 0));
        T += pr[k] ? 1 : 0;
    }
}

__global__ void __launch_bounds__(256) bvh_swap_kernel(const BvhChunk* ch, const BvhSeg* segs, const BvhAcc* acc,
                                                       int* order, const int* Fpos, const int* Tpos) {
    const BvhChunk c = ch[blockIdx.x];
    const BvhAcc& a = acc[c.seg];
    if (a.state) return;
    const int L = segs[c.seg].L, K = a.K;
    for (int p = c.start + (int)threadIdx.x; p < c.end; p += 256) {
        const int k = p - L;
        if (k < K) {
            const int x = Fpos[L + k], y = Tpos[L + k];
            const int t = order[x];
            order[x] = order[y];
            order[y] = t;
        }
    }
}

// node record + children for the next level, per range
__global__ void bvh_emit_kernel(const BvhSeg* segs, const BvhAcc* acc, int nseg, BvhTop* top, BvhSeg* nsegs,
                                BvhChunk* nchunks, BvhSmall* small, BvhCtr* ctr) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const BvhSeg sg = segs[s];
    const BvhAcc& a = acc[s];
    BvhTop t;
    for (int j = 0; j < 6; ++j) t.b[j] = a.bound[j];
    t.L = sg.L; t.R = sg.R; t.depth = sg.depth;
    t.axis = a.leaf ? -1 : a.d;
    t.left = t.right = 0;
    atomicMax(&ctr->max_depth, sg.depth);
    if (!a.leaf) {
        const int mid = sg.L + a.cnt;
        for (int side = 0; side < 2; ++side) {
            const int cl = side ? mid : sg.L, cr = side ? sg.R : mid, n = cr - cl;
            int ref;
            if (n > BVH_SMALL) {
                const int slot = atomicAdd(&ctr->nseg, 1);
                const int tmp = atomicAdd(&ctr->ntop, 1);
                const int nck = (n + BVH_CHUNK - 1) / BVH_CHUNK;
                const int c0 = atomicAdd(&ctr->nch, nck);
                BvhSeg ns; ns.L = cl; ns.R = cr; ns.depth = sg.depth + 1; ns.tmp = tmp; ns.chunk0 = c0;
                ns.pad[0] = ns.pad[1] = ns.pad[2] = 0;
                nsegs[slot] = ns;
                for (int i = 0; i < nck; ++i) {
                    BvhChunk k; k.seg = slot; k.start = cl + i * BVH_CHUNK; k.end = min(cl + (i + 1) * BVH_CHUNK, cr); k.pad = 0;
                    nchunks[c0 + i] = k;
                }
                ref = tmp;
            } else {
                const int k = atomicAdd(&ctr->nsmall, 1);
                BvhSmall m; m.L = cl; m.R = cr; m.depth = sg.depth + 1; m.base = 0; m.count = 0;
                m.pad[0] = m.pad[1] = m.pad[2] = 0;
                small[k] = m;
                ref = -(k + 1);
            }
            if (side) t.right = ref; else t.left = ref;
        }
    }
    top[sg.tmp] = t;
}

// =====================================================================================
// small ranges: one wave builds the whole subtree, depth-first in the reference's order
// =====================================================================================
__device__ __forceinline__ void bvh_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(256) bvh_small_kernel(BvhSmall* small, int nsmall, int* order, const float4* A,
                                                        const float4* B, const float* C, BvhLocal* out,
                                                        BvhCtr* ctr) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = blockIdx.x * 4 + w;
    if (k >= nsmall) return;                               // whole wave
    __shared__ int4 s_stk[4][64];
    __shared__ unsigned int s_n[4][BVH_BUCKETS], s_mn[4][BVH_BUCKETS * 3], s_mx[4][BVH_BUCKETS * 3];
    __shared__ int s_lst[4][2][64];
    const BvhSmall sm = small[k];
    const int n = sm.R - sm.L;
    int o = 0;
    float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f}, ce[3] = {0.f, 0.f, 0.f};
    if (lane < n) {
        o = order[sm.L + lane];
        const float4 a = A[o], b = B[o];
        mn[0] = a.x; mn[1] = a.y; mn[2] = a.z; mx[0] = b.x; mx[1] = b.y; mx[2] = b.z;
        ce[0] = a.w; ce[1] = b.w; ce[2] = C[o];
    }
    int base = 0;
    if (lane == 0) base = atomicAdd(&ctr->small_nodes, 2 * n - 1);
    base = __shfl(base, 0);
    int sp = 0, id = 0, maxd = 0;
    s_stk[w][0] = make_int4(0, n, sm.depth, -1);          // every lane writes the same entry
    sp = 1;
    const unsigned long long below = (1ull << lane) - 1ull;
    while (sp > 0) {
        --sp;
        const int4 e = s_stk[w][sp];
        const int l = e.x, r = e.y, dep = e.z, par = e.w;
        const int myid = id++;
        maxd = dep > maxd ? dep : maxd;
        if (par >= 0 && lane == 0) out[base + par].right = myid;
        const bool mem = lane >= l && lane < r;
        // node bound, bits of the first triangle attaining each extreme (:97-100)
        float bnd[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const float v = j < 3 ? mn[j] : mx[j - 3];
            const unsigned int key = bvh_ordc(v);
            const unsigned int red = j < 3 ? bvh_wmin(mem ? key : ~0u) : bvh_wmax(mem ? key : 0u);
            const unsigned long long win = __ballot(mem && key == red);
            bnd[j] = __shfl(v, __ffsll((long long)win) - 1);
        }
        const int nn = r - l;
        bool leaf = true;
        int axis = -1, mid = l;
        if (nn > 2) {
            float cn[3], cx[3], dg[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const unsigned int q = bvh_ord(ce[j]);
                cn[j] = bvh_unord(bvh_wmin(mem ? q : ~0u));
                cx[j] = bvh_unord(bvh_wmax(mem ? q : 0u));
                dg[j] = cx[j] - cn[j];
            }
            int d;
            if (dg[0] >= dg[1] && dg[0] >= dg[2]) d = 0;
            else if (dg[1] >= dg[0] && dg[1] >= dg[2]) d = 1;
            else d = 2;
            if (!(cx[d] == cn[d])) {
                const float lo = cn[d], ext = dg[d];
                const float myc = d == 0 ? ce[0] : (d == 1 ? ce[1] : ce[2]);
                const int pos = mem ? bvh_bucket(myc, lo, ext) : 0;
                if (lane < BVH_BUCKETS) s_n[w][lane] = 0u;
                if (lane < BVH_BUCKETS * 3) { s_mn[w][lane] = ~0u; s_mx[w][lane] = 0u; }
                bvh_wave_sync();
                if (mem) {
                    atomicAdd(&s_n[w][pos], 1u);
                    for (int j = 0; j < 3; ++j) {
                        atomicMin(&s_mn[w][3 * pos + j], bvh_ord(mn[j]));
                        atomicMax(&s_mx[w][3 * pos + j], bvh_ord(mx[j]));
                    }
                }
                bvh_wave_sync();
                unsigned int cnt12[BVH_BUCKETS];
                float bmn[BVH_BUCKETS * 3], bmx[BVH_BUCKETS * 3];
                for (int i = 0; i < BVH_BUCKETS; ++i) {
                    cnt12[i] = s_n[w][i];
                    for (int j = 0; j < 3; ++j) {
                        bmn[3 * i + j] = bvh_unord(s_mn[w][3 * i + j]);
                        bmx[3 * i + j] = bvh_unord(s_mx[w][3 * i + j]);
                    }
                }
                float minCost;
                int midBuc;
                bvh_best_split(cnt12, bmn, bmx, bvh_sa(bnd, bnd + 3), minCost, midBuc);
                const bool pred = mem && pos <= midBuc;
                const unsigned long long Tm = __ballot(pred);
                const int cnt = __popcll(Tm);
                mid = l + cnt;
                const unsigned long long memM = (r == 64 ? ~0ull : ((1ull << r) - 1ull)) & ~((1ull << l) - 1ull);
                const unsigned long long frontM = (mid == 64 ? ~0ull : ((1ull << mid) - 1ull)) & memM;
                const unsigned long long F = frontM & ~Tm, Tb = Tm & ~frontM;
                if (F != 0ull) {                               // std::partition's swaps
                    const bool inF = (F >> lane) & 1ull, inT = (Tb >> lane) & 1ull;
                    const int rf = __popcll(F & below);
                    const int rt = lane == 63 ? 0 : __popcll(Tb >> (lane + 1));
                    bvh_wave_sync();
                    if (inF) s_lst[w][0][rf] = lane;
                    if (inT) s_lst[w][1][rt] = lane;
                    bvh_wave_sync();
                    int src = lane;
                    if (inF) src = s_lst[w][1][rf];
                    if (inT) src = s_lst[w][0][rt];
                    o = __shfl(o, src);
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        mn[j] = __shfl(mn[j], src); mx[j] = __shfl(mx[j], src); ce[j] = __shfl(ce[j], src);
                    }
                }
                leaf = (nn <= BVH_LEAF_MAX && (float)nn <= minCost) || cnt == 0;
                axis = d;
            }
        }
        if (lane == 0) {
            BvhLocal rec;
            for (int j = 0; j < 6; ++j) rec.b[j] = bnd[j];
            rec.axis = leaf ? -1 : axis;
            rec.L = sm.L + l; rec.R = sm.L + r; rec.right = -1;
            out[base + myid] = rec;
        }
        if (!leaf) {                                      // left subtree first: pushed last
            bvh_wave_sync();
            s_stk[w][sp] = make_int4(mid, r, dep + 1, myid);
            s_stk[w][sp + 1] = make_int4(l, mid, dep + 1, -1);
            sp += 2;
            bvh_wave_sync();
        }
    }
    if (lane < n) order[sm.L + lane] = o;
    if (lane == 0) {
        small[k].base = base;
        small[k].count = id;
        atomicMax(&ctr->max_depth, maxd);
    }
}

// =====================================================================================
// final records (main.cpp:488-501 layout, 12 floats) at their pre-order ids
// =====================================================================================
__device__ __forceinline__ void bvh_put(float* out, int id, const float* b, int axis, int right, int L, int R) {
    float* q = out + 12 * (size_t)id;
    for (int j = 0; j < 6; ++j) q[j] = b[j];
    q[6] = (float)axis; q[7] = (float)right; q[8] = (float)L; q[9] = (float)R; q[10] = 0.f; q[11] = 0.f;
}

__global__ void bvh_scatter_top_kernel(const BvhTop* top, int ntop, const int* ftop, const int* fsmall, float* out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntop) return;
    const BvhTop n = top[t];
    int right = -1;
    if (n.axis != -1) right = n.right >= 0 ? ftop[n.right] : fsmall[-n.right - 1];
    bvh_put(out, ftop[t], n.b, n.axis, right, n.L, n.R);
}

__global__ void __launch_bounds__(256) bvh_scatter_small_kernel(const BvhSmall* small, int nsmall,
                                                                const BvhLocal* loc, const int* fsmall, float* out) {
    const int lane = threadIdx.x & 63;
    const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= nsmall) return;
    const BvhSmall m = small[k];
    const int f0 = fsmall[k];
    for (int j = lane; j < m.count; j += 64) {
        const BvhLocal r = loc[m.base + j];
        bvh_put(out, f0 + j, r.b, r.axis, r.right >= 0 ? f0 + r.right : -1, r.L, r.R);
    }
}
