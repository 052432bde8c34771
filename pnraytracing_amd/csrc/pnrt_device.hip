// pnraytracing_amd/csrc/pnrt_device.hip -- libpnrt.so: C ABI (include/pnrt.h),
// scene re-layout and the gfx950 radiance-integrator kernel that replaces
// PnRayTracing's shaders/ray_tracing.comp.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math
//        -fPIC -shared  (pnraytracing_amd/build.py)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pnrt.h"

#include "pt_path.h"
#include "pt_wf.h"
#include "pt_env.h"
#include "pt_bvh.h"

__global__ void pt_pack_rows_kernel(const float4* accum, float4* dst, int width, int rows, int band,
                                    int n_shards, int shard) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t total = (size_t)rows * width;
    if (i >= total) return;
    int r = (int)(i / width), x = (int)(i - (size_t)r * width);
    int y = shard_row(r, band, n_shards, shard);
    dst[i] = accum[(size_t)y * width + x];
}

// the inverse of pt_pack_rows_kernel: a shard's packed rows into their image rows
__global__ void pt_unpack_rows_kernel(const float4* src, float4* img, int width, int rows, int band, int n_shards,
                                      int shard) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t total = (size_t)rows * width;
    if (i >= total) return;
    int r = (int)(i / width), x = (int)(i - (size_t)r * width);
    int y = shard_row(r, band, n_shards, shard);
    img[(size_t)y * width + x] = src[i];
}

__global__ void pt_math_kernel(int fn, const float* a, const float* b, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i], r;
    uint32_t u;
    switch (fn) {
    case 0: r = pnm_sin(x); break;
    case 1: r = pnm_cos(x); break;
    case 2: r = pnm_atan2(x, y); break;
    case 3: r = pnm_asin(x); break;
    case 4: r = pnm_log(x); break;
    case 5: r = pnm_pow(x, y); break;
    case 6: r = pnm_exp2(x); break;
    case 7: r = sqrtf(x); break;
    case 8: r = x / y; break;
    case 9: u = __float_as_uint(x); r = (float)u; break;
    case 10: u = __float_as_uint(x); wang_hash(u); r = __uint_as_float(u); break;
    default: r = pnm_nan(); break;
    }
    out[i] = r;
}

// =====================================================================================
// host side
// =====================================================================================
struct pnrt_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // trace faults (pt_wf.h wf_fault): WF_FAULT_WORDS words in host-mapped memory the
    // kernels write only when a check trips; `faulted` latches until reset_accum
    uint32_t* fault_host = nullptr;
    uint32_t* fault_dev = nullptr;
    bool faulted = false;
    std::string fault_msg;
    // scene
    std::vector<void*> scene_allocs;
    DevScene scene{};
    bool has_scene = false;
    int max_depth = 0, n_interior = 0, root_is_leaf = 0;
    int64_t scene_bytes = 0;
    std::vector<int> light_mat;            // material of each light record's triangle (pnrt_update_materials)
    std::vector<float4> light_rec_host;    // host copy of the light records (patched, then one upload)
    std::vector<float> mat_emit;           // host copy of every material's emission (3 floats each)
    float env_max = 0.f;                   // largest |texel| component of the env image (NaN: a NaN texel)
    // env + textures
    void* hdr = nullptr;
    void* rnd = nullptr;
    void* hdr_q = nullptr;      // footprint records of both (DevScene::hdr_q)
    void* rnd_q = nullptr;
    void* tex[PT_MAX_TEXTURES] = {};
    int tex_w[PT_MAX_TEXTURES] = {}, tex_h[PT_MAX_TEXTURES] = {};
    float* unorm8 = nullptr;
    // frame
    int width = 0, height = 0, max_bounce = 4;
    pnrt_camera cam{};
    bool has_frame = false;
    float4* accum = nullptr;
    int mode = PNRT_TRAVERSE_ZCULL;
    bool boxes_finite = true;              // every BVH box coordinate finite: z-slab culling allowed (pt_wf.h box_slabs)
    int kernel = 3;                        // 3 = wavefront (default), 1 = v1 one-lane-per-pixel
    bool serial = false;                   // PNRT_SERIAL: one call in flight, full trace grid (measurement)
    // Pipelined wavefront rendering.  pnrt_render calls rotate over the pipes -- the
    // first WF_PIPES_LARGE of them, or all WF_PIPES for small calls (a multi-GPU
    // rank's share: its kernels are short, so a fourth call in flight fills the
    // gaps of the other three's dependent chains; measured at N = 8).  A pipe is its own
    // worker stream and primary / colour / path buffers, so call k+1 starts
    // while call k's kernels drain (one call's kernels fill the CUs the other's
    // trace kernel leaves idle while its last rays drain).  Only the blends are
    // ordered: they run in call order on the context stream, which therefore
    // sees each call's finished image.  The fourth pipe (small calls only) is
    // created only when the process has more than 4 hardware queues
    // (GPU_MAX_HW_QUEUES, HIP's default 4): with 4, its worker would share the
    // context stream's queue and serialise behind the blends, so small calls
    // rotate over the first three like large ones (n_pipes_small).
    // (Splitting a call into two concurrent half-batches on two worker streams
    // as well measured slower: 1 006 vs 1 105 Msamples/s.)
    struct PrimKey {        // what a pipe's primary records were traced for (render_wavefront)
        uint64_t epoch = 0; // scene_epoch at the time
        float cam[12] = {};
        int width = 0, height = 0, rows = 0, band = 0, n_shards = 0, shard = 0, mode = -1;
        bool valid = false;
    };
    struct Pipe {
        hipStream_t w = nullptr;
        hipEvent_t ev_join = nullptr, ev_blend = nullptr;
        hipEvent_t ev_stage = nullptr;   // WF_STAGGER: the call has reached its drain-heavy end
        bool stage_set = false;
        float4* primary = nullptr;  size_t primary_cap = 0;
        PrimKey prim;
        float4* colors = nullptr;   size_t colors_cap = 0;
        void* wf = nullptr;         size_t wf_cap = 0;
        uint2* ovf = nullptr;       size_t ovf_cap = 0;
        bool blend_pending = false;  // ev_blend guards the colour buffer's last reader
    };
    Pipe pipe[WF_PIPES];
    unsigned n_pipes_small = WF_PIPES;     // pipes small calls rotate over (pipes_init)
    size_t batch_bytes_cap = 0;            // PNRT_BATCH_BYTES: device bytes of one batch's buffers at most (0: none)
    unsigned last_pipe = 0;                // the pipe of the last call
    // bumped by every change of what the primary records depend on besides the
    // frame (camera, size, shard, traversal mode: compared per call): the scene
    // arrays, the materials (emission) and the environment (a miss's colour)
    uint64_t scene_epoch = 1;
    hipEvent_t ev_last = nullptr;          // recorded after every op the context queues on `stream`, so a
    bool last_valid = false;               // pnrt_set_stream orders the new stream after it without
                                           // touching the old stream (which the caller may have destroyed)
    bool pipes_ready = false;
    uint64_t ncall = 0;
    unsigned next_pipe = 0;
    int trace_grid = 0;
    int trace_grid_cc = 0;     // full occupancy of the lone calls' trace instantiation (WF_TRACE_WAVES_CC)
    int wf_stack_need = 0;                 // wide-traversal stack entries per lane (from upload)
    // per-kernel-class HIP event timing (pnrt_profile_enable / pnrt_profile_read)
    bool prof_on = false;
    int prof_mask = -1;     // kernel classes bracketed while profiling (pnrt_profile_select)
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
    double prof_ms[PNRT_K_COUNT] = {};
    int64_t prof_n[PNRT_K_COUNT] = {};
};

static int set_err(pnrt_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}

// PNRT_E_TRACE once a fault word is set by completed work (see pnrt.h)
static int check_fault(pnrt_ctx* c) {
    if (!c->faulted && c->fault_host) {
        static const char* what[WF_FAULT_WORDS] = {
            "a bounded wait of the trace kernel's block ray queue ran out",
            "a trace block loaded fewer rays than it dequeued",
            "a trace launch ended with ray-queue items never dequeued",
            "diagnostic bounds check: a fetch / store index out of range at site "};
        static const char* site[] = {"?", "node", "triangle", "leaf table", "stack spill", "trace result", "ray record",
                                     "hit attributes", "light record", "env footprint", "albedo texel", "primary record",
                                     "colour", "path state", "segment", "cooperative frontier"};
        std::string m;
        for (int k = 0; k < WF_FAULT_WORDS; ++k) {
            const uint32_t v = __atomic_load_n(c->fault_host + k, __ATOMIC_ACQUIRE);
            if (!v) continue;
            m += (m.empty() ? "" : "; ") + std::string(what[k]);
            if (k == WF_FAULT_BOUNDS) m += std::string(v < sizeof site / sizeof *site ? site[v] : "?") + " (" + std::to_string(v) + ")";
        }
        if (!m.empty()) {
            c->faulted = true;
            c->fault_msg = "trace fault: " + m + " -- queued rays may be untraced, the accumulation image is "
                           "invalid (pnrt_reset_accum clears it)";
        }
    }
    return c->faulted ? set_err(c, PNRT_E_TRACE, c->fault_msg) : PNRT_OK;
}
#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return set_err(ctx, PNRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

// Record ev_last after an op queued on c->stream (see pnrt_set_stream).
static int mark_stream(pnrt_ctx* c) {
    HIPCHK(c, c->ev_last ? hipSuccess : hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_last, c->stream));
    c->last_valid = true;
    return PNRT_OK;
}

// every stream the context launches on (the caller's / blend stream, the workers)
static hipError_t sync_all(pnrt_ctx* c) {
    hipError_t e = hipStreamSynchronize(c->stream);
    for (auto& P : c->pipe)
        if (e == hipSuccess && P.w) e = hipStreamSynchronize(P.w);
    return e;
}

// ---- event timing: a start/stop event pair around every launch of a class ----------------
static hipEvent_t ev_get(pnrt_ctx* c) {
    if (!c->ev_pool.empty()) { hipEvent_t e = c->ev_pool.back(); c->ev_pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
struct ProfScope {     // records on the launch stream, so it times exactly that stream's launches
    pnrt_ctx* c; int k; hipStream_t st; hipEvent_t a = nullptr;
    ProfScope(pnrt_ctx* c_, int k_, hipStream_t st_ = nullptr) : c(c_), k(k_), st(st_ ? st_ : c_->stream) {
        if (c->prof_on && ((c->prof_mask >> k) & 1) && (a = ev_get(c))) (void)hipEventRecord(a, st);
    }
    ~ProfScope() {
        if (!a) return;
        hipEvent_t b = ev_get(c);
        if (!b) { c->ev_pool.push_back(a); return; }
        (void)hipEventRecord(b, st);
        c->ev_pending.push_back({k, {a, b}});
    }
};
static int prof_collect(pnrt_ctx* c) {
    if (c->ev_pending.empty()) return PNRT_OK;
    HIPCHK(c, sync_all(c));
    for (auto& p : c->ev_pending) {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, p.second.first, p.second.second));
        c->prof_ms[p.first] += ms;
        c->prof_n[p.first] += 1;
        c->ev_pool.push_back(p.second.first);
        c->ev_pool.push_back(p.second.second);
    }
    c->ev_pending.clear();
    return PNRT_OK;
}

#ifndef WF_MAX_CHUNK_FRAMES
#define WF_MAX_CHUNK_FRAMES 128  // frames per batch at most (bench.py's calls: 16 frames of a 1080p frame; a
                                 // multi-GPU rank's share: its timed steps in as few one-batch calls as fit --
                                 // 80 frames of a quarter / eighth at N = 4 / 8, profiles/r06/h/: +3 to +5 %)
#endif

static int grow(pnrt_ctx* c, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return 0;
    if (*p) {                          // the old buffer may still be in use by calls in flight
        (void)sync_all(c);
        (void)hipFree(*p);
    }
    *p = nullptr;
    *cap = 0;
    HIPCHK(c, hipMalloc(p, bytes));
    *cap = bytes;
    return 0;
}

static void free_scene(pnrt_ctx* c) {
    for (void* p : c->scene_allocs) (void)hipFree(p);
    c->scene_allocs.clear();
    c->has_scene = false;
}

template <class T>
static int upload(pnrt_ctx* c, const std::vector<T>& v, const T** out) {
    void* p = nullptr;
    size_t bytes = v.size() * sizeof(T);
    if (bytes == 0) { *out = nullptr; return 0; }
    HIPCHK(c, hipMalloc(&p, bytes));
    c->scene_allocs.push_back(p);
    HIPCHK(c, hipMemcpy(p, v.data(), bytes, hipMemcpyHostToDevice));
    c->scene_bytes += (int64_t)bytes;
    *out = static_cast<const T*>(p);
    return 0;
}

static inline int fint(float f) { return (int)f; }   // GLSL int(float)

#ifndef WF_TRACE_GRID_PCT
#define WF_TRACE_GRID_PCT 50         // cap of the trace grid, % of full occupancy, for batches of fewer than
#endif                               // WF_SMALL_CALL_PATHS paths (multi-GPU shares: the calls in flight share the chip)
#ifndef WF_TRACE_GRID_PCT_LARGE
#define WF_TRACE_GRID_PCT_LARGE 80   // ... and for larger batches (16-frame 1080p calls: C2 +1.6 %, C5 +2.9 %, C4 -3.4 %)
#endif
#ifndef WF_TRACE_PATHS_PER_BLOCK
#define WF_TRACE_PATHS_PER_BLOCK (8 * WF_TRACE_BLOCK) // > 0: trace grid <= paths / this (small multi-GPU shares)
#endif
#ifndef WF_STAGGER
#define WF_STAGGER 3        // k > 0: calls of >= WF_STAGGER_PATHS paths run on two pipes with the full trace
#endif                      // grid, each starting when the previous one is k trace / shade launches from its end
#ifndef WF_TRACE_GRID_PCT_ONE
#define WF_TRACE_GRID_PCT_ONE 100   // trace grid of a staggered call, % of full occupancy
#endif
#ifndef WF_STAGGER_PATHS
#define WF_STAGGER_PATHS 12000000   // (1080p calls of >= 6 frames; a rank's share at N = 2 with 16-frame calls)
#endif
#ifndef WF_CC_MAX_PATHS
#define WF_CC_MAX_PATHS 4000000     // lone calls of fewer paths per batch run the CC trace instantiation (the
#endif                              // reference's 512x512 frame: 262k); larger ones the pipelined one at 8 waves
#ifndef WF_ALONE_ON_CALLER
#define WF_ALONE_ON_CALLER 1        // a call with nothing in flight runs on the caller's stream (no worker hop)
#endif
#ifndef WF_TRACE_PATHS_PER_BLOCK_ALONE
#define WF_TRACE_PATHS_PER_BLOCK_ALONE WF_TRACE_BLOCK  // ... for a call with no other call in flight
#endif

// Wavefront buffers of one batch of n path slots, carved from `base` (wf_layout):
// two path-state sets (P0-P7 + block counts), hit / occ, the env ray records,
// segment counts, dequeue counters + census words (+ the timing builds' stamps).
#define WF_SOBOL_BYTES (4 * WF_MAX_CHUNK_FRAMES * 8)   // the batch's Sobol table: bounces 1..3 x frames, float2
static size_t wf_bytes(size_t n) {
    const size_t npad = (n + 255) / 256 * 256, nseg = npad / 256;
    return 2 * (npad * 16 * 8 + nseg * 4 + 256) + n * (4 + 2) + 256 + npad * 32 + nseg * 12 + 256 + WF_SOBOL_BYTES +
           WF_COUNTER_BYTES + 512 +
           (WF_TIMING ? (size_t)64 * 1024 * 1024 : 0);
}
// The two path-state sets of a batch (entries are indexed up to npad: a block's
// live paths are compacted to the front of its 256 entries).
struct WfLayout {
    WfBufs b;
    PathSet set[2];
};
static WfLayout wf_layout(char* base, size_t n) {
    WfLayout L;
    WfBufs& b = L.b;
    const size_t npad = (n + 255) / 256 * 256;
    size_t off = 0;
    for (PathSet& ps : L.set) {
        float4** f4[] = {&ps.P0, &ps.P1, &ps.P2, &ps.P3, &ps.P4, &ps.P5, &ps.P6, &ps.P7};
        for (float4** q : f4) {
            *q = reinterpret_cast<float4*>(base + off); off += npad * 16;
        }
        ps.bcount = reinterpret_cast<uint32_t*>(base + off); off += (npad / 256) * 4;
        off = (off + 255) & ~(size_t)255;
    }
    b.rd = L.set[1];
    b.wr = L.set[0];
    b.hit = reinterpret_cast<int*>(base + off); off += n * 4;
    b.occ = reinterpret_cast<uint8_t*>(base + off); off += n * 2;
    off = (off + 255) & ~(size_t)255;
    b.npad = (uint32_t)((n + 255) / 256 * 256);
    b.nseg_k = b.npad / 256;
    // ray records of the queued kind (env shadow rays; the others are traced from the state)
    const size_t rec = (size_t)b.npad * 16;
    b.rayO = reinterpret_cast<float4*>(base + off); off += rec;
    b.rayD = reinterpret_cast<float4*>(base + off); off += rec;
    b.segcount = reinterpret_cast<unsigned int*>(base + off); off += (size_t)b.nseg_k * 12;
    off = (off + 255) & ~(size_t)255;
    b.sobol = reinterpret_cast<float2*>(base + off); off += WF_SOBOL_BYTES;
    b.counter = reinterpret_cast<unsigned int*>(base + off);               // WF_QSHARDS counters, WF_QSTRIDE dwords apart
    b.stats = reinterpret_cast<unsigned long long*>(base + off + WF_COUNTER_BYTES);
    b.n = (uint32_t)n;
    return L;
}

// Trace grid for a batch of n paths: small batches (a rank's share of a
// multi-GPU frame) take a proportional part of the chip, and no launch more than
// WF_TRACE_GRID_PCT % (WF_TRACE_GRID_PCT_LARGE % for large batches), so the calls
// in flight trace side by side instead of queueing.  A call submitted while no
// other call is in flight (`alone`: an interactive loop that waits for every
// frame, the reference's own 512x512 one-frame dispatch) has the chip to itself:
// full occupancy, one block per WF_TRACE_PATHS_PER_BLOCK_ALONE paths.
static unsigned trace_grid_for(const pnrt_ctx* c, size_t n, bool alone = false, bool one = false, bool cc = false) {
    const unsigned pct = (c->serial || alone) ? 100u : one ? WF_TRACE_GRID_PCT_ONE : n < (size_t)WF_SMALL_CALL_PATHS ? WF_TRACE_GRID_PCT : WF_TRACE_GRID_PCT_LARGE;
    // (cc: the lone calls' instantiation, resident at its own occupancy -- no block waits for a slot)
    const size_t gmax = (size_t)(cc && c->trace_grid_cc > 0 ? c->trace_grid_cc : c->trace_grid) * pct / 100;
    const size_t ppb = alone ? WF_TRACE_PATHS_PER_BLOCK_ALONE : WF_TRACE_PATHS_PER_BLOCK;
    return ppb ? (unsigned)std::min<size_t>(gmax, std::max<size_t>(64, (n + ppb - 1) / ppb)) : (unsigned)gmax;
}

// WF_STATS / WF_TIMING builds: the trace launch's census / per-wave drain
// timestamps, printed to stderr (tools/census.py, tools/trace_stats.py)
static int report_trace_diag(pnrt_ctx* c, const WfBufs& b, hipStream_t st, int bounce, unsigned grid) {
    if (WF_TIMING) {   // tail census: when the queue ran dry vs when the last wave ended
        const size_t nw = (size_t)grid * (WF_TRACE_BLOCK / 64);   // waves launched
        std::vector<unsigned long long> t(4 * nw);
        HIPCHK(c, hipStreamSynchronize(st));
        HIPCHK(c, hipMemcpy(t.data(), b.stats + 8, t.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, tex = ~0ull, tend = 0;
        std::vector<unsigned long long> ends;
        for (size_t w = 0; w < nw; ++w) {
            t0 = std::min(t0, t[4 * w]);
            if (t[4 * w + 1]) tex = std::min(tex, t[4 * w + 1]);
            tend = std::max(tend, t[4 * w + 2]);
            ends.push_back(t[4 * w + 2]);
        }
        std::sort(ends.begin(), ends.end());
        auto us = [&](unsigned long long v) { return (double)(v - t0) / 100.0; };
        fprintf(stderr, "[trace timing] bounce %d n=%u first-empty %.1f us, wave ends p10 %.1f p50 %.1f p90 %.1f "
                "max %.1f us\n", bounce, b.n, us(tex), us(ends[nw / 10]), us(ends[nw / 2]), us(ends[nw * 9 / 10]),
                us(tend));
        // the slowest 1 % of waves: end time and their longest last ray (kind, lane steps)
        std::vector<std::pair<unsigned long long, unsigned long long>> we;
        for (size_t w = 0; w < nw; ++w) we.push_back({t[4 * w + 2], w});
        std::sort(we.begin(), we.end());
        fprintf(stderr, "[trace tail] bounce %d (end us, kind/lane steps of the last ray, iterations and us after the queue ran dry):", bounce);
        for (size_t q = nw - std::max<size_t>(1, nw / 100); q < nw; q += std::max<size_t>(1, nw / 1000)) {
            const size_t w = we[q].second;
            const unsigned long long v = t[4 * w + 3];
            fprintf(stderr, " %.0f:k%llu/%llu:%llu/%.0f", us(t[4 * w + 2]), (v >> 16) & 0xffff, v & 0xffff, v >> 32,
                    (double)(t[4 * w + 2] - t[4 * w + 1]) / 100.0);
        }
        fprintf(stderr, "\n");
    }
    if (WF_DIAG_COOP) {   // cooperative-finish hand-overs of the launch (tests/test_gpu_coop.py)
        unsigned long long cc[5];
        HIPCHK(c, hipStreamSynchronize(st));
        HIPCHK(c, hipMemcpy(cc, b.stats, sizeof cc, hipMemcpyDeviceToHost));
        fprintf(stderr, "[coop] bounce %d n=%u anyhit=%llu closest=%llu restarts=%llu multi=%llu deep=%llu\n", bounce, b.n,
                cc[0], cc[1], cc[2], cc[3], cc[4]);
    }
    if (WF_DIAG_COOPSTAT) {   // the lone calls' drain finish (pt_wf.h): finishes, rays, waves it could not take
        unsigned long long cc[9];
        HIPCHK(c, hipStreamSynchronize(st));
        HIPCHK(c, hipMemcpy(cc, b.stats, sizeof cc, hipMemcpyDeviceToHost));
        fprintf(stderr, "[coopstat] bounce %d n=%u finishes=%llu rays=%llu deep_stacks=%llu given_back=%llu\n", bounce, b.n,
                cc[5], cc[8], cc[6], cc[7]);
    }
    if (WF_STATS) {
        unsigned long long stt[8 + 48 + 8];
        HIPCHK(c, hipStreamSynchronize(st));
        HIPCHK(c, hipMemcpy(stt, b.stats, sizeof stt, hipMemcpyDeviceToHost));
        // shadow rays the bounce's setup found moot (pt_wf.h WF_SKIP_MOOT: not traced)
        fprintf(stderr, "[trace moot] bounce %d light=%llu env=%llu cont=%llu\n", bounce, stt[56], stt[57], stt[58]);
        HIPCHK(c, hipMemsetAsync(b.stats + 56, 0, 64, st));
        for (int k = 0; k < 3; ++k) {        // lane steps per ray, log2 buckets, by ray kind
            fprintf(stderr, "[trace hist] bounce %d kind %d:", bounce, k);
            for (int q = 0; q < 16; ++q) fprintf(stderr, " %llu", stt[8 + 16 * k + q]);
            fprintf(stderr, "\n");
        }
        fprintf(stderr, "[trace stats] bounce %d n=%u iters=%llu active/iter=%.1f tri=%llu node=%llu uniform-fetch iters=%llu "
                "refills=%llu rays=%llu  lane-steps/ray=%.1f  continuation lane-steps=%.1f%%\n", bounce, b.n, stt[0],
                stt[0] ? (double)stt[1] / stt[0] : 0.0, stt[2], stt[3], stt[4], stt[5], stt[6],
                stt[6] ? (double)stt[1] / stt[6] : 0.0, stt[1] ? 100.0 * stt[7] / stt[1] : 0.0);
    }
    return PNRT_OK;
}

// One batch of frames (gen -> {trace -> shade/setup} x depth) on one stream;
// its colours land in frame slots [0, cf) of `colors`.
static int render_batch(pnrt_ctx* c, const DevScene& s, const FrameParams& fp, const WfLayout& L, hipStream_t st,
                        const float4* primary, float4* colors, bool alone, bool one, hipEvent_t stage = nullptr) {
    WfBufs b = L.b;
    if (b.n > WF_META_SLOT) return set_err(c, PNRT_E_ARG, "render: too many paths per batch");
    // the cooperative finish of closest-hit rays pays where the drain leaves the chip
    // idle -- a call with nothing else in flight (the reference's loop: D2 sync -19 %);
    // beside other calls' kernels the wave's 64 lanes on one ray cost more than they
    // save (C2 -2.3 %), so pipelined calls run the instantiation without it
    // (only for batches below WF_CC_MAX_PATHS: the lone call's instantiation runs at
    // WF_TRACE_WAVES_CC waves per SIMD, fewer than a large batch's stepping wants)
    const bool cc = alone && WF_COOP_TAIL >= 2 && (size_t)b.n < (size_t)WF_CC_MAX_PATHS;
    const dim3 g((unsigned)((b.n + 255) / 256));
    b.wr = L.set[0];
    if (WF_STATS) HIPCHK(c, hipMemsetAsync(b.stats + 56, 0, 64, st));    // the setups' moot-ray counts
    {   // path state + bounce-0 sampling
        ProfScope ps(c, PNRT_K_GEN, st);
        hipLaunchKernelGGL(pt_wf_gen_setup, g, dim3(256), 0, st, s, fp, b, primary, colors);
    }
    HIPCHK(c, hipGetLastError());
    const unsigned tg = trace_grid_for(c, b.n, alone, one, cc && !s.has_leaf_table);
    // (launch position 2 b: bounce b's trace, 2 b + 1: its shade)
    const int stage_at = std::max(2 * fp.max_depth - WF_STAGGER, 0);
    for (int bounce = 0; bounce < fp.max_depth; ++bounce) {
        if (stage && 2 * bounce == stage_at) HIPCHK(c, hipEventRecord(stage, st));
        // segment dequeue counters: zeroed by the setup kernel that queued the rays
        // (the census builds also clear their words)
        if (WF_STATS || WF_TIMING || WF_DIAG_COOP || WF_DIAG_COOPSTAT)
            HIPCHK(c, hipMemsetAsync(b.counter, 0, WF_COUNTER_BYTES + (WF_STATS ? 448 : 512), st));
        {
            ProfScope ps(c, PNRT_K_TRACE, st);
            if (s.has_leaf_table)       // (the kernel is instantiated per scene kind)
                hipLaunchKernelGGL((pt_wf_trace<WF_STACK, true>), dim3(tg), dim3(WF_TRACE_BLOCK), 0, st, s, b, fp.mode);
            else if (cc)
                hipLaunchKernelGGL((pt_wf_trace<WF_STACK, false, true>), dim3(tg), dim3(WF_TRACE_BLOCK), 0, st, s, b, fp.mode);
            else hipLaunchKernelGGL((pt_wf_trace<WF_STACK, false>), dim3(tg), dim3(WF_TRACE_BLOCK), 0, st, s, b, fp.mode);
        }
        HIPCHK(c, hipGetLastError());
        if (WF_STATS || WF_TIMING || WF_DIAG_COOP || WF_DIAG_COOPSTAT)
            if (int rc = report_trace_diag(c, b, st, bounce, tg)) return rc;
        if (stage && 2 * bounce + 1 == stage_at) HIPCHK(c, hipEventRecord(stage, st));
        {
            ProfScope ps(c, PNRT_K_SHADE, st);
            // MIS + continuation, then the next bounce's sampling (sets alternate)
            b.rd = L.set[bounce & 1];
            b.wr = L.set[(bounce + 1) & 1];
            if (bounce + 1 == fp.max_depth)   // every path ends: no setup half, no rays
                hipLaunchKernelGGL(pt_wf_shade_setup<true>, g, dim3(256), 0, st, s, fp, b, primary, colors);
            else
                hipLaunchKernelGGL(pt_wf_shade_setup<false>, g, dim3(256), 0, st, s, fp, b, primary, colors);
        }
        HIPCHK(c, hipGetLastError());
    }
    if (stage && fp.max_depth <= 0) HIPCHK(c, hipEventRecord(stage, st));
    return PNRT_OK;
}

static int pipes_init(pnrt_ctx* c) {
    if (c->pipes_ready) return PNRT_OK;
    c->pipes_ready = true;
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    const int hw_queues = (q && atoi(q) > 0) ? atoi(q) : 4;
    c->n_pipes_small = hw_queues > 4 ? WF_PIPES : WF_PIPES_LARGE;
    // a caller short of device memory (another tenant, a smaller part) caps one batch's
    // buffers; frames per batch shrink to fit, which changes no pixel
    const char* bb = getenv("PNRT_BATCH_BYTES");
    c->batch_bytes_cap = bb ? (size_t)strtoull(bb, nullptr, 10) : 0;
    for (unsigned i = 0; i < c->n_pipes_small; ++i) {
        auto& P = c->pipe[i];
        HIPCHK(c, hipStreamCreateWithFlags(&P.w, hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&P.ev_join, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&P.ev_blend, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&P.ev_stage, hipEventDisableTiming));
    }
    return PNRT_OK;
}

// v3 wavefront, one pnrt_render call on a pipe: the primary pass (unless the
// pipe's records are still valid, PrimKey), then per group of <= WF_MAX_CHUNK_FRAMES frames one
// batch (gen -> {trace -> shade} x depth) on the pipe's worker stream, then the
// frame-ordered blend on the context stream.  Consecutive calls are independent
// path sets, so running them concurrently changes nothing in the result; the
// blends keep frame order.
static int render_wavefront(pnrt_ctx* c, const DevScene& s, const FrameParams& fp, uint32_t first, uint32_t nf) {
    int rc;
    if ((rc = pipes_init(c))) return rc;
    const size_t pix = (size_t)fp.rows * c->width;
    const int tiles_x = (c->width + 7) / 8, tiles_y = (fp.rows + 7) / 8;
    const size_t per_frame = (size_t)tiles_x * tiles_y * 64;
    // frames per batch: at most WF_MAX_CHUNK_FRAMES, and few enough that every path
    // slot fits the path state's slot field (large frames take fewer per batch)
    if (per_frame > (size_t)WF_META_SLOT) return set_err(c, PNRT_E_ARG, "render: frame too large for one batch");
    const uint32_t fit = (uint32_t)std::min<size_t>(WF_MAX_CHUNK_FRAMES, (size_t)WF_META_SLOT / per_frame);
    uint32_t chunk = nf < fit ? nf : fit;
    // (PNRT_BATCH_BYTES: one batch's path state and colours within the cap, down to one frame)
    while (c->batch_bytes_cap && chunk > 1 &&
           wf_bytes(per_frame * chunk) + pix * 16 * chunk > c->batch_bytes_cap)
        chunk = (chunk + 1) / 2;
    // calls in flight by call size (paths per batch): small (< 5M: multi-GPU shares)
    // 4 with > 4 hardware queues; 5M-12M 2 -- their launches are long enough to fill
    // each other's drains (measured on 8-frame 1080p calls before the staggering: C2
    // +1.8 %, C3 +2.7 %, C4 +1.6 % against 3).
    // From 12M (1080p calls of 6+ frames, 4K calls) the calls are staggered (round 4):
    // two pipes, the full trace grid, and a call starts only when the previous one
    // has finished its second-to-last trace launch, so the two overlap just in the
    // drain-heavy end (last shade / trace / shade / blend) instead of contending for
    // the chip throughout (same box, 2 rounds: C2 +2.5 %, C3 +3.3 %, C4 +1.2 %, C5
    // +1.1 %; one call in flight: C2 +1.8 %, C4 -1.8 %).
    // Without staggering (WF_STAGGER 0): 2 pipes up to 32M, 3 above.
    const size_t call_paths = per_frame * chunk;
    const bool stagger = !c->serial && WF_STAGGER > 0 && call_paths >= (size_t)WF_STAGGER_PATHS;
    const bool one = c->serial || stagger;       // the trace launch may take the whole chip
    const unsigned want = stagger ? 2u : one ? 1u
                        : call_paths < (size_t)WF_SMALL_CALL_PATHS ? c->n_pipes_small
                        : call_paths < (size_t)WF_HUGE_CALL_PATHS ? WF_PIPES_MEDIUM : WF_PIPES_LARGE;
    const unsigned npipes = std::max(1u, std::min(want, c->n_pipes_small));   // only sets pipes_init made
    // no other call in flight: every pipe's last blend (its last work) has completed
    bool alone = !c->serial;
    for (auto& Q : c->pipe)
        if (alone && Q.blend_pending && hipEventQuery(Q.ev_blend) != hipSuccess) alone = false;
    // A call with nothing in flight stays on the last call's pipe (its buffers are
    // free, its primary records likely still valid, its lines still in the caches);
    // otherwise the calls rotate over the pipes
    const unsigned prev_pipe = c->last_pipe;
    const unsigned pi = (alone && c->last_pipe < npipes) ? c->last_pipe : c->next_pipe % npipes;
    c->next_pipe = (pi + 1) % npipes;
    c->last_pipe = pi;
    pnrt_ctx::Pipe& P = c->pipe[pi];
    if (c->trace_grid == 0) {
        int per_cu = 0, cus = 0;
        HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pt_wf_trace<WF_STACK, false>, WF_TRACE_BLOCK, 0));
        HIPCHK(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        c->trace_grid = (per_cu > 0 ? per_cu : 1) * cus;
        int per_cu_cc = 0;
        HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_cc, pt_wf_trace<WF_STACK, false, true>, WF_TRACE_BLOCK, 0));
        c->trace_grid_cc = std::min(c->trace_grid, (per_cu_cc > 0 ? per_cu_cc : 1) * cus);
    }
    // per-lane spill area of the trace kernel's stack: LDS holds WF_STACK entries
    const int ovf_stride = c->wf_stack_need > WF_STACK ? c->wf_stack_need - WF_STACK : 1;
    const size_t ovf_bytes = (size_t)c->trace_grid * WF_TRACE_BLOCK * ovf_stride * 8;
    // every buffer set this call size rotates over is sized now, so no later call of
    // the same size reallocates (a reallocation waits for all calls in flight)
    for (unsigned q = 0; q < npipes; ++q) {
        pnrt_ctx::Pipe& Q = c->pipe[(pi + q) % npipes];
        const float4* old_primary = Q.primary;
        if ((rc = grow(c, (void**)&Q.primary, &Q.primary_cap, pix * 48)) ||
            (rc = grow(c, (void**)&Q.colors, &Q.colors_cap, pix * 16 * chunk)) ||
            (rc = grow(c, &Q.wf, &Q.wf_cap, wf_bytes(per_frame * chunk) + 512)) ||
            (rc = grow(c, (void**)&Q.ovf, &Q.ovf_cap, ovf_bytes)))
            return rc;
        if (Q.primary != old_primary) Q.prim.valid = false;
    }
    ++c->ncall;
    // A call with nothing in flight runs on the caller's stream itself: no worker
    // stream to order against it, so no event wait before its first kernel and no
    // join before its blend (the reference's loop: one frame, then display)
    const bool on_caller = alone && WF_ALONE_ON_CALLER;
    hipStream_t w = on_caller ? c->stream : P.w;
    // this pipe's buffers were last read by the blend of the call that used it last
    // (already complete for a call with nothing in flight: `alone` queried it)
    if (P.blend_pending && !alone) HIPCHK(c, hipStreamWaitEvent(w, P.ev_blend, 0));
    // staggered calls: this one starts when the previous one reaches its last bounces
    if (stagger && !alone && prev_pipe != pi && prev_pipe < WF_PIPES && c->pipe[prev_pipe].stage_set)
        HIPCHK(c, hipStreamWaitEvent(w, c->pipe[prev_pipe].ev_stage, 0));
    P.stage_set = false;
    // The primary records (camera ray's closest hit per pixel of the shard) depend
    // on the camera, the frame size, the shard, the traversal mode and the scene
    // (scene_epoch: arrays, materials, environment) -- not on the frame number: the
    // camera ray has no jitter (ray_tracing.comp:205-211, 980).  A pipe whose
    // records were traced for the same key reuses them (read-only since), exactly.
    pnrt_ctx::PrimKey key;
    key.epoch = c->scene_epoch;
    std::memcpy(key.cam, fp.eye, 12); std::memcpy(key.cam + 3, fp.llc, 12);
    std::memcpy(key.cam + 6, fp.hor, 12); std::memcpy(key.cam + 9, fp.ver, 12);
    key.width = fp.width; key.height = fp.height; key.rows = fp.rows;
    key.band = fp.band; key.n_shards = fp.n_shards; key.shard = fp.shard; key.mode = fp.mode;
    key.valid = true;
    const bool prim_hit = P.prim.valid && P.prim.epoch == key.epoch && !std::memcmp(P.prim.cam, key.cam, sizeof key.cam) &&
                          P.prim.width == key.width && P.prim.height == key.height && P.prim.rows == key.rows &&
                          P.prim.band == key.band && P.prim.n_shards == key.n_shards && P.prim.shard == key.shard &&
                          P.prim.mode == key.mode;
    if (!prim_hit) {
        ProfScope ps(c, PNRT_K_PRIMARY, w);
        // the trace kernel's step, grid-stride, the pipe's spill area
        WfBufs pb{};
        pb.ovf = P.ovf;
        pb.fault = c->fault_dev;
        pb.ovf_stride = (uint32_t)ovf_stride;
        const unsigned gp = (unsigned)std::min<size_t>((pix + WF_TRACE_BLOCK - 1) / WF_TRACE_BLOCK, (size_t)c->trace_grid);
        if (s.has_leaf_table)
            hipLaunchKernelGGL((pt_primary_wf<WF_STACK, true>), dim3(gp), dim3(WF_TRACE_BLOCK), 0, w, s, fp, pb, P.primary);
        else hipLaunchKernelGGL((pt_primary_wf<WF_STACK, false>), dim3(gp), dim3(WF_TRACE_BLOCK), 0, w, s, fp, pb, P.primary);
        HIPCHK(c, hipGetLastError());
        P.prim = key;
    }
    for (uint32_t f0 = 0; f0 < nf; f0 += chunk) {
        const uint32_t cf = (nf - f0) < chunk ? (nf - f0) : chunk;
        WfLayout a = wf_layout(static_cast<char*>(P.wf), per_frame * cf);
        a.b.ovf = P.ovf;
        a.b.fault = c->fault_dev;
        a.b.ovf_stride = (uint32_t)ovf_stride;
        a.b.chunk_frames = (int)cf;
        a.b.tiles_x = tiles_x;
        a.b.first_frame = first + f0;
        if (f0 && w != c->stream) HIPCHK(c, hipStreamWaitEvent(w, P.ev_blend, 0));   // the previous group's blend has read the colours
        const bool last = f0 + cf >= nf;
        if ((rc = render_batch(c, s, fp, a, w, P.primary, P.colors, alone, one, stagger && last ? P.ev_stage : nullptr)))
            return rc;
        if (stagger && last) P.stage_set = true;
        if (w != c->stream) {
            HIPCHK(c, hipEventRecord(P.ev_join, w));
            HIPCHK(c, hipStreamWaitEvent(c->stream, P.ev_join, 0));
        }
        {   // the blends run in call order on the caller's stream
            ProfScope ps(c, PNRT_K_BLEND);
            hipLaunchKernelGGL(pt_blend_kernel, dim3((unsigned)((pix + 255) / 256)), dim3(256), 0, c->stream, fp,
                               (const float4*)P.colors, c->accum, (int)cf, first + f0);
        }
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(P.ev_blend, c->stream));
        P.blend_pending = true;
        if ((rc = mark_stream(c))) return rc;
    }
    return PNRT_OK;
}

static void free_env(pnrt_ctx* c);

extern "C" {

#ifndef PNRT_SRC_HASH
#define PNRT_SRC_HASH "unknown"
#endif
// the build stamps the sha256 of the device sources (pnraytracing_amd/build.py),
// so a stale prebuilt library shipped beside newer sources is detectable
const char* pnrt_version(void) {
    return PNRT_IS_DIAG_BUILD ? "pnrt-mi355x 0.2 (gfx950) DIAGNOSTIC BUILD src " PNRT_SRC_HASH
                              : "pnrt-mi355x 0.2 (gfx950) src " PNRT_SRC_HASH;
}

int pnrt_create(int device, pnrt_ctx** out) {
    if (!out) return PNRT_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PNRT_E_HIP;
    pnrt_ctx* c = new pnrt_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return PNRT_E_HIP;
    }
    c->stream = c->own_stream;
    // the pipelined renderer's worker streams are created with the context, so
    // they take hardware queues of their own before the caller creates more streams
    if (pipes_init(c) != PNRT_OK) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PNRT_E_HIP;
    }
    void* fh = nullptr;
    void* fd = nullptr;
    if (hipHostMalloc(&fh, 256, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&fd, fh, 0) != hipSuccess) {
        if (fh) (void)hipHostFree(fh);
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PNRT_E_HIP;
    }
    std::memset(fh, 0, 256);
    c->fault_host = static_cast<uint32_t*>(fh);
    c->fault_dev = static_cast<uint32_t*>(fd);
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_sobolV), kSobolV, sizeof kSobolV) != hipSuccess) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PNRT_E_HIP;
    }
    float lut[256];
    for (int i = 0; i < 256; ++i) lut[i] = (float)i / 255.0f;   // GL UNORM8 -> float
    if (hipMalloc(&c->unorm8, sizeof lut) != hipSuccess ||
        hipMemcpy(c->unorm8, lut, sizeof lut, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PNRT_E_HIP;
    }
    *out = c;
    return PNRT_OK;
}

void pnrt_destroy(pnrt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)sync_all(c);
    free_scene(c);
    free_env(c);
    for (void* t : c->tex) (void)hipFree(t);
    (void)hipFree(c->unorm8);
    (void)hipFree(c->accum);
    (void)sync_all(c);
    for (auto& P : c->pipe) {
        (void)hipFree(P.primary); (void)hipFree(P.colors); (void)hipFree(P.wf); (void)hipFree(P.ovf);
        if (P.w) (void)hipStreamDestroy(P.w);
        if (P.ev_join) (void)hipEventDestroy(P.ev_join);
        if (P.ev_blend) (void)hipEventDestroy(P.ev_blend);
        if (P.ev_stage) (void)hipEventDestroy(P.ev_stage);
    }

    for (auto& p : c->ev_pending) { c->ev_pool.push_back(p.second.first); c->ev_pool.push_back(p.second.second); }
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->ev_last) (void)hipEventDestroy(c->ev_last);
    if (c->fault_host) (void)hipHostFree(c->fault_host);
    (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* pnrt_last_error(pnrt_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* pnrt_get_stream(pnrt_ctx* c) { return c ? static_cast<void*>(c->own_stream) : nullptr; }

int pnrt_set_stream(pnrt_ctx* c, void* s) {
    if (!c) return PNRT_E_ARG;
    hipStream_t ns = s ? static_cast<hipStream_t>(s) : c->own_stream;
    if (ns == c->stream) return PNRT_OK;
    // blends (frame-ordered read-modify-writes of accum), pack_rows and
    // read_accum run on c->stream: the new stream starts after the last op the
    // context queued on the old one (ev_last, recorded with it), so no blend of
    // a later call overtakes a pending one -- and the old stream itself is not
    // touched (the caller may have destroyed it since)
    HIPCHK(c, hipSetDevice(c->device));
    if (c->last_valid) HIPCHK(c, hipStreamWaitEvent(ns, c->ev_last, 0));
    c->stream = ns;
    return PNRT_OK;
}

int pnrt_set_options(pnrt_ctx* c, int options) {
    if (!c) return PNRT_E_ARG;
    int mode = options & 0xff;
    if ((mode != PNRT_TRAVERSE_EXACT && mode != PNRT_TRAVERSE_ZCULL) || (options & ~0x3ff))
        return set_err(c, PNRT_E_ARG, "unknown option bits");
    c->mode = mode;
    c->kernel = (options & PNRT_KERNEL_V1) ? 1 : 3;
    const bool serial = (options & PNRT_SERIAL) != 0;
    if (serial != c->serial) HIPCHK(c, sync_all(c));   // the pipe rotation restarts from an idle context
    c->serial = serial;
    return PNRT_OK;
}

// DevScene::emit_max (pt_wf.h WF_SKIP_MOOT): a bound on every component of the
// emission a continuation ray can bring back -- any material's, or the env
// radiance (bilinear taps of the texels: 2^-16 above the largest texel covers the
// filter's rounding).  A NaN anywhere makes it NaN (then nothing is found moot).
static float abs_max(const float* v, size_t n, float m) {
    for (size_t k = 0; k < n; ++k) {
        const float a = std::fabs(v[k]);
        if (std::isnan(a) || std::isnan(m)) return std::numeric_limits<float>::quiet_NaN();
        m = std::max(m, a);
    }
    return m;
}
static void set_emit_max(pnrt_ctx* c) {
    float m = abs_max(c->mat_emit.data(), c->mat_emit.size(), 0.f);
    if (c->scene.has_hdr) {
        const float e = c->env_max * (1.0f + 0x1p-16f);
        m = (std::isnan(e) || std::isnan(m)) ? std::numeric_limits<float>::quiet_NaN() : std::max(m, e);
    }
    c->scene.emit_max = m;
}

int pnrt_upload_scene(pnrt_ctx* c, const float* V, int nv, const float* M, int nm, const float* T, int nt,
                      const float* N, int nn, const float* Lt, int nl, float lsum) {
    if (!c) return PNRT_E_ARG;
    if (!V || !M || !T || !N || nv <= 0 || nm <= 0 || nt <= 0 || nn <= 0 || nl < 0 || (nl > 0 && !Lt))
        return set_err(c, PNRT_E_ARG, "upload_scene: missing or empty arrays");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    free_scene(c);
    c->scene_bytes = 0;
    ++c->scene_epoch;                    // primary records of the old scene are stale

    // triangles: positions gathered in BVH order, ids validated
    std::vector<float4> tris((size_t)nt * 3 + 1);   // +1: the trace kernel reads 64 B per record
    std::vector<int4> tidx(nt);
    for (int i = 0; i < nt; ++i) {
        const float* t = T + 6 * (size_t)i;
        int id[3] = {fint(t[0]), fint(t[1]), fint(t[2])};
        for (int k = 0; k < 3; ++k)
            if (id[k] < 0 || id[k] >= nv) return set_err(c, PNRT_E_SCENE, "triangle " + std::to_string(i) + " has an out-of-range vertex index");
        int mat = fint(t[3]), tex = fint(t[4]);
        if (mat < 0 || mat >= nm) return set_err(c, PNRT_E_SCENE, "triangle " + std::to_string(i) + " has an out-of-range material id");
        const float* p0 = V + 15 * (size_t)id[0];
        const float* p1 = V + 15 * (size_t)id[1];
        const float* p2 = V + 15 * (size_t)id[2];
        float4 a, b, d;
        a.x = p0[0]; a.y = p0[1]; a.z = p0[2]; a.w = p1[0];
        b.x = p1[1]; b.y = p1[2]; b.z = p2[0]; b.w = p2[1];
        int mb, tb; std::memcpy(&mb, &mat, 4); std::memcpy(&tb, &tex, 4);
        d.x = p2[2];
        std::memcpy(&d.y, &mat, 4); std::memcpy(&d.z, &tex, 4); d.w = 0.f;
        (void)mb; (void)tb;
        tris[3 * (size_t)i] = a; tris[3 * (size_t)i + 1] = b; tris[3 * (size_t)i + 2] = d;
        tidx[i] = make_int4(id[0], id[1], id[2], 0);
    }
    std::vector<float4> verts((size_t)nv * 2);
    for (int i = 0; i < nv; ++i) {
        const float* v = V + 15 * (size_t)i;
        verts[2 * (size_t)i] = make_float4(v[0], v[1], v[2], v[3]);
        verts[2 * (size_t)i + 1] = make_float4(v[4], v[5], v[12], v[13]);
    }
    // per-triangle shading attributes (normals, uvs of its three vertices), so a
    // hit's attributes are one fetch away from the triangle index instead of two
    std::vector<float4> tattr((size_t)nt * 4);
    for (int i = 0; i < nt; ++i) {
        const float* v0 = V + 15 * (size_t)tidx[i].x;
        const float* v1 = V + 15 * (size_t)tidx[i].y;
        const float* v2 = V + 15 * (size_t)tidx[i].z;
        tattr[4 * (size_t)i + 0] = make_float4(v0[3], v0[4], v0[5], v1[3]);
        tattr[4 * (size_t)i + 1] = make_float4(v1[4], v1[5], v2[3], v2[4]);
        tattr[4 * (size_t)i + 2] = make_float4(v2[5], v0[12], v0[13], v1[12]);
        tattr[4 * (size_t)i + 3] = make_float4(v1[13], v2[12], v2[13], 0.f);
    }
    // BVH: validate the reference tree (pre-order, left = id + 1) from the root,
    // number interior nodes, and store child boxes in the parent.
    std::vector<int> dn(nn, -1), depth(nn, 0), order;
    std::vector<int> st{0};
    std::vector<char> seen(nn, 0);
    int maxd = 0;
    while (!st.empty()) {
        int i = st.back(); st.pop_back();
        if (i < 0 || i >= nn || seen[i]) return set_err(c, PNRT_E_SCENE, "BVH node array is not a tree");
        seen[i] = 1;
        const float* n = N + 12 * (size_t)i;
        int rc = fint(n[7]), s0 = fint(n[8]), e0 = fint(n[9]);
        if (rc == -1) {
            if (s0 < 0 || e0 > nt || s0 > e0) return set_err(c, PNRT_E_SCENE, "BVH leaf with bad triangle range");
            continue;
        }
        int ax = fint(n[6]);
        if (ax < 0 || ax > 2 || i + 1 >= nn || rc <= 0 || rc >= nn) return set_err(c, PNRT_E_SCENE, "BVH interior node with bad axis/children");
        dn[i] = (int)order.size();
        order.push_back(i);
        depth[i + 1] = depth[rc] = depth[i] + 1;
        if (depth[i] + 1 > maxd) maxd = depth[i] + 1;
        st.push_back(rc);
        st.push_back(i + 1);
    }
    if (maxd >= PT_STACK - 1)
        return set_err(c, PNRT_E_SCENE, "BVH depth " + std::to_string(maxd) + " exceeds the kernel stack");
    // device numbering: breadth-first, so the top levels are the first indices
    // (the top levels share cache lines); the visit order is
    // carried by the child refs and the axis, not by the numbering
    order.clear();
    if (fint(N[7]) != -1) order.push_back(0);
    for (size_t q = 0; q < order.size(); ++q) {
        const int i = order[q];
        dn[i] = (int)q;
        const float* n = N + 12 * (size_t)i;
        const int rc = fint(n[7]);
        if (fint(N[12 * (size_t)(i + 1) + 7]) != -1) order.push_back(i + 1);
        if (fint(N[12 * (size_t)rc + 7]) != -1) order.push_back(rc);
    }
    // child reference (pt_common.h): interior -> node index, leaf -> range, in the
    // packed encoding when every leaf fits it, else the wide one (+ leaf table)
    bool packed = nt < (1 << 24) - 1;
    for (size_t i = 0; i < (size_t)nn && packed; ++i) {
        const float* n = N + 12 * i;
        if (fint(n[7]) == -1 && fint(n[9]) - fint(n[8]) > 127) packed = false;
    }
    std::vector<int2> leaf_table;
    auto childref = [&](int ci) -> uint32_t {
        const float* n = N + 12 * (size_t)ci;
        if (fint(n[7]) != -1) return (uint32_t)dn[ci];
        int s0 = fint(n[8]), cnt = fint(n[9]) - s0;
        if (cnt <= 0) return REF_LEAF;
        if (packed) return REF_LEAF | ((uint32_t)cnt << 24) | (uint32_t)s0;
        if (cnt <= 127 && s0 < (1 << 23)) return REF_LEAF | ((uint32_t)s0 << 7) | (uint32_t)cnt;
        leaf_table.push_back(make_int2(s0, cnt));
        return REF_LEAF | REF_TABLE | (uint32_t)(leaf_table.size() - 1);
    };
    if ((int64_t)order.size() >= (1 << 25)) return set_err(c, PNRT_E_SCENE, "too many BVH nodes (2 GB node buffer limit)");
    if (nm >= (1 << 24)) return set_err(c, PNRT_E_SCENE, "too many materials");
    std::vector<float4> nodes(order.size() * 4);
    for (size_t k = 0; k < order.size(); ++k) {
        int i = order[k];
        const float* n = N + 12 * (size_t)i;
        int rc = fint(n[7]);
        const float* L = N + 12 * (size_t)(i + 1);
        const float* R = N + 12 * (size_t)rc;
        nodes[4 * k + 0] = make_float4(L[0], L[1], L[2], L[3]);
        nodes[4 * k + 1] = make_float4(L[4], L[5], R[0], R[1]);
        nodes[4 * k + 2] = make_float4(R[2], R[3], R[4], R[5]);
        uint32_t meta[4] = {childref(i + 1), childref(rc), 16u << fint(n[6]), (uint32_t)fint(n[6])};
        std::memcpy(&nodes[4 * k + 3], meta, 16);
    }
    uint32_t root_ref = childref(0);
    const int has_leaf_table = packed ? 0 : 1;
    if (leaf_table.empty()) leaf_table.push_back(make_int2(0, 0));

    // trace-kernel stack bound: at most one deferred sibling per BVH level
    c->wf_stack_need = maxd + 2;
    std::vector<float2> lights(nl > WF_LIGHT_SCAN ? nl : WF_LIGHT_SCAN, make_float2(0.f, 0.f));
    for (int i = 0; i < nl; ++i) {
        lights[i] = make_float2(Lt[3 * (size_t)i], Lt[3 * (size_t)i + 1]);
        int li = fint(Lt[3 * (size_t)i]);
        if (li < 0 || li >= nt) return set_err(c, PNRT_E_SCENE, "light references an out-of-range triangle");
    }
    std::vector<float> mats(M, M + 18 * (size_t)nm);
    // light records: what TriangleSample (:598-624) and the emission (:887) read for
    // light entry k -- its triangle's vertex records and material emission -- in one
    // place; entry nl is triangle 0 (GetLightIndex's fallback index)
    std::vector<float4> lrec((size_t)(nl + 1) * 7);
    c->light_mat.assign((size_t)nl + 1, 0);
    for (int e = 0; e <= nl; ++e) {
        const int t = e < nl ? fint(Lt[3 * (size_t)e]) : 0;
        for (int k = 0; k < 3; ++k) {
            const int vi = k == 0 ? tidx[t].x : (k == 1 ? tidx[t].y : tidx[t].z);
            lrec[7 * (size_t)e + 2 * k] = verts[2 * (size_t)vi];
            lrec[7 * (size_t)e + 2 * k + 1] = verts[2 * (size_t)vi + 1];
        }
        const int mat = fint(T[6 * (size_t)t + 3]);
        const float* em = M + 18 * (size_t)mat;
        lrec[7 * (size_t)e + 6] = make_float4(em[0], em[1], em[2], 0.f);
        c->light_mat[e] = mat;
    }
    c->light_rec_host = lrec;

    DevScene& s = c->scene;
    int rc;
    {   // nodes and triangle records in one allocation: the trace kernel addresses both
        // through one buffer resource with 32-bit offsets
        const size_t nb = nodes.size() * 16, tb = tris.size() * 16;
        if (nb + tb >= ((size_t)1 << 32) - 64)
            return set_err(c, PNRT_E_SCENE, "scene too large: nodes + triangles must stay below 4 GiB");
        void* g = nullptr;
        HIPCHK(c, hipMalloc(&g, nb + tb));
        c->scene_allocs.push_back(g);
        if (nb) HIPCHK(c, hipMemcpy(g, nodes.data(), nb, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(static_cast<char*>(g) + nb, tris.data(), tb, hipMemcpyHostToDevice));
        c->scene_bytes += (int64_t)(nb + tb);
        s.nodes = static_cast<const float4*>(g);
        s.tris = reinterpret_cast<const float4*>(static_cast<char*>(g) + nb);
        s.geo_tri_off = (uint32_t)nb;
        s.geo_bytes = (uint32_t)(nb + tb);
    }
    if ((rc = upload(c, leaf_table, &s.leaf_table)) || (rc = upload(c, tidx, &s.tri_idx)) ||
        (rc = upload(c, verts, &s.verts)) || (rc = upload(c, mats, &s.materials)) || (rc = upload(c, lights, &s.lights)) ||
        (rc = upload(c, tattr, &s.tri_attr)) || (rc = upload(c, lrec, &s.light_rec)) ||
        (rc = upload(c, std::vector<float4>(1, make_float4(0.f, 0.f, 0.f, 0.f)), &s.zero4)))
        return rc;
    s.n_nodes = (int)order.size(); s.n_tris = nt; s.n_verts = nv; s.n_materials = nm; s.n_lights = nl;
    s.lights_sum_area = lsum;
    const float* root = N;
    for (int k = 0; k < 3; ++k) { s.root_min[k] = root[k]; s.root_max[k] = root[3 + k]; }
    // z-slab culling's proof needs finite boxes (then a culling-enabled ray's
    // z-slab distances are never NaN); a scene with a non-finite box coordinate
    // is traversed without culling, which is the reference's exact traversal
    c->boxes_finite = true;
    for (size_t i = 0; i < (size_t)nn && c->boxes_finite; ++i)
        for (int k = 0; k < 6; ++k)
            if (!std::isfinite(N[12 * i + k])) { c->boxes_finite = false; break; }
    s.root_ref = root_ref;
    s.has_leaf_table = has_leaf_table;
    s.n_leaf_table = (int)leaf_table.size();
    {   // GetLightIndex is a lower bound: a linear scan returns the same index iff the
        // prefix areas are non-decreasing (they are for main.cpp:374-383's list)
        bool mono = nl <= WF_LIGHT_SCAN;
        for (int k = 1; mono && k < nl; ++k) mono = lights[k].y >= lights[k - 1].y;
        for (int k = 0; mono && k < nl; ++k) mono = lights[k].y == lights[k].y;
        s.light_scan = mono ? 1 : 0;
        for (int k = 0; k < WF_LIGHT_SCAN; ++k) s.lscan[k] = k < nl ? lights[k].y : 0.f;
    }
    c->mat_emit.resize(3 * (size_t)nm);
    for (int m = 0; m < nm; ++m)
        for (int k = 0; k < 3; ++k) c->mat_emit[3 * (size_t)m + k] = M[18 * (size_t)m + k];
    set_emit_max(c);
    c->root_is_leaf = fint(root[7]) == -1;
    c->n_interior = (int)order.size();
    c->max_depth = maxd;
    c->has_scene = true;
    return PNRT_OK;
}

int pnrt_update_materials(pnrt_ctx* c, int first, int count, const float* rec) {
    if (!c) return PNRT_E_ARG;
    if (!c->has_scene) return set_err(c, PNRT_E_STATE, "update_materials: upload_scene first");
    if (first < 0 || count < 0 || first > c->scene.n_materials - count || (count > 0 && !rec))
        return set_err(c, PNRT_E_ARG, "update_materials: material range outside the uploaded array");
    if (count == 0) return PNRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    // the calls in flight render with the old records (the reference's
    // glTexSubImage1D is ordered after the dispatches issued before it)
    HIPCHK(c, sync_all(c));
    HIPCHK(c, hipMemcpy(const_cast<float*>(c->scene.materials) + 18 * (size_t)first, rec, 18 * sizeof(float) * (size_t)count,
                        hipMemcpyHostToDevice));
    // light records carry a copy of their triangle's emission (upload_scene): patched
    // in the host copy, then the span of changed records goes up in ONE copy (an
    // emissive mesh of thousands of light triangles sharing one material is one
    // transfer per edit, as the reference's single glTexSubImage1D)
    size_t lo = c->light_mat.size(), hi = 0;
    for (size_t e = 0; e < c->light_mat.size(); ++e) {
        const int m = c->light_mat[e];
        if (m < first || m >= first + count) continue;
        const float* em = rec + 18 * (size_t)(m - first);
        c->light_rec_host[7 * e + 6] = make_float4(em[0], em[1], em[2], 0.f);
        lo = std::min(lo, e);
        hi = e + 1;
    }
    if (lo < hi)
        HIPCHK(c, hipMemcpy(const_cast<float4*>(c->scene.light_rec) + 7 * lo, c->light_rec_host.data() + 7 * lo,
                            (hi - lo) * 7 * sizeof(float4), hipMemcpyHostToDevice));
    for (int m = 0; m < count; ++m)
        for (int k = 0; k < 3; ++k) c->mat_emit[3 * (size_t)(first + m) + k] = rec[18 * (size_t)m + k];
    set_emit_max(c);
    ++c->scene_epoch;                    // primary records hold the hit material's emission
    return PNRT_OK;
}

int pnrt_upload_texture(pnrt_ctx* c, int slot, const uint8_t* px, int w, int h, int ch) {
    if (!c) return PNRT_E_ARG;
    if (slot < 0 || slot >= PT_MAX_TEXTURES || !px || w <= 0 || h <= 0 || ch < 1 || ch > 4)
        return set_err(c, PNRT_E_ARG, "upload_texture: bad arguments");
    HIPCHK(c, hipSetDevice(c->device));
    // glTexImage2D with the default GL_UNPACK_ALIGNMENT 4 (main.cpp:545): row j
    // starts at j * align4(w * ch) in the caller's tightly packed buffer; bytes
    // past the buffer read as 0.  GL_RED -> (r, 0, 0).
    size_t stride = ((size_t)w * ch + 3) & ~(size_t)3, avail = (size_t)w * h * ch;
    std::vector<uint32_t> texels((size_t)w * h);
    for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i) {
            uint32_t rgb[3] = {0, 0, 0};
            for (int k = 0; k < (ch >= 3 ? 3 : ch); ++k) {
                size_t o = (size_t)j * stride + (size_t)i * ch + k;
                rgb[k] = o < avail ? px[o] : 0;
            }
            texels[(size_t)j * w + i] = rgb[0] | (rgb[1] << 8) | (rgb[2] << 16);
        }
    HIPCHK(c, sync_all(c));             // pipelined calls may still sample the old texture
    (void)hipFree(c->tex[slot]);
    c->tex[slot] = nullptr;
    HIPCHK(c, hipMalloc(&c->tex[slot], texels.size() * 4));
    HIPCHK(c, hipMemcpy(c->tex[slot], texels.data(), texels.size() * 4, hipMemcpyHostToDevice));
    c->tex_w[slot] = w; c->tex_h[slot] = h;
    return PNRT_OK;
}

// Footprint records (DevScene::hdr_q / rnd_q) of a w x h image: record (qj, qi)
// = texels (bottom, left), (bottom, right), (top, left), (top, right) with
// left = clamp(qi - 1), right = clamp(qi), bottom = clamp(qj - 1), top = clamp(qj).
__global__ void env_quad_kernel(const float4* img, int w, int h, float4* q) {
    const size_t n = (size_t)(w + 1) * (h + 1);
    const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int qj = (int)(r / (size_t)(w + 1)), qi = (int)(r - (size_t)qj * (w + 1));
    const int l = qi > 0 ? qi - 1 : 0, rt = qi < w ? qi : w - 1;
    const int bo = qj > 0 ? qj - 1 : 0, tp = qj < h ? qj : h - 1;
    q[4 * r] = img[(size_t)bo * w + l];
    q[4 * r + 1] = img[(size_t)bo * w + rt];
    q[4 * r + 2] = img[(size_t)tp * w + l];
    q[4 * r + 3] = img[(size_t)tp * w + rt];
}

static void free_env(pnrt_ctx* c) {
    (void)hipFree(c->hdr); (void)hipFree(c->rnd); (void)hipFree(c->hdr_q); (void)hipFree(c->rnd_q);
    c->hdr = c->rnd = c->hdr_q = c->rnd_q = nullptr;
}

static int env_quads(pnrt_ctx* c, int w, int h) {
    const size_t n = (size_t)(w + 1) * (h + 1);
    HIPCHK(c, hipMalloc(&c->hdr_q, n * 64));
    HIPCHK(c, hipMalloc(&c->rnd_q, n * 64));
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(env_quad_kernel, dim3(g), dim3(256), 0, c->stream, (const float4*)c->hdr, w, h, (float4*)c->hdr_q);
    hipLaunchKernelGGL(env_quad_kernel, dim3(g), dim3(256), 0, c->stream, (const float4*)c->rnd, w, h, (float4*)c->rnd_q);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PNRT_OK;
}

int pnrt_upload_env(pnrt_ctx* c, const float* rgb, const float* rnd, int w, int h) {
    if (!c) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    free_env(c);
    c->scene.has_hdr = 0;
    set_emit_max(c);
    ++c->scene_epoch;                    // a primary miss records the env colour
    if (!rgb) return PNRT_OK;
    if (!rnd || w <= 0 || h <= 0) return set_err(c, PNRT_E_ARG, "upload_env: bad arguments");
    std::vector<float4> a((size_t)w * h), b((size_t)w * h);
    for (size_t i = 0; i < a.size(); ++i) {
        a[i] = make_float4(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 0.f);
        b[i] = make_float4(rnd[3 * i], rnd[3 * i + 1], rnd[3 * i + 2], 0.f);
    }
    HIPCHK(c, hipMalloc(&c->hdr, a.size() * 16));
    HIPCHK(c, hipMalloc(&c->rnd, b.size() * 16));
    HIPCHK(c, hipMemcpy(c->hdr, a.data(), a.size() * 16, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->rnd, b.data(), b.size() * 16, hipMemcpyHostToDevice));
    if (int rc = env_quads(c, w, h)) return rc;
    c->scene.has_hdr = 1;
    c->scene.hdr_w = w; c->scene.hdr_h = h;
    c->env_max = abs_max(rgb, 3 * (size_t)w * h, 0.f);
    set_emit_max(c);
    return PNRT_OK;
}

int pnrt_upload_env_build(pnrt_ctx* c, const float* rgb, int w, int h) {
    if (!c) return PNRT_E_ARG;
    if (!rgb || w <= 0 || h <= 0) return set_err(c, PNRT_E_ARG, "upload_env_build: bad arguments");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    free_env(c);
    c->scene.has_hdr = 0;
    set_emit_max(c);
    ++c->scene_epoch;                    // a primary miss records the env colour
    const size_t n = (size_t)w * h;
    std::vector<float4> a(n);
    for (size_t i = 0; i < n; ++i) a[i] = make_float4(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 0.f);
    HIPCHK(c, hipMalloc(&c->hdr, n * 16));
    HIPCHK(c, hipMalloc(&c->rnd, n * 16));
    HIPCHK(c, hipMemcpy(c->hdr, a.data(), n * 16, hipMemcpyHostToDevice));
    float* tmp = nullptr;                     // lumY/pdfY | lumX | cdfY | marginX | cdfX | sum
    HIPCHK(c, hipMalloc(&tmp, (3 * n + 2 * (size_t)w + 64) * 4));
    float *pdfY = tmp, *lumX = tmp + n, *cdfY = tmp + 2 * n, *marginX = tmp + 3 * n, *cdfX = marginX + w,
          *sum = cdfX + w;
    const unsigned gp = (unsigned)((n + 255) / 256), gx = (unsigned)((w + 255) / 256);
    hipLaunchKernelGGL(env_lumen_kernel, dim3(gp), dim3(256), 0, c->stream, (const float4*)c->hdr, pdfY, lumX, w, h);
    hipLaunchKernelGGL(env_sum_kernel, dim3(1), dim3(64), 0, c->stream, (const float*)lumX, n, sum);
    hipLaunchKernelGGL(env_margin_kernel, dim3(gx), dim3(256), 0, c->stream, pdfY, (const float*)sum, marginX, w, h);
    hipLaunchKernelGGL(env_cdfx_kernel, dim3(1), dim3(64), 0, c->stream, (const float*)marginX, cdfX, w);
    hipLaunchKernelGGL(env_cdfy_kernel, dim3(gx), dim3(256), 0, c->stream, (const float*)pdfY, (const float*)marginX, cdfY, w, h);
    hipLaunchKernelGGL(env_table_kernel, dim3(gp), dim3(256), 0, c->stream, (const float*)cdfX, (const float*)cdfY,
                       (const float*)pdfY, static_cast<float4*>(c->rnd), w, h);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(tmp);
    if (e != hipSuccess) return set_err(c, PNRT_E_HIP, std::string("upload_env_build: ") + hipGetErrorString(e));
    if (int rc = env_quads(c, w, h)) return rc;
    c->scene.has_hdr = 1;
    c->scene.hdr_w = w; c->scene.hdr_h = h;
    c->env_max = abs_max(rgb, 3 * n, 0.f);
    set_emit_max(c);
    return PNRT_OK;
}

int pnrt_read_env_table(pnrt_ctx* c, float* out) {
    if (!c || !out) return PNRT_E_ARG;
    if (!c->rnd) return set_err(c, PNRT_E_STATE, "read_env_table: no environment");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    const size_t n = (size_t)c->scene.hdr_w * c->scene.hdr_h;
    std::vector<float4> t(n);
    HIPCHK(c, hipMemcpy(t.data(), c->rnd, n * 16, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) { out[3 * i] = t[i].x; out[3 * i + 1] = t[i].y; out[3 * i + 2] = t[i].z; }
    return PNRT_OK;
}

int pnrt_set_frame(pnrt_ctx* c, int w, int h, const pnrt_camera* cam, int depth) {
    if (!c) return PNRT_E_ARG;
    if (w <= 0 || h <= 0 || !cam || depth < 0 || depth > 4)
        return set_err(c, PNRT_E_ARG, "set_frame: bad arguments (MAX_BOUNCE_DEPTH must be 0..4: 8 Sobol dims)");
    HIPCHK(c, hipSetDevice(c->device));
    if (w != c->width || h != c->height || !c->accum) {
        HIPCHK(c, sync_all(c));
        (void)hipFree(c->accum);
        c->accum = nullptr;
        HIPCHK(c, hipMalloc(&c->accum, (size_t)w * h * 16));
        HIPCHK(c, hipMemsetAsync(c->accum, 0, (size_t)w * h * 16, c->stream));
        c->width = w; c->height = h;
        if (int rc = mark_stream(c)) return rc;
    }
    c->cam = *cam;
    c->max_bounce = depth;
    c->has_frame = true;
    return PNRT_OK;
}

static int shard_rows(int h, int band, int n, int shard) {
    int rows = 0;
    for (int y0 = shard * band; y0 < h; y0 += band * n) rows += (h - y0 < band) ? h - y0 : band;
    return rows;
}

int pnrt_render(pnrt_ctx* c, uint32_t first, uint32_t nf, int band, int nsh, int shard) {
    if (!c) return PNRT_E_ARG;
    if (!c->has_scene || !c->has_frame) return set_err(c, PNRT_E_STATE, "render: upload_scene and set_frame first");
    if (band < 1 || nsh < 1 || shard < 0 || shard >= nsh) return set_err(c, PNRT_E_ARG, "render: bad shard selector");
    if (int rc = check_fault(c)) return rc;      // an earlier call's trace fault (completed work)
    if (nf == 0) return PNRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    FrameParams fp;
    std::memcpy(fp.eye, c->cam.eye, 12); std::memcpy(fp.llc, c->cam.lower_left, 12);
    std::memcpy(fp.hor, c->cam.horizontal, 12); std::memcpy(fp.ver, c->cam.vertical, 12);
    fp.width = c->width; fp.height = c->height; fp.max_depth = c->max_bounce;
    fp.first_frame = first; fp.n_frames = nf;
    fp.band = band; fp.n_shards = nsh; fp.shard = shard;
    fp.rows = shard_rows(c->height, band, nsh, shard);
    fp.mode = c->boxes_finite ? c->mode : PNRT_TRAVERSE_EXACT;
    if (fp.rows == 0) return PNRT_OK;
    DevScene s = c->scene;
    s.hdr = static_cast<const float4*>(c->hdr);
    s.rnd = static_cast<const float4*>(c->rnd);
    s.hdr_q = static_cast<const float4*>(c->hdr_q);
    s.rnd_q = static_cast<const float4*>(c->rnd_q);
    s.n_tex = PT_MAX_TEXTURES;
    for (int i = 0; i < PT_MAX_TEXTURES; ++i) {
        s.tex[i] = static_cast<const uint32_t*>(c->tex[i]);
        s.tex_w[i] = c->tex_w[i]; s.tex_h[i] = c->tex_h[i];
    }
    s.unorm8 = c->unorm8;
    s.fault = c->fault_dev;
    s.diag_force = 0;
    if (WF_DIAG_BOUNDS) {                // the bounds check's own test (diagnostic builds only)
        const char* f = getenv("PNRT_DIAG_FORCE_OOB");
        s.diag_force = (f && atoi(f) > 0) ? 1 : 0;
    }
    if (c->kernel == 1) {
        dim3 grid((c->width + 15) / 16, (fp.rows + 15) / 16);
        {
            ProfScope ps(c, PNRT_K_V1);
            hipLaunchKernelGGL(pt_render_kernel, grid, dim3(256), 0, c->stream, s, fp, c->accum);
        }
        HIPCHK(c, hipGetLastError());
        return mark_stream(c);           // (every op queued on c->stream records ev_last)
    }
    return render_wavefront(c, s, fp, first, nf);
}

int pnrt_reset_accum(pnrt_ctx* c) {
    if (!c) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    // a new accumulation: wait for the calls in flight first, so a fault of one of
    // them (whose contribution the reset erases) is read and cleared here, not
    // reported against the new accumulation later
    HIPCHK(c, sync_all(c));
    (void)check_fault(c);
    if (c->faulted) {
        for (int k = 0; k < WF_FAULT_WORDS; ++k) __atomic_store_n(c->fault_host + k, 0u, __ATOMIC_RELEASE);
        c->faulted = false;
        c->fault_msg.clear();
    }
    if (!c->accum) return PNRT_OK;
    HIPCHK(c, hipMemsetAsync(c->accum, 0, (size_t)c->width * c->height * 16, c->stream));
    return mark_stream(c);
}

int pnrt_read_accum(pnrt_ctx* c, float* out) {
    if (!c || !out) return PNRT_E_ARG;
    if (!c->accum) return set_err(c, PNRT_E_STATE, "read_accum: no frame");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(out, c->accum, (size_t)c->width * c->height * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, sync_all(c));
    return check_fault(c);
}

void* pnrt_accum_device_ptr(pnrt_ctx* c) { return c ? c->accum : nullptr; }

int pnrt_profile_enable(pnrt_ctx* c, int on) {
    if (!c) return PNRT_E_ARG;
    int rc = prof_collect(c);
    if (rc) return rc;
    c->prof_on = on != 0;
    for (int k = 0; k < PNRT_K_COUNT; ++k) { c->prof_ms[k] = 0.0; c->prof_n[k] = 0; }
    return PNRT_OK;
}

int pnrt_profile_select(pnrt_ctx* c, int mask) {
    if (!c) return PNRT_E_ARG;
    c->prof_mask = mask;
    return PNRT_OK;
}

int pnrt_profile_read(pnrt_ctx* c, pnrt_profile* out) {
    if (!c || !out) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = prof_collect(c);
    if (rc) return rc;
    for (int k = 0; k < PNRT_K_COUNT; ++k) { out->ms[k] = c->prof_ms[k]; out->launches[k] = c->prof_n[k]; }
    return PNRT_OK;
}

int pnrt_pack_rows(pnrt_ctx* c, void* dst, int band, int nsh, int shard) {
    if (!c || !dst) return PNRT_E_ARG;
    if (!c->accum) return set_err(c, PNRT_E_STATE, "pack_rows: no frame");
    if (band < 1 || nsh < 1 || shard < 0 || shard >= nsh) return set_err(c, PNRT_E_ARG, "pack_rows: bad shard selector");
    if (int rc = check_fault(c)) return rc;      // completed work that faulted
    HIPCHK(c, hipSetDevice(c->device));
    int rows = shard_rows(c->height, band, nsh, shard);
    size_t total = (size_t)rows * c->width;
    if (total == 0) return PNRT_OK;
    hipLaunchKernelGGL(pt_pack_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c->stream,
                       c->accum, static_cast<float4*>(dst), c->width, rows, band, nsh, shard);
    HIPCHK(c, hipGetLastError());
    return mark_stream(c);
}

int pnrt_unpack_rows(pnrt_ctx* c, const void* src, void* image, int band, int nsh, int shard) {
    if (!c || !src || !image) return PNRT_E_ARG;
    if (c->width <= 0 || c->height <= 0) return set_err(c, PNRT_E_STATE, "unpack_rows: no frame");
    if (band < 1 || nsh < 1 || shard < 0 || shard >= nsh) return set_err(c, PNRT_E_ARG, "unpack_rows: bad shard selector");
    HIPCHK(c, hipSetDevice(c->device));
    int rows = shard_rows(c->height, band, nsh, shard);
    size_t total = (size_t)rows * c->width;
    if (total == 0) return PNRT_OK;
    hipLaunchKernelGGL(pt_unpack_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c->stream,
                       static_cast<const float4*>(src), static_cast<float4*>(image), c->width, rows, band, nsh, shard);
    HIPCHK(c, hipGetLastError());
    return mark_stream(c);
}

int pnrt_synchronize(pnrt_ctx* c) {
    if (!c) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, sync_all(c));
    return check_fault(c);
}

int pnrt_get_device_info(pnrt_ctx* c, pnrt_device_info* info) {
    if (!c || !info) return PNRT_E_ARG;
    info->n_interior = c->n_interior;
    info->n_triangles = c->scene.n_tris;
    info->max_depth = c->max_depth;
    info->device_bytes = c->scene_bytes;
    info->root_is_leaf = c->root_is_leaf;
    info->stack_limit = PT_STACK;
    return PNRT_OK;
}

int pnrt_debug_math(pnrt_ctx* c, int fn, const float* a, const float* b, float* out, int n) {
    if (!c || !a || !out || n <= 0) return PNRT_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    float *da, *db, *dout;
    size_t bytes = (size_t)n * 4;
    HIPCHK(c, hipMalloc(&da, bytes));
    HIPCHK(c, hipMalloc(&db, bytes));
    HIPCHK(c, hipMalloc(&dout, bytes));
    HIPCHK(c, hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    if (b) HIPCHK(c, hipMemcpy(db, b, bytes, hipMemcpyHostToDevice));
    else HIPCHK(c, hipMemset(db, 0, bytes));
    hipLaunchKernelGGL(pt_math_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, fn, da, db, dout, n);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, sync_all(c));
    HIPCHK(c, hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
    return PNRT_OK;
}

}  // extern "C"

// ---- GPU BuildBVH (pt_bvh.h) -----------------------------------------------------------------
namespace {
struct DevAllocs {                     // device scratch of one build, freed on every return path
    std::vector<void*> p;
    ~DevAllocs() { for (void* q : p) (void)hipFree(q); }
    template <typename T> hipError_t get(T** out, size_t count) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, count * sizeof(T) + 16);
        if (e == hipSuccess) { p.push_back(q); *out = static_cast<T*>(q); }
        return e;
    }
};
}  // namespace

static unsigned blocks_for(long long n, int per) { return (unsigned)((n + per - 1) / per); }

extern "C" int pnrt_bvh_build(pnrt_ctx* c, const float* tb, int n, float* nodes_out, int cap, int* n_nodes_out,
                              int32_t* order_out, int* max_depth_out) {
    if (!c) return PNRT_E_ARG;
    if (!tb || n <= 0 || !nodes_out || !n_nodes_out || !order_out) return set_err(c, PNRT_E_ARG, "bvh_build: bad arguments");
    if (n >= (1 << 24)) return set_err(c, PNRT_E_ARG, "bvh_build: >= 2^24 triangles cannot be stored as exact floats");
    if (cap < 2 * n - 1) return set_err(c, PNRT_E_ARG, "bvh_build: node capacity must be >= 2 * n_triangles - 1");
    HIPCHK(c, hipSetDevice(c->device));
    // triangle bounds + centres: A = (pMin, cx), B = (pMax, cy), C = cz
    std::vector<float4> hA(n), hB(n);
    std::vector<float> hC(n);
    for (int i = 0; i < n; ++i) {
        const float* t = tb + 9 * (size_t)i;
        for (int k = 0; k < 9; ++k)
            if (!std::isfinite(t[k])) return set_err(c, PNRT_E_SCENE, "bvh_build: triangle " + std::to_string(i) + " has a non-finite bound");
        hA[i] = make_float4(t[0], t[1], t[2], t[6]);
        hB[i] = make_float4(t[3], t[4], t[5], t[7]);
        hC[i] = t[8];
    }
    const size_t segcap = (size_t)n / (BVH_SMALL + 1) + 2;
    const size_t chcap = (size_t)n / BVH_CHUNK + segcap + 2;
    DevAllocs m;
    float4 *A, *B; float* C; int *order, *Fpos, *Tpos, *ctrue, *excl;
    BvhSeg* segs[2]; BvhChunk* chunks[2]; BvhAcc* acc; BvhTop* top; BvhSmall* small; BvhLocal* loc; BvhCtr* ctr;
    HIPCHK(c, m.get(&A, n)); HIPCHK(c, m.get(&B, n)); HIPCHK(c, m.get(&C, n));
    HIPCHK(c, m.get(&order, n)); HIPCHK(c, m.get(&Fpos, n)); HIPCHK(c, m.get(&Tpos, n));
    HIPCHK(c, m.get(&ctrue, chcap)); HIPCHK(c, m.get(&excl, chcap));
    HIPCHK(c, m.get(&segs[0], segcap)); HIPCHK(c, m.get(&segs[1], segcap));
    HIPCHK(c, m.get(&chunks[0], chcap)); HIPCHK(c, m.get(&chunks[1], chcap));
    HIPCHK(c, m.get(&acc, segcap)); HIPCHK(c, m.get(&top, 2 * (size_t)n + 2));
    HIPCHK(c, m.get(&small, (size_t)n + 1)); HIPCHK(c, m.get(&loc, 2 * (size_t)n + 2));
    HIPCHK(c, m.get(&ctr, 1));
    hipStream_t st = c->stream;
    HIPCHK(c, hipMemcpyAsync(A, hA.data(), n * sizeof(float4), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(B, hB.data(), n * sizeof(float4), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(C, hC.data(), n * sizeof(float), hipMemcpyHostToDevice, st));
    {
        std::vector<int> iota(n);
        for (int i = 0; i < n; ++i) iota[i] = i;
        HIPCHK(c, hipMemcpyAsync(order, iota.data(), n * sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(c, hipStreamSynchronize(st));
    }
    BvhCtr h{};
    int nseg = 0, nch = 0, cur = 0;
    if (n > BVH_SMALL) {                      // root = large range 0 (temporary id 0)
        BvhSeg s0{}; s0.L = 0; s0.R = n; s0.depth = 0; s0.tmp = 0; s0.chunk0 = 0;
        std::vector<BvhChunk> ck;
        for (int p = 0; p < n; p += BVH_CHUNK) ck.push_back({0, p, std::min(p + BVH_CHUNK, n), 0});
        nseg = 1; nch = (int)ck.size();
        HIPCHK(c, hipMemcpy(segs[0], &s0, sizeof s0, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(chunks[0], ck.data(), ck.size() * sizeof(BvhChunk), hipMemcpyHostToDevice));
        h.ntop = 1;
    } else {                                  // root = small range 0
        BvhSmall s0{}; s0.L = 0; s0.R = n; s0.depth = 0;
        HIPCHK(c, hipMemcpy(small, &s0, sizeof s0, hipMemcpyHostToDevice));
        h.nsmall = 1;
    }
    HIPCHK(c, hipMemcpy(ctr, &h, sizeof h, hipMemcpyHostToDevice));
    int levels = 0;
    while (nseg > 0) {
        if (++levels > 100000) return set_err(c, PNRT_E_SCENE, "bvh_build: tree too deep");
        h.nseg = 0; h.nch = 0;
        HIPCHK(c, hipMemcpyAsync(ctr, &h, sizeof h, hipMemcpyHostToDevice, st));
        BvhSeg* sg = segs[cur]; BvhChunk* ck = chunks[cur];
        const unsigned gs = blocks_for(nseg, 256);
        hipLaunchKernelGGL(bvh_init_kernel, dim3(gs), dim3(256), 0, st, acc, nseg);
        hipLaunchKernelGGL(bvh_bounds_kernel, dim3(nch), dim3(256), 0, st, (const BvhChunk*)ck, acc, (const int*)order,
                           (const float4*)A, (const float4*)B, (const float*)C);
        hipLaunchKernelGGL(bvh_axis_kernel, dim3(gs), dim3(256), 0, st, (const BvhSeg*)sg, acc, nseg, (const int*)order,
                           (const float4*)A, (const float4*)B);
        hipLaunchKernelGGL(bvh_bucket_kernel, dim3(nch), dim3(256), 0, st, (const BvhChunk*)ck, acc, (const int*)order,
                           (const float4*)A, (const float4*)B, (const float*)C);
        hipLaunchKernelGGL(bvh_split_kernel, dim3(gs), dim3(256), 0, st, (const BvhSeg*)sg, acc, nseg);
        hipLaunchKernelGGL(bvh_count_kernel, dim3(nch), dim3(256), 0, st, (const BvhChunk*)ck, (const BvhAcc*)acc,
                           (const int*)order, (const float4*)A, (const float4*)B, (const float*)C, ctrue);
        hipLaunchKernelGGL(bvh_scan_kernel, dim3(1), dim3(1024), 0, st, (const int*)ctrue, excl, nch);
        hipLaunchKernelGGL(bvh_lists_kernel, dim3(nch), dim3(256), 0, st, (const BvhChunk*)ck, (const BvhSeg*)sg, acc,
                           (const int*)order, (const float4*)A, (const float4*)B, (const float*)C, (const int*)excl,
                           Fpos, Tpos);
        hipLaunchKernelGGL(bvh_swap_kernel, dim3(nch), dim3(256), 0, st, (const BvhChunk*)ck, (const BvhSeg*)sg,
                           (const BvhAcc*)acc, order, (const int*)Fpos, (const int*)Tpos);
        hipLaunchKernelGGL(bvh_emit_kernel, dim3(gs), dim3(256), 0, st, (const BvhSeg*)sg, (const BvhAcc*)acc, nseg, top,
                           segs[cur ^ 1], chunks[cur ^ 1], small, ctr);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(&h, ctr, sizeof h, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        nseg = h.nseg; nch = h.nch; cur ^= 1;
        if ((size_t)nseg > segcap || (size_t)nch > chcap || h.ntop > 2 * n + 2 || h.nsmall > n + 1)
            return set_err(c, PNRT_E_SCENE, "bvh_build: internal capacity exceeded");
    }
    if (h.nsmall > 0) {
        hipLaunchKernelGGL(bvh_small_kernel, dim3(blocks_for(h.nsmall, 4)), dim3(256), 0, st, small, h.nsmall, order,
                           (const float4*)A, (const float4*)B, (const float*)C, loc, ctr);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipMemcpyAsync(&h, ctr, sizeof h, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (h.ntop < 0 || h.ntop > 2 * n + 2 || h.nsmall < 0 || h.nsmall > n + 1 || h.small_nodes > 2 * n)
        return set_err(c, PNRT_E_SCENE, "bvh_build: internal capacity exceeded");
    std::vector<BvhTop> ht(h.ntop);
    std::vector<BvhSmall> hs(h.nsmall);
    if (h.ntop) HIPCHK(c, hipMemcpyAsync(ht.data(), top, h.ntop * sizeof(BvhTop), hipMemcpyDeviceToHost, st));
    if (h.nsmall) HIPCHK(c, hipMemcpyAsync(hs.data(), small, h.nsmall * sizeof(BvhSmall), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    // pre-order ids (the static nodeId counter of BVH.hpp:94-95): left subtree, then right
    std::vector<int> ftop(h.ntop + 1, 0), fsmall(h.nsmall + 1, 0);
    std::vector<int> stk{h.ntop ? 0 : -1};
    int counter = 0;
    while (!stk.empty()) {
        const int ref = stk.back();
        stk.pop_back();
        if (ref >= 0) {
            ftop[ref] = counter++;
            if (ht[ref].axis != -1) { stk.push_back(ht[ref].right); stk.push_back(ht[ref].left); }
        } else {
            fsmall[-ref - 1] = counter;
            counter += hs[-ref - 1].count;
        }
    }
    if (counter > cap) return set_err(c, PNRT_E_SCENE, "bvh_build: node capacity exceeded");
    int *dft, *dfs; float* dout;
    HIPCHK(c, m.get(&dft, ftop.size())); HIPCHK(c, m.get(&dfs, fsmall.size())); HIPCHK(c, m.get(&dout, 12 * (size_t)counter));
    HIPCHK(c, hipMemcpyAsync(dft, ftop.data(), ftop.size() * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(dfs, fsmall.data(), fsmall.size() * sizeof(int), hipMemcpyHostToDevice, st));
    if (h.ntop)
        hipLaunchKernelGGL(bvh_scatter_top_kernel, dim3(blocks_for(h.ntop, 256)), dim3(256), 0, st, (const BvhTop*)top,
                           h.ntop, (const int*)dft, (const int*)dfs, dout);
    if (h.nsmall)
        hipLaunchKernelGGL(bvh_scatter_small_kernel, dim3(blocks_for(h.nsmall, 4)), dim3(256), 0, st,
                           (const BvhSmall*)small, h.nsmall, (const BvhLocal*)loc, (const int*)dfs, dout);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(nodes_out, dout, 12 * (size_t)counter * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(order_out, order, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    *n_nodes_out = counter;
    if (max_depth_out) *max_depth_out = h.max_depth;
    return PNRT_OK;
}
