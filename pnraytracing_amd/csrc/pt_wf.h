// pnraytracing_amd/csrc/pt_wf.h -- v3 integrator: wavefront path tracing for gfx950.
//
// All samples (pixel, frame) of a pnrt_render chunk are paths held in SoA
// buffers in HBM.  Per bounce three kernels run over every path slot:
//   setup  -- material, light/env/BSDF sampling in the reference RNG order, and
//             every BRDF value the bounce needs (evaluated before the shadow
//             tests: same float ops, same bits); emits up to three rays
//   trace  -- ONE persistent traversal kernel for all rays of the bounce
//             (light shadow, env shadow: any-hit; continuation: closest-hit),
//             small register footprint -> high occupancy, LDS short stack
//   shade  -- "MIS" accumulation with the occlusion results, the continuation
//             hit (emission, throughput), next bounce or the final colour
// so each kernel is compact and coherent instead of one 240-VGPR megakernel.
#pragma once
#include <type_traits>
#include "pt_passes.h"

#ifndef WF_STACK
#define WF_STACK 8          // LDS stack entries per lane; deeper spills to global
#endif
#ifndef WF_REFILL_PCT
#define WF_REFILL_PCT 40    // refill a wave when at most this % of its lanes still trace (tuned at 8 waves)
#endif
#ifndef WF_PIPES
#define WF_PIPES 4          // buffer sets / worker streams: pnrt_render calls in flight at most
#endif
#ifndef WF_PIPES_LARGE
#define WF_PIPES_LARGE (WF_PIPES > 3 ? 3 : WF_PIPES)   // calls in flight for large calls (+ the context
#endif                                                // stream = the 4 HW queues of a process)
#ifndef WF_PIPES_MEDIUM
#define WF_PIPES_MEDIUM (WF_PIPES > 2 ? 2 : WF_PIPES)   // calls in flight for calls of WF_SMALL_CALL_PATHS ..
#endif                                                  // WF_HUGE_CALL_PATHS paths (never more than the sets made)
#ifndef WF_HUGE_CALL_PATHS
#define WF_HUGE_CALL_PATHS 32000000   // calls with more paths (4K frames) keep WF_PIPES_LARGE in flight
#endif
#ifndef WF_SMALL_CALL_PATHS
#define WF_SMALL_CALL_PATHS 5000000   // calls with fewer paths (multi-GPU shares: 2.1M at N = 8, 4.2M at N = 4 with 8-frame calls) use all WF_PIPES sets
#endif
#define WF_LIGHT_SCAN PT_LIGHT_SCAN
#ifndef WF_QSHARDS
#define WF_QSHARDS 16       // dequeue counters, one 128-B line apart
#endif
#ifndef WF_QSTRIDE
#define WF_QSTRIDE 32       // dwords between dequeue counters (one 128-B line each)
#endif
// bytes of the dequeue-counter area (the census / timing words follow it)
#define WF_COUNTER_BYTES (WF_QSHARDS * WF_QSTRIDE * 4 > 2048 ? WF_QSHARDS * WF_QSTRIDE * 4 : 2048)
#ifndef WF_TRACE_BLOCK
#define WF_TRACE_BLOCK 256   // trace workgroup size (128, 256 or 512)
#endif
#define WF_SPA_STRIDE (WF_TRACE_BLOCK * 8u)                 // LDS bytes per stack depth
#define WF_SPA_SHIFT (WF_TRACE_BLOCK == 512 ? 12 : WF_TRACE_BLOCK == 256 ? 11 : 10)
#define WF_BQ_GUARD (WF_DIAG_GUARD > 0 ? (uint32_t)WF_DIAG_GUARD : (1u << 10))   // block-queue claim attempts
// Ray kinds: 0 light shadow, 1 env shadow, 2 continuation.  Only env shadow rays
// are queued as ready-to-trace records (rayO / rayD): continuation and light
// shadow rays are traced from the path state the setup wrote (P0 with P1 / P7,
// see wf_enqueue; queued records for them measured 2 % / 3.3 % slower).
#define WF_QUEUED(k) ((k) == 1)

// Cache policy of the streamed path-state traffic (path state, ray records,
// frame colours): written once by a setup, read once by the trace and the next
// shade, never by the same CU's L2 while the line could still be there -- 1 GB
// per state set, far beyond the 4 MB L2 of an XCD, which the trace kernels of
// the calls in flight use for the BVH.  Loads are non-temporal (C2 +0.5 to
// +1.2 %, same box); stores plain (write-through sc1 stores: -4 %, nt: neutral).
PN_DEV void ps_st(float4* base, size_t i, float4 v) { base[i] = v; }
PN_DEV float4 ps_ld(const float4* p) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

// ray kinds a setup emitted (enqueue) ...
#define WF_RLIGHT 2u
#define WF_RENV 4u
#define WF_RCONT 8u
// ... and the path's meta word, P6.w: slot (pixel, frame) | light ray | env ray | bounce
// (WF_SLOT_BITS bits of slot bound the paths of one batch; the bounce takes the top
// bits above the two ray flags: 2 bits hold pnrt_set_frame's depth <= 4)
#ifndef WF_SLOT_BITS
#define WF_SLOT_BITS 28      // 2^28 paths per batch: 128 frames of a 1080p frame, 32 of a 4K frame (26 until late round 6)
#endif
static_assert(WF_SLOT_BITS >= 20 && WF_SLOT_BITS <= 28, "slot | RL | RE | bounce (>= 2 bits) in 32");
#define WF_META_SLOT ((1u << WF_SLOT_BITS) - 1u)
#define WF_META_RL (1u << WF_SLOT_BITS)
#define WF_META_RE (1u << (WF_SLOT_BITS + 1))
#define WF_META_BSHIFT (WF_SLOT_BITS + 2)

// Path state between a setup and the next shade: exactly what shade reads,
// 112 B per live path (the primary hit's base colour is re-read from the
// primary record).  A setup block writes its live paths compacted to the front
// of its 256-entry range (entry j = 256 * block + rank), so the next shade's
// lanes are all live paths and its empty waves exit at once; two sets
// alternate by bounce (a shade reads one and its setup writes the other).
struct PathSet {
    float4* P0;   // continuation origin (P + N*1e-4).xyz, dPDF
    float4* P1;   // L.xyz, |N.L|
    float4* P2;   // dBRDF.xyz, enPDF
    float4* P3;   // LDirect.xyz, lightPDF  written iff the path has a light ray, read iff it is unoccluded
    float4* P4;   // LEnvironment.xyz, -    written iff the path has an env ray, read iff it is unoccluded
    float4* P5;   // Lo.xyz, bits(seed)
    float4* P6;   // throughput.xyz, bits(meta)
    float4* P7;   // light shadow ray direction (read by trace only)
    uint32_t* bcount;   // live paths of each setup block
};

struct WfBufs {
    PathSet rd, wr;    // shade reads rd; its setup (and gen) writes wr
    // trace results, by path entry j
    uint8_t* occ;      // [2 * n]: light, env occluded
    int* hit;          // continuation hit triangle or -1
    uint2* ovf;        // traversal stack spill: per trace block ovf_stride depths x 2048 B (wf_ovf_rsrc)
    uint32_t ovf_stride;
    unsigned int* counter;   // ray dequeue counter (zeroed before each bounce)
    // ray queues, written by setup without atomics: segment (k, j) of kind k
    // (light | env | continuation) and setup block j = trace slots
    // [k * npad + 256 j, +segcount[k * nseg_k + j]).  The queued kind (env)
    // stores ready-to-trace records -- rayO = (origin, bits(path entry)), rayD =
    // (direction, -), at the slot's offset within its npad entries; the other
    // kinds are read from the path state (see wf_enqueue)
    float4* rayO;            // [npad]  (.w = path entry j)
    float4* rayD;            // [npad]
    unsigned int* segcount;  // [3 * nseg_k]
    uint32_t npad;           // n rounded up to 256
    uint32_t nseg_k;         // setup blocks = segments per kind
    unsigned long long* stats; // WF_STATS builds: traversal step census (8 counters)
    uint32_t* fault;   // the context's fault words (host-mapped, see wf_fault), WF_FAULT_* index
    uint32_t n;        // path slots
    int chunk_frames;
    int tiles_x;
    uint32_t first_frame;
    float2* sobol;     // [(bounce - 1) * chunk_frames + k]: the Sobol pair of bounces >= 1, frame k (gen writes it)
};

// Faults: a trace launch that could leave a queued ray untraced reports it
// instead of returning a silently wrong image (ray_tracing.comp:429-494 traces
// every ray).  One word per kind (pt_diag.h WF_FAULT_*) in the context's
// host-mapped fault area, written with a system-scope vector store only when a
// check trips (pnrt_render, pnrt_synchronize, pnrt_read_accum and pnrt_pack_rows
// then return PNRT_E_TRACE).
PN_DEV void wf_fault(const WfBufs& b, int kind) {
    __hip_atomic_store(b.fault + kind, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A setup kernel's block 0 resets the dequeue counters of the trace launch that
// follows it (the previous trace has completed: stream order).  The shade
// kernels first check that the previous trace handed out every queue item: item
// i is ticket i / WF_QSHARDS of counter i % WF_QSHARDS, so counter p must have
// passed all ceil((nseg - p) / WF_QSHARDS) tickets below nseg.  (Shards of
// contiguous image regions, one per XCD, each block starting on its XCD's shard:
// bit-exact, but C2 -0.5 %, C5 -2.3 %, profiles/r04/s4/summary.txt.)
PN_DEV void wf_check_drained(const WfBufs& b) {
    if (blockIdx.x == 0 && threadIdx.x < WF_QSHARDS) {
        const uint32_t nseg = 3u * b.nseg_k, p = threadIdx.x;
        const uint32_t need = nseg > p ? (nseg - p + WF_QSHARDS - 1) / WF_QSHARDS : 0u;
        if (b.counter[p * WF_QSTRIDE] < need) wf_fault(b, WF_FAULT_DRAIN);
    }
}
PN_DEV void wf_reset_counters(const WfBufs& b) {
    if (blockIdx.x == 0 && threadIdx.x < WF_QSHARDS) b.counter[threadIdx.x * WF_QSTRIDE] = 0u;
}

// path slot -> (x, local row, frame slot): 8x8-pixel tiles, frame-major inside a
// tile, so consecutive path slots (and the rays they spawn) are spatial neighbours
PN_DEV void wf_coords(const WfBufs& b, uint32_t s, int& x, int& lr, int& k) {
    uint32_t per_tile = 64u * (uint32_t)b.chunk_frames;
    uint32_t tile = s / per_tile, rem = s - tile * per_tile;
    k = (int)(rem >> 6);
    int p = (int)(rem & 63u);
    int ty = (int)(tile / (uint32_t)b.tiles_x), tx = (int)(tile - (uint32_t)ty * b.tiles_x);
    x = tx * 8 + (p & 7);
    lr = ty * 8 + (p >> 3);
}

// Number of set bits of m below this lane (v_mbcnt).
PN_DEV uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// A path's compacted entry within its block, without a block barrier between
// the waves' loads: each wave takes its range with one LDS atomic on the block's
// live-path counter (zeroed by wf_live_init at the kernel's start), so a wave
// whose records have arrived goes on to its next fetches instead of waiting for
// its block's slowest wave.  Which range a wave gets depends on arrival order --
// no result does: a path's entry only names where its state, rays and trace
// results live.  (Against a block-barrier rank: C2 shade -2.3 %; the barrier-free
// wf_enqueue below another -1.7 %, C2 +0.8 %, profiles/r03/s7/ab_enq_nobar_s15.txt.)
PN_DEV uint32_t* wf_live_ctr() {
    __shared__ uint32_t c;
    return &c;
}
PN_DEV uint32_t* wf_enq_ctr() {     // queued rays per kind, and the waves through wf_enqueue
    __shared__ uint32_t c[4];
    return c;
}
PN_DEV void wf_live_init() {
    if (threadIdx.x == 0) *wf_live_ctr() = 0u;
    if (threadIdx.x < 4) wf_enq_ctr()[threadIdx.x] = 0u;
    __syncthreads();
}
PN_DEV uint32_t wf_entry_rank(bool live) {
    const uint64_t m = __ballot(live);
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 0 && m != 0)
        base = __hip_atomic_fetch_add(wf_live_ctr(), (uint32_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(base) + lanes_below(m);
}

PN_DEV void wf_write_color(const WfBufs& b, const FrameParams& fp, float4* colors, int k, int lr, int x, f3 color) {
    color = mk3(clampf(color.x, 0.f, 1.f), clampf(color.y, 0.f, 1.f), clampf(color.z, 0.f, 1.f));
    const size_t at = PT_CHECK(b.fault, ((size_t)k * fp.rows + lr) * fp.width + x,
                               (size_t)b.chunk_frames * fp.rows * fp.width, PT_SITE_COLOR);
    ps_st(colors, at, make_float4(color.x, color.y, color.z, 0.f));
}
// the primary record of local row lr, column x
PN_DEV const float4* wf_primary(const WfBufs& b, const FrameParams& fp, const float4* primary, int lr, int x) {
    return primary + 3 * PT_CHECK(b.fault, (size_t)lr * fp.width + x, (size_t)fp.rows * fp.width, PT_SITE_PRIMARY);
}

// Path state a bounce's setup starts from (in registers: the fused kernels
// hand it over without a round trip through HBM).
struct PathIn {
    f3 P, N, V, cw, Lo;
    float u, v;
    int mt;            // material | (texture + 1) << 24
    uint32_t seed;
};

// ---- setup: one bounce's sampling and BRDF values (ray_tracing.comp:866-934) -----------------
// The bounce's three rays (:886-889 light: origin P + N*1e-4, unnormalised
// direction; :917-920 env: origin P; :949 continuation: origin P + N*1e-4).
struct BounceRays {
    f3 oOff, oP;          // offset origin, plain origin
    f3 dL, dE, dC;
};

// GetLightIndex (:237-251) as the light ENTRY it selects (the reference then
// uses entry.x, its triangle): a lower bound over the non-decreasing prefix
// areas.  Short lists (s.light_scan, checked monotone at upload) are scanned
// from the kernel arguments (s.lscan: scalar registers, no memory round trip)
// -- the same entry as the binary search.  No entry (u * sum beyond the last
// prefix) -> entry n_lights, whose record is triangle 0's, as the reference's
// fallback index 0.
PN_DEV int light_entry(const DevScene& s, float u) {
    const float randomArea = u * s.lights_sum_area;
    int ans = -1;
    if (s.light_scan) {
#pragma unroll
        for (int k = WF_LIGHT_SCAN - 1; k >= 0; --k)
            if (k < s.n_lights && s.lscan[k] >= randomArea) ans = k;
    } else {
        int L = 0, R = s.n_lights - 1;
        while (L <= R) {
            int mid = (L + R) >> 1;
            if (s.lights[mid].y >= randomArea) { ans = mid; R = mid - 1; }
            else L = mid + 1;
        }
    }
    return ans < 0 ? s.n_lights : ans;
}

// The light triangle's records (TriangleSample :598-624, emission :887), one
// fetch from the light entry.
struct LightFetch {
    float4 va0, vb0, va1, vb1, va2, vb2;
    f3 li;
};
PN_DEV LightFetch light_fetch(const DevScene& s, int entry) {
    entry = (int)PT_CHECK(s.fault, entry, s.n_lights + 1, PT_SITE_LIGHT_REC);
    LightFetch f;
    const float4* r = s.light_rec + 7 * (size_t)entry;
    f.va0 = r[0]; f.vb0 = r[1]; f.va1 = r[2]; f.vb1 = r[3]; f.va2 = r[4]; f.vb2 = r[5];
    const float4 em = r[6];
    f.li = mk3(em.x, em.y, em.z);
    return f;
}

#ifndef WF_SKIP_MOOT
#define WF_SKIP_MOOT 1        // shadow rays that cannot change the path are not traced (wf_setup_core)
#endif
#ifndef WF_MOOT_TSUM
#define WF_MOOT_TSUM 1        // the moot test's bound: T_U + T_E (1), or the numerator over the larger reciprocal (0)
#endif
#ifndef WF_MOOT_LDS
#define WF_MOOT_LDS 1         // the moot test reads the light / env candidates back from the lane's LDS slot
#endif                        // (0: from the P3 / P4 lines it just stored -- an L2 round trip)
// The lane's LDS copy of its light and env candidates (LDirect, lightPDF; LEnvironment)
// for the moot test: written where P3 / P4 are stored, read by the same lane.
PN_DEV float4* wf_moot_lds() {
    __shared__ float4 c[2 * 256];
    return c;
}

// The light record is always fetched with the material.  ENV_EARLY: the env
// table taps too (gen; in the shade kernel's setup they cost spills, -1.5 %).
// SOBOL_PAIR: both Sobol dimensions of the bounce in one pass over the set bits
// (sobol_pair: shade +1.1 %; in gen, where the bounce is the constant 0 and the
// per-bit loop folds, it lost 3.5 %).
// MOOT: the moot shadow-ray test (WF_SKIP_MOOT) -- not in gen: at bounce 0 Lo is
// zero, so only rays with an exactly zero term are moot (~1.7 % of C2's bounce-0
// light rays), fewer than the test costs.
// Returns the ray kinds the bounce emits; writes the path state P0-P7 of entry
// i of the write set (slot = the path's (pixel, frame) slot); the rays go to `rays`.
template <bool ENV_EARLY, bool SOBOL_PAIR, bool MOOT>
PN_DEV uint32_t wf_setup_core(const DevScene& s, const FrameParams& fp, const WfBufs& b, uint32_t i, uint32_t slot,
                              int bounce, int x, int py, uint32_t frame, const PathIn& q, BounceRays& rays) {
    const PathSet& w = b.wr;
    i = (uint32_t)PT_CHECK(b.fault, i, b.npad, PT_SITE_PATH);
    const f3 P = q.P, N = q.N, V = q.V;
    const int hmat = q.mt & 0x00ffffff, htex = (int)((uint32_t)q.mt >> 24) - 1;
    uint32_t seed = q.seed;
    // the bounce's light and environment draws (:880, :884, :918) come first in the
    // stream and depend on nothing else, so they are drawn up front (same order)
    const float uSel = rand01(seed);
    float u0 = 0.f, u1 = 0.f, r1 = 0.f, r2 = 0.f;
    if (s.n_lights > 0) { u0 = rand01(seed); u1 = rand01(seed); }
    if (s.has_hdr) { r1 = rand01(seed); r2 = rand01(seed); }
    // light record (and env table taps) in flight with the material fetch
    int lentry = light_entry(s, uSel);
    if (WF_DIAG_BOUNDS && s.diag_force && slot == 0) lentry = s.n_lights + 7;   // the check's own test
    const LightFetch lf = light_fetch(s, lentry);
    Taps4 envTaps;
    if constexpr (ENV_EARLY) {
        if (s.has_hdr) envTaps = taps_quad(s, s.rnd_q, r1, r2);
    }
    Material m = get_material(s, hmat);
    asm volatile("" ::: "memory");
    if (htex != -1) {
        if (texture_bound(s, htex)) m.baseColor = albedo_resolve(albedo_fetch(s, htex, q.u, q.v));
        else m.baseColor = mk3(0.f, 0.f, 0.f);                                        // unbound unit -> 0
    }
    f3 T, B;
    if (N.z > 0.9999995f) T = mk3(1.f, 0.f, 0.f);
    else T = normalize(cross(N, mk3(0.f, 0.f, 1.f)));
    B = cross(N, T);
    BrdfCtx bc = brdf_prepare(V, N, T, B, m);
    uint32_t nfl = 0;

    // direct light (:878-909): candidate values, used if the shadow ray is unoccluded
    f3 LD = mk3(0.f, 0.f, 0.f);
    float pl = 0.f;
    if (s.n_lights > 0) {                            // light_index() == -1 iff no lights
        float su0 = sqrtf(u0);
        float bx = 1.0f - su0, by = u1 * su0, bz = (1.0f - bx) - by;
        f3 p0 = mk3(lf.va0.x, lf.va0.y, lf.va0.z), p1 = mk3(lf.va1.x, lf.va1.y, lf.va1.z);
        f3 p2 = mk3(lf.va2.x, lf.va2.y, lf.va2.z);
        f3 n0 = mk3(lf.va0.w, lf.vb0.x, lf.vb0.y), n1 = mk3(lf.va1.w, lf.vb1.x, lf.vb1.y);
        f3 n2 = mk3(lf.va2.w, lf.vb2.x, lf.vb2.y);
        f3 lp = add(add(muls(p0, bx), muls(p1, by)), muls(p2, bz));
        f3 ln;
        if (iszero3(n0) || iszero3(n1) || iszero3(n2)) ln = normalize(cross(sub(p1, p0), sub(p2, p0)));
        else ln = add(add(muls(n0, bx), muls(n1, by)), muls(n2, bz));
        ln = normalize(ln);
        f3 ldir = sub(lp, P);
        float dis2 = (ldir.x * ldir.x + ldir.y * ldir.y) + ldir.z * ldir.z;
        f3 lightL = normalize(ldir);
        pl = dis2 / (pnm_fabs(dot(ln, neg(lightL))) * s.lights_sum_area);
        f3 lightBRDF = disney(bc, lightL);
        LD = divs(muls(mul(lightBRDF, lf.li), pnm_fabs(dot(N, lightL))), pl);
        rays.dL = ldir;
        ps_st(w.P7, i, make_float4(ldir.x, ldir.y, ldir.z, 0.f));
        nfl |= WF_RLIGHT;
    }
    // stored as soon as final (shorter live ranges), and only when shade can use it:
    // shade takes (0, 0) for a path without a light ray, as the reference's
    // initial LDirect / lightPDF (:878-879)
    if (nfl & WF_RLIGHT) ps_st(w.P3, i, make_float4(LD.x, LD.y, LD.z, pl));
    if (WF_SKIP_MOOT && WF_MOOT_LDS && MOOT)
        wf_moot_lds()[threadIdx.x] = (nfl & WF_RLIGHT) ? make_float4(LD.x, LD.y, LD.z, pl) : make_float4(0.f, 0.f, 0.f, 0.f);
    // environment (:911-926)
    f3 LE = mk3(0.f, 0.f, 0.f);
    float pe = 0.f;
    if (s.has_hdr) {
        f3 enL;
        f3 enLi;
        if constexpr (ENV_EARLY) enLi = taps_resolve(env_dir(s, envTaps, enL, pe));
        else enLi = sample_env(s, r1, r2, enL, pe);
        if (dot(enL, N) > 0) {
            f3 dB = disney(bc, enL);
            LE = divs(muls(mul(dB, enLi), dot(enL, N)), pe);
            rays.dE = enL;
            nfl |= WF_RENV;
        }
    }
    if (nfl & WF_RENV) ps_st(w.P4, i, make_float4(LE.x, LE.y, LE.z, 0.f));
    if (WF_SKIP_MOOT && WF_MOOT_LDS && MOOT)
        wf_moot_lds()[256 + threadIdx.x] = (nfl & WF_RENV) ? make_float4(LE.x, LE.y, LE.z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    // BRDF sample (:928-934) with Cranley-Patterson-rotated Sobol (:539-557)
    uint32_t pseed = ((uint32_t)(x * fp.width) * 1973u + (uint32_t)(py * fp.height) * 9277u +
                      (uint32_t)(114514 / 1919) * 26699u) | 1u;
    float cpu = rand01(pseed), cpv = rand01(pseed);
    const uint32_t g = (frame + 1u) ^ ((frame + 1u) >> 1);
    float su, sv;
    if constexpr (SOBOL_PAIR) {     // (the shade's setups, bounce >= 1: the batch's table, computed once by gen)
        const float2 v = b.sobol[(uint32_t)(bounce - 1) * (uint32_t)b.chunk_frames + (frame - b.first_frame)];
        su = v.x; sv = v.y;
    } else {
        su = sobol_dev(2u * (uint32_t)bounce, g);
        sv = sobol_dev(2u * (uint32_t)bounce + 1u, g);
    }
    su += cpu; if (su > 1) su -= 1; if (su < 0) su += 1;
    sv += cpv; if (sv > 1) sv -= 1; if (sv < 0) sv += 1;
    float rDiffuse = 1.0f - m.metallic;
    float rClearcoat = 0.25f * m.clearcoat;
    float invSum = 1.0f / ((rDiffuse + 1.0f) + rClearcoat);
    float pDiffuse = rDiffuse * invSum, pSpecular = 1.0f * invSum, pClearcoat = rClearcoat * invSum;
    float rl = rand01(seed);
    float alphaGTR1 = bc.alphaDr;
    float alphaGTR2 = fmax_(0.001f, sqr(m.roughness));
    f3 L;
    if (rl <= pDiffuse) {
        float theta = rand01(seed), rr = rand01(seed);
        float sth, cth;
        pnm_sincos(theta, sth, cth);
        float xx = rr * sth, yy = rr * cth;
        float zz = sqrtf((1.0f - sqr(xx)) - sqr(yy));
        L = tangent_to_world(T, B, N, mk3(xx, yy, zz));
    } else {
        float phiH = (2.0f * PT_PI) * su;
        float cosThetaH;
        if (rl <= pDiffuse + pSpecular)
            cosThetaH = sqrtf((1.0f - sv) / (1.0f + ((alphaGTR2 * alphaGTR2) - 1.0f) * sv));
        else {
            float a2 = alphaGTR1 * alphaGTR1;
            cosThetaH = sqrtf((1.0f - pnm_pow(a2, 1.0f - sv)) / (1.0f - a2));
        }
        float sinThetaH = fmax_(0.0f, 1.0f - sqr(cosThetaH));
        float sinPhiH = pnm_sin(phiH), cosPhiH = 1.0f - sqr(sinPhiH);
        f3 h = tangent_to_world(T, B, N, mk3(sinThetaH * cosPhiH, sinThetaH * sinPhiH, cosThetaH));
        L = sub(smul(2.0f * dot(V, h), h), V);
    }
    f3 H = normalize(add(L, V));
    float LdotH = dot(L, H), NdotH = dot(N, H), NdotLs = dot(N, L);
    float pdfDiffuse = NdotLs * PT_INVPI;
    float pdfSpecular = (gtr2(NdotH, alphaGTR2) * NdotH) / (4.0f * LdotH);
    float pdfClearcoat = (gtr1_ctx(bc, NdotH) * NdotH) / (4.0f * LdotH);
    float dPDF = (pDiffuse * pdfDiffuse + pSpecular * pdfSpecular) + pClearcoat * pdfClearcoat;
    f3 dBRDF = disney(bc, L);
    float NdotL = pnm_fabs(dot(N, L));
    rays.dC = L;
    rays.oP = P;
    rays.oOff = add(P, muls(N, 0.0001f));
    ps_st(w.P0, i, make_float4(rays.oOff.x, rays.oOff.y, rays.oOff.z, dPDF));
    ps_st(w.P2, i, make_float4(dBRDF.x, dBRDF.y, dBRDF.z, pe));
    ps_st(w.P5, i, make_float4(q.Lo.x, q.Lo.y, q.Lo.z, __uint_as_float(seed)));
    bool contMoot = false;
    if constexpr (WF_SKIP_MOOT && MOOT) {
        // Shadow rays whose outcome cannot change the path are not traced.  A
        // shadow ray's occlusion reaches nothing but the shade's MIS sum (:936-940),
        //   Lo1 = Lo + t,  t = (cw * (LE' pe + LD' pl')) * (1 / ((pe + pl') + dPDF)),
        // with (LD', pl') = (LD, pl) or (0, 0) (light ray unoccluded / occluded,
        // :890) and LE' = LE or 0 (env ray, :922).  Rounding to nearest is symmetric
        // and monotone, so |t| is at most the same chain on magnitudes in the same
        // order: T_U = (|cw| (|LE| pe + |LD| pl)) rU for the light-unoccluded
        // outcomes, T_E = (|cw| |LE| pe) rE for the occluded ones, each reciprocal
        // (of |(pe + pl) + dPDF|, |(pe + 0) + dPDF|) taken as rcp * (1 + 2^-20),
        // above the rounded quotient; T = T_U + T_E >= both (a sum, so a NaN in
        // either reaches T).  Lo + t is monotone in t: where Lo + T and Lo - T both
        // round back to Lo, every outcome gives Lo's bits (Lo is never -0: it starts
        // at +0 and only takes round-to-nearest sums, so Lo + (+-0) = Lo) -- the term
        // lies below Lo's rounding, or cw / LD / LE is zero.  Both rays are then
        // moot: their meta bits are cleared (the shade adds the "occluded" term,
        // which leaves Lo), the env ray is not queued, and the light ray (traced from
        // the path state) gets a NaN direction, which the trace's root box test
        // rejects.  A NaN or infinite operand, or a zero denominator, makes T NaN or
        // infinite: no skip; nor is there one where a reciprocal falls below 2^-126
        // (where v_rcp_f32 may return 0, no bound).
        //
        // The last bounce's continuation ray reaches only the term it adds to Lo1
        // (:950-969): ((cw * em) * dBRDF) * NdotL / dPDF, em the hit material's
        // emission, or the env radiance on a miss (or nothing), every component
        // within s.emit_max (host: the largest |emission| of any material and
        // |texel| of the env image).  Tc = (((|cw| emit_max) |dBRDF|) NdotL)
        // rcp(|dPDF|) (1 + 2^-20) bounds it the same way.  The ray is moot where Tc
        // is 0 (the term is +-0 for every outcome: Lo1 + +-0 = Lo1, Lo1 never -0) or
        // where Lo1 = Lo is proven (the test above) and Lo + Tc, Lo - Tc round to Lo.
        // Then P1 gets a NaN direction (the trace misses it) and NdotL = -1 (never
        // a real value, |N.L| >= 0), which the shade reads as "write Lo1".
        const bool last = bounce + 1 == fp.max_depth;
        if ((nfl & (WF_RLIGHT | WF_RENV)) || last) {
            // the candidates read back from the lane's own LDS slot (or from what P3 / P4
            // just got: same lane, same addresses, in order -- an L2 round trip); held in
            // registers through the BRDF sample they cost the kernel two spills
            asm volatile("" ::: "memory");
            float4 r3, r4;
            if constexpr (WF_MOOT_LDS) {
                r3 = wf_moot_lds()[threadIdx.x];
                r4 = wf_moot_lds()[256 + threadIdx.x];
            } else {
                r3 = (nfl & WF_RLIGHT) ? w.P3[i] : make_float4(0.f, 0.f, 0.f, 0.f);
                r4 = (nfl & WF_RENV) ? w.P4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            const f3 acw = mk3(fabsf(q.cw.x), fabsf(q.cw.y), fabsf(q.cw.z));
            const f3 mE = mk3(fabsf(r4.x) * fabsf(pe), fabsf(r4.y) * fabsf(pe), fabsf(r4.z) * fabsf(pe));
            const f3 mU = add(mE, mk3(fabsf(r3.x) * fabsf(r3.w), fabsf(r3.y) * fabsf(r3.w), fabsf(r3.z) * fabsf(r3.w)));
            const float rU = __builtin_amdgcn_rcpf(fabsf((pe + r3.w) + dPDF)) * (1.0f + 0x1p-20f);
            const float rE = __builtin_amdgcn_rcpf(fabsf((pe + 0.f) + dPDF)) * (1.0f + 0x1p-20f);
#if WF_MOOT_TSUM
            const f3 T = add(muls(mul(acw, mU), rU), muls(mul(acw, mE), rE));
#else
            const f3 T = muls(mul(acw, mU), fmaxf(rU, rE));     // (looser: the light term over rE)
#endif
            const f3 hi = add(q.Lo, T), lo = sub(q.Lo, T);
            // (a reciprocal below 2^-126 -- a denominator above 2^126 -- may come back
            // flushed to 0 from v_rcp_f32 and bound nothing: no skip)
            const bool moot = rU >= 0x1p-126f && rE >= 0x1p-126f && hi.x == q.Lo.x && hi.y == q.Lo.y &&
                              hi.z == q.Lo.z && lo.x == q.Lo.x && lo.y == q.Lo.y && lo.z == q.Lo.z;
            if (last) {
                const float rc = __builtin_amdgcn_rcpf(fabsf(dPDF)) * (1.0f + 0x1p-20f);
                const f3 Tc = muls(muls(mul(muls(acw, s.emit_max), mk3(fabsf(dBRDF.x), fabsf(dBRDF.y), fabsf(dBRDF.z))),
                                        NdotL), rc);
                const f3 hc = add(q.Lo, Tc), lc = sub(q.Lo, Tc);
                contMoot = rc >= 0x1p-126f &&
                           ((Tc.x == 0.f && Tc.y == 0.f && Tc.z == 0.f) ||
                            (moot && hc.x == q.Lo.x && hc.y == q.Lo.y && hc.z == q.Lo.z && lc.x == q.Lo.x &&
                             lc.y == q.Lo.y && lc.z == q.Lo.z));
                if (WF_STATS && contMoot) atomicAdd(&b.stats[58], 1ull);
            }
            if (moot && (nfl & (WF_RLIGHT | WF_RENV))) {
                if (WF_STATS) {     // census builds: moot rays per kind (pnrt_device.hip report_trace_diag)
                    if (nfl & WF_RLIGHT) atomicAdd(&b.stats[56], 1ull);
                    if (nfl & WF_RENV) atomicAdd(&b.stats[57], 1ull);
                }
                if (nfl & WF_RLIGHT)
                    ps_st(w.P7, i, make_float4(__uint_as_float(0x7fc00000u), __uint_as_float(0x7fc00000u),
                                               __uint_as_float(0x7fc00000u), 0.f));
                nfl &= ~(WF_RLIGHT | WF_RENV);
            }
        }
    }
    const float qnan = __uint_as_float(0x7fc00000u);
    ps_st(w.P1, i, contMoot ? make_float4(qnan, qnan, qnan, -1.f) : make_float4(L.x, L.y, L.z, NdotL));
    const uint32_t meta = slot | ((nfl & WF_RLIGHT) ? WF_META_RL : 0u) | ((nfl & WF_RENV) ? WF_META_RE : 0u) |
                          ((uint32_t)bounce << WF_META_BSHIFT);
    ps_st(w.P6, i, make_float4(q.cw.x, q.cw.y, q.cw.z, __uint_as_float(meta)));
    return nfl | WF_RCONT;
}

// Compact the block's rays of each kind into its own queue segment: a ballot
// per wave and one LDS atomic per wave for its slots, no global atomics, no
// barrier.  Each ray's traversal result is independent of every other ray and of
// its queue position.
//
// Rays traced from the path state: every live path has a continuation ray, and a
// light shadow ray whenever the scene has lights (the setup draws one for every
// path, :878-909), and the setup has just compacted the block's live paths to
// entries [256 j, 256 j + total) -- so the segment of such a kind IS that range
// of the path state: origin P0.xyz (the offset origin both kinds start from),
// direction P1.xyz (continuation) or P7.xyz (light), the same floats a ray
// record would copy.  Only the count is stored.  The env shadow rays (drawn only
// where the sampled direction is above the surface) are queued as records.  The
// wave that passes through here last writes the block's counts (its acquire sees
// every other wave's counter updates).  (Grouping a segment's rays by direction
// octant measured neutral for both queued and state-traced kinds.)
PN_DEV void wf_enqueue(const WfBufs& b, uint32_t i, uint32_t nfl, const BounceRays& rays, bool lights) {
    uint32_t* ec = wf_enq_ctr();
    const int lane = threadIdx.x & 63;
    {   // env shadow rays: ready-to-trace records
        const uint64_t m = __ballot((nfl & WF_RENV) != 0u);
        uint32_t base = 0;
        if (lane == 0 && m != 0)
            base = __hip_atomic_fetch_add(ec + 1, (uint32_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        base = __builtin_amdgcn_readfirstlane(base);
        if (nfl & WF_RENV) {
            const size_t slot = PT_CHECK(b.fault, (size_t)blockIdx.x * 256 + base + lanes_below(m), b.npad, PT_SITE_RAY);
            ps_st(b.rayO, slot, make_float4(rays.oP.x, rays.oP.y, rays.oP.z, __uint_as_float(i)));
            ps_st(b.rayD, slot, make_float4(rays.dE.x, rays.dE.y, rays.dE.z, 0.f));
        }
    }
    uint32_t done = 0;
    if (lane == 0) done = __hip_atomic_fetch_add(ec + 3, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__builtin_amdgcn_readfirstlane(done) == blockDim.x / 64 - 1) {
        const uint32_t tot = __hip_atomic_load(wf_live_ctr(), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane < 3) {
            const uint32_t qn = __hip_atomic_load(ec + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            b.segcount[lane * b.nseg_k + blockIdx.x] = WF_QUEUED(lane) ? qn : ((lane == 2 || lights) ? tot : 0u);
        }
        if (lane == 0) b.wr.bcount[blockIdx.x] = tot;
    }
}

#ifndef WF_SHADE_WAVES
#define WF_SHADE_WAVES 5      // waves per SIMD for the shade/setup kernel (<= 96 VGPRs without SLP packing)
#endif
#ifndef WF_GEN_WAVES
#define WF_GEN_WAVES WF_SHADE_WAVES   // waves per SIMD for the gen/setup kernel
#endif

// ---- gen + bounce-0 setup: start every path from its pixel's primary hit -------------------
__global__ void __launch_bounds__(256, WF_GEN_WAVES) pt_wf_gen_setup(DevScene s, FrameParams fp, WfBufs b, const float4* primary,
                                                       float4* colors) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;     // path slot
    wf_reset_counters(b);
    wf_live_init();
    // the Sobol pairs of bounces 1 .. depth-1 (:539-557) depend only on (bounce, frame):
    // computed here once per batch, read by the shade kernels' setups (the same
    // sobol_pair bits each lane would compute)
    if (i < (uint32_t)max(fp.max_depth - 1, 0) * (uint32_t)b.chunk_frames) {
        const uint32_t bn = 1u + i / (uint32_t)b.chunk_frames, k = i % (uint32_t)b.chunk_frames;
        const uint32_t f = b.first_frame + k, gk = (f + 1u) ^ ((f + 1u) >> 1);
        float su, sv;
        sobol_pair(2u * bn, gk, su, sv);
        b.sobol[(bn - 1u) * (uint32_t)b.chunk_frames + k] = make_float2(su, sv);
    }
    bool cont = false;
    PathIn q;
    int x = 0, py = 0;
    uint32_t frame = 0;
    if (i < b.n) {
        int lr, k;
        wf_coords(b, i, x, lr, k);
        if (x < fp.width && lr < fp.rows) {
            const float4* rec = wf_primary(b, fp, primary, lr, x);
            const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2];
            const int mt = __float_as_int(q0.w);
            const f3 base = mk3(q2.y, q2.z, q2.w);
            if (mt == -1) {                                   // primary miss: env colour only
                wf_write_color(b, fp, colors, k, lr, x, base);
            } else if (fp.max_depth == 0) {
                wf_write_color(b, fp, colors, k, lr, x, add(base, mk3(0.f, 0.f, 0.f)));
            } else {
                py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
                frame = b.first_frame + (uint32_t)k;
                q.P = mk3(q0.x, q0.y, q0.z); q.N = mk3(q1.x, q1.y, q1.z);
                q.u = q1.w; q.v = q2.x; q.mt = mt;
                q.V = neg(camera_dir(fp, x, py));
                q.cw = mk3(1.f, 1.f, 1.f);
                q.Lo = mk3(0.f, 0.f, 0.f);
                q.seed = ((uint32_t)x * 1973u + (uint32_t)py * 9277u + frame * 26699u) | 1u;
                cont = true;
            }
        }
    }
    const uint32_t j = blockIdx.x * 256u + wf_entry_rank(cont);    // compacted path entry
    uint32_t nfl = 0;
    BounceRays rays;
    if (cont) nfl = wf_setup_core<true, false, false>(s, fp, b, j, i, 0, x, py, frame, q, rays);
    wf_enqueue(b, j, nfl, rays, s.n_lights > 0);     // every lane of the wave reaches this point
}

// ---- trace: every ray of the bounce, persistent waves, LDS short stack ------------------------
// Leaf ref -> triangle range; the leaf-table lookup is behind a scene-uniform
// (scalar) branch, so scenes without table leaves pay no divergent branch.
// TBL = s.has_leaf_table, a template argument: the traversal kernels are
// instantiated per scene kind, so a scene without table leaves runs no test at
// all (against a scene-uniform run-time branch: C2 +1.4 %, trace -2.6 %, same box).
template <bool TBL>
PN_DEV void decode_leaf_fast(const DevScene& s, uint32_t ref, int& start, int& cnt) {
    start = (int)((ref >> 7) & 0x7fffffu);
    cnt = (int)(ref & 0x7fu);
    if (TBL) {
        if ((ref & (REF_LEAF | REF_TABLE)) == (REF_LEAF | REF_TABLE) && ref != REF_NONE) {
            const int2 e = s.leaf_table[PT_CHECK(s.fault, ref & 0x3fffffffu, s.n_leaf_table, PT_SITE_LEAF_TABLE)];
            start = e.x;
            cnt = e.y;
        }
    }
}

// The lane's stack position is one register: spa = sp * 2048 + 8 * tl, the LDS
// byte address of entry sp of lane tl (entries of one depth are 2048 B apart,
// 256 lanes x 8 B; WF_SPA_STRIDE in general), so sp = spa >> 11 and the lane's slot is spa & 2047 -- no
// separate per-lane base register (at 8 waves/SIMD the compiler spilled it).
// Entries deeper than STK go to the block's region of the global spill area
// (ovf_stride depths x 2048 B), laid out like the LDS stack, so the buffer
// access takes spa itself as its per-lane offset: the resource starts STK
// depths before the area and the block's region is the access's scalar
// offset -- no per-lane address arithmetic (the lane-major layout cost 2 VALU
// per step, hoisted out of the rare spill branches by the compiler).
PN_DEV __amdgpu_buffer_rsrc_t wf_ovf_rsrc(const WfBufs& b, int stk) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((char*)b.ovf - (size_t)stk * WF_SPA_STRIDE), (short)0, 0x7fffffff,
                                             0x00020000);
}
PN_DEV int wf_ovf_soff(const WfBufs& b) { return (int)(blockIdx.x * b.ovf_stride * WF_SPA_STRIDE); }
// Push and pop run without branches around the LDS access: every lane of the
// wave writes (push) or reads (pop) one LDS slot whether or not it moves its top
// -- the free slot above the top, or, when that depth is in the spill area (or
// the stack is empty), the lane's slot of one spare depth STK (the minimum of
// the two addresses) -- and only lanes that push/pop move spa.  Only the rare
// spill-area access stays in a branch.
// (Against a branch around the access: C2 +2.2 %, profiles/r03/ab_stack_bl_s11.txt.)
template <int STK>
PN_DEV uint32_t wf_spare() { return (STK * WF_SPA_STRIDE) | (threadIdx.x * 8u); }   // (= its spa & 2047, kept live: 2 VALU per step less)
template <int STK>
PN_DEV void wf_push(uint2* lds, const WfBufs& b, uint32_t& spa, bool push, uint32_t ref, float z) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const uint2 e = make_uint2(ref, __float_as_uint(z));
    *reinterpret_cast<uint2*>(reinterpret_cast<char*>(lds) + min(spa, wf_spare<STK>())) = e;
    if (push & (spa >= STK * WF_SPA_STRIDE)) {
        (void)PT_CHECK(b.fault, (spa >> WF_SPA_SHIFT) - STK, b.ovf_stride, PT_SITE_SPILL);
        const u2 v = {e.x, e.y};
        __builtin_amdgcn_raw_buffer_store_b64(v, wf_ovf_rsrc(b, STK), (int)spa, wf_ovf_soff(b), 0);
    }
    spa += push ? WF_SPA_STRIDE : 0u;
}
template <int STK>
PN_DEV uint2 wf_pop(const uint2* lds, const WfBufs& b, uint32_t& spa, bool pop) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const uint32_t pa = spa - WF_SPA_STRIDE;      // wraps for an empty stack -> the spare slot
    uint2 e = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(lds) + min(pa, wf_spare<STK>()));
    // the spill read is a buffer load, which the compiler cannot merge with the
    // LDS read into one flat load (a flat load waits for every outstanding
    // vector-memory operation, stores included)
    if (pop & (pa >= STK * WF_SPA_STRIDE)) {
        (void)PT_CHECK(b.fault, (pa >> WF_SPA_SHIFT) - STK, b.ovf_stride, PT_SITE_SPILL);
        const u2 v = __builtin_amdgcn_raw_buffer_load_b64(wf_ovf_rsrc(b, STK), (int)pa, wf_ovf_soff(b), 0);
        e = make_uint2(v.x, v.y);
    }
    spa = pop ? pa : spa;
    return e;
}

// BoundIntersect (:213-228) for traversal decisions.  v_min / v_max (IEEE
// minNum / maxNum) drop NaNs exactly like the oracle's min/max; the results only feed
// comparisons, where the sign of a zero cannot matter -> same booleans.
// box_slabs takes the six slab distances (far x y z, near x y z) and returns the
// box's z-slab lower end (zlo) in the triangle test's frame.
// (v_min / v_max written out: the slab distances are products, never signalling
// NaNs, so the IEEE-mode instructions are fminf / fmaxf here -- the compiler's
// own fminf inserted a quieting v_max x, x on two of them every step)
PN_DEV float vmin(float a, float b) { float r; asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
PN_DEV float vmax(float a, float b) { float r; asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
PN_DEV float vmin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
PN_DEV float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
template <bool IDENT = false>
PN_DEV bool box_slabs(const RayP& r, float fx, float fy, float fz, float nx, float ny, float nz, float& zlo) {
    const float zmin = vmin(fz, nz), zmax = vmax(fz, nz);
    float t1 = vmin3(vmax(fx, nx), vmax(fy, ny), zmax);
    float t0 = vmax3(vmin(fx, nx), vmin(fy, ny), zmin);
    const int kz = IDENT ? 2 : r.kz();
    float zf = kz == 2 ? fz : (kz == 0 ? fx : fy);
    float zn = kz == 2 ? nz : (kz == 0 ? nx : ny);
    // the z-slab ends only matter for culling-enabled rays, whose z-slab
    // distances are never NaN (finite ray, |d_kz| >= 1e-12, finite boxes: the
    // host disables culling otherwise), so min / max equal the compare-selects
    // of pt_kernel.h box_test -- and for kz = 2 they are the t0 / t1 terms above
    float lo = IDENT ? zmin : vmin(zn, zf), hi = IDENT ? zmax : vmax(zn, zf);
    zlo = lo;
    // zhi <= 0: the whole box is behind the ray in the triangle test's frame
    return (t1 >= t0) & !(r.cull_ok() & (hi <= 0.0f));
}
template <bool IDENT = false>
PN_DEV bool box_fast(const RayP& r, float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                     float& zlo) {
    float fx = (mxx - r.o.x) * r.inv.x, fy = (mxy - r.o.y) * r.inv.y, fz = (mxz - r.o.z) * r.inv.z;
    float nx = (mnx - r.o.x) * r.inv.x, ny = (mny - r.o.y) * r.inv.y, nz = (mnz - r.o.z) * r.inv.z;
    return box_slabs<IDENT>(r, fx, fy, fz, nx, ny, nz, zlo);
}

#ifndef WF_KIND_ORDER
#define WF_KIND_ORDER 0x210 // sweep order of the ray kinds, one hex digit each (0 light, 1 env, 2 continuation)
#endif

PN_DEV float4 geo_load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// One lane's traversal state (a ray being traced).
// The pending triangle range: in a wide-encoding scene (TBL) lt = first, lc =
// count; in a packed one (pt_common.h) lt holds the range as its leaf ref,
// REF_LEAF | count << 24 | first, and lc is unused -- the word a node or the
// stack supplies is the state itself (no decode), a pending triangle is one
// compare, a step one add, and the fetch offset's mad_u24 reads the first
// triangle from the low 24 bits; hitTri is then such a word too (or -1).
struct TravState {
    RayP r;
    float tMax;
    int hitTri, lt, lc;       // accepted triangle; pending triangle range [lt, lt + lc)
    uint32_t spa, cur;        // stack position (see wf_push); node to visit next
    uint32_t rid;             // kind << 30 | flags | path: kinds 0 / 1 (shadow rays) are any-hit, kind 2 closest-hit
    uint32_t nst;             // WF_STATS builds: lane steps of this ray
};

template <bool TBL>
PN_DEV bool wf_has_tri(const TravState& t) { return TBL ? t.lc > 0 : (uint32_t)t.lt >= (REF_LEAF | (1u << 24)); }
#define WF_RID_P WF_META_SLOT         // TravState::rid: kind << 30 | flags | path entry (< 2^WF_SLOT_BITS)
#define WF_RID_NOCOOP (1u << 29)      // the cooperative finish gave this ray back (traced alone to the end)
// A ray (t.r set) starts: the root box test (:433), tMax, no hit, empty stack.
template <bool TBL>
PN_DEV void wf_ray_start(const DevScene& s, TravState& t, float tmax) {
    float zlo;
    uint32_t root = REF_NONE;
    int nlt = 0, nlc = 0;
    if (box_fast(t.r, s.root_min[0], s.root_min[1], s.root_min[2], s.root_max[0], s.root_max[1], s.root_max[2], zlo)) {
        root = s.root_ref;
        if (root & REF_LEAF) { if (TBL) decode_leaf(s, root, nlt, nlc); else nlt = (int)root; root = REF_NONE; }
    }
    t.tMax = tmax;
    t.hitTri = -1; t.spa &= WF_SPA_STRIDE - 1u; t.cur = root; t.lt = nlt; t.lc = nlc;
    t.nst = 0;
}
// The triangle index of an accepted-hit word.  The mask goes through an opaque
// v_and: with a plain `h & 0xffffff` feeding a 64-bit address (hit_fetch) this
// compiler (ROCm 7.2 clang, gfx950) emitted v_mad_u64_u32 on the UNMASKED word
// -- the mask dropped as if the multiply were a 24-bit one -- and the primary
// pass read far outside the triangle array (a GPU memory fault).
template <bool TBL>
PN_DEV int wf_tri_index(int h) {
    if (TBL || h == -1) return h;
    int r;
    asm("v_and_b32 %0, 0xffffff, %1" : "=v"(r) : "v"(h));
    return r;
}

// One traversal step of a lane's ray; returns true when the ray is finished
// (an any-hit ray accepted a triangle, or nothing is left to visit).
template <int STK, bool ID, bool TBL>
PN_DEV __attribute__((always_inline)) bool wf_step(const DevScene& s, const WfBufs& b, __amdgpu_buffer_rsrc_t geo,
                                                   uint2* lds, TravState& t) {
    // One step, written branch-light: the triangle test and the node
    // visit are both evaluated (a wave almost always holds lanes of
    // both kinds, so both paths ran anyway) and their results are
    // selected per lane; only the rare memory side effects (the stack's
    // spill area, the result store) and the IEEE division stay in branches.
    const bool isTri = wf_has_tri<TBL>(t);
    const bool isNode = t.cur != REF_NONE;     // (a lane with pending triangles has cur = REF_NONE)
    if (WF_DIAG_BOUNDS) {                      // (the buffer loads below are range-checked by the hardware)
        if (isNode) (void)PT_CHECK(s.fault, t.cur, s.n_nodes, PT_SITE_NODE);
        if (isTri) (void)PT_CHECK(s.fault, TBL ? (uint32_t)t.lt : (uint32_t)t.lt & 0xffffffu, s.n_tris, PT_SITE_TRI);
    }
    // ---- the step's single fetch: a triangle record or a node; a lane with
    // neither asks for REF_NONE * 64, beyond the buffer's range, so its loads
    // return zeros without a cache access (it used to re-read node 0: +0.6 %)
    // (an arithmetic select: written as ?: the compiler branches around the two halves)
    const uint32_t offT = s.geo_tri_off + __umul24((uint32_t)t.lt, 48u), offN = t.cur * 64u;
    const uint32_t off = offN ^ ((offT ^ offN) & (0u - (uint32_t)isTri));
    // triangle lanes need no fourth quarter: their cur is REF_NONE (entering a
    // leaf clears it), so offN + 48 lies beyond the buffer's range too (zeros, no
    // cache access; it used to be one shared address)
    const uint32_t off3 = offN + 48u;
    const float4 q0 = geo_load(geo, off), q1 = geo_load(geo, off + 16u), q2 = geo_load(geo, off + 32u),
                 q3 = geo_load(geo, off3);
    // triangle test (:254-357 / :360-424)
    float e0, e1, e2, det, ts;
    const bool acc = tri_test<ID>(t.r, q0, q1, q2, t.tMax, e0, e1, e2, det, ts) & isTri;
    t.hitTri = acc ? t.lt : t.hitTri;
    const bool any = t.rid < (2u << 30);      // (a compare, not a bool kept in a register)
    bool done = acc & any;
    if (acc & !any) t.tMax = ts * (1.0f / det);
    if (TBL) {
        t.lt += isTri ? 1 : 0;
        t.lc -= isTri ? 1 : 0;
    } else {
        t.lt = isTri ? (int)((uint32_t)t.lt + (1u - (1u << 24))) : t.lt;     // first + 1, count - 1
    }
    // node visit: both child boxes (:447-457), z-slab culling
    const uint4 m = make_uint4(__float_as_uint(q3.x), __float_as_uint(q3.y), __float_as_uint(q3.z),
                               __float_as_uint(q3.w));
    // z > tMax * (1 + 1e-6) and z > 1e-20 as one compare: against the larger of
    // the two, keeping a NaN tMax (then nothing is culled, as before)
    const float tmc = t.tMax * 1.000001f;
    const float zc = tmc <= 1e-20f ? 1e-20f : tmc;
    float zloL, zloR;
    bool hL = box_fast<ID>(t.r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, zloL);
    bool hR = box_fast<ID>(t.r, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, zloR);
    const bool cull = t.r.cull_ok();
    hL = hL & !(cull & (zloL > zc)) & isNode;
    hR = hR & !(cull & (zloR > zc)) & isNode;
    const bool rightFirst = ((uint32_t)t.r.perm & m.z) != 0u;     // dir[axis] < 0 (:448; RayP::perm)
    const uint32_t farRef = rightFirst ? m.x : m.y;
    const float zFar = rightFirst ? zloL : zloR;
    // both children hit: continue with the near one, push the far one; one hit:
    // continue with it.  The right child is taken when it is hit and either the
    // left one is not or the right one is the near one -- one mask, two selects
    const bool both = hL & hR;
    wf_push<STK>(lds, b, t.spa, both, farRef, zFar);
    const uint32_t go = (hR & (!hL | rightFirst)) ? m.y : (hL ? m.x : REF_NONE);
    if (TBL) {
        const bool goLeaf = (go != REF_NONE) & ((go & REF_LEAF) != 0u);
        int gs, gc;
        decode_leaf_fast<TBL>(s, go, gs, gc);
        t.lt = goLeaf ? gs : t.lt;
        t.lc = goLeaf ? gc : t.lc;
    } else {
        t.lt = ((go != REF_NONE) & ((go & REF_LEAF) != 0u)) ? (int)go : t.lt;
    }
    // a leaf or REF_NONE (both negative as int) -> REF_NONE, a node index stays;
    // lanes that are no node lane keep REF_NONE (go is REF_NONE for them)
    t.cur = (uint32_t)max((int)go, -1);
    // ---- next fetch target: pop when nothing is pending
    const bool idle = !done & !wf_has_tri<TBL>(t) & (t.cur == REF_NONE);
    const bool stacked = t.spa >= WF_SPA_STRIDE;
    done = done | (idle & !stacked);
    {
        const bool pop = idle & stacked;
        const uint2 e = wf_pop<STK>(lds, b, t.spa, pop);
        const float z = __uint_as_float(e.y);
        const bool take = pop & !(cull & (z > zc));     // (zc: tMax after this step's acceptance, as before)
        const bool eLeaf = (e.x & REF_LEAF) != 0u;
        if (TBL) {
            int es, ec;
            decode_leaf_fast<TBL>(s, pop ? e.x : REF_NONE, es, ec);   // (a non-popping lane's word may be stale: no table lookup)
            t.lt = (take & eLeaf) ? es : t.lt;
            t.lc = (take & eLeaf) ? ec : t.lc;
            t.cur = (take & !eLeaf) ? e.x : t.cur;
        } else {
            // (as above: a popped node index reads as no pending triangle, a
            // popped leaf becomes REF_NONE in cur)
            t.lt = take ? (int)e.x : t.lt;
            t.cur = take ? (uint32_t)max((int)e.x, -1) : t.cur;
        }
    }
    return done;
}

// ---- wave-cooperative finish of a wave's last any-hit ray (WF_COOP_TAIL) ----------------------
// Once the ray queue is exhausted, the end of a trace launch is set by its
// slowest rays: a wave holding one last ray steps it alone, one dependent fetch
// per lane step (about 1 us each), while its other 63 lanes idle -- the drain
// tail that dominates a lone frame's trace launch (queues
// dry after 15-37 us of a 185-us launch at 512x512).  Those last rays are mostly
// shadow rays (the sweep ends on them), and an any-hit ray's result does not
// depend on the visit order: occlusion is the OR over every reachable triangle
// (every ancestor box passes the reference's slab test, :464-494) of the
// watertight test at the ray's FIXED tMax.  So the wave's 64 lanes finish it
// together: the ray's remaining work -- its LDS / spill stack entries, its node
// to visit and its pending triangle range -- becomes a frontier in the wave's
// LDS stack slots (free: every other lane is idle), and each iteration up to 64
// lanes take one entry each: a node tests both child boxes with the same box
// test and z-slab cull as wf_step and adds the children that pass; a leaf range
// tests its first triangle with the same triangle test and adds the rest.  The
// ray is occluded iff some lane accepts a triangle -- the same boolean, in
// about tree-depth iterations instead of one per visited box.
// Frontier capacity: (STK + 1) x 64 entries.  Up to 64 entries per iteration
// while the frontier holds at most CAP - 128, else one (depth-first: +1 per
// descent, at most the tree depth < 63 before a leaf), so it never overflows.
#ifndef WF_COOP_TAIL
#define WF_COOP_TAIL 2      // 0 off, 1 any-hit rays, 2 a wave's last rays of any kind together (wf_coop_multi)
#endif                      // in the launches of a call with nothing else in flight (pt_wf_trace<.., CC>, render_batch)
// The finishes' limits (pt_diag.h WF_DIAG_COOP_SMALL shrinks them so the fallbacks run):
// the frontier size above which one entry per iteration is taken (depth-first), the
// closest-hit candidates the fold takes (at most a wave), the key's sentinel bit
#if WF_DIAG_COOP_SMALL
#define WF_COOP_WIDE(cap) 8u
#define WF_COOP_MAXCAND 2u
#else
#define WF_COOP_WIDE(cap) ((cap) - 128u)
#define WF_COOP_MAXCAND 64u
#endif
// The owner's stack lives in `lds` (its slots, depth d at d * stride + 8 * otl, and the
// spill area); the frontier is built in the wave's slots of `fr` -- the same area as
// `lds` in the product library (every other lane of the wave is idle then), an area of
// its own in WF_DIAG_COOP builds (other lanes still trace).
template <int STK>
PN_DEV bool wf_coop_anyhit(const DevScene& s, const WfBufs& b, __amdgpu_buffer_rsrc_t geo, const uint2* lds, uint2* fr,
                           const RayP& r, float tMax, uint32_t cur, uint32_t lt, uint32_t spa, uint32_t otl) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    constexpr uint32_t CAP = (STK + 1) * 64u;
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    auto slot = [&](uint32_t e) -> uint32_t {      // LDS byte address of frontier entry e
        e = (uint32_t)PT_CHECK(b.fault, e, CAP, PT_SITE_COOP);
        return (e >> 6) * WF_SPA_STRIDE + 8u * (wbase + (e & 63u));
    };
    const float tmc = tMax * 1.000001f;
    const float zc = tmc <= 1e-20f ? 1e-20f : tmc;      // wf_step's cull bound (tMax is fixed)
    const bool cull = r.cull_ok();
    // the owner's stack: depth d < sp at spa = d * stride + 8 * otl (LDS below STK, spill area above)
    const uint32_t sp = spa >> WF_SPA_SHIFT;
    uint2 e = make_uint2(REF_NONE, 0u);
    if (lane < sp) {
        const uint32_t a = lane * WF_SPA_STRIDE + 8u * otl;
        if (lane < (uint32_t)STK) {
            e = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(lds) + a);
        } else {
            (void)PT_CHECK(b.fault, lane - (uint32_t)STK, b.ovf_stride, PT_SITE_SPILL);
            const u2 v = __builtin_amdgcn_raw_buffer_load_b64(wf_ovf_rsrc(b, STK), (int)a, wf_ovf_soff(b), 0);
            e = make_uint2(v.x, v.y);
        }
    }
    // + the node it would visit next and its pending triangle range (leaf word)
    if (lane == sp) e = make_uint2(cur, 0u);
    if (lane == sp + 1) e = make_uint2(lt, 0u);
    const bool valid = (lane < sp) | ((lane == sp) & (cur != REF_NONE)) |
                       ((lane == sp + 1) & ((uint32_t)lt >= (REF_LEAF | (1u << 24))));
    uint64_t m = __ballot(valid);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // every read of the owner's slots before the writes
    if (valid) *reinterpret_cast<uint2*>(reinterpret_cast<char*>(fr) + slot(lanes_below(m))) = e;
    uint32_t size = (uint32_t)__popcll(m);
    bool hit = false;
    while (size > 0) {
        const uint32_t k = size > WF_COOP_WIDE(CAP) ? 1u : min(size, 64u);
        const bool mine = lane < k;
        uint2 f = make_uint2(REF_NONE, 0u);
        if (mine) f = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(fr) + slot(size - 1u - lane));
        size -= k;
        // an entry's z: a pushed far child's z-slab lower end, culled as wf_pop culls it
        const bool take = mine & (f.x != REF_NONE) & !(cull & (__uint_as_float(f.y) > zc));
        const bool isTri = take & (f.x >= (REF_LEAF | (1u << 24)));
        const bool isNode = take & ((f.x & REF_LEAF) == 0u);
        const uint32_t offT = s.geo_tri_off + __umul24(f.x, 48u), offN = isNode ? f.x * 64u : REF_NONE * 64u;
        const uint32_t off = isTri ? offT : offN;
        const float4 q0 = geo_load(geo, off), q1 = geo_load(geo, off + 16u), q2 = geo_load(geo, off + 32u),
                     q3 = geo_load(geo, offN + 48u);
        float e0, e1, e2, det, ts;
        const bool acc = tri_test<false>(r, q0, q1, q2, tMax, e0, e1, e2, det, ts) & isTri;
        float zloL, zloR;
        bool hL = box_fast<false>(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, zloL);
        bool hR = box_fast<false>(r, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, zloR);
        hL = hL & !(cull & (zloL > zc)) & isNode;
        hR = hR & !(cull & (zloR > zc)) & isNode;
        // children to add: a node's passing children (a leaf child only if it holds
        // triangles), a leaf range's remaining triangles
        const uint32_t rest = f.x + (1u - (1u << 24));           // first + 1, count - 1
        const bool cA = isTri ? (rest >= (REF_LEAF | (1u << 24))) : (hL & (__float_as_uint(q3.x) != REF_LEAF));
        const bool cB = hR & (__float_as_uint(q3.y) != REF_LEAF);
        const uint2 eA = isTri ? make_uint2(rest, 0u) : make_uint2(__float_as_uint(q3.x), __float_as_uint(zloL));
        const uint2 eB = make_uint2(__float_as_uint(q3.y), __float_as_uint(zloR));
        if (__ballot(acc) != 0) { hit = true; break; }
        const uint64_t bA = __ballot(cA), bB = __ballot(cB);
        const uint32_t base = size + lanes_below(bA) + lanes_below(bB);
        if (cA) *reinterpret_cast<uint2*>(reinterpret_cast<char*>(fr) + slot(base)) = eA;
        if (cB) *reinterpret_cast<uint2*>(reinterpret_cast<char*>(fr) + slot(base + (cA ? 1u : 0u))) = eB;
        size += (uint32_t)(__popcll(bA) + __popcll(bB));
    }
    return hit;
}

// The same for closest-hit rays, whose result is the LAST triangle the
// reference's depth-first traversal (near child first, a leaf's triangles in
// order, :429-461) accepts against a shrinking tMax -- an order-dependent fold,
// exact only in that order -- and for a wave's last FEW rays at once, any-hit
// and closest-hit mixed (wf_coop_multi: up to WF_COOP_MAXRAYS rays, all 64 lanes
// on one shared frontier).  Two phases:
// 1. The frontier is walked in any order as above, each entry carrying its
//    ray's index and its place in the reference's order as a 64-bit key: ray
//    (2 or 3 bits), the rank of the hand-over entry (pending range 0, node 1, stack
//    top 2, ... bottom), then one bit per level below it (near child 0, far child
//    1) ended by a sentinel bit, and the triangle's place in its leaf in the low
//    8 bits -- the keys of a subtree lie between its entry's key and the next
//    one's.  A closest-hit ray's boxes are culled, and its triangles accepted,
//    against the relaxed bound E (1 + 1e-4), where E is the least hit distance
//    found for that ray so far (from its tMax at the hand-over; an LDS atomic
//    min per ray); each accepted triangle is a candidate (key, index).  An any-hit
//    ray uses its fixed tMax, and its first accepted triangle ends it (its
//    remaining entries are skipped).
// 2. Each closest-hit ray's candidates are folded in key order from the
//    hand-over (tMax, hit) with the exact test and tMax = ts * (1 / det): the
//    reference's result.
// Why the candidates suffice: let B be the least distance among the triangles
// the exact test accepts.  Every triangle within B (1 + 5e-5) of it is a
// candidate (E >= B, and the 1e-4 margin dwarfs the test's rounding); once the
// reference accepts one of those, tMax <= B (1 + 5e-5) and it accepts no
// triangle beyond B (1 + 1e-4) again, nor did anything it accepted before change
// which of them it accepts first (all lie beyond that with margin) -- so both
// folds accept the same triangles from there on and end on the same one.
// The frontier: the wave's LDS stack rows 0 .. STK-1 (16-B entries, (ref, z) +
// key); row STK holds the ray table (64 B per ray: origin, perm; direction,
// tMax; 1/direction, E; kind, done, hit at the hand-over, result).
// Fallback: a closest-hit key deeper than 45-46 levels below the hand-over, or a
// frontier plus candidates beyond the capacity, returns -2 for every ray; more
// than WF_COOP_MAXCAND candidates returns -2 for the closest-hit rays.  A -2 ray
// is traced again from its start by its own lane (WF_RID_NOCOOP; rare, exact
// either way).  The caller guarantees sum over the rays of (stack depth + 2) <= 64.
#ifndef WF_COOP_MAXRAYS
#define WF_COOP_MAXRAYS 8   // rays finished together (<= 8: the ray table fills row STK, 64 B per ray;
#endif                      // D2 synchronised: 2 / 4 / 6 / 8 rays 0.654 / 0.625 / 0.611 / 0.605 ms per frame)
#define WF_COOP_RAYBITS (WF_COOP_MAXRAYS > 4 ? 3 : 2)      // key bits 63.. : the ray
#define WF_COOP_RANKSHIFT (64 - WF_COOP_RAYBITS - 7)       // 7 bits below them: the hand-over rank
static_assert(WF_COOP_MAXRAYS >= 1 && WF_COOP_MAXRAYS <= 8, "the ray table holds at most 8 rays");
template <int STK>
PN_DEV int wf_coop_multi(const DevScene& s, __amdgpu_buffer_rsrc_t geo, const uint2* lds, uint2* fr, const WfBufs& b,
                         const TravState& t, uint64_t owners) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    constexpr uint32_t NSLOT = STK * 64u;              // the wave's 8-B frontier slots (rows 0 .. STK-1)
    constexpr uint32_t CAP = NSLOT / 2u;               // 16-B entries
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    auto at = [&](uint32_t i) -> char* {                // the wave's i-th 8-B frontier slot
        i = (uint32_t)PT_CHECK(b.fault, i, NSLOT, PT_SITE_COOP);
        return reinterpret_cast<char*>(fr) + (i >> 6) * WF_SPA_STRIDE + 8u * (wbase + (i & 63u));
    };
    auto put = [&](uint32_t e, uint2 v, uint64_t key) {
        *reinterpret_cast<uint2*>(at(2u * e)) = v;
        *reinterpret_cast<uint2*>(at(2u * e + 1u)) = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
    };
    // the ray table: row STK of the wave (512 contiguous bytes), 64 B per ray
    char* const tab = reinterpret_cast<char*>(fr) + STK * WF_SPA_STRIDE + 8u * wbase;
    auto row = [&](uint32_t r, uint32_t q) -> float4* {
        return reinterpret_cast<float4*>(tab + ((uint32_t)PT_CHECK(b.fault, r, WF_COOP_MAXRAYS, PT_SITE_COOP) * 64u + q * 16u));
    };
    // the key's sentinel bit below the ray and rank fields (the diagnostic small limits: bit 19)
    const uint64_t TOP = 1ull << (WF_DIAG_COOP_SMALL ? 19 : WF_COOP_RANKSHIFT - 1);
    constexpr int RS = 64 - WF_COOP_RAYBITS;
    const uint32_t nr = (uint32_t)__popcll(owners);
    const bool isOwner = ((owners >> lane) & 1ull) != 0;
    const uint32_t myr = lanes_below(owners);
    // the owners' rays into the table
    if (isOwner) {
        const bool closest = t.rid >= (2u << 30);
        row(myr, 0)[0] = make_float4(t.r.o.x, t.r.o.y, t.r.o.z, __int_as_float(t.r.perm));
        row(myr, 1)[0] = make_float4(t.r.d.x, t.r.d.y, t.r.d.z, t.tMax);
        row(myr, 2)[0] = make_float4(t.r.inv.x, t.r.inv.y, t.r.inv.z, t.tMax);
        row(myr, 3)[0] = make_float4(__int_as_float(closest ? 1 : 0), __int_as_float(0),
                                     __int_as_float(wf_tri_index<false>(t.hitTri)), __int_as_float(0));
    }
    // the initial frontier: ray r's stack entries, its node to visit and its pending
    // range, items [base_r, base_r + sp_r + 2) of at most 64 -- item l read by lane l,
    // every read before any write (the owners' stack slots lie in the rows the frontier
    // overwrites).  (Two items per lane, up to 128: the added registers spilled in the
    // lone-call kernel's step loop.)
    // ray q's items start at lane base_q (base_0 = 0, base_{q+1} = base_q + sp_q + 2: distinct
    // positions below 64) -- kept as one 64-bit mask of the bases, and ray q's owner lane in
    // lane q of `olist`: no per-ray arrays (indexed by a lane's ray they went to scratch)
    uint64_t bases = 0;
    uint32_t olist = 0;
    {
        uint64_t m = owners;
        uint32_t base = 0;
#pragma unroll
        for (int r = 0; r < WF_COOP_MAXRAYS; ++r) {
            if (m) {
                const int o = __ffsll((long long)m) - 1;
                bases |= 1ull << base;
                olist = lane == (uint32_t)r ? (uint32_t)o : olist;
                base += (((uint32_t)__builtin_amdgcn_readlane((int)t.spa, o)) >> WF_SPA_SHIFT) + 2u;
                m &= m - 1;
            }
        }
    }
    auto item = [&](uint32_t l, uint2& e, uint64_t& key) -> bool {
        // the lane's ray: the bases at or below l (l < 64)
        const uint64_t below = bases & (~0ull >> (63u - l));
        const uint32_t r = (uint32_t)__popcll(below) - 1u;
        const uint32_t jb = 63u - (uint32_t)__clzll((long long)below);
        const uint32_t o = (uint32_t)__shfl((int)olist, (int)r);
        const uint32_t ospa = (uint32_t)__shfl((int)t.spa, (int)o);
        const uint32_t ocur = (uint32_t)__shfl((int)t.cur, (int)o);
        const uint32_t olt = (uint32_t)__shfl(t.lt, (int)o);
        const uint32_t sp = ospa >> WF_SPA_SHIFT, otl = (ospa & (WF_SPA_STRIDE - 1u)) >> 3;
        const uint32_t j = l - jb;
        e = make_uint2(REF_NONE, 0u);
        key = (uint64_t)r << RS;
        const bool inRange = j < sp + 2u;
        if (inRange && j < sp) {
            const uint32_t a = j * WF_SPA_STRIDE + 8u * otl;
            if (j < (uint32_t)STK) {
                e = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(lds) + a);
            } else {
                (void)PT_CHECK(b.fault, j - (uint32_t)STK, b.ovf_stride, PT_SITE_SPILL);
                const u2 v = __builtin_amdgcn_raw_buffer_load_b64(wf_ovf_rsrc(b, STK), (int)a, wf_ovf_soff(b), 0);
                e = make_uint2(v.x, v.y);
            }
            key |= ((uint64_t)(2u + (sp - 1u - j)) << WF_COOP_RANKSHIFT) | TOP;
        }
        if (inRange && j == sp) { e = make_uint2(ocur, 0u); key |= (1ull << WF_COOP_RANKSHIFT) | TOP; }
        if (inRange && j == sp + 1u) { e = make_uint2(olt, 0u); key |= TOP; }
        return inRange & ((j < sp) | ((j == sp) & (ocur != REF_NONE)) |
                          ((j == sp + 1u) & (olt >= (REF_LEAF | (1u << 24)))));
    };
    uint2 e0;
    uint64_t key0;
    const bool v0 = item(lane, e0, key0);
    const uint64_t m0 = __ballot(v0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // the owners' slots are read before any write
    if (v0) put(lanes_below(m0), e0, key0);
    uint32_t size = (uint32_t)__popcll(m0), ncand = 0;
    bool fail = false;
    while (size > 0) {
        const uint32_t k = size + ncand > WF_COOP_WIDE(CAP) ? 1u : min(size, 64u);
        const bool mine = lane < k;
        uint2 f = make_uint2(REF_NONE, 0u);
        uint64_t fk = 0;
        if (mine) {
            f = *reinterpret_cast<const uint2*>(at(2u * (size - 1u - lane)));
            const uint2 kk = *reinterpret_cast<const uint2*>(at(2u * (size - 1u - lane) + 1u));
            fk = ((uint64_t)kk.y << 32) | kk.x;
        }
        size -= k;
        const uint32_t fr_r = (uint32_t)(fk >> RS);
        // the entry's ray (lanes without an entry read row 0: unused)
        const float4 T0 = row(fr_r, 0)[0], T1 = row(fr_r, 1)[0], T2 = row(fr_r, 2)[0], T3 = row(fr_r, 3)[0];
        RayP ry;
        ry.o = mk3(T0.x, T0.y, T0.z); ry.perm = __float_as_int(T0.w);
        ry.d = mk3(T1.x, T1.y, T1.z); ry.inv = mk3(T2.x, T2.y, T2.z);
        const bool closest = __float_as_int(T3.x) != 0, done = __float_as_int(T3.y) != 0;
        // closest hit: the relaxed bound from E; any hit: the fixed tMax
        const float er = closest ? T2.w * 1.0001f : T1.w;
        const float tmc = er * 1.000001f;
        const float zc = tmc <= 1e-20f ? 1e-20f : tmc;
        const bool cull = ry.cull_ok();
        const bool take = mine & !done & (f.x != REF_NONE) & !(cull & (__uint_as_float(f.y) > zc));
        const bool isTri = take & (f.x >= (REF_LEAF | (1u << 24)));
        const bool isNode = take & ((f.x & REF_LEAF) == 0u);
        const uint32_t offT = s.geo_tri_off + __umul24(f.x, 48u), offN = isNode ? f.x * 64u : REF_NONE * 64u;
        const uint32_t off = isTri ? offT : offN;
        const float4 q0 = geo_load(geo, off), q1 = geo_load(geo, off + 16u), q2 = geo_load(geo, off + 32u),
                     q3 = geo_load(geo, offN + 48u);
        float e0, e1, e2, det, ts;
        const bool acc = tri_test<false>(ry, q0, q1, q2, er, e0, e1, e2, det, ts) & isTri;
        const bool accC = acc & closest;
        if (acc & !closest) row(fr_r, 3)->y = __int_as_float(1);          // an any-hit ray is occluded
        if (accC) {
            const float th = ts * (1.0f / det);
            // E = the least distance found (a positive float: uint order); a non-finite one ends the cooperation
            fail |= !(pnm_fabs(th) < 3.0e38f);
            __hip_atomic_fetch_min(reinterpret_cast<uint32_t*>(&row(fr_r, 2)->w), __float_as_uint(th), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        float zloL, zloR;
        bool hL = box_fast<false>(ry, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, zloL);
        bool hR = box_fast<false>(ry, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, zloR);
        hL = hL & !(cull & (zloL > zc)) & isNode;
        hR = hR & !(cull & (zloR > zc)) & isNode;
        // children and their keys: near child (:448) = key - sent + sent / 2, far = key + sent / 2
        const uint64_t pk = fk & ~0xffull & ((1ull << WF_COOP_RANKSHIFT) - 1ull);
        const uint64_t sent = pk & (0ull - pk);
        fail |= isNode & closest & (sent <= 0x100ull);     // deeper than a closest-hit key holds
        const bool rightFirst = ((uint32_t)ry.perm & __float_as_uint(q3.z)) != 0u;
        // (an any-hit ray's entries keep their key: only its ray index is read, and the
        // key arithmetic past its depth must not carry into it)
        const uint64_t kNear = closest ? fk - sent + (sent >> 1) : fk, kFar = closest ? fk + (sent >> 1) : fk;
        const uint32_t rest = f.x + (1u - (1u << 24));           // first + 1, count - 1
        const bool cA = isTri ? (rest >= (REF_LEAF | (1u << 24))) : (hL & (__float_as_uint(q3.x) != REF_LEAF));
        const bool cB = hR & (__float_as_uint(q3.y) != REF_LEAF);
        const uint2 eA = isTri ? make_uint2(rest, 0u) : make_uint2(__float_as_uint(q3.x), __float_as_uint(zloL));
        const uint2 eB = make_uint2(__float_as_uint(q3.y), __float_as_uint(zloR));
        const uint64_t kA = isTri ? fk + (closest ? 1u : 0u) : (rightFirst ? kFar : kNear), kB = rightFirst ? kNear : kFar;
        const uint64_t bA = __ballot(cA), bB = __ballot(cB), bC = __ballot(accC);
        const uint32_t nnew = (uint32_t)(__popcll(bA) + __popcll(bB)), nc = (uint32_t)__popcll(bC);
        const bool wfail = (__ballot(fail) != 0) | (size + nnew + ncand + nc > CAP);
        if (wfail) { fail = true; break; }
        const uint32_t base = size + lanes_below(bA) + lanes_below(bB);
        if (cA) put(base, eA, kA);
        if (cB) put(base + (cA ? 1u : 0u), eB, kB);
        // candidates from the top of the area down: (key, triangle index)
        if (accC) put(CAP - 1u - ncand - lanes_below(bC), make_uint2(f.x & 0xffffffu, 0u), fk);
        size += nnew;
        ncand += nc;
    }
    // phase 2: per closest-hit ray, the exact fold over its candidates in key (= the reference's) order;
    // the results into the table's last word (-2: restart)
    const bool own = !fail && lane < ncand && ncand <= WF_COOP_MAXCAND;
    uint32_t tri = 0;
    uint64_t ck = ~0ull;
    if (own) {
        const uint2 v = *reinterpret_cast<const uint2*>(at(2u * (CAP - 1u - lane)));
        const uint2 kk = *reinterpret_cast<const uint2*>(at(2u * (CAP - 1u - lane) + 1u));
        tri = v.x;
        ck = ((uint64_t)kk.y << 32) | kk.x;
    }
    const uint32_t toff = own ? s.geo_tri_off + tri * 48u : REF_NONE * 64u;
    const float4 c0 = geo_load(geo, toff), c1 = geo_load(geo, toff + 16u), c2 = geo_load(geo, toff + 32u);
    for (uint32_t q = 0; q < nr; ++q) {
        const float4 T0 = row(q, 0)[0], T1 = row(q, 1)[0], T2 = row(q, 2)[0], T3 = row(q, 3)[0];
        const bool closest = __float_as_int(T3.x) != 0;
        int res;
        if (fail) {
            res = -2;
        } else if (!closest) {
            res = __float_as_int(T3.y);                   // occluded
        } else if (ncand > WF_COOP_MAXCAND) {
            res = -2;
        } else {
            RayP ry;
            ry.o = mk3(T0.x, T0.y, T0.z); ry.perm = __float_as_int(T0.w);
            ry.d = mk3(T1.x, T1.y, T1.z); ry.inv = mk3(T2.x, T2.y, T2.z);
            const bool mineq = own & ((uint32_t)(ck >> RS) == q);
            float tm = T1.w;
            int hit = __float_as_int(T3.z);
            uint64_t after = 0;               // keys <= after are behind the fold
            bool first = true;
            for (uint32_t guard = 0; guard <= ncand; ++guard) {
                float e0, e1, e2, det, ts;
                const bool pass = mineq & (first | (ck > after)) & tri_test<false>(ry, c0, c1, c2, tm, e0, e1, e2, det, ts);
                if (__ballot(pass) == 0) break;
                uint64_t kmin = pass ? ck : ~0ull;
                for (int w = 32; w > 0; w >>= 1) {
                    const uint64_t v = ((uint64_t)(uint32_t)__shfl_xor((int)(kmin >> 32), w) << 32) |
                                       (uint32_t)__shfl_xor((int)(uint32_t)kmin, w);
                    kmin = v < kmin ? v : kmin;
                }
                const int jw = __ffsll((long long)__ballot(pass & (ck == kmin))) - 1;
                tm = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ts * (1.0f / det)), jw));
                hit = __builtin_amdgcn_readlane((int)tri, jw);
                after = kmin;
                first = false;
            }
            res = hit;
        }
        if (lane == 0) row(q, 3)->w = __int_as_float(res);
    }
    int res = 0;
    if (isOwner) res = __float_as_int(row(myr, 3)->w);
    return res;
}

#ifndef WF_ENV_FAR_FIRST
#define WF_ENV_FAR_FIRST 1    // env shadow rays traverse far child first (wf_load_ray)
#endif
// Ray record `slot` of a kind-`kind` segment -> lane ray state.
PN_DEV void wf_load_ray(const WfBufs& b, uint32_t kind, uint32_t slot, int mode, RayP& r, float& tmax, bool& any,
                        uint32_t& p) {
    // slot = kind * npad + position e in the kind's range; kinds traced from the
    // state the setup wrote read path entry e, the queued kind its record (see
    // wf_enqueue)
    const uint32_t e = (uint32_t)PT_CHECK(b.fault, slot - kind * b.npad, b.npad, PT_SITE_RAY);
    const bool fromState = !WF_QUEUED(kind);     // wave-uniform
    const float4* O = fromState ? b.wr.P0 : b.rayO;
    const float4* D = fromState ? (kind == 0 ? b.wr.P7 : b.wr.P1) : b.rayD;
    const float4 ro = ps_ld(O + e), rd = ps_ld(D + e);
    p = fromState ? e : __float_as_uint(ro.w);
    tmax = kind == 0 ? 1.0f - PT_SHADOW_EPS : PT_FLOAT_MAX;
    any = kind != 2;
    r = make_ray(mk3(ro.x, ro.y, ro.z), mk3(rd.x, rd.y, rd.z), mode);
    // env shadow rays visit the FAR child first (the sign bits of the near-child
    // rule inverted): an any-hit ray's result is the OR over every reachable
    // triangle at its fixed tMax (:464-494; z-culling against a fixed tMax is
    // order-free too), so any visit order gives the same boolean, and an occluded
    // env ray leaving a closed room meets its wall sooner from the far side
    // (tools/step_model: env-ray lane steps -26 % on C2, -28 % on C3)
    if (WF_ENV_FAR_FIRST && kind == 1) r.perm ^= 0x70;
}

// Persistent traversal of every queued ray of the bounce.
//
// One "step" per lane and loop iteration, with a single memory fetch issued by
// the same instructions for every lane: a lane that has a triangle pending
// loads its 48-B record (tris are padded so the 64-B read is in bounds), a lane
// at an interior node loads the node's 64 B (both child boxes, refs, axis).
// The step then runs the triangle test or the node visit, and finally resolves
// the lane's next fetch target -- popping the LDS stack (z-culled entries are
// dropped) -- so a wave with lanes in both states waits for ONE memory latency
// per iteration, not two.  Per lane the sequence of triangle tests and node
// visits is exactly the reference's (near child first, :447-457).
// Control flow stays structured and loop-free inside a step with every
// wave-level decision (ballot) at a reconvergence point: the ray <-> lane
// refill runs between traversal phases.
#ifndef WF_TRACE_WAVES
#define WF_TRACE_WAVES 8      // waves per SIMD (64 VGPRs: no SLP packing, one-register stack position)
#endif
#ifndef WF_TRACE_WAVES_CC
#define WF_TRACE_WAVES_CC 6   // ... for the lone calls' instantiation (CC): 80 VGPRs, no scratch (at 8 waves its
#endif                        // multi-ray finish spilled 12 values, 80 B per lane); a lone call's grid is one block per
                              // 256 paths (the reference's 512x512 frame: 4 blocks per CU), within 6 waves per SIMD
// CC: a wave's last rays, closest-hit ones included, get the cooperative finish (wf_coop_multi) -- its own
// instantiation, launched for a call with nothing else in flight, so the
// pipelined launches run code without it (C2 -0.9 % with it compiled in)
// WF_DIAG_COOP builds: the lane steps after which a ray is handed to the cooperative
// finish, 0..WF_DIAG_COOP, a hash of its kind and path entry
PN_DEV uint32_t wf_coop_hash(uint32_t rid) {
    uint32_t h = (rid & ~WF_RID_NOCOOP) * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}
PN_DEV bool wf_coop_due(const TravState& t) {
    return !(t.rid & WF_RID_NOCOOP) && t.nst >= wf_coop_hash(t.rid) % (uint32_t)(WF_DIAG_COOP + 1) &&
           (t.spa >> WF_SPA_SHIFT) + 2u <= 64u;
}
template <int STK, bool TBL, bool CC = false>
__global__ void __launch_bounds__(WF_TRACE_BLOCK, CC ? WF_TRACE_WAVES_CC : WF_TRACE_WAVES) pt_wf_trace(DevScene s, WfBufs b, int mode) {
    __shared__ uint2 lds[(STK + 1) * WF_TRACE_BLOCK];     // STK depths + the spare one (wf_push)
    // the cooperative finishes' frontier: the wave's own stack slots (the other lanes
    // are idle then), an area of its own in WF_DIAG_COOP builds (they are not)
    __shared__ uint2 lds_coop[WF_DIAG_COOP ? (STK + 1) * WF_TRACE_BLOCK : 1];
    uint2* const fr = WF_DIAG_COOP ? lds_coop : lds;
    // nodes and triangle records through one buffer resource (32-bit offsets)
    const __amdgpu_buffer_rsrc_t geo =
        __builtin_amdgcn_make_buffer_rsrc((void*)s.nodes, (short)0, (int)s.geo_bytes, 0x00020000);
    const int tl = threadIdx.x, lane = tl & 63;
    // rays are dequeued one queue segment at a time (<= 256 rays of one kind from
    // 256 neighbouring paths, kind-major); one atomic per segment
    const uint32_t nseg = 3u * b.nseg_k;
    uint64_t t_start = WF_TIMING ? __builtin_amdgcn_s_memrealtime() : 0, t_exh = 0;
    // WF_STATS: per ray kind, a histogram of lane steps per ray (bucket = floor(log2(steps)))
    __shared__ unsigned int hist[WF_STATS ? 3 * 16 : 1];
    if (WF_STATS) {
        if (threadIdx.x < 48) hist[threadIdx.x] = 0u;
        __syncthreads();
    }
    uint32_t next = 0, end = 0, ckind = 0, qpart = 0;
    bool exhausted = false;

    TravState t;
    t.r = make_ray(mk3(0.f, 0.f, 0.f), mk3(0.f, 0.f, 1.f), 0);
    t.tMax = 0.f;
    t.hitTri = -1; t.lt = 0; t.lc = 0;
    t.spa = (uint32_t)threadIdx.x * 8u;      // stack position (see wf_push)
    t.cur = REF_NONE;
    t.rid = 0u;
    int busy = 0;
    // Ray accounting: when the block's last wave leaves, every ray the block took
    // off the global queue must have been loaded into a lane (a loaded ray is always
    // traced: the loop below ends only with no lane busy).  Generations of the block
    // queue advance only once a segment is fully claimed, and claimed rays are
    // loaded at once (a wave claims as many as it has idle lanes), so the check is
    // that the current generation's segment is used up.  bk_out counts the waves
    // that have left.
    uint64_t last_ray = 0;      // WF_TIMING builds: (iteration, kind, lane steps) of the lane's last finished ray
    uint32_t witer = 0, witer_exh = 0;
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // iters, active, tri, node, idle-pop, refill, rays, -

    // dequeue the wave's next queue item into [next, end) / ckind, or set `exhausted`
    // (wave-uniform; lane 0 issues the atomic)
    auto dequeue = [&]() {
        // WF_QSHARDS dequeue counters, item i on counter i % WF_QSHARDS: the
        // blocks sharing an XCD (blockIdx % 8) start on their own counter and
        // move on when it runs dry, so the global sweep order is unchanged
        // while each counter sees 1/WF_QSHARDS of the device-scope atomics
        uint32_t seg = nseg;
        while (qpart < WF_QSHARDS) {           // (qpart only grows: every shard it passed is dry)
            const uint32_t p = (blockIdx.x + qpart) % WF_QSHARDS;
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(b.counter + p * WF_QSTRIDE, 1u);
            t = __builtin_amdgcn_readfirstlane(t);
            const uint32_t item = t * WF_QSHARDS + p;
            if (item < nseg) {
                seg = item;
                break;
            }
            ++qpart;
        }
        if (seg >= nseg) { exhausted = true; if (WF_TIMING) { t_exh = __builtin_amdgcn_s_memrealtime(); witer_exh = witer; } }
        else {
            // one dequeue = one 256-ray segment.  Kind order of the sweep
            // (WF_KIND_ORDER): continuation rays (closest hit, the longest
            // traversals) first, then env shadow rays, so the launch ends
            // on the short light shadow rays (smaller dequeue grains: -2 to -7 %)
            const uint32_t qk = seg / b.nseg_k;
            const uint32_t j = seg - qk * b.nseg_k;
            ckind = (uint32_t)(WF_KIND_ORDER >> (4 * (2 - (int)qk))) & 0xfu;
            next = ckind * b.npad + j * 256u;
            end = next + b.segcount[ckind * b.nseg_k + j];
        }
    };
    // Block-level ray queue: the block's four waves share one dequeued segment; a
    // wave claims as many rays as it has idle lanes with an LDS atomic on bq_claim
    // = (generation << 16 | rays claimed), the segment of generation g is
    // bq_seg[g & 15] = {first slot, end slot, kind}; the first wave to find it used
    // up (a compare-and-swap on bq_refill) dequeues the next global segment and
    // publishes it as generation g + 1, the others sleep until then.  The last
    // segment of a block is thus worked through by all its waves, not by one.
    // (Fetching the block's next segment ahead of need measured -0.5 %.)
    __shared__ uint32_t bq_claim, bq_refill, bq_done, bk_out;
    __shared__ uint32_t bq_seg[16][3];
    if (threadIdx.x == 0) {
        bq_claim = 0u; bq_refill = 0u; bq_done = 0u; bk_out = 0u;
        bq_seg[0][0] = bq_seg[0][1] = 0u; bq_seg[0][2] = 0u;
    }
    __syncthreads();
    // the next non-empty global segment into next / end / ckind, or exhausted
    auto fetch_segment = [&]() {
        do {
            dequeue();
        } while (!exhausted && next >= end);
    };
    // Every wait is bounded (WF_BQ_GUARD claim attempts, 2^16 sleeps).  A wave that
    // runs out of attempts stops claiming; the rays stay queued for the block's other
    // waves, and a real loss (a published segment left unclaimed, items never
    // dequeued) trips the block / drain checks (WF_FAULT_BLOCK / _DRAIN).  The block's
    // waves are co-resident, so the waits end; diagnostic builds report the guard too.
    auto bclaim = [&](uint32_t want) {
        for (uint32_t guard = 0; guard < WF_BQ_GUARD; ++guard) {
            uint32_t c = 0;
            if (lane == 0) c = __hip_atomic_fetch_add(&bq_claim, want, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            c = __builtin_amdgcn_readfirstlane(c);
            const uint32_t g = c >> 16, old = c & 0xffffu;
            const uint32_t lo = __builtin_amdgcn_readfirstlane(bq_seg[g & 15][0]);
            const uint32_t hi = __builtin_amdgcn_readfirstlane(bq_seg[g & 15][1]);
            if (old < hi - lo) {
                next = lo + old; end = min(next + want, hi);
                ckind = __builtin_amdgcn_readfirstlane(bq_seg[g & 15][2]);
                return;
            }
            if (__hip_atomic_load(&bq_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                exhausted = true;        // (another wave of the block found the queue empty)
                if (WF_TIMING) { t_exh = __builtin_amdgcn_s_memrealtime(); witer_exh = witer; }
                return;
            }
            uint32_t won = 0;
            if (lane == 0) {
                uint32_t e = g;
                won = __hip_atomic_compare_exchange_strong(&bq_refill, &e, g + 1, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP) ? 1u : 0u;
            }
            won = __builtin_amdgcn_readfirstlane(won);
            if (won) {                          // this wave publishes generation g + 1
                fetch_segment();                // skips empty segments
                if (lane == 0) {
                    const uint32_t q = (g + 1) & 15;
                    bq_seg[q][0] = exhausted ? 0u : next;
                    bq_seg[q][1] = exhausted ? 0u : end;
                    bq_seg[q][2] = ckind;
                    if (exhausted) __hip_atomic_store(&bq_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&bq_claim, (g + 1) << 16, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                exhausted = false;              // re-claimed below (every wave leaves through bq_done)
                next = end = 0;
                continue;
            }
            // another wave is fetching generation g + 1
            for (uint32_t w = 0; w < (1u << 16); ++w) {
                const uint32_t c2 = __hip_atomic_load(&bq_claim, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if ((c2 >> 16) != g) break;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        exhausted = true;                       // guard: this wave stops claiming (see above)
        if (PNRT_IS_DIAG_BUILD && lane == 0) wf_fault(b, WF_FAULT_GUARD);
    };
    // one traversal step of a busy lane, the result stored when its ray is done
    auto step_lane = [&](auto ident_tag) {
        constexpr bool ID = decltype(ident_tag)::value;
        if (WF_STATS) {
            st[0] += 1;
            st[1] += __popcll(__ballot(busy != 0));
            st[2] += __popcll(__ballot(busy != 0 && wf_has_tri<TBL>(t)));
            st[3] += __popcll(__ballot(busy != 0 && !wf_has_tri<TBL>(t) && t.cur != REF_NONE));
            st[7] += __popcll(__ballot(busy != 0 && (t.rid >> 30) == 2u));     // continuation-ray lane steps
            {   // steps whose fetch address is the same for every active lane
                const uint64_t act = __ballot(busy != 0);
                const uint32_t fo = wf_has_tri<TBL>(t) ? 0x80000000u + (uint32_t)(t.lt & 0xffffff) : t.cur;
                const uint32_t f0 = __shfl(fo, act ? __ffsll((long long)act) - 1 : 0);
                st[4] += (act != 0 && __ballot(busy != 0 && fo != f0) == 0) ? 1 : 0;
            }
        }
        if (WF_TIMING) ++witer;
        // every lane steps: a lane without a ray holds a finished state (nothing
        // pending, empty stack), whose step fetches beyond the buffer's range,
        // tests nothing and touches only its own free LDS slot -- no branch
        // around the step (against `if (busy)`: C2 +3.5 %, trace -4 %)
        {
            const bool done = wf_step<STK, ID, TBL>(s, b, geo, lds, t) & (busy != 0);
            if (WF_STATS || WF_TIMING || WF_DIAG_COOP) t.nst += busy ? 1 : 0;
            if (WF_STATS && done) atomicAdd(&hist[(t.rid >> 30) * 16 + min(15, 31 - __clz((int)t.nst))], 1u);
            if (WF_TIMING && done) last_ray = (uint64_t)witer << 32 | (t.rid >> 30) << 16 | min(t.nst, 0xffffu);
            if (done) {
                const uint32_t kind = t.rid >> 30, p = (uint32_t)PT_CHECK(b.fault, t.rid & WF_RID_P, b.n, PT_SITE_RESULT);
                if (kind == 2) b.hit[p] = wf_tri_index<TBL>(t.hitTri);
                else b.occ[2 * (size_t)p + kind] = t.hitTri != -1 ? 1 : 0;
                busy = 0;
                t.lt = 0; t.lc = 0; t.cur = REF_NONE; t.spa &= WF_SPA_STRIDE - 1u;     // (an any-hit ray may stop mid-tree)
            }
        }
    };

    for (;;) {
        // ---- refill: idle lanes take the wave's next queued rays; more passes when a
        // segment runs out part-way (wave-uniform control flow only)
        const int busy0 = WF_STATS ? __popcll(__ballot(busy != 0)) : 0;
        auto refill = [&]() {
            const uint64_t idle = __ballot(busy == 0);
            if (idle != 0 && next >= end && !exhausted) bclaim((uint32_t)__popcll(idle));
            if (idle != 0 && next < end) {
                const uint32_t myid = next + lanes_below(idle);
                next = min(next + (uint32_t)__popcll(idle), end);
                if (busy == 0 && myid < end) {
                    const uint32_t kind = ckind;
                    uint32_t p;
                    RayP nr;
                    float ntmax;
                    bool nany;
                    wf_load_ray(b, kind, myid, mode, nr, ntmax, nany, p);
                    t.r = nr;
                    wf_ray_start<TBL>(s, t, ntmax);
                    t.rid = (kind << 30) | p;
                    busy = 1;
                }
            }
        };
        for (int pass = 0; pass < 4 && !exhausted && __ballot(busy == 0) != 0; ++pass) refill();
        if (WF_STATS) { st[5] += 1; st[6] += __popcll(__ballot(busy != 0)) - busy0; }
        const uint64_t busym = __ballot(busy != 0);
        if (busym == 0) {
            if (exhausted) break;
            continue;
        }
        int thr = (__popcll(busym) * WF_REFILL_PCT) / 100;
        // the cooperative finishes.  Owner lanes take the result -- or, for -2 (beyond a
        // finish's limits), restart their ray from the root, traced alone to the end
        auto coop_result = [&](bool owner, int res) {
            if (WF_DIAG_COOP && owner) {          // rays handed over (any-hit, closest-hit), restarts
                atomicAdd(b.stats + (t.rid >= (2u << 30) ? 1 : 0), 1ull);
                if (res == -2) atomicAdd(b.stats + 2, 1ull);
            }
            if (owner) {
                const uint32_t kind = t.rid >> 30;
                if (res == -2) {
                    wf_ray_start<TBL>(s, t, kind == 0 ? 1.0f - PT_SHADOW_EPS : PT_FLOAT_MAX);
                    t.rid |= WF_RID_NOCOOP;
                } else {
                    const uint32_t p = (uint32_t)PT_CHECK(b.fault, t.rid & WF_RID_P, b.n, PT_SITE_RESULT);
                    if (kind == 2) b.hit[p] = res;
                    else b.occ[2 * (size_t)p + kind] = (uint8_t)res;
                    busy = 0;
                    t.lt = 0; t.lc = 0; t.cur = REF_NONE; t.spa &= WF_SPA_STRIDE - 1u;
                }
            }
        };
        // one any-hit ray (lane o, wave-uniform), 8-B frontier entries
        auto coop_anyhit = [&](int o) {
            const uint32_t ospa = (uint32_t)__builtin_amdgcn_readlane((int)t.spa, o);
            auto rdf = [&](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), o)); };
            RayP r;
            r.o = mk3(rdf(t.r.o.x), rdf(t.r.o.y), rdf(t.r.o.z));
            r.d = mk3(rdf(t.r.d.x), rdf(t.r.d.y), rdf(t.r.d.z));
            r.inv = mk3(rdf(t.r.inv.x), rdf(t.r.inv.y), rdf(t.r.inv.z));
            r.perm = __builtin_amdgcn_readlane(t.r.perm, o);
            const uint32_t ocur = (uint32_t)__builtin_amdgcn_readlane((int)t.cur, o);
            const uint32_t olt = (uint32_t)__builtin_amdgcn_readlane(t.lt, o);
            const uint32_t otl = (ospa & (WF_SPA_STRIDE - 1u)) >> 3;
            const int res = wf_coop_anyhit<STK>(s, b, geo, lds, fr, r, rdf(t.tMax), ocur, olt, ospa, otl) ? 1 : 0;
            coop_result(WF_DIAG_COOP ? lane == o : busy != 0, res);   // (the owner: the wave's one busy lane in product builds)
        };
        // the rays of lanes `owners` (<= WF_COOP_MAXRAYS, any kinds), one shared frontier
        // (pipelined launches keep the one-ray any-hit finish: the multi-ray finish there
        // measured C2 -1.8 %, C4 -1.0 %, N = 8 shares -3 %, and gated on half the
        // block's waves having left -2.5 % -- profiles/r05/s3, s12, s13)
        constexpr bool MULTI = CC || WF_DIAG_COOP;
        auto coop_multi = [&](uint64_t owners) {
            if (WF_DIAG_COOP && lane == 0 && __popcll(owners) > 1) atomicAdd(b.stats + 3, 1ull);
            if (WF_DIAG_COOP && ((owners >> lane) & 1ull) && (t.spa >> WF_SPA_SHIFT) > (uint32_t)STK)
                atomicAdd(b.stats + 4, 1ull);       // rays handed over with stack entries in the spill area
            const int res = wf_coop_multi<STK>(s, geo, lds, fr, b, t, owners);
            coop_result(((owners >> lane) & 1ull) != 0, res);
        };
        if (WF_DIAG_COOP && !TBL && !WF_STATS) {
            // diagnostic: every ray goes through a cooperative finish once, at its
            // hash-chosen step (the run loop below stops when one is due): up to
            // WF_COOP_MAXRAYS due rays together, or a lone any-hit ray alone (by hash)
            uint64_t due = __ballot(busy != 0 && wf_coop_due(t));
            if (due != 0) {
                // (greedily, while the rays' stack entries fit the 64 initial items: deep
                // stacks -- entries in the spill area -- are handed over too)
                uint64_t own = 0;
                uint32_t need = 0;
                for (int q = 0; q < WF_COOP_MAXRAYS && due; ++q) {
                    const uint64_t bit = due & (0ull - due);
                    const uint32_t n = ((uint32_t)__builtin_amdgcn_readlane((int)t.spa, __ffsll((long long)bit) - 1) >>
                                        WF_SPA_SHIFT) + 2u;
                    due &= due - 1;
                    if (need + n > 64u) continue;
                    need += n;
                    own |= bit;
                }
                const int o = __ffsll((long long)own) - 1;
                const uint32_t orid = (uint32_t)__builtin_amdgcn_readlane((int)t.rid, o);
                if (__popcll(own) == 1 && orid < (2u << 30) && (wf_coop_hash(orid) & 1u)) coop_anyhit(o);
                else coop_multi(own);
                continue;
            }
        }
        if (WF_COOP_TAIL && !TBL && !WF_STATS) {
            const int nb = __popcll(busym);
            if (MULTI && WF_COOP_TAIL >= 2) {
                // lone calls: once the queue is exhausted -- the drain -- a wave down to
                // WF_COOP_MAXRAYS rays finishes them with all its lanes together
                if (exhausted && nb <= WF_COOP_MAXRAYS) {
                    bool ok = __ballot(busy != 0 && (t.rid & WF_RID_NOCOOP) != 0) == 0;
                    uint32_t need = 0;
                    for (uint64_t m = busym; m; m &= m - 1)
                        need += ((uint32_t)__builtin_amdgcn_readlane((int)t.spa, __ffsll((long long)m) - 1) >> WF_SPA_SHIFT) + 2u;
                    if (WF_DIAG_COOPSTAT && lane == 0) {    // diagnostic census of the drain finish
                        atomicAdd(b.stats + ((ok && need <= 64u) ? 5 : !ok ? 7 : 6), 1ull);
                        if (ok && need <= 64u) atomicAdd(b.stats + 8, (unsigned long long)nb);
                    }
                    if (ok && need <= 64u) {
                        coop_multi(busym);
                        continue;
                    }
                    thr = nb - 1;        // step until one of them is done, then look again
                } else {
                    thr = exhausted ? max(thr, WF_COOP_MAXRAYS) : (nb == 1 ? 0 : max(thr, 1));
                }
            } else {
                // pipelined launches: a wave never steps a lone ray while it could refill
                // around it (back here at one busy lane), and once the queue is exhausted
                // a wave down to one any-hit ray finishes it with all its lanes
                if (nb == 1 && exhausted) {
                    const int o = __ffsll((long long)busym) - 1;
                    const uint32_t orid = (uint32_t)__builtin_amdgcn_readlane((int)t.rid, o);
                    const uint32_t ospa = (uint32_t)__builtin_amdgcn_readlane((int)t.spa, o);
                    if (!(orid & WF_RID_NOCOOP) && (ospa >> WF_SPA_SHIFT) + 2u <= 64u && orid < (2u << 30)) {
                        coop_anyhit(o);
                        continue;
                    }
                    thr = 0;             // not for the cooperative finish: step it to the end
                } else {
                    thr = nb == 1 ? 0 : max(thr, 1);   // come back here when one ray is left
                }
            }
        }
        // ---- traverse until WF_REFILL_PCT % of the lanes have finished their ray --------
        // (IDENT: no lane of the wave needs the triangle test's axis permutation)
        auto run = [&](auto ident_tag) {
            for (;;) {
                step_lane(ident_tag);
                if (__popcll(__ballot(busy != 0)) <= thr) break;
                if (WF_DIAG_COOP && !TBL && !WF_STATS && __ballot(busy != 0 && wf_coop_due(t)) != 0) break;
            }
        };
        if (__ballot(busy != 0 && t.r.kz() != 2) == 0) run(std::true_type{});
        else run(std::false_type{});
    }
    if (lane == 0) {      // the block's last wave out checks the ray accounting
        const uint32_t out = __hip_atomic_fetch_add(&bk_out, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (out == WF_TRACE_BLOCK / 64 - 1) {
            const uint32_t c = __hip_atomic_load(&bq_claim, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t q = (c >> 16) & 15;
            if ((c & 0xffffu) < bq_seg[q][1] - bq_seg[q][0]) wf_fault(b, WF_FAULT_BLOCK);
        }
    }
    if (WF_TIMING && lane == 0) {      // diagnostic builds: per-wave start / queue-empty / end (100 MHz clock)
        unsigned long long* t = b.stats + 8 + 4 * ((size_t)blockIdx.x * (WF_TRACE_BLOCK / 64) + (threadIdx.x >> 6));
        t[0] = t_start; t[1] = t_exh; t[2] = __builtin_amdgcn_s_memrealtime();
        t[3] = 0;
    }
    if (WF_TIMING) {    // the wave's last ray to finish: kind << 16 | its lane steps (max over the wave's lanes)
        uint64_t lr = last_ray;
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t v = ((uint64_t)__shfl_xor((unsigned)(lr >> 32), o) << 32) | (unsigned)__shfl_xor((unsigned)lr, o);
            lr = v > lr ? v : lr;
        }
        if (lane == 0)
            b.stats[8 + 4 * ((size_t)blockIdx.x * (WF_TRACE_BLOCK / 64) + (threadIdx.x >> 6)) + 3] =
                (uint64_t)(witer - witer_exh) << 32 | (lr & 0xffffffffu);
    }
    if (WF_STATS) {
        __syncthreads();
        if (threadIdx.x < 48 && hist[threadIdx.x]) atomicAdd(b.stats + 8 + threadIdx.x, (unsigned long long)hist[threadIdx.x]);
    }
    if (WF_STATS && lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(b.stats + k, st[k]);
}

// ---- primary hits through the trace kernel's step --------------------------------------------
// The primary ray has no jitter (ray_tracing.comp:980), so its closest hit is
// traced once per pixel and reused by every frame of a call -- and of later calls
// while the camera, frame, shard and scene stay the same (pnrt_device.hip
// PrimKey).  The branch-light unified step of pt_wf_trace: one camera ray per
// lane, grid-stride over 256-pixel chunks (grid <= the trace grid, so the trace's
// stack spill area serves it), the same visit order and culling.  (Against a
// one-lane-per-pixel node / leaf loop pass: primary 0.27 -> 0.22 ms per 1080p call,
// D2 synchronised -4 %.)
// Record: q0 = (P.xyz, bits(mat | (tex + 1) << 24)), q1 = (N.xyz, u), q2 = (v,
// base.xyz); mat = -1 on a miss (base = emissive of the hit material, or the env
// colour of the primary direction).
#ifndef PT_PRIM_WF_WAVES
#define PT_PRIM_WF_WAVES 7
#endif
template <int STK, bool TBL>
__global__ void __launch_bounds__(WF_TRACE_BLOCK, PT_PRIM_WF_WAVES) pt_primary_wf(DevScene s, FrameParams fp, WfBufs b,
                                                                               float4* rec) {
    __shared__ uint2 lds[(STK + 1) * WF_TRACE_BLOCK];     // STK depths + the spare one (wf_push)
    const __amdgpu_buffer_rsrc_t geo =
        __builtin_amdgcn_make_buffer_rsrc((void*)s.nodes, (short)0, (int)s.geo_bytes, 0x00020000);
    const size_t npix = (size_t)fp.rows * fp.width;
    for (size_t base = (size_t)blockIdx.x * WF_TRACE_BLOCK; base < npix; base += (size_t)gridDim.x * WF_TRACE_BLOCK) {
        const size_t i = base + threadIdx.x;
        const bool mine = i < npix;
        const int lr = mine ? (int)(i / fp.width) : 0, px = mine ? (int)(i - (size_t)lr * fp.width) : 0;
        const int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
        const f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
        const f3 dir = camera_dir(fp, px, py);
        TravState t;
        t.r = make_ray(eye, dir, fp.mode);
        t.tMax = PT_FLOAT_MAX;
        t.hitTri = -1; t.lt = 0; t.lc = 0;
        t.spa = (uint32_t)threadIdx.x * 8u;
        t.cur = REF_NONE;
        t.rid = 2u << 30;       // closest hit
        float zlo;
        if (mine && box_fast(t.r, s.root_min[0], s.root_min[1], s.root_min[2], s.root_max[0], s.root_max[1],
                             s.root_max[2], zlo)) {
            t.cur = s.root_ref;
            if (t.cur & REF_LEAF) { if (TBL) decode_leaf(s, t.cur, t.lt, t.lc); else t.lt = (int)t.cur; t.cur = REF_NONE; }
        }
        int busy = mine && (t.cur != REF_NONE || wf_has_tri<TBL>(t));
        auto run = [&](auto ident_tag) {
            constexpr bool ID = decltype(ident_tag)::value;
            for (;;) {
                if (wf_step<STK, ID, TBL>(s, b, geo, lds, t)) busy = 0;     // (a finished lane's step is a no-op)
                if (__ballot(busy != 0) == 0) break;
            }
        };
        if (__ballot(busy != 0 && t.r.kz() != 2) == 0) run(std::true_type{});
        else run(std::false_type{});
        if (!mine) continue;
        float4 q0, q1, q2;
        if (t.hitTri != -1) {
            Hit h = make_hit(s, t.r, wf_tri_index<TBL>(t.hitTri));
            f3 em = get_emissive(s, h.mat);
            q0 = make_float4(h.P.x, h.P.y, h.P.z, __int_as_float((h.mat & 0x00ffffff) | ((h.tex + 1) << 24)));
            q1 = make_float4(h.N.x, h.N.y, h.N.z, h.u);
            q2 = make_float4(h.v, em.x, em.y, em.z);
        } else {
            f3 c = env_color(s, dir);
            q0 = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
            q1 = make_float4(0.f, 0.f, 0.f, 0.f);
            q2 = make_float4(0.f, c.x, c.y, c.z);
        }
        rec[3 * i] = q0;
        rec[3 * i + 1] = q1;
        rec[3 * i + 2] = q2;
    }
}

// ---- shade: MIS, continuation hit, next bounce or final colour (:936-972) --------------------
// Path entry i of the read set.  Returns whether the path continues; then q,
// bounce, slot and the pixel / frame carry its next bounce to the setup.
PN_DEV bool wf_shade_path(const DevScene& s, const FrameParams& fp, const WfBufs& b, const float4* primary,
                          float4* colors, uint32_t i, PathIn& q, int& bounce, uint32_t& slot, int& x, int& py,
                          uint32_t& frame) {
    const PathSet& rd = b.rd;
    i = (uint32_t)PT_CHECK(b.fault, i, b.npad, PT_SITE_PATH);
    const float4 p0 = ps_ld(rd.P0 + i), p1 = ps_ld(rd.P1 + i), p6 = ps_ld(rd.P6 + i);
    const float4 p2 = ps_ld(rd.P2 + i), p5 = ps_ld(rd.P5 + i);
    const int ht = b.hit[i];
    // the light / env candidates are read only where they count: an occluded
    // light ray zeroes LDirect and lightPDF (:890), an occluded or absent env ray
    // zeroes LEnvironment (:922; enPDF is kept, in P2.w).  Lanes that need neither
    // read the scene's zero float4 instead (no branch: both loads issue together).
    const uint32_t oc = reinterpret_cast<const uint16_t*>(b.occ)[i];      // both bytes in one load
    asm volatile("" ::: "memory");     // keep the hit load in this first batch (the scheduler sinks it)
    const uint32_t meta = __float_as_uint(p6.w);
    bounce = (int)(meta >> WF_META_BSHIFT);
    slot = meta & WF_META_SLOT;
    const bool useL = (meta & WF_META_RL) && !(oc & 0xffu);
    const bool useE = (meta & WF_META_RE) && !(oc >> 8);
    const float4 p3 = ps_ld(useL ? rd.P3 + i : s.zero4);
    const float4 p4 = ps_ld(useE ? rd.P4 + i : s.zero4);
    // the continuation hit's records, in flight while the MIS sum waits for P3/P4
    // (a miss reads triangle 0's, unused; so does an index a faulted trace left
    // stale -- reported as PNRT_E_TRACE, never a wild read)
    const HitFetch hf = hit_fetch(s, (uint32_t)ht < (uint32_t)s.n_tris ? ht : 0);
    asm volatile("" ::: "memory");     // issue them here (the scheduler would sink them past the MIS wait)
    f3 LD = mk3(p3.x, p3.y, p3.z), LE = mk3(p4.x, p4.y, p4.z);
    float pl = p3.w, pe = p2.w;
    f3 dBRDF = mk3(p2.x, p2.y, p2.z), L = mk3(p1.x, p1.y, p1.z);
    float NdotL = p1.w, dPDF = p0.w;
    f3 Lo = mk3(p5.x, p5.y, p5.z), cw = mk3(p6.x, p6.y, p6.z);
    float invPDFSum = 1.0f / ((pe + pl) + dPDF);
    f3 mis = add(muls(LE, pe), muls(LD, pl));
    Lo = add(Lo, muls(mul(cw, mis), invPDFSum));
    int lr, k;
    wf_coords(b, slot, x, lr, k);
    if (ht < 0) {      // (a moot continuation ray -- NdotL = -1, WF_SKIP_MOOT -- is a miss that adds nothing)
        if (s.has_hdr && !(NdotL < 0.f)) {
            f3 enLi = env_color(s, normalize(L));
            Lo = add(Lo, divs(muls(mul(mul(cw, enLi), dBRDF), NdotL), dPDF));
        }
        const float4 q2 = wf_primary(b, fp, primary, lr, x)[2];     // the primary hit's base colour
        wf_write_color(b, fp, colors, k, lr, x, add(mk3(q2.y, q2.z, q2.w), Lo));
        return false;
    }
    RayP r = make_ray(mk3(p0.x, p0.y, p0.z), L, 0);        // the continuation ray as traced
    Hit h = hit_resolve(r, hf);
    f3 em = get_emissive(s, h.mat);
    Lo = add(Lo, divs(muls(mul(mul(cw, em), dBRDF), NdotL), dPDF));
    cw = mul(cw, divs(muls(dBRDF, NdotL), dPDF));
    ++bounce;
    if (bounce >= fp.max_depth) {
        const float4 q2 = wf_primary(b, fp, primary, lr, x)[2];
        wf_write_color(b, fp, colors, k, lr, x, add(mk3(q2.y, q2.z, q2.w), Lo));
        return false;
    }
    // the next bounce starts here: its setup runs on the state in registers
    q.P = h.P; q.N = h.N; q.u = h.u; q.v = h.v;
    q.mt = (h.mat & 0x00ffffff) | ((h.tex + 1) << 24);
    q.V = neg(L); q.cw = cw; q.Lo = Lo; q.seed = __float_as_uint(p5.w);
    py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    frame = b.first_frame + (uint32_t)k;
    return true;
}

// ---- shade + next-bounce setup: MIS, continuation hit (:936-972), then the next
// bounce's sampling for the paths that continue.  FINAL: the last bounce (every
// path ends here), compiled without the setup half -> fewer registers, more waves.
template <bool FINAL>
__global__ void __launch_bounds__(256, FINAL ? 8 : WF_SHADE_WAVES) pt_wf_shade_setup(DevScene s, FrameParams fp, WfBufs b,
                                                                     const float4* primary, float4* colors) {
    // the block's live paths are its first b.rd.bcount[block] entries
    wf_check_drained(b);                      // (the previous trace's counters, then reset)
    if (!FINAL) wf_reset_counters(b);
    const uint32_t live = b.rd.bcount[blockIdx.x];
    if (live == 0) {                          // no path: nothing to shade, no rays, empty next block
        if (threadIdx.x < 3) b.segcount[threadIdx.x * b.nseg_k + blockIdx.x] = 0u;
        if (threadIdx.x == 0) b.wr.bcount[blockIdx.x] = 0u;
        return;
    }
    if (!FINAL) wf_live_init();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool cont = false;
    PathIn q;
    int bounce = 0, x = 0, py = 0;
    uint32_t slot = 0, frame = 0;
    if (threadIdx.x < live) cont = wf_shade_path(s, fp, b, primary, colors, i, q, bounce, slot, x, py, frame);
    if (FINAL) return;                        // bounce + 1 == max_depth: cont is false for every path
    const uint32_t j = blockIdx.x * 256u + wf_entry_rank(cont);
    uint32_t nfl = 0;
    BounceRays rays;
    if (cont) nfl = wf_setup_core<false, true, true>(s, fp, b, j, slot, bounce, x, py, frame, q, rays);
    wf_enqueue(b, j, nfl, rays, s.n_lights > 0);     // every lane of the wave reaches this point
}
