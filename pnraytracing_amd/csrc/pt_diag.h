// pnraytracing_amd/csrc/pt_diag.h -- the ONE place the diagnostic build switches
// live.  All default to 0, which is the product library; the others exist for
// measurement and fault-injection builds (build.py DIAG_VARIANTS,
// tools/build_variants.sh -> pnraytracing_amd/variants/) and never ship as
// libpnrt.so (pnrt_version() then says DIAGNOSTIC BUILD):
//   WF_STATS        trace-kernel census: lane steps / rays per launch (tools/census.py)
//   WF_TIMING       per-wave timestamps of the trace kernel (drain-tail analysis)
//   WF_DIAG_GUARD   N > 0: the trace kernel's block-queue claim gives up after N
//                   attempts instead of 1024, so waves quit with rays unclaimed --
//                   WRONG IMAGES; exercises the fault report (PNRT_E_TRACE)
//   WF_DIAG_BOUNDS  every fetch / store index of the integrator kernels (nodes,
//                   triangles, attributes, leaf table, stack spill area, ray and
//                   path-state entries, light records, env footprints, albedo
//                   texels, primary records, colours, trace results) is checked
//                   against its array (PT_CHECK); a violation writes its site into
//                   fault word WF_FAULT_BOUNDS (pnrt_* then return PNRT_E_TRACE) and
//                   the index is clamped to 0, so no access leaves its array.  Same
//                   images when nothing trips.  PNRT_DIAG_FORCE_OOB=1 in the
//                   environment makes one gen fetch out of range (the check's test)
//   WF_DIAG_COOP    k > 0: every ray of every trace launch (any-hit and closest-hit)
//                   is handed to the cooperative finish (pt_wf.h wf_coop_anyhit /
//                   wf_coop_closest) after a hash-chosen 0..k lane steps, whatever the
//                   wave's busy count -- the product library reaches it only at a
//                   drained wave's last ray.  The frontier gets an LDS area of its own
//                   (the other lanes' stacks stay intact).  Same images: the finishes
//                   are exact.  Hand-overs and restarts are counted per launch and
//                   printed ("[coop]" lines on stderr)
//   WF_DIAG_COOP_SMALL  with WF_DIAG_COOP: the finishes' limits shrunk -- the one-entry
//                   depth-first regime above 8 frontier entries, at most 2 closest-hit
//                   candidates, keys at most 12 levels below the hand-over -- so the
//                   -2 restart (the ray traced again by its own lane) happens routinely
//   WF_DIAG_COOPSTAT  census of the lone calls' drain finish per trace launch: finishes,
//                   rays finished, waves down to <= 8 rays that could not take it (stack
//                   entries beyond 64, or a ray given back before) -- "[coopstat]" lines
// The measured-and-dropped variants and the knockouts of rounds 1-3 (DESIGN.md
// section 8) live in git history, not here.
#pragma once
#ifndef WF_STATS
#define WF_STATS 0
#endif
#ifndef WF_TIMING
#define WF_TIMING 0
#endif
#ifndef WF_DIAG_GUARD
#define WF_DIAG_GUARD 0
#endif
#ifndef WF_DIAG_BOUNDS
#define WF_DIAG_BOUNDS 0
#endif
#ifndef WF_DIAG_COOP
#define WF_DIAG_COOP 0
#endif
#ifndef WF_DIAG_COOP_SMALL
#define WF_DIAG_COOP_SMALL 0
#endif
#if WF_DIAG_GUARD && !defined(PNRT_DIAG_BUILD)
#error "result-changing diagnostic switches need -DPNRT_DIAG_BUILD (measurement builds only)"
#endif
#if (WF_DIAG_COOP || WF_DIAG_COOP_SMALL) && !defined(PNRT_DIAG_BUILD)
#error "WF_DIAG_COOP builds are diagnostic builds: add -DPNRT_DIAG_BUILD"
#endif
#ifndef WF_DIAG_COOPSTAT
#define WF_DIAG_COOPSTAT 0
#endif
#if WF_DIAG_COOP_SMALL && !WF_DIAG_COOP
#error "WF_DIAG_COOP_SMALL shrinks the product finishes' limits: only with WF_DIAG_COOP"
#endif
#define PNRT_IS_DIAG_BUILD (WF_STATS || WF_TIMING || WF_DIAG_GUARD || WF_DIAG_BOUNDS || WF_DIAG_COOP || \
                            WF_DIAG_COOP_SMALL || WF_DIAG_COOPSTAT)

// Fault words (the context's host-mapped fault area, see pt_wf.h wf_fault)
#define WF_FAULT_GUARD 0     // a bounded wait of the block-level ray queue ran out (diagnostic builds)
#define WF_FAULT_BLOCK 1     // a trace block loaded fewer rays than it dequeued
#define WF_FAULT_DRAIN 2     // a trace launch ended with queue items never dequeued
#define WF_FAULT_BOUNDS 3    // WF_DIAG_BOUNDS: an index outside its array (the word holds its PtSite)
#define WF_FAULT_WORDS 4

// PT_CHECK(fault, index, n, site): the index itself in product builds; in
// WF_DIAG_BOUNDS builds an index outside [0, n) records `site` and reads as 0.
#if WF_DIAG_BOUNDS
PN_DEV long long pt_check_bound(uint32_t* fault, long long idx, long long n, int site) {
    if ((unsigned long long)idx < (unsigned long long)n) return idx;
    if (fault) __hip_atomic_store(fault + WF_FAULT_BOUNDS, (uint32_t)site, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return 0;
}
#define PT_CHECK(fault, idx, n, site) pt_check_bound((fault), (long long)(idx), (long long)(n), (site))
#else
#define PT_CHECK(fault, idx, n, site) (idx)
#endif
// check sites (the number a WF_FAULT_BOUNDS report carries; pnrt_device.hip check_fault names them)
enum PtSite {
    PT_SITE_NODE = 1, PT_SITE_TRI, PT_SITE_LEAF_TABLE, PT_SITE_SPILL, PT_SITE_RESULT, PT_SITE_RAY,
    PT_SITE_HIT_ATTR, PT_SITE_LIGHT_REC, PT_SITE_ENV_QUAD, PT_SITE_TEXEL, PT_SITE_PRIMARY, PT_SITE_COLOR,
    PT_SITE_PATH, PT_SITE_SEGMENT, PT_SITE_COOP
};
