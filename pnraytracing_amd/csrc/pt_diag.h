// pnraytracing_amd/csrc/pt_diag.h -- the ONE place the diagnostic build switches
// live.  All default to 0, which is the product library; the others exist for
// measurement builds (tools/build_variants.sh -> pnraytracing_amd/variants/)
// and never ship as libpnrt.so:
//   WF_STATS        trace-kernel census: lane steps / rays per launch (tools/census.py)
//   WF_TIMING       per-wave timestamps of the trace kernel (drain-tail analysis)
//   WF_KO_ATTR      knockout: hit attributes without the vertex fetches   -- WRONG IMAGES
//   WF_KO_ENV       knockout: env lookups without math (1) or memory (2)  -- WRONG IMAGES
//   WF_DIAG_NOSTORE knockout: trace results dropped                       -- WRONG IMAGES
//   WF_DIAG_VALU    N extra VALU instructions per traversal step (issue-bound probe)
//   WF_KO_STATE     knockout: the path state the trace does not read (P2-P5: BRDF
//                   value, MIS candidates, Lo, seed) neither stored by the setups nor
//                   loaded by the shade -- register stand-ins; P0 / P1 / P7 (the
//                   rays) and P6 (throughput, meta: control flow) kept -- WRONG IMAGES
//   WF_DIAG_GUARD   N > 0: the trace kernel's block-queue claim gives up after N
//                   iterations instead of 1024, so waves quit with rays unclaimed --
//                   WRONG IMAGES; exercises the fault report (PNRT_E_TRACE)
// The knockouts change results, so they require -DPNRT_DIAG_BUILD as well.
#pragma once
#ifndef WF_STATS
#define WF_STATS 0
#endif
#ifndef WF_TIMING
#define WF_TIMING 0
#endif
#ifndef WF_KO_ATTR
#define WF_KO_ATTR 0
#endif
#ifndef WF_KO_ENV
#define WF_KO_ENV 0
#endif
#ifndef WF_DIAG_NOSTORE
#define WF_DIAG_NOSTORE 0
#endif
#ifndef WF_DIAG_VALU
#define WF_DIAG_VALU 0
#endif
#ifndef WF_KO_STATE
#define WF_KO_STATE 0
#endif
#ifndef WF_DIAG_GUARD
#define WF_DIAG_GUARD 0
#endif
#if (WF_KO_ATTR || WF_KO_ENV || WF_KO_STATE || WF_DIAG_NOSTORE || WF_DIAG_GUARD) && !defined(PNRT_DIAG_BUILD)
#error "result-changing knockout switches need -DPNRT_DIAG_BUILD (measurement builds only)"
#endif
#define PNRT_IS_DIAG_BUILD (WF_STATS || WF_TIMING || WF_KO_ATTR || WF_KO_ENV || WF_KO_STATE || WF_DIAG_NOSTORE || WF_DIAG_VALU || WF_DIAG_GUARD)
