#!/usr/bin/env python3
"""bench.py -- Msamples/s of the MI355X path tracer on the BASELINE workload.

Workload (BASELINE.json metric / configs[1]; SURVEY 8d "C2"): Cornell box +
~70k-triangle bunny stand-in + vignaioli_night_1k HDR environment,
1920x1080, one step = one 4-spp iteration (frames 4k..4k+3 blended in order),
MAX_BOUNCE_DEPTH 4.  Synthetic scene data (procedural mesh stand-ins; the
reference's OBJ assets do not exist), the reference's real 1k HDR.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

N > 1: one process per GPU; the image rows are dealt in 8-row bands
(rank r owns bands b with b % N == r), each rank renders its rows, and the
accumulated rows are gathered to rank 0 over RCCL every step (strong
scaling: the frame is fixed, its rows are split).  `bench.py --gpus N` run
directly (no WORLD_SIZE in the environment) launches its own N ranks: the
parent never touches the GPU, starts `torch.distributed.run --nproc-per-node N`
as a child process, relays rank 0's line and exits with the worst rank's exit
code; with --backend nccl and fewer than N visible GPUs it exits non-zero
before anything runs (never a 1-GPU line under --gpus N).  Rank 0 runs the live
PMC passes over its own share of the rows before it initialises the GPU, so
an N > 1 line carries live traffic too.

Prints ONE JSON line (rank 0).  Roofline of the dominant kernel (pt_wf_trace),
every figure measured by this run:
  traffic   fabric bytes per trace launch from two rocprofv3 --pmc passes that
            this script runs as child processes BEFORE it touches the GPU
            (N = 1): FETCH_SIZE (the node / triangle gathers, tallied exactly) +
            the streamed ray records / 2 (tallied at half; ray count from the
            census of these sources) + WRITE_SIZE -- calibrated on known bytes,
            profiles/r03/fetch_calibration.json; traffic_bounds = [1x, 2x]
            FETCH_SIZE + WRITE_SIZE;
  kernel_ms the trace launch's EXCLUSIVE duration: HIP events around every
            trace launch during extra steps rendered with PNRT_SERIAL (one call
            in flight, full-occupancy grid), after the timed region;
  achieved  traffic / kernel_ms, against the 8 TB/s HBM peak (frac).
The kernel's own request stream (device-layout fetches from the census of a
WF_STATS build, profiles/census.json, used only when its source hash matches
the loaded library) is reported beside it against the L2 bandwidth, and the
SURVEY 8d reference-literal byte count as reference_bytes (never divided by a
peak).  The timed steps themselves run the default pipelined renderer.

After the timed region the CPU leg (rank 0) has the oracle render row sets of
the timed image itself -- every 36th row over all its frames -- and reports
"parity" (pixels differing, bit for bit; the run exits non-zero on any) and,
at N = 1, the oracle's rate as cpu_baseline.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import platform
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BAND = 8
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md: L2 (8 XCDs) ~34.5 TB/s
# FETCH_SIZE (KiB) -> fabric read bytes, calibrated on known byte counts over a 1 GiB table
# (tools/microtests/fetch_calib.hip, tools/fetch_calib.py -> profiles/r03/fetch_calibration.json):
# wide coalesced streaming reads (16 B per lane) are tallied at HALF their bytes (known /
# FETCH_SIZE = 2.00, 128 B per TCC_EA0_RDREQ; MI355X_MICROARCH.md says the same), scattered
# 64-B record gathers EXACTLY (0.994, 64 B per request; one 64-B half of each 128-B line:
# 0.993).  The trace kernel mixes both: its ray records (origin + direction, 32 B per ray,
# read once, streamed) and its node / triangle gathers (64-B requests).  So its fabric read
# bytes = FETCH_SIZE + the streamed ray bytes / 2 (they were tallied at half), the ray count
# from the census of these sources; the other kernels (path-state streams + gathers) are
# reported at 2 x FETCH_SIZE, an upper bound.
STREAM_FACTOR, GATHER_FACTOR = 2.0, 1.0
CALIBRATION = "profiles/r03/fetch_calibration.json"
# rocprofv3 --pmc passes (one run each; TCC block: FETCH_SIZE uses 3 counters, WRITE_SIZE 2; the third
# pass: 6 SQ, 1 GRBM and 1 TA counter, within the 8 / 2 / 2 a pass may hold)
PMC_PASSES = [("FETCH_SIZE",), ("WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"),
              ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES",
               "GRBM_GUI_ACTIVE", "TA_BUSY_avr")]
# VALU issue: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles (MI355X_MICROARCH.md); 1024
# SIMDs; GRBM_GUI_ACTIVE is reported summed over the 8 XCDs (per-XCD busy cycles = value / 8)
N_SIMD, N_XCD, VALU_CYC = 1024, 8, 2.0
VALU_BOUND = 0.6       # derive_bound: "valu-issue" when the kernel issues VALU on >= this share of SIMD cycles
KSHORT = {"pt_wf_trace": "trace", "pt_wf_gen_setup": "gen", "pt_wf_shade_setup": "shade",
          "pt_primary_kernel": "primary", "pt_primary_wf": "primary", "pt_blend_kernel": "blend", "pt_render_kernel": "v1"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5", "D2", "D3"],
                    help="C2-C5: BASELINE configs; D2 / D3: the C2 / C3 scene at the reference's own dispatch "
                         "shape -- 512x512 (PnRT.hpp:41-42), 1 spp per frame, one pnrt_render per frame "
                         "(main.cpp:569-615): a step is one frame")
    ap.add_argument("--sync-per-frame", action="store_true",
                    help="D configs: synchronise after every call (an interactive loop that displays each frame)")
    ap.add_argument("--sync-with", default="torch", choices=["torch", "pnrt"],
                    help="--sync-per-frame: wait with torch.cuda.synchronize() (device-wide) or pnrt_synchronize "
                         "(the library's own streams: what a C caller of the drop-in calls)")
    ap.add_argument("--mode", default="zcull", choices=["exact", "zcull"])
    ap.add_argument("--kernel", default="v3", choices=["v1", "v3"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU leg: the oracle renders parity row sets of the timed image for ~this long")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU leg's baseline timing (the parity check still renders one row set)")
    ap.add_argument("--no-parity", action="store_true", help="skip the CPU leg entirely (no parity check)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 PMC passes")
    ap.add_argument("--pmc-timeout", type=int, default=240, help="seconds per PMC pass (killed after)")
    ap.add_argument("--serial-steps", type=int, default=2,
                    help="extra PNRT_SERIAL steps after the timed region for exclusive kernel times (0: skip)")
    ap.add_argument("--serial", action="store_true",
                    help="time the steps themselves with PNRT_SERIAL (one call in flight): for the rocprofv3 "
                         "--stats run whose trace-kernel average is the roofline's exclusive kernel_ms")
    ap.add_argument("--save-image", default="")
    ap.add_argument("--spp", type=int, default=0, help="experiment: samples per step other than the config's 4")
    ap.add_argument("--iters-per-call", type=int, default=0,
                    help="4-spp iterations per pnrt_render call and per gather of the accumulated rows "
                         "(the primary pass and each launch's drain amortised over them; the image is the "
                         "same); steps stay 4-spp iterations, the last call of the warm-up / the timed "
                         "region takes what is left.  Default: 4 (16 frames) where they fit one batch, "
                         "else 2 (a whole 4K frame); DESIGN.md section 6")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="experiment: no HIP events around launches in the timed region")
    ap.add_argument("--kernel-times", action="store_true",
                    help="time every kernel class with HIP events in the timed region (default: only the dominant kernel)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL over xGMI; gloo = host-staged rehearsal)")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)   # a PMC pass's workload: no output
    ap.add_argument("--shard-world", type=int, default=1, help=argparse.SUPPRESS)   # child: rank 0's share of N
    return ap.parse_args(argv)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ---- host facts ------------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


# ---- live PMC (child processes, before this process initialises the GPU) --------------------
def _read_counters(d):
    """{kernel class: {counter: average per dispatch}, "_dispatches": {class: n}}"""
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
            if k not in KSHORT:
                continue
            key = (KSHORT[k], r["Dispatch_Id"])
            per.setdefault(key, {})
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    acc, nd = {}, {}
    for (k, _), cs in per.items():
        nd[k] = nd.get(k, 0) + 1
        for c, v in cs.items():
            acc.setdefault(k, {}).setdefault(c, []).append(v)
    out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    out["_dispatches"] = nd
    return out


def pmc_child_cmd(args, shard_world: int, exe: str, group, d: str) -> list:
    """One PMC pass: rocprofv3 over `bench.py --child` rendering rank 0's share of a
    shard_world-way split in calls of the timed calls' size (pmc_iters_per_call),
    2 calls timed after 1 of warm-up."""
    ipc = pmc_iters_per_call(args, shard_world)
    cmd = ["timeout", "-s", "KILL", str(args.pmc_timeout), exe, "--kernel-trace", "--pmc", *group,
           "-d", d, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--child", "--config", args.config, "--mode", args.mode,
           "--kernel", args.kernel, "--steps", str(2 * ipc), "--warmup", str(ipc)]
    if args.spp:
        cmd += ["--spp", str(args.spp)]
    return cmd + ["--iters-per-call", str(ipc), "--shard-world", str(shard_world)]


def live_pmc(args, shard_world: int = 1):
    """Two rocprofv3 --kernel-trace --pmc passes over a short run of this same
    workload (child processes: this process has not touched the GPU yet) -- at
    N > 1 over rank 0's share of an N-way split (shard_world), rendered alone.
    Returns {class: {"bytes_per_launch", "launches_per_step", "l2_hit_rate"}}
    or None when rocprofv3 is absent or a pass fails."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        log("rocprofv3 not found: no live PMC")
        return None
    tmp = tempfile.mkdtemp(prefix="pnrt_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", RC_DIR_ENV):
        env.pop(v, None)
    # whole calls of the TIMED calls' size, so every profiled launch covers the
    # iterations a timed launch covers: the share's call size computed here exactly
    # as the child (and the timed run) will compute it, and passed explicitly
    ipc = pmc_iters_per_call(args, shard_world)
    steps, warm = 2 * ipc, ipc
    counters = {}
    try:
        for i, group in enumerate(PMC_PASSES):
            d = os.path.join(tmp, f"p{i}")
            cmd = pmc_child_cmd(args, shard_world, exe, group, d)
            log(f"PMC pass {i + 1}/{len(PMC_PASSES)}: {' '.join(group)}")
            t = time.perf_counter()
            with open(os.path.join(tmp, f"p{i}.log"), "w") as lf:
                r = subprocess.run(cmd, stdout=lf, stderr=subprocess.STDOUT, env=env)
            if r.returncode != 0:
                log(f"PMC pass {i + 1} failed (rc {r.returncode}); see {tmp}/p{i}.log")
                return None
            log(f"PMC pass {i + 1} done in {time.perf_counter() - t:.1f}s")
            got = _read_counters(d)
            nd = got.pop("_dispatches")
            for k, cs in got.items():
                counters.setdefault(k, {}).update(cs)
                counters[k]["_n"] = nd.get(k, 0)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    res = {}
    for k, cs in counters.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        e = {"bytes_per_launch": (STREAM_FACTOR * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024.0,
             "fetch_bytes": cs["FETCH_SIZE"] * 1024.0, "write_bytes": cs["WRITE_SIZE"] * 1024.0,
             "launches_per_step": cs["_n"] / (steps + warm)}
        if "TCC_HIT_sum" in cs:
            e["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"], 1.0)
        e.update(issue_stats(cs))
        res[k] = e
    return res or None


def issue_stats(cs):
    """Issue-side figures of one kernel class from the third PMC pass (averages per
    dispatch): valu_util = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
    -- the share of SIMD cycles issuing VALU --; ta_busy = TA_BUSY_avr / (GRBM_GUI_ACTIVE /
    8), the texture-address units' busy share; VALU / SALU per wave; wait_frac =
    SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)."""
    out = {}
    g = cs.get("GRBM_GUI_ACTIVE")
    if not g:
        return out
    cyc = g / N_XCD
    if "SQ_INSTS_VALU" in cs:
        out["valu_util"] = cs["SQ_INSTS_VALU"] * VALU_CYC / (N_SIMD * cyc)
    if "TA_BUSY_avr" in cs:
        out["ta_busy"] = cs["TA_BUSY_avr"] / cyc
    w = cs.get("SQ_WAVES")
    if w:
        if "SQ_INSTS_VALU" in cs:
            out["valu_per_wave"] = cs["SQ_INSTS_VALU"] / w
        if "SQ_INSTS_SALU" in cs:
            out["salu_per_wave"] = cs["SQ_INSTS_SALU"] / w
    if cs.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in cs:
        out["wait_frac"] = cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"]
    return out


CONFIG_DIMS = {"C2": (1920, 1080), "C3": (1920, 1080), "C4": (1920, 1080), "C5": (3840, 2160),
               "D2": (512, 512), "D3": (512, 512)}


def pmc_iters_per_call(args, shard_world: int) -> int:
    """The iterations per call the PMC child (and the timed run) will use: as given;
    1 for the D configs (one frame per call); else iters_per_call() of the largest
    share of a shard_world-way split of the config's rows (ShardedFrame.max_rows)."""
    if args.iters_per_call > 0:
        return args.iters_per_call
    if args.config.startswith("D"):
        return 1
    from pnraytracing_amd.tracer import shard_rows      # (numpy only: loads no library)
    W, H = CONFIG_DIMS[args.config]
    rows = max(len(shard_rows(H, BAND, shard_world, r)) for r in range(shard_world))
    return iters_per_call(args, rows * W, shards=shard_world)


def stored_keyed(path, key, src_hash):
    """An entry of a profiles/*.json file, only if recorded for these sources."""
    path = os.path.join(REPO, "profiles", path)
    if not os.path.exists(path):
        return None
    e = json.load(open(path)).get(key)
    if not e or e.get("source_hash") != src_hash:
        return None
    return e


# ---- CPU baseline ------------------------------------------------------------------------------
def host_cpus():
    """(usable, facts): the CPUs this process may run on -- its affinity mask,
    capped by a cgroup v2 CPU quota when one is set (the GPU box gives a job a
    share of a larger host: nproc shows every CPU of the machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    return usable, {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota}


PARITY_STEP = 36     # the parity check's row sets: every 36th row, offsets interleaved


def parity_offsets(step: int = PARITY_STEP):
    """Row offsets of the successive parity row sets: 0, step/2, step/4, 3 step/4, ...
    (each set is every step-th row; the sets interleave, so any prefix of them
    spreads over the whole frame)."""
    out, k = [0], 1
    while k < step:
        out += [o for o in ((2 * j + 1) * step // (2 * k) for j in range(k)) if o not in out]
        k *= 2
    return out + [o for o in range(step) if o not in out]


def cpu_leg(cfg, gpu_image, frames: int, target_s: float):
    """The CPU leg: the oracle (oracle/pn_oracle.c, the C restatement of
    ray_tracing.comp, OpenMP over rows, every CPU the process may use) renders row
    sets of the TIMED image -- every PARITY_STEP-th row, frames 0 .. frames-1 in
    order, exactly what the GPU accumulated over the warm-up and the timed steps --
    until ~target_s (at least one set).  Its rate is the CPU baseline (a bounded
    sample of the same workload), and its rows are compared bit for bit with the
    GPU's image: the parity of the measured run itself (ray_tracing.comp:975-991).
    Returns (parity dict, cpu dict, counters)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    threads, cpu_facts = host_cpus()
    o = pyoracle.Oracle(cfg)
    H, W = cfg.height, cfg.width
    ref = np.zeros((H, W, 4), np.float32)
    tot, rows = None, []
    t = time.perf_counter()
    for off in parity_offsets():
        if off >= H:
            continue
        _, st = o.render(0, frames, rows=(off, H), y_step=PARITY_STEP, accum=ref, threads=threads)
        tot = st if tot is None else {k: tot[k] + st[k] for k in st}
        rows += list(range(off, H, PARITY_STEP))
        if time.perf_counter() - t >= target_s:
            break
    dt = time.perf_counter() - t
    rows = np.array(sorted(rows))
    g, r = gpu_image[rows].view(np.uint32), ref[rows].view(np.uint32)
    bad = np.argwhere(np.any(g != r, axis=-1))
    parity = {"rows": int(len(rows)), "row_step": PARITY_STEP, "pixels": int(len(rows) * W), "frames": frames,
              "differing": int(len(bad)), "tolerance": "0 ulp (bit-exact)",
              "oracle": "oracle/pn_oracle.c on the same scene arrays",
              "first_differing": ([int(rows[bad[0][0]]), int(bad[0][1])] if len(bad) else None)}
    n = tot["samples"]
    cpu = {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": f"{cfg.name}: {len(rows)} rows (every {PARITY_STEP}th, interleaved sets) x {W} px x {frames} frames "
                     f"= {n} samples in {dt:.1f}s -- the parity rows of the timed image; oracle/pn_oracle.c "
                     f"OpenMP {threads} threads",
           "cpu_model": cpu_model(), **cpu_facts}
    return parity, cpu, tot


def cpu_baseline_c1(cpu: dict):
    """C1 (the reference's CPU-runnable config, BASELINE configs[0]) at full size
    on the same threads, added to the CPU leg's record."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    from pnraytracing_amd import scenes
    threads = cpu["cores"]
    # C1: Cornell box, 256x256, 1 spp per frame, depth 4 (BASELINE configs[0]); frames until ~1 s
    c1 = scenes.cornell_c1()
    o1 = pyoracle.Oracle(c1)
    a1 = np.zeros((c1.height, c1.width, 4), np.float32)
    f1, t1 = 0, time.perf_counter()
    while f1 < 64 and (f1 < 4 or time.perf_counter() - t1 < 1.0):
        o1.render(f1, 1, accum=a1, threads=threads)
        f1 += 1
    d1 = time.perf_counter() - t1
    cpu["c1"] = {"value": round(f1 * c1.width * c1.height / d1 / 1e6, 4), "unit": "Msamples/s",
                 "sample": f"C1 256x256 x {f1} frames (1 spp each, depth 4) in {d1:.2f}s"}


BATCH_FRAMES_MAX = 128     # pnrt_device.hip WF_MAX_CHUNK_FRAMES: frames per batch at most
BATCH_SLOTS = 1 << 28      # pt_wf.h WF_SLOT_BITS: path slots per batch at most


def iters_per_call(args, paths_per_frame: int, batch_slots: int = BATCH_SLOTS, shards: int = 1) -> int:
    """4-spp iterations per pnrt_render call: as given, else
    * one GPU (shards == 1): calls of one whole batch -- as many frames as one
      batch holds (at most BATCH_FRAMES_MAX frames and BATCH_SLOTS path slots: 128
      frames of a 1080p frame, 32 of a 4K frame) but no more than the steps, the last
      call cut at the region's end (the driver's 20 steps of C2: one 80-frame call);
    * a rank of an N-way split (shards > 1): the timed steps in as few one-batch
      calls as fit, split evenly (20 steps: one call at every N).
    Multi-rank runs pass the LARGEST share (ShardedFrame.max_rows), so every rank
    issues the same calls and therefore the same gathers (batch_slots: a test
    override).  A batch's trace launches' drains and its gen / blend launches are
    fixed costs, so the larger the batch the smaller their share.  Measured
    (profiles/r06/h/, profiles/r06/j/, profiles/r06/k/): one GPU, bench.py C2, same box:
    16-frame calls (the plan since round 2) 1 887-1 893 Msamples/s, 32-frame calls
    (a whole batch of 2^26 slots) 1 921-1 928; with 2^28-slot batches one 80-frame
    call 1 915-1 926 against 1 893-1 897 for 32-frame calls (another box), C3 +1.1
    to +2 %, C5 8 frames -> 32 +2.2 %.  Rank 0's share through bench.py's gather path
    (tools/share_bench.py --collective): N = 8 16-iteration calls (64-frame batches)
    1 710-1 771 per rank, one 20-iteration call in one 80-frame batch 1 781-1 815;
    N = 4 1 811-1 871 -> 1 882-1 891; N = 2 two calls of 10 1 890-1 897 against
    16 + 4 1 860-1 868 (even split; on one GPU 8 + 8 + 4 beat 7 + 7 + 6)."""
    if args.iters_per_call > 0:
        return args.iters_per_call
    ppf = max(1, paths_per_frame)
    most = max(1, min(BATCH_FRAMES_MAX, batch_slots // ppf) // 4)
    steps = max(1, getattr(args, "steps", most))
    if shards > 1:
        ncalls = -(-steps // most)
        return -(-steps // ncalls)
    return min(most, steps)


def call_groups(lo: int, hi: int, ipc: int):
    """(first iteration, iterations) of each call covering iterations [lo, hi)
    exactly: groups of ipc, the last one cut at hi."""
    return [(k, min(ipc, hi - k)) for k in range(lo, hi, max(1, ipc))]


def sizing_calls(warmup: int, steps: int, ipc: int):
    """Iterations of the untimed calls issued before the warm-up: one per distinct call
    size of the warm-up and timed plans, the timed calls' size first.  A call size
    selects how many buffer sets ("pipes") calls of that size rotate over (by paths per
    batch), and the first call of a size sizes all of them -- so neither a shorter
    warm-up call (5 iterations beside the 20-iteration timed call of an N = 8 share)
    nor the cut last call of a plan allocates inside the warm-up or the timed region."""
    sizes = {m for _, m in call_groups(0, warmup, ipc) + call_groups(warmup, warmup + steps, ipc)}
    return [ipc] + sorted(sizes - {ipc}, reverse=True)


def issue_calls(sf, spp: int, lo: int, hi: int, ipc: int, world: int) -> int:
    """The pnrt_render calls of iterations [lo, hi): one per group of ipc
    iterations (the last group cut at hi); multi-GPU ranks start one gather of
    their rows after each (overlapped with the next call).  Returns the gathers
    issued -- a collective, so every rank must issue the same number."""
    n = 0
    for k, m in call_groups(lo, hi, ipc):
        sf.render(spp * k, spp * m)
        if world > 1:
            sf.gather_async()
            n += 1
    return n


def same_on_all_ranks(values, device) -> None:
    """Raise unless every rank holds the same integers (one all_reduce of
    (v, -v) with MAX): the call plan of a multi-rank run, checked before any
    gather is issued -- ranks issuing different numbers of gathers would hang."""
    import torch
    import torch.distributed as dist
    v = torch.tensor([int(x) for x in values] + [-int(x) for x in values], dtype=torch.int64, device=device)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    k = len(values)
    if v[:k].tolist() != [int(x) for x in values] or (-v[k:]).tolist() != [int(x) for x in values]:
        raise SystemExit(f"rank {dist.get_rank()}: call plan {list(values)} differs across ranks "
                         f"(max {v[:k].tolist()}, min {(-v[k:]).tolist()})")


def launches_per_step_of(k_launches: int, steps: int, excl: dict, kname: str):
    """Dominant-kernel launches per step, counted at the call size kernel_ms was
    measured on: from the PNRT_SERIAL steps (whole calls of iters_per_call
    iterations, as kernel_ms), else from the timed region's events, else unknown
    (None).  (A timed region shorter than one call -- steps < iters_per_call --
    issues shorter calls, whose launches are not the serial steps' launches.)"""
    if kname in excl and excl[kname].get("launches_per_step"):
        return excl[kname]["launches_per_step"]
    if k_launches:
        return k_launches / steps
    return None


L2_HIT_CYC, MISS_CYC = 200.0, 900.0   # MI355X_MICROARCH.md: global_load L2-hit / HBM-miss latency (cycles)


def derive_bound(hbm_frac, l2_hit, l2_frac, gather_hit=None, valu_util=None):
    """The roof that binds, from the counters: "hbm" (bandwidth) when the kernel's
    fabric traffic reaches half the HBM peak; "valu-issue" when, below that, the
    kernel issues VALU on at least VALU_BOUND of its SIMD cycles (valu_util, the
    third PMC pass: the trace step's branch-free VALU, VERDICT r5 "Next" 2); below
    both the kernel is bound by
    the latency of its dependent fetch chains -- "hbm-latency" when at least a
    third of that latency is spent on L2 misses (a miss costs ~900 cycles, a hit
    ~200: a gather miss rate above ~10 %, C5's 4.2M-triangle scene beyond the
    L2s), "l2-latency" otherwise (C2-C4: L1/L2-hit chains).
    The gathers' own hit rate (gather_hit: the streamed ray records, read once,
    miss by nature and are taken out) decides when known, else the kernel's whole
    L2 hit rate.  l2_frac (its own requests against the L2 bandwidth) is
    reported beside it."""
    if hbm_frac is None:
        return None
    if hbm_frac >= 0.5:
        return "hbm"
    if valu_util is not None and valu_util >= VALU_BOUND:
        return "valu-issue"
    hit = gather_hit if gather_hit is not None else l2_hit
    if hit is None:
        return "l2-latency"
    miss = (1.0 - hit) * MISS_CYC
    return "hbm-latency" if miss >= (miss + hit * L2_HIT_CYC) / 3.0 else "l2-latency"


def gather_hit_rate(fetch_bytes, streamed_bytes, requested_bytes, rays):
    """L2 hit rate of the trace kernel's node / triangle gathers alone, in bytes:
    1 - (fabric read bytes of the gathers) / (bytes the gathers requested).  The
    gathers' fabric bytes are FETCH_SIZE less the streamed ray records' share
    (tallied at half, CALIBRATION); their requests are the census's request
    stream less the ray records (32 B + the 4-B path entry per ray)."""
    req = requested_bytes - 36.0 * rays
    if req <= 0:
        return None
    return max(0.0, min(1.0, 1.0 - (fetch_bytes - streamed_bytes / 2.0) / req))


# ---- self-launch of N ranks (bench.py --gpus N without a launcher) ------------------------------
RC_DIR_ENV = "PNRT_BENCH_RC_DIR"     # the self-launch's directory of per-rank exit codes


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_launch_cmd(n: int, port: int, argv) -> list:
    """torch.distributed.run over this script with the same arguments (one rank per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def worst_exit_code(codes: dict, n: int, launcher_rc: int) -> int:
    """The worst (largest) exit code over the N ranks; a rank that left no code
    (killed, crashed before recording) counts as the launcher's code, at least 1."""
    worst = max(codes.values()) if codes else 0
    if len(codes) < n or (launcher_rc != 0 and worst == 0):
        worst = max(worst, launcher_rc if launcher_rc > 0 else 1)
    return worst


def launch_ranks(args, argv) -> int:
    """--gpus N > 1 and no WORLD_SIZE: start N ranks of this script as a CHILD
    torch.distributed.run (never an exec: a process that has touched the GPU must
    not replace itself, and this one never touches it -- device_count() does not
    initialise HIP on this image).  Rank 0's JSON line reaches stdout through the
    inherited descriptor; the return value is the worst rank's exit code."""
    import torch
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} with --backend nccl needs one GPU per rank, but {ndev} GPU(s) are "
              f"visible; no line is printed (a 1-GPU line under --gpus {args.gpus} would be wrong).  Use "
              f"--backend gloo to rehearse {args.gpus} ranks on fewer GPUs.", file=sys.stderr, flush=True)
        return 2
    if ndev == 0:
        print("bench.py: no GPU visible", file=sys.stderr, flush=True)
        return 2
    rc_dir = tempfile.mkdtemp(prefix="pnrt_bench_rc_", dir=os.environ.get("TMPDIR", "/tmp"))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env[RC_DIR_ENV] = rc_dir
    cmd = rank_launch_cmd(args.gpus, free_port(), argv)
    log(f"launching {args.gpus} ranks ({args.backend}): {' '.join(cmd[1:6])} ...")
    try:
        r = subprocess.run(cmd, env=env)
        codes = {}
        for f in os.listdir(rc_dir):
            if f.startswith("rc."):
                try:
                    codes[int(f[3:])] = int(open(os.path.join(rc_dir, f)).read().strip())
                except ValueError:
                    pass
    finally:
        shutil.rmtree(rc_dir, ignore_errors=True)
    rc = worst_exit_code(codes, args.gpus, r.returncode)
    if rc:
        log(f"rank exit codes {dict(sorted(codes.items()))}, launcher {r.returncode}: exit {rc}")
    return rc


def record_exit_code(rc: int) -> None:
    """A self-launched rank records its exit code for the parent (launch_ranks).  A
    PMC pass's child (--child) never does: its rank-0 slot belongs to rank 0."""
    if "--child" in sys.argv[1:]:
        return
    d = os.environ.get(RC_DIR_ENV)
    if d and os.path.isdir(d):
        with open(os.path.join(d, f"rc.{os.environ.get('RANK', '0')}"), "w") as f:
            f.write(str(int(rc)))


def step_rooflines(pmc, excl, ms_per_step):
    """The whole step against the HBM roof (VERDICT r4 "Next" 5): the fabric bytes
    of every kernel of a step (PMC, 2 x FETCH_SIZE + WRITE_SIZE per launch -- exact
    for the streamed path state, an upper bound for gathers) over the step's
    wall time; and per kernel class (gen, shade, blend, trace) its bytes per launch
    over its EXCLUSIVE launch time (PNRT_SERIAL steps), with the [1x, 2x]
    FETCH_SIZE bounds as frac_bounds.  (The dominant kernel's calibrated figure
    is roofline.frac.)  Returns (step, {class: ...}) or (None, None)."""
    if not pmc:
        return None, None
    tot = sum(e["bytes_per_launch"] * e["launches_per_step"] for e in pmc.values())
    step = {"bytes_per_step": round(tot), "ms_per_step": round(ms_per_step, 4),
            "achieved": round(tot / (ms_per_step * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(tot / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "counting": f"sum over the step's launches of {STREAM_FACTOR:g} x FETCH_SIZE + WRITE_SIZE "
                        f"(live PMC) / the timed ms_per_step (pipelined calls overlap: whole-step rate)"}
    per = {}
    for k, e in pmc.items():
        ms = (excl.get(k) or {}).get("ms_per_launch")
        if not ms:
            continue
        lo = GATHER_FACTOR * e["fetch_bytes"] + e["write_bytes"]
        hi = e["bytes_per_launch"]
        per[k] = {"traffic": round(hi), "kernel_ms": ms, "achieved": round(hi / (ms * 1e-3) / 1e9, 2),
                  "frac": round(hi / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                  "frac_bounds": [round(lo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                  round(hi / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)],
                  "launches_per_step": round(e["launches_per_step"], 3),
                  "l2_hit_rate": round(e["l2_hit_rate"], 4) if "l2_hit_rate" in e else None,
                  "valu_util": round(e["valu_util"], 4) if "valu_util" in e else None,
                  "ta_busy": round(e["ta_busy"], 4) if "ta_busy" in e else None}
    return step, (per or None)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None and not args.child:
        sys.exit(launch_ranks(args, argv))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not args.child:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: the line would not measure "
                         f"--gpus {args.gpus} ranks")
    # live PMC first, while this process has not initialised the GPU (the passes are
    # child processes under rocprofv3); at N > 1 rank 0 profiles its own share before
    # it joins the process group (the other ranks wait there)
    pmc = None
    if rank == 0 and not args.child and not args.no_pmc:
        pmc = live_pmc(args, shard_world=world)
    if world > 1:
        # multi-rank: RCCL adds a stream of its own beside the library's four (own +
        # three workers); 8 hardware queues keep it off theirs (set before HIP starts)
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:          # rehearsal of N ranks on fewer GPUs (gloo only)
        if args.backend == "nccl":
            raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPU(s): RCCL needs one GPU per rank")
        local = local % ndev
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from pnraytracing_amd import build, host, scenes
    from pnraytracing_amd.dist import ShardedFrame
    from pnraytracing_amd.tracer import KERNEL_V1, SERIAL, TRAVERSE_EXACT, TRAVERSE_ZCULL, PathTracer

    builders = {"C2": scenes.bunny_c2, "C3": scenes.marry_c3, "C4": scenes.teapot_c4, "C5": scenes.synthetic_c5}
    t = time.perf_counter()
    dispatch_shape = args.config.startswith("D")
    if dispatch_shape:                  # the reference's interactive shape: 512x512, one 1-spp frame per call
        cfg = builders["C" + args.config[1:]](width=512, height=512, spp=1)
        cfg.name = args.config + cfg.name[2:] + "@512"
        args.iters_per_call = 1
    else:
        cfg = builders[args.config]()
    scene_s = time.perf_counter() - t
    if args.spp:
        cfg.spp = args.spp
    W, H, spp = cfg.width, cfg.height, cfg.spp

    pt = PathTracer(local)
    # torch works on the library's own stream (created with the context, before its
    # worker streams): a further stream of torch's own would share one of the
    # process's 4 hardware queues with a busy stream (measured -4 %)
    stream = torch.cuda.ExternalStream(pt.stream_handle())
    torch.cuda.set_stream(stream)
    pt.set_stream(stream.cuda_stream)
    opts = (TRAVERSE_ZCULL if args.mode == "zcull" else TRAVERSE_EXACT) | {"v1": KERNEL_V1, "v3": 0}[args.kernel]
    if args.serial:
        opts |= SERIAL
    t = time.perf_counter()
    pt.load(cfg, opts)
    upload_s = time.perf_counter() - t
    info = pt.device_info()
    version = pt.version()

    sf = ShardedFrame(pt, band=BAND, device=torch.device("cuda", local),   # pnraytracing_amd/dist.py
                      shard=(args.shard_world, 0) if (args.child and args.shard_world > 1) else None)
    image = None

    # every rank plans its calls from the LARGEST share, so all issue the same gathers
    ipc = iters_per_call(args, sf.max_rows * W, shards=world)
    if world > 1:
        same_on_all_ranks([ipc, len(call_groups(0, args.warmup, ipc)),
                           len(call_groups(args.warmup, args.warmup + args.steps, ipc))],
                          "cuda" if args.backend == "nccl" else "cpu")

    def calls(lo, hi):
        if args.sync_per_frame:             # every frame completed before the next is submitted
            n = 0
            wait = pt.synchronize if args.sync_with == "pnrt" else torch.cuda.synchronize
            for k in range(lo, hi):
                n += issue_calls(sf, spp, k, k + 1, ipc, world)
                wait()
            return n
        return issue_calls(sf, spp, lo, hi, ipc, world)

    # the library sizes every buffer set at the first call of a size: one untimed call
    # of the timed calls' size first (then the accumulation is reset: the image is the
    # warm-up's and timed steps' frames as before), so that no later call -- a shorter
    # warm-up call included -- reallocates inside the warm-up or the timed region
    if not args.child:                         # (a PMC pass's warm-up is whole calls: it sizes them,
        for m in sizing_calls(args.warmup, args.steps, ipc):   # and its launch counts stay those of its steps)
            sf.render(0, spp * m)
        torch.cuda.synchronize()
        pt.reset_accum()
    calls(0, args.warmup)
    if world > 1:
        sf.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if args.child:                             # a PMC pass: the profiler sees the launches; done
        calls(args.warmup, args.warmup + args.steps)
        torch.cuda.synchronize()
        pt.close()
        return
    # live per-kernel timing: the library brackets every launch with HIP events
    # recorded on the stream it launches on (pnrt_profile_enable); only the dominant
    # kernel is bracketed unless --kernel-times (every event record is a queue packet
    # between launches of the overlapped calls)
    kname = {"v1": "v1", "v3": "trace"}[args.kernel]
    pt.profile_select(None if args.kernel_times else [kname])
    pt.profile_enable(not args.no_kernel_events)
    t0 = time.perf_counter()
    calls(args.warmup, args.warmup + args.steps)
    if world > 1:
        image = sf.finish()                    # every gather completes inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = pt.profile_read()
    pt.profile_enable(False)
    k_ms_total, k_launches = prof.get(kname, (0.0, 0))
    kern_ms_pipe = k_ms_total / k_launches if k_launches else None   # average launch duration, pipelined

    # the timed image itself (frames 0 .. (warmup + steps) * spp - 1), for the parity
    # check of the CPU leg below; read before the PNRT_SERIAL steps add frames to it
    timed_image = None
    if rank == 0 and (args.save_image or not args.no_parity):
        timed_image = image.cpu().numpy() if world > 1 else pt.read_accum()
    if args.save_image and rank == 0:
        np.save(args.save_image, timed_image)

    # exclusive kernel times: PNRT_SERIAL steps (one call in flight, full trace grid)
    excl = {}
    if args.serial_steps > 0:
        pt.set_options(opts | SERIAL)
        pt.profile_select(None)
        pt.profile_enable(True)
        for k in range(args.serial_steps):          # calls of the same size as the timed ones
            sf.render(spp * (args.warmup + args.steps + k * ipc), spp * ipc)
        torch.cuda.synchronize()
        ser = pt.profile_read()
        pt.profile_enable(False)
        pt.set_options(opts)
        excl = {k: {"ms_per_launch": round(ms / n, 4), "launches_per_step": n / (args.serial_steps * ipc)}
                for k, (ms, n) in ser.items() if n}
    kern_ms = excl[kname]["ms_per_launch"] if kname in excl else None
    launches_per_step = launches_per_step_of(k_launches, args.steps, excl, kname)
    if world > 1:
        t = torch.tensor([elapsed, kern_ms_pipe or 0.0, kern_ms or 0.0], dtype=torch.float64,
                         device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_pipe, kern_ms = float(t[0]), (float(t[1]) or None), (float(t[2]) or None)

    samples = W * H * spp * args.steps
    value = samples / elapsed / 1e6
    parity = None
    if rank == 0:
        # one-shot setup, reported beside the step rate: host scene build
        # (ModelOutput + BuildBVH + packing), the BuildBVH part alone on the host and on
        # the GPU (pnrt_bvh_build, incl. PCIe; same arrays), and the upload (pnrt_*)
        setup = {"scene_build_s": round(scene_s, 3), "bvh_build_host_s": round(cfg.packed.bvh_seconds, 4),
                 "upload_s": round(upload_s, 3)}
        if cfg.packed.tri_bounds is not None:
            tb = cfg.packed.tri_bounds
            pt.build_bvh(tb[: min(len(tb), 4096)])                    # module / allocation warm-up
            t = time.perf_counter()
            nodes, _, _ = pt.build_bvh(tb)
            setup["bvh_build_gpu_s"] = round(time.perf_counter() - t, 4)
            setup["bvh_gpu_identical"] = bool(np.array_equal(nodes.view(np.uint32), cfg.packed.nodes.view(np.uint32)))

        cpu = counts = None
        if not args.no_parity:
            # the CPU leg (rank 0): oracle rows of the timed image -- its parity, and at
            # N = 1 the CPU baseline; N > 1 checks one row set (the gathered image)
            timing = world == 1 and not args.no_cpu_baseline
            parity, cpu, counts = cpu_leg(cfg, timed_image, (args.warmup + args.steps) * spp,
                                          args.cpu_seconds if timing else 0.0)
            if timing:
                cpu_baseline_c1(cpu)
            else:
                cpu = None
            log(f"parity: {parity['differing']} of {parity['pixels']} pixels differ "
                f"({parity['rows']} rows x {parity['frames']} frames vs the oracle)")
        rows0 = sf.my_rows
        samples_per_step = rows0 * W * spp
        src_hash = build.device_source_hash()
        ref_bytes = None
        if counts and launches_per_step:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import pyoracle
            per = (pyoracle.bounce_traversal_bytes(counts) if args.kernel == "v3"
                   else pyoracle.algorithmic_bytes(counts)) / counts["samples"]
            ref_bytes = round(per * samples_per_step / launches_per_step)

        traffic = l2hit = ghit = None
        issue = {}
        traffic_src = None
        step_traffic = None
        census = stored_keyed("census.json", cfg.name, src_hash) if args.kernel == "v3" else None
        census_scale = (rows0 / census.get("rows", H) * spp * ipc / census.get("frames", 4)) if census else None
        traffic_bounds = None
        if pmc and kname in pmc:
            e = pmc[kname]
            l2hit = e.get("l2_hit_rate")
            issue = {k: round(e[k], 4) for k in ("valu_util", "ta_busy", "valu_per_wave", "salu_per_wave", "wait_frac")
                     if k in e}
            traffic_bounds = [round(GATHER_FACTOR * e["fetch_bytes"] + e["write_bytes"]),
                              round(STREAM_FACTOR * e["fetch_bytes"] + e["write_bytes"])]
            if census and args.kernel == "v3":
                # the launch's streamed ray records: 32 B per ray (census rays, scaled to the launch)
                rays = sum(b["rays"] for b in census["per_bounce"]) / census["trace_launches"] * census_scale
                streamed = min(32.0 * rays, e["fetch_bytes"] * STREAM_FACTOR)
                traffic = e["fetch_bytes"] * GATHER_FACTOR + streamed / 2.0 + e["write_bytes"]
                ghit = gather_hit_rate(e["fetch_bytes"], streamed, census["requested_bytes_per_launch"] * census_scale,
                                       rays)
                traffic_src = (f"live rocprofv3 --pmc: FETCH_SIZE + streamed ray bytes / 2 + WRITE_SIZE -- 64-B gathers "
                               f"tallied exactly, streamed reads at half ({CALIBRATION}); {rays / 1e6:.1f}M rays x 32 B "
                               f"per launch from profiles/census.json")
            else:
                traffic = traffic_bounds[0]
                traffic_src = (f"live rocprofv3 --pmc: FETCH_SIZE + WRITE_SIZE, every read tallied as a 64-B gather "
                               f"(lower bound; no census for these sources; {CALIBRATION})")
            step_traffic = {k: {"bytes_per_launch": round(e["bytes_per_launch"]),
                                "launches_per_step": round(e["launches_per_step"], 3),
                                "l2_hit_rate": round(e["l2_hit_rate"], 4) if "l2_hit_rate" in e else None}
                            for k, e in pmc.items()}
            step_traffic["counting"] = (f"{STREAM_FACTOR:g} x FETCH_SIZE + WRITE_SIZE per launch: exact for the "
                                        f"streamed path state, an upper bound for gathers ({CALIBRATION})")
            step_traffic["total_bytes_per_step"] = round(sum(e["bytes_per_launch"] * e["launches_per_step"]
                                                             for e in pmc.values()))
        else:
            # no live PMC (--no-pmc, rocprofv3 absent or a pass failed): the N = 1 live
            # figure recorded for these sources (tools/record_pmc.py), scaled to this
            # rank's launch -- its share of the rows and its frames per launch
            e = stored_keyed("pmc.json", f"{cfg.name}/{kname}", src_hash)
            if e and e.get("bytes_per_launch"):
                scale = rows0 / e["rows"] * (spp * ipc) / e["frames_per_launch"]
                traffic, l2hit = e["bytes_per_launch"] * scale, e.get("l2_hit_rate")
                traffic_src = (f"derived: N = 1 live PMC recorded for these sources (profiles/pmc.json, "
                               f"{e['bytes_per_launch']:.4g} B per {e['frames_per_launch']}-frame launch of "
                               f"{e['rows']} rows) x this rank's share ({rows0} rows, {spp * ipc} frames)")
        achieved = traffic / (kern_ms * 1e-3) / 1e9 if (traffic and kern_ms) else None
        requested = None
        if census and kern_ms:
            rb = census["requested_bytes_per_launch"] * census_scale      # the census traced 4-frame calls
            requested = {"bytes_per_launch": round(rb), "achieved": round(rb / (kern_ms * 1e-3) / 1e9, 1),
                         "peak": L2_PEAK_GBS, "unit": "GB/s",
                         "frac_of_l2": round(rb / (kern_ms * 1e-3) / 1e9 / L2_PEAK_GBS, 4),
                         "source": "profiles/census.json (WF_STATS build of these sources)"}
        checks = None
        if kern_ms and launches_per_step:
            checks = {"launches_x_kernel_ms": round(launches_per_step * kern_ms, 4),
                      "le_ms_per_step": launches_per_step * kern_ms <= elapsed / args.steps * 1e3,
                      "frac_le_1": (achieved / HBM_PEAK_GBS <= 1.0) if achieved else None}
        kernels = {k: {"ms_per_launch": round(ms / n, 4), "launches_per_step": n / args.steps}
                   for k, (ms, n) in prof.items() if n}
        step_roof, kernel_roofs = step_rooflines(pmc, excl, elapsed / args.steps * 1e3)
        kfull = {"v1": "pt_render_kernel", "v3": "pt_wf_trace"}[args.kernel]
        line = {
            "metric": "Msamples/sec (whole node) at 1920x1080, 4spp/iter; fraction of HBM roofline",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural stand-in meshes (reference OBJs absent), reference HDR/texture assets",
            "config": {"workload": f"{cfg.name}: {cfg.description}"
                                   + (" -- reference dispatch shape, one pnrt_render per frame"
                                      + (f", synchronised per frame ({args.sync_with})" if args.sync_per_frame else "")
                                      if dispatch_shape else ""), "width": W, "height": H,
                       "spp_per_step": spp, "max_bounce_depth": cfg.max_depth, "triangles": cfg.n_triangles,
                       "iters_per_call": ipc,
                       "traverse": args.mode, "kernel_version": args.kernel, "parallelism": f"row-bands{BAND}x{world}",
                       "kernel": kfull, "calls": "serial" if args.serial else "pipelined",
                       "primary": ("reused across calls (camera fixed): each pipe keeps its primary records while "
                                   "camera / frame / shard / mode / scene are unchanged, so the timed steps trace "
                                   "no primary pass (exact: no camera jitter, ray_tracing.comp:980; DESIGN.md "
                                   "section 15)"),
                       "moot_rays": ("shadow rays, and the last bounce's continuation rays, whose outcome is proven "
                                     "per ray not to change the path's radiance bits (monotone rounding bound on the "
                                     "MIS / emission term) are not traced; every timed image is checked against the "
                                     "oracle, which traces them all (DESIGN.md section 16)")},
            "roofline": {"bound": derive_bound(achieved / HBM_PEAK_GBS if achieved else None, l2hit,
                                               requested["frac_of_l2"] if requested else None, ghit,
                                               issue.get("valu_util")),
                         "bound_rule": "derived from the counters (bench.derive_bound): hbm (bandwidth) if frac >= 0.5; "
                                       f"else valu-issue if valu_util >= {VALU_BOUND} (SQ_INSTS_VALU x 2 cycles over the "
                                       "SIMDs' GRBM_GUI_ACTIVE cycles, live third PMC pass); else the latency of "
                                       "dependent fetch chains -- hbm-latency if L2 misses of the "
                                       "node / triangle gathers (gather_l2_hit_rate; l2_hit_rate when unknown) take "
                                       ">= 1/3 of the fetch latency (miss ~900, hit ~200 cycles), l2-latency otherwise; "
                                       "peak / frac stay against HBM",
                         "valu_util": issue.get("valu_util"), "ta_busy": issue.get("ta_busy"),
                         "issue": issue or None,
                         "achieved": round(achieved, 2) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src,
                         "traffic_bounds": traffic_bounds,
                         "l2_hit_rate": round(l2hit, 4) if l2hit is not None else None,
                         "gather_l2_hit_rate": round(ghit, 4) if ghit is not None else None,
                         "kernel": kfull, "kernel_ms": kern_ms, "kernel_ms_timing": "exclusive (PNRT_SERIAL steps)",
                         "kernel_ms_pipelined": round(kern_ms_pipe, 4) if kern_ms_pipe else None,
                         "launches_per_step": launches_per_step,
                         "checks": checks,
                         "requested": requested,
                         "reference_bytes_per_launch": ref_bytes,
                         "reference_bytes_note": ("SURVEY 8d's reference-literal count (no z-cull, no reuse, every record "
                                                  "access counted): a workload size, never divided by a peak -- over "
                                                  "kernel_ms it exceeds the HBM peak on the L2-resident scenes (C2: "
                                                  "~3x), since the tree and triangles are served from L2 (gather L2 "
                                                  "hit ~0.98); frac above is the counter-measured fabric traffic"),
                         "step": step_roof,
                         "kernels": kernel_roofs},
            "kernels": kernels,
            "kernels_exclusive": excl or None,
            "fabric_traffic": step_traffic,
            "setup": setup,
            "parity": parity,
            "cpu_baseline": cpu,
            "device": {"bvh_interior_nodes": info["n_interior"], "max_depth": info["max_depth"],
                       "scene_bytes": info["device_bytes"], "library": version},
        }
        print(json.dumps(line), flush=True)
    failed = bool(parity and parity["differing"])
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    pt.close()
    if failed:
        log("PARITY FAILURE: the timed image differs from the oracle")
        sys.exit(3)


if __name__ == "__main__":
    _rc = 1
    try:
        main()
        _rc = 0
    except SystemExit as _e:
        _rc = _e.code if isinstance(_e.code, int) else (0 if _e.code is None else 1)
        raise
    finally:
        record_exit_code(_rc)
