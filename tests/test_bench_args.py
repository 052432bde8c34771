"""bench.py's call shape (CPU): iterations per pnrt_render call by world size,
and the iteration -> call grouping that times exactly K 4-spp iterations."""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bench_mod"] = mod
    spec.loader.exec_module(mod)
    return mod


def test_iters_per_call_defaults():
    b = _bench()
    ns = type("A", (), {"iters_per_call": 0, "steps": 20})()
    # one GPU: a whole batch (BATCH_FRAMES_MAX frames, BATCH_SLOTS paths), no more than the steps
    assert b.iters_per_call(ns, 1920 * 1080) == 20         # 128 frames of 1080p fit: one 80-frame call
    assert b.iters_per_call(ns, 3840 * 2160) == 8          # 4K: 32 frames per batch
    assert b.iters_per_call(ns, 8192 * 4320) == 1          # 7 frames per batch: one iteration
    assert b.iters_per_call(ns, 512 * 512) == 20
    assert b.iters_per_call(ns, 1920 * 1080, batch_slots=1 << 26) == 8    # 2^26 slots: 32 frames
    # a rank's share of an N-way split: the timed steps in as few one-batch calls as fit, split evenly
    for n in (2, 4, 8):
        assert b.iters_per_call(ns, 1920 * (1080 // n), shards=n) == 20   # one call
    assert b.iters_per_call(ns, 1920 * 544, shards=2, batch_slots=1 << 26) == 10   # 64 frames: 2 calls of 10
    ns.steps = 100
    assert b.iters_per_call(ns, 1920 * 1080) == 32         # 32 + 32 + 32 + 4
    assert b.iters_per_call(ns, 1920 * 136, shards=8) == 25     # 4 calls of 100 frames
    assert b.iters_per_call(ns, 3840 * 2160) == 8
    for slots in (1 << 26, b.BATCH_SLOTS):
        for steps in range(1, 90):
            ns.steps = steps
            for rows, n in ((1080, 1), (544, 2), (272, 4), (136, 8)):
                ipc = b.iters_per_call(ns, 1920 * rows, shards=n, batch_slots=slots)
                fit = min(b.BATCH_FRAMES_MAX, slots // (1920 * rows))
                assert 4 * ipc <= fit                                  # every call one batch
                assert -(-steps // ipc) == -(-steps // (fit // 4))     # as few calls as fit
    ns.iters_per_call = 3
    assert b.iters_per_call(ns, 1920 * 1080) == 3 and b.iters_per_call(ns, 3840 * 2160) == 3
    assert b.iters_per_call(ns, 1920 * 136, shards=8) == 3


def test_call_groups_cover_exactly_the_region():
    """The calls of [lo, hi) render exactly its iterations, in order, none longer
    than ipc -- for any warm-up / step count and ipc."""
    b = _bench()
    for ipc in (1, 2, 3, 4):
        for lo, hi in ((0, 3), (3, 23), (1, 6), (5, 5), (0, 1), (2, 20)):
            groups = b.call_groups(lo, hi, ipc)
            its = [k + i for k, n in groups for i in range(n)]
            assert its == list(range(lo, hi)), (ipc, lo, hi, groups)
            assert all(1 <= n <= ipc for _, n in groups)
            assert len(groups) == -(-(hi - lo) // ipc)


def test_launch_count_without_kernel_events():
    """--no-kernel-events: the timed region records no launches; the launch count
    comes from the PNRT_SERIAL steps, or is unknown -- never a division by 0."""
    b = _bench()
    assert b.launches_per_step_of(16, 4, {}, "trace") == 4.0
    assert b.launches_per_step_of(0, 4, {"trace": {"ms_per_launch": 3.0, "launches_per_step": 1.0}}, "trace") == 1.0
    assert b.launches_per_step_of(0, 4, {}, "trace") is None
    # steps < iters_per_call: the timed region's short calls do not count at kernel_ms's call size
    assert b.launches_per_step_of(4, 1, {"trace": {"ms_per_launch": 3.0, "launches_per_step": 1.0}}, "trace") == 1.0


def test_bound_derived_from_counters():
    b = _bench()
    assert b.derive_bound(0.13, 0.95, 0.32) == "l2-latency"     # L1/L2-hit chains
    assert b.derive_bound(0.25, 0.52, 0.30) == "hbm-latency"    # half the L2 lookups miss
    assert b.derive_bound(0.62, 0.90, 0.30) == "hbm"
    assert b.derive_bound(None, 0.5, 0.3) is None
    # C4: the misses are the streamed ray records, the gathers hit
    assert b.derive_bound(0.08, 0.44, 0.3, gather_hit=0.998) == "l2-latency"    # C4 (round 4)
    assert b.derive_bound(0.15, 0.80, 0.4, gather_hit=0.985) == "l2-latency"    # C2
    assert b.derive_bound(0.28, 0.51, 0.36, gather_hit=0.878) == "hbm-latency"  # C5: 12 % of its gathers miss
    g = b.gather_hit_rate(fetch_bytes=1.0e9, streamed_bytes=1.2e9, requested_bytes=9.0e9, rays=25e6)
    assert abs(g - (1 - 0.4e9 / 8.1e9)) < 1e-9


def test_parity_row_sets_interleave():
    """The CPU leg's parity row sets: every PARITY_STEP-th row from offsets 0,
    step/2, step/4, 3 step/4, ...: a permutation of the offsets, so the sets
    partition the frame."""
    b = _bench()
    o = b.parity_offsets()
    assert o[:4] == [0, 18, 9, 27] and sorted(o) == list(range(b.PARITY_STEP))


def test_host_cpus_reports_affinity():
    b = _bench()
    n, facts = b.host_cpus()
    assert n >= 1 and facts["affinity_cpus"] >= n and facts["nproc"] >= facts["affinity_cpus"]


def test_self_launch_exit_codes_and_command():
    """bench.py --gpus N without WORLD_SIZE starts its own N ranks (VERDICT r4 "Next"
    1): the child torch.distributed.run command carries the same arguments, and the
    parent's exit code is the worst rank's (a rank that left no code counts as a
    failure)."""
    b = _bench()
    cmd = b.rank_launch_cmd(8, 29999, ["--gpus", "8", "--steps", "3"])
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=8" in cmd
    assert "127.0.0.1" in cmd and cmd[-4:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "3"][-4:]
    assert b.worst_exit_code({0: 0, 1: 0}, 2, 0) == 0
    assert b.worst_exit_code({0: 3, 1: 0}, 2, 1) == 3          # rank 0's parity failure is the job's code
    assert b.worst_exit_code({0: 0}, 2, 0) == 1                # a rank vanished without a code
    assert b.worst_exit_code({0: 0, 1: 0}, 2, -9) == 1
    assert b.worst_exit_code({}, 2, 137) == 137


def test_gpus_n_with_nccl_and_too_few_gpus_prints_no_line():
    """--gpus 8 --backend nccl with fewer than 8 visible GPUs (here: none) exits
    non-zero before anything runs and prints no JSON line -- never a 1-GPU line
    under --gpus N; and a WORLD_SIZE that disagrees with --gpus is refused."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    # no GPU visible to the child on any host: the refusal path, never a real 8-rank launch
    env.update(HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "{" not in r.stdout and "needs one GPU per rank" in r.stderr, r.stderr[-2000:]
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "{" not in r.stdout and "WORLD_SIZE 1" in r.stderr, r.stderr[-2000:]


def test_step_rooflines():
    """roofline.step (the whole step's fabric bytes over ms_per_step) and the
    per-kernel figures (bytes per launch over the exclusive launch time)."""
    b = _bench()
    pmc = {"trace": {"bytes_per_launch": 3.0e9, "fetch_bytes": 1.4e9, "write_bytes": 0.2e9, "launches_per_step": 1.0,
                     "l2_hit_rate": 0.8},
           "shade": {"bytes_per_launch": 8.0e9, "fetch_bytes": 3.8e9, "write_bytes": 0.4e9, "launches_per_step": 1.0}}
    excl = {"trace": {"ms_per_launch": 2.5}, "shade": {"ms_per_launch": 2.0}}
    step, per = b.step_rooflines(pmc, excl, 5.0)
    assert step["bytes_per_step"] == 11e9 and abs(step["achieved"] - 2200.0) < 1e-6
    assert abs(step["frac"] - 0.275) < 1e-9
    assert abs(per["shade"]["frac"] - 0.5) < 1e-9 and per["shade"]["frac_bounds"][0] == round(4.2e9 / 2e-3 / 1e9 / 8000, 4)
    assert per["trace"]["l2_hit_rate"] == 0.8 and per["shade"]["l2_hit_rate"] is None
    assert b.step_rooflines(None, excl, 5.0) == (None, None)


def test_pmc_child_runs_the_timed_call_size():
    """at N > 1 rank 0's PMC child renders its share in calls of the size
    the timed run issues (driver's 20 steps: one 80-frame call at every N), passed explicitly, with
    2 calls timed after 1 of warm-up -- so bytes per launch and launches per step
    are those of the timed launches."""
    b = _bench()
    for n, ipc in ((1, 20), (2, 20), (4, 20), (8, 20)):
        a = b.parse(["--gpus", str(n), "--steps", "20"])
        cmd = b.pmc_child_cmd(a, n, "rocprofv3", ("FETCH_SIZE",), "/tmp/x")
        i = cmd.index("--child")
        child = cmd[i:]
        assert child[child.index("--iters-per-call") + 1] == str(ipc), (n, child)
        assert child[child.index("--steps") + 1] == str(2 * ipc) and child[child.index("--warmup") + 1] == str(ipc)
        assert child[child.index("--shard-world") + 1] == str(n)
        # the timed run's own call size for rank 0's share (ShardedFrame.max_rows x W)
        from pnraytracing_amd.tracer import shard_rows
        rows = max(len(shard_rows(1080, b.BAND, n, r)) for r in range(n))
        assert b.iters_per_call(a, rows * 1920, shards=n) == ipc
    assert b.pmc_iters_per_call(b.parse(["--config", "C5"]), 1) == 8      # 32 4K frames a batch
    assert b.pmc_iters_per_call(b.parse(["--config", "D2"]), 1) == 1
    assert b.pmc_iters_per_call(b.parse(["--iters-per-call", "3"]), 4) == 3


def test_issue_stats_and_valu_bound():
    """The third PMC pass's issue figures (VERDICT r5 "Next" 2): round 5's recorded
    trace counters (profiles/r05/s23/pmc_valu.txt) give VALU issue 0.65, and the
    bound reads valu-issue at >= 0.6, the latency classes below it."""
    b = _bench()
    st = b.issue_stats({"GRBM_GUI_ACTIVE": 3.154e7, "SQ_INSTS_VALU": 1.312e9, "SQ_WAVES": 8192.0,
                        "SQ_INSTS_SALU": 5.684e8, "SQ_WAVE_CYCLES": 7.744e9, "SQ_WAIT_ANY": 3.752e9})
    assert abs(st["valu_util"] - 0.65) < 0.005 and abs(st["valu_per_wave"] - 160156.25) < 1e-6
    assert abs(st["wait_frac"] - 0.4845) < 1e-3 and "ta_busy" not in st
    assert b.derive_bound(0.15, 0.8, 0.4, 0.98, 0.65) == "valu-issue"
    assert b.derive_bound(0.15, 0.8, 0.4, 0.98, 0.5) == "l2-latency"
    assert b.derive_bound(0.6, 0.8, 0.4, 0.98, 0.7) == "hbm"
    assert b.derive_bound(0.27, 0.5, 0.4, 0.87, None) == "hbm-latency"


def test_batch_frames_match_the_library():
    """bench.BATCH_FRAMES_MAX / BATCH_SLOTS (the call plan's one-batch limits) are the
    library's WF_MAX_CHUNK_FRAMES / 2^WF_SLOT_BITS: a plan computed against a larger
    limit would split a call into two batches (profiles/r06/h/summary.txt)."""
    import re
    b = _bench()
    src = open(os.path.join(REPO, "pnraytracing_amd", "csrc", "pnrt_device.hip")).read()
    m = re.search(r"#define WF_MAX_CHUNK_FRAMES (\d+)", src)
    assert m and int(m.group(1)) == b.BATCH_FRAMES_MAX
    wf = open(os.path.join(REPO, "pnraytracing_amd", "csrc", "pt_wf.h")).read()
    m = re.search(r"#define WF_SLOT_BITS (\d+)", wf)
    assert m and 1 << int(m.group(1)) == b.BATCH_SLOTS
