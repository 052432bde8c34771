"""bench.py's multi-rank path on one GPU: 2 ranks (torch.distributed.run)
render their 8-row bands and gather them (gloo, host-staged); the gathered
image must equal the single-rank image bit for bit.  (On an 8-GPU node the
same code gathers over RCCL; see DESIGN.md "Multi-GPU".)"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_gather_equals_one(tmp_path):
    args = ["--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--config", "C4"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    a, b = str(tmp_path / "n1.npy"), str(tmp_path / "n2.npy")
    subprocess.run([sys.executable, "bench.py", *args, "--save-image", a], cwd=REPO, env=env, check=True,
                   timeout=400, stdout=subprocess.DEVNULL)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", "29541", "bench.py", "--gpus", "2",
                    "--backend", "gloo", *args, "--save-image", b], cwd=REPO, env=env, check=True, timeout=600,
                   stdout=subprocess.DEVNULL)
    x, y = np.load(a), np.load(b)
    assert x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_eight_gloo_ranks_gather_equals_one(tmp_path):
    """bench.py's N = 8 plan (8-way row bands, padding of the short shares,
    same_on_all_ranks, 8 hardware queues and four calls in flight per rank)
    rehearsed with 8 gloo ranks on the box's one GPU: the gathered C2 image
    equals the N = 1 image bit for bit, and each run's own parity check (the
    CPU leg's oracle rows of its timed image) passes (VERDICT r3 "Next" 8)."""
    args = ["--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-pmc", "--serial-steps", "1", "--config", "C2"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    a, b = str(tmp_path / "n1.npy"), str(tmp_path / "n8.npy")
    subprocess.run([sys.executable, "bench.py", *args, "--save-image", a], cwd=REPO, env=env, check=True,
                   timeout=400, stdout=subprocess.DEVNULL)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29547", "bench.py", "--gpus", "8",
                        "--backend", "gloo", *args, "--save-image", b], cwd=REPO, env=env, timeout=600,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    import json
    d = json.loads(line)
    assert d["n_gpus"] == 8 and d["parity"]["differing"] == 0 and d["config"]["parallelism"] == "row-bands8x8"
    x, y = np.load(a), np.load(b)
    assert x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_bench_self_launch_gloo_two_ranks(tmp_path):
    """`python3 bench.py --gpus 2 --backend gloo ...` with NO launcher around it
    (the driver's command shape) starts its own two ranks (VERDICT r4 "Next" 1):
    the line says n_gpus 2, carries live PMC traffic (rank 0's share, profiled
    before it joined the group), its own parity check passes, and the gathered
    image equals the N = 1 image bit for bit."""
    base = ["--steps", "1", "--warmup", "1", "--config", "C2", "--serial-steps", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    a, b = str(tmp_path / "n1.npy"), str(tmp_path / "n2.npy")
    subprocess.run([sys.executable, "bench.py", *base, "--no-pmc", "--no-cpu-baseline", "--save-image", a], cwd=REPO,
                   env=env, check=True, timeout=400, stdout=subprocess.DEVNULL)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", *base, "--save-image", b],
                       cwd=REPO, env=env, timeout=700, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    import json
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "row-bands8x2"
    assert d["parity"]["differing"] == 0 and d["parity"]["pixels"] > 0
    assert d["roofline"]["traffic"] and d["roofline"]["traffic_source"].startswith("live"), d["roofline"]
    x, y = np.load(a), np.load(b)
    assert x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_bench_gpus8_nccl_refused_on_one_gpu():
    """--gpus 8 over RCCL on this one-GPU box: a non-zero exit and no line, before
    any rank starts."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "1", "--warmup", "1"], cwd=REPO, env=env,
                       timeout=120, capture_output=True, text=True)
    assert r.returncode != 0 and not [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert "needs one GPU per rank" in r.stderr


def _single_rank_c4(path):
    from pnraytracing_amd import scenes
    from pnraytracing_amd.tracer import PathTracer
    cfg = scenes.teapot_c4(320, 176)
    with PathTracer(0) as pt:
        pt.load(cfg)
        for k in range(3):
            pt.render(4 * k, 4)
        return pt.read_accum()


def _run_worker(tmp_path, nproc, port):
    out = str(tmp_path / f"rccl{nproc}.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "tests/rccl_worker.py", out],
                       cwd=REPO, env=env, timeout=300, capture_output=True, text=True)
    return r, out


def test_rccl_gather_one_rank(tmp_path):
    """The RCCL gather path of ShardedFrame (dist.gather on device tensors, async,
    double-buffered) executed with one rank: image = the plain render."""
    r, out = _run_worker(tmp_path, 1, 29551)
    assert r.returncode == 0, r.stderr[-3000:]
    x, y = _single_rank_c4(None), np.load(out)
    assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_rccl_gather_two_ranks_one_gpu(tmp_path):
    """Two RCCL ranks on the box's one GPU, when RCCL accepts that (it may refuse a
    duplicate device): the gathered bands = the single-rank image."""
    r, out = _run_worker(tmp_path, 2, 29553)
    if r.returncode != 0:
        msg = r.stderr[-3000:]
        if "uplicate GPU" in msg or "invalid usage" in msg.lower():
            why = [ln for ln in msg.splitlines() if "uplicate GPU" in ln or "invalid usage" in ln.lower()]
            pytest.skip("RCCL refuses two ranks on one GPU: " + (why[0].strip()[:200] if why else "duplicate device"))
        raise AssertionError(msg)
    x, y = _single_rank_c4(None), np.load(out)
    assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_bench_iters_per_call_same_image(tmp_path):
    """bench.py --iters-per-call 2 renders two 4-spp iterations per pnrt_render
    call (and per gather): the accumulated image equals one call per iteration."""
    args = ["--steps", "2", "--warmup", "2", "--no-cpu-baseline", "--no-pmc", "--serial-steps", "0", "--config", "C4"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    a, b = str(tmp_path / "ipc1.npy"), str(tmp_path / "ipc2.npy")
    for out, ipc in ((a, "1"), (b, "2")):
        subprocess.run([sys.executable, "bench.py", *args, "--iters-per-call", ipc, "--save-image", out], cwd=REPO,
                       env=env, check=True, timeout=400, stdout=subprocess.DEVNULL)
    x, y = np.load(a), np.load(b)
    assert x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
