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
