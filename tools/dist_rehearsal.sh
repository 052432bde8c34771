#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: NPROC (default 2) ranks share the GPU,
# gather staged through gloo; the gathered image must equal the 1-rank image.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --config C2"}
timeout -k 10 300 python bench.py $ARGS --save-image gpurun_out/img_n1.npy > gpurun_out/dist_n1.log 2>&1 || exit $?
NP=${NPROC:-2}
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus $NP --backend gloo $ARGS --save-image gpurun_out/img_n2.npy \
    > gpurun_out/dist_n2.log 2>&1 || exit $?
python - <<'PY'
import numpy as np, json
a = np.load("gpurun_out/img_n1.npy"); b = np.load("gpurun_out/img_n2.npy")
print("shape", a.shape, b.shape, "bitwise equal:", bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))))
for f in ("gpurun_out/dist_n1.log", "gpurun_out/dist_n2.log"):
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["n_gpus"], d["value"], d["config"]["parallelism"])
PY
