#!/bin/bash
# Widened fuzz campaign on the final round-3 build: random scenes x 3 kernel modes vs the C oracle.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fuzz3; mkdir -p $O
export TMPDIR=/tmp
PNRT_FUZZ_SEEDS=${SEEDS:-40000} timeout -k 10 1100 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
rc=$?; echo "fuzz rc=$rc"; tail -2 $O/fuzz.log; exit $rc
