#!/bin/bash
# GPU session: parity tests, then A/B bench of kernel variants (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log; { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
for v in ${VARIANTS:-"--kernel v2" "--kernel v1"}; do
  timeout -k 10 240 python bench.py --no-cpu-baseline $v > gpurun_out/ab.log 2>&1
  rc=$?; echo "bench [$v] rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/ab.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
