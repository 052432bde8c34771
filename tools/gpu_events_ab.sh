#!/bin/bash
# bench (torch stream / the library's own stream) vs the bare render loop, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/e.log 2>&1 || exit 1; echo "torch stream: $(grep -o '"value": [0-9.]*' gpurun_out/e.log)"
  PNRT_BENCH_OWN_STREAM=1 timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/e.log 2>&1 || exit 1; echo "own stream: $(grep -o '"value": [0-9.]*' gpurun_out/e.log)"
  timeout -k 10 100 python tools/shard_sim_one.py 1 20 > gpurun_out/e.log 2>&1 || exit 1; echo "bare: $(tail -1 gpurun_out/e.log | cut -c1-60)"
done
