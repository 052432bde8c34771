cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=$PWD/pnraytracing_amd/variants
for q in 4 8; do for p in p3 p5 p7; do
  GPU_MAX_HW_QUEUES=$q PNRT_DEVICE_LIB=$V/libpnrt_$p.so timeout -k 10 100 python tools/shard_sim_one.py 8 30 > gpurun_out/hwq.log 2>&1 || exit 1
  echo "q=$q $p N=8: $(tail -1 gpurun_out/hwq.log)"
  GPU_MAX_HW_QUEUES=$q PNRT_DEVICE_LIB=$V/libpnrt_$p.so timeout -k 10 100 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/hwq.log 2>&1 || exit 1
  echo "q=$q $p C2: $(grep -o '"value": [0-9.]*' gpurun_out/hwq.log)"
done; done
