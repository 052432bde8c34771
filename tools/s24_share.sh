cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05s24; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_moot.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2; do
  for spec in "8 16" "4 16" "2 8" "1 4" "8 4" "4 4" "2 4"; do
    set -- $spec
    timeout -k 10 120 python tools/share_bench.py $1 $2 20 5 >> $O/share.txt 2>> $O/share.err || exit 1
  done
done
cat $O/share.txt
