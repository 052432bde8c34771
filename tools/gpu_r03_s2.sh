#!/bin/bash
# Round-3 session 2: C++ multi-GPU caller test, FETCH_SIZE calibration, path-state
# knockout A/B, the reference dispatch shape (D2/D3, v3 and v1), and the roofline
# reproducibility pair (default bench line + rocprofv3 stats of the --serial run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s2; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);k=d.get('kernels_exclusive') or {};print(d['value'],d['ms_per_step'],' '.join(f'{n}={e[\"ms_per_launch\"]}' for n,e in k.items()))" 2>/dev/null || tail -3 $1; }
step c-abi timeout -k 10 300 python -u -m pytest tests/test_gpu_c_abi.py -x -q -rs --timeout 200 --timeout-method thread > $O/c_abi.log 2>&1
tail -2 $O/c_abi.log
step fetch-calib timeout -k 10 300 python tools/fetch_calib.py $O/fetch_calibration.json > $O/fetch_calib.log 2>&1
cat $O/fetch_calib.log
for rep in 1 2; do
  for v in cur kostate; do
    step ab-$v env PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 150 python bench.py --no-cpu-baseline --no-pmc > $O/ab_$v.log 2>&1
    echo "  $v $(val $O/ab_$v.log)"
  done
done
for c in D2 D3; do
  for k in v3 v1; do
    for sync in "" "--sync-per-frame"; do
      step $c-$k$sync timeout -k 10 200 python bench.py --config $c --kernel $k $sync --steps 240 --warmup 16 --no-cpu-baseline --no-pmc --serial-steps 0 > $O/${c}_${k}${sync}.json 2> $O/${c}_${k}${sync}.err
      echo "  $c $k $sync $(val $O/${c}_${k}${sync}.json)"
    done
  done
done
step bench-C2 timeout -k 10 600 python bench.py > $O/bench_C2.json 2> $O/bench_C2.err
python -c "import json;d=json.loads(open('$O/bench_C2.json').read().strip().splitlines()[-1]);r=d['roofline'];print('C2', d['value'], r['bound'], r['frac'], r['kernel_ms'], r['traffic'])"
step prof-serial timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- \
  python bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-pmc --serial > $O/serial.json 2> $O/serial.err
s=$(ls $O/serial/*kernel_stats.csv $O/serial/*/*kernel_stats.csv 2>/dev/null | head -1); cut -d, -f1-8 $s | head -8
exit 0
