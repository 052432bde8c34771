#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench (pipelined) and of the
# PNRT_SERIAL bench (exclusive launches), + per-class timelines.
#   OUT=gpurun_out/prof_x bash tools/gpu_prof.sh [extra bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/prof}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pipe -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --serial-steps 0 "$@" > $O/pipe.json 2> $O/pipe.err
rc=$?; echo "pipelined rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- \
  python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pmc --serial-steps 0 --serial "$@" > $O/serial.json 2> $O/serial.err
rc=$?; echo "serial rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(ls $O/pipe/*kernel_trace.csv $O/pipe/*/*kernel_trace.csv 2>/dev/null | head -1)
python tools/timeline2.py $f 24 | tee $O/timeline.txt
for m in pipe serial; do
  s=$(ls $O/$m/*kernel_stats.csv $O/$m/*/*kernel_stats.csv 2>/dev/null | head -1); echo "== $m"; cut -d, -f1-6 $s | head -8
  python -c "import json;d=json.load(open('$O/$m.json'));print('$m', d['value'], d['ms_per_step'], d['kernels'])"
done
