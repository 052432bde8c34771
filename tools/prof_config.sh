# rocprofv3 kernel trace of one config's bench run (serialised calls), per-kernel per-bounce durations
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pc}; mkdir -p $O
for c in ${CONFIGS:-C4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$c -o run --output-format csv -- \
    python bench.py --config $c --steps 8 --warmup 4 --no-cpu-baseline --no-pmc --no-parity --serial > $O/prof_$c.json 2> $O/prof_$c.err || exit 1
done
exit 0
