#!/bin/bash
# One GPU-box session (rounds 4-5), steps chosen by STEPS (space-separated, in order):
#   smoke    __graft_entry__.smoke()
#   tests    the whole -m gpu suite (TESTS= to narrow it, e.g. TESTS="tests/test_gpu_parity.py")
#   bench    bench.py C2 default (live PMC, CPU leg with the parity check)   [CONFIGS= for others]
#   d2       the reference's dispatch shape D2 / D3, pipelined and synchronised per frame (no HIP events;
#            + a synchronised run with every kernel timed)
#   ab       A/B of prebuilt variants (VARIANTS="name ...", ROUNDS=n): C2 (+ AB_CONFIGS) per variant
#   prof     rocprofv3 --kernel-trace --stats of bench.py --serial and of the default command
#   census   trace census of these sources -> profiles/census.json (needs the stats variant)
#   record   profiles/pmc.json from this session's N = 1 bench lines
#   shard    the multi-GPU share simulation (per-rank rates at N = 1/2/4/8 on one GPU)
#   tail     WF_TIMING drain census of the lone-frame (D2) trace launches
#   coopv    the cooperative-finish tests, verbose (hand-over / restart counts)
#   abd      A/B of prebuilt variants on D2 / D3 synchronised per frame, no HIP events (VARIANTS, ROUNDS)
#   dloop    D2 / D3 through the compiled C caller alone (tools/dloop.py), synchronised and pipelined
#   profd    rocprofv3 kernel trace of D2 / D3 synchronised per frame; tools/frame_gaps.py splits each frame
#   fuzz     the widened fuzz campaign (SEEDS=40000 random scenes x 3 kernel modes vs the oracle)
# Output under gpurun_out/$TAG.  Every GPU step has its own time limit; the first failing
# step ends the session (no retries).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-s}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
summ() {
  python3 - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    try:
        d = [json.loads(x) for x in open(f) if x.startswith("{")][-1]
    except Exception as e:
        print(" ", f, "no line", e); continue
    r = d.get("roofline") or {}
    p = d.get("parity") or {}
    print(" ", f.split("/")[-1], d["value"], "ms/step", d["ms_per_step"], "trace", r.get("kernel_ms"), "frac", r.get("frac"),
          r.get("bound"), "parity", p.get("differing"), "/", p.get("pixels"),
          "prim", (d.get("kernels") or {}).get("primary"))
PY
}
for s in ${STEPS:-smoke tests bench}; do
  case $s in
    smoke) step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    tests)
      step gpu-tests timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -rs --timeout 300 \
        --timeout-method thread > $O/gpu_tests.log 2>&1
      tail -3 $O/gpu_tests.log ;;
    census)    # trace census of these sources (profiles/census.json, read by bench.py): needs
               # variants/libpnrt_stats.so built from them (tools/build_variants.sh stats:"-DWF_PIPES=1 -DWF_STATS=1")
      step census timeout -k 10 600 python tools/census.py ${CONFIGS:-C2 C3 C4 C5} > $O/census.log 2>&1
      cp profiles/census.json $O/census.json ;;
    record)    # profiles/pmc.json from the N = 1 bench lines of this session (read by N > 1 lines)
      step record timeout -k 10 60 python tools/record_pmc.py $O/bench_C*.json
      cp profiles/pmc.json $O/pmc.json ;;
    tail)      # WF_TIMING drain census of the lone-frame trace launches (needs variants/libpnrt_timing.so)
      for c in ${DCONFIGS:-D2}; do
        step tail-$c env PNRT_DEVICE_LIB=pnraytracing_amd/variants/libpnrt_timing.so timeout -k 10 200 python bench.py \
          --config $c --sync-per-frame --steps 8 --warmup 4 --no-parity --no-pmc --serial-steps 0 > $O/tail_$c.json \
          2> $O/tail_$c.err
      done ;;
    shard)     # the multi-GPU share simulation: rank 0's rows of an N-way split on one GPU (16-frame calls)
      step shard env GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/shard_sim.py 30 ${SHARD_FPC:-auto} > $O/shard_sim.txt 2>&1
      cat $O/shard_sim.txt ;;
    fuzz)
      step fuzz env PNRT_FUZZ_SEEDS=${SEEDS:-40000} PNRT_FUZZ_FIRST=${FIRST:-0} timeout -k 10 1100 python -u -m pytest tests/test_gpu_fuzz.py -x -q \
        --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
      tail -2 $O/fuzz.log ;;
    bench)
      for c in ${CONFIGS:-C2}; do
        extra=""; [ $c = C5 ] && extra="--steps 10"; [ $c != C2 ] && extra="$extra --cpu-seconds 6"
        step bench-$c timeout -k 10 600 python bench.py --config $c $extra ${BENCH_ARGS:-} > $O/bench_$c.json 2> $O/bench_$c.err
        summ $O/bench_$c.json
      done ;;
    d2)        # the headline lines without HIP events (an event pair around each of a frame's 10
               # launches costs ~12 % of a synchronised 512x512 frame); + one with every kernel timed
      for c in ${DCONFIGS:-D2 D3}; do
        for sync in "" "--sync-per-frame"; do
          step $c$sync timeout -k 10 200 python bench.py --config $c $sync --steps 240 --warmup 16 --no-cpu-baseline \
            --no-pmc --serial-steps 0 --no-kernel-events > $O/${c}${sync}.json 2> $O/${c}${sync}.err
          summ $O/${c}${sync}.json
        done
        step $c-kt timeout -k 10 200 python bench.py --config $c --sync-per-frame --steps 240 --warmup 16 --no-cpu-baseline \
          --no-pmc --serial-steps 0 --kernel-times > $O/${c}--sync-per-frame-kernel-times.json 2> $O/${c}-kt.err
        summ $O/${c}--sync-per-frame-kernel-times.json
      done ;;
    coopv)     # the cooperative-finish tests verbose: the hand-over / restart counts of the diagnostic libraries
      step coop-tests timeout -k 10 900 python -u -m pytest tests/test_gpu_coop.py -m gpu -x -v -s --timeout 400 \
        --timeout-method thread > $O/coop_tests.log 2>&1
      grep -E "rays handed over|passed|failed" $O/coop_tests.log | tail -8 ;;
    abd)       # A/B of the reference's dispatch shape (D2 / D3: 512x512, one 1-spp frame per call), synchronised
               # per frame, no HIP events; VARIANTS as for ab
      for r in $(seq 1 ${ROUNDS:-2}); do
        for v in ${VARIANTS}; do
          lib=""; [ $v != base ] && lib=pnraytracing_amd/variants/libpnrt_$v.so
          for c in ${AB_DCONFIGS:-D2 D3}; do
            step abd-$v-$c-$r env PNRT_DEVICE_LIB=$lib timeout -k 10 200 python bench.py --config $c --sync-per-frame \
              --steps 240 --warmup 16 --no-parity --no-pmc --no-cpu-baseline --serial-steps 0 --no-kernel-events \
              ${ABD_ARGS:-} > $O/abd_${v}_${c}_$r.json 2> $O/abd_${v}_${c}_$r.err
            summ $O/abd_${v}_${c}_$r.json
          done
        done
      done ;;
    ab)
      for r in $(seq 1 ${ROUNDS:-2}); do
        for v in ${VARIANTS}; do
          lib=""; [ $v != base ] && lib=pnraytracing_amd/variants/libpnrt_$v.so
          for c in C2 ${AB_CONFIGS:-}; do
            step ab-$v-$c-$r env PNRT_DEVICE_LIB=$lib timeout -k 10 300 python bench.py --config $c --no-pmc \
              --no-parity --serial-steps 0 ${AB_ARGS:-} > $O/ab_${v}_${c}_$r.json 2> $O/ab_${v}_${c}_$r.err
            summ $O/ab_${v}_${c}_$r.json
          done
          for c in ${AB_DCONFIGS:-}; do
            step ab-$v-$c-$r env PNRT_DEVICE_LIB=$lib timeout -k 10 200 python bench.py --config $c --sync-per-frame \
              --steps 240 --warmup 16 --no-parity --no-pmc --serial-steps 0 --kernel-times > $O/ab_${v}_${c}_$r.json \
              2> $O/ab_${v}_${c}_$r.err
            summ $O/ab_${v}_${c}_$r.json
          done
        done
      done ;;
    prof)
      step prof-serial timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run --output-format csv -- \
        python bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-pmc --serial > $O/prof_serial.json 2> $O/prof_serial.err
      step prof-pipe timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pipe -o run --output-format csv -- \
        python bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-pmc > $O/prof_pipe.json 2> $O/prof_pipe.err
      for m in serial pipe; do     # rocprof's trace-kernel average vs the line's kernel_ms (CPU only)
        python3 tools/prof_summary.py $O/prof_$m/run_kernel_trace.csv $O/prof_$m.json $O/prof_${m}_check.json > /dev/null \
          && python3 -c "import json; print('  prof-$m', json.load(open('$O/prof_${m}_check.json'))['check'])"
      done ;;
    profd)     # rocprofv3 kernel trace of the reference's dispatch shape, synchronised per frame, no events
      for c in ${DCONFIGS:-D2 D3}; do
        step profd-$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profd_$c -o run --output-format csv -- \
          python bench.py --config $c --sync-per-frame --steps 120 --warmup 16 --no-parity --no-pmc --no-cpu-baseline \
          --serial-steps 0 --no-kernel-events > $O/profd_$c.json 2> $O/profd_$c.err
        python3 tools/frame_gaps.py $O/profd_$c/run_kernel_trace.csv | tail -12
      done ;;
    dloop)     # the reference's loop through the C ABI alone (no Python): D2 / D3, synchronised and pipelined
      step dloop timeout -k 10 300 python tools/dloop.py ${DCONFIGS:-D2 D3} > $O/dloop.json 2> $O/dloop.err
      cat $O/dloop.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
