# D2 / D3 synchronised per frame with every kernel bracketed by HIP events
# (--kernel-times), only the trace kernel (default) and none (--no-kernel-events)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-ev}; mkdir -p $O
for r in 1 2; do
  for c in D2 D3; do
    for m in kt def none; do
      a=""; [ $m = kt ] && a="--kernel-times"; [ $m = none ] && a="--no-kernel-events"
      timeout -k 10 200 python bench.py --config $c --sync-per-frame --steps 240 --warmup 16 --no-cpu-baseline --no-pmc \
        --serial-steps 0 $a > $O/${c}_${m}_$r.json 2> $O/${c}_${m}_$r.err || exit 1
      python3 -c "import json; d=[json.loads(x) for x in open('$O/${c}_${m}_$r.json') if x.startswith('{')][-1]; print('$c $m $r', d['ms_per_step'], (d.get('parity') or {}).get('differing'))"
    done
  done
done
exit 0
