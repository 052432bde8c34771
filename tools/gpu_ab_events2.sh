cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/ev; mkdir -p $O
v() { python -c "import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);print(d['value'])"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc > $O/a$r.log 2>&1 || exit 1; echo "events    $(v $O/a$r.log)"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-kernel-events > $O/b$r.log 2>&1 || exit 1; echo "no-events $(v $O/b$r.log)"
done
timeout -k 10 200 python tools/shard_sim.py 20 16 > $O/ss.txt 2>&1 || exit 1; grep "N=1" $O/ss.txt
