"""Per-class view of a pipelined rocprofv3 kernel trace: over the window of the
timed steps, the share of time with >= 1 kernel of each class running, the
mean duration of each class, and the share of time the trace kernel runs
alone / beside shade / beside gen.
    python tools/timeline2.py gpurun_out/.../run_kernel_trace.csv [skip_first_n]"""
import csv
import sys

CLS = {"pt_wf_trace": "trace", "pt_wf_shade_setup": "shade", "pt_wf_gen_setup": "gen", "pt_primary_kernel": "primary", "pt_primary_wf": "primary",
       "pt_blend_kernel": "blend"}
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0].strip()
    if k in CLS:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), CLS[k]))
rows.sort()
rows = rows[int(sys.argv[2]) if len(sys.argv) > 2 else 0:]
t0, t1 = rows[0][0], max(e for _, e, _ in rows)
ev = []
for s, e, c in rows:
    ev.append((s, 1, c))
    ev.append((e, -1, c))
ev.sort()
act = {c: 0 for c in CLS.values()}
share = {}
last = t0
for t, d, c in ev:
    if t > last:
        key = tuple(sorted(k for k, v in act.items() if v))
        share[key] = share.get(key, 0) + (t - last)
    act[c] += d
    last = t
win = t1 - t0
print(f"window {win / 1e6:.3f} ms, {len(rows)} kernels")
for c in CLS.values():
    durs = [e - s for s, e, k in rows if k == c]
    if durs:
        on = sum(v for k, v in share.items() if c in k)
        print(f"  {c:8s} n={len(durs):4d} mean {sum(durs) / len(durs) / 1e3:8.1f} us  active {100 * on / win:5.1f} % of window")
print("  top concurrency patterns (% of window):")
for k, v in sorted(share.items(), key=lambda kv: -kv[1])[:10]:
    print(f"    {100 * v / win:5.1f} %  {'+'.join(k) or 'idle'}")
