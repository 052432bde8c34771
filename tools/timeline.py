"""Step timeline from a rocprofv3 kernel trace: per step (primary kernel to the next
primary), the wall time, the busy time (union of kernel intervals), the sum of kernel
durations (> busy when kernels overlap) and the idle gaps.
    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("pt_", "void pt_"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps, cur = [], []
for r in rows:
    if "pt_primary_kernel" in r["Kernel_Name"] and cur:
        steps.append(cur)
        cur = []
    cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
steps.append(cur)
for k, st in enumerate(steps[1:-1][-4:]):
    t0, t1 = st[0][0], max(e for _, e, _ in st)
    busy, last = 0, t0
    ivs = sorted((s, e) for s, e, _ in st)
    cs, ce = ivs[0]
    for s, e in ivs[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    tot = sum(e - s for s, e, _ in st)
    print(f"step: wall {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f}  sum of kernels {tot / 1e6:.3f}  "
          f"idle {(t1 - t0 - busy) / 1e6:.3f}  kernels {len(st)}")
