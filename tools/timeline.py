"""GPU busy time from a rocprofv3 kernel trace: over the window from the first to the
last pt_* kernel, the union of kernel intervals (busy), the sum of kernel durations
(> busy when kernels overlap) and the idle time.
    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [skip_first_n_kernels]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("pt_", "void pt_"))]
ivs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
ivs = ivs[int(sys.argv[2]) if len(sys.argv) > 2 else 0:]
t0, t1 = ivs[0][0], max(e for _, e in ivs)
busy, (cs, ce) = 0, ivs[0]
for s, e in ivs[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
tot = sum(e - s for s, e in ivs)
print(f"window {(t1 - t0) / 1e6:.3f} ms: busy {busy / 1e6:.3f} ms ({100 * busy / (t1 - t0):.1f} %), "
      f"sum of kernel durations {tot / 1e6:.3f} ms (mean concurrency {tot / busy:.2f}), {len(ivs)} kernels")
