"""The measurement tools that tie the committed profiles to the bench lines
(CPU): prof_summary.py (rocprof kernel trace vs a line's kernel_ms, the sizing
call excluded) and record_pmc.py (an N = 1 line's traffic -> profiles/pmc.json
for N > 1 lines), on synthetic inputs."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(kms, kpipe, traffic=3.2e9, n=1):
    return {"metric": "m", "value": 1.0, "n_gpus": n,
            "config": {"workload": "C2-bunny: x", "height": 1080, "spp_per_step": 4, "iters_per_call": 4},
            "roofline": {"kernel": "pt_wf_trace", "kernel_ms": kms, "kernel_ms_pipelined": kpipe, "traffic": traffic,
                         "traffic_source": "live", "l2_hit_rate": 0.8},
            "device": {"library": "pnrt-mi355x 0.2 (gfx950) src abcdef0123456789"}}


def test_prof_summary_excludes_the_sizing_call(tmp_path):
    rows, t = [], 0
    for call in range(3):                    # sizing call (slow), then two timed calls
        # each call starts with its ray generation; the primary pass runs in the
        # first call only (its records are reused while the camera stays)
        prim = [("pt_primary_wf", 0.2)] if call == 0 else []
        for k, ms in prim + [("pt_wf_gen_setup", 1.8)] + [("pt_wf_trace<8, false>", 3.4 if call == 0 else 3.0)] * 4:
            rows.append({"Kernel_Name": f"void {k}(DevScene)", "Start_Timestamp": t, "End_Timestamp": t + int(ms * 1e6)})
            t += int(ms * 1e6) + 1000
    tr = tmp_path / "trace.csv"
    with open(tr, "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader(); w.writerows(rows)
    ln = tmp_path / "line.json"
    line = _line(3.0, 3.1)
    line["config"]["calls"] = "serial"       # a --serial command: compared with the exclusive kernel_ms
    ln.write_text("noise\n" + json.dumps(line) + "\n")
    out = tmp_path / "out.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_summary.py"), str(tr), str(ln), str(out)],
                   check=True, capture_output=True)
    r = json.load(open(out))
    assert r["kernels"]["trace"]["launches"] == 12 and r["kernels"]["trace"]["launches_after_sizing_call"] == 8
    assert abs(r["check"]["rel_diff"]) < 1e-6 and r["check"]["compared_with"] == "kernel_ms"


def test_record_pmc_keys_by_source_hash(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import record_pmc
    out = tmp_path / "pmc.json"
    monkeypatch.setattr(record_pmc, "OUT", str(out))
    a, b = tmp_path / "a.json", tmp_path / "b.json"
    a.write_text(json.dumps(_line(3.0, 3.5)) + "\n")
    b.write_text(json.dumps(_line(3.0, 3.5, n=2)) + "\n")      # N > 1 lines are not recorded
    record_pmc.main([str(a), str(b)])
    db = json.load(open(out))
    e = db["C2-bunny/trace"]
    assert e["source_hash"] == "abcdef0123456789" and e["frames_per_launch"] == 16 and e["rows"] == 1080
    assert e["bytes_per_launch"] == 3.2e9 and len(db) == 1
