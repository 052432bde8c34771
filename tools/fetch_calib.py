#!/usr/bin/env python3
"""FETCH_SIZE calibration for scattered 64-B gathers.

Runs tools/microtests/fetch_calib (four dispatches, known byte counts over a
1 GiB table: stream / gather64 / half64 / line128) once plain (timing) and
under separate rocprofv3 --kernel-trace --pmc passes, and writes per pattern
known bytes, FETCH_SIZE bytes, TCC_EA0_RDREQ and the ratios to a JSON file:

    python tools/fetch_calib.py OUT.json

bench.py's FETCH_FACTOR (fabric read bytes = FETCH_FACTOR x FETCH_SIZE KiB) is
set from the gather64 / half64 rows of the committed result
(profiles/r03/fetch_calibration.json)."""
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "microtests", "fetch_calib")
PASSES = [("FETCH_SIZE",), ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"), ("TCC_HIT_sum", "TCC_MISS_sum")]


def counters(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"calib<(\d)>", r["Kernel_Name"])
            if not m:
                continue
            k = int(m.group(1))
            per.setdefault(k, {})
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main():
    out = sys.argv[1]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    plain = subprocess.run(["timeout", "-s", "KILL", "60", EXE], capture_output=True, text=True, env=env)
    if plain.returncode != 0:
        raise SystemExit(f"fetch_calib failed: {plain.stdout}{plain.stderr}")
    rows = {}
    for line in plain.stdout.splitlines():
        if line.startswith("{"):
            r = json.loads(line)
            rows[r["dispatch"]] = r
    tmp = tempfile.mkdtemp(prefix="fcal_", dir=env["TMPDIR"])
    errors = {}
    try:
        for i, group in enumerate(PASSES):
            d = os.path.join(tmp, f"p{i}")
            r = subprocess.run(["timeout", "-s", "KILL", "60", "rocprofv3", "--kernel-trace", "--pmc", *group, "-d", d,
                                "-o", "run", "--output-format", "csv", "--", EXE], capture_output=True, text=True, env=env)
            if r.returncode != 0:
                errors[" ".join(group)] = (r.stdout + r.stderr)[-600:]
                continue
            for k, cs in counters(d).items():
                rows[k].update({c: v for c, v in cs.items()})
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    for r in rows.values():
        if "FETCH_SIZE" in r:
            fb = r["FETCH_SIZE"] * 1024.0
            r["fetch_size_bytes"] = fb
            r["known_over_fetch_size"] = round(r["known_bytes"] / fb, 4) if fb else None
            r["lines_over_fetch_size"] = round(r["lines_touched_bytes"] / fb, 4) if fb else None
        if r.get("TCC_EA0_RDREQ_sum"):
            r["known_bytes_per_rdreq"] = round(r["known_bytes"] / r["TCC_EA0_RDREQ_sum"], 2)
            r["lines_bytes_per_rdreq"] = round(r["lines_touched_bytes"] / r["TCC_EA0_RDREQ_sum"], 2)
    res = {"what": "FETCH_SIZE vs known bytes, 1 GiB table (4x Infinity Cache), one dispatch per pattern "
                   "(tools/microtests/fetch_calib.hip)", "patterns": [rows[k] for k in sorted(rows)], "errors": errors}
    json.dump(res, open(out, "w"), indent=1)
    for r in res["patterns"]:
        print(r["pattern"], "ms", r["ms"], "known GB/s", r["known_GBps"], "known/FETCH", r.get("known_over_fetch_size"),
              "B/RDREQ", r.get("known_bytes_per_rdreq"), "hit", r.get("TCC_HIT_sum"), "miss", r.get("TCC_MISS_sum"))
    if errors:
        print("pass errors:", json.dumps(errors)[:800])


if __name__ == "__main__":
    main()
