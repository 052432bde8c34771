#!/usr/bin/env python3
"""Condense a round's A/B session directories (profiles/rNN/sK/) into one
summary.txt each (VERDICT r4 "Next" 7): every bench line's headline figures
(value, ms per step, exclusive / pipelined trace launch, parity) and the tail
of every text record, one line per run.  The raw files stay in git history.

    python tools/condense_profiles.py profiles/r04 [--keep s1/tail_D2_timing.txt ...] [--apply]

Without --apply it only prints what it would write and remove.  A session that
already has a summary.txt keeps it (the figures quoted in DESIGN.md were taken
from it); the other files of the session are removed either way, except the
--keep paths (records DESIGN.md cites by name) and the final/ directory.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess


def line_of(path: str) -> str | None:
    try:
        txt = open(path).read()
    except OSError:
        return None
    for ln in reversed(txt.splitlines()):
        ln = ln.strip()
        if ln.startswith("{") and '"value"' in ln:
            try:
                d = json.loads(ln)
            except ValueError:
                continue
            r = d.get("roofline") or {}
            par = d.get("parity") or {}
            ex = (d.get("kernels_exclusive") or {}).get("trace", {})
            return (f"{d.get('value')} Msamples/s  {d.get('ms_per_step')} ms/step  trace excl "
                    f"{ex.get('ms_per_launch')} ms  pipelined {r.get('kernel_ms_pipelined')} ms  frac {r.get('frac')}  "
                    f"parity {par.get('differing', '-')}/{par.get('pixels', '-')}  "
                    f"[{(d.get('config') or {}).get('workload', '')[:40]}]")
    return None


def summarise(sdir: str, files: list[str]) -> str:
    out = [f"# {sdir}: condensed from {len(files)} raw files (git history holds them)"]
    for f in sorted(files):
        p = os.path.join(sdir, f)
        if f.endswith(".json"):
            s = line_of(p)
            if s is None:
                try:
                    d = json.load(open(p))
                    s = json.dumps(d)[:300]
                except (OSError, ValueError):
                    s = "(unreadable)"
            out.append(f"{f}: {s}")
        elif f.endswith((".txt", ".log")):
            lines = open(p, errors="replace").read().splitlines()
            out.append(f"== {f} (last {min(25, len(lines))} of {len(lines)} lines)")
            out += ["  " + ln for ln in lines[-25:]]
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round_dir")
    ap.add_argument("--keep", nargs="*", default=[])
    ap.add_argument("--apply", action="store_true")
    a = ap.parse_args()
    tracked = subprocess.run(["git", "ls-files", a.round_dir], capture_output=True, text=True, check=True).stdout.split()
    sessions: dict[str, list[str]] = {}
    for t in tracked:
        rel = os.path.relpath(t, a.round_dir)
        parts = rel.split(os.sep)
        if len(parts) < 2 or parts[0] == "final":
            continue
        sessions.setdefault(parts[0], []).append(os.sep.join(parts[1:]))
    keep = set(a.keep)
    for s, files in sorted(sessions.items()):
        sdir = os.path.join(a.round_dir, s)
        has = "summary.txt" in files
        raw = [f for f in files if f != "summary.txt" and os.path.join(s, f) not in keep]
        if not has:
            text = summarise(sdir, raw)
            print(f"{sdir}/summary.txt: {len(text.splitlines())} lines from {len(raw)} files")
            if a.apply:
                open(os.path.join(sdir, "summary.txt"), "w").write(text)
        print(f"{sdir}: remove {len(raw)} raw files")
        if a.apply and raw:
            subprocess.run(["git", "rm", "-q", "--"] + [os.path.join(sdir, f) for f in raw], check=True)
        if a.apply and not has:
            subprocess.run(["git", "add", os.path.join(sdir, "summary.txt")], check=True)


if __name__ == "__main__":
    main()
