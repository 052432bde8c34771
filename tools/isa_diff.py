#!/usr/bin/env python3
"""Compare the per-kernel instruction streams of two device-assembly files
(hipcc --cuda-device-only -S), e.g. before and after a source refactor that
must not change the product kernels:

    tools/isa_diff.py old.s new.s [name-map old=new ...]

Comments, directives and basic-block label numbers are normalised away; a
kernel whose instruction stream is identical prints "same".  Kernels present
on one side only are listed.  Exit status 1 when any common kernel differs."""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+|[A-Za-z_]\w*):\s*(;.*)?$", line)
        if m and not line.startswith(".L"):
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            out[cur] = body
            cur = None
            continue
        t = line.split(";")[0].strip()
        if not t or t.startswith("."):
            if re.match(r"^\.LBB\d+_\d+:", t):
                body.append("LBB:")
            continue
        body.append(re.sub(r"\.LBB\d+_\d+", "LBB", t))
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    rename = dict(x.split("=", 1) for x in sys.argv[3:])
    bad = 0
    for k in sorted(a):
        kb = rename.get(k, k)
        if kb not in b:
            print(f"only in old: {k}")
            continue
        if a[k] == b[kb]:
            print(f"same      {len(a[k]):6d} lines  {k[:90]}")
        else:
            bad += 1
            va = sum(1 for x in a[k] if x.startswith("v_"))
            vb = sum(1 for x in b[kb] if x.startswith("v_"))
            print(f"DIFFERENT {len(a[k]):6d} -> {len(b[kb]):6d} lines, VALU {va} -> {vb}  {k[:90]}")
    for k in sorted(set(b) - {rename.get(x, x) for x in a}):
        print(f"only in new: {k}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
