#!/usr/bin/env python3
"""Instruction census of the trace kernel's step loops (the innermost loops that
issue the geometry fetch), from the assembly tools/isa_count.sh leaves in
/tmp/isa_trace.s: every basic block whose loop comment names the loop's header.

    python tools/isa_loop.py [/tmp/isa_trace.s]
"""
import re
import sys
from collections import Counter


def main(path):
    lines = open(path).read().splitlines()
    blocks, cur = [], None
    for ln in lines:
        m = re.match(r'^(\.LBB\d+_\d+|; %bb\.\d+):?\s*(;.*)?$', ln)
        if m:
            cur = {"name": m.group(1), "comment": ln, "ins": []}
            blocks.append(cur)
            continue
        if cur is not None:
            t = ln.split(";")[0].strip()
            if t and not t.startswith("."):
                cur["ins"].append(t)
    # a loop header block carries "Loop Header"; members say "Header=BB<id>" (or are the header)
    for i, b in enumerate(blocks):
        if "Inner Loop Header" not in b["comment"] and "Inner Loop Header" not in " ".join(
                lines[lines.index(b["comment"]) + 1:lines.index(b["comment"]) + 4]):
            continue
        hid = b["name"].lstrip(".L")
        members = [x for x in blocks if x is b or f"Header={hid} " in x["comment"] + " "]
        ins = [x for m in members for x in m["ins"]]
        if not any("buffer_load_dwordx4" in x for x in ins):
            continue
        op = Counter(x.split()[0] for x in ins)
        v = sum(c for k, c in op.items() if k.startswith("v_"))
        s = sum(c for k, c in op.items() if k.startswith("s_"))
        print(f"loop {hid}: blocks {len(members)}  VALU {v}  SALU {s}  cndmask {sum(c for k, c in op.items() if k.startswith('v_cndmask'))}"
              f"  cmp {sum(c for k, c in op.items() if k.startswith('v_cmp'))}  branches {sum(c for k, c in op.items() if k.startswith('s_cbranch'))}"
              f"  LDS {sum(c for k, c in op.items() if k.startswith('ds_'))}  VMEM {sum(c for k, c in op.items() if k.startswith(('buffer_', 'global_', 'scratch_')))}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa_trace.s")
