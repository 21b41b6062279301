#!/usr/bin/env python
"""Instruction mix of a kernel's hottest loop in a hipcc -S listing:
python tools/asmstats.py file.s <kernel-substring>.  Reports, per loop
(backward branch target), counts of MFMA / VALU / LDS / VMEM / SALU / waitcnt."""
import re
import sys
from collections import Counter


def main(path, pat):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^[A-Za-z_]\S*:", l) and pat in l.split(":")[0]:
            start = i
            break
    if start is None:
        print("kernel not found")
        return
    end = start
    while end < len(lines) and not lines[end].strip().startswith(".Lfunc_end"):
        end += 1
    body = lines[start:end]
    labels = {l.strip()[:-1]: j for j, l in enumerate(body) if re.match(r"^\.LBB\S+:$", l.strip())}
    loops = []
    for j, l in enumerate(body):
        m = re.match(r"\s*s_cbranch_\w+\s+(\.LBB\S+)|\s*s_branch\s+(\.LBB\S+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < j:
                loops.append((labels[tgt], j))
    print(f"kernel lines {len(body)}; loops {len(loops)}")
    for a, b in loops:
        c = Counter()
        for l in body[a:b + 1]:
            t = l.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            op = t[0]
            if "mfma" in op:
                c["mfma"] += 1
            elif op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_")):
                c["vmem"] += 1
            elif op.startswith("s_waitcnt"):
                c["waitcnt"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
        print(f"  loop lines {a}-{b}: {dict(c)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
