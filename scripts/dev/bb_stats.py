#!/usr/bin/env python3
"""Per-basic-block instruction mix of an extracted loop (.s), to separate hot paths from rare ones."""
import collections
import re
import sys

blocks, cur, name = [], [], "entry"
for ln in open(sys.argv[1]):
    s = ln.strip()
    m = re.match(r"^(\.LBB\S+|; %bb\.\d+):", s) or re.match(r"^(; %bb\.\d+)", s)
    if m:
        blocks.append((name, cur))
        name, cur = m.group(1), []
        continue
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur.append(s.split()[0])
blocks.append((name, cur))
for name, ins in blocks:
    if not ins:
        continue
    c = collections.Counter(ins)
    top = ", ".join(f"{k}:{v}" for k, v in c.most_common(8))
    print(f"{name:14s} n={len(ins):4d}  {top}")
