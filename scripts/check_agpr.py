#!/usr/bin/env python3
"""Fail if hipcc itself touches an AGPR in fa_fwd_w4 (only the pinned inline asm may).

fa_fwd_w4 keeps its O accumulators in literal AGPRs a0..a127 that only inline asm reads and writes
(csrc/fa_agpr_asm.inc); a compiler-generated v_accvgpr_* or AGPR operand (e.g. a VGPR spill to an
AGPR) outside ;;#ASMSTART/;;#ASMEND would silently corrupt them. Usage: check_agpr.py file.s
"""
import re
import sys


PINNED = 192  # a0..a127 (O) and a128..a191 (Q) belong to the inline asm (fa_agpr_asm.inc)


def check(path: str) -> list[str]:
    bad, in_asm, fn = [], False, None
    pat = re.compile(r"\ba\[(\d+)(?::\d+)?\]|\ba(\d+)\b")
    for ln in open(path):
        if ln.startswith("_ZN2fa9fa_fwd_w4") and ln.rstrip().endswith(":") or re.match(r"^_ZN2fa9fa_fwd_w4\S*:", ln):
            fn = ln.split(":")[0]
        elif re.match(r"^_Z\S*:", ln):
            fn = None
        if ";;#ASMSTART" in ln:
            in_asm = True
        elif ";;#ASMEND" in ln:
            in_asm = False
        elif fn and not in_asm and not ln.lstrip().startswith(";"):
            for m in pat.finditer(ln.split(";")[0]):
                reg = int(m.group(1) or m.group(2))
                if reg < PINNED:
                    bad.append(f"{fn}: {ln.strip()}")
                    break
    return bad


if __name__ == "__main__":
    bad = check(sys.argv[1])
    for b in bad[:20]:
        print(b)
    print(f"{len(bad)} compiler uses of the pinned AGPRs a0..a{PINNED - 1} in fa_fwd_w4")
    sys.exit(1 if bad else 0)
