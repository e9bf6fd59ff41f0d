"""Build gate on the device assembly of every kernel instantiation (called by ``_build.build_abi``).

``fa_fwd_w4`` keeps O (a0..a127) and the Q fragments (a128..a191) in literal AGPRs that only its
inline asm reads and writes (csrc/fa_agpr_asm.inc); ``fa_fwd_p8`` likewise O (a0..a63) and Q
(a64..a95). The compiler does not know these registers are
live across the separate asm statements, so a compiler-generated AGPR use in that range (for example
a VGPR spill to an AGPR after a toolchain or code change) would silently corrupt the output. This
module scans the ``-save-temps`` assembly: any use of those AGPRs (a0..a63 at D = 64) outside ``;;#ASMSTART``/``;;#ASMEND``
inside ``fa_fwd_w4``, or any kernel with ``.vgpr_spill_count`` > 0, fails the build.

CLI: ``python -m flash_attention_cute_amd._asm_check file.s [...]``
"""
from __future__ import annotations

import re
import sys

QBASE, QEND = 128, 192  # the Q fragments a128..a191 belong to the inline asm (fa_agpr_asm.inc)
_REG = re.compile(r"\ba\[(\d+)(?::\d+)?\]|\ba(\d+)\b")
_TILE = re.compile(r"ELi(64|128)ELb")  # the head-dim tile template argument of the mangled name


def pinned_p8(fn: str, reg: int) -> bool:
    """fa_fwd_p8 (256 registers per wave): O^T of its one 32-row block in a0..a(D/2 - 1), the Q
    fragments in a64..a95 (a64..a79 at D = 64)."""
    m = _TILE.search(fn)
    d = int(m.group(1)) if m else 128
    return reg < d // 2 or 64 <= reg < 64 + d // 4


def pinned(fn: str, reg: int) -> bool:
    """a0..a(head-dim tile - 1) hold O^T of both 32-row blocks (D/32 d-tiles x 16 each x 2 blocks),
    a128..a191 the Q fragments; at D = 64 the compiler may use a64..a127."""
    m = _TILE.search(fn)
    o_end = int(m.group(1)) if m else 128
    return reg < o_end or QBASE <= reg < QEND


def agpr_violations(text: str) -> list[str]:
    """Compiler-generated uses of the pinned AGPRs inside fa_fwd_w4 (one entry per offending line)."""
    bad, in_asm, fn = [], False, None
    for ln in text.splitlines():
        m = re.match(r"^(_Z\S*):", ln)
        if m:
            fn = m.group(1) if m.group(1).startswith(("_ZN2fa9fa_fwd_w4", "_ZN2fa9fa_fwd_p8")) else None
            continue
        if ";;#ASMSTART" in ln:
            in_asm = True
        elif ";;#ASMEND" in ln:
            in_asm = False
        elif fn and not in_asm and not ln.lstrip().startswith(";"):
            for r in _REG.finditer(ln.split(";")[0]):
                rule = pinned_p8 if fn.startswith("_ZN2fa9fa_fwd_p8") else pinned
                if rule(fn, int(r.group(1) or r.group(2))):
                    bad.append(f"{fn}: {ln.strip()}")
                    break
    return bad


def spills(text: str) -> list[str]:
    """Kernels whose metadata reports VGPR spills to memory."""
    out = []
    for block in re.split(r"\n\s*- \.", text):
        name = re.search(r"\.name:\s+(\S+)", block)
        vs = re.search(r"\.vgpr_spill_count:\s+(\d+)", block)
        if name and vs and int(vs.group(1)) > 0:
            out.append(f"{name.group(1)}: vgpr_spill_count {vs.group(1)}")
    return out


def check_file(path) -> list[str]:
    text = open(path).read()
    if "fa_fwd_w4" not in text:
        return [f"{path}: no fa_fwd_w4 kernel in the assembly (stale or wrong file)"]
    return agpr_violations(text) + spills(text)


if __name__ == "__main__":
    problems = [p for f in sys.argv[1:] for p in check_file(f)]
    for p in problems[:40]:
        print(p)
    print(f"{len(problems)} problems")
    sys.exit(1 if problems else 0)
