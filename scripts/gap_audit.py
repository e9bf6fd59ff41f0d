"""Per-gap issue audit of fa_fwd_w4's hot loop.

One wave per SIMD issues one instruction per ~4 cycles whatever its kind, and a 32x32x16 MFMA holds
the SIMD's issue for 8 of its 32 cycles, so the fillers between two MFMAs hide only while their issue
costs stay within ~24 cycles: at most 5 single-issue fillers, at most one of them an 8-cycle
transcendental (MI355X_MICROARCH.md, 'single-issue instructions HIDDEN per v_mfma_f32_32x32x16_bf16
gap'). This script reads the build's -save-temps assembly of one instantiation, finds the unmasked
pipelined loop (the loop of two tiles, 128 MFMAs, with the fewest instructions) and lists, for
every gap between consecutive MFMAs in program order, its fillers by kind and an issue-cost estimate
from the guide's constants table:

    MFMA 8, v_exp/v_log/v_rcp/... 8, other VALU 4, SALU / s_waitcnt / branch 4, s_nop N 4 (N + 1),
    ds_read 4, LDS-DMA piece (buffer_load ... lds) 60 (the guide: ~60 among bare MFMAs).

Usage: python scripts/gap_audit.py [build/obj/f16_c0_d128_x1/fa_inst-hip-amdgcn-amd-amdhsa-gfx950.s]
"""
from __future__ import annotations

import collections
import pathlib
import re
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from flash_attention_cute_amd import _asm_check as A  # noqa: E402

TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_")


def kind(mn: str, ops) -> str:
    if mn.startswith("v_mfma"):
        return "mfma"
    if TRANS.match(mn):
        return "trans"
    if mn.startswith("buffer_load") and "lds" in " ".join(ops).split():
        return "ldsdma"
    if mn.startswith(("ds_read", "ds_load")):
        return "lds"
    if mn.startswith(("buffer_", "global_")):
        return "vmem"
    if mn.startswith("s_nop"):
        return "nop"
    if mn == "s_waitcnt":
        return "wait"
    if mn in ("s_barrier",):
        return "barrier"
    if mn.startswith("s_"):
        return "salu"
    if mn.startswith("v_"):
        return "valu"
    return "other"


def cost(k: str, mn: str, ops) -> int:
    if k in ("mfma", "trans"):
        return 8
    if k == "ldsdma":
        return 60
    if k == "nop":
        return 4 * (int(ops[0], 0) + 1 if ops and ops[0] else 1)
    return 4


def hot_loop(insns):
    """(start, end) block indices of the two-tile loop with 128 MFMAs and the fewest instructions."""
    blocks, succ = A._blocks(insns)
    best = None
    for i, s in enumerate(succ):
        for j in s:
            if j > i:
                continue
            body = [it for b in blocks[j:i + 1] for it in b[1]]
            n = sum(1 for it in body if it[1].startswith("v_mfma"))
            if n == 128 and (best is None or len(body) < best[0]):
                best = (len(body), j, i)
    if best is None:
        raise SystemExit("no two-tile loop with 128 MFMAs found")
    return blocks, best[1], best[2]


def audit(path: str):
    text = open(path).read()
    kernels = A._parse(text)
    out = []
    for fn, insns in kernels.items():
        blocks, j, i = hot_loop(insns)
        body = [it for b in blocks[j:i + 1] for it in b[1]]
        gaps, cur, first = [], None, True
        for _, mn, ops, _, _ in body:
            k = kind(mn, ops)
            if k == "mfma":
                if cur is not None:
                    gaps.append(cur)
                cur = collections.Counter()
                cur["_cost"] = 8
                continue
            if cur is None:  # the loop head before its first MFMA: counted with the last gap
                continue
            cur[k] += 1
            cur["_cost"] += cost(k, mn, ops)
        gaps.append(cur)  # last MFMA -> loop end (barrier, branch): the tile boundary
        out.append((fn, gaps, len(body)))
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "build/obj/f16_c0_d128_x1/fa_inst-hip-amdgcn-amd-amdhsa-gfx950.s")
    for fn, gaps, n in audit(path):
        print(f"{fn}\n  hot loop: {n} instructions, {len(gaps)} MFMA gaps (two tiles)")
        kinds = ["valu", "trans", "lds", "ldsdma", "salu", "wait", "nop", "barrier", "vmem", "other"]
        print("  gap  phase  " + " ".join(f"{k:>6}" for k in kinds) + "  fillers  cost(cyc)")
        over5 = overexp = overcost = 0
        per_phase = collections.defaultdict(lambda: [0, 0, 0])
        for g, c in enumerate(gaps):
            fill = sum(c[k] for k in kinds)
            ph = (g // 32) % 2 + 1
            per_phase[ph][0] += fill
            per_phase[ph][1] += c["_cost"]
            per_phase[ph][2] += max(32, c["_cost"])
            flag = []
            if fill > 5:
                over5 += 1
                flag.append(">5")
            if c["trans"] > 1:
                overexp += 1
                flag.append(">1exp")
            if c["_cost"] > 32:
                overcost += 1
                flag.append(">32")
            print(f"  {g:3d}  p{ph}     " + " ".join(f"{c[k]:6d}" for k in kinds)
                  + f"  {fill:7d}  {c['_cost']:5d} {' '.join(flag)}")
        print(f"  gaps with > 5 fillers: {over5}; with > 1 transcendental: {overexp}; "
              f"issue estimate > 32 cycles: {overcost} of {len(gaps)}")
        for ph, (f, cst, eff) in sorted(per_phase.items()):
            print(f"  phase {ph} (both tiles): {f} fillers, issue estimate {cst} cycles, "
                  f"max(32, gap) sum {eff} cycles (MFMA floor {32 * 64})")


if __name__ == "__main__":
    main()
