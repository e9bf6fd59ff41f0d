"""Build gate on the device assembly of every kernel instantiation (called by ``_build.build_abi``).

``fa_fwd_w4`` keeps O (a0..a127) and the Q fragments (a128..a191) in literal AGPRs that only its
inline asm reads and writes (csrc/fa_agpr_asm.inc); ``fa_fwd_p8`` likewise O (a0..a63) and Q
(a64..a95). The compiler does not know these registers are
live across the separate asm statements, so a compiler-generated AGPR use in that range (for example
a VGPR spill to an AGPR after a toolchain or code change) would silently corrupt the output. This
module scans the ``-save-temps`` assembly: any use of those AGPRs (a0..a63 at D = 64) outside ``;;#ASMSTART``/``;;#ASMEND``
inside ``fa_fwd_w4``, or any kernel with ``.vgpr_spill_count`` > 0, fails the build; so does a
violation of the MFMA data-hazard rules R1-R5 around the inline-asm MFMAs (``hazards``, below).

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


# ---------------------------------------------------------------------------------------------------
# MFMA data hazards of the hand-placed (inline-asm) MFMAs: hipcc's hazard recognizer inserts the wait
# states between a visible MFMA and its neighbours, but it does not know that an inline-asm statement
# is an MFMA, so every wait around the asm MFMAs of fa_fwd_w4 is the kernel author's. The rules, with
# the counts hipcc itself inserts for the same pairs on gfx950 when the MFMA is a builtin (probed with
# hipcc 7.2 --offload-arch=gfx950, scripts/microbench/mfma_hazard_probe.hip):
#   R1  VALU write of a VGPR / AGPR  -> asm MFMA reads it as SrcA or SrcB        >= 1 wait state
#   R2  VALU write                   -> asm MFMA reads it as SrcC                >= 2
#   R3  asm MFMA writes a register   -> a non-MFMA instruction reads it          >= passes + 4
#                                       (VALU, v_accvgpr_read, LDS / VMEM data)   (12 for 32x32x16, 8 for
#                                                                                  16x16x32)
#   R4  asm MFMA writes a register   -> another MFMA reads it as SrcA / SrcB     >= passes + 4
#   (an MFMA reading as SrcC exactly the previous MFMA's destination is interlocked: 0)
#   R5  an asm MFMA reads an AGPR as SrcC (an accumulator) that is undefined (kernel entry) or was consumed by a
#       v_accvgpr_read (the epilogue's O read-out) and not written since, on some path: the stale
#       accumulator of a previous Q block (a logic error, not a wait state; the round-3 "O zeroing by
#       C = 0 MFMAs" build failed this way -- DESIGN.md section 5)
# A wait state is one issue slot: an instruction counts 1, s_nop N counts N + 1, and an MFMA that
# follows another within its pipeline occupancy first stalls until the pipe frees (passes - 1 slots
# after the previous MFMA's issue), which the walk adds as elapsed time (back-to-back 32x32x16 MFMAs
# issue 8 slots apart, MI355X_MICROARCH 'back-to-back issue'). The walk is a dataflow over the basic
# blocks of the kernel (the minimum elapsed time since each register's last write over every path),
# so a write before a branch and a read after the join are paired too.
_INSN = re.compile(r"^\s+([a-z_][a-z0-9_]*)(?:\s+(.*))?$")
_OPREG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")
_BRANCH = re.compile(r"^s_(cbranch_\w+|branch)$")
_STORE = re.compile(r"^(ds_write|ds_store|buffer_store|global_store|flat_store|scratch_store)")
_LOAD = re.compile(r"^(ds_read|ds_load|buffer_load|global_load|flat_load|scratch_load)")
HORIZON = 40  # wait states after which no rule applies any more
MAX_CTX = 8  # path contexts (branch-flag values) kept per basic block
MAX_FLAGS = 4  # branch flags tracked at once


def _regs(op: str):
    out = []
    for m in _OPREG.finditer(op):
        if m.group(1):
            out += [(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)]
        else:
            out.append((m.group(4), int(m.group(5))))
    return out


def _passes(mn: str) -> int:
    return 8 if "32x32" in mn else 4 if "16x16" in mn else 16


def _parse(text: str):
    """{kernel: [(label | None, mnemonic, operand strings, in_asm, line)]} of the fa_fwd_w4 kernels."""
    kernels, fn, in_asm = {}, None, False
    for ln in text.splitlines():
        m = re.match(r"^(_Z\S*):", ln)
        if m:
            fn = m.group(1) if m.group(1).startswith("_ZN2fa9fa_fwd_w4") else None
            if fn:
                kernels[fn] = []
            continue
        if fn is None:
            continue
        if re.match(r"^\s*\.(section|amdhsa_kernel)\b|^\.Lfunc_end", ln):  # the kernel's code ends (an
            fn = None                                                     # s_endpgm need not be last)
            continue
        if ";;#ASMSTART" in ln:
            in_asm = True
            continue
        if ";;#ASMEND" in ln:
            in_asm = False
            continue
        lab = re.match(r"^(\.?L\w+):", ln)
        if lab:
            kernels[fn].append((lab.group(1), None, [], in_asm, ln))
            continue
        code = ln.split(";")[0]
        im = _INSN.match(code)
        if not im or im.group(1).startswith("."):
            continue
        ops = [o.strip() for o in (im.group(2) or "").split(",")]
        kernels[fn].append((None, im.group(1), ops, in_asm, ln))
    return kernels


_LONGJMP = re.compile(r"\((\.?L\w+)-\.Lpost_getpc\d+\)")


def _blocks(insns):
    """Basic blocks: [(label, [insn]), ...] and successor label lists. A long branch (hipcc's
    ``s_getpc_b64`` / ``s_add_u32 s, s, (.LBBn-.Lpost_getpcM)`` / ``s_setpc_b64`` sequence in a
    kernel too large for 16-bit branch offsets) is an unconditional jump to .LBBn."""
    blocks, cur, lab = [], [], None
    for it in insns:
        if it[0] is not None:  # label
            if cur or lab is not None:
                blocks.append((lab, cur))
            lab, cur = it[0], []
            continue
        cur.append(it)
        if _BRANCH.match(it[1]) or it[1] in ("s_endpgm", "s_setpc_b64"):
            blocks.append((lab, cur))
            lab, cur = None, []
    if cur or lab is not None:
        blocks.append((lab, cur))
    index = {lab: i for i, (lab, _) in enumerate(blocks) if lab is not None}
    succ = []
    for i, (_, body) in enumerate(blocks):
        s = []
        last = body[-1][1] if body else None
        if last and _BRANCH.match(last):
            tgt = body[-1][2][0] if body[-1][2] else None
            if tgt in index:
                s.append(index[tgt])
            if last != "s_branch" and i + 1 < len(blocks):
                s.append(i + 1)
        elif last == "s_setpc_b64":
            # the target: the (.LBBn-.Lpost_getpcM) term of the s_add_u32 before it (this block or,
            # since the .Lpost_getpc label starts a block, the one before)
            tgt = None
            for j in (i, i - 1):
                for it in blocks[j][1] if j >= 0 else []:
                    m = _LONGJMP.search(it[4])
                    if m:
                        tgt = m.group(1)
            if tgt in index:
                s.append(index[tgt])
            else:  # unknown target: every block (conservative)
                s.extend(range(len(blocks)))
        elif last != "s_endpgm" and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    return blocks, succ


def _classify(mn, ops):
    """(kind, dst regs, srcA, srcB, srcC, other sources) of one instruction."""
    if mn.startswith(("v_mfma", "v_smfmac")):
        r = [_regs(o) for o in ops[:4]] + [[]] * 4
        return "mfma", r[0], r[1], r[2], r[3], []
    all_regs = [_regs(o) for o in ops]
    if _STORE.match(mn):
        return "mem", [], [], [], [], [x for rs in all_regs for x in rs]
    if _LOAD.match(mn):
        dst = [] if ops and ops[-1] == "lds" or "lds" in ops else (all_regs[0] if all_regs else [])
        return "load", dst, [], [], [], [x for rs in all_regs[1:] for x in rs]
    if mn.startswith("v_"):
        dst = all_regs[0] if all_regs and not mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) else []
        return "valu", dst, [], [], [], [x for rs in all_regs[1:] for x in rs]
    return "other", [], [], [], [], []


_SREG = re.compile(r"^s\[(\d+):(\d+)\]$|^s(\d+)$")


def _sregs(op: str):
    m = _SREG.match(op)
    if not m:
        return None
    return (int(m.group(1)), int(m.group(2))) if m.group(1) else (int(m.group(3)), int(m.group(3)))


def _flow_const(kc: dict, vcc, mn: str, ops: list):
    """Branch-flag constants (the walk prunes the infeasible edges of hipcc's structurised control flow):
    hipcc sets an SGPR pair to -1 / 0 on each incoming edge of a join and tests it after the join
    (``s_mov_b64 s[x:y], -1`` ... ``s_and_b64 vcc, exec, s[x:y]`` / ``s_cbranch_vccz``). kc maps a pair to
    its known value; vcc is "nz" / "z" / None. Returns the new vcc; kc is updated in place. Conservative:
    any other instruction naming vcc makes it unknown, and any SGPR a VALU instruction names or an SALU
    instruction writes (its first operand) drops the pairs it overlaps."""
    if mn in ("s_and_b64", "s_andn2_b64") and len(ops) == 3 and ops[0] == "vcc" and ops[1] == "exec":
        # (a flag is tested once after its join: it is forgotten here, which keeps the contexts few)
        v = kc.pop(_sregs(ops[2]), None)
        if v is None:
            return None
        nz = (v != 0) if mn == "s_and_b64" else (v == 0)  # (exec is not empty inside the kernel)
        return "nz" if nz else "z"
    if any(o.startswith("vcc") for o in ops):
        vcc = None
    named = [r for r in (_sregs(o) for o in (ops if mn.startswith("v_") else ops[:1])) if r is not None]
    for dst in named:
        for k in [k for k in kc if not (k[1] < dst[0] or k[0] > dst[1])]:
            del kc[k]
    if mn == "s_mov_b64" and len(ops) == 2 and ops[1] in ("-1", "0") and named and named[0][1] == named[0][0] + 1:
        kc[named[0]] = int(ops[1])
        while len(kc) > MAX_FLAGS:  # (the most recently set flags only)
            del kc[next(iter(kc))]
    return vcc


def hazards(text: str) -> list[str]:
    """Violations of R1-R4 around the inline-asm MFMAs of every fa_fwd_w4 kernel in ``text``."""
    out = []
    for fn, insns in _parse(text).items():
        blocks, succ = _blocks(insns)
        if not blocks:
            continue
        # state: valu[reg] = slots since its last VALU write; mf[reg] = (slots since an asm MFMA wrote
        # it, required); pipe = slots until the MFMA pipe is free
        # Path contexts: a block keeps one state per (known branch flags, vcc) combination it is entered
        # with (at most MAX_CTX, then they are merged into the flag-free context), so a state that
        # reaches a join only on the edge whose flag value skips a branch is not paired with it
        entry = [dict() for _ in blocks]
        entry[0][((), None)] = ({}, {}, 0, frozenset(("a", r) for r in range(256)))
        work = [(0, ((), None))]
        seen_err = set()
        while work:
            bi, key = work.pop()
            if key not in entry[bi]:
                continue
            valu, mf, pipe = (dict(entry[bi][key][0]), dict(entry[bi][key][1]), entry[bi][key][2])
            stale = set(entry[bi][key][3])
            kc, vcc = dict(key[0]), key[1]

            def advance(n):
                nonlocal pipe
                for d in (valu,):
                    for k in list(d):
                        d[k] += n
                        if d[k] > HORIZON:
                            del d[k]
                for k in list(mf):
                    t, req = mf[k]
                    if t + n > HORIZON:
                        del mf[k]
                    else:
                        mf[k] = (t + n, req)
                pipe = max(0, pipe - n)

            for _, mn, ops, in_asm, ln in blocks[bi][1]:
                vcc = _flow_const(kc, vcc, mn, ops)
                kind, dst, sa, sb, sc, srcs = _classify(mn, ops)
                if kind == "mfma":
                    advance(pipe)  # stall until the pipe accepts it
                    if in_asm:
                        for reg in sa + sb:
                            if valu.get(reg, HORIZON + 1) < 1:
                                seen_err.add(f"{fn}: R1 VALU write of {reg[0]}{reg[1]} -> asm MFMA SrcA/B with "
                                             f"{valu[reg]} wait states (>= 1): {ln.strip()}")
                        for reg in sc:
                            if valu.get(reg, HORIZON + 1) < 2:
                                seen_err.add(f"{fn}: R2 VALU write of {reg[0]}{reg[1]} -> asm MFMA SrcC with "
                                             f"{valu[reg]} wait states (>= 2): {ln.strip()}")
                    if in_asm:
                        for reg in sc:  # (accumulators; operand AGPRs -- the Q fragments -- are written on
                            # paths a path-insensitive walk cannot pair: the first block vs the next ones)
                            if reg in stale:
                                seen_err.add(f"{fn}: R5 asm MFMA reads {reg[0]}{reg[1]}, undefined or consumed by "
                                             f"v_accvgpr_read on some path: {ln.strip()}")
                    for reg in sa + sb:
                        if reg in mf and mf[reg][0] < mf[reg][1]:
                            seen_err.add(f"{fn}: R4 asm MFMA write of {reg[0]}{reg[1]} -> MFMA SrcA/B after "
                                         f"{mf[reg][0]} wait states (>= {mf[reg][1]}): {ln.strip()}")
                    advance(1)
                    pipe = _passes(mn) - 1
                    for reg in dst:
                        stale.discard(reg)
                        valu.pop(reg, None)
                        if in_asm:
                            mf[reg] = (0, _passes(mn) + 4)
                        else:
                            mf.pop(reg, None)
                    continue
                for reg in srcs:
                    if reg in mf and mf[reg][0] < mf[reg][1]:
                        seen_err.add(f"{fn}: R3 asm MFMA write of {reg[0]}{reg[1]} -> {mn} after {mf[reg][0]} "
                                     f"wait states (>= {mf[reg][1]}): {ln.strip()}")
                nop = re.match(r"s_nop", mn)
                advance(int(ops[0], 0) + 1 if nop and ops and ops[0] else 1)
                if mn.startswith("v_accvgpr_read"):
                    stale.update(r for r in srcs if r[0] == "a")
                for reg in dst:
                    stale.discard(reg)
                    mf.pop(reg, None)
                    if kind == "valu":
                        valu[reg] = 0
                    else:
                        valu.pop(reg, None)
            body = blocks[bi][1]
            nxt = list(succ[bi])
            if body and body[-1][1] in ("s_cbranch_vccz", "s_cbranch_vccnz") and vcc is not None and len(nxt) == 2:
                taken = (vcc == "z") == (body[-1][1] == "s_cbranch_vccz")
                nxt = [nxt[0]] if taken else [nxt[1]]  # (succ: [branch target, fall-through])
            for s in nxt:
                nkey = (tuple(sorted(kc.items())), vcc)
                if nkey not in entry[s] and len(entry[s]) >= MAX_CTX:
                    nkey = ((), None)
                    if nkey not in entry[s]:  # merge every context into the flag-free one
                        for k in list(entry[s]):
                            st = entry[s].pop(k)
                            if nkey not in entry[s]:
                                entry[s][nkey] = st
                                continue
                            a, b_ = entry[s][nkey], st
                            mv = dict(a[0])
                            for kk, vv in b_[0].items():
                                mv[kk] = min(vv, mv.get(kk, HORIZON + 1))
                            mm = dict(a[1])
                            for kk, (t, req) in b_[1].items():
                                if kk not in mm or t < mm[kk][0]:
                                    mm[kk] = (t, max(req, mm.get(kk, (0, 0))[1]))
                            entry[s][nkey] = (mv, mm, min(a[2], b_[2]), a[3] | b_[3])
                if nkey not in entry[s]:
                    entry[s][nkey] = ({k: v for k, v in valu.items()}, dict(mf), pipe, frozenset(stale))
                    work.append((s, nkey))
                    continue
                ov, om, op_, ost = entry[s][nkey]
                nv = dict(ov)
                for k, v in valu.items():
                    nv[k] = min(v, nv.get(k, HORIZON + 1))
                nm = dict(om)
                for k, (t, req) in mf.items():
                    if k not in nm or t < nm[k][0]:
                        nm[k] = (t, max(req, nm.get(k, (0, 0))[1]))
                npipe = min(op_, pipe)  # (the smaller stall: elapsed time is a lower bound)
                nst = ost | frozenset(stale)
                if (nv, nm, npipe, nst) != (ov, om, op_, ost):
                    entry[s][nkey] = (nv, nm, npipe, nst)
                    work.append((s, nkey))
        out += sorted(seen_err)
    return out


def check_file(path) -> list[str]:
    text = open(path).read()
    if "fa_fwd_w4" not in text:
        return [f"{path}: no fa_fwd_w4 kernel in the assembly (stale or wrong file)"]
    return agpr_violations(text) + spills(text) + hazards(text)


if __name__ == "__main__":
    problems = [p for f in sys.argv[1:] for p in check_file(f)]
    for p in problems[:40]:
        print(p)
    print(f"{len(problems)} problems")
    sys.exit(1 if problems else 0)
