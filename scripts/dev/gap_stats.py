"""Per-MFMA-gap instruction mix of a loop listing (build/asm/loop.s from scripts/dev/asm_loop.sh).
Issue cost model (MI355X_MICROARCH.md 'vector-instruction ISSUE cost'): trans 8, VALU 4, MFMA 8,
ds 4 (rough), DMA 25 (measured here), s_nop N -> 4(N+1)/4.. rough."""
import re
import sys

lines = [l.strip() for l in open(sys.argv[1] if len(sys.argv) > 1 else "build/asm/loop.s")
         if l.strip() and not l.strip().startswith(";") and not l.strip().startswith(".")]
gaps, cur = [], []
for l in lines:
    op = l.split()[0]
    if op.startswith("v_mfma"):
        gaps.append(cur)
        cur = []
    else:
        cur.append(op)
gaps.append(cur)


def cost(ops):
    c = 0
    for o in ops:
        if o.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
            c += 8
        elif o.startswith("v_accvgpr") or o.startswith("v_"):
            c += 4
        elif o.startswith("ds_"):
            c += 4
        elif o.startswith("buffer_load") and "lds" in o:
            c += 25
        elif o.startswith("buffer_") or o.startswith("global_"):
            c += 8
        elif o == "s_nop":
            c += 4
    return c


for i, g in enumerate(gaps):
    ex = sum(o.startswith("v_exp") for o in g)
    va = sum(o.startswith("v_") and not o.startswith("v_exp") for o in g)
    ds = sum(o.startswith("ds_") for o in g)
    bl = sum(o.startswith("buffer") for o in g)
    sa = sum(o.startswith("s_") for o in g)
    print(f"gap {i:3d}: cost {cost(g)+8:3d}  exp {ex} valu {va:2d} ds {ds} dma {bl} salu {sa:2d} | {' '.join(g)[:150]}")
