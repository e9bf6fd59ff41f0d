"""CPU model of fa_fwd_w4's persistent block walk on one XCD: which K/V tiles hit its 4 MiB L2.

Each of the XCD's workgroups walks the XCD's range of the logical block order round by round (snake),
as the kernel does (fa_fwd_kernels.hpp: block_of / decode_work); a block (batch, head, q-tile)
streams K/V tiles 0 .. n_end - 1 at one tile per time unit after a switch cost. Tiles are 32 KiB of
K + V per (kv-head, tile) in an LRU of 4 MiB. Prints the misses per algorithmic tile read (1.0 = every
head's K/V fetched once per XCD ... ideal is one miss per distinct (kv-head, tile) the XCD touches)
and the makespan, for candidate orders.
usage: python scripts/experiments/l2_walk_sim.py [c3|c4|c5|window|...]

Measured against it (round 3, profiles/r3_ab_halfmask_walk_rejected.log): the model predicts C3
1.5 -> 1.0 misses per distinct tile for hg = g instead of the kernel's max(64 / nq, g), but that
build ran C3 -0.6 % (A/B, identical output): the over-fetch the model sees is served by the
Infinity Cache and is not what limits C3, so the kernel keeps its order.
"""
import heapq
import sys
from collections import OrderedDict

CFG = {"c3": (4, 32, 32, 8192, 0), "c4": (4, 32, 8, 4096, 0), "c5": (1, 32, 8, 4096, 0),
       "window": (1, 32, 8, 32768, 4096), "mha16k": (2, 32, 32, 16384, 0), "mha2k": (8, 32, 32, 2048, 0),
       "gqa16k": (1, 64, 8, 16384, 0), "mha4k": (4, 32, 32, 4096, 0)}
B, HQ, HKV, S, W = CFG[sys.argv[1] if len(sys.argv) > 1 else "c3"]
G = HQ // HKV
NQ = S // 256
NWG = NQ * HQ * B
GRID = min(NWG, 256)
SWITCH = 4.5  # block switch in tile times (stamps: ~13k cycles vs ~2.9k per tile)
L2_TILES = (4 << 20) // (64 * 128 * 2 * 2)  # 4 MiB of 32 KiB K+V tiles


def decode(k_xcd, start, cnt, hg_rule):
    """(b, hq, qtile) of the XCD's k-th block: causal heavy-first, heads in groups of hg."""
    nb = cnt // NQ
    hg = hg_rule(nb)
    grp, kk = divmod(k_xcd, hg * NQ)
    t, hoff = divmod(kk, hg)
    bh = start // NQ + grp * hg + hoff
    return bh // HQ, bh % HQ, NQ - 1 - t


def tiles_of(qtile):
    hi = min(S // 64, (qtile + 1) * 4)
    lo = 0 if not W else max(0, (qtile * 256 - W) // 64)
    return lo, hi


def simulate(hg_rule, xcd=0):
    q8, r8 = NWG // 8, NWG % 8
    start = xcd * (q8 + 1) if xcd < r8 else r8 * (q8 + 1) + (xcd - r8) * q8
    cnt = q8 + (1 if xcd < r8 else 0)
    gx = (GRID - xcd + 7) // 8
    lru = OrderedDict()
    misses = reads = 0
    distinct = set()
    ev = [(0.0, cx, 0) for cx in range(gx)]  # (time, workgroup, round)
    heapq.heapify(ev)
    # each workgroup streams its current block tile by tile; interleave by time
    state = {}
    while ev:
        t, cx, rnd = heapq.heappop(ev)
        if cx not in state:
            kb = rnd * gx + ((gx - 1 - cx) if rnd & 1 else cx)
            if kb >= cnt:
                continue
            b, hq, qt = decode(kb, start, cnt, hg_rule)
            lo, hi = tiles_of(qt)
            state[cx] = [b, hq // G, lo, hi]
        b, hk, j, hi = state[cx]
        if j >= hi:
            del state[cx]
            heapq.heappush(ev, (t + SWITCH, cx, rnd + 1))
            continue
        key = (b, hk, j)
        reads += 1
        distinct.add(key)
        if key in lru:
            lru.move_to_end(key)
        else:
            misses += 1
            lru[key] = 1
            if len(lru) > L2_TILES:
                lru.popitem(last=False)
        state[cx][2] = j + 1
        heapq.heappush(ev, (t + 1.0, cx, rnd))
        last = t + 1.0
    return misses / len(distinct), last


rules = {
    "kernel (hg = max(64/nq, g))": lambda nb: _fit(max(64 // NQ, G), nb),
    "hg = 1 head": lambda nb: _fit(1, nb),
    "hg = g (one GQA group)": lambda nb: _fit(G, nb),
    "hg = 2g": lambda nb: _fit(2 * G, nb),
    "hg = all heads": lambda nb: nb,
}


def _fit(hg, nb):
    hg = max(1, min(hg, nb))
    while nb % hg:
        hg -= 1
    return hg


for name, rule in rules.items():
    m, span = simulate(rule)
    print(f"{sys.argv[1] if len(sys.argv) > 1 else 'c3'}: {name:28s} misses / distinct tiles {m:.3f}  makespan {span:.0f}")
