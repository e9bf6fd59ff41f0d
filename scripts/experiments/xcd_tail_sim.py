#!/usr/bin/env python3
"""What a finer tail could recover from the XCD clock skew (the 'half-block
XCD tail' prototype, as a model driven by measured per-XCD end times).

Input: the per-XCD end times of a C2 launch from the round-3 realtime stamps
(profiles/r3_st_rt_c2.log: 8 XCDs x 256 blocks, equal blocks, static schedule; the XCDs run the same
cycles at different clocks). Each XCD's block rate follows from its end time. The model then schedules
the LAST round of blocks three ways and reports the launch span:

  static     every XCD keeps its 32 last blocks (the kernel today; reproduces the measured span)
  whole      the last round's 256 blocks claimed dynamically by whichever workgroup is free first
             (a global counter; one claim costs `claim_us`, an unprefetched Q / K_0 load)
  half       the last round split by keys into 512 half-blocks claimed dynamically; every pair then
             needs a combine (partial O and row statistics through HBM: `combine_us` on the
             workgroup that finishes last)
  quarter    the same with 1024 quarter-blocks

usage: python scripts/experiments/xcd_tail_sim.py [claim_us] [combine_us]
"""
import heapq
import sys

END_US = [941.0, 962.4, 966.2, 983.4, 956.7, 967.7, 921.8, 962.5]  # r3_st_rt_c2.log, xcd 0..7
BLOCKS_PER_WG = 8  # C2: 2048 blocks / 256 workgroups
WG_PER_XCD = 32


def simulate(claim_us: float, combine_us: float):
    per_block = [e / BLOCKS_PER_WG for e in END_US]  # us per block on a workgroup of XCD x
    out = {"static": max(END_US)}
    # the first BLOCKS_PER_WG - 1 rounds stay static; the last round is pooled
    free = [(per_block[x] * (BLOCKS_PER_WG - 1), x) for x in range(8) for _ in range(WG_PER_XCD)]
    for mode, items, frac in (("whole", 256, 1.0), ("half", 512, 0.5), ("quarter", 1024, 0.25)):
        heap = list(free)
        heapq.heapify(heap)
        ends = []
        for _ in range(items):
            t, x = heapq.heappop(heap)
            t += claim_us + per_block[x] * frac
            ends.append(t)
            heapq.heappush(heap, (t, x))
        span = max(ends)
        if mode != "whole":
            span += combine_us  # the last block's combine runs after its last piece
        out[mode] = span
    return out


def main():
    claim = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    comb = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    print(f"per-XCD end (measured, static): {END_US} us; mean {sum(END_US) / 8:.1f}, max {max(END_US):.1f}")
    for c, m in ((0.0, 0.0), (claim, 0.0), (claim, comb), (claim, 2 * comb)):
        r = simulate(c, m)
        print(f"claim {c:4.1f} us, combine {m:4.1f} us: static {r['static']:.1f}  whole-block tail {r['whole']:.1f} "
              f"({r['static'] / r['whole'] - 1:+.1%})  half-block tail {r['half']:.1f} ({r['static'] / r['half'] - 1:+.1%})"
              f"  quarter-block tail {r['quarter']:.1f} ({r['static'] / r['quarter'] - 1:+.1%})")
    print("(the bound: every XCD ending at the mean, "
          f"{max(END_US) / (sum(END_US) / 8) - 1:+.1%})")


if __name__ == "__main__":
    main()
