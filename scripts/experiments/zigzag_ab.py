#!/usr/bin/env python3
"""Same-process A/B of the zigzag causal Q-block layout (knob 0 = plain blocks, 1 = the default rule)
on one-round causal grids: C4's share of the 8-way split (B1 Hq16 Hkv4 S4096 fp16) and smaller
single-sequence prefills. Prints TFLOP/s per mode and whether zigzag ran."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import flash_attention_cute_amd  # noqa: E402,F401
from flash_attention_cute_amd import _debug  # noqa: E402

dev = torch.device("cuda:0")
shapes = [("c4 share B1 Hq16/4 S4096 f16", 1, 16, 4, 4096, torch.float16),
          ("B1 Hq8/8 S8192 bf16", 1, 8, 8, 8192, torch.bfloat16),
          ("B1 Hq32/8 S2048 bf16", 1, 32, 8, 2048, torch.bfloat16)]
op = torch.ops.flash_attention.forward
for name, b, hq, hkv, s, dt in shapes:
    q = torch.randn(b, hq, s, 128, device=dev, dtype=dt)
    k = torch.randn(b, hkv, s, 128, device=dev, dtype=dt)
    v = torch.randn(b, hkv, s, 128, device=dev, dtype=dt)
    flops = 4 * b * hq * s * s * 128 / 2
    res = {0: [], 1: []}
    outs = {}
    for rep in range(7):
        for mode in (0, 1):
            _debug.set_zigzag(mode)
            o = op(q, k, v, 128 ** -0.5, True)
            torch.cuda.synchronize()
            outs[mode] = (o, _debug.last_zigzag())
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            a.record()
            for _ in range(n):
                op(q, k, v, 128 ** -0.5, True)
            e.record()
            torch.cuda.synchronize()
            res[mode].append(flops * n / (a.elapsed_time(e) * 1e-3) / 1e12)
    _debug.set_zigzag(None)
    med = {m: sorted(r)[len(r) // 2] for m, r in res.items()}
    same = torch.equal(outs[0][0], outs[1][0])
    print(f"{name}: plain {med[0]:.1f} TF/s, zigzag-rule {med[1]:.1f} TF/s (ran zigzag: {bool(outs[1][1])}), "
          f"x{med[1] / med[0]:.3f}, bit-identical {same}", flush=True)
