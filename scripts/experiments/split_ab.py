#!/usr/bin/env python3
"""Same-process A/B of the causal block layouts on one-round grids: key-split (the default; the op
passes its workspace), zigzag (split 0) and plain (split 0, zigzag 0). C4's 8-way share and smaller
single-sequence prefills. TFLOP/s per layout (useful causal FLOPs) and the max |difference|."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import flash_attention_cute_amd  # noqa: E402,F401
from flash_attention_cute_amd import _debug  # noqa: E402

dev = torch.device("cuda:0")
shapes = [("c4 share B1 Hq16/4 S4096 f16", 1, 16, 4, 4096, torch.float16),
          ("c5-like B1 Hq32/8 S2048 bf16", 1, 32, 8, 2048, torch.bfloat16),
          ("B1 Hq8/8 S8192 bf16", 1, 8, 8, 8192, torch.bfloat16),
          ("B2 Hq8/2 S4096 f16", 2, 8, 2, 4096, torch.float16)]
if "--sweep" in sys.argv:  # where the layout pays: sequence length x one-round grid fill (256 CUs)
    shapes = [(f"B1 Hq{h}/{max(h // 4, 1)} S{s} bf16 ({h * ((s + 255) // 256)} blocks)", 1, h, max(h // 4, 1), s, torch.bfloat16)
              for s in (1024, 2048, 3072, 4096, 6144, 8192) for h in (4, 8, 16, 32, 64)
              if 64 <= h * ((s + 255) // 256) <= 256]
modes = {"split": (1, None), "zigzag": (0, None), "plain": (0, 0)}
op = torch.ops.flash_attention.forward
for name, b, hq, hkv, s, dt in shapes:
    q = torch.randn(b, hq, s, 128, device=dev, dtype=dt)
    k = torch.randn(b, hkv, s, 128, device=dev, dtype=dt)
    v = torch.randn(b, hkv, s, 128, device=dev, dtype=dt)
    flops = 4 * b * hq * s * s * 128 / 2
    res = {m: [] for m in modes}
    outs, lay = {}, {}
    for rep in range(7):
        for mname, (sp, zz) in modes.items():
            _debug.set_split(sp)
            _debug.set_zigzag(zz)
            outs[mname] = op(q, k, v, 128 ** -0.5, True)
            lay[mname] = _debug.last_layout()
            torch.cuda.synchronize()
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            a.record()
            for _ in range(n):
                op(q, k, v, 128 ** -0.5, True)
            e.record()
            torch.cuda.synchronize()
            res[mname].append(flops * n / (a.elapsed_time(e) * 1e-3) / 1e12)
    _debug.set_split(None)
    _debug.set_zigzag(None)
    med = {m: sorted(r)[len(r) // 2] for m, r in res.items()}
    d = (outs["split"].float() - outs["plain"].float()).abs().max().item()
    print(f"{name}: " + ", ".join(f"{m} ({lay[m]}) {med[m]:.1f}" for m in modes)
          + f" TF/s; split/zigzag x{med['split'] / med['zigzag']:.3f}, split/plain x{med['split'] / med['plain']:.3f}; "
          f"max|split - plain| {d:.2e}", flush=True)
