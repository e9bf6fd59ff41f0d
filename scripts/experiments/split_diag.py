#!/usr/bin/env python3
"""Key-split diagnostic: run the split layout several times on one shape and report, against the
plain layout, which (head, row) ranges differ and by how much (torn combine vs rounding)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import flash_attention_cute_amd  # noqa: E402,F401
from flash_attention_cute_amd import _debug  # noqa: E402

dev = torch.device("cuda:0")
op = torch.ops.flash_attention.forward
for (b, hq, hkv, s, d) in [(1, 4, 2, 1024, 128), (2, 2, 1, 640, 64)]:
    torch.manual_seed(0)
    q = torch.randn(b, hq, s, d, device=dev, dtype=torch.float16)
    k = torch.randn(b, hkv, s, d, device=dev, dtype=torch.float16)
    v = torch.randn(b, hkv, s, d, device=dev, dtype=torch.float16)
    _debug.set_split(0)
    _debug.set_zigzag(0)
    plain = op(q, k, v, d ** -0.5, True).float()
    _debug.set_split(1)
    _debug.set_zigzag()
    for rep in range(6):
        out = op(q, k, v, d ** -0.5, True)
        lay = _debug.last_layout()
        torch.cuda.synchronize()
        diff = (out.float() - plain).abs()
        rows = diff.amax(dim=-1)  # [b, hq, s]
        bad = (rows > 2e-2).nonzero().tolist()
        print(f"B{b} Hq{hq} S{s} D{d} rep {rep} layout {lay}: max diff {diff.max().item():.3e}, "
              f"nan {torch.isnan(out).sum().item()}, bad rows {len(bad)}", flush=True)
        if bad:
            runs = {}
            for bb, hh, ss in bad:
                runs.setdefault((bb, hh, ss // 128, (ss % 128) // 32), []).append(ss)
            for key, ss in sorted(runs.items())[:12]:
                print(f"   (b, h, qtile, 32-row block) {key}: rows {min(ss)}..{max(ss)} ({len(ss)})", flush=True)
    _debug.set_split()
