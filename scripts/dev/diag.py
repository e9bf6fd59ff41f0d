"""Small GPU diagnostic: error statistics of a few cases vs the oracle (no asserts)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from flash_attention_cute_amd import flash_attn_func  # noqa: E402
from oracle import fa_oracle_c as OC  # noqa: E402

dev = torch.device("cuda:0")
cases = [(1, 1, 1, 32, 64, 128, False), (1, 1, 1, 256, 64, 128, False), (1, 1, 1, 256, 256, 128, False),
         (1, 2, 2, 300, 300, 128, True), (1, 2, 1, 64, 100, 64, False), (1, 8, 2, 1, 257, 128, False)]
for dt in (torch.float16, torch.bfloat16):
    for (b, hq, hkv, sq, sk, d, causal) in cases:
        g = torch.Generator().manual_seed(1)
        q = torch.randn(b, hq, sq, d, generator=g).to(dt)
        k = torch.randn(b, hkv, sk, d, generator=g).to(dt)
        v = torch.randn(b, hkv, sk, d, generator=g).to(dt)
        o = flash_attn_func(q.to(dev), k.to(dev), v.to(dev), causal=causal).float().cpu()
        r = OC.forward(q, k, v, d ** -0.5, causal).float()
        e = (o - r).abs()
        print(dt, (b, hq, hkv, sq, sk, d, causal), "max", f"{e.max().item():.3e}", "mean", f"{e.mean().item():.3e}",
              "worst row", e.amax(dim=(0, 1, 3)).argmax().item(), "worst col", e.amax(dim=(0, 1, 2)).argmax().item(),
              "nan", torch.isnan(o).sum().item(), flush=True)
