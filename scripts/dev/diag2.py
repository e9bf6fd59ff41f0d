"""Error map of the w4 kernel on causal / ragged shapes (rows grouped by 32-row block)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from flash_attention_cute_amd import flash_attn_func  # noqa: E402
from oracle import fa_oracle_c as OC  # noqa: E402

dev = torch.device("cuda:0")
os.environ["FA_GFX950_VARIANT"] = sys.argv[1] if len(sys.argv) > 1 else "w4"
for (sq, sk, causal) in [(64, 64, True), (128, 128, True), (256, 256, True), (300, 300, True), (512, 512, True),
                         (256, 300, False), (100, 333, True), (256, 256, False)]:
    g = torch.Generator().manual_seed(1)
    q = torch.randn(1, 1, sq, 128, generator=g).half()
    k = torch.randn(1, 1, sk, 128, generator=g).half()
    v = torch.randn(1, 1, sk, 128, generator=g).half()
    o = flash_attn_func(q.to(dev), k.to(dev), v.to(dev), causal=causal).float().cpu()
    r = OC.forward(q, k, v, 128 ** -0.5, causal).float()
    e = (o - r).abs()[0, 0].amax(dim=1)
    blocks = [f"{e[i:i + 32].max().item():.0e}" for i in range(0, sq, 32)]
    print((sq, sk, causal), "max", f"{e.max().item():.2e}", " ".join(blocks), flush=True)
