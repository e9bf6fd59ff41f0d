"""GPU helper: padded decode (bench.py decode_padded) at several split targets (the decode plan's
knob), interleaved in one process: GB/s of algorithmic bytes per setting."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from flash_attention_cute_amd import _debug, flash_attn_padded_func  # noqa: E402

c = bench.CONFIGS["decode_padded"]
dev = torch.device("cuda:0")
q = torch.randn(c["B"], c["Hq"], 1, c["D"], device=dev, dtype=torch.bfloat16)
k = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], device=dev, dtype=torch.bfloat16)
v = torch.randn_like(k)
lens = torch.tensor(c["lens"], dtype=torch.int32, device=dev)
ke = torch.full_like(lens, c["Sk"])
ks = ke - lens
targets = [int(x) for x in sys.argv[1:]] or [160, 512, 1024, 2048]
res = {t: [] for t in targets}
ref = None
for rep in range(7):
    for t in targets:
        _debug.set_knobs(dec_target=t)
        for _ in range(20):
            flash_attn_padded_func(q, k, v, ks, ke, causal=True)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(100):
            o = flash_attn_padded_func(q, k, v, ks, ke, causal=True)
        b.record()
        torch.cuda.synchronize()
        res[t].append(bench.algo_bytes(c) / (a.elapsed_time(b) / 100 * 1e-3) / 1e9)
        if ref is None:
            ref = o.float()
        assert (o.float() - ref).abs().max().item() < 2e-2
        path = _debug.last_path()
for t in targets:
    r = sorted(res[t])
    print(f"dec_target {t}: median {r[len(r) // 2]:.0f} GB/s (min {r[0]:.0f} max {r[-1]:.0f}) path {path}")
