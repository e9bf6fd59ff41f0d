"""Host-side cost per call of the public op vs the bare extension vs a captured HIP graph (GPU box).

usage: python scripts/dev/host_overhead.py"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from flash_attention_cute_amd import flash_attn_func  # noqa: E402
from flash_attention_cute_amd import flash_attention as fam  # noqa: E402

dev = torch.device("cuda:0")


def per_call(fn, n=2000):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6, (time.perf_counter() - t0) / n * 1e6


for name, (b, hq, hkv, sq, sk) in {"tiny decode": (1, 32, 8, 1, 64), "decode B32": (32, 32, 8, 1, 4096)}.items():
    q = torch.randn(b, hq, sq, 128, device=dev, dtype=torch.float16)
    k = torch.randn(b, hkv, sk, 128, device=dev, dtype=torch.float16)
    v = torch.randn(b, hkv, sk, 128, device=dev, dtype=torch.float16)
    s = 128 ** -0.5
    res = {
        "flash_attn_func": per_call(lambda: flash_attn_func(q, k, v)),
        "torch.ops.flash_attention.forward": per_call(lambda: torch.ops.flash_attention.forward(q, k, v, s, False)),
        "extension flash_attention_fwd": per_call(lambda: fam.flash_attention_cuda.flash_attention_fwd(q, k, v, s, False)),
    }
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            flash_attn_func(q, k, v)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        out = flash_attn_func(q, k, v)
    res["hip graph replay"] = per_call(g.replay)
    # GPU-only duration: fill the queue behind a sleep so events see back-to-back kernels
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    torch.cuda._sleep(200_000_000)
    for a, e in ev:
        a.record()
        flash_attn_func(q, k, v)
        e.record()
    torch.cuda.synchronize()
    gpu_us = sum(a.elapsed_time(e) for a, e in ev) / len(ev) * 1e3
    print(f"{name}: GPU kernel {gpu_us:.1f} us/call (queue pre-filled)")
    for k_, (host, wall) in res.items():
        print(f"  {k_:36s} host {host:7.1f} us/call   wall {wall:7.1f} us/call")
