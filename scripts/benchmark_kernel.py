#!/usr/bin/env python3
"""Kernel benchmark with the reference's CLI (reference scripts/benchmark_kernel.py:15-160):
this op ("custom") vs a library flash attention ("official") vs fp32 eager attention, then MSE and
allclose(atol=1e-3) between them.

The reference's "official" is Dao-AILab flash_attn 2 (CUDA), which does not exist on this machine;
its stand-in is torch.nn.functional.scaled_dot_product_attention on the GPU (PyTorch-ROCm's fused
flash backend), called on the same [B, H, S, D] tensors with ``enable_gqa``. Causal masks follow
each library's convention: this op and the reference are bottom-right aligned, SDPA / eager
top-left, so causal comparisons use Sq == Sk (where both agree).

  python scripts/benchmark_kernel.py --batch-size 16 --num-heads-q 64 --num-heads-kv 8 --seqlen-q 1024 \\
      --seqlen-kv 1024 --dim 128 --dtype half [--causal]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from flash_attention import flash_attn_func as flash_attn_custom  # noqa: E402

torch.set_grad_enabled(False)


def eager_attention(query, key, value, softmax_scale=None, is_causal=False):
    """fp32 eager reference (reference scripts/benchmark_kernel.py:15-43)."""
    scale = 1 / (query.size(-1) ** 0.5) if softmax_scale is None else softmax_scale
    L, S = query.size(-2), key.size(-2)
    dt = query.dtype
    q, k, v = query.float(), key.float(), value.float()
    bias = torch.zeros(L, S, dtype=q.dtype, device=q.device)
    if is_causal:
        bias.masked_fill_(torch.ones(L, S, dtype=torch.bool, device=q.device).tril(0).logical_not(), float("-inf"))
    k = k.repeat_interleave(q.size(-3) // k.size(-3), -3)
    v = v.repeat_interleave(q.size(-3) // v.size(-3), -3)
    w = torch.softmax(torch.matmul(q, k.transpose(-2, -1)) * scale + bias, dim=-1)
    return torch.matmul(w, v).to(dt)


def flash_attention_custom(q, k, v, softmax_scale=None, is_causal=False):
    return flash_attn_custom(q, k, v, softmax_scale=softmax_scale, causal=is_causal)


def flash_attention_official(q, k, v, softmax_scale=None, is_causal=False):
    return torch.nn.functional.scaled_dot_product_attention(q, k, v, scale=softmax_scale, is_causal=is_causal,
                                                            enable_gqa=q.size(1) != k.size(1))


def mse(a, b):
    return torch.mean((a.float() - b.float()) ** 2)


def _time(fn, iters, sync):
    sync()
    t0 = time.time()
    for _ in range(iters):
        fn()
    sync()
    return (time.time() - t0) * 1e3


def run_benchmark(batch_size, num_heads_q, num_heads_kv, seqlen_q, seqlen_kv, dim, iters, is_causal, dtype, device):
    q = torch.randn((batch_size, num_heads_q, seqlen_q, dim), dtype=dtype, device=device)
    k = torch.randn((batch_size, num_heads_kv, seqlen_kv, dim), dtype=dtype, device=device)
    v = torch.randn((batch_size, num_heads_kv, seqlen_kv, dim), dtype=dtype, device=device)
    print("\nBenchmark Configuration:")
    print(f"Batch size: {batch_size}")
    print(f"Query heads: {num_heads_q}, Key/Value heads: {num_heads_kv}")
    print(f"Query length: {seqlen_q}, Key/Value length: {seqlen_kv}")
    print(f"Dimension: {dim}, Causal: {is_causal}")
    print(f"Data type: {dtype}, Device: {device}")
    print(f"Iterations: {iters}\n")
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    flops = 4.0 * batch_size * num_heads_q * seqlen_q * seqlen_kv * dim * (0.5 if is_causal else 1.0)
    res = {}
    print("Running benchmarks...")
    for name, fn in (("Custom", flash_attention_custom), ("Official", flash_attention_official),
                     ("Eager", eager_attention)):
        n = iters if name != "Eager" else max(1, iters // 10)
        fn(q, k, v, is_causal=is_causal)  # warm-up (first-call JIT / autotune of the library)
        ms = _time(lambda: fn(q, k, v, is_causal=is_causal), n, sync)
        res[name] = {"ms_per_iter": ms / n, "tflops": flops / (ms / n * 1e-3) / 1e12}
        print(f"[{name}] Total: {ms:.3f}ms | Per iter: {ms / n:.3f}ms | {res[name]['tflops']:.1f} TFLOPS")

    print("\nChecking accuracy...")
    o_custom = flash_attention_custom(q, k, v, is_causal=is_causal)
    o_official = flash_attention_official(q, k, v, is_causal=is_causal)
    o_eager = eager_attention(q, k, v, is_causal=is_causal)
    acc = {"mse_custom_official": mse(o_custom, o_official).item(), "mse_custom_eager": mse(o_custom, o_eager).item(),
           "allclose_custom_official": bool(torch.allclose(o_custom, o_official, atol=1e-3)),
           "allclose_custom_eager": bool(torch.allclose(o_custom, o_eager, atol=1e-3))}
    print(f"MSE between implementations (custom, official): {acc['mse_custom_official']:.4e}")
    print(f"MSE between implementations (custom, eager): {acc['mse_custom_eager']:.4e}")
    print(f"AllClose check (custom, official): {acc['allclose_custom_official']}")
    print(f"AllClose check (custom, eager): {acc['allclose_custom_eager']}")
    res.update(acc)
    return res


def main(argv=None):
    p = argparse.ArgumentParser(description="Flash Attention Benchmark Tool")
    p.add_argument("--batch-size", type=int, default=16)
    p.add_argument("--num-heads-q", type=int, default=64)
    p.add_argument("--num-heads-kv", type=int, default=8)
    p.add_argument("--seqlen-q", type=int, default=1024)
    p.add_argument("--seqlen-kv", type=int, default=1024)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--iter", type=int, default=100)
    p.add_argument("--dtype", type=str, default="half")
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--causal", action="store_true")
    a = p.parse_args(argv)
    dtype = getattr(torch, a.dtype)
    assert isinstance(dtype, torch.dtype)
    res = run_benchmark(a.batch_size, a.num_heads_q, a.num_heads_kv, a.seqlen_q, a.seqlen_kv, a.dim, a.iter,
                        a.causal, dtype, torch.device(a.device))
    print(json.dumps({"config": vars(a), **res}), flush=True)
    return res


if __name__ == "__main__":
    main()
