#!/usr/bin/env python3
"""Prefill / decode throughput of an HF causal LM with the gfx950 attention patch vs HF's own
attention -- the reference's LLM harness (reference scripts/benchmark_llm.py:27-118, ``run_perf``)
restated for this machine: no hub download (no network), so the model is built from a local
config with random seeded weights and the prompt is synthetic token ids of the requested length.

  python scripts/benchmark_llm.py --model llama3-8b --attn custom --prompt-len 4096 --max-new-tokens 64
  python scripts/benchmark_llm.py --model qwen2-7b --attn sdpa --num-layers 4

--attn custom patches ``LlamaAttention.forward`` / ``Qwen2Attention.forward`` with
models/patch_{llama,qwen2}.patch_attn (the reference's ``--attn custom``); any other value is passed
to HF as ``attn_implementation`` (sdpa, eager). Timing follows the reference: prefill = mean of
``num_trials`` full-prompt forwards with ``use_cache=True``; decode = mean per-token time of greedy
steps on the prefill's KV cache. Prints the reference's two lines plus one JSON summary line.
Random weights make the generated tokens meaningless; throughput is what is measured.
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

# Local configs: the published layer dimensions of the models the reference benchmarks
# (reference README / scripts/benchmark_llm.py --model), built without the hub.
MODELS = {
    "llama3-8b": ("llama", dict(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                                num_key_value_heads=8, num_hidden_layers=32, vocab_size=128256,
                                rope_theta=500000.0, max_position_embeddings=8192, rms_norm_eps=1e-5)),
    "qwen2-7b": ("qwen2", dict(hidden_size=3584, intermediate_size=18944, num_attention_heads=28,
                               num_key_value_heads=4, num_hidden_layers=28, vocab_size=152064,
                               rope_theta=1000000.0, max_position_embeddings=32768, rms_norm_eps=1e-6)),
    # small shapes for CPU tests / smoke runs (MHA: the op's CPU default, torch SDPA, has no GQA --
    # reference flash_attention/flash_attention.py:6-15)
    "llama-tiny": ("llama", dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                                 num_key_value_heads=4, num_hidden_layers=2, vocab_size=1000,
                                 rope_theta=10000.0, max_position_embeddings=2048)),
    "qwen2-tiny": ("qwen2", dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                                 num_key_value_heads=4, num_hidden_layers=2, vocab_size=1000,
                                 rope_theta=10000.0, max_position_embeddings=2048)),
}


def build_model(name: str, attn: str, dtype: torch.dtype, device: torch.device, num_layers: int | None,
                seed: int = 0):
    import transformers

    family, kw = MODELS[name]
    kw = dict(kw)
    if num_layers:
        kw["num_hidden_layers"] = num_layers
    impl = "eager" if attn == "custom" else attn
    if family == "llama":
        cfg = transformers.LlamaConfig(**kw, attn_implementation=impl)
        cls = transformers.LlamaForCausalLM
    else:
        cfg = transformers.Qwen2Config(**kw, attn_implementation=impl, use_sliding_window=False)
        cls = transformers.Qwen2ForCausalLM
    torch.manual_seed(seed)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        with torch.device(device):  # weights initialised in place (no host copy of 8B params)
            model = cls(cfg)
    finally:
        torch.set_default_dtype(prev)
    model.eval()
    if attn == "custom":
        if family == "llama":
            from models.patch_llama import patch_attn
        else:
            from models.patch_qwen2 import patch_attn
        patch_attn()
    return model, cfg


class _Timer:
    """CUDA events on a GPU, perf_counter on CPU (the reference times with CUDA events)."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"

    def __enter__(self):
        if self.cuda:
            torch.cuda.synchronize()
            self.a, self.b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            self.a.record()
        else:
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            self.b.record()
            torch.cuda.synchronize()
            self.s = self.a.elapsed_time(self.b) / 1000
        else:
            self.s = time.perf_counter() - self.t0


def run_perf(model, input_ids, max_new_tokens: int, num_trials: int, num_warmup: int) -> dict:
    """reference scripts/benchmark_llm.py:27-96 (run_perf), same measurement order."""
    device = input_ids.device
    seq_len = input_ids.shape[1]
    with torch.no_grad():
        for _ in range(num_warmup):
            model(input_ids, use_cache=True)
        pre = []
        for _ in range(num_trials):
            with _Timer(device) as t:
                model(input_ids, use_cache=True)
            pre.append(t.s)
        prefill_s = sum(pre) / len(pre)
        print(f"[Prefill] Throughput: {seq_len * input_ids.shape[0] / prefill_s:.2f} tokens/s | SeqLen: {seq_len} "
              f"| AvgTime: {prefill_s:.4f}s")

        total, steps = 0.0, 0
        for _ in range(num_trials):
            out = model(input_ids, use_cache=True, return_dict=True)
            past = out.past_key_values
            nxt = out.logits[:, -1, :].argmax(dim=-1).unsqueeze(-1)
            for _ in range(max_new_tokens):
                with _Timer(device) as t:
                    out = model(nxt, past_key_values=past, use_cache=True)
                past = out.past_key_values
                nxt = out.logits[:, -1, :].argmax(dim=-1).unsqueeze(-1)
                total += t.s
                steps += 1
        decode_s = total / max(steps, 1)
        print(f"[Decode ] Throughput: {input_ids.shape[0] / decode_s:.2f} tokens/s | AvgTime: {decode_s * 1000:.2f}ms/token")
    return {"prefill_s": prefill_s, "prefill_tokens_per_s": seq_len * input_ids.shape[0] / prefill_s,
            "decode_ms_per_token": decode_s * 1000, "decode_tokens_per_s": input_ids.shape[0] / decode_s}


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model", default="llama3-8b", choices=sorted(MODELS))
    ap.add_argument("--attn", default="custom", help="custom (the gfx950 patch) | sdpa | eager")
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--max-new-tokens", type=int, default=64)
    ap.add_argument("--num-trials", type=int, default=3)
    ap.add_argument("--num-warmup", type=int, default=1)
    ap.add_argument("--num-layers", type=int, default=None, help="override the layer count (quick runs)")
    ap.add_argument("--torch-dtype", default="bfloat16", choices=["bfloat16", "float16", "float32"])
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    args = ap.parse_args(argv)

    device = torch.device(args.device)
    dtype = getattr(torch, args.torch_dtype)
    model, cfg = build_model(args.model, args.attn, dtype, device, args.num_layers)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (args.batch, args.prompt_len), generator=g).to(device)
    res = run_perf(model, ids, args.max_new_tokens, args.num_trials, args.num_warmup)
    res.update({"model": args.model, "attn": args.attn, "layers": cfg.num_hidden_layers, "dtype": args.torch_dtype,
                "batch": args.batch, "prompt_len": args.prompt_len, "max_new_tokens": args.max_new_tokens,
                "device": str(device), "weights": "random (seeded), local config"})
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
