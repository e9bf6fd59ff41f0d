"""The LLM harness (scripts/benchmark_llm.py, reference scripts/benchmark_llm.py:27-118): locally
built configs, prefill + decode timing, patched vs HF attention."""
import importlib.util
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent


def _harness():
    spec = importlib.util.spec_from_file_location("benchmark_llm", ROOT / "scripts" / "benchmark_llm.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["benchmark_llm"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("model", ["llama-tiny", "qwen2-tiny"])
def test_harness_runs_patched_on_cpu(model):
    from flash_attention_cute_amd import hf_attention  # noqa: F401  (patch restored below)
    import transformers.models.llama.modeling_llama as ml
    import transformers.models.qwen2.modeling_qwen2 as mq

    saved = (ml.LlamaAttention.forward, mq.Qwen2Attention.forward)
    try:
        res = _harness().main(["--model", model, "--attn", "custom", "--prompt-len", "24", "--max-new-tokens", "3",
                               "--num-trials", "1", "--num-warmup", "0", "--device", "cpu",
                               "--torch-dtype", "float32"])
    finally:
        ml.LlamaAttention.forward, mq.Qwen2Attention.forward = saved
    assert res["prefill_tokens_per_s"] > 0 and res["decode_tokens_per_s"] > 0
    assert res["layers"] == 2


@pytest.mark.gpu
def test_harness_llama3_layers_on_gpu():
    import transformers.models.llama.modeling_llama as ml

    saved = ml.LlamaAttention.forward
    try:
        res = _harness().main(["--model", "llama3-8b", "--num-layers", "2", "--attn", "custom", "--prompt-len", "512",
                               "--max-new-tokens", "4", "--num-trials", "1", "--device", "cuda"])
    finally:
        ml.LlamaAttention.forward = saved
    assert res["prefill_tokens_per_s"] > 0 and res["decode_tokens_per_s"] > 0
