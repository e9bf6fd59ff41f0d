"""The HF attention monkey-patches (reference models/patch_{llama,qwen2}.py, models/rope_attn_fwd.py).

CPU tests run the patched forward through the op's CPU default (torch SDPA, exactly as the
reference's op does on CPU) and compare against the unpatched transformers attention; they pin the
three fixes of SURVEY.md 3.2 (sliding-window attribute, ``past_key_values`` name, decode causal
flag). GPU tests compare the patched layer / model on the gfx950 kernel against unpatched
transformers (SDPA) on the same device.
"""
from __future__ import annotations

import copy
import warnings

import pytest
import torch

transformers = pytest.importorskip("transformers")
from transformers import DynamicCache, LlamaConfig, Qwen2Config  # noqa: E402
from transformers.models.llama import modeling_llama as ml  # noqa: E402
from transformers.models.qwen2 import modeling_qwen2 as mq  # noqa: E402

from flash_attention_cute_amd import hf_attention  # noqa: E402


def tiny_llama(hq=4, hkv=4, d=32, layers=2):
    return LlamaConfig(hidden_size=hq * d, intermediate_size=2 * hq * d, num_attention_heads=hq,
                       num_key_value_heads=hkv, head_dim=d, num_hidden_layers=layers, vocab_size=97,
                       max_position_embeddings=512, rope_theta=5e5, attn_implementation="sdpa")


def tiny_qwen2(hq=4, hkv=4, d=32, layers=2):
    return Qwen2Config(hidden_size=hq * d, intermediate_size=2 * hq * d, num_attention_heads=hq,
                       num_key_value_heads=hkv, num_hidden_layers=layers, vocab_size=97,
                       max_position_embeddings=512, attn_implementation="sdpa")


class patched:
    """Context manager: swap ``cls.forward`` for the gfx950 attention forward, restore on exit."""

    def __init__(self, cls):
        self.cls = cls

    def __enter__(self):
        self.orig = self.cls.forward
        self.cls.forward = hf_attention.attention_forward

    def __exit__(self, *exc):
        self.cls.forward = self.orig


def run_layer(attn_cls, cfg, dev, dtype, seqs=(7, 1, 1), patch=False, seed=0):
    """Prefill seqs[0] tokens, then decode the rest one step at a time, through a DynamicCache."""
    torch.manual_seed(seed)
    layer = attn_cls(cfg, layer_idx=0).to(dev, dtype).eval()
    rope = (ml.LlamaRotaryEmbedding if attn_cls is ml.LlamaAttention else mq.Qwen2RotaryEmbedding)(cfg).to(dev)
    cache = DynamicCache(config=cfg)
    total = sum(seqs)
    x = torch.randn(2, total, cfg.hidden_size, device=dev, dtype=dtype)
    outs, pos = [], 0
    paths = []  # kernel launched per step (patched GPU runs): flash_attention_cute_amd._debug
    ctx = patched(attn_cls) if patch else _null()
    with ctx, torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for s in seqs:
            pid = torch.arange(pos, pos + s, device=dev)[None].expand(2, -1)
            pe = rope(x, pid)
            # unpatched HF builds no mask for SDPA here; pass is_causal through the module
            o, _ = layer(x[:, pos:pos + s], position_embeddings=pe, attention_mask=None, past_key_values=cache,
                         cache_position=pid[0])
            outs.append(o)
            if patch and torch.device(dev).type == "cuda":
                from flash_attention_cute_amd import _debug

                paths.append(_debug.last_path())
            pos += s
    out = torch.cat(outs, dim=1)
    run_layer.paths = paths
    return out


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


# ------------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("attn_cls,mk", [(ml.LlamaAttention, tiny_llama), (mq.Qwen2Attention, tiny_qwen2)])
def test_patch_prefill_and_decode_match_hf_on_cpu(attn_cls, mk):
    cfg = mk()
    ref = run_layer(attn_cls, cfg, "cpu", torch.float32, patch=False)
    got = run_layer(attn_cls, cfg, "cpu", torch.float32, patch=True)
    # prefill rows equal SDPA exactly up to fp32 op-order; decode rows see the whole cache
    torch.testing.assert_close(got, ref, atol=2e-5, rtol=1e-4)


def test_llama_config_without_use_sliding_window_does_not_crash():
    cfg = tiny_llama()
    assert not hasattr(cfg, "use_sliding_window")  # the attribute the reference reads (rope_attn_fwd.py:97)
    run_layer(ml.LlamaAttention, cfg, "cpu", torch.float32, seqs=(5,), patch=True)


def test_past_key_value_singular_name_is_accepted():
    cfg = tiny_llama()
    torch.manual_seed(0)
    layer = ml.LlamaAttention(cfg, layer_idx=0).eval()
    rope = ml.LlamaRotaryEmbedding(cfg)
    x = torch.randn(1, 4, cfg.hidden_size)
    pid = torch.arange(4)[None]
    c1, c2 = DynamicCache(config=cfg), DynamicCache(config=cfg)
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a, _ = hf_attention.attention_forward(layer, x, rope(x, pid), None, past_key_value=c1)
        b, _ = hf_attention.attention_forward(layer, x, rope(x, pid), None, past_key_values=c2)
    assert torch.equal(a, b)
    assert c1.get_seq_length() == 4 and c2.get_seq_length() == 4


def test_decode_step_sees_whole_cache_on_cpu():
    """Reference bug 3: Sq == 1 with is_causal must attend to every cached key."""
    cfg = tiny_llama()
    ref = run_layer(ml.LlamaAttention, cfg, "cpu", torch.float32, seqs=(6, 1), patch=False)
    got = run_layer(ml.LlamaAttention, cfg, "cpu", torch.float32, seqs=(6, 1), patch=True)
    torch.testing.assert_close(got[:, -1], ref[:, -1], atol=2e-5, rtol=1e-4)


def window_mask4(b, s, pos, w):
    """HF's 4-D SDPA mask [B, 1, s, pos + s] of a sliding-window causal layer (True = attend) for s new
    tokens at positions pos.. (transformers sliding_window_causal_mask_function: p - w < n <= p)."""
    p_ = torch.arange(pos, pos + s)[:, None]
    n = torch.arange(pos + s)[None, :]
    return ((n <= p_) & (n > p_ - w))[None, None].expand(b, 1, s, pos + s)


def run_window_layer(cfg, dev, dtype, seqs, w, patch, seed=0):
    """A Qwen2 sliding-window layer (use_sliding_window, window w) through a DynamicCache, with the 4-D
    sliding-window mask HF builds for SDPA passed to both the patched and the unpatched forward."""
    torch.manual_seed(seed)
    layer = mq.Qwen2Attention(cfg, layer_idx=0).to(dev, dtype).eval()
    rope = mq.Qwen2RotaryEmbedding(cfg).to(dev)
    # a cache that keeps every key (no sliding-window truncation), so the mask spans pos + s keys and
    # the window itself is what hides the old ones
    cache = DynamicCache()
    x = torch.randn(2, sum(seqs), cfg.hidden_size, device=dev, dtype=dtype)
    outs, pos = [], 0
    ctx = patched(mq.Qwen2Attention) if patch else _null()
    with ctx, torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for s in seqs:
            pid = torch.arange(pos, pos + s, device=dev)[None].expand(2, -1)
            mask = window_mask4(2, s, pos, w).to(dev)
            o, _ = layer(x[:, pos:pos + s], position_embeddings=rope(x, pid), attention_mask=mask,
                         past_key_values=cache, cache_position=pid[0])
            outs.append(o)
            pos += s
    return torch.cat(outs, dim=1)


def sliding_qwen2(w, **kw):
    cfg = tiny_qwen2(**kw)
    cfg.use_sliding_window = True
    cfg.sliding_window = w
    cfg.max_window_layers = 0
    cfg.layer_types = ["sliding_attention"] * cfg.num_hidden_layers
    return cfg


def test_active_sliding_window_runs_the_window_op_not_ignored():
    """Reference models/rope_attn_fwd.py:95-101 computes the window and ignores it; the patch runs the
    local-window op: same output as unpatched HF under HF's own sliding-window mask (prefill longer
    than the window, then decode steps past it)."""
    cfg = sliding_qwen2(4)
    ref = run_window_layer(cfg, "cpu", torch.float32, (9, 1, 1), 4, patch=False)
    got = run_window_layer(cfg, "cpu", torch.float32, (9, 1, 1), 4, patch=True)
    torch.testing.assert_close(got, ref, atol=2e-5, rtol=1e-4)
    # the window matters here: plain causal attention over the same tokens differs
    full = run_layer(mq.Qwen2Attention, tiny_qwen2(), "cpu", torch.float32, seqs=(9, 1, 1), patch=True)
    assert not torch.allclose(full, got, atol=1e-3)


def padded_window_mask4(valid, s, pos, w):
    """HF's 4-D SDPA mask of a sliding-window layer over a padded batch: the window on cache indices
    (p - w < n <= p) AND the key is a real token."""
    return window_mask4(valid.shape[0], s, pos, w).to(valid.device) & valid[:, None, None, :pos + s]


def test_sliding_window_over_a_padded_batch_on_cpu():
    """Left-padded batch through a Qwen2 sliding-window layer (window 4): the patch lowers the mask to
    the varlen op with the window per sequence; real tokens match unpatched HF (prefill + decode)."""
    from flash_attention_cute_amd import hf_attention as hfa

    cfg = sliding_qwen2(4, hq=4, hkv=2)
    torch.manual_seed(0)
    layer = mq.Qwen2Attention(cfg, layer_idx=0).eval()
    rope = mq.Qwen2RotaryEmbedding(cfg)
    lens, s = [9, 5, 7], 9
    valid = torch.zeros(3, s + 1, dtype=torch.bool)
    for b, n in enumerate(lens):
        valid[b, s - n:] = True
    valid[:, s] = True
    x = torch.randn(3, s + 1, cfg.hidden_size)
    pid = (valid.long().cumsum(1) - 1).clamp(min=0)
    outs = {}
    for patch in (False, True):
        cache = DynamicCache()
        with torch.no_grad(), warnings.catch_warnings(), (patched(mq.Qwen2Attention) if patch else _null()):
            warnings.simplefilter("ignore")
            a, _ = layer(x[:, :s], position_embeddings=rope(x, pid[:, :s]),
                         attention_mask=padded_window_mask4(valid, s, 0, 4), past_key_values=cache)
            d, _ = layer(x[:, s:], position_embeddings=rope(x, pid[:, s:]),
                         attention_mask=padded_window_mask4(valid, 1, s, 4), past_key_values=cache)
        outs[patch] = (a, d)
    real = valid[:, :s]
    torch.testing.assert_close(outs[True][0][real], outs[False][0][real], atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(outs[True][1], outs[False][1], atol=2e-5, rtol=1e-4)
    # the lowering: padding found, the window accepted; a window the caller did not declare raises
    assert torch.equal(hfa.key_padding(padded_window_mask4(valid, s, 0, 4), s, s, True, 3), valid[:, :s])
    with pytest.raises(NotImplementedError, match="only causal"):
        hfa.key_padding(padded_window_mask4(valid, s, 0, 4), s, s, True, None)
    # padding inside a sequence: cache-index and packed-token windows differ -> rejected
    holes = valid.clone()
    holes[0, 4] = False
    with pytest.raises(NotImplementedError, match="contiguous"):
        hfa.key_padding(padded_window_mask4(holes, s, 0, 4), s, s, True, 3)


def test_patch_attn_entry_points_swap_forward():
    from models import patch_llama, patch_qwen2

    o1, o2 = ml.LlamaAttention.forward, mq.Qwen2Attention.forward
    try:
        patch_llama.patch_attn()
        patch_qwen2.patch_attn()
        assert ml.LlamaAttention.forward is hf_attention.attention_forward
        assert mq.Qwen2Attention.forward is hf_attention.attention_forward
    finally:
        ml.LlamaAttention.forward, mq.Qwen2Attention.forward = o1, o2


# ------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("attn_cls,mk", [(ml.LlamaAttention, tiny_llama), (mq.Qwen2Attention, tiny_qwen2)])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_patch_gqa_layer_matches_hf_on_gpu(device, attn_cls, mk, dtype):
    cfg = mk(hq=8, hkv=2, d=128)
    seqs = (300, 1, 1, 37)  # prefill, two decode steps (q-head pack), a chunk with Sq < Sk
    from flash_attention_cute_amd import _debug

    _debug.set_knobs()  # product defaults
    ref = run_layer(attn_cls, cfg, device, torch.float32, seqs=seqs, patch=False)
    got = run_layer(attn_cls, cfg, device, dtype, seqs=seqs, patch=True)
    # prefill on the pipelined w4 kernel; the Sq == 1 steps on the decode kernel; the 37-row chunk
    # (4 q-heads x 37 rows > 64) on w4
    assert run_layer.paths[0] == "w4" and run_layer.paths[3] == "w4", run_layer.paths
    assert all(p_ in ("decode", "decode_split") for p_ in run_layer.paths[1:3]), run_layer.paths
    # the last chunk (Sq < Sk): unpatched HF SDPA with attention_mask=None uses is_causal only when
    # q_len > 1 and Sq == Sk; compare prefill + decode rows, and the chunk against a bottom-right ref
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    n = seqs[0] + seqs[1] + seqs[2]
    torch.testing.assert_close(got[:, :n].float(), ref[:, :n], atol=tol, rtol=0)


@pytest.mark.gpu
def test_patched_llama_model_generates_same_tokens_as_hf(device):
    cfg = tiny_llama(hq=8, hkv=2, d=128, layers=2)
    torch.manual_seed(0)
    model = transformers.LlamaForCausalLM(cfg).to(device, torch.bfloat16).eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 64), device=device)
    with torch.no_grad():
        ref = model(ids).logits.float()
        with patched(ml.LlamaAttention):
            got = model(ids).logits.float()
    assert (got - ref).abs().max().item() < 5e-2
    assert (got.argmax(-1) == ref.argmax(-1)).float().mean().item() > 0.95


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_patch_sliding_window_layer_matches_hf_on_gpu(device, dtype):
    """Qwen2 sliding-window layer (window 128) on the GPU: a 300-token prefill (the window kernel)
    and decode steps past the window (keys cut, decode kernel), against unpatched HF in fp32 under
    HF's own sliding-window mask."""
    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    cfg = sliding_qwen2(128, hq=8, hkv=2, d=128)
    seqs = (300, 1, 1)
    ref = run_window_layer(cfg, device, torch.float32, seqs, 128, patch=False)
    got = run_window_layer(cfg, device, dtype, seqs, 128, patch=True)
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    torch.testing.assert_close(got.float(), ref, atol=tol, rtol=0)
