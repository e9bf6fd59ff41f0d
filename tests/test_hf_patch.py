"""The HF attention monkey-patches (reference models/patch_{llama,qwen2}.py, models/rope_attn_fwd.py).

CPU tests run the patched forward through the op's CPU default (torch SDPA, exactly as the
reference's op does on CPU) and compare against the unpatched transformers attention; they pin the
three fixes of SURVEY.md 3.2 (sliding-window attribute, ``past_key_values`` name, decode causal
flag). GPU tests compare the patched layer / model on the gfx950 kernel against unpatched
transformers (SDPA) on the same device.
"""
from __future__ import annotations

import copy
import sys
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


def bottom_right_mask4(b, s, pos, dev):
    """[B, 1, s, pos + s] bool (True = attend): s new tokens at positions pos.. see every key up to
    their own position -- the kernel's bottom-right causal alignment (reference csrc/mask.cuh:37-39)
    written as the explicit mask an unpatched HF layer honours."""
    p_ = torch.arange(pos, pos + s, device=dev)[:, None]
    n = torch.arange(pos + s, device=dev)[None, :]
    return (n <= p_)[None, None].expand(b, 1, s, pos + s)


def run_layer(attn_cls, cfg, dev, dtype, seqs=(7, 1, 1), patch=False, seed=0, explicit_mask=False):
    """Prefill seqs[0] tokens, then decode the rest one step at a time, through a DynamicCache.
    explicit_mask: pass the bottom-right causal mask of every step (unpatched reference runs of steps
    with Sq < Sk, where HF's mask-free SDPA call would be top-left causal)."""
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
            mask = bottom_right_mask4(2, s, pos, dev) if explicit_mask else None
            o, _ = layer(x[:, pos:pos + s], position_embeddings=pe, attention_mask=mask, past_key_values=cache,
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
    # the reference: unpatched transformers in fp32 with the bottom-right causal mask written out, so
    # the Sq < Sk chunk is compared too (mask-free SDPA would be top-left causal there)
    ref = run_layer(attn_cls, cfg, device, torch.float32, seqs=seqs, patch=False, explicit_mask=True)
    got = run_layer(attn_cls, cfg, device, dtype, seqs=seqs, patch=True)
    # prefill on the pipelined w4 kernel; the Sq == 1 steps on the decode kernel; the 37-row chunk
    # (4 q-heads x 37 rows > 64) on w4
    assert run_layer.paths[0] == "w4" and run_layer.paths[3] == "w4", run_layer.paths
    assert all(p_ in ("decode", "decode_split") for p_ in run_layer.paths[1:3]), run_layer.paths
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    assert got.shape[1] == sum(seqs)
    torch.testing.assert_close(got.float(), ref, atol=tol, rtol=0)  # every row, the chunk included


def greedy_margins(model, seq, n_prompt, mask):
    """Top-1 minus top-2 logit (fp32 model) at every generated position of ``seq``: how far each greedy
    choice is from a tie."""
    full = torch.cat([mask, torch.ones_like(seq[:, n_prompt:])], dim=1)
    pid = (full.long().cumsum(1) - 1).clamp(min=0)
    with torch.no_grad():
        logits = model(seq, attention_mask=full, position_ids=pid).logits.float()[:, n_prompt - 1:-1]
    top2 = logits.topk(2, dim=-1).values
    return (top2[..., 0] - top2[..., 1])


def tiny_generator(device, padded):
    """A 2-layer GQA Llama (Hq 8, Hkv 2, D 128; seeded random weights, initializer_range 0.3 so the
    logits spread over several units) and a 48-token prompt batch of 2 (row 1 left-padded by 17),
    generated on ``device``."""
    cfg = tiny_llama(hq=8, hkv=2, d=128, layers=2)
    cfg.initializer_range = 0.3
    # seed 8: on MI355X the fp32 greedy trajectory's top-2 margins are >= 0.15 for both prompts and
    # unpatched fp16 reproduces it (scripts/experiments/gen_seed_search.py, profiles/r3_gen_seed.log)
    torch.manual_seed(8)
    model = transformers.LlamaForCausalLM(cfg).to(device).eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 48), device=device)
    mask = torch.ones_like(ids)
    if padded:
        mask[1, :17] = 0
        ids[1, :17] = 0
    return model, ids, mask


@pytest.mark.gpu
@pytest.mark.parametrize("padded", [False, True], ids=["dense", "left_padded"])
def test_patched_llama_greedy_generate_matches_hf_fp16(device, padded):
    """Greedy ``generate`` of 24 tokens through a DynamicCache in fp16 (prefill + 23 decode steps on the
    split-KV kernel; with left padding, the padded path in place): the patched model produces exactly
    the token ids of unpatched transformers (SDPA) in fp16 and of the fp32 model. Premise, checked: the
    fp32 greedy trajectory has a top-2 logit margin >= 0.1 at every step, far above fp16 error."""
    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    model, ids, mask = tiny_generator(device, padded)
    kw = dict(attention_mask=mask, max_new_tokens=24, do_sample=False, pad_token_id=0)
    with torch.no_grad():
        ref32 = model.generate(ids, **kw)
    margins = greedy_margins(model, ref32, ids.shape[1], mask)
    assert margins.min().item() >= 0.1, margins.min().item()  # the premise
    model = model.half()
    with torch.no_grad():
        ref = model.generate(ids, **kw)
        with patched(ml.LlamaAttention):
            got = model.generate(ids, **kw)
    assert got.shape == (2, 48 + 24)
    assert torch.equal(got, ref), (got[:, 48:], ref[:, 48:])
    assert torch.equal(got, ref32), (got[:, 48:], ref32[:, 48:])


def teacher_forced_decode(model, seq, mask, n_prompt, patch):
    """Logits of every generated position of ``seq``: prefill of the prompt, then one decode step per
    token of ``seq`` through a DynamicCache (the decode path), fp32 copies."""
    full = torch.cat([mask, torch.ones_like(seq[:, n_prompt:])], dim=1)
    pid = (full.long().cumsum(1) - 1).clamp(min=0)
    cache = DynamicCache()
    outs = []
    with torch.no_grad(), warnings.catch_warnings(), (patched(ml.LlamaAttention) if patch else _null()):
        warnings.simplefilter("ignore")
        o = model(seq[:, :n_prompt], attention_mask=full[:, :n_prompt], position_ids=pid[:, :n_prompt],
                  past_key_values=cache, use_cache=True)
        outs.append(o.logits[:, -1].float())
        for t in range(n_prompt, seq.shape[1] - 1):
            o = model(seq[:, t:t + 1], attention_mask=full[:, :t + 1], position_ids=pid[:, t:t + 1],
                      past_key_values=cache, use_cache=True)
            outs.append(o.logits[:, -1].float())
    return torch.stack(outs, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("padded", [False, True], ids=["dense", "left_padded"])
def test_patched_llama_decode_logits_bf16_bar(device, padded):
    """bf16: greedy token ids are not a stable bar here (unpatched HF bf16 itself departs from the fp32
    trajectory), so the bar is BASELINE.md's: teacher-forced along the fp32 greedy trajectory (prefill,
    then 23 single-token decode steps through a DynamicCache -- the split-KV kernel, padded path with
    left padding), the patched model's logits stay within 2x the error of unpatched transformers bf16
    against fp32 (max and mean), and its greedy choice agrees with fp32 at least as often."""
    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    model, ids, mask = tiny_generator(device, padded)
    with torch.no_grad():
        seq = model.generate(ids, attention_mask=mask, max_new_tokens=24, do_sample=False, pad_token_id=0)
    l32 = teacher_forced_decode(model, seq, mask, 48, patch=False)
    model = model.to(torch.bfloat16)
    lhf = teacher_forced_decode(model, seq, mask, 48, patch=False)
    lgot = teacher_forced_decode(model, seq, mask, 48, patch=True)
    assert _debug.last_path() in ("decode", "decode_split"), _debug.last_path()
    e_hf, e_got = (lhf - l32).abs(), (lgot - l32).abs()
    assert e_got.max().item() <= 2 * e_hf.max().item(), (e_got.max().item(), e_hf.max().item())
    assert e_got.mean().item() <= 2 * e_hf.mean().item(), (e_got.mean().item(), e_hf.mean().item())
    tok32 = l32.argmax(-1)
    agree_got = (lgot.argmax(-1) == tok32).float().mean().item()
    agree_hf = (lhf.argmax(-1) == tok32).float().mean().item()
    assert agree_got >= agree_hf - 0.05, (agree_got, agree_hf)


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


# ---- masks lowered on the device: static caches, graph capture ----------
def _generate_tokens(model, ids, mask, patch, **kw):
    with torch.no_grad(), warnings.catch_warnings(), (patched(ml.LlamaAttention) if patch else _null()):
        warnings.simplefilter("ignore")
        return model.generate(ids, attention_mask=mask, do_sample=False, pad_token_id=0, **kw)


@pytest.mark.parametrize("cache", ["dynamic", "static"])
def test_patched_generate_with_left_padding_matches_hf_on_cpu(cache):
    """Left-padded greedy generate through a DynamicCache and a StaticCache (whose keys past the current
    position are empty slots the 4-D mask hides: the query rows sit mid-way through the keys) gives the
    token ids of unpatched transformers."""
    cfg = tiny_llama(hq=4, hkv=2, d=32)
    torch.manual_seed(0)
    model = transformers.LlamaForCausalLM(cfg).eval()
    ids = torch.randint(1, cfg.vocab_size, (3, 12))
    mask = torch.ones_like(ids)
    mask[1, :5] = 0
    mask[2, :11] = 0
    ids[mask == 0] = 0
    kw = dict(max_new_tokens=6, cache_implementation=cache)
    assert torch.equal(_generate_tokens(model, ids, mask, True, **kw), _generate_tokens(model, ids, mask, False, **kw))


def _static_masks(valid, pos, s, total):
    """HF's 4-D SDPA mask of s new tokens at positions pos.. over a static cache of ``total`` slots."""
    p_ = torch.arange(pos, pos + s)[:, None]
    n = torch.arange(total)[None, :]
    return ((n <= p_)[None] & valid[:, None, :total])[:, None]


def test_lower_mask_static_cache_and_padding_kinds():
    from flash_attention_cute_amd.hf_attention import lower_mask

    total = 10
    valid = torch.zeros(3, total, dtype=torch.bool)
    valid[0, :7] = True          # no padding, 7 tokens so far
    valid[1, 3:7] = True         # left padding
    valid[2, :7] = True
    valid[2, 4] = False          # a hole
    low = lower_mask(_static_masks(valid, 0, 7, total)[:, :, :7], 7, total, True)  # prefill rows 0..6
    # (row 2: six real tokens, not one run -- its ranges are not used, the varlen path packs it)
    assert low.k_start.tolist() == [0, 3, 0] and low.k_end.tolist() == [7, 7, 6]
    assert low.q_start.tolist() == [0, 3, 0] and low.q_end.tolist() == [7, 7, 6]
    assert low.shape_ok.tolist() == [True, True, True] and low.run_ok.tolist() == [True, True, False]
    assert not bool(low.dense)  # the static cache's empty slots are hidden: not the dense kernel
    dec = lower_mask(_static_masks(valid, 6, 1, total), 1, total, False)  # decode at position 6
    assert dec.k_start.tolist() == [0, 3, 0] and dec.k_end.tolist() == [7, 7, 6]
    assert dec.run_ok.tolist() == [True, True, False]
    # a document (block-diagonal) mask is not causal + padding
    doc = _static_masks(torch.ones(1, total, dtype=torch.bool), 0, 7, total)[:, :, :7].clone()
    doc[0, 0, 4:, :4] = False
    assert lower_mask(doc, 7, total, True).shape_ok.tolist() == [False]


def test_lower_mask_unmasked_left_padding_rows():
    """transformers / torch "unmask" query rows that attend nothing (left padding) to attend EVERY key.
    Such a row must not set the causal offset (it made the padding row the only valid
    query and zeroed the real rows); a real row left out of the query range is rejected, not zeroed."""
    from flash_attention_cute_amd.hf_attention import lower_mask

    sq = sk = 8
    valid = torch.zeros(2, sk, dtype=torch.bool)
    valid[0, 3:] = True  # three left-padding tokens
    valid[1, :] = True
    m = _static_masks(valid, 0, sq, sk).clone()  # [B, 1, Sq, Sk], dynamic-cache prefill
    m[0, 0, :3, :] = True  # the padding rows unmasked
    low = lower_mask(m, sq, sk, True)
    assert low.q_start.tolist() == [3, 0] and low.q_end.tolist() == [8, 8]
    assert low.k_start.tolist() == [3, 0] and low.k_end.tolist() == [8, 8]
    assert low.shape_ok.tolist() == [True, True] and low.run_ok.tolist() == [True, True]
    # the additive float form of the same mask
    lowf = lower_mask(torch.where(m, 0.0, float("-inf")), sq, sk, True)
    assert lowf.q_start.tolist() == [3, 0] and lowf.shape_ok.tolist() == [True, True]
    # every row unmasked (a sequence of padding only, but its last token): only the last row is real
    m2 = torch.ones(1, 1, sq, sk, dtype=torch.bool)
    low2 = lower_mask(m2, sq, sk, True)
    assert low2.q_start.tolist() == [7] and low2.q_end.tolist() == [8]
    # a real row that hides its own key (not causal + padding) is rejected instead of being dropped
    m3 = _static_masks(torch.ones(1, sk, dtype=torch.bool), 0, sq, sk).clone()
    m3[0, 0, 5, 5] = False
    assert lower_mask(m3, sq, sk, True).shape_ok.tolist() == [False]


def test_eager_padded_forward_reads_the_host_once_per_forward(monkeypatch):
    """the layers of one forward share the lowering of their (identical) mask,
    so an eager left-padded forward through a 4-layer model does ONE host read, not one per layer; a new
    mask (or an in-place change) is lowered again."""
    cfg = tiny_llama(hq=4, hkv=2, d=32, layers=4)
    torch.manual_seed(0)
    model = transformers.LlamaForCausalLM(cfg).eval()
    ids = torch.randint(1, cfg.vocab_size, (2, 9))
    mask = torch.ones_like(ids)
    mask[1, :4] = 0
    reads = []  # host reads made by the attention patch (transformers' own code makes others)
    orig = torch.Tensor.tolist

    def counted(self):
        if sys._getframe(1).f_code.co_filename.endswith("hf_attention.py"):
            reads.append(1)
        return orig(self)

    monkeypatch.setattr(torch.Tensor, "tolist", counted)
    lowers = []
    monkeypatch.setattr(hf_attention, "lower_mask", lambda *a, _f=hf_attention.lower_mask: (lowers.append(1), _f(*a))[1])
    hf_attention._LOWER_MEMO[0] = None
    with torch.no_grad(), warnings.catch_warnings(), patched(ml.LlamaAttention):
        warnings.simplefilter("ignore")
        out = model(ids, attention_mask=mask).logits
        assert len(reads) == 1 and len(lowers) == 1
        model(ids, attention_mask=mask)
        assert len(reads) == 2 and len(lowers) == 2  # (a new forward builds a new mask tensor)
    ref = model(ids, attention_mask=mask).logits
    assert torch.allclose(out[1, 4:], ref[1, 4:], atol=1e-4, rtol=1e-4) and torch.allclose(out[0], ref[0], atol=1e-4)


class _NoHostReads:
    """Any read-back of a tensor value on the host (item / tolist / bool / int) raises."""

    NAMES = ("item", "tolist", "__bool__", "__int__", "__index__")

    def __enter__(self):
        self.saved = {n: getattr(torch.Tensor, n) for n in self.NAMES}
        for n in self.NAMES:
            setattr(torch.Tensor, n, lambda *a, _n=n, **k: (_ for _ in ()).throw(AssertionError(f"host read {_n}")))

    def __exit__(self, *exc):
        for n, f in self.saved.items():
            setattr(torch.Tensor, n, f)


def test_lowering_under_capture_reads_nothing_back_and_counts_bad_rows(monkeypatch):
    """Under HIP-graph capture (simulated on CPU) the patched core reads no tensor back, runs the padded
    op on the lowered ranges, and gives a row whose mask it cannot express an empty range + a count."""
    from flash_attention_cute_amd import hf_attention as hfa

    calls = []

    def fake_padded(q, k, v, ks, ke, qs=None, qe=None, softmax_scale=None, causal=False, window_left=-1):
        calls.append((ks.clone(), ke.clone(), None if qs is None else qs.clone(), None if qe is None else qe.clone()))
        return torch.zeros_like(q)

    monkeypatch.setattr(hfa, "_capturing", lambda t: True)
    monkeypatch.setattr(hfa, "flash_attn_padded_func", fake_padded)
    hfa._MASK_ERRORS.clear()
    total, b, h, d = 10, 3, 2, 8
    valid = torch.zeros(b, total, dtype=torch.bool)
    valid[:, 2:8] = True
    mask = _static_masks(valid, 0, 8, total)[:, :, :8].clone()
    mask[2, 0, 6, 3] = False  # row 2: a score hidden that padding does not explain
    q, k = torch.randn(b, h, 8, d), torch.randn(b, h, total, d)
    mod = type("M", (), {"is_causal": True})()
    with _NoHostReads():
        hfa._flash_attention_forward(mod, q, k, k, mask, scaling=0.3)
    ks, ke, qs, qe = calls[-1]
    assert ks.tolist() == [2, 2, 2] and ke.tolist() == [8, 8, 2]  # row 2: empty key range
    assert qs.tolist() == [2, 2, 2] and qe.tolist() == [8, 8, 2]
    assert hfa.mask_errors("cpu") == 1


@pytest.mark.gpu
def test_patched_llama_static_cache_decode_steps_replay_one_hip_graph(device):
    """a left-padded greedy generation whose decode steps replay ONE captured
    HIP graph of the patched model's decode step (StaticCache, TRUST_PADDING_MASK left False, the mask
    lowered on the device) produces the token ids of unpatched transformers' eager generate."""
    from transformers import StaticCache

    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    assert hf_attention.TRUST_PADDING_MASK is False
    model, ids, mask = tiny_generator(device, True)
    model = model.half()
    # no EOS: the config's eos id (2) ends row 0 after two tokens in fp16 and generate pads the rest,
    # while the step loop below keeps generating
    model.generation_config.eos_token_id = None
    n_new = 24
    with torch.no_grad():
        ref = model.generate(ids, attention_mask=mask, max_new_tokens=n_new, do_sample=False, pad_token_id=0,
                             cache_implementation="static")
    b, n0 = ids.shape
    total = n0 + n_new
    cache = StaticCache(config=model.config, max_cache_len=total)
    full = torch.zeros(b, total, dtype=torch.long, device=device)  # the 2-D mask over every slot
    full[:, :n0] = mask
    pid = (mask.long().cumsum(1) - 1).clamp(min=0)
    toks = []
    with torch.no_grad(), warnings.catch_warnings(), patched(ml.LlamaAttention):
        warnings.simplefilter("ignore")
        out = model(ids, attention_mask=full[:, :n0], position_ids=pid, past_key_values=cache, use_cache=True,
                    cache_position=torch.arange(n0, device=device))
        toks.append(out.logits[:, -1].argmax(-1, keepdim=True))
        tok_buf, pos_buf = toks[-1].clone(), pid[:, -1:] + 1
        # the cache slot of the fed token, a device tensor advanced in place: without it the model
        # derives the slot from the cache's host-side length, which a captured graph bakes in
        slot_buf = torch.tensor([n0], device=device)
        full[:, n0] = 1

        def step():
            return model(tok_buf, attention_mask=full, position_ids=pos_buf, past_key_values=cache,
                         use_cache=True, cache_position=slot_buf).logits[:, -1]

        def advance(logits, i):  # token i + 1 generated: feed it at the next slot
            toks.append(logits.argmax(-1, keepdim=True))
            tok_buf.copy_(toks[-1])
            full[:, n0 + i] = 1
            pos_buf.add_(1)
            slot_buf.add_(1)

        advance(step(), 1)  # decode step 1 eagerly (it also warms every lazy initialisation up)
        torch.cuda.synchronize()
        errors0 = hf_attention.mask_errors(device)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            logits_buf = step()
        assert _debug.last_path() in ("decode", "decode_split"), _debug.last_path()
        for i in range(2, n_new):
            graph.replay()
            advance(logits_buf, i)
        torch.cuda.synchronize()
    got = torch.cat([ids] + toks[:n_new], dim=1)
    assert got.shape == ref.shape
    assert torch.equal(got, ref), (got[:, n0:], ref[:, n0:])
    assert hf_attention.mask_errors(device) == errors0 == 0
