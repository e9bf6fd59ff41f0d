"""GPU parity of the local-window path (include/fa_gfx950.h fa_fwd_gfx950_window) against the
oracle's window (oracle/fa_oracle.c fa_oracle_fwd_window), through ``flash_attn_window_func``.

Covers windows narrower than a tile, exactly one and several tiles wide, wider than the
sequence (the plain path), Sq < Sk and Sq > Sk, GQA, an inexact head dim, decode (Sq == 1: the keys
left of the window are cut and the split-KV decode kernel runs on the rest) and a short query block
whose window still binds (prefill kernel). Tolerances as tests/test_gpu_parity.py:
  fp16 |gpu - oracle| <= 2e-3 + 2e-3*|oracle|, bf16 1.6e-2 + 1.6e-2*|oracle|.
The reference has no window (it ignores Qwen2's, reference models/rope_attn_fwd.py:95-101): the
semantics are pinned to transformers' sliding-window mask in tests/test_window.py.
"""
from __future__ import annotations

import pytest
import torch

from oracle import fa_oracle_c as OC
from tests.test_gpu_parity import make

pytestmark = pytest.mark.gpu

TOL = {torch.float16: 2e-3, torch.bfloat16: 1.6e-2}

CASES = [  # (B, Hq, Hkv, Sq, Sk, D, window_left)
    (2, 4, 2, 1000, 1000, 128, 0),
    (2, 4, 2, 1000, 1000, 128, 63),
    (2, 4, 2, 1000, 1000, 128, 64),
    (2, 4, 2, 1000, 1000, 128, 100),
    (1, 4, 2, 1000, 1000, 128, 255),
    (1, 4, 2, 1000, 1000, 128, 511),
    (1, 4, 2, 1000, 1000, 128, 998),
    (1, 4, 2, 1000, 1000, 128, 5000),  # wider than the sequence: the plain path
    (1, 8, 2, 300, 1200, 128, 200),    # Sq < Sk
    (1, 4, 4, 700, 300, 64, 150),      # Sq > Sk: causal rows without a key are 0
    (2, 4, 1, 513, 513, 72, 130),      # inexact head dim
    (1, 8, 2, 1, 5000, 128, 100),      # decode: cut, then the split-KV decode kernel
    (1, 8, 2, 4, 3000, 128, 100),      # 4 positions x 4 q-heads: the window binds (prefill kernel)
]


def _ids(c):
    return "B{}_H{}-{}_S{}-{}_D{}_w{}".format(*c)


@pytest.fixture
def wfn(device):
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attention as fam
    from flash_attention_cute_amd import flash_attn_window_func

    assert fam.flash_attention_cuda is not None, f"gfx950 extension failed to load: {fam._load_error!r}"
    _debug.set_knobs()
    try:
        yield flash_attn_window_func
    finally:
        _debug.set_knobs()


def _check(out, q, k, v, scale, causal, wl, dtype):
    ref = OC.forward(q, k, v, scale, causal, window_left=wl).float()
    got = out.float().cpu()
    assert got.shape == ref.shape and torch.isfinite(got).all()
    tol = TOL[dtype]
    err = (got - ref).abs()
    assert bool((err <= tol + tol * ref.abs()).all()), f"max err {err.max().item():.3e}"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [True, False], ids=["causal", "full"])
@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_window_matches_oracle(wfn, device, case, causal, dtype):
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d, wl = case
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, 7000 + sq + wl)
    out = wfn(q.to(device), k.to(device), v.to(device), wl, causal=causal)
    torch.cuda.synchronize()
    path = _debug.last_path()
    cut = max(0, sk - sq - wl)
    if sk - cut - 1 <= wl and (hq // hkv) * sq <= 64 and sq == 1:
        assert path in ("decode", "decode_split"), path
    elif sk - cut - 1 > wl:
        assert path == "w4", path
    _check(out, q, k, v, d ** -0.5, causal and sq > 1, wl, dtype)


@pytest.mark.parametrize("variant", ["w8", "p8", "w4slow"])
def test_window_under_other_variants(device, variant):
    """In the debug library (lib/libfa_gfx950_debug.so) the window runs on fa_fwd_w4 whatever prefill
    variant is selected (w8 / p8 have no window mask), and through the debug body under w4slow."""
    from flash_attention_cute_amd import _debug

    q, k, v = make(1, 4, 2, 900, 900, 128, torch.float16, 11)
    try:
        out = _debug.forward(q.to(device), k.to(device), v.to(device), causal=True, variant=variant,
                             window_left=200)
        torch.cuda.synchronize()
        assert _debug.last_path(debug=True) == ("w4slow" if variant == "w4slow" else "w4")
    finally:
        _debug.set_knobs(debug=True)
    _check(out, q, k, v, 128 ** -0.5, True, 200, torch.float16)


def test_window_persistent_grid_block_switches(device):
    """Many Q blocks per workgroup (grid capped at 16): every block starts at its own first window
    tile j_lo with the ring parity restarted, across block switches; two launches bit-equal."""
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attn_window_func

    q, k, v = make(2, 8, 2, 2048, 2048, 128, torch.bfloat16, 12)
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    _debug.set_knobs(w4_grid=16)
    try:
        a = flash_attn_window_func(qd, kd, vd, 300, causal=True)
        b_ = flash_attn_window_func(qd, kd, vd, 300, causal=True)
        torch.cuda.synchronize()
    finally:
        _debug.set_knobs()
    assert torch.equal(a, b_)
    _check(a, q, k, v, 128 ** -0.5, True, 300, torch.bfloat16)


def test_window_qwen2_7b_dims_sampled_heads(device):
    """Qwen2-7B attention dims (Hq 28, Hkv 4, D 128) at S = 8192 with its 4096-token sliding window,
    bf16 causal; q-heads 0, 13 and 27 (first, middle, last kv group) against the oracle."""
    from flash_attention_cute_amd import flash_attn_window_func

    q, k, v = make(1, 28, 4, 8192, 8192, 128, torch.bfloat16, 13)
    out = flash_attn_window_func(q.to(device), k.to(device), v.to(device), 4095, causal=True).cpu()
    for h in (0, 13, 27):
        hk = h // 7
        _check(out[:, h:h + 1], q[:, h:h + 1], k[:, hk:hk + 1], v[:, hk:hk + 1], 128 ** -0.5, True, 4095,
               torch.bfloat16)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [True, False], ids=["causal", "full"])
@pytest.mark.parametrize("wl", [0, 40, 200])
def test_varlen_window_matches_oracle(device, wl, causal, dtype):
    """The window per sequence of a packed batch (fa_fwd_gfx950_varlen_window): ragged, empty and
    Sq != Sk sequences against the per-sequence oracle window."""
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attn_varlen_func
    from tests.test_varlen import CASES as VCASES
    from tests.test_varlen import pack

    _debug.set_knobs()
    for ci, case in enumerate(VCASES):
        q, k, v, cu_q, cu_k, mq, mk = pack(case, dtype, 31 + ci + wl)
        out = flash_attn_varlen_func(q.to(device), k.to(device), v.to(device), cu_q.to(device), cu_k.to(device), mq,
                                     mk, causal=causal, window_left=wl)
        torch.cuda.synchronize()
        assert _debug.last_path() == "w4"
        ref = OC.forward_varlen(q, k, v, cu_q, cu_k, case[2] ** -0.5, causal, window_left=wl).float()
        got = out.float().cpu()
        tol = TOL[dtype]
        err = (got - ref).abs()
        assert bool((err <= tol + tol * ref.abs()).all()), f"case {ci}: max err {err.max().item():.3e}"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_hf_sliding_window_padded_batch_on_gpu(device, dtype):
    """Left-padded batch through a Qwen2 sliding-window layer (window 100) on the GPU: the varlen
    kernel with the window per sequence; real tokens match unpatched HF in fp32."""
    from transformers import DynamicCache
    from transformers.models.qwen2 import modeling_qwen2 as mq

    from flash_attention_cute_amd import _debug
    from tests.test_hf_patch import _null, padded_window_mask4, patched, sliding_qwen2

    _debug.set_knobs()
    cfg = sliding_qwen2(100, hq=8, hkv=2, d=128)
    lens, s = [300, 17, 250, 299], 300
    valid = torch.zeros(4, s + 1, dtype=torch.bool, device=device)
    for b, n in enumerate(lens):
        valid[b, s - n:] = True
    valid[:, s] = True
    torch.manual_seed(0)
    x = torch.randn(4, s + 1, cfg.hidden_size, device=device)
    pid = (valid.long().cumsum(1) - 1).clamp(min=0)
    outs = {}
    for patch, dt in ((False, torch.float32), (True, dtype)):
        torch.manual_seed(1)
        layer = mq.Qwen2Attention(cfg, layer_idx=0).to(device, dt).eval()
        rope = mq.Qwen2RotaryEmbedding(cfg).to(device)
        cache = DynamicCache()
        xx = x.to(dt)
        with torch.no_grad(), (patched(mq.Qwen2Attention) if patch else _null()):
            a, _ = layer(xx[:, :s], position_embeddings=rope(xx, pid[:, :s]),
                         attention_mask=padded_window_mask4(valid, s, 0, 100), past_key_values=cache)
            d, _ = layer(xx[:, s:], position_embeddings=rope(xx, pid[:, s:]),
                         attention_mask=padded_window_mask4(valid, 1, s, 100), past_key_values=cache)
        outs[patch] = (a.float(), d.float())
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    real = valid[:, :s]
    torch.testing.assert_close(outs[True][0][real], outs[False][0][real], atol=tol, rtol=0)
    torch.testing.assert_close(outs[True][1], outs[False][1], atol=tol, rtol=0)
