"""RoPE next to the attention call -- SURVEY.md 8(f) row 3.

The reference rotates q and k with HF's rotate-half RoPE in elementwise torch ops before the call
(reference models/rope_attn_fwd.py:8-38, :88). This repo rotates k with one HIP pass
(``apply_rope``, C-ABI fa_rope_gfx950) and q inside the attention kernel's Q load
(``flash_attn_rope_func``, C-ABI fa_fwd_gfx950_rope).

Oracle: ``oracle.fa_oracle.rope_rotate`` (the kernels' arithmetic: fp32 fma, one rounding to T),
pinned here to the reference's convention (``hf_attention.apply_rotary_pos_emb``, the reference's
function, and transformers' own) in fp32; then the dense oracle on the rotated q.
GPU bars: the standalone kernel is bit-exact against the oracle; the fused op is bit-equal to
rotate-then-attend through the same kernel, and within TOL (tests/test_gpu_parity.py) of the oracle.
"""
from __future__ import annotations

import warnings
import zlib

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O
from oracle import fa_oracle_c as OC


def tables(b, s, d, dtype, seed, theta=5e5, batch_shared=False):
    """cos / sin [B|1, S, D] of rotary angles pos * theta^(-2i/D), as HF builds them (duplicated halves),
    for random positions (as after left padding / with a cache)."""
    g = torch.Generator().manual_seed(seed)
    pos = torch.randint(0, 8192, (1 if batch_shared else b, s), generator=g).double()
    inv = theta ** (-torch.arange(0, d, 2, dtype=torch.float64) / d)
    ang = pos[..., None] * inv
    emb = torch.cat([ang, ang], dim=-1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def oracle_rope(x, cos, sin):
    dt = "f16" if x.dtype == torch.float16 else "bf16"
    c = cos.double().numpy()[:, None]
    s = sin.double().numpy()[:, None]
    return torch.from_numpy(O.rope_rotate(x.double().numpy(), c, s, dt)).to(x.dtype)


# ------------------------------------------------------------------------------------------- CPU
def test_rope_oracle_matches_reference_convention():
    from flash_attention_cute_amd.hf_attention import apply_rotary_pos_emb
    from transformers.models.llama.modeling_llama import apply_rotary_pos_emb as hf_rope

    q = torch.randn(2, 4, 33, 128, dtype=torch.float64).half().double()
    k = torch.randn(2, 2, 33, 128, dtype=torch.float64).half().double()
    cos, sin = tables(2, 33, 128, torch.float16, 0)
    a, b = apply_rotary_pos_emb(q.float(), k.float(), cos.float(), sin.float())
    c, d = hf_rope(q.float(), k.float(), cos.float(), sin.float())
    assert torch.equal(a, c) and torch.equal(b, d)  # the restated caller is transformers' function
    got = O.rope_rotate(q.numpy(), cos.double().numpy()[:, None], sin.double().numpy()[:, None], "f32")
    np.testing.assert_allclose(got, a.double().numpy(), rtol=2e-7, atol=1e-7)


def test_rope_ops_cpu_defaults():
    from flash_attention_cute_amd import apply_rope, flash_attn_rope_func

    q = torch.randn(1, 4, 40, 64)
    k = torch.randn(1, 4, 40, 64)
    cos, sin = tables(1, 40, 64, torch.float32, 1)
    np.testing.assert_allclose(apply_rope(q, cos, sin).numpy(),
                               O.rope_rotate(q.double().numpy(), cos.double().numpy()[:, None],
                                             sin.double().numpy()[:, None], "f32"), rtol=1e-6, atol=1e-6)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out = flash_attn_rope_func(q, k, k, cos, sin, causal=True)
    ref = torch.nn.functional.scaled_dot_product_attention(apply_rope(q, cos, sin), k, k, is_causal=True)
    torch.testing.assert_close(out, ref)


def test_rope_op_registration():
    import flash_attention_cute_amd  # noqa: F401

    q = torch.randn(1, 2, 16, 64)
    cos, sin = tables(1, 16, 64, torch.float32, 2)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        torch.library.opcheck(torch.ops.flash_attention.rope_apply.default, (q, cos, sin),
                              test_utils=("test_schema", "test_faketensor"))
        torch.library.opcheck(torch.ops.flash_attention.rope_forward.default, (q, q, q, cos, sin, 0.125, True),
                              test_utils=("test_schema", "test_faketensor"))


# ------------------------------------------------------------------------------------------- GPU
@pytest.fixture
def gpu(device):
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attention as fam

    assert fam.flash_attention_cuda is not None, f"gfx950 extension failed to load: {fam._load_error!r}"
    _debug.set_knobs()
    return device


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("d", [128, 64, 72, 40])
def test_apply_rope_bit_exact(gpu, dtype, d):
    from flash_attention_cute_amd import apply_rope

    b, s, h = 4, 777, 8
    gen = torch.Generator().manual_seed(d)
    x4 = torch.randn(b, s, h, d, generator=gen).to(dtype)  # HF projection layout [B, S, H, D] -> [B, H, S, D]
    cos, sin = tables(b, s, d, dtype, d)
    out = apply_rope(x4.to(gpu).transpose(1, 2), cos.to(gpu), sin.to(gpu))
    assert out.stride() == x4.transpose(1, 2).stride()  # keeps the caller's layout
    ref = oracle_rope(x4.transpose(1, 2), cos, sin)
    bad = (out.cpu() != ref).nonzero().tolist()
    if bad:
        bi, hi, si, di = bad[0]
        x = x4.transpose(1, 2)
        pd = (di + d // 2) % d
        raise AssertionError(f"{len(bad)} mismatches; first at {bad[0]}: got {out.cpu()[bi, hi, si, di].item()!r} "
                             f"ref {ref[bi, hi, si, di].item()!r} x {x[bi, hi, si, di].item()!r} "
                             f"partner {x[bi, hi, si, pd].item()!r} cos {cos[bi, si, di].item()!r} "
                             f"sin {sin[bi, si, di].item()!r}")


@pytest.mark.gpu
def test_apply_rope_shared_table(gpu):
    from flash_attention_cute_amd import apply_rope

    x = torch.randn(3, 8, 100, 128, dtype=torch.bfloat16)
    cos, sin = tables(3, 100, 128, torch.bfloat16, 5, batch_shared=True)
    out = apply_rope(x.to(gpu), cos[0].to(gpu), sin[0].to(gpu))  # [S, D] tables
    assert torch.equal(out.cpu(), oracle_rope(x, cos, sin))


CASES = [  # (B, Hq, Hkv, Sq, Sk, D, causal)
    (2, 8, 2, 300, 300, 128, True),     # fused, GQA prefill
    (1, 4, 4, 257, 500, 64, True),      # fused, D = 64 tile, Sq < Sk (a cache)
    (2, 4, 1, 700, 700, 128, False),    # fused, several Q blocks
    (2, 8, 2, 1, 400, 128, False),      # decode (Sq == 1 pack): rotate, then the decode kernel
    (1, 8, 2, 6, 90, 128, True),        # short chunk (g * Sq <= 64): rotate, then the decode kernel
    (1, 4, 2, 130, 130, 96, True),      # other head dim: rotate, then the plain path
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_fused_rope_attention(gpu, dtype, case):
    from flash_attention_cute_amd import _debug, apply_rope, flash_attn_func, flash_attn_rope_func
    from tests.test_gpu_parity import check

    b, hq, hkv, sq, sk, d, causal = case
    seed = zlib.crc32(repr((case, str(dtype))).encode())
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(b, hq, sq, d, generator=g).to(dtype)
    k = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    v = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    cos, sin = tables(b, sq, d, dtype, seed)
    qd, kd, vd, cd, sd = (t.to(gpu) for t in (q, k, v, cos, sin))
    out = flash_attn_rope_func(qd, kd, vd, cd, sd, causal=causal)
    fused = d in (64, 128) and sq > 1 and (hq // hkv) * sq > 64
    assert _debug.last_path() == ("w4" if fused or d == 96 else "decode"), _debug.last_path()
    # the same computation unfused: the standalone kernel, then the plain op -- bit for bit
    assert torch.equal(out, flash_attn_func(apply_rope(qd, cd, sd), kd, vd, causal=causal))
    torch.cuda.synchronize()
    check(out, oracle_rope(q, cos, sin), k, v, d ** -0.5, causal and sq > 1, dtype)


@pytest.mark.gpu
def test_fused_rope_strided_hf_views(gpu):
    from flash_attention_cute_amd import apply_rope, flash_attn_func, flash_attn_rope_func

    b, s, hq, hkv, d = 2, 300, 8, 2, 128
    q = torch.randn(b, s, hq, d, device=gpu, dtype=torch.bfloat16).transpose(1, 2)
    k = torch.randn(b, s, hkv, d, device=gpu, dtype=torch.bfloat16).transpose(1, 2)
    cos, sin = (t.to(gpu) for t in tables(b, s, d, torch.bfloat16, 9))
    out = flash_attn_rope_func(q, k, k, cos, sin, causal=True)
    assert out.stride() == q.stride()
    assert torch.equal(out, flash_attn_func(apply_rope(q, cos, sin), k, k, causal=True))


@pytest.mark.gpu
def test_hf_patch_fused_rope_equals_unfused(gpu):
    """The patched layer with the fused RoPE path (default) and with the reference's torch RoPE:
    the same numbers up to the one rounding the fusion saves (q rotated in fp32 once)."""
    from tests.test_hf_patch import run_layer, tiny_llama
    from transformers.models.llama import modeling_llama as ml

    from flash_attention_cute_amd import hf_attention

    cfg = tiny_llama(hq=8, hkv=2, d=128)
    seqs = (300, 1, 1, 37)
    fused = run_layer(ml.LlamaAttention, cfg, gpu, torch.bfloat16, seqs=seqs, patch=True)
    hf_attention.FUSE_ROPE = False
    try:
        plain = run_layer(ml.LlamaAttention, cfg, gpu, torch.bfloat16, seqs=seqs, patch=True)
    finally:
        hf_attention.FUSE_ROPE = True
    torch.testing.assert_close(fused.float(), plain.float(), atol=2e-2, rtol=0)
