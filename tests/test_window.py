"""Local (sliding-window) attention -- include/fa_gfx950.h fa_fwd_gfx950_window, the op
``flash_attention::window_forward`` / ``flash_attn_window_func`` and the HF patch's Qwen2 sliding
window (the reference computes it and then ignores it, reference models/rope_attn_fwd.py:95-101).

The reference has no window mask, so no reference output pins it: the semantics are pinned to
transformers' own ``sliding_window_causal_mask_function`` (parity unpinned against the reference,
pinned against the library whose models the patch serves). CPU tests here: the mask convention,
the oracle's window against a float64 restatement, the op's CPU default, and the HF mask lowering.
The GPU parity sweep is tests/test_gpu_window.py.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from flash_attention_cute_amd.flash_attention import _window_mask
from oracle import fa_oracle_c as OC


def _ref64(q, k, v, scale, causal, window_left):
    """float64 attention under the window mask; rows that see no key are 0."""
    qd, kd, vd = (t.double() for t in (q, k, v))
    g = qd.shape[1] // kd.shape[1]
    kd = kd.repeat_interleave(g, dim=1)
    vd = vd.repeat_interleave(g, dim=1)
    sq, sk = q.shape[2], k.shape[2]
    if sq == 1:  # the decode convention: the one query sits at position Sk - 1
        mask = torch.arange(sk)[None, :] >= sk - 1 - window_left
    else:
        mask = _window_mask(sq, sk, window_left, causal, "cpu")
    s = torch.einsum("bhmd,bhnd->bhmn", qd, kd) * scale
    s = s.masked_fill(~mask, float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    return torch.einsum("bhmn,bhnd->bhmd", p, vd)


@pytest.mark.parametrize("sq,sk", [(7, 7), (5, 12), (12, 5), (1, 9)])
@pytest.mark.parametrize("w", [1, 2, 4, 16])
def test_window_mask_matches_transformers(sq, sk, w):
    """``_window_mask(window_left = W - 1)`` is transformers' sliding_window_causal_mask_function(W)
    with the queries at the last Sq positions (the KV-cache convention)."""
    masking_utils = pytest.importorskip("transformers.masking_utils")
    fn = masking_utils.sliding_window_causal_mask_function(w)
    off = sk - sq
    t = torch.tensor
    ref = torch.tensor([[bool(fn(t(0), t(0), t(m + off), t(n))) for n in range(sk)] for m in range(sq)])
    assert torch.equal(_window_mask(sq, sk, w - 1, True, "cpu"), ref)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [True, False], ids=["causal", "full"])
@pytest.mark.parametrize("shape,wl", [((1, 2, 2, 150, 150, 32), 0), ((1, 4, 2, 150, 150, 32), 37),
                                      ((2, 2, 1, 70, 200, 16), 64), ((1, 2, 2, 200, 70, 16), 20),
                                      ((1, 4, 1, 1, 300, 32), 99)])
def test_oracle_window_against_float64(dtype, causal, shape, wl):
    b, hq, hkv, sq, sk, d = shape
    g = torch.Generator().manual_seed(sq * 1000 + sk + wl)
    q = torch.randn(b, hq, sq, d, generator=g).to(dtype)
    k = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    v = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    scale = d ** -0.5
    got = OC.forward(q, k, v, scale, causal, window_left=wl).double()
    ref = _ref64(q, k, v, scale, causal and sq > 1, wl)
    tol = 2e-3 if dtype == torch.float16 else 1.6e-2
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=tol, rtol=tol)


def test_oracle_without_window_is_unchanged():
    g = torch.Generator().manual_seed(3)
    q, k, v = (torch.randn(1, 2, 90, 32, generator=g).half() for _ in range(3))
    assert torch.equal(OC.forward(q, k, v, 0.2, True), OC.forward(q, k, v, 0.2, True, window_left=-1))


def test_op_cpu_default_matches_oracle():
    from flash_attention_cute_amd import flash_attn_window_func

    g = torch.Generator().manual_seed(5)
    q = torch.randn(1, 4, 120, 32, generator=g).half()
    k = torch.randn(1, 2, 160, 32, generator=g).half()
    v = torch.randn(1, 2, 160, 32, generator=g).half()
    with pytest.warns(UserWarning):
        out = flash_attn_window_func(q.float(), k.float(), v.float(), 31, causal=True)
    ref = OC.forward(q, k, v, 32 ** -0.5, True, window_left=31).float()
    torch.testing.assert_close(out, ref, atol=2e-3, rtol=2e-3)


def test_window_op_schema_and_fake():
    schema = str(torch.ops.flash_attention.window_forward.default._schema)
    assert schema.startswith("flash_attention::window_forward(Tensor q, Tensor k, Tensor v, SymInt window_left")
    q = torch.empty(1, 2, 8, 16, device="meta")
    assert torch.ops.flash_attention.window_forward(q, q, q, 3, 0.25, True).shape == q.shape
