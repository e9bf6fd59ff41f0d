"""Variable-length (packed) batches and padding masks -- SURVEY.md 8(f) row 4.

No reference counterpart: varlen is a TODO at reference README.md:18 and the reference's HF
patch drops ``attention_mask`` (models/rope_attn_fwd.py:40-64; its vendored models raise on one,
models/modeling_llama.py:296-297). The semantics pinned here: every sequence of the pack is the
dense operator on its own rows (bottom-right causal per sequence, rows that see no key are 0), so
the varlen oracle is the dense oracle per sequence (which tests/test_oracle.py pins to the
reference's golden vectors), itself checked here against a plain float64 softmax.

CPU: the oracle, the op's CPU default, op registration, and the HF mask lowering.
GPU (-m gpu): the HIP kernel (C-ABI fa_fwd_gfx950_varlen through the op) against the oracle,
bit-equality with the dense launch, strided packs, graph capture, padded HF batches.
Tolerances: tests/test_gpu_parity.py TOL (fp16 2e-3 + 2e-3|ref|, bf16 1.6e-2 + 1.6e-2|ref|).
"""
from __future__ import annotations

import warnings
import zlib

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O
from oracle import fa_oracle_c as OC

CASES = [  # (Hq, Hkv, D, [(Sq_b, Sk_b), ...])
    (4, 4, 128, [(130, 130), (1, 1), (300, 300), (64, 64)]),
    (8, 2, 128, [(100, 333), (333, 333), (7, 20), (256, 256), (513, 513)]),   # GQA, Sq < Sk
    (4, 1, 64, [(50, 50), (0, 0), (77, 77), (0, 9), (260, 260)]),             # empty sequences
    (2, 2, 72, [(40, 30), (1, 100), (129, 129)]),                            # Sq > Sk (no-key rows)
]


def pack(case, dtype, seed):
    hq, hkv, d, lens = case
    g = torch.Generator().manual_seed(seed)
    tq = sum(a for a, _ in lens)
    tk = sum(b for _, b in lens)
    q = torch.randn(tq, hq, d, generator=g).to(dtype)
    k = torch.randn(tk, hkv, d, generator=g).to(dtype)
    v = torch.randn(tk, hkv, d, generator=g).to(dtype)
    cu_q = torch.tensor([0] + list(np.cumsum([a for a, _ in lens])), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(np.cumsum([b for _, b in lens])), dtype=torch.int32)
    return q, k, v, cu_q, cu_k, max(a for a, _ in lens), max(b for _, b in lens)


def f64_reference(q, k, v, cu_q, cu_k, scale, causal):
    """Plain float64 softmax(QK^T) V per sequence (bottom-right causal), no-key rows 0."""
    out = np.zeros(q.shape)
    cq, ck = cu_q.tolist(), cu_k.tolist()
    for b in range(len(cq) - 1):
        q0, q1, k0, k1 = cq[b], cq[b + 1], ck[b], ck[b + 1]
        if q1 == q0 or k1 == k0:
            continue
        qs, ks, vs = (t.double().numpy().transpose(1, 0, 2)[None] for t in (q[q0:q1], k[k0:k1], v[k0:k1]))
        o = O.sdpa_reference_f64(qs, ks, vs, scale, causal)[0]
        o[:, O.fully_masked_rows(q1 - q0, k1 - k0, causal)] = 0
        out[q0:q1] = o.transpose(1, 0, 2)
    return out


# ------------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_varlen_oracle_matches_float64(ci, causal):
    q, k, v, cu_q, cu_k, _, _ = pack(CASES[ci], torch.float16, ci)
    scale = CASES[ci][2] ** -0.5
    got = OC.forward_varlen(q, k, v, cu_q, cu_k, scale, causal).double().numpy()
    ref = f64_reference(q, k, v, cu_q, cu_k, scale, causal)
    np.testing.assert_allclose(got, ref, atol=3e-3, rtol=3e-3)


def test_varlen_oracle_equals_dense_oracle_on_equal_lengths():
    q, k, v = (torch.randn(3 * 200, 4, 128).half() for _ in range(3))
    cu = torch.tensor([0, 200, 400, 600], dtype=torch.int32)
    got = OC.forward_varlen(q, k, v, cu, cu, 0.1, True)
    dense = OC.forward(*(t.view(3, 200, 4, 128).transpose(1, 2).contiguous() for t in (q, k, v)), 0.1, True)
    assert torch.equal(got.view(3, 200, 4, 128), dense.transpose(1, 2))


@pytest.mark.parametrize("causal", [False, True])
def test_varlen_op_cpu_default(causal):
    from flash_attention_cute_amd import flash_attn_varlen_func

    q, k, v, cu_q, cu_k, mq, mk = pack(CASES[1], torch.float32, 5)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out = flash_attn_varlen_func(q, k, v, cu_q, cu_k, mq, mk, causal=causal)
    ref = f64_reference(q, k, v, cu_q, cu_k, 128 ** -0.5, causal)
    np.testing.assert_allclose(out.double().numpy(), ref, atol=2e-5, rtol=1e-4)


def test_varlen_max_seqlen_check(monkeypatch):
    """FA_CHECK_VARLEN=1: a max_seqlen below the longest sequence raises instead of silently leaving
    rows uncomputed (off by default: no host sync)."""
    from flash_attention_cute_amd import flash_attention as fam

    q, k, v, cu_q, cu_k, mq, mk = pack(CASES[1], torch.float32, 5)
    fam._check_varlen_maxima(cu_q, cu_k, mq, mk)  # true maxima pass
    with pytest.raises(ValueError, match="max_seqlen_q"):
        fam._check_varlen_maxima(cu_q, cu_k, mq - 1, mk)
    with pytest.raises(ValueError, match="max_seqlen_k"):
        fam._check_varlen_maxima(cu_q, cu_k, mq, mk - 1)
    monkeypatch.setenv("FA_CHECK_VARLEN", "1")  # set after import: read at the call
    with pytest.raises(ValueError):
        fam.flash_attn_varlen_func(q, k, v, cu_q, cu_k, mq - 1, mk)
    monkeypatch.setenv("FA_CHECK_VARLEN", "0")


def test_varlen_op_registration():
    import flash_attention_cute_amd  # noqa: F401

    sch = str(torch.ops.flash_attention.varlen_forward.default._schema)
    assert sch == ("flash_attention::varlen_forward(Tensor q, Tensor k, Tensor v, Tensor cu_seqlens_q, "
                   "Tensor cu_seqlens_k, SymInt max_seqlen_q, SymInt max_seqlen_k, float softmax_scale=None, "
                   "bool causal=False, SymInt window_left=-1) -> Tensor")
    q, k, v, cu_q, cu_k, mq, mk = pack(CASES[0], torch.float32, 1)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        torch.library.opcheck(torch.ops.flash_attention.varlen_forward.default,
                              (q, k, v, cu_q, cu_k, mq, mk, 0.125, True),
                              test_utils=("test_schema", "test_faketensor"))


def hf_mask_4d(valid: torch.Tensor, sq: int):
    """The 4-D bool mask transformers builds for SDPA: causal AND key not padding."""
    b, sk = valid.shape
    ar = torch.arange(max(sk, sq), device=valid.device)
    causal = ar[None, :sk] <= ar[:sq, None] + (sk - sq)
    return (causal[None] & valid[:, None, :])[:, None]


def test_key_padding_lowering():
    from flash_attention_cute_amd.hf_attention import key_padding

    valid = torch.tensor([[0, 0, 1, 1, 1, 1], [1, 1, 1, 1, 1, 1], [1, 1, 1, 1, 0, 0]], dtype=torch.bool)
    assert torch.equal(key_padding(valid.int(), 6, 6, True), valid)                   # 2-D padding mask
    assert torch.equal(key_padding(hf_mask_4d(valid, 6), 6, 6, True), valid)          # 4-D bool, prefill
    add = torch.where(hf_mask_4d(valid, 6), 0.0, torch.finfo(torch.float32).min)
    assert torch.equal(key_padding(add, 6, 6, True), valid)                           # 4-D additive
    assert torch.equal(key_padding(hf_mask_4d(valid, 1), 1, 6, False), valid)         # decode step
    full = torch.ones(3, 6, dtype=torch.bool)
    assert key_padding(hf_mask_4d(full, 6), 6, 6, True) is None                       # plain causal
    assert key_padding(None, 6, 6, True) is None
    sliding = hf_mask_4d(full, 6) & (torch.arange(6)[None, :] > torch.arange(6)[:, None] - 3)[None, None]  # noqa
    with pytest.raises(NotImplementedError, match="causal \\+ key-padding"):
        key_padding(sliding, 6, 6, True)


@pytest.mark.parametrize("side", ["left", "right"])
def test_hf_padded_batch_on_cpu(side):
    """A padded batch through the patched layer (op CPU default) matches unpatched HF SDPA on the
    real tokens, prefill and one decode step."""
    from tests.test_hf_patch import patched, tiny_llama
    from transformers import DynamicCache
    from transformers.models.llama import modeling_llama as ml

    cfg = tiny_llama(hq=4, hkv=2, d=32)
    torch.manual_seed(0)
    layer = ml.LlamaAttention(cfg, layer_idx=0).eval()
    rope = ml.LlamaRotaryEmbedding(cfg)
    lens = [9, 5, 7]
    s = 9
    valid = torch.zeros(3, s + 1, dtype=torch.bool)
    for b, n in enumerate(lens):
        if side == "left":
            valid[b, s - n:] = True
        else:
            valid[b, :n] = True
    valid[:, s] = True  # the decode token
    x = torch.randn(3, s + 1, cfg.hidden_size)
    pid = (valid.long().cumsum(1) - 1).clamp(min=0)
    outs = {}
    for patch in (False, True):
        cache = DynamicCache(config=cfg)
        with torch.no_grad(), warnings.catch_warnings(), (patched(ml.LlamaAttention) if patch else _null()):
            warnings.simplefilter("ignore")
            a, _ = layer(x[:, :s], position_embeddings=rope(x, pid[:, :s]),
                         attention_mask=hf_mask_4d(valid[:, :s], s), past_key_values=cache)
            d, _ = layer(x[:, s:], position_embeddings=rope(x, pid[:, s:]),
                         attention_mask=hf_mask_4d(valid, 1), past_key_values=cache)
        outs[patch] = (a, d)
    real = valid[:, :s]
    torch.testing.assert_close(outs[True][0][real], outs[False][0][real], atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(outs[True][1], outs[False][1], atol=2e-5, rtol=1e-4)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


# ------------------------------------------------------------------------------------------- GPU
def check_varlen(out, q, k, v, cu_q, cu_k, scale, causal, dtype):
    from tests.test_gpu_parity import TOL

    ref = OC.forward_varlen(q, k, v, cu_q, cu_k, scale, causal).float()
    got = out.float().cpu()
    assert torch.isfinite(got).all()
    atol, rtol, mean_tol = TOL[dtype]
    err = (got - ref).abs()
    worst = (err - (atol + rtol * ref.abs())).max().item() if err.numel() else 0.0
    assert worst <= 0, f"max err {err.max().item():.3e} exceeds bound by {worst:.3e}"
    assert err.numel() == 0 or err.mean().item() <= mean_tol


@pytest.fixture
def gpu_varlen(device):
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attention as fam
    from flash_attention_cute_amd import flash_attn_varlen_func

    assert fam.flash_attention_cuda is not None, f"gfx950 extension failed to load: {fam._load_error!r}"
    _debug.set_knobs()

    def run(*a, **kw):
        out = flash_attn_varlen_func(*a, **kw)
        assert _debug.last_path() == "w4", _debug.last_path()
        return out

    return run


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [False, True], ids=["full", "causal"])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_varlen_parity(gpu_varlen, device, ci, causal, dtype):
    seed = zlib.crc32(repr((ci, causal, str(dtype))).encode())
    q, k, v, cu_q, cu_k, mq, mk = pack(CASES[ci], dtype, seed)
    out = gpu_varlen(q.to(device), k.to(device), v.to(device), cu_q.to(device), cu_k.to(device), mq, mk,
                     causal=causal)
    torch.cuda.synchronize()
    check_varlen(out, q, k, v, cu_q, cu_k, CASES[ci][2] ** -0.5, causal, dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_varlen_bit_equal_to_dense_on_equal_lengths(gpu_varlen, device, causal):
    from flash_attention_cute_amd import flash_attn_func

    b, s, hq, hkv, d = 3, 700, 8, 2, 128
    q, k, v = (torch.randn(b, s, h, d, device=device, dtype=torch.bfloat16) for h in (hq, hkv, hkv))
    cu = torch.arange(0, (b + 1) * s, s, device=device, dtype=torch.int32)
    got = gpu_varlen(q.view(b * s, hq, d), k.view(b * s, hkv, d), v.view(b * s, hkv, d), cu, cu, s, s, causal=causal)
    dense = flash_attn_func(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal=causal)
    assert torch.equal(got.view(b, s, hq, d), dense.transpose(1, 2))


@pytest.mark.gpu
def test_varlen_strided_pack(gpu_varlen, device):
    # q, k, v as slices of one packed qkv projection [total, Hq + 2 Hkv, D] (row stride (Hq+2Hkv)*D)
    hq, hkv, d = 8, 2, 128
    lens = [(300, 300), (45, 45), (128, 128)]
    tot = sum(a for a, _ in lens)
    qkv = torch.randn(tot, hq + 2 * hkv, d, device=device, dtype=torch.float16)
    q, k, v = qkv[:, :hq], qkv[:, hq:hq + hkv], qkv[:, hq + hkv:]
    cu = torch.tensor([0, 300, 345, 473], dtype=torch.int32)
    out = gpu_varlen(q, k, v, cu.to(device), cu.to(device), 300, 300, causal=True)
    assert out.shape == q.shape  # (empty_like of a non-dense view is contiguous, as for the dense op)
    check_varlen(out, q.cpu(), k.cpu(), v.cpu(), cu, cu, d ** -0.5, True, torch.float16)


@pytest.mark.gpu
def test_varlen_graph_capture(gpu_varlen, device):
    q, k, v, cu_q, cu_k, mq, mk = (t.to(device) if torch.is_tensor(t) else t for t in pack(CASES[1], torch.float16, 3))
    gpu_varlen(q, k, v, cu_q, cu_k, mq, mk, causal=True)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = gpu_varlen(q, k, v, cu_q, cu_k, mq, mk, causal=True)
    q.copy_(torch.randn_like(q))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, gpu_varlen(q, k, v, cu_q, cu_k, mq, mk, causal=True))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_hf_padded_batch_on_gpu(device, dtype):
    """Left-padded batch (generation-style) through the patched Llama layer on the GPU: prefill and
    two decode steps run the padded path in place; real tokens match unpatched HF in fp32."""
    from tests.test_hf_patch import patched, tiny_llama
    from transformers import DynamicCache
    from transformers.models.llama import modeling_llama as ml

    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    cfg = tiny_llama(hq=8, hkv=2, d=128)
    torch.manual_seed(0)
    lens, s, steps = [300, 17, 250, 299], 300, 2
    valid = torch.zeros(4, s + steps, dtype=torch.bool, device=device)
    for b, n in enumerate(lens):
        valid[b, s - n:] = True
    valid[:, s:] = True
    x = torch.randn(4, s + steps, cfg.hidden_size, device=device)
    pid = (valid.long().cumsum(1) - 1).clamp(min=0)
    outs = {}
    for patch, dt in ((False, torch.float32), (True, dtype)):
        torch.manual_seed(1)  # the same weights for both runs
        layer = ml.LlamaAttention(cfg, layer_idx=0).to(device, dt).eval()
        rope = ml.LlamaRotaryEmbedding(cfg).to(device)
        cache = DynamicCache(config=cfg)
        res, paths = [], []
        with torch.no_grad(), warnings.catch_warnings(), (patched(ml.LlamaAttention) if patch else _null()):
            warnings.simplefilter("ignore")
            pos = 0
            for n in (s,) + (1,) * steps:
                xs = x[:, pos:pos + n].to(dt)
                o, _ = layer(xs, position_embeddings=rope(xs, pid[:, pos:pos + n]),
                             attention_mask=hf_mask_4d(valid[:, :pos + n], n), past_key_values=cache)
                res.append(o.float())
                if patch:
                    paths.append(_debug.last_path())
                pos += n
        outs[patch] = torch.cat(res, 1)
        if patch:
            # prefill: the padded batch in place on the prefill kernel; decode steps: the q-head
            # pack on the split-KV decode kernel over each sequence's key range
            assert paths[0] == "w4" and all(p in ("decode", "decode_split") for p in paths[1:]), paths
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    real = valid
    torch.testing.assert_close(outs[True][real], outs[False][real], atol=tol, rtol=0)
