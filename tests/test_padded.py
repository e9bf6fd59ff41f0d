"""Padded batches read in place -- per-sequence query / key ranges inside dense tensors.

No reference counterpart: the reference's HF patch drops ``attention_mask``
(reference models/rope_attn_fwd.py:40-64). ``flash_attn_padded_func`` (C-ABI
``fa_fwd_gfx950_padded``) is what an HF left / right padding mask is lowered to: the projections
and the KV cache are read where they are (no ``index_select`` packing), and a decode step keeps
the reference's Sq == 1 q-head pack (reference csrc/flash_attention_api.cpp:72-83) on the split-KV
kernel, now with each sequence's own key range.

Semantics pinned here: batch row b is the dense operator on its real rows (bottom-right causal per
sequence, rows that see no key 0, rows outside the query range 0). The oracle is the packed-varlen
oracle (``fa_oracle_c.forward_varlen``, itself the dense oracle per sequence, which
tests/test_oracle.py pins to the reference's golden vectors) on the gathered real rows.
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


def make_batch(b, hq, hkv, sq, sk, d, dtype, seed, layout="bshd"):
    """Dense q [B, Hq, Sq, D], k / v [B, Hkv, Sk, D]; "bshd": HF projection views (seq stride H * D)."""
    g = torch.Generator().manual_seed(seed)
    if layout == "bshd":
        q = torch.randn(b, sq, hq, d, generator=g).to(dtype).transpose(1, 2)
        k = torch.randn(b, sk, hkv, d, generator=g).to(dtype).transpose(1, 2)
        v = torch.randn(b, sk, hkv, d, generator=g).to(dtype).transpose(1, 2)
    else:  # KV-cache layout [B, H, S, D] contiguous
        q = torch.randn(b, hq, sq, d, generator=g).to(dtype)
        k = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
        v = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    return q, k, v


def oracle_padded(q, k, v, ks, ke, qs, qe, scale, causal, window_left=-1):
    """The packed-varlen oracle on the gathered real rows, scattered back; other rows 0."""
    b, hq, sq, d = q.shape
    ks, ke = ks.tolist(), ke.tolist()
    qs = qs.tolist() if qs is not None else [0] * b
    qe = qe.tolist() if qe is not None else [sq] * b
    qp = torch.cat([q[i, :, qs[i]:qe[i]].transpose(0, 1) for i in range(b)])
    kp = torch.cat([k[i, :, ks[i]:ke[i]].transpose(0, 1) for i in range(b)])
    vp = torch.cat([v[i, :, ks[i]:ke[i]].transpose(0, 1) for i in range(b)])
    cu_q = torch.tensor([0] + list(np.cumsum([qe[i] - qs[i] for i in range(b)])), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(np.cumsum([ke[i] - ks[i] for i in range(b)])), dtype=torch.int32)
    op = OC.forward_varlen(qp.contiguous(), kp.contiguous(), vp.contiguous(), cu_q, cu_k, scale, causal,
                           window_left=window_left)
    out = torch.zeros(b, sq, hq, d, dtype=q.dtype)
    for i in range(b):
        out[i, qs[i]:qe[i]] = op[int(cu_q[i]):int(cu_q[i + 1])]
    return out.transpose(1, 2)


def ranges(b, sq, sk, seed, side="left", min_len=0):
    """Random real-token runs: keys [ks, ke) of Sk; the queries are the last Sq token positions."""
    rng = np.random.default_rng(seed)
    n = rng.integers(min_len, sk + 1, size=b)
    n[0] = sk  # one full row
    if b > 2:
        n[-1] = min_len  # and a shortest one
    ks = np.where(side == "left", sk - n, 0) if side != "mixed" else np.where(np.arange(b) % 2, sk - n, 0)
    ke = ks + n
    off = sk - sq
    qs = np.clip(ks - off, 0, sq)
    qe = np.clip(ke - off, 0, sq)
    t = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    return t(ks), t(ke), t(qs), t(qe)


# ------------------------------------------------------------------------------------------- CPU
def test_padding_ranges_lowering():
    from flash_attention_cute_amd.hf_attention import padding_ranges

    valid = torch.tensor([[0, 0, 1, 1, 1, 1], [1, 1, 1, 1, 1, 1], [1, 1, 1, 1, 0, 0], [0, 0, 0, 0, 0, 0]],
                         dtype=torch.bool)
    ks, ke, qs, qe = padding_ranges(valid, 6)
    assert ks.tolist() == [2, 0, 0, 0] and ke.tolist() == [6, 6, 4, 0]
    assert qs.tolist() == [2, 0, 0, 0] and qe.tolist() == [6, 6, 4, 0]
    ks, ke, qs, qe = padding_ranges(valid, 1)  # decode: the query is the last position
    assert qs.tolist() == [0, 0, 0, 0] and qe.tolist() == [1, 1, 0, 0]
    holes = valid.clone()
    holes[1, 3] = False
    assert padding_ranges(holes, 6) is None  # not one run: the packed varlen path
    assert padding_ranges(holes, 6, check=False) is not None  # trusted: no host synchronisation


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("sq", [1, 37])
def test_padded_op_cpu_default_matches_oracle(causal, sq):
    from flash_attention_cute_amd import flash_attn_padded_func

    b, hq, hkv, sk, d = 4, 4, 2, 90, 64
    q, k, v = make_batch(b, hq, hkv, sq, sk, d, torch.float16, 3)
    ks, ke, qs, qe = ranges(b, sq, sk, 5, side="mixed", min_len=sq)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out = flash_attn_padded_func(q.float(), k.float(), v.float(), ks, ke, qs, qe, causal=causal)
    ref = oracle_padded(q, k, v, ks, ke, qs, qe, d ** -0.5, causal).float()
    torch.testing.assert_close(out, ref, atol=3e-3, rtol=3e-3)


def test_padded_op_registration():
    import flash_attention_cute_amd  # noqa: F401

    sch = str(torch.ops.flash_attention.padded_forward.default._schema)
    assert sch == ("flash_attention::padded_forward(Tensor q, Tensor k, Tensor v, Tensor k_start, Tensor k_end, "
                   "Tensor? q_start=None, Tensor? q_end=None, float softmax_scale=None, bool causal=False, "
                   "SymInt window_left=-1) -> Tensor")
    q, k, v = make_batch(2, 4, 2, 16, 16, 32, torch.float32, 1)
    ks, ke, qs, qe = ranges(2, 16, 16, 2)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        torch.library.opcheck(torch.ops.flash_attention.padded_forward.default,
                              (q, k, v, ks, ke, qs, qe, 0.125, True, -1),
                              test_utils=("test_schema", "test_faketensor"))


# ------------------------------------------------------------------------------------------- GPU
def check_padded(out, ref, dtype):
    from tests.test_gpu_parity import TOL

    got = out.float().cpu()
    ref = ref.float()
    assert torch.isfinite(got).all()
    atol, rtol, mean_tol = TOL[dtype]
    err = (got - ref).abs()
    worst = (err - (atol + rtol * ref.abs())).max().item()
    assert worst <= 0, f"max err {err.max().item():.3e} exceeds bound by {worst:.3e}"
    assert err.mean().item() <= mean_tol


@pytest.fixture
def padded_op(device):
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attention as fam
    from flash_attention_cute_amd import flash_attn_padded_func

    assert fam.flash_attention_cuda is not None, f"gfx950 extension failed to load: {fam._load_error!r}"
    _debug.set_knobs()

    def run(*a, **kw):
        out = flash_attn_padded_func(*a, **kw)
        return out, _debug.last_path()

    return run


PREFILL = [  # (B, Hq, Hkv, Sq, Sk, D, layout, side)
    (4, 8, 2, 300, 300, 128, "bshd", "left"),
    (3, 4, 4, 517, 517, 64, "bhsd", "right"),
    (5, 8, 1, 100, 700, 128, "bshd", "mixed"),   # Sq < Sk: a chunk on a cache
    (2, 4, 2, 260, 260, 72, "bhsd", "left"),     # padded head dim
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [False, True], ids=["full", "causal"])
@pytest.mark.parametrize("ci", range(len(PREFILL)))
def test_padded_prefill_parity(padded_op, device, ci, causal, dtype):
    b, hq, hkv, sq, sk, d, layout, side = PREFILL[ci]
    seed = zlib.crc32(repr((ci, causal, str(dtype))).encode())
    q, k, v = make_batch(b, hq, hkv, sq, sk, d, dtype, seed, layout)
    ks, ke, qs, qe = ranges(b, sq, sk, seed, side)
    dv = lambda t: t.to(device)  # noqa: E731
    out, path = padded_op(dv(q), dv(k), dv(v), dv(ks), dv(ke), dv(qs), dv(qe), causal=causal)
    torch.cuda.synchronize()
    assert path == "w4"
    check_padded(out, oracle_padded(q, k, v, ks, ke, qs, qe, d ** -0.5, causal), dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("shape", [(32, 32, 8, 4096, "left"), (3, 32, 8, 20000, "mixed"), (8, 16, 16, 333, "right"),
                                   (6, 8, 1, 1000, "left")], ids=["b32", "b3_long", "mha", "mqa"])
def test_padded_decode_runs_the_decode_kernel(padded_op, device, shape, dtype):
    """A decode step (Sq == 1) over a padded KV cache: the q-head pack and the split-KV decode kernel on
    each sequence's own key range, against the per-sequence oracle."""
    b, hq, hkv, sk, side = shape
    d = 128
    seed = zlib.crc32(repr((shape, str(dtype))).encode())
    q, k, v = make_batch(b, hq, hkv, 1, sk, d, dtype, seed, "bhsd")
    ks, ke, _, _ = ranges(b, 1, sk, seed, side, min_len=1)
    dv = lambda t: t.to(device)  # noqa: E731
    out, path = padded_op(dv(q), dv(k), dv(v), dv(ks), dv(ke), causal=True)
    torch.cuda.synchronize()
    assert path in ("decode", "decode_split"), path
    check_padded(out, oracle_padded(q, k, v, ks, ke, None, None, d ** -0.5, False), dtype)


@pytest.mark.gpu
def test_padded_decode_empty_and_single_key_rows(padded_op, device):
    b, hq, hkv, sk, d = 4, 8, 2, 4096, 128
    q, k, v = make_batch(b, hq, hkv, 1, sk, d, torch.float16, 7, "bhsd")
    ks = torch.tensor([0, 4095, 100, 4096], dtype=torch.int32)
    ke = torch.tensor([4096, 4096, 100, 4096], dtype=torch.int32)  # full, one key, empty, empty at the end
    dv = lambda t: t.to(device)  # noqa: E731
    out, _ = padded_op(dv(q), dv(k), dv(v), dv(ks), dv(ke))
    torch.cuda.synchronize()
    o = out.float().cpu()
    assert torch.isfinite(o).all()
    assert (o[2] == 0).all() and (o[3] == 0).all()
    g = hq // hkv
    torch.testing.assert_close(o[1], v[1, :, 4095:4096].float().repeat_interleave(g, 0), atol=0, rtol=0)
    check_padded(out[:1], oracle_padded(q[:1], k[:1], v[:1], ks[:1], ke[:1], None, None, d ** -0.5, False),
                 torch.float16)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_padded_full_ranges_bit_equal_to_dense(padded_op, device, causal):
    from flash_attention_cute_amd import flash_attn_func

    b, hq, hkv, s, d = 3, 8, 2, 700, 128
    q, k, v = (t.to(device) for t in make_batch(b, hq, hkv, s, s, d, torch.bfloat16, 11))
    full = torch.full((b,), s, dtype=torch.int32, device=device)
    zero = torch.zeros(b, dtype=torch.int32, device=device)
    got, path = padded_op(q, k, v, zero, full, zero, full, causal=causal)
    assert path == "w4"
    assert torch.equal(got, flash_attn_func(q, k, v, causal=causal))
    # key ranges alone (the library derives every-row query ranges in its workspace)
    got2, _ = padded_op(q, k, v, zero, full, causal=causal)
    assert torch.equal(got2, got)


@pytest.mark.gpu
def test_padded_window(padded_op, device):
    b, hq, hkv, sq, sk, d, wl = 3, 4, 2, 400, 400, 128, 99
    q, k, v = make_batch(b, hq, hkv, sq, sk, d, torch.float16, 13)
    ks, ke, qs, qe = ranges(b, sq, sk, 13, "left", min_len=50)
    dv = lambda t: t.to(device)  # noqa: E731
    out, path = padded_op(dv(q), dv(k), dv(v), dv(ks), dv(ke), dv(qs), dv(qe), causal=True, window_left=wl)
    torch.cuda.synchronize()
    assert path == "w4"
    check_padded(out, oracle_padded(q, k, v, ks, ke, qs, qe, d ** -0.5, True, window_left=wl), torch.float16)
    # decode with a window: the key range is narrowed on the device, the decode kernel runs
    q1 = q[:, :, -1:]
    out1, path1 = padded_op(dv(q1), dv(k), dv(v), dv(ks), dv(ke), causal=True, window_left=wl)
    torch.cuda.synchronize()
    assert path1 in ("decode", "decode_split")
    ks1 = torch.maximum(ks, ke - (wl + 1))
    check_padded(out1, oracle_padded(q1, k, v, ks1, ke, None, None, d ** -0.5, False), torch.float16)


@pytest.mark.gpu
def test_padded_decode_graph_capture(padded_op, device):
    """The padded decode step makes no host synchronisation: it captures into a HIP graph, and the
    replay follows new q / range values."""
    b, hq, hkv, sk, d = 16, 32, 8, 2048, 128
    q, k, v = (t.to(device) for t in make_batch(b, hq, hkv, 1, sk, d, torch.bfloat16, 17, "bhsd"))
    ks, ke, _, _ = (t.to(device) for t in ranges(b, 1, sk, 17, "left", min_len=1))
    padded_op(q, k, v, ks, ke)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out, _ = padded_op(q, k, v, ks, ke)
    q.copy_(torch.randn_like(q))
    ks.copy_(torch.clamp(ks - 7, min=0))
    g.replay()
    torch.cuda.synchronize()
    ref, path = padded_op(q, k, v, ks, ke)
    assert path in ("decode", "decode_split")
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_padded_prefill_seqlen_sliced_q(padded_op, device, causal):
    """q a seqlen slice of a longer buffer (not dense): empty_like would give a contiguous o with a
    different rows-per-batch multiple than q, so the binding makes q contiguous."""
    b, hq, hkv, sq, sk, d = 3, 8, 2, 200, 200, 128
    q, k, v = make_batch(b, hq, hkv, sq + 56, sk, d, torch.float16, 19, "bhsd")
    q = q[:, :, :sq]
    assert not q.is_contiguous()
    ks, ke, qs, qe = ranges(b, sq, sk, 19, "left", min_len=30)
    dv = lambda t: t.to(device)  # noqa: E731
    out, path = padded_op(dv(q), dv(k), dv(v), dv(ks), dv(ke), dv(qs), dv(qe), causal=causal)
    torch.cuda.synchronize()
    assert path == "w4"
    check_padded(out, oracle_padded(q, k, v, ks, ke, qs, qe, d ** -0.5, causal), torch.float16)


@pytest.mark.gpu
def test_padded_out_of_range_positions_are_clamped(padded_op, device):
    """Ranges past the tensors (negative starts, ends past Sq / Sk, end < start) are clamped on the
    device (include/fa_gfx950.h): the result equals the call with the clamped ranges, and nothing
    outside the output tensor is written (guard rows around it stay untouched)."""
    b, hq, hkv, s, d = 4, 8, 2, 300, 128
    q, k, v = make_batch(b, hq, hkv, s, s, d, torch.bfloat16, 23, "bhsd")
    bad = [torch.tensor(x, dtype=torch.int32) for x in
           ([-50, 10, 290, 400], [250, 900, 280, 500], [-5, 0, 100, 301], [320, 300, 90, 1000])]
    ks, ke, qs, qe = bad
    clamp = lambda a, lo, hi: torch.minimum(torch.maximum(a, lo), hi)  # noqa: E731
    z, n = torch.zeros(b, dtype=torch.int32), torch.full((b,), s, dtype=torch.int32)
    ks_c, qs_c = clamp(ks, z, n), clamp(qs, z, n)
    ke_c, qe_c = clamp(ke, ks_c, n), clamp(qe, qs_c, n)
    dv = lambda t: t.to(device)  # noqa: E731
    # q / k / v with guard rows on both sides inside one allocation, NaN-poisoned
    def guarded(t):
        buf = torch.full((t.shape[0], t.shape[1], t.shape[2] + 64, d), float("nan"), dtype=t.dtype, device=device)
        buf[:, :, 32:32 + t.shape[2]] = dv(t)
        return buf, buf[:, :, 32:32 + t.shape[2]]
    _, qg = guarded(q)
    _, kg = guarded(k)
    _, vg = guarded(v)
    for causal in (False, True):
        out, path = padded_op(qg, kg, vg, dv(ks), dv(ke), dv(qs), dv(qe), causal=causal)
        ref, _ = padded_op(qg, kg, vg, dv(ks_c), dv(ke_c), dv(qs_c), dv(qe_c), causal=causal)
        torch.cuda.synchronize()
        assert path == "w4"
        assert torch.isfinite(out).all()  # the NaN guard rows were never read
        assert torch.equal(out, ref)
        check_padded(out, oracle_padded(q, k, v, ks_c, ke_c, qs_c, qe_c, d ** -0.5, causal), torch.bfloat16)
    # decode (Sq == 1, split-KV kernel): key ranges clamped the same way
    q1 = qg[:, :, -1:]
    out1, path1 = padded_op(q1, kg, vg, dv(ks), dv(ke), causal=True)
    ref1, _ = padded_op(q1, kg, vg, dv(ks_c), dv(ke_c), causal=True)
    torch.cuda.synchronize()
    assert path1 in ("decode", "decode_split")
    assert torch.isfinite(out1).all() and torch.equal(out1, ref1)
