"""GPU parity of the split-KV decode kernel (csrc/fa_decode.hpp) against the CPU oracle.

The decode kernel serves every call with at most 64 (q-head, position) rows per (batch, kv-head):
the reference's Sq == 1 q-head pack (reference csrc/flash_attention_api.cpp:72-83, which also
forces non-causal) and unpacked GQA / MHA with a few query positions (causal per position,
bottom-right aligned as reference csrc/mask.cuh:37-39). Cases cover: key counts around the 32-key
tile and the 4-wave / split boundaries, single-key and very long K/V (many splits, combine
kernel), D tiles 64 / 128 and ragged D, two row blocks, fully masked rows (Sq > Sk causal), the HF
[B, S, H, D] strided layout, and the unsplit C-ABI entry (fa_fwd_gfx950, no workspace).

Tolerances as tests/test_gpu_parity.py (written in TOL there): the split only changes which
running max a P is rounded against.
"""
from __future__ import annotations

import ctypes
import zlib

import pytest
import torch

from tests.test_gpu_parity import TOL, check, make

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa(device):
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attention as fam
    from flash_attention_cute_amd import flash_attn_func

    assert fam.flash_attention_cuda is not None, f"gfx950 extension failed to load: {fam._load_error!r}"
    _debug.set_knobs()  # the product defaults (w4 + split-KV decode)

    def run(*a, **kw):
        out = flash_attn_func(*a, **kw)
        assert _debug.last_path() in ("decode", "decode_split"), _debug.last_path()
        return out

    return run


DECODE = [  # (B, Hq, Hkv, Sk): Sq == 1, q-head pack
    (1, 8, 2, 1),
    (2, 8, 2, 31),
    (1, 4, 4, 32),
    (3, 8, 1, 33),       # MQA: 8 rows per row block
    (2, 32, 8, 257),
    (1, 32, 8, 4096),    # batch 1: split over the keys + combine
    (4, 16, 2, 5000),
    (1, 64, 1, 3000),    # 64 q-heads on one kv-head: two row blocks
    (1, 2, 1, 70000),    # many splits, long K/V
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("shape", DECODE, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("d", [128, 64])
def test_decode_pack(fa, device, dtype, shape, d):
    b, hq, hkv, sk = shape
    seed = zlib.crc32(repr((shape, d, str(dtype))).encode())
    q, k, v = make(b, hq, hkv, 1, sk, d, dtype, seed)
    for causal in (False, True):  # Sq == 1: the pack forces non-causal (reference :81)
        out = fa(q.to(device), k.to(device), v.to(device), causal=causal)
        torch.cuda.synchronize()
        check(out, q, k, v, d ** -0.5, False, dtype)


SHORT = [  # (B, Hq, Hkv, Sq, Sk): unpacked rows = (Hq / Hkv) * Sq <= 64
    (2, 8, 2, 4, 300),    # speculative decode, 16 rows
    (1, 16, 2, 8, 1000),  # 64 rows: two row blocks
    (1, 4, 4, 16, 200),   # MHA, 16 positions
    (1, 8, 2, 5, 3),      # Sq > Sk: causal rows with no visible key are 0
    (2, 4, 1, 3, 4100),   # split + per-position causal
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [False, True], ids=["full", "causal"])
@pytest.mark.parametrize("shape", SHORT, ids=lambda s: "x".join(map(str, s)))
def test_decode_short_queries(fa, device, dtype, causal, shape):
    b, hq, hkv, sq, sk = shape
    seed = zlib.crc32(repr((shape, causal, str(dtype))).encode())
    q, k, v = make(b, hq, hkv, sq, sk, 128, dtype, seed)
    out = fa(q.to(device), k.to(device), v.to(device), causal=causal)
    torch.cuda.synchronize()
    check(out, q, k, v, 128 ** -0.5, causal, dtype)


@pytest.mark.parametrize("d", [8, 40, 72, 120])
def test_decode_headdims(fa, device, d):
    q, k, v = make(2, 8, 2, 1, 777, d, torch.float16, d)
    out = fa(q.to(device), k.to(device), v.to(device))
    check(out, q, k, v, d ** -0.5, False, torch.float16)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_decode_strided_hf_layout(fa, device, dtype):
    # HF decode: q/k/v are transpose(1, 2) views of [B, S, H, D] (models/rope_attn_fwd.py:81-85)
    b, sk, hq, hkv, d = 3, 1111, 32, 8, 128
    g = torch.Generator().manual_seed(3)
    q4 = torch.randn(b, 1, hq, d, generator=g).to(dtype)
    k4 = torch.randn(b, sk, hkv, d, generator=g).to(dtype)
    v4 = torch.randn(b, sk, hkv, d, generator=g).to(dtype)
    qd, kd, vd = (t.to(device).transpose(1, 2) for t in (q4, k4, v4))
    out = fa(qd, kd, vd, causal=True)
    check(out, *(t.transpose(1, 2).contiguous() for t in (q4, k4, v4)), d ** -0.5, False, dtype)


def test_decode_matches_prefill_kernel(fa, device):
    # the same decode step through the decode kernel and through the prefill kernel
    q, k, v = (t.to(device) for t in make(4, 32, 8, 1, 2048, 128, torch.bfloat16, 21))
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attn_func

    a = fa(q, k, v)
    with _debug.knobs(decode=False):
        b = flash_attn_func(q, k, v)
        assert _debug.last_path() == "w4"
    assert (a.float() - b.float()).abs().max().item() <= 1.6e-2


FUSE = [  # (B, Hq, Hkv, Sq, Sk, D): split-KV launches (n_split > 1)
    (1, 32, 8, 1, 16384, 128),   # decode_long's class: 8 units, one per XCD
    (1, 12, 3, 1, 9000, 128),    # 3 units: XCDs 3..7 get none (their padded workgroups leave)
    (2, 64, 1, 1, 5000, 64),     # MQA with 64 q-heads: two row blocks per (batch, kv-head)
    (1, 8, 2, 3, 7000, 128),     # 3 query positions per q-head (unpacked rows)
]


@pytest.mark.parametrize("shape", FUSE, ids=lambda s: "x".join(map(str, s)))
def test_decode_fused_merge(fa, device, shape):
    """The last split of a (batch, kv-head, row block) merges the partials inside fa_decode (a.cnt:
    the unit's splits on one XCD, the stream's persistent zeroed counters): bit-identical to the
    separate fa_decode_combine launch at D = 128 (one output ulp at D = 64), against the oracle, and
    twice in a row (the counters are left zero)."""
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d = shape
    q, k, v = (t.to(device) for t in make(b, hq, hkv, sq, sk, d, torch.float16, zlib.crc32(repr(shape).encode())))
    try:
        fused = fa(q, k, v)
        assert _debug.last_path() == "decode_split"
        again = fa(q, k, v)
        _debug.set_dec_fuse(0)
        sep = fa(q, k, v)
        assert _debug.last_path() == "decode_split"
    finally:
        _debug.set_dec_fuse()
    assert torch.equal(fused, again)
    if d == 128:
        assert torch.equal(fused, sep)
    else:  # (hipcc folds fa_decode_combine's D = 64 O * 1/l into the f16 conversion, v_fma_mix: one
        # rounding instead of two -- at most one output ulp apart)
        assert (fused.float() - sep.float()).abs().max().item() <= 2 ** -10
    check(fused.cpu(), q.cpu(), k.cpu(), v.cpu(), d ** -0.5, False, torch.float16)


def test_decode_deterministic(fa, device):
    q, k, v = (t.to(device) for t in make(1, 32, 8, 1, 9000, 128, torch.float16, 4))
    assert torch.equal(fa(q, k, v), fa(q, k, v))


def test_unsplit_c_abi_entry(fa, device):
    """fa_fwd_gfx950 (no workspace) runs the decode kernel unsplit: one workgroup per row block."""
    from flash_attention_cute_amd import _build
    from tests.test_abi import FaFwdParams

    lib = ctypes.CDLL(str(_build.ABI_LIB))
    b, hkv, g, sk, d = 1, 2, 4, 3000, 128
    q, k, v = make(b, hkv * g, hkv, 1, sk, d, torch.float16, 8)
    qd = q.to(device).reshape(b, hkv, g, d).contiguous()  # the pack, as the torch host API does it
    kd, vd = k.to(device), v.to(device)
    od = torch.empty_like(qd)
    p = FaFwdParams(q_ptr=qd.data_ptr(), k_ptr=kd.data_ptr(), v_ptr=vd.data_ptr(), o_ptr=od.data_ptr(),
                    batch_size=b, num_heads_q=hkv, num_heads_kv=hkv, seqlen_q=g, seqlen_kv=sk, headdim=d,
                    head_q_per_group=1, softmax_scale=d ** -0.5 * 1.4426950408889634)
    for name, t in (("q", qd), ("k", kd), ("v", vd), ("o", od)):
        setattr(p, f"{name}_batch_stride", t.stride(0))
        setattr(p, f"{name}_head_stride", t.stride(1))
        setattr(p, f"{name}_seqlen_stride", t.stride(2))
    lib.fa_fwd_gfx950.restype = ctypes.c_int
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.fa_fwd_gfx950(ctypes.byref(p), 0, 0, ctypes.c_void_p(stream)) == 0
    from flash_attention_cute_amd import _debug

    assert _debug.last_path() == "decode"  # no workspace: unsplit
    torch.cuda.synchronize()
    check(od.reshape(b, hkv * g, 1, d), q, k, v, d ** -0.5, False, torch.float16)
