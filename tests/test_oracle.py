"""Pin the CPU oracle before trusting it (CPU only).

(a) against golden vectors produced by the REFERENCE's own operator (tests/golden/make_golden.py,
    reference flash_attention/flash_attention.py:6-15 CPU path);
(b) numpy float64 restatement (oracle/fa_oracle.py) vs the fp32 C port (oracle/fa_oracle.c);
(c) against a plain float64 softmax(QK^T)V with bottom-right causal alignment, for the cases the
    reference's CPU path cannot express (Sq != Sk causal, GQA, decode pack);
(d) the documented divergence from the reference's -FLT_MAX convention on fully masked rows.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O
from oracle import fa_oracle_c as OC

GOLD = Path(__file__).resolve().parent / "golden"


def as_f64(a: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "bf16":
        return O.bf16_bits_to_f64(a)
    return a.astype(np.float64)


def test_golden_c1_config1():
    g = np.load(GOLD / "golden_c1.npz")
    q, k, v, o = g["q"], g["k"], g["v"], g["o"]
    assert q.shape == (1, 2, 128, 64) and q.dtype == np.float32
    out = O.flash_attention_fwd(q.astype(np.float64), k.astype(np.float64), v.astype(np.float64),
                                float(g["scale"]), False, "f32")
    np.testing.assert_allclose(out, o, atol=2e-6, rtol=1e-5)


@pytest.mark.parametrize("i", range(json.loads((GOLD / "golden_meta.json").read_text())["n_small_cases"]))
def test_golden_small_cases(i):
    g = np.load(GOLD / "golden_small.npz")
    dtype = str(g[f"case{i}_dtype"])
    b, h, s, d, causal = (int(x) for x in g[f"case{i}_meta"])
    q, k, v, o = (as_f64(g[f"case{i}_{n}"], dtype) for n in "qkvo")
    out = O.flash_attention_fwd(q, k, v, float(g[f"case{i}_scale"]), bool(causal), dtype)
    # the reference's CPU path is SDPA in T (no P rounding, one final rounding): differences are
    # one or two output ulps of T
    atol = {"f32": 2e-6, "f16": 2e-3, "bf16": 1.6e-2}[dtype]
    np.testing.assert_allclose(out, o, atol=atol, rtol=atol)
    assert np.abs(out - o).mean() < atol / 8


def load_multi_case(g, i):
    """(q, k, v, o) float64 [B, H, S, D], dtype name, scale, causal, layout of golden_multi case i."""
    dtype = str(g[f"case{i}_dtype"])
    b, h, sq, sk, d, causal = (int(x) for x in g[f"case{i}_meta"])
    q, k, v, o = (as_f64(g[f"case{i}_{n}"], dtype) for n in "qkvo")
    assert q.shape == (b, h, sq, d) and k.shape == (b, h, sk, d) and o.shape == q.shape
    return q, k, v, o, dtype, float(g[f"case{i}_scale"]), bool(causal), str(g[f"case{i}_layout"])


@pytest.mark.parametrize("i", range(json.loads((GOLD / "golden_meta.json").read_text())["n_multi_cases"]))
def test_golden_multi_block_cases(i):
    """Multi-block reference-generated cases (several Q blocks, >= 10 KV tiles, Sq != Sk, Sq == 1,
    D in {40, 72, 100}, strided input): the restatement agrees with the reference's op."""
    g = np.load(GOLD / "golden_multi.npz")
    q, k, v, o, dtype, scale, causal, _ = load_multi_case(g, i)
    out = O.flash_attention_fwd(q, k, v, scale, causal, dtype)
    atol = {"f16": 2e-3, "bf16": 1.6e-2}[dtype]
    np.testing.assert_allclose(out, o, atol=atol, rtol=atol)
    assert np.abs(out - o).mean() < atol / 8


def test_golden_multi_covers_the_kernel_shapes():
    g = np.load(GOLD / "golden_multi.npz")
    n = json.loads((GOLD / "golden_meta.json").read_text())["n_multi_cases"]
    metas = [tuple(int(x) for x in g[f"case{i}_meta"]) for i in range(n)]
    assert any(sq == sk and sq > 512 and c for _, _, sq, sk, _, c in metas)  # causal, >= 3 Q blocks
    assert any(sq == sk and sq > 512 and not c for _, _, sq, sk, _, c in metas)
    assert any(sk >= 640 for _, _, _, sk, _, _ in metas)  # >= 10 KV tiles
    assert any(1 < sq < sk for _, _, sq, sk, _, _ in metas) and any(sq > sk for _, _, sq, sk, _, _ in metas)
    assert any(sq == 1 for _, _, sq, _, _, _ in metas)
    assert {40, 72, 100} <= {d for *_, d, _ in metas}
    assert "bshd" in {str(g[f"case{i}_layout"]) for i in range(n)}


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 4, 2, 100, 130, 64), (2, 4, 1, 1, 77, 128), (1, 2, 2, 129, 65, 40),
                                   (1, 3, 3, 64, 64, 128)])
def test_numpy_oracle_matches_c_port(dtype, causal, shape):
    b, hq, hkv, sq, sk, d = shape
    g = torch.Generator().manual_seed(sum(shape))
    q = torch.randn(b, hq, sq, d, generator=g).to(dtype)
    k = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    v = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    name = "f16" if dtype == torch.float16 else "bf16"
    c = OC.forward(q, k, v, d ** -0.5, causal).double().numpy()
    n = O.flash_attention_fwd(q.double().numpy(), k.double().numpy(), v.double().numpy(), d ** -0.5, causal, name)
    ulp = 2 ** -10 if name == "f16" else 2 ** -7
    assert np.abs(c - n).max() <= 2 * ulp * max(1.0, np.abs(n).max())


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 2, 2, 70, 200, 64), (1, 4, 1, 200, 70, 32), (2, 8, 2, 1, 300, 64),
                                   (1, 2, 2, 130, 130, 128)])
def test_oracle_vs_f64_softmax_bottom_right(causal, shape):
    b, hq, hkv, sq, sk, d = shape
    rng = np.random.default_rng(sum(shape))
    q = O.round_to(rng.standard_normal((b, hq, sq, d)), "f16")
    k = O.round_to(rng.standard_normal((b, hkv, sk, d)), "f16")
    v = O.round_to(rng.standard_normal((b, hkv, sk, d)), "f16")
    out = O.flash_attention_fwd(q, k, v, d ** -0.5, causal, "f16", rounded=False)
    ref = O.sdpa_reference_f64(q, k, v, d ** -0.5, causal and sq > 1)
    keep = ~O.fully_masked_rows(sq, sk, causal)
    # only P's rounding to fp16 separates the two (relative 2^-11 per probability)
    np.testing.assert_allclose(out[..., keep, :], ref[..., keep, :], atol=1.5e-3, rtol=1e-3)
    assert np.all(out[..., ~keep, :] == 0)


def test_decode_pack_equals_per_head():
    rng = np.random.default_rng(3)
    b, hq, hkv, sk, d = 2, 8, 2, 90, 64
    q = O.round_to(rng.standard_normal((b, hq, 1, d)), "bf16")
    k = O.round_to(rng.standard_normal((b, hkv, sk, d)), "bf16")
    v = O.round_to(rng.standard_normal((b, hkv, sk, d)), "bf16")
    packed = O.flash_attention_fwd(q, k, v, 0.125, True, "bf16")  # causal ignored when Sq == 1
    g = hq // hkv
    for h in range(hq):
        one = O.flash_attention_fwd(q[:, h:h + 1], k[:, h // g:h // g + 1], v[:, h // g:h // g + 1], 0.125, False,
                                    "bf16")
        np.testing.assert_array_equal(packed[:, h:h + 1], one)


def test_flt_max_quirk_documented():
    """Reference -FLT_MAX convention vs ours: identical except rows that see no key."""
    rng = np.random.default_rng(5)
    sq, sk, d = 300, 100, 64
    q = O.round_to(rng.standard_normal((1, 1, sq, d)), "f16")
    k = O.round_to(rng.standard_normal((1, 1, sk, d)), "f16")
    v = O.round_to(rng.standard_normal((1, 1, sk, d)), "f16")
    ours = O.flash_attention_fwd(q, k, v, d ** -0.5, True, "f16", mask="inf")
    refq = O.flash_attention_fwd(q, k, v, d ** -0.5, True, "f16", mask="flt_max")
    fm = O.fully_masked_rows(sq, sk, True)
    assert fm.sum() == sq - sk
    np.testing.assert_array_equal(ours[..., ~fm, :], refq[..., ~fm, :])
    assert np.all(ours[..., fm, :] == 0)
    # the reference gives a (non-zero) average over the visited tile's columns on those rows
    assert np.abs(refq[..., fm, :]).max() > 0


def test_host_scale_matches_cpp_float_arithmetic():
    s = np.float32(128 ** -0.5)
    assert O.host_scale(float(s)) == float(np.float32(np.float64(s) * 1.4426950408889634))


def test_flops_and_bytes_formulas():
    assert O.attention_flops(4, 32, 4096, 4096, 128, False) == pytest.approx(1.0995e12, rel=1e-4)
    assert O.attention_flops(4, 32, 8192, 8192, 128, True) == pytest.approx(2.1990e12, rel=1e-4)
    assert O.attention_bytes(4, 32, 32, 4096, 4096, 128, 2) == 536870912
    assert O.attention_bytes(4, 32, 8, 4096, 4096, 128, 2) == 335544320


def load_gqa_case(g, i):
    """(q, k, v, o) float64 (q / o [B, Hq, Sq, D], k / v [B, Hkv, Sk, D] -- NOT expanded), dtype, scale,
    causal, (Hq, Hkv) of golden_gqa case i (tests/golden/make_golden.py: the reference op on K / V
    expanded with repeat_interleave, reference scripts/benchmark_kernel.py:37-38)."""
    dtype = str(g[f"case{i}_dtype"])
    b, hq, hkv, sq, sk, d, causal = (int(x) for x in g[f"case{i}_meta"])
    cs = float(g["code_scale"])
    q, k, v = (g[f"case{i}_{n}c"].astype(np.float64) / cs for n in "qkv")
    o = as_f64(g[f"case{i}_o"], dtype)
    assert q.shape == (b, hq, sq, d) and k.shape == (b, hkv, sk, d) and o.shape == q.shape
    return q, k, v, o, dtype, float(g[f"case{i}_scale"]), bool(causal), (hq, hkv)


@pytest.mark.parametrize("i", range(json.loads((GOLD / "golden_meta.json").read_text())["n_gqa_cases"]))
def test_golden_gqa_cases(i):
    """GQA / MQA and the Sq == 1 q-head pack with g = 4 and g = 8 against the reference op's outputs:
    the restatement's kv-head mapping h // g (reference csrc/flash_attention_template.cuh:157-160) and
    pack (reference csrc/flash_attention_api.cpp:72-83) reproduce the reference on unexpanded K / V."""
    g = np.load(GOLD / "golden_gqa.npz")
    q, k, v, o, dtype, scale, causal, _ = load_gqa_case(g, i)
    out = O.flash_attention_fwd(q, k, v, scale, causal, dtype)
    atol = {"f16": 2e-3, "bf16": 1.6e-2}[dtype]
    np.testing.assert_allclose(out, o, atol=atol, rtol=atol)
    assert np.abs(out - o).mean() < atol / 8


@pytest.mark.parametrize("i", range(json.loads((GOLD / "golden_meta.json").read_text())["n_gqa128_cases"]))
def test_golden_gqa128_cases(i):
    """The same at D = 128 (golden_gqa128.npz): causal g = 4 in fp16 (C4's class)
    and bf16 (C5's), the Sq == 1 pack at D = 128, one long causal head (the GPU's key-split layout)."""
    g = np.load(GOLD / "golden_gqa128.npz")
    q, k, v, o, dtype, scale, causal, _ = load_gqa_case(g, i)
    assert q.shape[-1] == 128
    out = O.flash_attention_fwd(q, k, v, scale, causal, dtype)
    atol = {"f16": 2e-3, "bf16": 1.6e-2}[dtype]
    np.testing.assert_allclose(out, o, atol=atol, rtol=atol)
    assert np.abs(out - o).mean() < atol / 8


def pairs_codes(*args):
    """golden_pairs.npz's input codes, regenerated from its seed by the generator's own function."""
    import sys

    sys.path.insert(0, str(GOLD))
    from make_golden import pairs_codes as gen

    return gen(*args)


PAIRS_FILES = json.loads((GOLD / "golden_meta.json").read_text())["pairs_files"]


@pytest.mark.parametrize("fname", PAIRS_FILES)
def test_golden_pairs_case(fname):
    """The key-split pairs fixtures (golden_pairs.npz fp16, golden_pairs_bf16.npz bf16: the reference op
    on a causal GQA launch that the default rule runs as pairs; inputs regenerated from the stored seed):
    the restatement on the three sampled q-heads reproduces the reference's sampled rows."""
    g = np.load(GOLD / fname)
    meta = json.loads((GOLD / "golden_meta.json").read_text())
    assert meta["n_pairs_cases"] == 2 and set(PAIRS_FILES) == {"golden_pairs.npz", "golden_pairs_bf16.npz"}
    dtype = str(g["dtype"])
    b, hq, hkv, sq, sk, d, causal = (int(x) for x in g["meta"])
    qc, kc, vc = pairs_codes(int(g["seed"]), b, hq, hkv, sq, sk, d)
    cs, heads, rows = float(g["code_scale"]), g["heads"], g["rows"]
    grp = hq // hkv
    q = qc[:, heads].astype(np.float64) / cs
    k, v = (c[:, heads // grp].astype(np.float64) / cs for c in (kc, vc))
    out = O.flash_attention_fwd(q, k, v, float(g["scale"]), bool(causal), dtype)[:, :, rows]
    o = as_f64(g["o"], dtype)
    assert out.shape == o.shape
    atol = {"f16": 2e-3, "bf16": 1.6e-2}[dtype]
    np.testing.assert_allclose(out, o, atol=atol, rtol=atol)
    assert np.abs(out - o).mean() < atol / 8


def test_golden_gqa_covers_the_pack_and_the_mapping():
    g = np.load(GOLD / "golden_gqa.npz")
    n = json.loads((GOLD / "golden_meta.json").read_text())["n_gqa_cases"]
    metas = [tuple(int(x) for x in g[f"case{i}_meta"]) for i in range(n)]
    assert {hq // hkv for _, hq, hkv, sq, *_ in metas if sq == 1} >= {4, 8}  # the pack at g = 4 and 8
    assert any(sq > 256 and hkv > 1 and c for _, hq, hkv, sq, sk, _, c in metas)  # causal GQA, >= 2 Q blocks
    assert any(hq == 32 and hkv == 8 for _, hq, hkv, *_ in metas)
    assert (GOLD / "golden_gqa.npz").stat().st_size <= 1 << 20
    # the mapping matters: the same case with q-head h reading kv-head h % Hkv gives other outputs
    q, k, v, o, dtype, scale, causal, (hq, hkv) = load_gqa_case(g, 0)
    wrong = O.flash_attention_fwd(q, k[:, np.arange(hq) % hkv], v[:, np.arange(hq) % hkv], scale, causal, dtype)
    assert np.abs(wrong - o).max() > 0.1
