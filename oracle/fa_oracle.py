"""CPU oracle for the FlashAttention-2 forward hot path -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it. The gfx950 operator never routes through it.

It restates, in numpy float64, the algorithm of the reference CUDA kernel (which cannot be built
or run here: CUTLASS is an empty submodule and there is no nvcc / NVIDIA GPU -- SURVEY.md 8(c)):

  host   reference csrc/flash_attention_api.cpp:64-135   Sq==1 q-head packing, scale*log2(e)
  kernel reference csrc/flash_attention_template.cuh:327-528
         - S = Q K^T per 64-key block, fp32 accumulation            (:362-373)
         - OOB and bottom-right causal mask                          (csrc/mask.cuh:37-43, 54-87)
         - causal block skip                                          (csrc/mask.cuh:45-52, template :344-349)
         - running max on unscaled S, alpha = exp2((m_old-m_new)*s') (:445-471)
         - P = exp2(S*s' - m*s'), row sum of fp32 P                  (:475-487)
         - P rounded to T (RNE) before P.V                           (:493-514)
         - O / l with l == 0 -> 1, rounded to T                      (:516-530)

Two mask conventions are provided:

* ``mask="inf"`` (default) -- the semantics of this repository's kernel: masked scores are -inf and
  a row that sees no key at all (causal with Sq > Sk, rows m < Sq - Sk) is defined as 0.
  For every other row this is identical to the reference (a masked score contributes exactly 0
  either way).
* ``mask="flt_max"`` -- bit-level restatement of the reference's -FLT_MAX convention, including its
  128-row q-tile block skip, which makes fully masked rows of a non-skipped tile an average of V
  over the tile's columns (SURVEY.md Appendix A, quirk iii). Used only to document that quirk.

Parity pinning: this oracle is checked against (a) golden vectors produced by the reference's own
Python operator on CPU (tests/golden/make_golden.py, reference flash_attention/flash_attention.py)
and (b) torch SDPA in float64 -- see tests/test_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np

FLT_MAX = float(np.finfo(np.float32).max)
LOG2E = 1.4426950408889634  # M_LOG2E


# --------------------------------------------------------------------------------------------
# dtype helpers (T in {fp16, bf16, fp32})
# --------------------------------------------------------------------------------------------
def round_bf16(x: np.ndarray) -> np.ndarray:
    """Round to the nearest bf16 (ties to even) via fp32, returned as float64."""
    f = np.ascontiguousarray(x, dtype=np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def round_to(x: np.ndarray, dtype: str) -> np.ndarray:
    """Round float64 values as the kernel does (value in fp32, then RNE to T)."""
    if dtype == "f16":
        return np.asarray(x, dtype=np.float32).astype(np.float16).astype(np.float64)
    if dtype == "bf16":
        return round_bf16(x)
    if dtype == "f32":
        return np.asarray(x, dtype=np.float32).astype(np.float64)
    raise ValueError(dtype)


def bf16_bits_to_f64(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def f64_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    f = np.ascontiguousarray(x, dtype=np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    return (((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF).astype(np.uint16)


def host_scale(softmax_scale: float) -> float:
    """`softmax_scale *= M_LOG2E` on a C++ float (reference csrc/flash_attention_api.cpp:87)."""
    return float(np.float32(np.float64(np.float32(softmax_scale)) * LOG2E))


# --------------------------------------------------------------------------------------------
# kernel restatement for one (batch, q-head)
# --------------------------------------------------------------------------------------------
def _attend_head(q: np.ndarray, k: np.ndarray, v: np.ndarray, s2: float, causal: bool, dtype: str,
                 block_n: int = 64, mask: str = "inf", block_m_ref: int = 128) -> np.ndarray:
    """O (float64, unrounded) for q [Sq, D], k/v [Sk, D] (float64 holding T values)."""
    sq, d = q.shape
    sk = k.shape[0]
    n_blocks = -(-sk // block_n)
    rows = np.arange(sq)[:, None]
    out = np.zeros((sq, d), dtype=np.float64)

    if mask == "inf":
        m = np.full((sq, 1), -np.inf)
        l = np.zeros((sq, 1))
        o = np.zeros((sq, d))
        # (the kernel's causal block skip only drops blocks whose scores are all masked for every
        #  row of a wave; such blocks contribute exactly 0 here, so all blocks are visited)
        for j in range(n_blocks):
            cols = np.arange(j * block_n, (j + 1) * block_n)[None, :]
            kb = k[j * block_n:(j + 1) * block_n]
            vb = v[j * block_n:(j + 1) * block_n]
            s = q @ kb.T
            if kb.shape[0] < block_n:  # OOB columns of the tail block
                s = np.concatenate([s, np.zeros((sq, block_n - kb.shape[0]))], axis=1)
                vb = np.concatenate([vb, np.zeros((block_n - vb.shape[0], d))], axis=0)
            masked = cols >= sk
            if causal:
                masked = masked | (sq - rows > sk - cols)
            s = np.where(masked, -np.inf, s)
            m_new = np.maximum(m, s.max(axis=1, keepdims=True))
            m_sc = np.where(m_new == -np.inf, 0.0, m_new * s2)
            with np.errstate(invalid="ignore"):
                alpha = np.exp2(m * s2 - m_sc)
            p = np.exp2(s * s2 - m_sc)
            l = l * alpha + p.sum(axis=1, keepdims=True)
            o = o * alpha + round_to(p, dtype) @ vb
            m = m_new
        inv = np.where(l == 0, 1.0, 1.0 / np.where(l == 0, 1.0, l))
        return o * inv

    if mask != "flt_max":
        raise ValueError(mask)
    # reference convention: -FLT_MAX everywhere, per-128-row tile block skip (mask.cuh:45-52)
    for t0 in range(0, sq, block_m_ref):
        qt = q[t0:t0 + block_m_ref]
        bm = qt.shape[0]
        trows = np.arange(t0, t0 + bm)[:, None]
        m = np.full((bm, 1), -FLT_MAX)
        l = np.zeros((bm, 1))
        o = np.zeros((bm, d))
        for j in range(n_blocks):
            if causal:
                n_block_max = -(-((sk - sq) + (t0 // block_m_ref + 1) * block_m_ref) // block_n)
                if j >= n_block_max:
                    continue
            cols = np.arange(j * block_n, (j + 1) * block_n)[None, :]
            kb = k[j * block_n:(j + 1) * block_n]
            vb = v[j * block_n:(j + 1) * block_n]
            s = qt @ kb.T
            if kb.shape[0] < block_n:
                s = np.concatenate([s, np.zeros((bm, block_n - kb.shape[0]))], axis=1)
                vb = np.concatenate([vb, np.zeros((block_n - vb.shape[0], d))], axis=0)
            masked = cols >= sk
            if causal:
                masked = masked | (sq - trows > sk - cols)
            s = np.where(masked, -FLT_MAX, s)
            m_old = m
            m = np.maximum(m, s.max(axis=1, keepdims=True))
            alpha = np.exp2((m_old - m) * s2)
            l = l * alpha
            o = o * alpha
            p = np.exp2(s * s2 - m * s2)
            l = l + p.sum(axis=1, keepdims=True)
            o = o + round_to(p, dtype) @ vb
        inv = np.where(l == 0, 1.0, 1.0 / np.where(l == 0, 1.0, l))
        out[t0:t0 + bm] = o * inv
    return out


def flash_attention_fwd(q: np.ndarray, k: np.ndarray, v: np.ndarray, softmax_scale: float, causal: bool,
                        dtype: str, mask: str = "inf", rounded: bool = True) -> np.ndarray:
    """Restatement of the host API + kernel (reference csrc/flash_attention_api.cpp:14-135).

    q [B, Hq, Sq, D], k/v [B, Hkv, Sk, D] as float64 arrays holding T-representable values.
    Returns O [B, Hq, Sq, D] in float64 (rounded to T when ``rounded``).
    """
    b, hq, sq, d = q.shape
    hkv, sk = k.shape[1], k.shape[2]
    if hq % hkv != 0:
        raise ValueError("number of heads in q must be multiple of number of heads in k and v")
    group = hq // hkv
    s2 = host_scale(softmax_scale)
    pack = sq == 1  # reference :72-83
    if pack:
        q = q.reshape(b, hkv, group, d)
        causal = False
        hq_eff, g_eff = hkv, 1
    else:
        hq_eff, g_eff = hq, group
    out = np.zeros(q.shape, dtype=np.float64)
    for bi in range(b):
        for h in range(hq_eff):
            out[bi, h] = _attend_head(q[bi, h], k[bi, h // g_eff], v[bi, h // g_eff], s2, causal, dtype,
                                      mask=mask)
    if pack:
        out = out.reshape(b, hq, 1, d)
    return round_to(out, dtype) if rounded else out


def fully_masked_rows(sq: int, sk: int, causal: bool) -> np.ndarray:
    """Boolean [Sq] of rows that see no key (where the two mask conventions differ)."""
    m = np.arange(sq)
    if not causal or sq == 1:
        return np.zeros(sq, dtype=bool)
    return m < sq - sk


def attention_flops(b: int, hq: int, sq: int, sk: int, d: int, causal: bool) -> float:
    """FA convention: 4*B*Hq*Sq*Sk*D, halved when causal."""
    f = 4.0 * b * hq * sq * sk * d
    return f / 2 if causal else f


def attention_bytes(b: int, hq: int, hkv: int, sq: int, sk: int, d: int, elem: int) -> int:
    """Algorithmic HBM bytes: |Q| + |O| + |K| + |V|."""
    return (2 * b * hq * sq * d + 2 * b * hkv * sk * d) * elem


def sdpa_reference_f64(q: np.ndarray, k: np.ndarray, v: np.ndarray, softmax_scale: float, causal: bool,
                       bottom_right: bool = True) -> np.ndarray:
    """Plain softmax(QK^T*scale)V in float64 (no online softmax, no P rounding); GQA by head index."""
    b, hq, sq, d = q.shape
    hkv, sk = k.shape[1], k.shape[2]
    g = hq // hkv
    out = np.zeros((b, hq, sq, d))
    for bi in range(b):
        for h in range(hq):
            s = q[bi, h] @ k[bi, h // g].T * softmax_scale
            if causal:
                rows = np.arange(sq)[:, None]
                cols = np.arange(sk)[None, :]
                off = (sk - sq) if bottom_right else 0
                s = np.where(cols > rows + off, -np.inf, s)
            mx = s.max(axis=1, keepdims=True)
            mx = np.where(np.isfinite(mx), mx, 0.0)
            p = np.exp(s - mx)
            den = p.sum(axis=1, keepdims=True)
            out[bi, h] = (p / np.where(den == 0, 1.0, den)) @ v[bi, h // g]
    return out


def rope_rotate(x: np.ndarray, cos: np.ndarray, sin: np.ndarray, dtype: str) -> np.ndarray:
    """Rotate-half RoPE as the gfx950 kernels compute it (csrc/fa_rope.hip, fa_fwd_kernels.hpp rope8).

    Convention of the reference's caller (reference models/rope_attn_fwd.py:8-12 rotate_half,
    :14-38 apply_rotary_pos_emb): out = x * cos + rotate_half(x) * sin, rotate_half([a, b]) = [-b, a]
    over the last dim. Arithmetic: t = fp32(rot * sin), out = fp32(x * cos + t) (one fma), rounded
    once (RNE) to T. x [..., S, D], cos / sin broadcastable to it, float64 arrays holding T values.
    """
    half = x.shape[-1] // 2
    rot = np.concatenate([-x[..., half:], x[..., :half]], axis=-1)
    t = round_to(rot * sin, "f32")
    return round_to(round_to(x * cos + t, "f32"), dtype)


__all__ = ["rope_rotate", "flash_attention_fwd", "sdpa_reference_f64", "round_to", "round_bf16", "host_scale",
           "bf16_bits_to_f64", "f64_to_bf16_bits", "fully_masked_rows", "attention_flops",
           "attention_bytes", "FLT_MAX", "LOG2E", "math"]
