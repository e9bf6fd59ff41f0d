"""``flash_attention::forward`` custom op and ``flash_attn_func`` for MI355X.

Host-side mirror of reference flash_attention/flash_attention.py:1-53 -- same op name, schema,
registrations, default-scale rule and wrapper behaviour:

* ``torch.library.custom_op("flash_attention::forward", mutates_args=())`` whose default (CPU)
  implementation is ``F.scaled_dot_product_attention`` (reference :6-15);
* ``register_kernel(..., "cuda")`` -- ROCm devices report device type "cuda" -- which zero-pads
  the head dim to a multiple of 8, makes the last dim contiguous, calls the gfx950 extension
  (``flash_attention_fwd``) and slices the padding off again (reference :17-38);
* ``register_fake`` returning ``empty_like(q)`` (reference :40-43);
* ``flash_attn_func(q, k, v, softmax_scale=None, causal=False)`` with ``scale = D ** -0.5``
  computed on the UNPADDED head dim (reference :46-53).

GPU tensors always go through the hand-written HIP kernel: if the extension failed to load, the
"cuda" kernel raises instead of falling back to a PyTorch implementation.

Beyond the reference (its README.md:18 lists varlen as a TODO): ``flash_attention::varlen_forward``
/ ``flash_attn_varlen_func`` over packed variable-length sequences described by int32 ``cu_seqlens``
prefix sums (the layout a padding mask is lowered to; ``hf_attention`` does that lowering), with the
same registrations (CPU default, "cuda" kernel, fake) and the same pad / contiguity wrapper.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional

import torch

from .load_cpp_extention import load_extension

try:
    flash_attention_cuda = load_extension()
    _load_error = None
except Exception as e:  # noqa: BLE001 -- surfaced when a GPU tensor reaches the op
    flash_attention_cuda = None
    _load_error = e


@torch.library.custom_op("flash_attention::forward", mutates_args=())
def flash_attention_forward(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, softmax_scale: float = None,
                            causal: bool = False) -> torch.Tensor:
    # q: [batch_size, n_heads, q_seq_len, d]; k, v: [batch_size, n_heads_kv, kv_seq_len, d]
    # Non-GPU default, as in the reference: torch SDPA (top-left causal, no GQA expansion).
    warnings.warn("Flash Attention only support cuda now, fallback to pytorch implementation.",
                  stacklevel=2)
    return torch.nn.functional.scaled_dot_product_attention(q, k, v, scale=softmax_scale, is_causal=causal)


@torch.library.register_kernel("flash_attention::forward", "cuda")
def flash_attention_forward_cuda(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, softmax_scale: float = None,
                                 causal: bool = False) -> torch.Tensor:
    if flash_attention_cuda is None:
        raise RuntimeError(f"gfx950 flash attention extension is not available: {_load_error!r}")
    head_dim = q.size(3)
    need_padding = head_dim % 8 != 0
    if need_padding:
        pad = [0, 8 - head_dim % 8]
        q = torch.nn.functional.pad(q, pad)
        k = torch.nn.functional.pad(k, pad)
        v = torch.nn.functional.pad(v, pad)
    q = q.contiguous() if q.stride(3) != 1 else q
    k = k.contiguous() if k.stride(3) != 1 else k
    v = v.contiguous() if v.stride(3) != 1 else v
    attn = flash_attention_cuda.flash_attention_fwd(q, k, v, softmax_scale, causal)
    if need_padding:
        attn = attn[:, :, :, :head_dim]
    return attn


@torch.library.register_fake("flash_attention::forward")
def flash_attention_forward_fake(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, softmax_scale: float = None,
                                 causal: bool = False) -> torch.Tensor:
    return torch.empty_like(q)


def flash_attn_func(q, k, v, softmax_scale=None, causal=False):
    # q: [batch_size, n_heads, q_seq_len, d]; k, v: [batch_size, n_heads_kv, kv_seq_len, d]
    softmax_scale = (q.size(-1) ** -0.5) if softmax_scale is None else softmax_scale
    return torch.ops.flash_attention.forward(q, k, v, softmax_scale, causal)


# ---------------------------------------------------------------------------------------------
# variable-length (packed) sequences -- no reference counterpart (reference README.md:18 TODO)
# ---------------------------------------------------------------------------------------------
def split_errors(reset: bool = False) -> int:
    """Key-split hand-offs on the current device that timed out since the last reset (include/fa_gfx950.h
    ``fa_split_errors``): a causal block split over two workgroups whose second piece did not see its
    partner's partial result within ~1 s, so its rows are wrong. 0 in a healthy run; one host
    synchronisation."""
    from . import _debug

    return int(_debug.lib().fa_split_errors(1 if reset else 0))


def _bottom_right_causal(sq: int, sk: int, device) -> torch.Tensor:
    """[sq, sk] bool, True = visible: key n is visible to query m iff n <= m + sk - sq
    (the kernel's causal convention, reference csrc/mask.cuh:37-39)."""
    m = torch.arange(sq, device=device)[:, None]
    n = torch.arange(sk, device=device)[None, :]
    return n <= m + (sk - sq)


@torch.library.custom_op("flash_attention::varlen_forward", mutates_args=())
def flash_attention_varlen_forward(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_seqlens_q: torch.Tensor,
                                   cu_seqlens_k: torch.Tensor, max_seqlen_q: int, max_seqlen_k: int,
                                   softmax_scale: float = None, causal: bool = False,
                                   window_left: int = -1) -> torch.Tensor:
    # q: [total_q, n_heads, d]; k, v: [total_k, n_heads_kv, d]; cu_seqlens_*: int32 [batch_size + 1].
    # Non-GPU default: per-sequence torch SDPA with the kernel's semantics (bottom-right causal,
    # GQA, rows that see no key are 0; window_left >= 0: the local window per sequence).
    warnings.warn("Flash Attention only support cuda now, fallback to pytorch implementation.", stacklevel=2)
    out = torch.zeros_like(q)
    cq, ck = cu_seqlens_q.tolist(), cu_seqlens_k.tolist()
    for b in range(len(cq) - 1):
        q0, q1, k0, k1 = cq[b], cq[b + 1], ck[b], ck[b + 1]
        if q1 == q0 or k1 == k0:
            continue
        qs, ks, vs = (t.transpose(0, 1).unsqueeze(0) for t in (q[q0:q1], k[k0:k1], v[k0:k1]))
        if window_left >= 0:
            mask = _window_mask(q1 - q0, k1 - k0, window_left, causal, q.device)
        else:
            mask = _bottom_right_causal(q1 - q0, k1 - k0, q.device) if causal else None
        o = torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, attn_mask=mask, scale=softmax_scale,
                                                             enable_gqa=True)
        if mask is not None:  # rows with no visible key (Sq_b > Sk_b) are 0, as on the GPU
            o = o.masked_fill(~mask.any(dim=1)[None, None, :, None], 0)
        out[q0:q1] = o[0].transpose(0, 1)
    return out


@torch.library.register_kernel("flash_attention::varlen_forward", "cuda")
def flash_attention_varlen_forward_cuda(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                                        cu_seqlens_q: torch.Tensor, cu_seqlens_k: torch.Tensor, max_seqlen_q: int,
                                        max_seqlen_k: int, softmax_scale: float = None,
                                        causal: bool = False, window_left: int = -1) -> torch.Tensor:
    if flash_attention_cuda is None:
        raise RuntimeError(f"gfx950 flash attention extension is not available: {_load_error!r}")
    head_dim = q.size(2)
    need_padding = head_dim % 8 != 0
    if need_padding:
        pad = [0, 8 - head_dim % 8]
        q = torch.nn.functional.pad(q, pad)
        k = torch.nn.functional.pad(k, pad)
        v = torch.nn.functional.pad(v, pad)
    q = q.contiguous() if q.stride(2) != 1 else q
    k = k.contiguous() if k.stride(2) != 1 else k
    v = v.contiguous() if v.stride(2) != 1 else v
    attn = flash_attention_cuda.flash_attention_varlen_fwd(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                                                           max_seqlen_k, softmax_scale, causal, int(window_left))
    if need_padding:
        attn = attn[:, :, :head_dim]
    return attn


@torch.library.register_fake("flash_attention::varlen_forward")
def flash_attention_varlen_forward_fake(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                                        softmax_scale=None, causal=False, window_left=-1):
    return torch.empty_like(q)


def _check_varlen_enabled() -> bool:
    """FA_CHECK_VARLEN, read at every call (setting it after import takes effect)."""
    return os.environ.get("FA_CHECK_VARLEN", "0") not in ("", "0")


def _check_varlen_maxima(cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k):
    """Raise if a sequence is longer than the max_seqlen the caller passed (FA_CHECK_VARLEN=1)."""
    for name, cu, mx in (("q", cu_seqlens_q, max_seqlen_q), ("k", cu_seqlens_k, max_seqlen_k)):
        longest = int((cu[1:] - cu[:-1]).max()) if cu.numel() > 1 else 0
        if longest > mx:
            raise ValueError(f"max_seqlen_{name}={mx} is smaller than the longest sequence ({longest}) "
                             f"in cu_seqlens_{name}")


def flash_attn_varlen_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, softmax_scale=None,
                           causal=False, window_left=-1):
    """Attention over packed sequences: q [total_q, Hq, D], k/v [total_k, Hkv, D]; sequence b owns rows
    [cu_seqlens_q[b], cu_seqlens_q[b+1]) of q and [cu_seqlens_k[b], cu_seqlens_k[b+1]) of k/v
    (int32, on q's device). ``max_seqlen_q`` / ``max_seqlen_k`` must be the true maxima: the GPU grid
    is sized by ``max_seqlen_q``, so a smaller value leaves the rows of longer sequences uncomputed.
    With ``FA_CHECK_VARLEN=1`` in the environment (read at every call) both are verified against
    ``cu_seqlens_*`` (one host sync per call; off by default, as in the reference's varlen API).
    ``window_left >= 0``: the local window of ``flash_attn_window_func`` within each sequence."""
    softmax_scale = (q.size(-1) ** -0.5) if softmax_scale is None else softmax_scale
    if _check_varlen_enabled():
        _check_varlen_maxima(cu_seqlens_q, cu_seqlens_k, int(max_seqlen_q), int(max_seqlen_k))
    return torch.ops.flash_attention.varlen_forward(q, k, v, cu_seqlens_q, cu_seqlens_k, int(max_seqlen_q),
                                                    int(max_seqlen_k), softmax_scale, causal, int(window_left))


# ---------------------------------------------------------------------------------------------
# padded batches -- per-sequence ranges inside dense tensors (include/fa_gfx950.h
# fa_fwd_gfx950_padded); no reference counterpart (the reference drops attention_mask,
# models/rope_attn_fwd.py:40-64). An HF left / right padding mask is lowered to this: the KV cache
# and the projections are read in place, decode steps keep the q-head pack and split-KV kernel.
# ---------------------------------------------------------------------------------------------
@torch.library.custom_op("flash_attention::padded_forward", mutates_args=())
def flash_attention_padded_forward(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, k_start: torch.Tensor,
                                   k_end: torch.Tensor, q_start: Optional[torch.Tensor] = None,
                                   q_end: Optional[torch.Tensor] = None, softmax_scale: float = None,
                                   causal: bool = False, window_left: int = -1) -> torch.Tensor:
    # q: [B, Hq, Sq, D]; k, v: [B, Hkv, Sk, D]; batch row b's keys are positions [k_start[b], k_end[b])
    # and (optional) its queries [q_start[b], q_end[b]). Non-GPU default: per-sequence torch SDPA with
    # the kernel's semantics (bottom-right causal per sequence, GQA, rows outside / with no key 0).
    warnings.warn("Flash Attention only support cuda now, fallback to pytorch implementation.", stacklevel=2)
    out = torch.zeros_like(q)
    sq = q.size(2)
    ks, ke = k_start.tolist(), k_end.tolist()
    qs = q_start.tolist() if q_start is not None else [0] * q.size(0)
    qe = q_end.tolist() if q_end is not None else [sq] * q.size(0)
    for b in range(q.size(0)):
        q0, q1, k0, k1 = qs[b], qe[b], ks[b], ke[b]
        if q1 <= q0 or k1 <= k0:
            continue
        if window_left >= 0:
            mask = _window_mask(q1 - q0, k1 - k0, window_left, causal, q.device)
        else:
            # bottom-right per sequence (one query row sees every key, as the Sq == 1 pack's non-causal)
            mask = _bottom_right_causal(q1 - q0, k1 - k0, q.device) if causal else None
        o = torch.nn.functional.scaled_dot_product_attention(q[b:b + 1, :, q0:q1], k[b:b + 1, :, k0:k1],
                                                             v[b:b + 1, :, k0:k1], attn_mask=mask,
                                                             scale=softmax_scale, enable_gqa=True)
        if mask is not None:
            o = o.masked_fill(~mask.any(dim=1)[None, None, :, None], 0)
        out[b:b + 1, :, q0:q1] = o
    return out


@torch.library.register_kernel("flash_attention::padded_forward", "cuda")
def flash_attention_padded_forward_cuda(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, k_start: torch.Tensor,
                                        k_end: torch.Tensor, q_start: Optional[torch.Tensor] = None,
                                        q_end: Optional[torch.Tensor] = None, softmax_scale: float = None,
                                        causal: bool = False, window_left: int = -1) -> torch.Tensor:
    if flash_attention_cuda is None:
        raise RuntimeError(f"gfx950 flash attention extension is not available: {_load_error!r}")
    head_dim = q.size(3)
    need_padding = head_dim % 8 != 0
    if need_padding:
        pad = [0, 8 - head_dim % 8]
        q = torch.nn.functional.pad(q, pad)
        k = torch.nn.functional.pad(k, pad)
        v = torch.nn.functional.pad(v, pad)
    q = q.contiguous() if q.stride(3) != 1 else q
    k = k.contiguous() if k.stride(3) != 1 else k
    v = v.contiguous() if v.stride(3) != 1 else v
    attn = flash_attention_cuda.flash_attention_padded_fwd(q, k, v, q_start, q_end, k_start, k_end, softmax_scale,
                                                           causal, int(window_left))
    if need_padding:
        attn = attn[:, :, :, :head_dim]
    return attn


@torch.library.register_fake("flash_attention::padded_forward")
def flash_attention_padded_forward_fake(q, k, v, k_start, k_end, q_start=None, q_end=None, softmax_scale=None,
                                        causal=False, window_left=-1):
    return torch.empty_like(q)


def flash_attn_padded_func(q, k, v, k_start, k_end, q_start=None, q_end=None, softmax_scale=None, causal=False,
                           window_left=-1):
    """Attention over a padded batch read in place: q [B, Hq, Sq, D], k / v [B, Hkv, Sk, D] (any strides,
    e.g. HF projection views and the KV cache), batch row b's real keys at positions
    ``[k_start[b], k_end[b])`` and, optionally, its real queries at ``[q_start[b], q_end[b])`` (int32 [B]
    on q's device; default: every query row). Causal / window masks are bottom-right aligned per
    sequence; output rows outside the query ranges are 0. No host synchronisation (graph-capturable);
    Sq == 1 takes the q-head pack and the split-KV decode kernel."""
    softmax_scale = (q.size(-1) ** -0.5) if softmax_scale is None else softmax_scale
    return torch.ops.flash_attention.padded_forward(q, k, v, k_start, k_end, q_start, q_end, softmax_scale, causal,
                                                    int(window_left))


# ---------------------------------------------------------------------------------------------
# RoPE: the reference rotates q and k with elementwise torch ops before the
# call (reference models/rope_attn_fwd.py:8-38, :88). Here k is rotated in one HIP pass
# (``apply_rope``; the KV cache stores rotated keys) and q inside the attention kernel's Q load
# (``flash_attn_rope_func``).
# ---------------------------------------------------------------------------------------------
def _rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, H, S, D] * cos + rotate_half(x) * sin with cos / sin [B|1, S, D] or [S, D], in fp32,
    rounded once to x's dtype (the kernels' arithmetic up to the fma)."""
    cos = cos if cos.dim() == 3 else cos[None]
    sin = sin if sin.dim() == 3 else sin[None]
    xf = x.float()
    half = x.shape[-1] // 2
    rot = torch.cat((-xf[..., half:], xf[..., :half]), dim=-1)
    return (xf * cos.float()[:, None] + rot * sin.float()[:, None]).to(x.dtype)


@torch.library.custom_op("flash_attention::rope_apply", mutates_args=())
def flash_attention_rope_apply(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    return _rope_reference(x, cos, sin)


@torch.library.register_kernel("flash_attention::rope_apply", "cuda")
def flash_attention_rope_apply_cuda(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    if flash_attention_cuda is None:
        raise RuntimeError(f"gfx950 flash attention extension is not available: {_load_error!r}")
    x = x.contiguous() if x.stride(3) != 1 else x
    return flash_attention_cuda.rope_apply(x, cos.to(x.dtype), sin.to(x.dtype))


@torch.library.register_fake("flash_attention::rope_apply")
def flash_attention_rope_apply_fake(x, cos, sin):
    return torch.empty_like(x)


@torch.library.custom_op("flash_attention::rope_forward", mutates_args=())
def flash_attention_rope_forward(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cos: torch.Tensor,
                                 sin: torch.Tensor, softmax_scale: float = None, causal: bool = False) -> torch.Tensor:
    # q unrotated [B, Hq, Sq, D]; k (already rotated), v [B, Hkv, Sk, D]; cos / sin of q's positions.
    warnings.warn("Flash Attention only support cuda now, fallback to pytorch implementation.", stacklevel=2)
    return torch.nn.functional.scaled_dot_product_attention(_rope_reference(q, cos, sin), k, v, scale=softmax_scale,
                                                            is_causal=causal)


@torch.library.register_kernel("flash_attention::rope_forward", "cuda")
def flash_attention_rope_forward_cuda(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cos: torch.Tensor,
                                      sin: torch.Tensor, softmax_scale: float = None,
                                      causal: bool = False) -> torch.Tensor:
    if flash_attention_cuda is None:
        raise RuntimeError(f"gfx950 flash attention extension is not available: {_load_error!r}")
    cos, sin = cos.to(q.dtype), sin.to(q.dtype)
    if q.size(3) % 8 != 0:  # padded head dims: rotate first (the halves are those of the real D)
        return flash_attention_forward_cuda(flash_attention_rope_apply_cuda(q, cos, sin), k, v, softmax_scale, causal)
    q = q.contiguous() if q.stride(3) != 1 else q
    k = k.contiguous() if k.stride(3) != 1 else k
    v = v.contiguous() if v.stride(3) != 1 else v
    return flash_attention_cuda.flash_attention_rope_fwd(q, k, v, cos, sin, softmax_scale, causal)


@torch.library.register_fake("flash_attention::rope_forward")
def flash_attention_rope_forward_fake(q, k, v, cos, sin, softmax_scale=None, causal=False):
    return torch.empty_like(q)


def apply_rope(x, cos, sin):
    """Rotate-half RoPE of x [B, H, S, D] with cos / sin [B|1, S, D] or [S, D] (one HIP pass on GPU)."""
    return torch.ops.flash_attention.rope_apply(x, cos, sin)


def flash_attn_rope_func(q, k, v, cos, sin, softmax_scale=None, causal=False):
    """``flash_attn_func(apply_rope(q, cos, sin), k, v, ...)`` with the rotation of q fused into the
    attention kernel's Q load; k must already be rotated (``apply_rope``)."""
    softmax_scale = (q.size(-1) ** -0.5) if softmax_scale is None else softmax_scale
    return torch.ops.flash_attention.rope_forward(q, k, v, cos, sin, softmax_scale, causal)


# ---------------------------------------------------------------------------------------------
# Local (sliding-window) attention -- the reference computes the Qwen2 sliding window and then
# ignores it (reference models/rope_attn_fwd.py:95-101); include/fa_gfx950.h fa_fwd_gfx950_window.
# ---------------------------------------------------------------------------------------------
def _window_mask(sq: int, sk: int, window_left: int, causal: bool, device) -> torch.Tensor:
    """[sq, sk] bool, True = visible: key n is visible to query m iff n >= m + sk - sq - window_left
    and, with causal, n <= m + sk - sq (transformers' sliding_window_causal_mask_function with
    sliding_window = window_left + 1, bottom-right aligned as the kernel's causal mask)."""
    m = torch.arange(sq, device=device)[:, None]
    n = torch.arange(sk, device=device)[None, :]
    vis = n >= m + (sk - sq) - window_left
    if causal:
        vis = vis & (n <= m + (sk - sq))
    return vis


@torch.library.custom_op("flash_attention::window_forward", mutates_args=())
def flash_attention_window_forward(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, window_left: int,
                                   softmax_scale: float = None, causal: bool = False) -> torch.Tensor:
    # q: [B, Hq, Sq, D]; k, v: [B, Hkv, Sk, D]. Non-GPU default: torch SDPA under the window mask
    # (GQA expanded; rows that see no key are 0, as on the GPU).
    warnings.warn("Flash Attention only support cuda now, fallback to pytorch implementation.", stacklevel=2)
    mask = _window_mask(q.size(2), k.size(2), window_left, causal, q.device)
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=softmax_scale,
                                                         enable_gqa=True)
    return o.masked_fill(~mask.any(dim=1)[None, None, :, None], 0)


@torch.library.register_kernel("flash_attention::window_forward", "cuda")
def flash_attention_window_forward_cuda(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, window_left: int,
                                        softmax_scale: float = None, causal: bool = False) -> torch.Tensor:
    if flash_attention_cuda is None:
        raise RuntimeError(f"gfx950 flash attention extension is not available: {_load_error!r}")
    if window_left < 0:
        raise ValueError(f"window_left must be >= 0 (got {window_left})")
    head_dim = q.size(3)
    need_padding = head_dim % 8 != 0
    if need_padding:
        pad = [0, 8 - head_dim % 8]
        q = torch.nn.functional.pad(q, pad)
        k = torch.nn.functional.pad(k, pad)
        v = torch.nn.functional.pad(v, pad)
    q = q.contiguous() if q.stride(3) != 1 else q
    k = k.contiguous() if k.stride(3) != 1 else k
    v = v.contiguous() if v.stride(3) != 1 else v
    attn = flash_attention_cuda.flash_attention_window_fwd(q, k, v, int(window_left), softmax_scale, causal)
    if need_padding:
        attn = attn[:, :, :, :head_dim]
    return attn


@torch.library.register_fake("flash_attention::window_forward")
def flash_attention_window_forward_fake(q, k, v, window_left, softmax_scale=None, causal=False):
    return torch.empty_like(q)


def flash_attn_window_func(q, k, v, window_left, softmax_scale=None, causal=False):
    """``flash_attn_func`` where query m sees only keys n >= m + Sk - Sq - window_left: a sliding
    window of ``window_left + 1`` keys ending at the (bottom-right) diagonal with ``causal``.
    transformers' ``sliding_window`` W is ``window_left = W - 1`` (flash-attn ``window_size=(W - 1,
    -1)``)."""
    softmax_scale = (q.size(-1) ** -0.5) if softmax_scale is None else softmax_scale
    return torch.ops.flash_attention.window_forward(q, k, v, int(window_left), softmax_scale, causal)
