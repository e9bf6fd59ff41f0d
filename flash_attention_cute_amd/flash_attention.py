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
"""
from __future__ import annotations

import warnings

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
