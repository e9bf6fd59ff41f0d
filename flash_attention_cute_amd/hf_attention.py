"""Drop-in HF attention ``forward`` that routes the attention core through ``flash_attn_func``.

Mirror of reference models/rope_attn_fwd.py:1-120 (the caller of the hot path),
kept call-site identical -- q/k/v projections viewed as strided [B, H, S, D] (seq stride H*D), RoPE,
KV-cache update, ``flash_attn_func(q, k, v, causal=module.is_causal, softmax_scale=self.scaling)``,
``transpose(1, 2)``, ``reshape(...).contiguous()``, ``o_proj`` -- with the three defects SURVEY.md 3.2
verified against the installed transformers fixed:

1. ``self.config.use_sliding_window`` raised AttributeError on ``LlamaConfig``
   (reference models/rope_attn_fwd.py:97): read with ``getattr(..., False)``; a sliding window
   that cuts the visible keys runs the local-window kernel (``flash_attn_window_func``,
   window_left = sliding_window - 1) instead of being ignored as in the reference (:95-101);
2. HF passes the cache as ``past_key_values=`` (plural) while the reference takes
   ``past_key_value`` (:71) and silently drops the cache on decode: both names are accepted;
3. decode (Sq == 1) with ``is_causal=True`` must see every cached key: the GPU kernel's causal mask
   is bottom-right aligned (key n visible to query m iff n <= m + Sk - Sq) and the host API drops
   the causal flag for Sq == 1 (reference csrc/flash_attention_api.cpp:81), but the op's CPU
   default (torch SDPA, top-left) would let the query see only key 0 -- so the flag is passed as
   ``module.is_causal and Sq > 1``, which is the same computation on the GPU and correct on CPU.

Because the op's output inherits q's strides (reference csrc/flash_attention_api.cpp:85, kept in
csrc/flash_attention_api.cpp), ``attn.transpose(1, 2).reshape(B, S, -1)`` is copy-free.
"""
from __future__ import annotations

import weakref
from typing import NamedTuple, Optional, Tuple

import torch
from torch import nn

from .flash_attention import (_bottom_right_causal, _window_mask, apply_rope, flash_attn_func, flash_attn_padded_func,
                              flash_attn_rope_func, flash_attn_varlen_func, flash_attn_window_func)

# On GPU tensors the patched forward rotates k with one HIP pass (apply_rope) and q inside the
# attention kernel (flash_attn_rope_func) instead of the reference's elementwise torch ops
# (reference models/rope_attn_fwd.py:14-38). False restores the reference's order of operations
# (A/B measurements, scripts/benchmark_llm.py --no-fused-rope).
FUSE_ROPE = True

# How an HF attention mask is lowered (``lower_mask``: every check computed on the device):
#  * eager calls read the checks back with ONE host synchronisation per call and take the exact
#    path -- the dense kernels when the mask hides nothing beyond causal / window, the padded kernel
#    in place when each sequence's real tokens are one run, the packed varlen kernel for other
#    padding, NotImplementedError for masks none of them expresses;
#  * under HIP-graph capture (torch.cuda.is_current_stream_capturing()) nothing is read back: the
#    padded kernel always runs, and a batch row whose mask it cannot express gets an empty range
#    (output 0) and is counted in a device-side error counter (``mask_errors()`` reads it);
#  * TRUST_PADDING_MASK = True skips the checks altogether (no synchronisation in eager calls
#    either): the mask is trusted to be causal + key padding with one real-token run per sequence
#    (left or right padding, what ``generate`` builds).
TRUST_PADDING_MASK = False

_MASK_ERRORS = {}  # device -> int32 [1] count of batch rows whose mask the padded kernel could not express


def mask_errors(device=None, reset: bool = False) -> int:
    """Batch rows (summed over calls) whose attention mask was not expressible while lowering without
    a host synchronisation (graph capture); their outputs were zeroed. One host synchronisation."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    t = _MASK_ERRORS.get(dev)
    if t is None:
        return 0
    n = int(t.item())
    if reset:
        t.zero_()
    return n


def _error_counter(dev: torch.device) -> torch.Tensor:
    t = _MASK_ERRORS.get(dev)
    if t is None:  # (created by the first eager call, ahead of a capture's warm-up)
        t = _MASK_ERRORS[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return t


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    """[x1, x2] -> [-x2, x1] over the last dim (reference models/rope_attn_fwd.py:8-12)."""
    half = x.shape[-1] // 2
    return torch.cat((-x[..., half:], x[..., :half]), dim=-1)


def apply_rotary_pos_emb(q, k, cos, sin, position_ids=None, unsqueeze_dim=1):
    """RoPE on q [B,Hq,S,D] and k [B,Hkv,S,D] (reference models/rope_attn_fwd.py:14-38).

    Elementwise on the strided projection views, so the outputs keep the [B,S,H,D] physical layout.
    """
    cos = cos.unsqueeze(unsqueeze_dim)
    sin = sin.unsqueeze(unsqueeze_dim)
    return q * cos + rotate_half(q) * sin, k * cos + rotate_half(k) * sin


class Lowering(NamedTuple):
    """An HF attention mask lowered to per-sequence ranges (all device tensors; ``lower_mask``)."""

    kv_valid: torch.Tensor  # [B, Sk] bool: keys some real query row attends
    q_valid: torch.Tensor   # [B, Sq] bool: query rows whose own token is real
    k_start: torch.Tensor   # [B] int32: the real keys are positions [k_start, k_end) ...
    k_end: torch.Tensor
    q_start: torch.Tensor   # ... the real query rows [q_start, q_end)
    q_end: torch.Tensor
    shape_ok: torch.Tensor  # [B] bool: on every real query row the mask is "causal / window AND key real"
    run_ok: torch.Tensor    # [B] bool: real keys and real query rows each one run, the last real query's
                            # own key the last real key (the kernels' bottom-right alignment)
    dense: torch.Tensor     # [] bool: every range is the whole dimension (nothing hidden beyond the shape)


def _first_last_count(valid: torch.Tensor):
    n = valid.shape[1]
    idx = torch.arange(n, device=valid.device)[None]
    first = torch.where(valid, idx, n).amin(1)
    last = torch.where(valid, idx, -1).amax(1)
    return first, last, valid.sum(1)


def lower_mask(attention_mask: Optional[torch.Tensor], sq: int, sk: int, causal: bool,
               window_left: Optional[int] = None) -> Optional[Lowering]:
    """Lower an HF attention mask to per-sequence query / key ranges, computed on the device with no
    host synchronisation (None: no mask).

    Accepted: a 2-D padding mask ``[B, Sk]`` (1 = real token; the queries are the last Sq keys, a
    dynamic cache), or the 4-D mask HF builds for SDPA / eager ``[B, 1, Sq, Sk]`` (bool, True =
    attend; or additive float, 0 = attend). With a causal 4-D mask each query row's own key position
    is read from the mask itself -- the last key a real row attends is its own token -- so the queries
    may sit anywhere in the keys: the last Sq of a dynamic cache, or mid-way through a static cache
    whose later slots are empty (the mask hides them). Padding query rows attend no key (left
    padding) or sit after the real rows (right padding). ``shape_ok`` holds where the mask is exactly
    "causal (up to the row's own key) AND inside the window AND key real" on every real row; anything
    else (chunked / document / custom masks) is for the caller to reject instead of being silently
    dropped as in the reference (models/rope_attn_fwd.py:40-64 ignores ``attention_mask``).
    """
    if attention_mask is None:
        return None
    m = attention_mask
    if sq > sk:
        raise NotImplementedError("flash_attention_cute_amd: attention_mask with more queries than keys")
    dev = m.device
    ar_q = torch.arange(sq, device=dev)
    n_ = torch.arange(sk, device=dev)
    if m.dim() == 2:
        if tuple(m.shape[1:]) != (sk,):
            raise NotImplementedError(f"flash_attention_cute_amd: 2-D attention_mask of shape {tuple(m.shape)} "
                                      f"does not cover the {sk} keys")
        kv_valid = m.bool()
        qpos = (ar_q + (sk - sq))[None]  # [1, Sq]
        q_valid = kv_valid[:, qpos[0]]
        shape_ok = torch.ones(m.shape[0], dtype=torch.bool, device=dev)
    elif m.dim() == 4:
        if m.shape[1] != 1 or m.shape[2] != sq or m.shape[3] != sk:
            raise NotImplementedError(f"flash_attention_cute_amd: 4-D attention_mask of shape {tuple(m.shape)} "
                                      f"(expected [B, 1, {sq}, {sk}])")
        a = m[:, 0] if m.dtype == torch.bool else (m[:, 0] == 0)
        own = torch.where(a, n_[None, None], -1).amax(2)  # [B, Sq] the last key each row attends
        if causal:
            # real rows: own key = offset + row; padding rows attend only earlier keys (right padding,
            # holes), none (left padding) or -- transformers / torch "unmask" rows that attend nothing --
            # every key. The offset is the largest own - row over the rows that attend some key but not
            # all of them; when no row qualifies (every row attends every key) the last query row is
            # the last key's.
            full = a.all(2)
            rel = torch.where((own >= 0) & ~full, own - ar_q[None], -1 - sk)
            off = rel.amax(1)
            off = torch.where(off < -sk, torch.full_like(off, sk - sq), off)
            q_valid = (own >= 0) & (own - ar_q[None] == off[:, None])
            qpos = off[:, None] + ar_q[None]  # [B, Sq]
        else:  # (a decode row, Sq == 1, no query range: computed whatever its position; real iff it
            # attends a key)
            q_valid = own >= 0
            qpos = own
        kv_valid = (a & q_valid[:, :, None]).any(1)
        shape = torch.ones(1, 1, sk, dtype=torch.bool, device=dev)
        if causal:
            shape = shape & (n_[None, None] <= qpos[:, :, None])
            if window_left is not None:
                shape = shape & (n_[None, None] >= qpos[:, :, None] - window_left)
        allowed = kv_valid[:, None, :] & shape
        # (rows that do not attend their own key are padding: their output is discarded)
        shape_ok = ~((a != allowed) & q_valid[:, :, None]).any(2).any(1)
        if causal:
            # ... and a padding row's own position holds a padding key: a row left out whose own key a
            # real row attends would be a real row the lowering drops (its output would be 0)
            inside = (qpos >= 0) & (qpos < sk)
            own_real = kv_valid.gather(1, qpos.clamp(0, sk - 1)) & inside
            shape_ok = shape_ok & ~(own_real & ~q_valid).any(1)
    else:
        raise NotImplementedError(f"flash_attention_cute_amd: attention_mask with {m.dim()} dims")
    k_first, k_last, k_cnt = _first_last_count(kv_valid)
    q_first, q_last, q_cnt = _first_last_count(q_valid)
    k_start = torch.where(k_cnt > 0, k_first, 0)
    k_end = k_start + k_cnt
    q_start = torch.where(q_cnt > 0, q_first, 0)
    q_end = q_start + q_cnt
    run_ok = ((k_last - k_first + 1 == k_cnt) | (k_cnt == 0)) & ((q_last - q_first + 1 == q_cnt) | (q_cnt == 0))
    if causal:  # the kernels' bottom-right alignment: the last real query's own key is the last real key
        last_own = qpos.expand(q_end.shape[0], sq).gather(1, (q_end - 1).clamp(min=0)[:, None])[:, 0]
        run_ok = run_ok & ((q_cnt == 0) | (k_end == last_own + 1))
    dense = ((k_start == 0) & (k_end == sk) & (q_start == 0) & (q_end == sq)).all()
    i32 = lambda t: t.to(torch.int32)  # noqa: E731
    return Lowering(kv_valid, q_valid, i32(k_start), i32(k_end), i32(q_start), i32(q_end), shape_ok, run_ok, dense)


def key_padding(attention_mask: Optional[torch.Tensor], sq: int, sk: int, causal: bool,
                window_left: Optional[int] = None) -> Optional[torch.Tensor]:
    """Per-token validity ``[B, Sk]`` (True = real token) of an HF attention mask, or None when it
    masks nothing beyond the plain causal (and, with ``window_left``, sliding-window) shape; masks the
    kernels cannot express raise NotImplementedError. ``lower_mask`` plus one host synchronisation."""
    low = lower_mask(attention_mask, sq, sk, causal, window_left)
    if low is None:
        return None
    if TRUST_PADDING_MASK:
        return low.kv_valid
    shape_ok, run_ok, dense = torch.stack([low.shape_ok.all(), low.run_ok.all(), low.dense]).tolist()
    _raise_unexpressible(shape_ok, run_ok, window_left)
    return None if dense else low.kv_valid


def _raise_unexpressible(shape_ok: bool, run_ok: bool, window_left: Optional[int]) -> None:
    if not shape_ok:
        raise NotImplementedError("flash_attention_cute_amd: only causal + key-padding attention masks are "
                                  "supported (this mask masks other scores)")
    if not run_ok and window_left is not None:
        # HF places the window on cache indices, the varlen kernel on the packed real tokens: the two
        # agree only when each sequence's real tokens are one contiguous run (left or right padding)
        raise NotImplementedError("flash_attention_cute_amd: a sliding window over padding that is not one "
                                  "contiguous run per sequence")


def padding_ranges(kv_valid: torch.Tensor, sq: int, check: bool = True):
    """[B, Sk] per-token validity -> int32 device tensors (k_start, k_end, q_start, q_end): batch row b's
    real keys are positions [k_start, k_end) and its real queries (the last Sq token positions) rows
    [q_start, q_end). None when some row's real tokens are not one contiguous run (``check``: one host
    synchronisation; check=False trusts the mask)."""
    sk = kv_valid.shape[1]
    idx = torch.arange(sk, device=kv_valid.device, dtype=torch.int32)[None]
    cnt = kv_valid.sum(1, dtype=torch.int32)
    first = torch.where(kv_valid, idx, sk).amin(1)
    if check:
        last = torch.where(kv_valid, idx, -1).amax(1)
        if bool(((last - first + 1 != cnt) & (cnt > 0)).any()):
            return None
    k_start = torch.where(cnt > 0, first, 0).to(torch.int32)
    k_end = k_start + cnt
    off = sk - sq  # query row i is token position off + i
    q_start = (k_start - off).clamp(0, sq).to(torch.int32)
    q_end = (k_end - off).clamp(0, sq).to(torch.int32)
    return k_start, k_end, q_start, q_end


def _padded_attention(query, key, value, ranges, causal, scaling, window_left=-1):
    """Padded batch read in place (``flash_attn_padded_func``) -> [B, Sq, Hq, D], padding rows 0. A decode
    step (Sq == 1) passes no query ranges, so it keeps the q-head pack and the split-KV kernel."""
    k_start, k_end, q_start, q_end = ranges
    if query.shape[2] == 1:
        q_start = q_end = None
    o = flash_attn_padded_func(query, key, value, k_start, k_end, q_start, q_end, softmax_scale=scaling,
                               causal=causal, window_left=window_left)
    return o.transpose(1, 2)


def _varlen_attention(query, key, value, kv_valid, q_valid, causal, scaling, window_left=-1):
    """Padded batch -> packed sequences -> ``flash_attn_varlen_func`` -> padded [B, Sq, Hq, D] (padding
    rows 0). q/k/v are [B, H, S, D] views. Every sequence's real query rows are the last of its real
    keys (``lower_mask``'s alignment), so the packed bottom-right causal mask is the original one."""
    b, hq, sq, d = query.shape
    hkv, sk = key.shape[1], key.shape[2]
    lens_q = q_valid.sum(1, dtype=torch.int32)
    lens_k = kv_valid.sum(1, dtype=torch.int32)
    cu_q = torch.nn.functional.pad(torch.cumsum(lens_q, 0, dtype=torch.int32), (1, 0))
    cu_k = torch.nn.functional.pad(torch.cumsum(lens_k, 0, dtype=torch.int32), (1, 0))
    idx_q = q_valid.flatten().nonzero().squeeze(1)
    idx_k = kv_valid.flatten().nonzero().squeeze(1)
    qp = query.transpose(1, 2).reshape(b * sq, hq, d).index_select(0, idx_q)
    kp = key.transpose(1, 2).reshape(b * sk, hkv, d).index_select(0, idx_k)
    vp = value.transpose(1, 2).reshape(b * sk, hkv, d).index_select(0, idx_k)
    o = flash_attn_varlen_func(qp, kp, vp, cu_q, cu_k, int(lens_q.max()), int(lens_k.max()), softmax_scale=scaling,
                               causal=causal, window_left=window_left)
    out = query.new_zeros(b * sq, hq, d)
    out.index_copy_(0, idx_q, o)
    return out.view(b, sq, hq, d)


def _capturing(t: torch.Tensor) -> bool:
    return t.is_cuda and torch.cuda.is_current_stream_capturing()


# The eager lowering of the last mask seen: (weak reference to the mask, its key, (lowering, path)). The
# decoder layers of one forward receive the SAME mask tensor, so the device lowering and its one host
# read run once per forward (per decode token), not once per layer. A hit needs the same live tensor
# object (a weak reference: a freed mask whose id or storage is reused never matches) at the same
# version counter (an in-place update misses). Never consulted under graph capture, whose lowering must
# be recorded in the graph itself.
_LOWER_MEMO: list = [None]


def _lowered_eager(attention_mask: Optional[torch.Tensor], sq: int, sk: int, causal: bool,
                   window_left: Optional[int]):
    """``lower_mask`` + the path it allows (one host read), memoised across the layers of one forward:
    (None, "dense") without a mask, else (lowering, "dense" | "padded" | "varlen")."""
    if attention_mask is None:
        return None, "dense"
    key = (tuple(attention_mask.shape), attention_mask.dtype, attention_mask.device, attention_mask._version, sq, sk,
           causal, window_left, TRUST_PADDING_MASK)
    memo = _LOWER_MEMO[0]
    if memo is not None and memo[0]() is attention_mask and memo[1] == key:
        return memo[2]
    low = lower_mask(attention_mask, sq, sk, causal, window_left)
    if TRUST_PADDING_MASK:
        path = "padded"
    else:
        shape_ok, run_ok, dense = torch.stack([low.shape_ok.all(), low.run_ok.all(), low.dense]).tolist()
        _raise_unexpressible(shape_ok, run_ok, window_left)
        path = "dense" if dense else "padded" if run_ok else "varlen"
    _LOWER_MEMO[0] = (weakref.ref(attention_mask), key, (low, path))
    return low, path


def _flash_attention_forward(module: nn.Module, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                             attention_mask: Optional[torch.Tensor], dropout: float = 0.0,
                             scaling: Optional[float] = None, sliding_window: Optional[int] = None,
                             softcap: Optional[float] = None, **kwargs) -> Tuple[torch.Tensor, None]:
    """Attention core (reference models/rope_attn_fwd.py:40-64): returns [B, Sq, Hq, D], None.

    Unlike the reference, ``attention_mask`` is honoured (``lower_mask``): a mask that hides nothing
    beyond causal / window runs the dense kernels; one real-token run per sequence (left / right
    padding, a static cache's empty slots) runs the padded kernel on the tensors in place; other
    padding is packed for the varlen kernel; masks none of them expresses raise. Under HIP-graph
    capture the padded kernel always runs and nothing is read back (module header)."""
    kwargs.pop("is_causal", None)
    if softcap is not None:
        raise NotImplementedError("flash_attention_cute_amd: attention logit softcapping is not supported")
    if dropout:
        raise NotImplementedError("flash_attention_cute_amd: attention dropout is not supported (forward only)")
    sq, sk = query.shape[2], key.shape[2]
    causal = bool(getattr(module, "is_causal", True)) and sq > 1
    # a sliding window of W keys (transformers: key n visible to the query at position p iff
    # p - W < n <= p) that cuts the visible keys: the local-window kernel, window_left = W - 1
    window_left = sliding_window - 1 if sliding_window is not None and sk > sliding_window else None
    wl = -1 if window_left is None else window_left
    rope = kwargs.pop("rope_q", None)  # (cos, sin): q still to be rotated (fused path)
    kwargs.pop("cache_position", None)
    if attention_mask is not None and _capturing(query):
        low = lower_mask(attention_mask, sq, sk, causal, window_left)
        path = "padded"
        ranges = (low.k_start, low.k_end, low.q_start, low.q_end)
        if not TRUST_PADDING_MASK:
            # no host read-back: rows the padded kernel cannot express get empty ranges and are counted
            ok = low.shape_ok & low.run_ok
            _error_counter(query.device).add_((~ok).sum(dtype=torch.int32))
            ranges = (low.k_start, torch.where(ok, low.k_end, low.k_start), low.q_start,
                      torch.where(ok, low.q_end, low.q_start))
    else:
        low, path = _lowered_eager(attention_mask, sq, sk, causal, window_left)
        if low is not None:
            ranges = (low.k_start, low.k_end, low.q_start, low.q_end)
            if query.is_cuda:
                _error_counter(query.device)
    if low is not None:
        if path != "dense":
            if rope is not None:
                query = apply_rope(query, *rope)
            if path == "padded":
                return _padded_attention(query, key, value, ranges, causal, scaling, wl), None
            return _varlen_attention(query, key, value, low.kv_valid, low.q_valid, causal, scaling, wl), None
    if window_left is not None:
        if rope is not None:
            query = apply_rope(query, *rope)
        attn_output = flash_attn_window_func(query, key, value, window_left, softmax_scale=scaling, causal=causal)
        return attn_output.transpose(1, 2), None
    if rope is not None:
        attn_output = flash_attn_rope_func(query, key, value, *rope, causal=causal, softmax_scale=scaling)
    else:
        attn_output = flash_attn_func(query, key, value, causal=causal, softmax_scale=scaling)
    return attn_output.transpose(1, 2), None


def attention_forward(self: nn.Module, hidden_states: torch.Tensor,
                      position_embeddings: Tuple[torch.Tensor, torch.Tensor],
                      attention_mask: Optional[torch.Tensor] = None, past_key_value=None,
                      cache_position: Optional[torch.LongTensor] = None, **kwargs):
    """Replacement for ``LlamaAttention.forward`` / ``Qwen2Attention.forward``
    (reference models/rope_attn_fwd.py:66-120)."""
    cache = kwargs.pop("past_key_values", None)
    if cache is None:
        cache = past_key_value
    input_shape = hidden_states.shape[:-1]
    hidden_shape = (*input_shape, -1, self.head_dim)

    # strided [B, H, S, D] views of the projections (seq stride H * D); no copies
    query_states = self.q_proj(hidden_states).view(hidden_shape).transpose(1, 2)
    key_states = self.k_proj(hidden_states).view(hidden_shape).transpose(1, 2)
    value_states = self.v_proj(hidden_states).view(hidden_shape).transpose(1, 2)

    cos, sin = position_embeddings
    rope_q = None
    if FUSE_ROPE and query_states.is_cuda:
        # k: one HIP pass (the cache stores rotated keys); q: rotated in the attention kernel
        key_states = apply_rope(key_states, cos, sin)
        rope_q = (cos, sin)
    else:
        query_states, key_states = apply_rotary_pos_emb(query_states, key_states, cos, sin)

    if cache is not None:
        cache_kwargs = {"sin": sin, "cos": cos, "cache_position": cache_position}
        key_states, value_states = cache.update(key_states, value_states, self.layer_idx, cache_kwargs)

    cfg = self.config
    sliding_window = None
    if (getattr(cfg, "use_sliding_window", False) and getattr(cfg, "sliding_window", None) is not None
            and self.layer_idx >= getattr(cfg, "max_window_layers", 0)):
        sliding_window = cfg.sliding_window
    elif getattr(self, "sliding_window", None) is not None:
        sliding_window = self.sliding_window

    attn_output, attn_weights = _flash_attention_forward(
        self, query_states, key_states, value_states, attention_mask,
        dropout=0.0 if not self.training else self.attention_dropout, scaling=self.scaling,
        sliding_window=sliding_window, rope_q=rope_q, **kwargs)

    attn_output = attn_output.reshape(*input_shape, -1).contiguous()
    attn_output = self.o_proj(attn_output)
    return attn_output, attn_weights
