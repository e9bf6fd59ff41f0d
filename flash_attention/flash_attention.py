"""Drop-in for reference module ``flash_attention.flash_attention`` (flash_attention/flash_attention.py:1-53).

The reference module builds its extension at import (``flash_attention_cuda = load_extension()``,
:4) and registers ``flash_attention::forward`` with a CPU default (:6-15), a "cuda" kernel
(:17-38) and a fake (:40-43), then defines ``flash_attn_func`` (:46-53). Here the op is registered
exactly once, in ``flash_attention_cute_amd.flash_attention``; this module re-binds the SAME
objects under the reference's names, so code that imports from the reference's submodule path
reaches the gfx950 op without a second registration:

* ``flash_attention_cuda``        -- the loaded gfx950 extension (``flash_attention_fwd`` et al.),
                                     or ``None`` when it could not be loaded (GPU calls then raise);
* ``flash_attention_forward``     -- the ``flash_attention::forward`` custom op object;
* ``flash_attention_forward_cuda`` -- its "cuda" kernel (pad D, last-dim contiguity, slice);
* ``flash_attention_forward_fake`` -- its fake (``empty_like(q)``);
* ``flash_attn_func``             -- ``scale = D ** -0.5`` by default, then the op.
"""
from flash_attention_cute_amd.flash_attention import (  # noqa: F401
    flash_attention_cuda,
    flash_attention_forward,
    flash_attention_forward_cuda,
    flash_attention_forward_fake,
    flash_attn_func,
)
from flash_attention_cute_amd.flash_attention import flash_attn_varlen_func  # noqa: F401  (beyond the reference)

from .load_cpp_extention import load_extension  # noqa: F401  (the reference module imports it, :2)

__all__ = ["flash_attention_cuda", "flash_attention_forward", "flash_attention_forward_cuda",
           "flash_attention_forward_fake", "flash_attn_func", "load_extension"]
