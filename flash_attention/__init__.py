"""Drop-in import name of the reference package (reference flash_attention/__init__.py:1).

``from flash_attention import flash_attn_func`` resolves to the gfx950 implementation, and so do
the reference's submodule paths ``flash_attention.flash_attention`` and
``flash_attention.load_cpp_extention``.
"""
from .flash_attention import flash_attn_func  # noqa: F401
from .flash_attention import flash_attn_varlen_func  # noqa: F401  (beyond the reference: varlen)
