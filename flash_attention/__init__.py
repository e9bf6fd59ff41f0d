"""Drop-in import name of the reference package (reference flash_attention/__init__.py:1).

``from flash_attention import flash_attn_func`` resolves to the gfx950 implementation.
"""
from flash_attention_cute_amd import flash_attn_func  # noqa: F401
from flash_attention_cute_amd import flash_attn_varlen_func  # noqa: F401,E402  (beyond the reference: varlen)
