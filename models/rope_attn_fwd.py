"""Reference module path models/rope_attn_fwd.py -> flash_attention_cute_amd.hf_attention."""
from flash_attention_cute_amd.hf_attention import (  # noqa: F401
    _flash_attention_forward, apply_rotary_pos_emb, attention_forward, rotate_half)
