"""MI355X-native FlashAttention-2 forward (drop-in for izmttk/flash_attention_cute)."""
from .flash_attention import (apply_rope, flash_attention_forward, flash_attention_padded_forward,  # noqa: F401
                              flash_attention_varlen_forward, flash_attention_window_forward, flash_attn_func,
                              flash_attn_padded_func, flash_attn_rope_func, flash_attn_varlen_func,
                              flash_attn_window_func, split_errors)

__all__ = ["flash_attn_func", "flash_attention_forward", "flash_attn_varlen_func", "flash_attention_varlen_forward",
           "flash_attn_rope_func", "apply_rope", "flash_attn_window_func", "flash_attention_window_forward",
           "flash_attn_padded_func", "flash_attention_padded_forward", "split_errors"]
