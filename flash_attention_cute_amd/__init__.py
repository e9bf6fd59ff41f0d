"""MI355X-native FlashAttention-2 forward (drop-in for izmttk/flash_attention_cute)."""
from .flash_attention import flash_attn_func, flash_attention_forward  # noqa: F401

__all__ = ["flash_attn_func", "flash_attention_forward"]
