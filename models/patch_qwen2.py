"""``patch_attn()``: Qwen2Attention.forward -> gfx950 flash attention (reference models/patch_qwen2.py:1-5)."""
from transformers.models.qwen2.modeling_qwen2 import Qwen2Attention

from flash_attention_cute_amd.hf_attention import attention_forward


def patch_attn():
    Qwen2Attention.forward = attention_forward
