"""``patch_attn()``: LlamaAttention.forward -> gfx950 flash attention (reference models/patch_llama.py:1-5)."""
from transformers.models.llama.modeling_llama import LlamaAttention

from flash_attention_cute_amd.hf_attention import attention_forward


def patch_attn():
    LlamaAttention.forward = attention_forward
