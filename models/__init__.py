"""Drop-in import path of the reference's model integration (reference models/).

``from models.patch_llama import patch_attn`` / ``from models.patch_qwen2 import patch_attn``
monkey-patch the installed transformers' attention to run the gfx950 kernel
(flash_attention_cute_amd/hf_attention.py). The reference's vendored full-model copies
(models/modeling_{llama,qwen2}.py) are not imported by anything there and are out of scope.
"""
