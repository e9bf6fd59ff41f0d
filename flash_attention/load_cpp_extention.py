"""Drop-in for reference module ``flash_attention.load_cpp_extention`` (flash_attention/load_cpp_extention.py:11-53).

The reference's ``load_extension()`` JIT-compiles ``csrc/flash_attention_api.cpp`` +
``flash_attention_impl.cu`` with nvcc and returns the module exposing ``flash_attention_fwd``.
Here it returns the prebuilt gfx950 extension (hipcc, built in-tree by
``flash_attention_cute_amd._build``; built once on first call if missing and a ROCm toolchain is
present), which exposes ``flash_attention_fwd(q, k, v, softmax_scale, causal)`` with the
reference's pybind signature (reference csrc/flash_attention_api.cpp:14-15, :137-141).
"""
from flash_attention_cute_amd.load_cpp_extention import load_extension  # noqa: F401

__all__ = ["load_extension"]
