"""Loader for the prebuilt gfx950 extension.

Mirrors reference flash_attention/load_cpp_extention.py:11-53 (``load_extension()`` returning the
module that exposes ``flash_attention_fwd``), but never JIT-compiles at import and never hipifies:
the extension is built in-tree by ``flash_attention_cute_amd._build`` (called from
``__graft_entry__.build()``) and this function only imports it. If the artefact is missing and a
ROCm toolchain is present, it is built once; otherwise the import error is raised to the caller.
"""
from __future__ import annotations

import importlib
import os

from . import _build


def load_extension():
    """Import ``flash_attention_cute_amd._C`` (building it first if it does not exist)."""
    import torch  # noqa: F401  -- loads libc10/libtorch/libamdhip64 before the extension

    if not _build.ext_path().exists() or not _build.ABI_LIB.exists():
        if os.environ.get("FA_GFX950_NO_BUILD") or not _build.HIPCC.exists():
            raise ImportError(
                f"gfx950 extension not built ({_build.ext_path().name}); run "
                "`python -m flash_attention_cute_amd._build`")
        _build.build_all()
    return importlib.import_module("flash_attention_cute_amd._C")
