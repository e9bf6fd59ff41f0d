"""Diagnostic hooks of the C-ABI library (not part of include/fa_gfx950.h; tests and A/B scripts).

The dispatcher reads its tuning / debug knobs ONCE per process (from the environment, at the first
launch) and never per launch (csrc/fa_launch.h ``Knobs``). Tests that need another kernel variant or
grid cap switch them with :func:`knobs`, which restores the defaults on exit, and check which kernel
actually ran with :func:`last_path`.
"""
from __future__ import annotations

import contextlib
import ctypes

from . import _build

PATHS = {0: "none", 1: "w4", 2: "w8", 3: "w4slow", 4: "decode", 5: "decode_split", 6: "p8"}
VARIANTS = {"w4": 0, "w8": 1, "w4slow": 2, "p8": 3}

_lib = None


def lib() -> ctypes.CDLL:
    """The already-loaded libfa_gfx950.so (the torch binding links it; dlopen returns that handle)."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  -- the HIP runtime first, as in the product

        lib = ctypes.CDLL(str(_build.ABI_LIB))
        lib.fa_debug_set_knobs.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int]
        lib.fa_debug_set_knobs.restype = None
        lib.fa_debug_last_path.restype = ctypes.c_int
        _lib = lib
    return _lib


def set_knobs(variant: str | None = None, w4_grid: int | None = None, decode: bool | None = None,
              dec_target: int | None = None, dec_flags: int | None = None) -> None:
    """Override knobs for the following launches; None restores that knob's default."""
    lib().fa_debug_set_knobs(-1 if variant is None else VARIANTS[variant], -1 if w4_grid is None else int(w4_grid),
                             -1 if decode is None else int(bool(decode)), -1 if dec_target is None else int(dec_target),
                             -1 if dec_flags is None else int(dec_flags))


@contextlib.contextmanager
def knobs(**kw):
    """``with knobs(variant="w8"): ...`` -- every knob back to its default afterwards."""
    set_knobs(**kw)
    try:
        yield
    finally:
        set_knobs()


def last_path() -> str:
    """Kernel the last op call on this thread launched ("w4", "decode_split", ...)."""
    return PATHS.get(lib().fa_debug_last_path(), "unknown")
