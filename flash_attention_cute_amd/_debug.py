"""Diagnostic hooks of the C-ABI library (not part of include/fa_gfx950.h; tests and A/B scripts).

The dispatcher reads its tuning / debug knobs ONCE per process (from the environment, at the first
launch) and never per launch (csrc/fa_launch.h ``Knobs``). Tests that need another grid cap or the
decode kernel off switch them with :func:`knobs`, which restores the defaults on exit, and check
which kernel actually ran with :func:`last_path`.

The debug / A-B kernel bodies (``fa_fwd_w8``, ``fa_fwd_p8``, the non-pipelined ``w4slow`` body) are
NOT in the product library the op loads: they live in ``lib/libfa_gfx950_debug.so`` (the same
C-ABI built with -DFA_DEBUG_VARIANTS). :func:`forward` runs one of them through that library's
C-ABI with the host steps of the op restated (default scale, head-dim pad, the Sq == 1 q-head pack
of reference csrc/flash_attention_api.cpp:72-83, the stride-preserving output), for the GPU parity
sweep.
"""
from __future__ import annotations

import contextlib
import ctypes

from . import _build

PATHS = {0: "none", 1: "w4", 2: "w8", 3: "w4slow", 4: "decode", 5: "decode_split", 6: "p8", 7: "m32", 8: "m16"}
VARIANTS = {"w4": 0, "w8": 1, "w4slow": 2, "p8": 3, "m32": 4, "m16": 5}
LOG2E = 1.4426950408889634

_libs = {}


class FaFwdParams(ctypes.Structure):
    """include/fa_gfx950.h ``fa_fwd_params`` (field order of reference csrc/flash_attention.h:5-37)."""

    _fields_ = ([(n, ctypes.c_void_p) for n in ("q_ptr", "k_ptr", "v_ptr", "o_ptr")]
                + [(n, ctypes.c_int64) for n in ("batch_size", "num_heads_q", "num_heads_kv", "seqlen_q", "seqlen_kv",
                                                 "headdim", "head_q_per_group")]
                + [(f"{t}_{s}_stride", ctypes.c_int64) for s in ("batch", "head", "seqlen") for t in "qkvo"]
                + [("softmax_scale", ctypes.c_float)])


def lib(debug: bool = False) -> ctypes.CDLL:
    """The already-loaded libfa_gfx950.so (the torch binding links it; dlopen returns that handle), or
    (``debug``) lib/libfa_gfx950_debug.so."""
    if debug not in _libs:
        import torch  # noqa: F401  -- the HIP runtime first, as in the product

        path = _build.DEBUG_LIB if debug else _build.ABI_LIB
        if not path.exists():
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(str(path))
        lib.fa_debug_set_knobs.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int]
        lib.fa_debug_set_knobs.restype = None
        lib.fa_debug_last_path.restype = ctypes.c_int
        lib.fa_last_error.restype = ctypes.c_char_p
        lib.fa_debug_set_zigzag.argtypes = [ctypes.c_int]
        lib.fa_debug_set_zigzag.restype = None
        lib.fa_debug_set_split.argtypes = [ctypes.c_int]
        lib.fa_debug_set_split.restype = None
        lib.fa_debug_set_split_pairs.argtypes = [ctypes.c_int]
        lib.fa_debug_set_split_pairs.restype = None
        lib.fa_debug_set_dec_fuse.argtypes = [ctypes.c_int]
        lib.fa_debug_set_dec_fuse.restype = None
        lib.fa_debug_last_zigzag.restype = ctypes.c_int
        lib.fa_split_errors.argtypes = [ctypes.c_int]
        lib.fa_split_errors.restype = ctypes.c_int64
        lib.fa_debug_set_xccs.argtypes = [ctypes.c_int]
        lib.fa_debug_set_xccs.restype = None
        lib.fa_debug_set_split_fault.argtypes = [ctypes.c_int]
        lib.fa_debug_set_split_fault.restype = None
        lib.fa_debug_last_dec_fused.restype = ctypes.c_int
        lib.fa_debug_set_head_pack.argtypes = [ctypes.c_int]
        lib.fa_debug_set_split_rr.argtypes = [ctypes.c_int]
        lib.fa_debug_set_split_rr.restype = None
        lib.fa_debug_set_head_pack.restype = None
        lib.fa_fwd_gfx950_workspace_size.restype = ctypes.c_int64
        lib.fa_fwd_gfx950_ws.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_void_p]
        _libs[debug] = lib
    return _libs[debug]


def set_knobs(variant: str | None = None, w4_grid: int | None = None, decode: bool | None = None,
              dec_target: int | None = None, dec_flags: int | None = None, debug: bool = False) -> None:
    """Override knobs for the following launches; None restores that knob's default. ``variant`` other
    than w4 exists only in the debug library."""
    if variant not in (None, "w4") and not debug:
        raise ValueError(f"variant {variant!r} is only in the debug library (debug=True, forward())")
    lib(debug).fa_debug_set_knobs(-1 if variant is None else VARIANTS[variant],
                                  -1 if w4_grid is None else int(w4_grid),
                                  -1 if decode is None else int(bool(decode)),
                                  -1 if dec_target is None else int(dec_target),
                                  -1 if dec_flags is None else int(dec_flags))


@contextlib.contextmanager
def knobs(debug: bool = False, **kw):
    """``with knobs(w4_grid=16): ...`` -- every knob back to its default afterwards."""
    set_knobs(debug=debug, **kw)
    try:
        yield
    finally:
        set_knobs(debug=debug)


def last_path(debug: bool = False) -> str:
    """Kernel the last call on this thread launched ("w4", "decode_split", ...)."""
    return PATHS.get(lib(debug).fa_debug_last_path(), "unknown")


def set_zigzag(mode: int | None = None, debug: bool = False) -> None:
    """Causal Q-block layout of fa_fwd_w4: 0 never zigzag, 1 when the blocks fit one round of the
    persistent grid (the default), 2 always where it applies; None restores the default."""
    lib(debug).fa_debug_set_zigzag(-1 if mode is None else int(mode))


def last_zigzag(debug: bool = False) -> bool:
    """Whether the last prefill launch on this thread ran zigzag Q blocks."""
    return lib(debug).fa_debug_last_zigzag() == 1


def set_split(mode: int | None = None, debug: bool = False) -> None:
    """Key-split causal blocks (the op passes the workspace they need): 0 never, 1 where measured
    faster than zigzag (the default: one-round grids with long enough keys, fa_launch.h use_split),
    2 whenever a workspace is passed; None restores the default."""
    lib(debug).fa_debug_set_split(-1 if mode is None else int(mode))


def set_split_pairs(mode: int | None = None, debug: bool = False) -> None:
    """Key-split pairs (a heavy and a light q-tile on two workgroups, one pass; fa_launch.h
    use_split_pairs): 0 never, 1 where they fit one pass of the grid (the default); None restores it."""
    lib(debug).fa_debug_set_split_pairs(-1 if mode is None else int(mode))


def set_split_rr(mode: int | None = None, debug: bool = False) -> None:
    """Work order of the key-split halves: 1 level-major (every XCD a share of every q-tile level, the
    default), 0 decode_work's XCD-contiguous ranges; None restores the default."""
    lib(debug).fa_debug_set_split_rr(-1 if mode is None else int(mode))


def set_dec_fuse(mode: int | None = None, debug: bool = False) -> None:
    """Split-KV decode merge: 1 the last split of a unit merges inside fa_decode (the default), 0 the
    separate fa_decode_combine launch; None restores the default."""
    lib(debug).fa_debug_set_dec_fuse(-1 if mode is None else int(mode))


def set_xccs(n: int | None = None, debug: bool = False) -> None:
    """XCDs per device seen by the placement check (fa_launch.h same_xcd_placement: key-split and the
    fused decode merge need the count to divide 8); None restores the device's own count."""
    lib(debug).fa_debug_set_xccs(-1 if n is None else int(n))


def set_split_fault(on: bool) -> None:
    """DEBUG library only: force one key-split hand-off per launch (slot 0, wave 0) to time out."""
    lib(debug=True).fa_debug_set_split_fault(1 if on else 0)


def last_dec_fused(debug: bool = False) -> bool:
    """Whether the last split-KV decode launch on this thread merged its partials in-kernel."""
    return lib(debug).fa_debug_last_dec_fused() == 1


def set_head_pack(mode: int | None = None, debug: bool = False) -> None:
    """Head-packed causal GQA blocks (4 q-heads per kv-head, one per wave, 64 rows; fa_launch.h
    use_head_pack, use_head_pack_split): 0 never, 1 on multi-round grids and for key-split pieces (the
    default), 2 wherever they apply; None restores it."""
    lib(debug).fa_debug_set_head_pack(-1 if mode is None else int(mode))


def last_layout(debug: bool = False) -> str:
    """Causal block layout of the last prefill launch on this thread: "plain", "zigzag", "split"
    (key-split, as halves or as pairs: last_split_pairs; over head-packed blocks: last_head_pack) or
    "headpack"."""
    return {0: "plain", 1: "zigzag", 2: "split", 3: "split", 4: "headpack", 5: "split",
            6: "split"}[lib(debug).fa_debug_last_zigzag()]


def last_split_pairs(debug: bool = False) -> bool:
    """Whether the last prefill launch on this thread laid its key-split pieces out as pairs."""
    return lib(debug).fa_debug_last_zigzag() in (3, 6)


def last_head_pack(debug: bool = False) -> bool:
    """Whether the last prefill launch on this thread ran head-packed blocks (key-split pieces or not)."""
    return lib(debug).fa_debug_last_zigzag() in (4, 5, 6)


def forward(q, k, v, softmax_scale=None, causal=False, variant="w8", window_left=-1, w4_grid=None,
            workspace=False):
    """Attention through a kernel body of the DEBUG library (tests: the parity sweep over w8 / w4slow /
    p8): the op's host steps (reference flash_attention/flash_attention.py:17-53 and
    csrc/flash_attention_api.cpp:64-133, restated) over lib/libfa_gfx950_debug.so's C-ABI;
    ``workspace``: through fa_fwd_gfx950_ws with the workspace it asks for, as the op does."""
    import torch

    dl = lib(debug=True)
    set_knobs(variant=variant, w4_grid=w4_grid, debug=True)
    d0 = q.size(-1)
    scale = d0 ** -0.5 if softmax_scale is None else softmax_scale
    if d0 % 8:
        pad = [0, 8 - d0 % 8]
        q, k, v = (torch.nn.functional.pad(t, pad) for t in (q, k, v))
    q, k, v = (t if t.stride(3) == 1 else t.contiguous() for t in (q, k, v))
    b, hq, sq, d = q.shape
    hkv, sk = k.size(1), k.size(2)
    g = hq // hkv
    qx = q
    pack = sq == 1 and window_left < 0
    if pack:  # the q-heads of a kv group become the rows of one (batch, kv-head) problem
        qx = q.reshape(b, hkv, g, d)
        causal = False
    o = torch.empty_like(qx)
    st = lambda t, i: t.stride(i) if t.size(i) > 1 else 0  # noqa: E731
    p = FaFwdParams(qx.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, qx.size(1), hkv, qx.size(2), sk, d,
                    1 if pack else g, *(st(t, i) for i in range(3) for t in (qx, k, v, o)),
                    float(torch.tensor(scale, dtype=torch.float32).double() * LOG2E))
    dtype = 0 if q.dtype == torch.float16 else 1
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if window_left >= 0:
        rc = dl.fa_fwd_gfx950_window(ctypes.byref(p), dtype, int(causal), ctypes.c_int64(window_left), stream)
    elif workspace:
        need = dl.fa_fwd_gfx950_workspace_size(ctypes.byref(p), dtype, int(causal))
        ws = torch.empty(max(need, 16), dtype=torch.uint8, device=q.device)
        rc = dl.fa_fwd_gfx950_ws(ctypes.byref(p), dtype, int(causal), ws.data_ptr(), need, stream)
    else:
        rc = dl.fa_fwd_gfx950(ctypes.byref(p), dtype, int(causal), stream)
    if rc != 0:
        raise RuntimeError(f"debug library call failed ({rc}): {dl.fa_last_error().decode()}")
    o = o.reshape(q.shape)
    return o[..., :d0] if d0 % 8 else o
