"""ctypes front-end of oracle/fa_oracle.c -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

``forward(q, k, v, scale, causal)`` takes CPU torch tensors (fp16 / bf16, [B, H, S, D]) and returns
the oracle output as a tensor of the same dtype, computed with the kernel's arithmetic widths
(fp32 accumulation, P rounded to T) on ``threads`` host cores.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB = HERE / "lib" / "libfa_oracle.so"
_lib = None


def build(force: bool = False) -> Path:
    src = HERE / "fa_oracle.c"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        cmd = ["make", "-C", str(HERE), "-s"] + (["-B"] if force else [])
        subprocess.run(cmd, check=True, capture_output=True)
    return LIB


def _load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = ctypes.CDLL(str(LIB))
        i64 = ctypes.c_int64
        lib.fa_oracle_fwd.argtypes = [ctypes.c_void_p] * 5 + [i64] * 6 + [ctypes.c_float, ctypes.c_int,
                                                                         ctypes.c_int, ctypes.c_int]
        lib.fa_oracle_fwd.restype = ctypes.c_int
        lib.fa_oracle_fwd_window.argtypes = lib.fa_oracle_fwd.argtypes + [i64]
        lib.fa_oracle_fwd_window.restype = ctypes.c_int
        lib.fa_oracle_max_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def max_threads() -> int:
    return _load().fa_oracle_max_threads()


def forward(q, k, v, softmax_scale: float, causal: bool, threads: int = 0, want_f32: bool = False,
            window_left: int = -1):
    """window_left >= 0: the local window of fa_fwd_gfx950_window (key n visible to query m only if
    n >= m + Sk - Sq - window_left)."""
    import torch

    lib = _load()
    assert q.dtype in (torch.float16, torch.bfloat16) and q.dtype == k.dtype == v.dtype
    dtype = 0 if q.dtype == torch.float16 else 1
    q = q.detach().cpu().contiguous()
    k = k.detach().cpu().contiguous()
    v = v.detach().cpu().contiguous()
    b, hq, sq, d = q.shape
    hkv, sk = k.shape[1], k.shape[2]
    o = torch.empty_like(q)
    o32 = torch.empty(q.shape, dtype=torch.float32) if want_f32 else None
    rc = lib.fa_oracle_fwd_window(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                  o32.data_ptr() if o32 is not None else None, b, hq, hkv, sq, sk, d,
                                  float(softmax_scale), int(bool(causal)), dtype, int(threads), int(window_left))
    if rc != 0:
        raise ValueError("fa_oracle_fwd: invalid shapes")
    return (o, o32) if want_f32 else o


if __name__ == "__main__":
    print(build(force=bool(os.environ.get("FORCE"))))


def forward_varlen(q, k, v, cu_seqlens_q, cu_seqlens_k, softmax_scale: float, causal: bool, threads: int = 0,
                   window_left: int = -1):
    """Oracle of the varlen entry (include/fa_gfx950.h fa_fwd_gfx950_varlen): packed q [total_q, Hq, D],
    k/v [total_k, Hkv, D]; each sequence is the dense forward above on its own rows (bottom-right
    causal per sequence); a sequence without keys gives 0 rows."""
    import torch

    cq = [int(x) for x in cu_seqlens_q.tolist()]
    ck = [int(x) for x in cu_seqlens_k.tolist()]
    q, k, v = (t.detach().cpu() for t in (q, k, v))
    out = torch.zeros_like(q)
    for b in range(len(cq) - 1):
        q0, q1, k0, k1 = cq[b], cq[b + 1], ck[b], ck[b + 1]
        if q1 == q0 or k1 == k0:
            continue
        qs, ks, vs = (t.transpose(0, 1).unsqueeze(0) for t in (q[q0:q1], k[k0:k1], v[k0:k1]))
        out[q0:q1] = forward(qs, ks, vs, softmax_scale, causal, threads=threads,
                             window_left=window_left)[0].transpose(0, 1)
    return out
