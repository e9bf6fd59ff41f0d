#!/usr/bin/env python3
"""Round-3 "O zeroed by C = 0 P.V MFMAs" experiment, rebuilt (-DFA_EXP_CZERO: no v_accvgpr_write
zeroing in the block prologue; the block's first UNMASKED iteration writes O with C = 0): the same
inputs through it and through the product library, for causal / windowless non-causal shapes and two
grid caps. The failure it shows is the one _asm_check rule R5 rejects on CPU: a Q block whose first
tile is masked (causal first q-tiles) accumulates into the previous block's O (or, at kernel entry,
into whatever the AGPRs held), so the output depends on the schedule.
usage: python scripts/experiments/czero_repro.py <czero lib> [product lib]"""
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from flash_attention_cute_amd._debug import FaFwdParams, LOG2E  # noqa: E402

bad = ctypes.CDLL(sys.argv[1])
good = ctypes.CDLL(sys.argv[2] if len(sys.argv) > 2 else str(ROOT / "flash_attention_cute_amd/lib/libfa_gfx950.so"))
for lib in (bad, good):
    lib.fa_debug_set_knobs.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int]
dev = torch.device("cuda:0")


def run(lib, q, k, v, causal, grid):
    lib.fa_debug_set_knobs(-1, grid, -1, -1, -1)
    o = torch.empty_like(q)
    b, hq, sq, d = q.shape
    hkv, sk = k.shape[1], k.shape[2]
    p = FaFwdParams(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, hq, hkv, sq, sk, d, hq // hkv,
                    *(t.stride(i) for i in range(3) for t in (q, k, v, o)), d ** -0.5 * LOG2E)
    rc = lib.fa_fwd_gfx950(ctypes.byref(p), 0, int(causal), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
    return o


torch.manual_seed(0)
for causal in (False, True):
    q = torch.randn(2, 8, 1024, 128, device=dev, dtype=torch.float16)
    k = torch.randn(2, 2, 1024, 128, device=dev, dtype=torch.float16)
    v = torch.randn(2, 2, 1024, 128, device=dev, dtype=torch.float16)
    ref = run(good, q, k, v, causal, 0)
    for grid in (0, 16, 8):
        o = run(bad, q, k, v, causal, grid)
        d = (o.float() - ref.float()).abs()
        rows = (d.amax(-1) > 1e-2)
        print(f"causal={causal} grid={grid or 'default'}: max|czero - product| {d.max().item():.3e}, "
              f"rows off {int(rows.sum())} of {rows.numel()}, q-tiles with a wrong row "
              f"{sorted(set((rows.nonzero()[:, 2] // 256).tolist()))}", flush=True)
