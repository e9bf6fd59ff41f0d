#!/usr/bin/env python3
"""Interleaved A/B timing of several builds of the C-ABI library on one bench config (same process,
same device, same inputs), so device-to-device clock differences cancel out.
usage: python scripts/ab_libs.py <cfg> <lib.so>[@variant[:knob=value,...]] [...]   (env AB_REPS, AB_ITERS)
       variant: w4 | w8 | w4slow | p8 | m32 | m16, set through the library's fa_debug_set_knobs before its runs;
       knobs (debug setters of that library, applied before its runs): hp (head-packed blocks), zz (zigzag),
       split, pairs, rr. A library named twice is loaded from a copy, so each entry keeps its own knobs.
"""
import ctypes
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

cfg = dict(bench.CONFIGS[sys.argv[1]])
if os.environ.get("AB_SHAPE"):  # B,Hq,Hkv,S,D,dtype,causal: a shape of its own (e.g. one rank's share)
    b_, hq_, hkv_, s_, d_, dt_, c_ = os.environ["AB_SHAPE"].split(",")
    cfg.update(B=int(b_), Hq=int(hq_), Hkv=int(hkv_), Sq=int(s_), Sk=int(s_), D=int(d_), dtype=dt_, causal=c_ == "1")
    cfg.pop("W", None)
VARIANTS = {"w4": 0, "w8": 1, "w4slow": 2, "p8": 3, "m32": 4, "m16": 5}
SETTERS = {"hp": "fa_debug_set_head_pack", "zz": "fa_debug_set_zigzag", "split": "fa_debug_set_split",
           "pairs": "fa_debug_set_split_pairs", "rr": "fa_debug_set_split_rr"}
specs = [a.split("@") for a in sys.argv[2:]]
libs, seen = [], set()
for i, sp in enumerate(specs):
    path = os.path.abspath(sp[0])
    if path in seen:  # (dlopen of the same path returns the same handle and its knobs: load a copy)
        import shutil
        copy = f"/tmp/ab_libs_copy_{os.getpid()}_{i}.so"
        shutil.copyfile(path, copy)
        path = copy
    seen.add(os.path.abspath(sp[0]))
    libs.append(ctypes.CDLL(path))
variants = [VARIANTS[sp[1].split(":")[0] or "w4"] if len(sp) > 1 else -1 for sp in specs]
knob_sets = [[kv.split("=") for kv in sp[1].split(":")[1].split(",")] if len(sp) > 1 and ":" in sp[1] else []
             for sp in specs]
for lib, ks in zip(libs, knob_sets):
    for k, v in ks:
        getattr(lib, SETTERS[k]).argtypes = [ctypes.c_int]
        getattr(lib, SETTERS[k])(int(v))


class P(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_void_p) for n in ("q", "k", "v", "o")]
                + [(n, ctypes.c_int64) for n in ("B", "Hq", "Hkv", "Sq", "Sk", "D", "g")]
                + [(f"s{i}", ctypes.c_int64) for i in range(12)] + [("scale", ctypes.c_float)])


dev = torch.device("cuda:0")
dt = torch.float16 if cfg["dtype"] == "fp16" else torch.bfloat16
torch.manual_seed(0)
q = torch.randn(cfg["B"], cfg["Hq"], cfg["Sq"], cfg["D"], device=dev, dtype=dt)
k = torch.randn(cfg["B"], cfg["Hkv"], cfg["Sk"], cfg["D"], device=dev, dtype=dt)
v = torch.randn_like(k)
outs = [torch.empty_like(q) for _ in libs]
stream = torch.cuda.current_stream().cuda_stream


def params(o):
    st = (q, k, v, o)
    return P(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), cfg["B"], cfg["Hq"], cfg["Hkv"], cfg["Sq"],
             cfg["Sk"], cfg["D"], cfg["Hq"] // cfg["Hkv"], *[t.stride(0) for t in st], *[t.stride(1) for t in st],
             *[t.stride(2) for t in st], cfg["D"] ** -0.5 * 1.4426950408889634)


ps = [params(o) for o in outs]
dcode = 0 if dt == torch.float16 else 1
wss = [None] * len(libs)
if os.environ.get("AB_WS") == "1":
    for i, lib in enumerate(libs):
        lib.fa_fwd_gfx950_workspace_size.restype = ctypes.c_int64
        n = lib.fa_fwd_gfx950_workspace_size(ctypes.byref(ps[i]), dcode, int(cfg["causal"]))
        wss[i] = torch.empty(max(n, 256), dtype=torch.uint8, device=dev) if n > 0 else None


def run(i, n):
    libs[i].fa_debug_set_knobs(variants[i], -1, -1, -1, -1)
    for _ in range(n):
        if cfg.get("W"):  # local-window configs: fa_fwd_gfx950_window
            rc = libs[i].fa_fwd_gfx950_window(ctypes.byref(ps[i]), dcode, int(cfg["causal"]),
                                              ctypes.c_int64(cfg["W"] - 1), ctypes.c_void_p(stream))
        elif wss[i] is not None:  # AB_WS=1: the workspace the library asks for (key-split blocks)
            rc = libs[i].fa_fwd_gfx950_ws(ctypes.byref(ps[i]), dcode, int(cfg["causal"]), ctypes.c_void_p(wss[i].data_ptr()),
                                          ctypes.c_int64(wss[i].numel()), ctypes.c_void_p(stream))
        else:
            rc = libs[i].fa_fwd_gfx950(ctypes.byref(ps[i]), dcode, int(cfg["causal"]), ctypes.c_void_p(stream))
        assert rc == 0


flops = bench.flops(cfg)
iters = int(os.environ.get("AB_ITERS", "30"))
for i in range(len(libs)):
    run(i, 10)
torch.cuda.synchronize()
res = [[] for _ in libs]
for rep in range(int(os.environ.get("AB_REPS", "5"))):
    for i in range(len(libs)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run(i, iters)
        b.record()
        torch.cuda.synchronize()
        res[i].append(flops * iters / (a.elapsed_time(b) * 1e-3) / 1e12)
for i, p in enumerate(sys.argv[2:]):
    r = sorted(res[i])
    d = (outs[i].float() - outs[0].float()).abs().max().item()
    print(f"{sys.argv[1]} {p}: median {r[len(r) // 2]:.1f} TFLOPS  (min {r[0]:.1f} max {r[-1]:.1f})  max|o-o0| {d:.2e}")
