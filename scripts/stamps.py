#!/usr/bin/env python3
"""In-kernel phase stamps of fa_fwd_w4 (diagnostic; needs the -DFA_STAMPS=1 build:
python -c "from flash_attention_cute_amd import _build; _build.build_abi(stamps=True)").

Loads build/stamps/libfa_gfx950.so through its C-ABI, runs ~2 s of back-to-back launches of one
bench config (DVFS settles), then one stamped launch, and prints per-wave medians of the cycle
split: phase 1 (S = K.Q^T || softmax 2 || DMA), phase 2 (O += P.V || softmax 1) + rescale, the
DMA wait, the barrier; plus the in-kernel clock (s_memtime / s_memrealtime x 100 MHz).
usage: python scripts/stamps.py [c2|c3|c4|c5] [w4|p8]   (p8: 8 waves per Q block; p1 = phase A, p2 = B)
env: STAMPS_SHAPE (another shape), STAMPS_WS=1 (pass the workspace: key-split causal blocks, two records
per block), STAMPS_WIDTH (record width of the build)
"""
import ctypes
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"])
if os.environ.get("STAMPS_SHAPE"):  # "B,Hq,Hkv,S,causal,dtype", e.g. "1,16,4,4096,1,fp16" (C4's 8-way share)
    b_, hq_, hkv_, s_, c_, dt_ = os.environ["STAMPS_SHAPE"].split(",")
    cfg.update(B=int(b_), Hq=int(hq_), Hkv=int(hkv_), Sq=int(s_), Sk=int(s_), causal=bool(int(c_)), dtype=dt_,
               workload=f"shape {os.environ['STAMPS_SHAPE']}")
variant = sys.argv[2] if len(sys.argv) > 2 else "w4"
WAVES = 8 if variant == "p8" else 4


lib = ctypes.CDLL(os.environ.get("FA_STAMPS_LIB", str(ROOT / "build" / "stamps" / "libfa_gfx950.so")))


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
o = torch.empty_like(q)
st = []
for t in (q, k, v, o):
    st.append(t)
p = P(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), cfg["B"], cfg["Hq"], cfg["Hkv"], cfg["Sq"],
      cfg["Sk"], cfg["D"], cfg["Hq"] // cfg["Hkv"],
      *[t.stride(0) for t in st], *[t.stride(1) for t in st], *[t.stride(2) for t in st],
      cfg["D"] ** -0.5 * 1.4426950408889634)
nwg = cfg["B"] * cfg["Hq"] * ((cfg["Sq"] + 255) // 256) * (2 if os.environ.get("STAMPS_WS") == "1" else 1)
W = int(os.environ.get("STAMPS_WIDTH", "15"))  # 19: a -DFA_STAMPS_FINE build (phase sub-splits); 12 / 16: builds
# before round 5 (no prologue-wait / next-block-issue / first-tile fields)
buf = torch.zeros(nwg * WAVES * W, dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream().cuda_stream
lib.fa_debug_set_stamps(ctypes.c_void_p(0))
lib.fa_debug_set_knobs({"w4": 0, "p8": 3}[variant], -1, -1, -1, -1)
if os.environ.get("STAMPS_ZIGZAG"):  # 0 plain causal blocks, 1 the default rule, 2 always
    lib.fa_debug_set_zigzag(int(os.environ["STAMPS_ZIGZAG"]))
import time  # noqa: E402

dcode = 0 if dt == torch.float16 else 1
ws = None
if os.environ.get("STAMPS_WS") == "1":  # the workspace the library asks for (key-split causal blocks)
    lib.fa_fwd_gfx950_workspace_size.restype = ctypes.c_int64
    nws = lib.fa_fwd_gfx950_workspace_size(ctypes.byref(p), dcode, int(cfg["causal"]))
    ws = torch.empty(max(nws, 256), dtype=torch.uint8, device=dev) if nws > 0 else None


def launch():
    if ws is not None:
        rc = lib.fa_fwd_gfx950_ws(ctypes.byref(p), dcode, int(cfg["causal"]), ctypes.c_void_p(ws.data_ptr()),
                                  ctypes.c_int64(ws.numel()), ctypes.c_void_p(stream))
    else:
        rc = lib.fa_fwd_gfx950(ctypes.byref(p), dcode, int(cfg["causal"]), ctypes.c_void_p(stream))
    assert rc == 0


t0 = time.time()
n = 0
while time.time() - t0 < 2.0:
    launch()
    n += 1
    if n % 20 == 0:
        torch.cuda.synchronize()
lib.fa_debug_set_stamps(ctypes.c_void_p(buf.data_ptr()))
launch()
torch.cuda.synchronize()
lib.fa_debug_set_stamps(ctypes.c_void_p(0))
s = buf.view(-1, W).cpu().double()
s = s[s[:, 0] > 0]  # records of Q blocks that ran (an empty q-tile block writes none)
names = ["total", "p1", "p2+resc", "dma_wait", "barrier", "tiles", "drain", "prologue", "epilogue", "realtime"]
med = s.median(dim=0).values
print(f"{cfg['workload']} [{variant}]: {n} warm launches, {s.shape[0]} waves")
for i, nm in enumerate(names):
    print(f"  {nm:10s} median {med[i]:12.0f}  mean {s[:, i].mean():12.0f}")
tiles = s[:, 5].clamp(min=1)
for i, nm in [(1, "p1"), (2, "p2+resc"), (3, "dma_wait"), (4, "barrier")]:
    print(f"  per tile {nm:10s} {float((s[:, i] / tiles).median()):8.0f} cycles")
if W in (16, 19):  # FA_STAMPS_FINE: phase 2 in quarters (8 of its 32 MFMA gaps each), phase 1 in halves
    q = [float((s[:, i] / tiles).median()) for i in (12, 13, 14)]
    p2t = float((s[:, 2] / tiles).median())
    h1 = float((s[:, 15] / tiles).median())
    p1t = float((s[:, 1] / tiles).median())
    print(f"  per tile p1 halves          {h1:6.0f} {p1t - h1:6.0f}")
    print(f"  per tile p2 quarters (+resc) {q[0]:6.0f} {q[1]:6.0f} {q[2]:6.0f} {p2t - sum(q):6.0f}")
clk = (s[:, 0] / s[:, 9] * 100e6 / 1e9)
print(f"  in-kernel clock median {float(clk.median()):.3f} GHz")

# whole-launch accounting in s_memrealtime ticks (100 MHz, one clock for all XCDs; record field 10 is
# the block's realtime start, 9 its realtime duration), wave 0 of each Q block: busy share of the
# launch span over the grid's workgroups (ramp-up and end-of-launch imbalance), per XCD too
w0 = s[torch.arange(s.shape[0]) % WAVES == 0]
t_end = w0[:, 10] + w0[:, 9]
span = float(t_end.max() - w0[:, 10].min())
grid = min(nwg, 256)
busy = float(w0[:, 9].sum())
switch = float((w0[:, 6] + w0[:, 7] + w0[:, 8]).sum())
loop = float((w0[:, 1] + w0[:, 2] + w0[:, 3] + w0[:, 4]).sum())
print(f"  launch span {span / 100:.1f} us; utilisation (busy / (span x {grid} workgroups)) {busy / (span * grid):.3f}; "
      f"of the busy cycles: tiles {loop / float(w0[:, 0].sum()):.3f}, switch {switch / float(w0[:, 0].sum()):.3f}")
first = float(w0[:, 10].min())
print(f"  first block start spread {float(torch.quantile(w0[:, 10] - first, 0.99)) / 100:.2f} us (p99 over blocks), "
      f"last end - p50 end of the XCDs' last blocks:")
for x in range(8):
    sel = (w0[:, 11].long() & 255) == x
    if sel.any():
        e = t_end[sel]
        xs = w0[sel]
        print(f"    xcd {x}: blocks {int(sel.sum())}, end {float(e.max() - first) / 100:.1f} us, "
              f"busy {float(xs[:, 9].sum()) / 100:.0f} us, cycles {float(xs[:, 0].sum()) / 1e6:.2f} M, "
              f"clock {float((xs[:, 0] / xs[:, 9]).median()) / 10:.3f} GHz")
bt = torch.quantile(w0[:, 0], torch.tensor([0.1, 0.5, 0.9, 1.0], dtype=torch.float64))
btl = torch.quantile(w0[:, 5], torch.tensor([0.1, 0.5, 0.9, 1.0], dtype=torch.float64))
print(f"  block cycles (wave 0) p10 {bt[0]:.0f}  p50 {bt[1]:.0f}  p90 {bt[2]:.0f}  max {bt[3]:.0f}; "
      f"tiles p10 {btl[0]:.0f}  p50 {btl[1]:.0f}  p90 {btl[2]:.0f}  max {btl[3]:.0f}")
fields = [(6, "drain"), (7, "prologue"), (8, "epilogue")] + (
    [(W - 3, "pro. wait"), (W - 2, "next issue"), (W - 1, "first tile")] if W in (15, 19) else [])
for i, nm in fields:
    qs = torch.quantile(s[:, i], torch.tensor([0.1, 0.5, 0.9, 0.99], dtype=torch.float64))
    print(f"  {nm:10s} p10 {qs[0]:8.0f}  p50 {qs[1]:8.0f}  p90 {qs[2]:8.0f}  p99 {qs[3]:8.0f}")
role = s[:, 11].long() >> 8  # key-split role (fa_fwd_w4 split_role): 1 the first piece to arrive, 3 the second
for rl, nm in ((1, "1st, gave all"), (2, "1st, did A"), (3, "2nd, did both"), (4, "2nd, did B")):  # (2 / 4: the
    # one-block-each hand-off of stamps builds from profiles/r5i_*, not kept)
    sel = role == rl
    if sel.any():
        qs = torch.quantile(s[sel][:, 8], torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"  epilogue of {nm:13s} ({int(sel.sum()):5d} waves) p10 {qs[0]:8.0f}  p50 {qs[1]:8.0f}  p90 {qs[2]:8.0f}")
if WAVES == 8:  # leaders (waves 0-3) and followers (4-7) of every block
    w = torch.arange(s.shape[0]) % 8
    for nm, sel in (("leaders", w < 4), ("followers", w >= 4)):
        ss = s[sel]
        t = ss[:, 5].clamp(min=1)
        print(f"  {nm}: per tile A {float((ss[:, 1] / t).median()):.0f}  B {float((ss[:, 2] / t).median()):.0f}"
              f"  wait {float((ss[:, 3] / t).median()):.0f}  barrier {float((ss[:, 4] / t).median()):.0f}"
              f"  drain {float(ss[:, 6].median()):.0f}  prologue {float(ss[:, 7].median()):.0f}"
              f"  epilogue {float(ss[:, 8].median()):.0f}")
