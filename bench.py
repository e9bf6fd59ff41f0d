#!/usr/bin/env python3
"""bench.py -- attention-forward TFLOPS and % of MFMA peak of the gfx950 FlashAttention-2 kernel.

Metric (BASELINE.json): attn fwd TFLOPS + %MFMA peak at (B,H,S,D) = (4,32,4096,128) fp16
(BASELINE configs[1], "C2": MHA, non-causal). A step is one call of the public op
``flash_attn_func`` (custom op -> C++ host API -> C-ABI -> HIP kernel) over one batch of
synthetic N(0,1) q, k, v already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|c5_layer|decode|window|...]
                  [--weak] [--world W --rank R]

Multi-GPU (launched by torch.distributed.run, one process per GPU; attention tiles are independent,
so there is no data-path collective -- SURVEY.md 8(e)). A gloo process group carries only the
barrier and the max-over-ranks of the timings.
  default ("strong"): ONE global problem (batch = --global-batch, default the
                    config's; C5: global batch 8) is split into (batch, kv-head) units by
                    flash_attention_cute_amd/shard.py and each rank runs only its units (strided
                    views, no copies); value = global FLOPs / slowest rank. C2 at N = 8: 128 (b, h)
                    units -> 16 per GPU. At N = 1 this is the whole configured workload.
  --weak          : every rank runs the whole configured workload on its own seeded inputs.
  --world W --rank R (no torch.distributed): THIS process runs exactly rank R's share of a W-way
                    strong split on one GPU -- the per-GPU work of the N = W run, measured on one
                    device (``shard_of`` in the line); value = that share's FLOPs / its time.
c5_layer: a step is one patched ``LlamaAttention.forward`` (Llama-3-8B dims, random weights,
reference models/rope_attn_fwd.py:66-120 with this repo's fused RoPE) -- value in tokens/s, with the
bare op and unpatched HF (SDPA) timed beside it in the same run.

Rank 0 prints ONE JSON line. Besides the contract fields it carries
  roofline     : the kernel's achieved TFLOP/s (algorithmic FLOPs / the HIP-event time of the
                 timed region's back-to-back launches, per launch) against the dense fp16 MFMA
                 peak; ``traffic`` is
                 the HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), or null;
  cpu_baseline : torch SDPA fp32 on the host cores (the reference op's CPU path, BASELINE.md's CPU
                 baseline) on the same workload; ``port`` = oracle/fa_oracle.c on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import struct
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "attn fwd TFLOPS + %MFMA peak, (B,H,S,D)=(4,32,4096,128) fp16"  # BASELINE.json (config c2)
PEAK_TFLOPS = 2516.6  # 256 CU x 4 SIMD x 1024 FLOP/clk (32x32x16 f16/bf16 MFMA) x 2.4 GHz, dense
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    "c2": dict(workload="C2 MHA fp16 B4 H32 S4096 D128 non-causal", B=4, Hq=32, Hkv=32, Sq=4096,
               Sk=4096, D=128, dtype="fp16", causal=False),
    "c3": dict(workload="C3 MHA bf16 B4 H32 S8192 D128 causal", B=4, Hq=32, Hkv=32, Sq=8192, Sk=8192,
               D=128, dtype="bf16", causal=True),
    "c4": dict(workload="C4 GQA fp16 B4 Hq32 Hkv8 S4096 D128 causal", B=4, Hq=32, Hkv=8, Sq=4096,
               Sk=4096, D=128, dtype="fp16", causal=True),
    # C5: Llama-3-8B attention (Hq32 Hkv8 D128), bf16 causal prefill S4096; by default global batch 8
    # (strong_batch) sharded over (batch, kv-head) units -- one batch row per GPU at N=8
    # (flash_attention_cute_amd/shard.py, strong scaling); --weak: a B1 replica per GPU
    "c5": dict(workload="C5 Llama-3-8B attn bf16 causal Hq32 Hkv8 S4096 D128", B=1, Hq=32, Hkv=8,
               Sq=4096, Sk=4096, D=128, dtype="bf16", causal=True, strong_batch=8),
    # the patched HF attention layer around the op at C5's dims (prefill of S tokens, B per GPU)
    "c5_layer": dict(workload="C5 layer: patched Llama-3-8B LlamaAttention.forward bf16 causal B1(per GPU) S4096 "
                              "(hidden 4096, Hq32 Hkv8 D128, rope_theta 5e5)", B=1, Hq=32, Hkv=8, Sq=4096, Sk=4096,
                     D=128, dtype="bf16", causal=True, hidden=4096),
    "decode": dict(workload="decode GQA fp16 B32 Hq32 Hkv8 Sq1 Sk4096 D128 (q-head pack)", B=32, Hq=32,
                   Hkv=8, Sq=1, Sk=4096, D=128, dtype="fp16", causal=False),
    # long-context decode at batch 1: the same K/V bytes as "decode" in 8 (batch, kv-head) streams,
    # split over the keys (split-KV + combine)
    "decode_long": dict(workload="decode GQA bf16 B1 Hq32 Hkv8 Sq1 Sk131072 D128 (split-KV)", B=1, Hq=32, Hkv=8,
                        Sq=1, Sk=131072, D=128, dtype="bf16", causal=False),
    # local (sliding-window) attention: each query sees the last W keys up to itself (Mistral-7B-style
    # window of 4096 on Llama-3-8B attention dims, 32k-token prefill); flash_attn_window_func
    "window": dict(workload="sliding window GQA bf16 B1 Hq32 Hkv8 S32768 W4096 D128 causal", B=1, Hq=32, Hkv=8,
                   Sq=32768, Sk=32768, D=128, dtype="bf16", causal=True, W=4096),
    # a decode step of a left-padded batch (HF generate): the KV cache [B, Hkv, 4096, D] read in
    # place, sequence b's real keys the last lens[b] positions (mixed lengths 1024 .. 4000);
    # flash_attn_padded_func -> q-head pack + split-KV decode kernel on each sequence's key range
    "decode_padded": dict(workload="padded decode GQA bf16 B32 Hq32 Hkv8 Sq1 Sk<=4096 (lens 1024..4000, left "
                                   "padding) D128", B=32, Hq=32, Hkv=8, Sq=1, Sk=4096, D=128, dtype="bf16",
                          causal=True, lens=[1024 + 96 * i for i in range(32)]),
}


def metric_of(key: str, c) -> str:
    """BASELINE.json's metric string for C2; the same metric named after the workload elsewhere."""
    if key == "c2":
        return METRIC
    if key == "c5_layer":
        return f"patched LlamaAttention.forward tokens/s, {c['workload']}"
    return f"attn fwd TFLOPS + %MFMA peak, {c['workload']}"


def flops(c) -> float:
    if c.get("lens"):  # padded batch: each row's real keys
        return 4.0 * c["Hq"] * c["Sq"] * c["D"] * sum(c["lens"][:c["B"]])
    if c.get("W"):  # visible (query, key) pairs under the causal window (Sq == Sk >= W)
        w, s_ = c["W"], c["Sq"]
        return 4.0 * c["B"] * c["Hq"] * c["D"] * (w * (w + 1) / 2 + (s_ - w) * w)
    f = 4.0 * c["B"] * c["Hq"] * c["Sq"] * c["Sk"] * c["D"]
    return f / 2 if c["causal"] else f


def algo_bytes(c) -> int:
    if c.get("lens"):  # padded batch: q / o of every row, K / V of the real keys only
        return (2 * c["B"] * c["Hq"] * c["Sq"] * c["D"] + 2 * c["Hkv"] * c["D"] * sum(c["lens"][:c["B"]])) * 2
    return (2 * c["B"] * c["Hq"] * c["Sq"] * c["D"] + 2 * c["B"] * c["Hkv"] * c["Sk"] * c["D"]) * 2


def _lib_path(path=None) -> Path:
    return Path(path) if path else ROOT / "flash_attention_cute_amd" / "lib" / "libfa_gfx950.so"


def lib_sha16(path=None) -> str:
    """First 16 hex digits of the sha256 of the C-ABI library in the tree (the one the op loads)."""
    import hashlib

    p = _lib_path(path)
    return hashlib.sha256(p.read_bytes()).hexdigest()[:16] if p.exists() else "missing"


def _elf_sections(blob: bytes) -> dict:
    """{name: [(offset, size)]} of an ELF64 little-endian image (section headers only)."""
    shoff, = struct.unpack_from("<Q", blob, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", blob, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQ", blob, shoff + i * shentsize) for i in range(shnum)]
    stro = hdrs[shstrndx][4]
    out = {}
    for h in hdrs:
        name = blob[stro + h[0]: blob.index(b"\0", stro + h[0])].decode()
        out.setdefault(name, []).append((h[4], h[5]))
    return out


def code_sha16(path=None) -> str:
    """First 16 hex digits of a sha256 over the gfx950 DEVICE code of the library: the ``.text`` and
    ``.rodata`` (kernel descriptors) of every amdgcn code object in its ``.hip_fatbin`` offload bundles,
    one digest per object, sorted. Host code, symbol tables and the per-compile unique ids hipcc puts in
    each object are left out, so a rebuild of identical source keeps the value (the whole-file
    ``lib_sha16`` changes with every build)."""
    import hashlib

    p = _lib_path(path)
    if not p.exists():
        return "missing"
    blob = p.read_bytes()
    secs = _elf_sections(blob).get(".hip_fatbin")
    if not secs:
        return "no-device-code"
    off, size = secs[0]
    fat = blob[off: off + size]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    digests, pos = [], 0
    while (i := fat.find(magic, pos)) >= 0:
        n, = struct.unpack_from("<Q", fat, i + 24)
        q = i + 32
        for _ in range(n):
            eoff, esize, tl = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24: q + 24 + tl].decode()
            q += 24 + tl
            if "amdgcn" in triple and esize:
                co = fat[i + eoff: i + eoff + esize]
                cs = _elf_sections(co)
                h = hashlib.sha256()
                for name in (".text", ".rodata"):
                    for so, ss in cs.get(name, []):
                        h.update(co[so: so + ss])
                digests.append(h.hexdigest())
        pos = q
    return hashlib.sha256("".join(sorted(digests)).encode()).hexdigest()[:16]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(q, k, v, c, target_s: float) -> dict:
    """BASELINE.md's CPU baseline: torch SDPA fp32 (the reference op's own CPU implementation,
    reference flash_attention/flash_attention.py:6-15) on the host cores, on the whole workload when
    that fits ~20 s, else on batch 0; plus, as the "port" sub-key, oracle/fa_oracle.c (fp32,
    OpenMP) on a bounded sample of batch 0's heads."""
    import torch

    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    torch.set_num_threads(cores)
    f_all = flops(c)
    nb = c["B"] if f_all <= 20 * 1.5e12 else 1  # SDPA fp32 runs ~1.5 TFLOP/s on 16 EPYC cores
    if c.get("lens"):  # padded decode: per sequence on its real keys
        try:
            qf, kf, vf = (t.float().cpu() for t in (q, k, v))
            sk = c["Sk"]

            def run_all():
                for b, n in enumerate(c["lens"][:c["B"]]):
                    torch.nn.functional.scaled_dot_product_attention(qf[b:b + 1], kf[b:b + 1, :, sk - n:],
                                                                     vf[b:b + 1, :, sk - n:], enable_gqa=True)
            run_all()
            nrep = 5
            t0 = time.perf_counter()
            for _ in range(nrep):
                run_all()
            t_sdpa = (time.perf_counter() - t0) / nrep
            gbs = algo_bytes(c) / t_sdpa / 1e9
            return {"value": round(gbs, 3), "unit": "GB/s", "cores": torch.get_num_threads(), "kind": "reference",
                    "tflops": round(f_all / t_sdpa / 1e12, 6),
                    "sample": f"the whole workload ({c['workload']}, {t_sdpa * 1e3:.2f} ms per step, mean of {nrep} "
                              "after 1 warm-up): torch SDPA fp32 per sequence on its real keys, the reference op's "
                              "CPU path (flash_attention/flash_attention.py:6-15); bf16 algorithmic bytes",
                    "cpu_model": cpu_model()}
        except Exception as e:  # noqa: BLE001
            return {"value": None, "unit": "GB/s", "cores": cores, "kind": "reference", "error": repr(e),
                    "cpu_model": cpu_model()}
    try:
        qf, kf, vf = (t[:nb].float().cpu() for t in (q, k, v))
        causal = c["causal"] and c["Sq"] > 1
        kw = {"is_causal": causal}
        if c.get("W"):  # the window as an explicit mask
            from flash_attention_cute_amd.flash_attention import _window_mask

            kw = {"attn_mask": _window_mask(c["Sq"], c["Sk"], c["W"] - 1, causal, "cpu")}
        torch.nn.functional.scaled_dot_product_attention(qf[:, :1], kf[:, :1], vf[:, :1], **kw)
        nrep = 3
        t0 = time.perf_counter()
        for _ in range(nrep):
            torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, enable_gqa=True, **kw)
        t_sdpa = (time.perf_counter() - t0) / nrep
        f_s = flops(dict(c, B=nb))
        out = {"value": round(f_s / t_sdpa / 1e12, 6), "unit": "TFLOPS", "cores": torch.get_num_threads(),
               "kind": "reference",
               "sample": f"{'the whole workload' if nb == c['B'] else 'batch 0'} of {c['workload']} "
                         f"({f_s / 1e9:.1f} GFLOP, {t_sdpa:.3f} s per call, mean of {nrep} after 1 warm-up): "
                         "torch SDPA fp32, the reference op's CPU path (flash_attention/flash_attention.py:6-15)",
               "cpu_model": cpu_model()}
        del qf, kf, vf
    except Exception as e:  # noqa: BLE001
        out = {"value": None, "unit": "TFLOPS", "cores": cores, "kind": "reference", "error": repr(e),
               "cpu_model": cpu_model()}
    out["port"] = cpu_port(q, k, v, c, target_s, cores)
    return out


def cpu_layer_baseline(c, seed: int) -> dict:
    """c5_layer's CPU baseline: the unpatched HF LlamaAttention (fp32, SDPA, the reference's CPU
    path) on the host cores, same dims, one warm-up + 2 timed calls, in tokens/s."""
    import torch
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml

    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    torch.set_num_threads(cores)
    cfg = LlamaConfig(hidden_size=c["hidden"], intermediate_size=14336, num_attention_heads=c["Hq"],
                      num_key_value_heads=c["Hkv"], head_dim=c["D"], num_hidden_layers=1, vocab_size=128256,
                      max_position_embeddings=8192, rope_theta=5e5, attn_implementation="sdpa")
    torch.manual_seed(seed)
    attn = ml.LlamaAttention(cfg, layer_idx=0).eval()
    x = torch.randn(c["B"], c["Sq"], c["hidden"])
    pe = ml.LlamaRotaryEmbedding(cfg)(x, torch.arange(c["Sq"])[None].expand(c["B"], -1))
    with torch.no_grad():
        attn(x, pe, None)
        t0 = time.perf_counter()
        for _ in range(2):
            attn(x, pe, None)
        t = (time.perf_counter() - t0) / 2
    return {"value": round(c["B"] * c["Sq"] / t, 1), "unit": "tokens/s", "cores": torch.get_num_threads(),
            "kind": "reference", "cpu_model": cpu_model(),
            "sample": f"the whole workload ({c['B']} x {c['Sq']} tokens, {t:.2f} s per call): unpatched HF "
                      "LlamaAttention fp32 with torch SDPA (the reference op's CPU path) on the host"}


def cpu_port(q, k, v, c, target_s: float, cores: int) -> dict:
    """oracle/fa_oracle.c (the CPU restatement, fp32 arithmetic, OpenMP) on a bounded sample."""
    from oracle import fa_oracle_c as OC

    g = c["Hq"] // c["Hkv"]

    def sample(nh):
        nkv = max(1, -(-nh // g))
        return (q[:1, :nh].cpu(), k[:1, :nkv].cpu(), v[:1, :nkv].cpu())

    scale = c["D"] ** -0.5
    # calibrate on one kv group, then size the sample to about target_s seconds of CPU work
    wl = c["W"] - 1 if c.get("W") else -1
    qs, ks, vs = sample(g)
    t0 = time.perf_counter()
    OC.forward(qs, ks, vs, scale, c["causal"], threads=cores, window_left=wl)
    t1 = max(time.perf_counter() - t0, 1e-3)
    nh = int(min(c["Hq"], max(g, (target_s / t1) * g)))
    nh = max(g, (nh // g) * g)
    qs, ks, vs = sample(nh)
    t0 = time.perf_counter()
    OC.forward(qs, ks, vs, scale, c["causal"], threads=cores, window_left=wl)
    t_port = time.perf_counter() - t0
    f_sample = flops(dict(c, B=1, Hq=nh))
    return {"value": round(f_sample / t_port / 1e12, 6), "unit": "TFLOPS", "cores": cores, "kind": "port",
            "sample": f"batch 0, q-heads 0..{nh - 1} of {c['workload']} ({f_sample / 1e9:.1f} GFLOP, "
                      f"{t_port:.2f} s, oracle/fa_oracle.c fp32 OpenMP)"}


def run_mode(config_key: str, weak: bool = False, global_batch: int = 0, world: int = 1, rank: int = 0,
             emu_world: int = 0, emu_rank: int = 0) -> dict:
    """How this process's timed launches relate to the job.

    strong (default): one global problem of ``global_batch`` rows (default the config's
    ``strong_batch``, else its B) split over ``split_world`` ranks by shard.plan; this process runs
    the share of ``split_rank``. ``emu_world`` > 0 runs rank ``emu_rank``'s share of an
    ``emu_world``-way split in this one process (no torch.distributed). weak: every rank runs the
    whole configured workload (c5_layer always: a layer call per GPU)."""
    c = CONFIGS[config_key]
    emulated = emu_world > 0
    if emulated and world > 1:
        raise ValueError("--world/--rank emulate one rank's share in a single process; not under --gpus > 1")
    strong = not weak and config_key != "c5_layer"
    if emulated and not strong:
        raise ValueError("--world/--rank need the strong split (not --weak, not c5_layer)")
    split_world, split_rank = (emu_world, emu_rank) if emulated else (world, rank)
    if not 0 <= split_rank < split_world:
        raise ValueError(f"rank {split_rank} outside world {split_world}")
    default_gb = c.get("strong_batch", c["B"])
    gb = (global_batch or default_gb) if strong else c["B"]
    # the committed PMC pass (profiles/pmc_<config>.json) profiled the default N = 1 run: its traffic
    # describes these launches only when they are that whole workload
    whole = (split_world == 1 and gb == default_gb) if strong else default_gb == c["B"]
    return {"strong": strong, "split_world": split_world, "split_rank": split_rank, "emulated": emulated,
            "global_batch": gb, "whole_default_workload": whole}


def strong_calls(c, q, k, v, runs, dense_fn, window_fn, padded_fn):
    """One op call per shard.Run of a rank (strided views of the global q [B, Hq, Sq, D] / k, v
    [B, Hkv, Sk, D], no copies): [(run, call)], and the FLOPs and algorithmic bytes of those calls.
    Padded configs (``lens``: left padding) pass each run's rows' own key ranges, windowed configs
    the window."""
    import torch

    g = c["Hq"] // c["Hkv"]
    lens_all = c.get("lens")
    out, fl, by = [], 0.0, 0
    for r in runs:
        qv, kv, vv = q[r.b:r.b_end, r.h0 * g:r.h1 * g], k[r.b:r.b_end, r.h0:r.h1], v[r.b:r.b_end, r.h0:r.h1]
        cr = dict(c, B=r.b_end - r.b, Hq=(r.h1 - r.h0) * g, Hkv=r.h1 - r.h0)
        if lens_all:
            cr["lens"] = list(lens_all[r.b:r.b_end])
            k_end = torch.full((cr["B"],), c["Sk"], dtype=torch.int32, device=q.device)
            k_start = k_end - torch.tensor(cr["lens"], dtype=torch.int32, device=q.device)
            call = (lambda a=qv, b_=kv, v_=vv, s=k_start, e=k_end: padded_fn(a, b_, v_, s, e, causal=c["causal"]))
        elif c.get("W"):
            call = (lambda a=qv, b_=kv, v_=vv: window_fn(a, b_, v_, c["W"] - 1, causal=c["causal"]))
        else:
            call = (lambda a=qv, b_=kv, v_=vv: dense_fn(a, b_, v_, causal=c["causal"]))
        out.append((r, call))
        fl += flops(cr)
        by += algo_bytes(cr)
    return out, fl, by


def load_traffic(config_key: str):
    """(HBM bytes per launch, provenance) from profiles/pmc_<config>.json -- only when that PMC pass
    profiled THIS library's device code (its ``code_sha16`` equals the loaded library's: a rebuild of
    the same source keeps it); otherwise (None, why)."""
    p = ROOT / "profiles" / f"pmc_{config_key}.json"
    if not p.exists():
        return None, {"traffic_source": None}
    try:
        d = json.loads(p.read_text())
    except Exception:  # noqa: BLE001
        return None, {"traffic_source": None}
    prof, cur = d.get("code_sha16"), code_sha16()
    if prof != cur:
        return None, {"traffic_stale": True, "traffic_profiled_lib": prof, "traffic_this_lib": cur,
                      "traffic_of_profiled_lib": d.get("hbm_bytes_per_launch")}
    return d.get("hbm_bytes_per_launch"), {"traffic_stale": False, "traffic_source": f"profiles/pmc_{config_key}.json"}


def roofline(c, kern_ms: float, traffic, rank_flops=None, rank_bytes=None, median=None):
    """Roofline of the attention kernel: MFMA-bound for prefill (intensity ~2 kFLOP/B at S=4096),
    HBM-bound for decode (Sq = 1: one pass over K/V per q-head group). ``rank_*``: the work of the
    launches timed (one rank's shard under --strong), default the whole config. ``achieved`` is the mean
    over the timed launches; ``median`` = (median ms per launch, launches) of individually timed
    launches (BASELINE.md's statistic), reported beside it as ``kernel_ms_median`` / ``frac_median``."""
    fl = flops(c) if rank_flops is None else rank_flops
    by = algo_bytes(c) if rank_bytes is None else rank_bytes
    gbs = by / (kern_ms * 1e-3) / 1e9
    tf = fl / (kern_ms * 1e-3) / 1e12
    traffic, prov = traffic if isinstance(traffic, tuple) else (traffic, {})
    base = {"traffic": traffic, **prov, "kernel_ms": round(kern_ms, 4), "algorithmic_bytes": by,
            "algorithmic_flops": fl}
    if median is not None:
        med_ms, n_med = median
        rate = by / (med_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if c["Sq"] == 1 else fl / (med_ms * 1e-3) / 1e12 / PEAK_TFLOPS
        base.update({"kernel_ms_median": round(med_ms, 4), "median_launches": n_med, "frac_median": round(rate, 4)})
    if c["Sq"] == 1:
        return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "achieved_TFLOPs": round(tf, 3), **base}
    return {"bound": "mfma", "achieved": round(tf, 3), "peak": PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / PEAK_TFLOPS, 4), "algorithmic_GBs": round(gbs, 1), **base}


def layer_setup(c, dev, dt, seed):
    """C5's caller: one Llama-3-8B attention layer (random weights; transformers' LlamaAttention with
    its forward patched to flash_attention_cute_amd.hf_attention.attention_forward, as reference
    models/patch_llama.py:4-5 does) over B x S tokens of prefill. Returns the patched step and, for
    timing beside it, the unpatched HF (SDPA) layer and the patched layer with the reference's
    unfused torch RoPE."""
    import torch
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml

    from flash_attention_cute_amd import hf_attention

    cfg = LlamaConfig(hidden_size=c["hidden"], intermediate_size=14336, num_attention_heads=c["Hq"],
                      num_key_value_heads=c["Hkv"], head_dim=c["D"], num_hidden_layers=1, vocab_size=128256,
                      max_position_embeddings=8192, rope_theta=5e5, attn_implementation="sdpa")
    torch.manual_seed(seed)
    attn = ml.LlamaAttention(cfg, layer_idx=0).to(dev, dt).eval()
    rope = ml.LlamaRotaryEmbedding(cfg).to(dev)
    x = torch.randn(c["B"], c["Sq"], c["hidden"], device=dev, dtype=dt)
    pe = rope(x, torch.arange(c["Sq"], device=dev)[None].expand(c["B"], -1))
    orig = ml.LlamaAttention.forward

    def patched_call():
        with torch.no_grad():
            return hf_attention.attention_forward(attn, x, pe, None)[0]

    def hf_call():
        with torch.no_grad():
            return orig(attn, x, pe, None)[0]

    def unfused_call():
        hf_attention.FUSE_ROPE = False
        try:
            return patched_call()
        finally:
            hf_attention.FUSE_ROPE = True

    proj = 2.0 * c["B"] * c["Sq"] * c["hidden"] * (2 * c["Hq"] * c["D"] + 2 * c["Hkv"] * c["D"])
    info = {"projection_flops": proj, "attention_flops": flops(c), "_hf_step": hf_call, "_unfused_step": unfused_call}
    return patched_call, info


def reduce_max(world: int, *vals: float):
    """Max over ranks of host-side timings (gloo, CPU tensor): the harness's only cross-rank traffic."""
    if world <= 1:
        return vals
    import torch
    import torch.distributed as dist

    t = torch.tensor(vals, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return tuple(float(x) for x in t)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="CPU port sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--strong", action="store_true", help="(the default) split one global problem over the ranks")
    ap.add_argument("--weak", action="store_true", help="every rank runs the whole configured workload instead")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong split: global batch (default: the config's; C5: 8)")
    ap.add_argument("--world", type=int, default=0,
                    help="run rank --rank's share of a --world-way strong split in this one process")
    ap.add_argument("--rank", type=int, default=0, help="see --world")
    ap.add_argument("--warmup-seconds", type=float, default=2.0,
                    help="back-to-back op calls before the W warm-up steps (the clock settles)")
    args = ap.parse_args()
    if args.strong and args.weak:
        ap.error("--strong and --weak exclude each other")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not started by torch.distributed.run: start it as a child (never exec) and pass its status on
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={29500 + os.getpid() % 1000}", __file__, *sys.argv[1:]]
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    n_gpus = world
    # BENCH_SHARE_GPU=1 (rehearsal only): every rank uses cuda:0, so the multi-rank flow can be run on
    # a one-GPU box; the numbers of such a run are not scaling numbers
    gpu = 0 if os.environ.get("BENCH_SHARE_GPU") == "1" else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    from flash_attention_cute_amd import flash_attn_func, flash_attn_padded_func, flash_attn_window_func

    c = CONFIGS[args.config]
    dt = torch.float16 if c["dtype"] == "fp16" else torch.bfloat16
    layer = args.config == "c5_layer"
    extra = {}
    try:
        mode = run_mode(args.config, weak=args.weak, global_batch=args.global_batch, world=world, rank=rank,
                        emu_world=args.world, emu_rank=args.rank)
    except ValueError as e:
        ap.error(str(e))
    if mode["strong"]:
        # one global problem, this rank's (batch, kv-head) units (shard.py); same seed on every rank
        from flash_attention_cute_amd import shard

        gb, W, R = mode["global_batch"], mode["split_world"], mode["split_rank"]
        if W == 1 and gb == c["B"]:
            c = dict(c, B=gb)
        elif mode["emulated"]:
            c = dict(c, B=gb, workload=f"{c['workload']}, global batch {gb}: rank {R}'s share of a {W}-way split")
        else:
            c = dict(c, B=gb, workload=f"{c['workload']}, global batch {gb} split over {W} GPU(s)")
        gen = torch.Generator(device=dev).manual_seed(args.seed)
        q = torch.randn(gb, c["Hq"], c["Sq"], c["D"], device=dev, dtype=dt, generator=gen)
        k = torch.randn(gb, c["Hkv"], c["Sk"], c["D"], device=dev, dtype=dt, generator=gen)
        v = torch.randn(gb, c["Hkv"], c["Sk"], c["D"], device=dev, dtype=dt, generator=gen)
        runs = shard.rank_runs(gb, c["Hkv"], W, R)
        run_calls, rank_flops, rank_bytes = strong_calls(c, q, k, v, runs, flash_attn_func, flash_attn_window_func,
                                                         flash_attn_padded_func)

        def step():
            return [f() for _, f in run_calls]

        extra["shard"] = {"units": f"{c['B'] * c['Hkv']} (batch, kv-head)", "world": W, "rank": R,
                          "rank_runs": len(runs), "rank_units": sum((r.b_end - r.b) * (r.h1 - r.h0) for r in runs)}
        if mode["emulated"]:
            extra["shard_of"] = {"world": W, "rank": R, "global_flops": flops(c), "rank_flops": rank_flops,
                                 "note": "one rank's share of the W-way strong split, run alone on this GPU"}
    else:
        if world > 1 or c.get("strong_batch", c["B"]) != c["B"]:
            c = dict(c, workload=f"{c['workload']}, B{c['B']} replica per GPU")
        gen = torch.Generator(device=dev).manual_seed(args.seed + rank)  # per-rank replica
        q = torch.randn(c["B"], c["Hq"], c["Sq"], c["D"], device=dev, dtype=dt, generator=gen)
        k = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], device=dev, dtype=dt, generator=gen)
        v = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], device=dev, dtype=dt, generator=gen)
        rank_flops, rank_bytes = flops(c), algo_bytes(c)
        if c.get("lens"):  # padded batch: left padding, sequence b's real keys the last lens[b] positions
            lens = torch.tensor(c["lens"][:c["B"]], dtype=torch.int32, device=dev)
            k_end = torch.full_like(lens, c["Sk"])
            k_start = k_end - lens

        def step():
            if c.get("lens"):
                return flash_attn_padded_func(q, k, v, k_start, k_end, causal=c["causal"])
            if c.get("W"):
                return flash_attn_window_func(q, k, v, c["W"] - 1, causal=c["causal"])
            return flash_attn_func(q, k, v, causal=c["causal"])

    if layer:
        layer_step, layer_info = layer_setup(c, dev, dt, args.seed + rank)
        extra["layer"] = layer_info

    def timed(fn, n):
        """n back-to-back calls of fn between synchronisations: (wall s, HIP-event ms per call).

        One event pair brackets the n launches on the current stream (the stream the kernel runs
        on). An event pair around EVERY launch, as round 1 / 2 had it, puts ≈6-10 µs between
        consecutive kernels on ROCm (rocprof kernel trace: 0 µs between back-to-back launches, ≈10 µs
        with the per-launch records), which is measurement overhead, not the op's."""
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record()
        for _ in range(n):
            fn()
        b.record()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, a.elapsed_time(b) / n

    def per_launch_median(fn, n):
        """(median HIP-event ms of n launches of fn, each bracketed by its own event pair, n)."""
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        torch.cuda.synchronize()
        for a, b in evs:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) for a, b in evs), n

    main_step = layer_step if layer else step
    # Device warm-up: the MI355X ramps its clock over the first ~second of sustained load, so a
    # few warm-up steps leave the timed steps on a still-rising clock (C2: 1043 TFLOPS after 5
    # warm-up steps vs 1099 after 1000, same binary and box). Run the same op back to back for
    # --warmup-seconds first, then the W warm-up steps; the timed region is still exactly K steps.
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < args.warmup_seconds:
        for _ in range(10):
            main_step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        main_step()
    torch.cuda.synchronize()

    if layer:  # the bare op and unpatched HF at the same dims, timed beside the patched layer
        for key, fn in (("bare_op_ms", step), ("hf_sdpa_layer_ms", layer_info.pop("_hf_step")),
                        ("unfused_rope_layer_ms", layer_info.pop("_unfused_step"))):
            timed(fn, 10)  # warm-up (library heuristics, first-call setup)
            extra["layer"][key] = round(timed(fn, max(args.steps, 10))[1], 4)
        for _ in range(args.warmup):
            main_step()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed, step_ms = timed(main_step, args.steps)
    if world > 1:
        dist.barrier()
    # the attention kernel alone (roofline): HIP events around the op's launches on the current stream
    kern_ms = step_ms if not layer else extra["layer"]["bare_op_ms"]
    # BASELINE.md's statistic beside the mean: the median over >= 50 launches, each between its own
    # event pair (after the timed region, so the pairs' gaps do not touch `value`)
    kern_med_ms, n_med = per_launch_median(step, max(50, args.steps))

    (elapsed,) = reduce_max(world, elapsed)

    if layer:
        tokens = n_gpus * c["B"] * c["Sq"] * args.steps
        value, unit = tokens / elapsed, "tokens/s"
        extra["layer"]["layer_ms"] = round(elapsed * 1e3 / args.steps, 4)
        extra["layer"]["hf_sdpa_tokens_per_s"] = round(c["B"] * c["Sq"] / (extra["layer"]["hf_sdpa_layer_ms"] * 1e-3), 1)
        extra["layer"]["layer_TFLOPS"] = round((extra["layer"]["projection_flops"] + extra["layer"]["attention_flops"])
                                               / (elapsed / args.steps) / 1e12, 2)
    elif mode["emulated"]:  # the one GPU's share, timed alone
        value, unit = rank_flops * args.steps / elapsed / 1e12, "TFLOPS"
    elif mode["strong"]:
        value, unit = flops(c) * args.steps / elapsed / 1e12, "TFLOPS"
    else:
        value, unit = n_gpus * flops(c) * args.steps / elapsed / 1e12, "TFLOPS"
    tf_per_gpu = value / n_gpus
    result = {
        "metric": metric_of(args.config, c),
        "value": round(value, 3),
        "unit": unit,
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "device_warmup_s": args.warmup_seconds,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if mode["strong"] else "weak",
        "vs_baseline": None,
        "dtype": c["dtype"],
        "data": ("synthetic N(0,1) q/k/v, one global seed, sharded by (batch, kv-head)" if mode["strong"] else
                 "synthetic N(0,1) q/k/v, seed + rank, resident in HBM") +
                ("; random-init Llama-3-8B attention weights, no checkpoint" if layer else ""),
        "config": {"workload": c["workload"], "batch": c["B"], "heads_q": c["Hq"], "heads_kv": c["Hkv"],
                   "seqlen_q": c["Sq"], "seqlen_kv": c["Sk"], "headdim": c["D"], "causal": c["causal"],
                   **({"window": c["W"]} if c.get("W") else {}),
                   "parallelism": (f"one rank of dp{mode['split_world']} (its (batch, kv-head) units, run alone)"
                                   if mode["emulated"] else
                                   f"dp{n_gpus}: (batch, kv-head) units of one problem split over ranks, no collective"
                                   if mode["strong"] else
                                   f"dp{n_gpus} (independent replica of the workload per GPU, no collective)")},
        "pct_mfma_peak": None if layer else round(100.0 * tf_per_gpu / PEAK_TFLOPS, 2),
        # rank 0's kernel: its FLOPs / bytes over the mean HIP-event time of its launches; the PMC
        # traffic only when these launches are the profiled (default N = 1) workload
        "roofline": roofline(c, kern_ms, load_traffic(args.config) if mode["whole_default_workload"] else
                             (None, {"traffic_source": None, "traffic_note": "launches differ from the profiled "
                                     "workload (a shard or another batch)"}),
                             rank_flops=rank_flops, rank_bytes=rank_bytes, median=(kern_med_ms, n_med)),
        "cpu_baseline": None,
        **extra,
    }
    if rank == 0 and n_gpus == 1 and not mode["emulated"] and not args.no_cpu_baseline:
        result["cpu_baseline"] = (cpu_layer_baseline(c, args.seed) if layer else
                                  cpu_baseline(q, k, v, c, args.cpu_seconds))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
