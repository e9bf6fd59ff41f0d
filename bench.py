#!/usr/bin/env python3
"""bench.py -- attention-forward TFLOPS and % of MFMA peak of the gfx950 FlashAttention-2 kernel.

Metric (BASELINE.json): attn fwd TFLOPS + %MFMA peak at (B,H,S,D) = (4,32,4096,128) fp16
(BASELINE configs[1], "C2": MHA, non-causal). A step is one call of the public op
``flash_attn_func`` (custom op -> C++ host API -> C-ABI -> HIP kernel) over one batch of
synthetic N(0,1) q, k, v already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|decode]

Multi-GPU (launched by torch.distributed.run, one process per GPU): every rank runs the full
workload on its own seeded shard of batch x heads (weak scaling; attention tiles are independent,
so there is no data-path collective -- SURVEY.md 8(e)). A gloo process group carries only the
barrier and the max-over-ranks of the timings.

Rank 0 prints ONE JSON line. Besides the contract fields it carries
  roofline     : the kernel's achieved TFLOP/s (algorithmic FLOPs / mean HIP-event duration of
                 the launches in the timed region) against the dense fp16 MFMA peak; ``traffic`` is
                 the HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), or null;
  cpu_baseline : the oracle/fa_oracle.c port (fp32 arithmetic, OpenMP) timed on the host cores on
                 a bounded sample of the same workload, plus torch SDPA fp32 on the same sample
                 (the CPU reference of BASELINE.md).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "attn fwd TFLOPS + %MFMA peak, (B,H,S,D)=(4,32,4096,128) fp16"
PEAK_TFLOPS = 2516.6  # 256 CU x 4 SIMD x 1024 FLOP/clk (32x32x16 f16/bf16 MFMA) x 2.4 GHz, dense
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    "c2": dict(workload="C2 MHA fp16 B4 H32 S4096 D128 non-causal", B=4, Hq=32, Hkv=32, Sq=4096,
               Sk=4096, D=128, dtype="fp16", causal=False),
    "c3": dict(workload="C3 MHA bf16 B4 H32 S8192 D128 causal", B=4, Hq=32, Hkv=32, Sq=8192, Sk=8192,
               D=128, dtype="bf16", causal=True),
    "c4": dict(workload="C4 GQA fp16 B4 Hq32 Hkv8 S4096 D128 causal", B=4, Hq=32, Hkv=8, Sq=4096,
               Sk=4096, D=128, dtype="fp16", causal=True),
    # C5: Llama-3-8B attention (Hq32 Hkv8 D128), bf16 causal prefill S4096; global batch 8 sharded
    # over (batch, kv-head) units -- one batch row per GPU at N=8 (flash_attention_cute_amd/shard.py)
    "c5": dict(workload="C5 Llama-3-8B attn bf16 causal B1(per GPU) Hq32 Hkv8 S4096 D128", B=1, Hq=32, Hkv=8,
               Sq=4096, Sk=4096, D=128, dtype="bf16", causal=True),
    "decode": dict(workload="decode GQA fp16 B32 Hq32 Hkv8 Sq1 Sk4096 D128 (q-head pack)", B=32, Hq=32,
                   Hkv=8, Sq=1, Sk=4096, D=128, dtype="fp16", causal=False),
    # long-context decode at batch 1: the same K/V bytes as "decode" in 8 (batch, kv-head) streams,
    # split over the keys (split-KV + combine)
    "decode_long": dict(workload="decode GQA bf16 B1 Hq32 Hkv8 Sq1 Sk131072 D128 (split-KV)", B=1, Hq=32, Hkv=8,
                        Sq=1, Sk=131072, D=128, dtype="bf16", causal=False),
}


def flops(c) -> float:
    f = 4.0 * c["B"] * c["Hq"] * c["Sq"] * c["Sk"] * c["D"]
    return f / 2 if c["causal"] else f


def algo_bytes(c) -> int:
    return (2 * c["B"] * c["Hq"] * c["Sq"] * c["D"] + 2 * c["B"] * c["Hkv"] * c["Sk"] * c["D"]) * 2


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(q, k, v, c, target_s: float) -> dict:
    """Time the oracle port and torch SDPA (fp32) on a bounded sample of batch 0's heads."""
    import torch
    from oracle import fa_oracle_c as OC

    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    torch.set_num_threads(cores)
    g = c["Hq"] // c["Hkv"]

    def sample(nh):
        nkv = max(1, -(-nh // g))
        return (q[:1, :nh].cpu(), k[:1, :nkv].cpu(), v[:1, :nkv].cpu())

    scale = c["D"] ** -0.5
    # calibrate on one kv group, then size the sample to about target_s seconds of CPU work
    qs, ks, vs = sample(g)
    t0 = time.perf_counter()
    OC.forward(qs, ks, vs, scale, c["causal"], threads=cores)
    t1 = max(time.perf_counter() - t0, 1e-3)
    nh = int(min(c["Hq"], max(g, (target_s / t1) * g)))
    nh = max(g, (nh // g) * g)
    qs, ks, vs = sample(nh)
    t0 = time.perf_counter()
    OC.forward(qs, ks, vs, scale, c["causal"], threads=cores)
    t_port = time.perf_counter() - t0
    f_sample = flops(dict(c, B=1, Hq=nh))
    out = {"value": round(f_sample / t_port / 1e12, 6), "unit": "TFLOPS", "cores": cores, "kind": "port",
           "sample": f"batch 0, q-heads 0..{nh - 1} of {c['workload']} ({f_sample / 1e9:.1f} GFLOP, "
                     f"{t_port:.2f} s, oracle/fa_oracle.c fp32 OpenMP)",
           "cpu_model": cpu_model()}
    # torch SDPA fp32 on the same sample (BASELINE.md's CPU reference): 1 warm-up + 3 reps
    try:
        qf, kf, vf = (t.float() for t in (qs, ks, vs))
        nrep = 3
        torch.nn.functional.scaled_dot_product_attention(qf[:, :1], kf[:, :1], vf[:, :1], is_causal=c["causal"])
        t0 = time.perf_counter()
        for _ in range(nrep):
            torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, is_causal=c["causal"] and c["Sq"] > 1,
                                                             enable_gqa=True)
        t_sdpa = (time.perf_counter() - t0) / nrep
        out["sdpa_fp32"] = {"value": round(f_sample / t_sdpa / 1e12, 6), "unit": "TFLOPS",
                            "threads": torch.get_num_threads(), "seconds": round(t_sdpa, 3)}
    except Exception as e:  # noqa: BLE001
        out["sdpa_fp32"] = {"error": repr(e)}
    return out


def load_traffic(config_key: str):
    p = ROOT / "profiles" / f"pmc_{config_key}.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text()).get("hbm_bytes_per_launch")
    except Exception:  # noqa: BLE001
        return None


def roofline(c, kern_ms: float, traffic):
    """Roofline of the attention kernel: MFMA-bound for prefill (intensity ~2 kFLOP/B at S=4096),
    HBM-bound for decode (Sq = 1: one pass over K/V per q-head group)."""
    gbs = algo_bytes(c) / (kern_ms * 1e-3) / 1e9
    tf = flops(c) / (kern_ms * 1e-3) / 1e12
    base = {"traffic": traffic, "kernel_ms": round(kern_ms, 4), "algorithmic_bytes": algo_bytes(c),
            "algorithmic_flops": flops(c)}
    if c["Sq"] == 1:
        return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "achieved_TFLOPs": round(tf, 3), **base}
    return {"bound": "mfma", "achieved": round(tf, 3), "peak": PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / PEAK_TFLOPS, 4), "algorithmic_GBs": round(gbs, 1), **base}


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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--warmup-seconds", type=float, default=2.0,
                    help="back-to-back op calls before the W warm-up steps (the clock settles)")
    args = ap.parse_args()

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

    from flash_attention_cute_amd import flash_attn_func

    c = CONFIGS[args.config]
    dt = torch.float16 if c["dtype"] == "fp16" else torch.bfloat16
    gen = torch.Generator(device=dev).manual_seed(args.seed + rank)  # per-rank shard of batch x heads
    q = torch.randn(c["B"], c["Hq"], c["Sq"], c["D"], device=dev, dtype=dt, generator=gen)
    k = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], device=dev, dtype=dt, generator=gen)
    v = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], device=dev, dtype=dt, generator=gen)

    def step():
        return flash_attn_func(q, k, v, causal=c["causal"])

    # Device warm-up: the MI355X ramps its clock over the first ~second of sustained load, so a
    # few warm-up steps leave the timed steps on a still-rising clock (C2: 1043 TFLOPS after 5
    # warm-up steps vs 1099 after 1000, same binary and box). Run the same op back to back for
    # --warmup-seconds first, then the W warm-up steps; the timed region is still exactly K steps.
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < args.warmup_seconds:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        step()
        ev[i][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    elapsed, kern_ms = reduce_max(world, elapsed, kern_ms)

    f_step = flops(c)
    value = n_gpus * f_step * args.steps / elapsed / 1e12
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "TFLOPS",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "device_warmup_s": args.warmup_seconds,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": c["dtype"],
        "data": "synthetic N(0,1) q/k/v, seed + rank, resident in HBM",
        "config": {"workload": c["workload"], "batch": c["B"], "heads_q": c["Hq"], "heads_kv": c["Hkv"],
                   "seqlen_q": c["Sq"], "seqlen_kv": c["Sk"], "headdim": c["D"], "causal": c["causal"],
                   "parallelism": f"dp{n_gpus} (independent batch x head shard per GPU, no collective)"},
        "pct_mfma_peak": round(100.0 * value / n_gpus / PEAK_TFLOPS, 2),
        "roofline": roofline(c, kern_ms, load_traffic(args.config)),
        "cpu_baseline": None,
    }
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(q, k, v, c, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
