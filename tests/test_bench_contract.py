"""bench.py's measurement bookkeeping on CPU: the PMC traffic it reports is tied to the library that
ran ("roofline.traffic is a stored constant"), and the roofline arithmetic uses the
algorithmic FLOPs / bytes of DESIGN.md section 5. No GPU needed."""
import json
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


_KERNEL = """#include <hip/hip_runtime.h>
__global__ void k(float *x) { x[threadIdx.x] *= %s; }
extern "C" int run(float *x, hipStream_t s) { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, x); return 0; }
"""


@pytest.fixture(scope="module")
def tiny_libs(tmp_path_factory):
    """Three gfx950 libraries built here by hipcc: a and b from the SAME source (two compiles), c from a
    kernel with another constant."""
    hipcc = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "bin" / "hipcc"
    if not hipcc.exists():
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("tiny")
    out = {}
    for name, const in (("a", "2.f"), ("b", "2.f"), ("c", "3.f")):
        src = d / f"{name}.hip"
        src.write_text(_KERNEL % const)
        subprocess.run([str(hipcc), "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", str(src), "-o",
                        str(d / f"{name}.so")], check=True, capture_output=True)
        out[name] = d / f"{name}.so"
    return out


def _fake_tree(tmp_path, lib: Path, pmc: dict | None):
    (tmp_path / "flash_attention_cute_amd" / "lib").mkdir(parents=True, exist_ok=True)
    shutil.copyfile(lib, tmp_path / "flash_attention_cute_amd" / "lib" / "libfa_gfx950.so")
    (tmp_path / "profiles").mkdir(exist_ok=True)
    if pmc is not None:
        (tmp_path / "profiles" / "pmc_c2.json").write_text(json.dumps(pmc))


def test_device_code_hash_survives_a_rebuild(tiny_libs):
    """Two compiles of one source differ as files (hipcc's per-compile ids) but not in device code;
    another kernel differs in both ("traffic provenance breaks on any rebuild")."""
    a, b, c = (tiny_libs[n] for n in "abc")
    assert bench.lib_sha16(a) != bench.lib_sha16(b)
    assert bench.code_sha16(a) == bench.code_sha16(b)
    assert bench.code_sha16(a) != bench.code_sha16(c)
    assert all(len(bench.code_sha16(x)) == 16 for x in (a, b, c))


def test_traffic_is_used_only_for_the_profiled_device_code(tmp_path, monkeypatch, tiny_libs):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    _fake_tree(tmp_path, tiny_libs["a"], None)
    code = bench.code_sha16()
    (tmp_path / "profiles" / "pmc_c2.json").write_text(
        json.dumps({"lib_sha16": bench.lib_sha16(), "code_sha16": code, "hbm_bytes_per_launch": 123.0}))
    traffic, why = bench.load_traffic("c2")
    assert traffic == 123.0 and why["traffic_stale"] is False
    # a rebuild of the same source: another file, the same device code -> still this traffic
    _fake_tree(tmp_path, tiny_libs["b"], None)
    traffic, why = bench.load_traffic("c2")
    assert traffic == 123.0 and why["traffic_stale"] is False
    # other device code, the committed PMC file unchanged: no stale number, and the reason says why
    _fake_tree(tmp_path, tiny_libs["c"], None)
    traffic, why = bench.load_traffic("c2")
    assert traffic is None and why["traffic_stale"] is True
    assert why["traffic_profiled_lib"] == code and why["traffic_this_lib"] != code
    assert why["traffic_of_profiled_lib"] == 123.0


def test_traffic_absent_without_a_pmc_file(tmp_path, monkeypatch, tiny_libs):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    _fake_tree(tmp_path, tiny_libs["a"], None)
    assert bench.load_traffic("c2") == (None, {"traffic_source": None})


def test_committed_pmc_files_carry_a_library_hash():
    for p in sorted((ROOT / "profiles").glob("pmc_*.json")):
        d = json.loads(p.read_text())
        assert len(d.get("lib_sha16", "")) == 16 and len(d.get("code_sha16", "")) == 16, p.name
        assert d["hbm_bytes_per_launch"] > 0, p.name


def test_algorithmic_counts_of_the_headline_config():
    c = bench.CONFIGS["c2"]
    assert bench.flops(c) == 4 * 4 * 32 * 4096 * 4096 * 128  # 4 Sq Sk D per (b, head), non-causal
    assert bench.algo_bytes(c) == 536870912  # q, k, v, o once each


# ---- multi-GPU mode of bench.py: strong split by default, one rank's share alone ----
import os  # noqa: E402
import socket  # noqa: E402

import pytest  # noqa: E402


def test_run_mode_defaults_to_the_strong_split():
    m = bench.run_mode("c2")
    assert m["strong"] and m["split_world"] == 1 and m["global_batch"] == 4 and m["whole_default_workload"]
    m = bench.run_mode("c2", world=8, rank=3)
    assert m["strong"] and (m["split_world"], m["split_rank"]) == (8, 3) and not m["whole_default_workload"]
    m = bench.run_mode("c5")  # BASELINE C5: global batch 8, also at N = 1 (the PMC-profiled workload)
    assert m["strong"] and m["global_batch"] == 8 and m["whole_default_workload"]
    m = bench.run_mode("c5", weak=True)  # a B1 replica: not the profiled launches
    assert not m["strong"] and m["global_batch"] == 1 and not m["whole_default_workload"]
    m = bench.run_mode("c2", weak=True, world=8, rank=1)
    assert not m["strong"] and m["whole_default_workload"]
    assert not bench.run_mode("c5_layer")["strong"]


def test_run_mode_emulates_one_rank_share():
    m = bench.run_mode("c2", emu_world=8, emu_rank=0)
    assert m["emulated"] and m["strong"] and (m["split_world"], m["split_rank"]) == (8, 0)
    assert not m["whole_default_workload"]  # no PMC traffic for a shard
    for kw in (dict(emu_world=8, emu_rank=8), dict(emu_world=2, world=2), dict(emu_world=2, weak=True)):
        with pytest.raises(ValueError):
            bench.run_mode("c2", **kw)


def test_c5_workload_label_names_the_mode():
    assert "replica" not in bench.CONFIGS["c5"]["workload"]  # the strong (default) line's label


class _FakeRun:
    def __init__(self, b, b_end, h0, h1):
        self.b, self.b_end, self.h0, self.h1 = b, b_end, h0, h1


def test_strong_calls_count_each_shards_own_work():
    import torch

    from flash_attention_cute_amd import shard

    for key in ("c2", "c4", "decode_padded", "window"):
        c = dict(bench.CONFIGS[key])
        B = c["B"]
        q = torch.empty(B, c["Hq"], 1, 8)  # (shapes only: the calls are not run)
        k = torch.empty(B, c["Hkv"], 1, 8)
        tot_f = tot_b = 0
        for r in range(8):
            calls, f, b = bench.strong_calls(c, q, k, k, shard.rank_runs(B, c["Hkv"], 8, r), None, None, None)
            assert calls
            tot_f += f
            tot_b += b
        assert abs(tot_f - bench.flops(c)) <= 1e-9 * bench.flops(c), key
        assert tot_b == bench.algo_bytes(c), key


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _strong_worker(rank, world, port, ret):
    """bench.py's strong path with the reference op's CPU implementation (torch SDPA, what
    torch.ops.flash_attention.forward runs on CPU tensors): each rank runs only its shard's calls."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flash_attention_cute_amd import shard

        c = dict(bench.CONFIGS["c4"], B=2, Sq=48, Sk=48, D=32)
        g = torch.Generator().manual_seed(0)  # one global problem on every rank
        q = torch.randn(c["B"], c["Hq"], c["Sq"], c["D"], generator=g)
        k = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], generator=g)
        v = torch.randn(c["B"], c["Hkv"], c["Sk"], c["D"], generator=g)

        def dense(a, b_, v_, causal):
            return torch.nn.functional.scaled_dot_product_attention(a, b_, v_, is_causal=causal, enable_gqa=True)

        m = bench.run_mode("c4", world=world, rank=rank)
        runs = shard.rank_runs(c["B"], c["Hkv"], m["split_world"], m["split_rank"])
        calls, f, _ = bench.strong_calls(c, q, k, v, runs, dense, None, None)
        out = torch.zeros_like(q)
        shard.assemble([(r, fn()) for r, fn in calls], out)
        dist.all_reduce(out)
        tf = torch.tensor([f], dtype=torch.float64)
        dist.all_reduce(tf)
        (tmax,) = bench.reduce_max(world, float(rank + 1))
        if rank == 0:
            ref = dense(q, k, v, True)
            ret.put((float((out - ref).abs().max()), float(tf[0]) / bench.flops(c), tmax))
    finally:
        dist.destroy_process_group()


def test_world2_gloo_strong_split_reassembles_the_global_problem():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, 2, port, ret)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    err, frac, tmax = ret.get(timeout=5)
    assert err <= 1e-6 and frac == pytest.approx(1.0) and tmax == 2.0
