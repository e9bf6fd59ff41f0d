"""Multi-GPU partitioning on CPU: shard planner properties, and a world_size-2
gloo run in which every rank computes its (batch, kv-head) shard with the oracle and the shards
reassemble into the single-process result. The gloo all-reduce here is the TEST's check, not part of
the path (the path has no collective)."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flash_attention_cute_amd import shard


@pytest.mark.parametrize("B,H,W", [(4, 32, 8), (4, 8, 8), (1, 8, 3), (3, 5, 4), (2, 2, 8), (32, 8, 8)])
def test_plan_is_a_balanced_partition(B, H, W):
    p = shard.plan(B, H, W)
    assert len(p) == W and p[0][0] == 0 and p[-1][1] == B * H
    assert all(a[1] == b[0] for a, b in zip(p, p[1:]))
    sizes = [e - s for s, e in p]
    assert max(sizes) - min(sizes) <= 1
    seen = []
    for r in range(W):
        runs = shard.rank_runs(B, H, W, r)
        for run in runs:
            assert 0 <= run.b < run.b_end <= B and 0 <= run.h0 < run.h1 <= H
            assert run.b_end == run.b + 1 or (run.h0, run.h1) == (0, H)  # multi-row runs are whole rows
            seen += [(b, h) for b in range(run.b, run.b_end) for h in range(run.h0, run.h1)]
        assert len(runs) <= 3  # a partial row, whole rows in one call, a partial row
    assert sorted(seen) == [(b, h) for b in range(B) for h in range(H)]


def test_plan_rejects_bad_arguments():
    with pytest.raises(ValueError):
        shard.plan(0, 8, 2)
    with pytest.raises(ValueError):
        shard.rank_runs(2, 8, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import fa_oracle_c as OC

        B, Hq, Hkv, Sq, Sk, D, causal = case
        g = torch.Generator().manual_seed(0)  # every rank draws the same global tensors
        q = torch.randn(B, Hq, Sq, D, generator=g).half()
        k = torch.randn(B, Hkv, Sk, D, generator=g).half()
        v = torch.randn(B, Hkv, Sk, D, generator=g).half()
        scale = D ** -0.5
        parts = shard.sharded_forward(q, k, v, rank, world,
                                      lambda a, b_, c: OC.forward(a.contiguous(), b_.contiguous(), c.contiguous(),
                                                                  scale, causal, threads=1))
        out = shard.assemble(parts, torch.zeros(B, Hq, Sq, D, dtype=torch.float32))
        cover = torch.zeros(B, Hq)
        for run, _ in parts:
            cover[run.b:run.b_end, run.h0 * (Hq // Hkv):run.h1 * (Hq // Hkv)] = 1
        dist.all_reduce(out)
        dist.all_reduce(cover)
        if rank == 0:
            ref = OC.forward(q, k, v, scale, causal, threads=2).float()
            ret.put((float((out - ref).abs().max()), float(cover.min()), float(cover.max())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", [(2, 8, 2, 40, 40, 64, True), (3, 4, 4, 17, 33, 32, False)])
def test_world2_gloo_shards_reassemble_to_single_process_result(case):
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, ret)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    err, cmin, cmax = ret.get(timeout=5)
    assert err == 0.0 and cmin == 1.0 and cmax == 1.0
