"""Multi-GPU partitioning of the attention forward.

Every (q-tile, q-head, batch) workgroup of the kernel is independent (reference
csrc/flash_attention_template.cuh:148-160: a CTA reads one q tile and the K/V of head
``h / head_q_per_group``), so the path shards with NO data-path collective. The unit of
distribution is a (batch, kv-head) pair together with its whole GQA group of q-heads, so K/V never
crosses devices and each rank streams only the K/V it owns. One process per GPU; the only
cross-rank traffic is the harness's barrier and max-of-timings (bench.py), never tensor data.

``plan(B, Hkv, world)`` splits the B*Hkv units into ``world`` contiguous, balanced ranges;
``rank_runs(...)`` turns one rank's range into runs -- whole batch rows merged into one, partial rows
as consecutive kv-heads -- each of which is ONE call of the op on strided views (no copies);
``sharded_forward`` runs them.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Tuple


@dataclass(frozen=True)
class Run:
    """Batch rows ``[b, b1)`` x kv-heads ``[h0, h1)`` (q-heads ``[h0*g, h1*g)``): one op call. A run
    spans several batch rows only when it covers all their kv-heads (``b1`` defaults to ``b + 1``)."""

    b: int
    h0: int
    h1: int
    b1: int = -1

    @property
    def b_end(self) -> int:
        return self.b + 1 if self.b1 < 0 else self.b1


def plan(batch: int, heads_kv: int, world: int) -> List[Tuple[int, int]]:
    """Balanced contiguous split of the ``batch * heads_kv`` units: [(start, stop)] per rank."""
    if batch <= 0 or heads_kv <= 0 or world <= 0:
        raise ValueError("batch, heads_kv and world must be positive")
    n = batch * heads_kv
    q, r = divmod(n, world)
    out, s = [], 0
    for i in range(world):
        e = s + q + (1 if i < r else 0)
        out.append((s, e))
        s = e
    return out


def rank_runs(batch: int, heads_kv: int, world: int, rank: int) -> List[Run]:
    """The runs of consecutive kv-heads (within one batch row) that ``rank`` owns."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    s, e = plan(batch, heads_kv, world)[rank]
    runs: List[Run] = []
    u = s
    while u < e:
        b, h = divmod(u, heads_kv)
        if h == 0 and e - u >= heads_kv:  # whole batch rows: one call over [b, b + n)
            n = (e - u) // heads_kv
            runs.append(Run(b, 0, heads_kv, b + n))
            u += n * heads_kv
            continue
        h1 = min(heads_kv, h + (e - u))
        runs.append(Run(b, h, h1))
        u += h1 - h
    return runs


def sharded_forward(q, k, v, rank: int, world: int, fn: Callable, **kw):
    """Run ``fn(q_view, k_view, v_view, **kw)`` over this rank's runs.

    ``q`` [B, Hq, Sq, D], ``k``/``v`` [B, Hkv, Sk, D] (any strides). Returns [(Run, out)] with
    ``out`` [b_end - b, (h1-h0)*g, Sq, D]: a run spans batch rows b .. b_end - 1 (one row, or whole rows of
    every kv-head). Views only: the op reads the shard in place.
    """
    B, Hq = q.shape[0], q.shape[1]
    Hkv = k.shape[1]
    if Hq % Hkv:
        raise ValueError("num_heads_q must be a multiple of num_heads_kv")
    g = Hq // Hkv
    res = []
    for run in rank_runs(B, Hkv, world, rank):
        qs = q[run.b:run.b_end, run.h0 * g:run.h1 * g]
        ks = k[run.b:run.b_end, run.h0:run.h1]
        vs = v[run.b:run.b_end, run.h0:run.h1]
        res.append((run, fn(qs, ks, vs, **kw)))
    return res


def assemble(shards, out):
    """Write [(Run, out)] from ``sharded_forward`` into the global output ``out`` [B, Hq, Sq, D]."""
    for run, o in shards:
        g = o.shape[1] // (run.h1 - run.h0)
        out[run.b:run.b_end, run.h0 * g:run.h1 * g] = o
    return out
