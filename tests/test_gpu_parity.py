"""GPU parity of the gfx950 kernel against the CPU oracle (and torch SDPA), through the public op.

Every case calls ``flash_attn_func`` (reference flash_attention/flash_attention.py:46-53) on
cuda:0, i.e. the custom op -> C++ host API -> C-ABI ``fa_fwd_gfx950`` -> HIP kernel, and compares
with oracle/fa_oracle.c run on the same seeded inputs (same arithmetic widths: fp32 accumulation,
P rounded to T before P.V). The sweep follows SURVEY.md section 4: dtype x causal x
{MHA, GQA, MQA} x {Sq == Sk, Sq == 1 (decode pack), Sq < Sk, Sq > Sk} x D x ragged lengths x
strided (transposed-view) inputs.

Tolerances (written per test):
  fp16: |gpu - oracle| <= 2e-3 + 2e-3*|oracle|, mean error <= 1e-4
  bf16: |gpu - oracle| <= 1.6e-2 + 1.6e-2*|oracle|, mean error <= 1e-3
One output ulp is 9.8e-4 (fp16) / 7.8e-3 (bf16) at |O| ~ 1; the bounds allow the one-ulp flips that
a different fp32 summation order and the hardware exp2 produce, nothing systematic.
"""
from __future__ import annotations

import zlib

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O
from oracle import fa_oracle_c as OC

pytestmark = pytest.mark.gpu

TOL = {torch.float16: (2e-3, 2e-3, 1e-4), torch.bfloat16: (1.6e-2, 1.6e-2, 1e-3)}


class _Variant:
    """A debug / A-B kernel body (w8, w4slow, p8) of lib/libfa_gfx950_debug.so through its C-ABI with
    the op's host steps restated (flash_attention_cute_amd._debug.forward); the product library the op
    loads compiles fa_fwd_w4 only."""

    def __init__(self, variant):
        self.variant = variant

    def __call__(self, q, k, v, softmax_scale=None, causal=False):
        from flash_attention_cute_amd import _debug

        return _debug.forward(q, k, v, softmax_scale, causal, variant=self.variant)


@pytest.fixture(params=["w4", "w8", "w4slow", "p8", "m16", "m32"])
def fa(device, request):
    """The public op (the product kernel w4), or one of the debug library's bodies (the 8-wave
    cross-check w8, the non-pipelined w4slow, the paired 8-wave p8). Function-scoped: the knobs are
    restored to their defaults after every test."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug
    from flash_attention_cute_amd import flash_attention as fam

    assert fam.flash_attention_cuda is not None, f"gfx950 extension failed to load: {fam._load_error!r}"
    _debug.set_knobs()
    if request.param == "w4":
        m.flash_attn_func.variant = "w4"
        yield m.flash_attn_func
        return
    try:
        yield _Variant(request.param)
    finally:
        _debug.set_knobs(debug=True)


def assert_path(variant, hq, hkv, sq):
    """The kernel the last call launched: the decode kernel for few rows per kv-head under the
    default variant (g * Sq <= 64, the Sq == 1 pack included), else the selected prefill body."""
    from flash_attention_cute_amd import _debug

    rows = (hq // hkv) * sq if sq > 1 else hq // hkv
    if variant == "w4" and rows <= 64:
        assert _debug.last_path() in ("decode", "decode_split"), _debug.last_path()
    else:
        path = _debug.last_path(debug=variant != "w4")
        assert path == variant, (path, variant)


def make(b, hq, hkv, sq, sk, d, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(b, hq, sq, d, generator=g).to(dtype)
    k = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    v = torch.randn(b, hkv, sk, d, generator=g).to(dtype)
    return q, k, v


def check(out_gpu, q, k, v, scale, causal, dtype):
    ref = OC.forward(q, k, v, scale, causal).float()
    got = out_gpu.float().cpu()
    assert got.shape == ref.shape
    sq, sk = q.shape[2], k.shape[2]
    keep = torch.from_numpy(~O.fully_masked_rows(sq, sk, causal))
    fm = ~keep
    if fm.any():  # rows that see no key are defined as 0
        assert torch.all(got[:, :, fm, :] == 0)
    got, ref = got[:, :, keep, :], ref[:, :, keep, :]
    assert torch.isfinite(got).all()
    atol, rtol, mean_tol = TOL[dtype]
    err = (got - ref).abs()
    bound = atol + rtol * ref.abs()
    worst = (err - bound).max().item()
    assert worst <= 0, f"max err {err.max().item():.3e} exceeds bound by {worst:.3e}"
    assert err.mean().item() <= mean_tol, f"mean err {err.mean().item():.3e}"


SHAPES = [  # (B, Hq, Hkv, Sq, Sk)
    (1, 2, 2, 128, 128),      # MHA, exact tiles
    (2, 4, 1, 300, 300),      # MQA, ragged (not a multiple of 64 / 256)
    (1, 8, 2, 1, 257),        # GQA decode -> q-head pack path
    (1, 4, 2, 100, 333),      # Sq < Sk (bottom-right causal offset)
    (1, 2, 2, 333, 100),      # Sq > Sk (fully masked rows when causal)
    (1, 2, 1, 520, 77),       # several q tiles, short kv
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("causal", [False, True], ids=["full", "causal"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("d", [128, 64])
def test_parity_sweep(fa, device, dtype, causal, shape, d):
    b, hq, hkv, sq, sk = shape
    seed = zlib.crc32(repr((shape, d, causal, str(dtype))).encode())
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, seed)
    out = fa(q.to(device), k.to(device), v.to(device), causal=causal)
    assert_path(fa.variant, hq, hkv, sq)
    torch.cuda.synchronize()
    check(out, q, k, v, d ** -0.5, causal, dtype)


@pytest.mark.parametrize("d", [8, 40, 72, 96, 120])
def test_headdims_multiple_of_8(fa, device, d):
    q, k, v = make(1, 2, 2, 200, 190, d, torch.float16, d)
    out = fa(q.to(device), k.to(device), v.to(device), causal=True)
    check(out, q, k, v, d ** -0.5, True, torch.float16)


@pytest.mark.parametrize("d", [36, 100])
def test_headdim_padding_path(fa, device, d):
    # D % 8 != 0: the python wrapper zero-pads to a multiple of 8 (reference flash_attention.py:26-31)
    q, k, v = make(1, 2, 2, 130, 130, d, torch.float16, d)
    out = fa(q.to(device), k.to(device), v.to(device))
    assert out.shape == q.shape
    pad = [0, 8 - d % 8]
    qp, kp, vp = (torch.nn.functional.pad(t, pad) for t in (q, k, v))
    ref = OC.forward(qp, kp, vp, d ** -0.5, False)[..., :d].float()
    assert (out.float().cpu() - ref).abs().max().item() < 2e-3


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_strided_hf_layout(fa, device, dtype):
    # HF attention passes q/k/v as transpose(1, 2) views of [B, S, H, D] (models/rope_attn_fwd.py:81-85)
    b, s, hq, hkv, d = 2, 257, 8, 2, 128
    g = torch.Generator().manual_seed(7)
    q4 = torch.randn(b, s, hq, d, generator=g).to(dtype)
    k4 = torch.randn(b, s, hkv, d, generator=g).to(dtype)
    v4 = torch.randn(b, s, hkv, d, generator=g).to(dtype)
    qd, kd, vd = (t.to(device).transpose(1, 2) for t in (q4, k4, v4))
    assert not qd.is_contiguous()
    out = fa(qd, kd, vd, causal=True)
    # stride-preserving output: o inherits q's physical [B, S, H, D] layout (api.cpp:85)
    assert out.stride() == qd.stride()
    assert out.transpose(1, 2).is_contiguous()
    check(out, *(t.transpose(1, 2).contiguous() for t in (q4, k4, v4)), d ** -0.5, True, dtype)


def test_custom_scale_and_default_scale(fa, device):
    q, k, v = make(1, 2, 2, 64, 64, 128, torch.float16, 3)
    out = fa(q.to(device), k.to(device), v.to(device), softmax_scale=0.3)
    check(out, q, k, v, 0.3, False, torch.float16)
    out2 = fa(q.to(device), k.to(device), v.to(device))
    check(out2, q, k, v, 128 ** -0.5, False, torch.float16)


def test_online_softmax_rescale_forced(fa, device):
    # A key aligned with a component shared by every query makes the running max of every row jump
    # at KV tile 5 (guide rule 26): the O / l rescale branch is taken by all waves at that tile.
    q, k, v = make(1, 2, 2, 256, 512, 128, torch.float16, 11)
    u = torch.randn(128, generator=torch.Generator().manual_seed(1))
    u = u / u.norm()
    q = (q.float() + 3 * u).to(torch.float16)
    k[:, :, 5 * 64 + 3, :] = (12 * u).to(torch.float16)
    v[:, :, 5 * 64 + 3, :] = 3.0
    out = fa(q.to(device), k.to(device), v.to(device))
    check(out, q, k, v, 128 ** -0.5, False, torch.float16)


def test_against_sdpa_reference_bar(fa, device):
    # The reference's own accuracy bar (scripts/benchmark_kernel.py:120-123): allclose(atol=1e-3)
    # against fp32 eager attention, fp16, Sq == Sk so the top-left mask of SDPA equals ours.
    q, k, v = make(2, 8, 2, 1024, 1024, 128, torch.float16, 5)
    for causal in (False, True):
        out = fa(q.to(device), k.to(device), v.to(device), causal=causal)
        ref = torch.nn.functional.scaled_dot_product_attention(
            q.to(device).float(), k.to(device).float(), v.to(device).float(), is_causal=causal,
            enable_gqa=True)
        assert torch.allclose(out.float(), ref, atol=1e-3), (out.float() - ref).abs().max().item()


def test_deterministic(fa, device):
    q, k, v = (t.to(device) for t in make(2, 8, 8, 777, 777, 128, torch.bfloat16, 9))
    a = fa(q, k, v, causal=True)
    b = fa(q, k, v, causal=True)
    assert torch.equal(a, b)


def test_inputs_not_mutated(fa, device):
    q, k, v = (t.to(device) for t in make(1, 4, 2, 100, 100, 64, torch.float16, 13))
    c = [t.clone() for t in (q, k, v)]
    fa(q, k, v, causal=True)
    assert all(torch.equal(a, b) for a, b in zip((q, k, v), c))


def test_errors_are_runtime_errors(fa, device):
    """The op's validation (reference csrc/flash_attention_api.cpp:17-59 messages): host code, the same
    whatever kernel body the library carries -- checked on the product op."""
    if fa.variant != "w4":
        pytest.skip("host-side validation of the op: product library only")
    q = torch.randn(1, 3, 64, 64, device=device, dtype=torch.float16)
    k = torch.randn(1, 2, 64, 64, device=device, dtype=torch.float16)
    with pytest.raises(RuntimeError, match="multiple of number of heads"):
        fa(q, k, k)
    q32 = torch.randn(1, 2, 64, 64, device=device)
    with pytest.raises(RuntimeError, match="fp16 or bf16"):
        fa(q32, q32, q32)
    big = torch.randn(1, 2, 64, 192, device=device, dtype=torch.float16)
    with pytest.raises(RuntimeError, match="<= 128"):
        fa(big, big, big)


@pytest.mark.parametrize("grid", ["1", "5", "8", "13", "20", "64"])
def test_persistent_grid_sizes(device, grid):
    """fa_fwd_w4 is persistent (a workgroup walks Q blocks, snake-ordered rounds per XCD residue
    class); forcing small grids (the w4_grid knob, rounded by the host to >= 8 / multiples of 8)
    must cover every block and give the default launch's output bit for bit."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    cases = [(2, 8, 2, 700, 700, 128, torch.float16, True), (3, 6, 6, 513, 640, 64, torch.bfloat16, False),
             (1, 12, 4, 1100, 1100, 96, torch.float16, True)]
    for i, (b, hq, hkv, sq, sk, d, dt, causal) in enumerate(cases):
        q, k, v = make(b, hq, hkv, sq, sk, d, dt, 300 + i)
        qd, kd, vd = (t.to(device) for t in (q, k, v))
        ref = m.flash_attn_func(qd, kd, vd, causal=causal)
        assert _debug.last_path() == "w4"
        with _debug.knobs(w4_grid=int(grid)):
            got = m.flash_attn_func(qd, kd, vd, causal=causal)
            assert _debug.last_path() == "w4"
        torch.cuda.synchronize()
        assert torch.equal(got, ref), (grid, i, (got.float() - ref.float()).abs().max().item())
        if i == 0:
            check(got, q, k, v, d ** -0.5, causal, dt)


@pytest.mark.parametrize("shape", [(2, 8, 2, 640, 640, 128, True), (4, 32, 8, 1, 3000, 128, False)])
def test_hip_graph_capture_replay(device, shape):
    """The op launches asynchronously on the caller's stream with no host sync, so it can be
    captured into a HIP graph (torch.cuda.CUDAGraph) and replayed: prefill (persistent fa_fwd_w4)
    and Sq == 1 decode (split-KV kernel + combine, stream-ordered workspace)."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d, causal = shape
    q, k, v = (t.to(device) for t in make(b, hq, hkv, sq, sk, d, torch.float16, 77))
    ref = m.flash_attn_func(q, k, v, causal=causal)
    # the product path, not a variant left behind by another test: w4, or split-KV decode + combine
    assert _debug.last_path() == ("decode_split" if sq == 1 else "w4"), _debug.last_path()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up on the side stream, as torch's graph docs prescribe
        m.flash_attn_func(q, k, v, causal=causal)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = m.flash_attn_func(q, k, v, causal=causal)
    for seed in (78, 79):  # replay on new inputs written in place
        q2, k2, v2 = make(b, hq, hkv, sq, sk, d, torch.float16, seed)
        q.copy_(q2)
        k.copy_(k2)
        v.copy_(v2)
        g.replay()
        torch.cuda.synchronize()
        eager = m.flash_attn_func(q, k, v, causal=causal)
        assert torch.equal(out, eager)
    assert not torch.equal(out, ref)


ZIGZAG = [  # (B, Hq, Hkv, Sq, Sk, D): causal launches that fit one round of the grid
    (1, 4, 2, 1024, 1024, 128),   # 8 segments -> 4 blocks per head
    (2, 2, 1, 640, 640, 64),      # 5 segments: the middle one has no partner
    (1, 2, 2, 700, 900, 128),     # Sq < Sk: bottom-right offset, ragged last segment
    (1, 2, 1, 600, 333, 128),     # Sq > Sk: rows that see no key
    (1, 3, 3, 200, 200, 96),      # 2 segments, padded head dim tile
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
@pytest.mark.parametrize("shape", ZIGZAG, ids=lambda s: "x".join(map(str, s)))
def test_zigzag_causal_blocks(device, shape, dtype):
    """Causal launches whose 256-row blocks fit one round of the persistent grid pair the 128-row
    segments t and nseg - 1 - t (fa_fwd_w4 "Zigzag Q blocks": equal work per block); with the layout
    forced on and off, both against the oracle, two launches bit-identical."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d = shape
    seed = zlib.crc32(repr((shape, str(dtype), "zz")).encode())
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, seed)
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    _debug.set_knobs()
    _debug.set_split(0)  # (the op's default for these grids is the key-split layout: tested below)
    try:
        out = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_path() == "w4" and _debug.last_zigzag()  # picked for a small grid
        again = m.flash_attn_func(qd, kd, vd, causal=True)
        _debug.set_zigzag(0)
        plain = m.flash_attn_func(qd, kd, vd, causal=True)
        assert not _debug.last_zigzag()
        torch.cuda.synchronize()
    finally:
        _debug.set_zigzag()
        _debug.set_split()
    assert torch.equal(out, again)
    check(out, q, k, v, d ** -0.5, True, dtype)
    check(plain, q, k, v, d ** -0.5, True, dtype)


def test_zigzag_only_where_it_applies(device):
    """Non-causal, windowed and large-grid causal launches keep the plain layout; mode 2 forces the
    zigzag on a large causal grid too (and stays exact), mode 0 keeps it off on a small one."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    q, k, v = (t.to(device) for t in make(1, 2, 2, 512, 512, 128, torch.float16, 5))
    _debug.set_split(0)
    try:
        m.flash_attn_func(q, k, v, causal=False)
        assert not _debug.last_zigzag()
        m.flash_attn_window_func(q, k, v, 100, causal=True)
        assert not _debug.last_zigzag()
        big = [t.to(device) for t in make(8, 32, 8, 1024, 1024, 128, torch.float16, 6)]  # 1024 blocks
        ref = m.flash_attn_func(*big, causal=True)
        assert not _debug.last_zigzag()
        _debug.set_zigzag(2)
        zz = m.flash_attn_func(*big, causal=True)
        assert _debug.last_zigzag()
        torch.cuda.synchronize()
        assert (zz.float() - ref.float()).abs().max().item() < 4e-3
        _debug.set_zigzag(0)
        m.flash_attn_func(q, k, v, causal=True)
        assert not _debug.last_zigzag()
    finally:
        _debug.set_zigzag()
        _debug.set_split()


SPLIT = [  # (B, Hq, Hkv, Sq, Sk, D): causal launches whose 256-row blocks fit one round of the grid
    (1, 4, 2, 1024, 1024, 128),
    (2, 2, 1, 640, 640, 64),
    (1, 8, 8, 2048, 2048, 128),
    (1, 4, 4, 700, 1500, 128),   # Sq < Sk: every row sees both key halves
    (1, 4, 4, 1500, 700, 64),    # Sq > Sk: the first rows see no key at all (output 0)
    (3, 2, 2, 200, 200, 128),    # one q-tile per head, a single key tile: piece 0 empty
]


@pytest.mark.parametrize("shape", SPLIT, ids=[str(s) for s in SPLIT])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_key_split_causal_blocks(device, shape, dtype):
    """Key-split causal blocks (fa_fwd_w4 "Key-split causal blocks": each block's key tiles in two
    pieces on two workgroups, the second combining), knob 2 (always; the default rule picks long
    one-round grids);
    against the oracle, two launches bit-identical (the combine does not depend on which piece
    arrives second), any persistent grid size bit-identical, and close to the unsplit layout."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d = shape
    seed = zlib.crc32(repr((shape, str(dtype), "split")).encode())
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, seed)
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    _debug.set_knobs()
    _debug.set_split(2)
    m.split_errors(reset=True)
    try:
        out = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_path() == "w4" and _debug.last_layout() == "split"
        again = m.flash_attn_func(qd, kd, vd, causal=True)
        with _debug.knobs(w4_grid=8):  # many rounds per workgroup: pieces meet in every order
            small = m.flash_attn_func(qd, kd, vd, causal=True)
            assert _debug.last_layout() == "split"
        _debug.set_split(0)
        _debug.set_zigzag(0)
        plain = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_layout() == "plain"
        torch.cuda.synchronize()
    finally:
        _debug.set_split()
        _debug.set_zigzag()
    # (the counters of the persistent per-stream area were left zeroed by every launch: a stale one
    # would have sent the next launch's pieces to the wrong records)
    assert m.split_errors() == 0
    assert torch.equal(out, again) and torch.equal(out, small)
    check(out, q, k, v, d ** -0.5, True, dtype)
    tol = 4e-3 if dtype == torch.float16 else 3e-2
    assert (out.float() - plain.float()).abs().max().item() < tol


PAIRS = [  # (B, Hq, Hkv, Sq, Sk, D): one-round causal grids with more plain blocks than half the CUs
    (1, 16, 4, 4096, 4096, 128),  # C4's 8-way share: 16 q-tiles per head, pairs (15, 0) .. (8, 7)
    (1, 24, 24, 1536, 1536, 64),  # 6 q-tiles: short pairs, the split point clamps to 0 (no hand-off)
    (1, 16, 8, 2304, 2304, 128),  # 9 q-tiles: the middle one halves over its two workgroups
    (1, 32, 8, 1280, 2000, 128),  # Sq < Sk, 5 q-tiles
    (2, 12, 4, 1500, 700, 64),    # Sq > Sk: the first rows see no key (output 0)
]


@pytest.mark.parametrize("shape", PAIRS, ids=[str(s) for s in PAIRS])
def test_key_split_pairs(device, shape):
    """Key-split pairs (fa_fwd_w4 "key-split blocks", fa_launch.h use_split_pairs): the heavy q-tile
    Q - 1 - p split between two workgroups, one of which also runs the light q-tile p. Against the
    oracle, two launches bit-identical, close to the plain layout and to the halves layout
    (different split points: summation order only), no hand-off error; a capped grid (no room for a
    pass) falls back to the halves."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d = shape
    dtype = torch.float16
    seed = zlib.crc32(repr((shape, "pairs")).encode())
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, seed)
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    _debug.set_knobs()
    _debug.set_split(2)
    m.split_errors(reset=True)
    try:
        out = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_layout() == "split" and _debug.last_split_pairs()
        again = m.flash_attn_func(qd, kd, vd, causal=True)
        _debug.set_split_pairs(0)
        halves = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_layout() == "split" and not _debug.last_split_pairs()
        _debug.set_split_pairs()
        with _debug.knobs(w4_grid=64):
            capped = m.flash_attn_func(qd, kd, vd, causal=True)
            assert _debug.last_layout() == "split" and not _debug.last_split_pairs()
        _debug.set_split(0)
        _debug.set_zigzag(0)
        plain = m.flash_attn_func(qd, kd, vd, causal=True)
        torch.cuda.synchronize()
    finally:
        _debug.set_split()
        _debug.set_split_pairs()
        _debug.set_zigzag()
    assert m.split_errors() == 0
    assert torch.equal(out, again) and torch.equal(halves, capped)
    check(out, q, k, v, d ** -0.5, True, dtype)
    for other in (plain, halves):
        assert (out.float() - other.float()).abs().max().item() < 4e-3


def test_key_split_pairs_by_default_on_the_c4_share(device):
    """The default rule sends C4's 8-way share (B1 Hq16 Hkv4 S4096 causal) to key-split pairs over
    head-packed blocks; a half-round grid (B1 Hq8 Hkv2 S4096: the halves layout) keeps plain blocks
    (head-packed halves measured slower, profiles/r6_split_rule_sweep.log); key-split from 1024 keys on
    a half-round grid and from 2048 on a fuller one; below, zigzag at half fill or less and head-packed
    blocks above."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    def run(b, hq, hkv, s):
        q, k, v = (torch.randn(b, h, s, 128, device=device, dtype=torch.float16) for h in (hq, hkv, hkv))
        m.flash_attn_func(q, k, v, causal=True)
        return _debug.last_layout(), _debug.last_split_pairs(), _debug.last_head_pack()

    _debug.set_knobs()
    _debug.set_split()
    _debug.set_split_pairs()
    _debug.set_head_pack()
    assert run(1, 16, 4, 4096) == ("split", True, True)
    assert run(1, 8, 2, 4096) == ("split", False, False)
    assert run(1, 32, 8, 2048) == ("split", True, True)  # 256 blocks, 2048 keys
    assert run(1, 32, 32, 2048) == ("split", True, False)  # MHA: plain-block pairs
    assert run(1, 16, 4, 1024) == ("split", False, False)  # 64 blocks: the halves from 1024 keys
    assert run(2, 32, 8, 1024)[0] == "headpack"  # 256 blocks of 1024 keys: no key-split, a full round
    assert run(1, 16, 4, 768)[0] == "zigzag"


HP_SPLIT = [  # (B, Hq, Hkv, Sq, Sk, D): one-round causal GQA grids, g % 4 == 0
    (1, 16, 4, 4096, 4096, 128),  # C4's 8-way share: pairs over 64 q-tiles of 4 quads
    (1, 8, 2, 1024, 1024, 128),   # halves (16 q-tiles x 2 quads x 2 pieces)
    (1, 32, 8, 1280, 2000, 128),  # Sq < Sk
    (2, 8, 1, 1500, 700, 64),     # Sq > Sk: the first rows see no key (output 0); g = 8, D = 64
    (1, 4, 1, 300, 300, 128),     # ragged: a 44-row last q-tile
]


@pytest.mark.parametrize("shape", HP_SPLIT, ids=[str(s) for s in HP_SPLIT])
@pytest.mark.parametrize("pairs", [1, 0], ids=["pairs", "halves"])
def test_head_packed_key_split(device, shape, pairs):
    """Key-split pieces over head-packed blocks (fa_launch.h use_head_pack_split: the halves or pairs
    layout over (batch, q-head quad, 64-row q-tile) units, one hand-off per (block, wave); knob 2, as
    the default rule takes them under the pairs layout only): against the
    oracle, two launches and a capped persistent grid bit-identical, no hand-off error, close to the
    plain-block key-split layout (different split points: summation order only)."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d = shape
    dtype = torch.bfloat16 if pairs else torch.float16
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, zlib.crc32(repr((shape, pairs, "hpsplit")).encode()))
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    _debug.set_knobs()
    _debug.set_split(2)
    _debug.set_split_pairs(pairs)
    _debug.set_head_pack(2)  # (the default rule head-packs the pairs layout only)
    m.split_errors(reset=True)
    try:
        out = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_layout() == "split" and _debug.last_head_pack()
        layout_pairs = _debug.last_split_pairs()
        again = m.flash_attn_func(qd, kd, vd, causal=True)
        with _debug.knobs(w4_grid=16):  # many rounds per workgroup: the halves, pieces in every order
            small = m.flash_attn_func(qd, kd, vd, causal=True)
            assert _debug.last_head_pack() and not _debug.last_split_pairs()
        _debug.set_head_pack(0)
        plain = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_layout() == "split" and not _debug.last_head_pack()
        torch.cuda.synchronize()
    finally:
        _debug.set_split()
        _debug.set_split_pairs()
        _debug.set_head_pack()
    assert m.split_errors() == 0
    assert torch.equal(out, again)
    if not layout_pairs:
        assert torch.equal(out, small)
    check(out, q, k, v, d ** -0.5, True, dtype)
    check(small, q, k, v, d ** -0.5, True, dtype)
    tol = 4e-3 if dtype == torch.float16 else 3e-2
    assert (out.float() - plain.float()).abs().max().item() < tol


@pytest.mark.parametrize("hp", [0, 2], ids=["plain", "headpack"])
def test_key_split_halves_order_is_bit_identical(device, hp):
    """The halves' work order (knob split_rr: level-major, the default, or decode_work's XCD-contiguous
    ranges) moves pieces between workgroups only: the split points and the order-independent combine
    are the same, so the outputs are bit-identical; no hand-off error either way."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    q, k, v = (t.to(device) for t in make(1, 8, 2, 2048, 2048, 128, torch.bfloat16, 41))
    _debug.set_knobs()
    _debug.set_split(2)
    _debug.set_split_pairs(0)
    _debug.set_head_pack(hp)
    m.split_errors(reset=True)
    try:
        outs = []
        for rr in (1, 0):
            _debug.set_split_rr(rr)
            outs.append(m.flash_attn_func(q, k, v, causal=True))
            assert _debug.last_layout() == "split" and not _debug.last_split_pairs()
            assert _debug.last_head_pack() == (hp == 2)
        torch.cuda.synchronize()
    finally:
        _debug.set_split_rr()
        _debug.set_split()
        _debug.set_split_pairs()
        _debug.set_head_pack()
    assert torch.equal(outs[0], outs[1])
    assert m.split_errors() == 0
    check(outs[0], q.cpu(), k.cpu(), v.cpu(), 128 ** -0.5, True, torch.bfloat16)


def test_key_split_only_with_a_workspace(device):
    """The C-ABI runs key-split blocks only when the caller passes the workspace
    fa_fwd_gfx950_workspace_size asks for (the torch op does); without one (plain fa_fwd_gfx950) the
    same launch runs zigzag blocks; non-causal launches ask for none, nor (default knob) large causal
    grids or short keys."""
    import ctypes

    from flash_attention_cute_amd import _debug

    lib = _debug.lib()
    lib.fa_fwd_gfx950_workspace_size.restype = ctypes.c_int64
    _debug.set_split(2)
    try:
        q, k, v = (t.to(device) for t in make(1, 4, 2, 1024, 1024, 128, torch.float16, 9))
        o = torch.empty_like(q)
        p = _debug.FaFwdParams(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), 1, 4, 2, 1024, 1024, 128, 2,
                               *(t.stride(i) for i in range(3) for t in (q, k, v, o)), 128 ** -0.5 * _debug.LOG2E)
        need = lib.fa_fwd_gfx950_workspace_size(ctypes.byref(p), 0, 1)
        assert need > 0 and lib.fa_fwd_gfx950_workspace_size(ctypes.byref(p), 0, 0) == 0
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert lib.fa_fwd_gfx950(ctypes.byref(p), 0, 1, stream) == 0
        assert _debug.last_layout() == "zigzag"
        ws = torch.empty(need, dtype=torch.uint8, device=device)
        o2 = torch.empty_like(q)
        p.o_ptr = o2.data_ptr()
        lib.fa_fwd_gfx950_ws.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_void_p]
        o3 = torch.empty_like(q)
        p.o_ptr = o3.data_ptr()
        # (ABI 7: a workspace too small for the partials runs the unsplit zigzag layout, no error)
        assert lib.fa_fwd_gfx950_ws(ctypes.byref(p), 0, 1, ws.data_ptr(), need - 256, stream) == 0
        assert _debug.last_layout() == "zigzag"
        p.o_ptr = o2.data_ptr()
        assert lib.fa_fwd_gfx950_ws(ctypes.byref(p), 0, 1, ws.data_ptr(), need, stream) == 0
        assert _debug.last_layout() == "split"
        torch.cuda.synchronize()
        assert torch.equal(o, o3)
        assert (o.float() - o2.float()).abs().max().item() < 4e-3
        # default knob: 8 x 32 heads x 4 q-tiles = 1024 blocks, four rounds, and a one-round 768-key
        # launch ask for none; this one-round 1024-key launch (16 blocks) and 8 heads x 16 q-tiles of
        # 4096 keys (128 blocks) do (contiguous strides)
        _debug.set_split()
        assert lib.fa_fwd_gfx950_workspace_size(ctypes.byref(p), 0, 1) > 0

        def params(b, hq, hkv, s):
            hs = {"q": hq, "k": hkv, "v": hkv, "o": hq}
            strides = [hs[t] * s * 128 for t in "qkvo"] + [s * 128] * 4 + [128] * 4
            return _debug.FaFwdParams(0x10000, 0x10000, 0x10000, 0x10000, b, hq, hkv, s, s, 128, 4, *strides, 0.1)

        assert lib.fa_fwd_gfx950_workspace_size(ctypes.byref(params(8, 32, 8, 1024)), 0, 1) == 0
        assert lib.fa_fwd_gfx950_workspace_size(ctypes.byref(params(1, 8, 2, 768)), 0, 1) == 0
        assert lib.fa_fwd_gfx950_workspace_size(ctypes.byref(params(1, 8, 2, 4096)), 0, 1) > 0
    finally:
        _debug.set_split()


def test_key_split_under_graph_capture(device):
    """A key-split launch captured into a HIP graph: the capturing stream has no counter area yet, so its
    counters go to the workspace, zeroed by a memset node of the graph; replays equal the eager launch
    bit for bit, and no hand-off times out."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    q, k, v = (t.to(device) for t in make(1, 4, 2, 1024, 1024, 128, torch.bfloat16, 21))
    _debug.set_split(2)
    m.split_errors(reset=True)
    try:
        eager = m.flash_attn_func(q, k, v, causal=True)
        assert _debug.last_layout() == "split"
        g = torch.cuda.CUDAGraph()  # (captures on a stream of its own)
        with torch.cuda.graph(g):
            out = m.flash_attn_func(q, k, v, causal=True)
        outs = []
        for _ in range(3):
            g.replay()
            outs.append(out.clone())
        torch.cuda.synchronize()
    finally:
        _debug.set_split()
    assert all(torch.equal(o, eager) for o in outs)
    assert m.split_errors() == 0


@pytest.mark.parametrize("layout", ["halves", "pairs", "halves_hp", "pairs_hp"])
def test_key_split_timeout_leaves_the_next_launch_correct(device, layout):
    """A hand-off that times out (debug library: wave 0 of the last q-tile of (batch 0, q-head 0) holds
    its ready mark until its partner has abandoned the pair) is counted exactly once, and the NEXT
    launches on the same stream are correct against the oracle with no further error: the abandoned
    pair's arrivals word was left 0, so no launch inherits a stale ready mark (fa_fwd_w4 key-split
    hand-off). Both layouts, over plain and head-packed blocks (_hp: 64-row q-tiles of q-head quads).
    Reference behaviour kept by the good launches: plain blocks, template.cuh:516-563."""
    from flash_attention_cute_amd import _debug

    pairs, hp = layout.startswith("pairs"), layout.endswith("_hp")
    shape = (1, 16, 4, 4096, 4096, 128) if pairs else (1, 8, 2, 1024, 1024, 128)
    b, hq, hkv, sq, sk, d = shape
    dtype = torch.float16
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, zlib.crc32(repr((shape, "fault")).encode()))
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    dl = _debug.lib(debug=True)
    _debug.set_split(2, debug=True)
    _debug.set_split_pairs(1 if pairs else 0, debug=True)
    _debug.set_head_pack(2 if hp else 0, debug=True)
    dl.fa_split_errors(1)
    try:
        _debug.set_split_fault(True)
        bad = _debug.forward(qd, kd, vd, causal=True, variant="w4", workspace=True)
        assert _debug.last_path(debug=True) == "w4" and _debug.last_layout(debug=True) == "split"
        assert _debug.last_split_pairs(debug=True) == pairs and _debug.last_head_pack(debug=True) == hp
        torch.cuda.synchronize()
        assert dl.fa_split_errors(0) == 1
        _debug.set_split_fault(False)
        good = _debug.forward(qd, kd, vd, causal=True, variant="w4", workspace=True)
        again = _debug.forward(qd, kd, vd, causal=True, variant="w4", workspace=True)
        torch.cuda.synchronize()
        assert dl.fa_split_errors(1) == 1  # (nothing new: the faulted pair left its word zeroed)
    finally:
        _debug.set_split_fault(False)
        _debug.set_split(debug=True)
        _debug.set_split_pairs(debug=True)
        _debug.set_head_pack(debug=True)
        _debug.set_knobs(debug=True)
    assert torch.equal(good, again)
    check(good, q, k, v, d ** -0.5, True, dtype)
    # the faulted launch can differ from the good one only in the abandoned block's rows (wave 0 of
    # q-tile nq - 1 of (batch 0, q-head 0): rows 0-31 and 128-159 of that 256-row block, or head-packed
    # all 64 rows of that 64-row q-tile; the partner's records are usually written by the time it gives
    # up, so they may well be right)
    rows = 64 if hp else 256
    nq = (sq + rows - 1) // rows
    for bb, hh, m in (bad.float() != good.float()).any(dim=-1).nonzero().tolist():
        assert (bb, hh) == (0, 0) and m // rows == nq - 1 and (hp or (m % 256) % 128 < 32), (bb, hh, m)


def test_split_layouts_need_same_xcd_placement(device):
    """With an XCD count that does not divide 8 (knob), the dispatcher takes the layouts without a
    hand-off: causal prefill runs zigzag and asks for no workspace, split-KV decode merges in the
    separate combine launch; both equal their placement-checked counterparts within the bar."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    q, k, v = (t.to(device) for t in make(1, 4, 2, 1024, 1024, 128, torch.float16, 31))
    qd, kd, vd = (t.to(device) for t in make(1, 8, 1, 1, 65536, 128, torch.bfloat16, 32))
    _debug.set_knobs()
    _debug.set_split(2)
    try:
        split = m.flash_attn_func(q, k, v, causal=True)
        assert _debug.last_layout() == "split"
        dec = m.flash_attn_func(qd, kd, vd)
        assert _debug.last_path() == "decode_split" and _debug.last_dec_fused()
        _debug.set_xccs(3)
        fallback = m.flash_attn_func(q, k, v, causal=True)
        assert _debug.last_layout() == "zigzag"
        dec_fb = m.flash_attn_func(qd, kd, vd)
        assert _debug.last_path() == "decode_split" and not _debug.last_dec_fused()
        _debug.set_xccs(4)  # (DPX-like: 4 XCDs, b and b + 8 still share one)
        m.flash_attn_func(q, k, v, causal=True)
        assert _debug.last_layout() == "split"
        torch.cuda.synchronize()
    finally:
        _debug.set_xccs()
        _debug.set_split()
    assert (split.float() - fallback.float()).abs().max().item() < 4e-3
    assert (dec.float() - dec_fb.float()).abs().max().item() < 3e-2


def test_first_key_split_call_beside_a_graph_capture(device):
    """A stream's first key-split / fused-decode call allocates its counter area (hipMalloc with the
    thread in relaxed capture mode) and zeroes it with a memset on that stream -- no device-wide
    synchronisation -- so it may run while another stream is capturing a graph in global mode (torch's
    default); the captured graph, which never holds a shared area, replays bit-identical to its eager
    launch. The side-stream calls go through the C-ABI with buffers allocated beforehand (torch's own
    caching allocator is not what is tested here)."""
    import ctypes

    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    lib = _debug.lib()
    q, k, v = (t.to(device) for t in make(1, 4, 2, 1024, 1024, 128, torch.float16, 41))
    qd, kd, vd = (t.to(device) for t in make(1, 8, 1, 1, 65536, 128, torch.float16, 42))
    _debug.set_split(2)
    m.split_errors(reset=True)

    def abi_call(qx, kx, vx, causal, stream):
        """fa_fwd_gfx950_ws on `stream` with preallocated output and workspace (the op's host steps:
        Sq == 1 q-head pack for decode)."""
        b, hq, sq, d = qx.shape
        hkv = kx.size(1)
        pack = sq == 1
        qp = qx.reshape(b, hkv, hq // hkv, d) if pack else qx
        o = torch.empty_like(qp)
        p = _debug.FaFwdParams(qp.data_ptr(), kx.data_ptr(), vx.data_ptr(), o.data_ptr(), b, qp.size(1), hkv,
                               qp.size(2), kx.size(2), d, 1 if pack else hq // hkv,
                               *(t.stride(i) for i in range(3) for t in (qp, kx, vx, o)), d ** -0.5 * _debug.LOG2E)
        need = lib.fa_fwd_gfx950_workspace_size(ctypes.byref(p), 0, int(causal))
        ws = torch.empty(max(need, 16), dtype=torch.uint8, device=device)
        run = lambda: lib.fa_fwd_gfx950_ws(ctypes.byref(p), 0, int(causal), ws.data_ptr(), need,  # noqa: E731
                                           ctypes.c_void_p(stream.cuda_stream))
        return run, o.reshape(qx.shape)

    try:
        eager = m.flash_attn_func(q, k, v, causal=True)
        eager_dec = m.flash_attn_func(qd, kd, vd)
        side = torch.cuda.Stream()  # (new: no counter area yet)
        run_pf, side_out = abi_call(q, k, v, True, side)
        run_dec, side_dec = abi_call(qd, kd, vd, False, side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = m.flash_attn_func(q, k, v, causal=True)
            out_dec = m.flash_attn_func(qd, kd, vd)
            assert not _debug.last_dec_fused()  # (under capture: the combine launch)
            # an eager first call on another stream mid-capture: allocates that stream's area
            assert run_pf() == 0 and _debug.last_layout() == "split"
            assert run_dec() == 0 and _debug.last_dec_fused()
        side.synchronize()
        outs = []
        for _ in range(3):
            g.replay()
            outs.append((out.clone(), out_dec.clone()))
        torch.cuda.synchronize()
    finally:
        _debug.set_split()
    assert torch.equal(side_out, eager) and torch.equal(side_dec, eager_dec)
    assert all(torch.equal(o, eager) and torch.equal(od, eager_dec) for o, od in outs)
    assert m.split_errors() == 0


HEADPACK = [  # (B, Hq, Hkv, Sq, Sk, D): causal GQA with a multiple of 4 q-heads per kv-head
    (1, 8, 2, 1024, 1024, 128),
    (2, 4, 1, 300, 300, 128),     # ragged: a 44-row last q-tile
    (1, 4, 1, 700, 1500, 128),    # Sq < Sk
    (1, 8, 2, 1500, 700, 64),     # Sq > Sk: the first rows see no key (output 0)
    (1, 4, 1, 130, 130, 64),      # three 64-row q-tiles, one key tile
    (1, 16, 2, 600, 600, 128),    # g = 8: two q-head quads per kv group
]


@pytest.mark.parametrize("shape", HEADPACK, ids=[str(s) for s in HEADPACK])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_head_packed_blocks(device, shape, dtype):
    """Head-packed causal blocks (fa_fwd_w4 "Head-packed blocks": a block is (batch, kv-head, 64 rows),
    wave w on q-head 4 kv-head + w), forced with knob 2: against the oracle, and BIT-identical to the
    plain 256-row layout -- every row keeps its 32-row group and its tile order."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    b, hq, hkv, sq, sk, d = shape
    q, k, v = make(b, hq, hkv, sq, sk, d, dtype, zlib.crc32(repr((shape, str(dtype), "hp")).encode()))
    qd, kd, vd = q.to(device), k.to(device), v.to(device)
    _debug.set_knobs()
    _debug.set_split(0)  # (one-round shapes of 1024+ keys take key-split by default)
    try:
        _debug.set_head_pack(2)
        out = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_path() == "w4" and _debug.last_layout() == "headpack"
        with _debug.knobs(w4_grid=8):  # many rounds per workgroup
            small = m.flash_attn_func(qd, kd, vd, causal=True)
        _debug.set_head_pack(0)
        _debug.set_zigzag(0)
        _debug.set_split(0)
        plain = m.flash_attn_func(qd, kd, vd, causal=True)
        assert _debug.last_layout() == "plain"
        torch.cuda.synchronize()
    finally:
        _debug.set_head_pack()
        _debug.set_zigzag()
        _debug.set_split()
    assert torch.equal(out, plain) and torch.equal(out, small)
    check(out, q, k, v, d ** -0.5, True, dtype)


@pytest.mark.parametrize("entry", ["rope", "varlen", "padded", "window63", "window300", "window0", "varlen_window"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["f16", "bf16"])
def test_head_packed_blocks_on_rope_ranges_and_window(device, entry, dtype):
    """Head-packed blocks on the other causal entries that carry GQA prefill: the fused-RoPE launch
    (the patched Llama layer's call), packed varlen and padded batches in place (ragged and empty
    sequences, Sq < Sk), the local window (narrower than, one less than and wider than a 64-key tile)
    alone and per packed sequence. Knob 2 against knob 0: bit-identical; and against the oracle."""
    from flash_attention_cute_amd import (_debug, flash_attn_padded_func, flash_attn_rope_func, flash_attn_varlen_func,
                                          flash_attn_window_func)
    from tests.test_padded import check_padded, make_batch, oracle_padded, ranges
    from tests.test_rope import oracle_rope, tables
    from tests.test_varlen import check_varlen, pack

    seed = zlib.crc32(repr((entry, str(dtype), "hp")).encode())
    dv = lambda t: t.to(device)  # noqa: E731
    if entry == "rope":
        b, hq, hkv, s, d = 2, 8, 2, 700, 128
        q, k, v = make_batch(b, hq, hkv, s, s, d, dtype, seed, "bshd")  # HF projection views
        cos, sin = tables(b, s, d, dtype, seed)
        args = tuple(map(dv, (q, k, v, cos, sin)))
        run = lambda: flash_attn_rope_func(*args, causal=True)  # noqa: E731
        ref = lambda out: check(out, oracle_rope(q, cos, sin), k, v, d ** -0.5, True, dtype)  # noqa: E731
    elif entry == "varlen":
        case = (8, 2, 128, [(700, 700), (130, 130), (0, 0), (45, 300), (300, 300), (64, 64)])
        q, k, v, cu_q, cu_k, mq, mk = pack(case, dtype, seed)
        args = tuple(map(dv, (q, k, v, cu_q, cu_k)))
        run = lambda: flash_attn_varlen_func(*args, mq, mk, causal=True)  # noqa: E731
        ref = lambda out: check_varlen(out, q, k, v, cu_q, cu_k, 128 ** -0.5, True, dtype)  # noqa: E731
    elif entry.startswith("window"):
        wl = int(entry[6:])
        b, hq, hkv, sq, sk, d = 2, 8, 2, 1000, 1100, 128
        q, k, v = make(b, hq, hkv, sq, sk, d, dtype, seed)
        args = tuple(map(dv, (q, k, v)))
        run = lambda: flash_attn_window_func(*args, wl, causal=True)  # noqa: E731

        def ref(out):
            r = OC.forward(q, k, v, d ** -0.5, True, window_left=wl).float()
            err = (out.float().cpu() - r).abs()
            tol = TOL[dtype][0]
            assert bool((err <= tol + tol * r.abs()).all()), f"max err {err.max().item():.3e}"
    elif entry == "varlen_window":
        case = (8, 2, 128, [(700, 700), (130, 130), (0, 0), (45, 300), (300, 300), (64, 64)])
        q, k, v, cu_q, cu_k, mq, mk = pack(case, dtype, seed)
        args = tuple(map(dv, (q, k, v, cu_q, cu_k)))
        run = lambda: flash_attn_varlen_func(*args, mq, mk, causal=True, window_left=100)  # noqa: E731

        def ref(out):
            r = OC.forward_varlen(q, k, v, cu_q, cu_k, 128 ** -0.5, True, window_left=100).float()
            err = (out.float().cpu() - r).abs()
            tol = TOL[dtype][0]
            assert bool((err <= tol + tol * r.abs()).all()), f"max err {err.max().item():.3e}"
    else:
        b, hq, hkv, sq, sk, d = 4, 8, 2, 600, 700, 128
        q, k, v = make_batch(b, hq, hkv, sq, sk, d, dtype, seed, "bshd")
        rg = ranges(b, sq, sk, seed, "mixed")
        args = tuple(map(dv, (q, k, v) + rg))
        run = lambda: flash_attn_padded_func(*args, causal=True)  # noqa: E731
        ref = lambda out: check_padded(out, oracle_padded(q, k, v, *rg, d ** -0.5, True), dtype)  # noqa: E731
    _debug.set_knobs()
    try:
        _debug.set_head_pack(2)
        out = run()
        assert _debug.last_path() == "w4" and _debug.last_layout() == "headpack"
        with _debug.knobs(w4_grid=8):
            small = run()
        _debug.set_head_pack(0)
        plain = run()
        assert _debug.last_layout() != "headpack"
        torch.cuda.synchronize()
    finally:
        _debug.set_head_pack()
    assert torch.equal(out, plain) and torch.equal(out, small)
    ref(out)


def test_head_packed_blocks_by_default(device):
    """The default rule: multi-round causal grids with g = 4 take head-packed blocks (C4 / C5's class),
    and one-round grids more than half full that key-split leaves (short keys); g = 8 too (two q-head
    quads per kv group); g = 2, non-causal, half-full short grids (zigzag) and long one-round grids
    (key-split) do not."""
    import flash_attention_cute_amd as m
    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    _debug.set_head_pack()
    big = [torch.randn(2, h, 2048, 128, device=device, dtype=torch.float16) for h in (32, 8, 8)]  # 512 blocks
    m.flash_attn_func(*big, causal=True)
    assert _debug.last_layout() == "headpack"
    m.flash_attn_func(*big, causal=False)
    assert _debug.last_layout() == "plain"
    cs = torch.randn(2, 2048, 128, device=device, dtype=torch.float16)
    m.flash_attn_rope_func(*big, cs, cs, causal=True)  # the patched Llama layer's launch
    assert _debug.last_layout() == "headpack"
    m.flash_attn_window_func(*big, 1000, causal=True)  # the local window too
    assert _debug.last_layout() == "headpack"
    g2 = [torch.randn(2, h, 2048, 128, device=device, dtype=torch.float16) for h in (32, 16, 16)]
    m.flash_attn_func(*g2, causal=True)
    assert _debug.last_layout() != "headpack"
    g8 = [torch.randn(2, h, 2048, 128, device=device, dtype=torch.float16) for h in (32, 4, 4)]
    m.flash_attn_func(*g8, causal=True)
    assert _debug.last_layout() == "headpack"
    one = [torch.randn(1, h, 1024, 128, device=device, dtype=torch.float16) for h in (8, 2, 2)]  # 32 blocks
    m.flash_attn_func(*one, causal=True)
    assert _debug.last_layout() == "split"  # (1024 keys at half fill: key-split)
    short = [torch.randn(2, h, 512, 128, device=device, dtype=torch.float16) for h in (32, 8, 8)]  # 128 blocks
    m.flash_attn_func(*short, causal=True)
    assert _debug.last_layout() == "zigzag"  # (half fill, short keys)
    full = [torch.randn(4, h, 512, 128, device=device, dtype=torch.float16) for h in (32, 8, 8)]  # 256 blocks
    m.flash_attn_func(*full, causal=True)
    assert _debug.last_layout() == "headpack"  # (a full round of short keys)
