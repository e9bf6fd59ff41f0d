"""The C-ABI boundary (include/fa_gfx950.h): the library loads, exports every declared symbol, and
validates parameters with the documented error codes -- host-only calls, no GPU needed."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "fa_gfx950.h"
LIB = ROOT / "flash_attention_cute_amd" / "lib" / "libfa_gfx950.so"

FA_OK, FA_ERR_INVALID_ARGUMENT, FA_ERR_UNSUPPORTED, FA_ERR_LAUNCH = 0, 1, 2, 3


class FaFwdParams(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_void_p) for n in ("q_ptr", "k_ptr", "v_ptr", "o_ptr")]
                + [(n, ctypes.c_int64) for n in ("batch_size", "num_heads_q", "num_heads_kv", "seqlen_q", "seqlen_kv",
                                                 "headdim", "head_q_per_group")]
                + [(f"{t}_{s}_stride", ctypes.c_int64) for s in ("batch", "head", "seqlen") for t in "qkvo"]
                + [("softmax_scale", ctypes.c_float)])


def declared_functions() -> list[str]:
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return re.findall(r"\b(fa_\w+)\s*\(", text)


@pytest.fixture(scope="module")
def lib():
    if not LIB.exists():
        pytest.skip("libfa_gfx950.so not built (run __graft_entry__.build())")
    import torch  # noqa: F401  -- same process layout as the product (torch's HIP runtime first)

    return ctypes.CDLL(str(LIB))


def test_header_declares_the_boundary():
    assert set(declared_functions()) == {"fa_fwd_gfx950", "fa_fwd_gfx950_check", "fa_last_error", "fa_abi_version",
                                         "fa_fwd_gfx950_geometry", "fa_fwd_gfx950_ws",
                                         "fa_fwd_gfx950_workspace_size", "fa_fwd_gfx950_varlen",
                                         "fa_fwd_gfx950_varlen_check", "fa_fwd_gfx950_rope", "fa_rope_gfx950",
                                         "fa_fwd_gfx950_window", "fa_fwd_gfx950_varlen_window", "fa_fwd_gfx950_padded",
                                         "fa_fwd_gfx950_padded_workspace_size", "fa_split_errors"}


def test_every_declared_symbol_is_exported(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (fa_\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_struct_layout_matches_header():
    # 4 pointers + 7 sizes + 12 strides (int64) + float, padded to 8
    assert ctypes.sizeof(FaFwdParams) == 4 * 8 + 7 * 8 + 12 * 8 + 8
    assert FaFwdParams.softmax_scale.offset == 4 * 8 + 19 * 8


def good_params(**kw) -> FaFwdParams:
    b, hq, hkv, s, d = 2, 8, 2, 300, 128
    p = FaFwdParams(q_ptr=0x10000, k_ptr=0x20000, v_ptr=0x30000, o_ptr=0x40000, batch_size=b, num_heads_q=hq,
                    num_heads_kv=hkv, seqlen_q=s, seqlen_kv=s, headdim=d, head_q_per_group=hq // hkv,
                    softmax_scale=0.1275)
    for t, h in (("q", hq), ("k", hkv), ("v", hkv), ("o", hq)):
        setattr(p, f"{t}_batch_stride", h * s * d)
        setattr(p, f"{t}_head_stride", s * d)
        setattr(p, f"{t}_seqlen_stride", d)
    for key, val in kw.items():
        setattr(p, key, val)
    return p


def check(lib, p, dtype=0, causal=0):
    lib.fa_fwd_gfx950_check.restype = ctypes.c_int
    rc = lib.fa_fwd_gfx950_check(ctypes.byref(p), dtype, causal)
    lib.fa_last_error.restype = ctypes.c_char_p
    return rc, lib.fa_last_error().decode()


def test_abi_version(lib):
    lib.fa_abi_version.restype = ctypes.c_int
    assert lib.fa_abi_version() == 8


def test_check_accepts_valid(lib):
    assert check(lib, good_params()) == (FA_OK, "")
    assert check(lib, good_params(), dtype=1, causal=1)[0] == FA_OK


@pytest.mark.parametrize("kw,code,msg", [
    ({"headdim": 100}, FA_ERR_INVALID_ARGUMENT, "multiple of 8"),
    ({"headdim": 136}, FA_ERR_UNSUPPORTED, "<= 128"),
    ({"head_q_per_group": 3}, FA_ERR_INVALID_ARGUMENT, "head_q_per_group"),
    ({"seqlen_kv": 0}, FA_ERR_INVALID_ARGUMENT, "at least one element"),
    ({"q_ptr": 0x10008}, FA_ERR_INVALID_ARGUMENT, "16-byte aligned"),
    ({"k_seqlen_stride": 132}, FA_ERR_INVALID_ARGUMENT, "multiples of 8"),
    ({"o_ptr": None}, FA_ERR_INVALID_ARGUMENT, "non-NULL"),
])
def test_check_rejects(lib, kw, code, msg):
    rc, err = check(lib, good_params(**kw))
    assert rc == code and msg in err


def test_check_rejects_dtype(lib):
    rc, err = check(lib, good_params(), dtype=7)
    assert rc == FA_ERR_UNSUPPORTED and "dtype" in err


def test_null_params(lib):
    lib.fa_fwd_gfx950_check.restype = ctypes.c_int
    assert lib.fa_fwd_gfx950_check(None, 0, 0) == FA_ERR_INVALID_ARGUMENT


def test_launch_entry_validates_before_touching_the_device(lib):
    lib.fa_fwd_gfx950.restype = ctypes.c_int
    p = good_params(headdim=100)
    assert lib.fa_fwd_gfx950(ctypes.byref(p), 0, 0, None) == FA_ERR_INVALID_ARGUMENT


def test_window_entry_validates_before_touching_the_device(lib):
    lib.fa_fwd_gfx950_window.restype = ctypes.c_int
    lib.fa_fwd_gfx950_window.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p]
    p = good_params(headdim=100)
    assert lib.fa_fwd_gfx950_window(ctypes.byref(p), 0, 1, 63, None) == FA_ERR_INVALID_ARGUMENT
    assert lib.fa_fwd_gfx950_window(None, 0, 1, 63, None) == FA_ERR_INVALID_ARGUMENT


def test_geometry(lib):
    lib.fa_fwd_gfx950_geometry.restype = ctypes.c_int
    vals = [ctypes.c_int64() for _ in range(4)]
    rc = lib.fa_fwd_gfx950_geometry(ctypes.byref(good_params()), 0, *[ctypes.byref(x) for x in vals])
    assert rc == FA_OK
    bm, bn, thr, wg = (x.value for x in vals)
    assert (bm, bn, thr) == (256, 64, 256)  # fa_fwd_w4: 4 waves
    assert wg == 2 * 8 * ((300 + bm - 1) // bm)


def decode_params(b=32, hq=32, hkv=8, sk=4096, d=128, sq=1, pack=True) -> FaFwdParams:
    """Parameters as the torch host API passes them for a decode step: Sq == 1 q-heads packed into
    the rows of one (batch, kv-head) problem (reference csrc/flash_attention_api.cpp:72-83)."""
    g = hq // hkv
    if pack:
        hq, sq, g = hkv, g * sq, 1
    p = good_params(batch_size=b, num_heads_q=hq, num_heads_kv=hkv, seqlen_q=sq, seqlen_kv=sk, headdim=d,
                    head_q_per_group=g)
    for t, h, s in (("q", hq, sq), ("k", hkv, sk), ("v", hkv, sk), ("o", hq, sq)):
        setattr(p, f"{t}_batch_stride", h * s * d)
        setattr(p, f"{t}_head_stride", s * d)
        setattr(p, f"{t}_seqlen_stride", d)
    return p


def geometry(lib, p):
    lib.fa_fwd_gfx950_geometry.restype = ctypes.c_int
    vals = [ctypes.c_int64() for _ in range(4)]
    assert lib.fa_fwd_gfx950_geometry(ctypes.byref(p), 0, *[ctypes.byref(x) for x in vals]) == FA_OK
    return tuple(x.value for x in vals)


def ws_size(lib, p, dtype=0, causal=0):
    lib.fa_fwd_gfx950_workspace_size.restype = ctypes.c_int64
    return lib.fa_fwd_gfx950_workspace_size(ctypes.byref(p), dtype, causal)


def test_decode_geometry_and_workspace(lib):
    # B32 x Hkv8 = 256 row blocks already fill the chip: one workgroup each, no split, no workspace
    p = decode_params()
    assert geometry(lib, p) == (32, 32, 256, 256)
    assert ws_size(lib, p) == 0
    # batch 1: 8 row blocks, split over the keys -> fp32 partials (32 rows x 128) + lse per split
    p1 = decode_params(b=1, sk=32768)
    n = ws_size(lib, p1)
    assert n > 0 and n % (8 * 32 * (128 * 4 + 4)) == 0
    splits = n // (8 * 32 * (128 * 4 + 4))
    assert 2 <= splits <= 64
    # short K/V: no split (every wave keeps >= 4 tiles of 32 keys)
    assert ws_size(lib, decode_params(b=1, sk=256)) == 0
    # prefill shapes need no workspace; invalid parameters report -1
    assert ws_size(lib, good_params()) == 0
    assert ws_size(lib, good_params(headdim=100)) == -1


def test_decode_rows_threshold(lib):
    # unpacked GQA with a few query positions also runs the decode kernel while g * Sq <= 64 rows
    assert geometry(lib, decode_params(sq=8, pack=False))[0] == 32   # 4 heads x 8 positions
    assert geometry(lib, decode_params(sq=17, pack=False))[0] == 256  # 68 rows -> prefill kernel


def test_ws_entry_rejects_small_workspace(lib):
    lib.fa_fwd_gfx950_ws.restype = ctypes.c_int
    p = decode_params(b=1, sk=32768)
    need = ws_size(lib, p)
    rc = lib.fa_fwd_gfx950_ws(ctypes.byref(p), 0, 0, ctypes.c_void_p(0x100000), ctypes.c_int64(need - 16), None)
    assert rc == FA_ERR_INVALID_ARGUMENT
    lib.fa_last_error.restype = ctypes.c_char_p
    assert b"workspace" in lib.fa_last_error()
    rc = lib.fa_fwd_gfx950_ws(ctypes.byref(p), 0, 0, ctypes.c_void_p(0x100008), ctypes.c_int64(need), None)
    assert rc == FA_ERR_INVALID_ARGUMENT  # misaligned


def test_knobs_are_set_through_the_debug_hook_not_per_launch_env(lib, monkeypatch):
    """The dispatcher reads its tuning knobs once per process; a variable set later changes
    nothing, only fa_debug_set_knobs does (flash_attention_cute_amd/_debug.py)."""
    from flash_attention_cute_amd import _debug

    _debug.set_knobs()
    dlib = _debug.lib(debug=True)  # the debug / A-B library (-DFA_DEBUG_VARIANTS), its knobs read now
    dlib.fa_fwd_gfx950_geometry.restype = ctypes.c_int
    assert geometry(dlib, good_params())[2] == 256
    monkeypatch.setenv("FA_GFX950_VARIANT", "w8")
    monkeypatch.setenv("FA_GFX950_DECODE", "0")
    assert geometry(lib, good_params())[2] == 256          # still fa_fwd_w4 (4 waves)
    assert geometry(lib, decode_params())[0] == 32         # still the decode kernel
    with pytest.raises(ValueError):  # the product library compiles fa_fwd_w4 only
        _debug.set_knobs(variant="w8")
    with _debug.knobs(variant="w8", debug=True):
        assert geometry(dlib, good_params())[2] == 512      # fa_fwd_w8: 8 waves
        assert geometry(dlib, decode_params())[0] == 256    # variants other than w4 never use decode
    assert geometry(dlib, good_params())[2] == 256
    with _debug.knobs(decode=False):
        assert geometry(lib, decode_params())[0] == 256
    assert geometry(lib, good_params())[2] == 256 and geometry(lib, decode_params())[0] == 32
    assert _debug.last_path() == "none"  # host-only calls launch nothing


def test_asm_check_detects_pinned_agpr_use_and_spills():
    from flash_attention_cute_amd import _asm_check as A

    ok = ("_ZN2fa9fa_fwd_w4IXEEv:\n\t;;#ASMSTART\n\tv_mfma_f32_32x32x16_f16 a[0:15], v[0:3], v[4:7], a[0:15]\n"
          "\t;;#ASMEND\n\tv_accvgpr_write_b32 a200, v1\n\ts_endpgm\n")
    assert A.agpr_violations(ok) == []
    bad = ok.replace("a200", "a17")
    assert len(A.agpr_violations(bad)) == 1
    other = bad.replace("fa_fwd_w4", "fa_decode")  # only fa_fwd_w4 pins AGPRs
    assert A.agpr_violations(other) == []
    # the head-dim tile sets the O range: a64..a127 are free at D = 64, pinned at D = 128
    d64 = ok.replace("IXEE", "INS_3F16ELb0ELi64ELb1EE").replace("a200", "a70")
    assert A.agpr_violations(d64) == []
    assert len(A.agpr_violations(d64.replace("Li64E", "Li128E"))) == 1
    assert len(A.agpr_violations(d64.replace("a70", "a130"))) == 1  # Q: pinned at every D
    meta = "amdhsa.kernels:\n  - .agpr_count: 0\n    .name: k1\n    .vgpr_spill_count: 0\n" \
           "  - .agpr_count: 0\n    .name: k2\n    .vgpr_spill_count: 3\n"
    assert A.spills(meta) == ["k2: vgpr_spill_count 3"]


def test_build_asm_gate_passes_on_the_built_instantiations():
    from flash_attention_cute_amd import _asm_check as A
    from flash_attention_cute_amd import _build

    files = sorted((_build.ROOT / "build" / "obj").glob("*/fa_inst-hip-amdgcn-amd-amdhsa-gfx950.s"))
    if not files:
        pytest.skip("no -save-temps assembly (library built elsewhere)")
    assert len(files) == len(_build.INSTANCES)
    assert [p for f in files for p in A.check_file(f)] == []


class FaVarlenParams(ctypes.Structure):
    _fields_ = [("base", FaFwdParams), ("cu_seqlens_q", ctypes.c_void_p), ("cu_seqlens_k", ctypes.c_void_p)]


def test_varlen_struct_layout():
    assert ctypes.sizeof(FaVarlenParams) == ctypes.sizeof(FaFwdParams) + 16
    assert FaVarlenParams.cu_seqlens_q.offset == ctypes.sizeof(FaFwdParams)


def test_varlen_check(lib):
    lib.fa_fwd_gfx950_varlen_check.restype = ctypes.c_int
    lib.fa_last_error.restype = ctypes.c_char_p
    base = good_params(q_batch_stride=3, k_batch_stride=5)  # batch strides are ignored by varlen
    vp = FaVarlenParams(base, 0x50000, 0x60000)
    assert lib.fa_fwd_gfx950_varlen_check(ctypes.byref(vp), 0, 1) == FA_OK
    vp = FaVarlenParams(base, None, 0x60000)
    assert lib.fa_fwd_gfx950_varlen_check(ctypes.byref(vp), 0, 1) == FA_ERR_INVALID_ARGUMENT
    assert b"cu_seqlens" in lib.fa_last_error()
    vp = FaVarlenParams(base, 0x50002, 0x60000)
    assert lib.fa_fwd_gfx950_varlen_check(ctypes.byref(vp), 0, 1) == FA_ERR_INVALID_ARGUMENT
    vp = FaVarlenParams(good_params(headdim=136), 0x50000, 0x60000)
    assert lib.fa_fwd_gfx950_varlen_check(ctypes.byref(vp), 0, 1) == FA_ERR_UNSUPPORTED
    lib.fa_fwd_gfx950_varlen.restype = ctypes.c_int
    assert lib.fa_fwd_gfx950_varlen(ctypes.byref(vp), 0, 1, None) == FA_ERR_UNSUPPORTED  # validated, no launch


def test_q_o_stride_bound_covers_the_interleaved_wave_slab(lib):
    """fa_fwd_w4 addresses a wave's Q / O slab (block A + block B, 160 rows) with 32-bit offsets:
    the q / o seqlen strides are bounded so that 160 rows fit, K / V by their 64-row tile."""
    lim_qo = (0x7fffffff - 256) // (2 * 160) // 8 * 8   # largest multiple of 8 that fits
    lim_kv = (0x7fffffff - 256) // (2 * 64) // 8 * 8
    for t in "qo":
        assert check(lib, good_params(**{f"{t}_seqlen_stride": lim_qo}))[0] == FA_OK
        rc, err = check(lib, good_params(**{f"{t}_seqlen_stride": lim_qo + 8}))
        assert rc == FA_ERR_UNSUPPORTED and "32-bit" in err
    for t in "kv":
        assert check(lib, good_params(**{f"{t}_seqlen_stride": lim_qo + 8}))[0] == FA_OK
        assert check(lib, good_params(**{f"{t}_seqlen_stride": lim_kv + 8}))[0] == FA_ERR_UNSUPPORTED


class FaPaddedParams(ctypes.Structure):
    _fields_ = [("base", FaFwdParams)] + [(n, ctypes.c_void_p) for n in ("q_start", "q_end", "k_start", "k_end")]


def test_padded_struct_layout():
    assert ctypes.sizeof(FaPaddedParams) == ctypes.sizeof(FaFwdParams) + 32


def test_padded_entry_validates_before_touching_the_device(lib):
    lib.fa_fwd_gfx950_padded.restype = ctypes.c_int
    lib.fa_fwd_gfx950_padded.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                         ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    lib.fa_fwd_gfx950_padded_workspace_size.restype = ctypes.c_int64
    lib.fa_fwd_gfx950_padded_workspace_size.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64]
    lib.fa_last_error.restype = ctypes.c_char_p
    # decode shape with key positions: the split-KV plan of the dense call
    dec = FaPaddedParams(decode_params(b=1, sk=32768), None, None, 0x50000, 0x50100)
    assert lib.fa_fwd_gfx950_padded_workspace_size(ctypes.byref(dec), 0, 0, -1) == ws_size(lib, dec.base)
    # prefill shape: the [2, B] query and key row arrays (B = 2: 4 * 2 * 4 = 32 bytes)
    pre = FaPaddedParams(good_params(), None, None, 0x50000, 0x50100)
    assert lib.fa_fwd_gfx950_padded_workspace_size(ctypes.byref(pre), 0, 1, -1) == 32
    assert lib.fa_fwd_gfx950_padded_workspace_size(ctypes.byref(dec), 0, 1, 100) == 16  # window: prefill kernel
    # ... which refuses to launch without that workspace
    assert lib.fa_fwd_gfx950_padded(ctypes.byref(pre), 0, 1, -1, None, 0, None) == FA_ERR_INVALID_ARGUMENT
    assert b"workspace" in lib.fa_last_error()
    half = FaPaddedParams(good_params(), None, None, 0x50000, None)
    assert lib.fa_fwd_gfx950_padded(ctypes.byref(half), 0, 1, -1, None, 0, None) == FA_ERR_INVALID_ARGUMENT
    assert b"together" in lib.fa_last_error()
    odd = FaPaddedParams(good_params(), None, None, 0x50002, 0x50100)
    assert lib.fa_fwd_gfx950_padded(ctypes.byref(odd), 0, 1, -1, None, 0, None) == FA_ERR_INVALID_ARGUMENT
    # prefill needs batch strides that are multiples of the seqlen strides (rows are addressed)
    skew = FaPaddedParams(good_params(k_batch_stride=2 * 300 * 128 + 8), None, None, 0x50000, 0x50100)
    rc = lib.fa_fwd_gfx950_padded(ctypes.byref(skew), 0, 1, -1, ctypes.c_void_p(0x70000), 32, None)
    assert rc == FA_ERR_INVALID_ARGUMENT and b"multiple" in lib.fa_last_error()
    bad = FaPaddedParams(good_params(headdim=136), None, None, 0x50000, 0x50100)
    assert lib.fa_fwd_gfx950_padded(ctypes.byref(bad), 0, 1, -1, None, 0, None) == FA_ERR_UNSUPPORTED
    assert lib.fa_fwd_gfx950_padded_workspace_size(ctypes.byref(bad), 0, 1, -1) == -1
    assert lib.fa_fwd_gfx950_padded(None, 0, 1, -1, None, 0, None) == FA_ERR_INVALID_ARGUMENT


def test_debug_bodies_only_in_the_debug_library():
    """The product library compiles fa_fwd_w4 (+ decode) only; fa_fwd_w8 / fa_fwd_p8 and the
    non-pipelined w4slow body are in lib/libfa_gfx950_debug.so (-DFA_DEBUG_VARIANTS)."""
    from flash_attention_cute_amd import _build

    prod = LIB.read_bytes()
    assert b"fa_fwd_w4" in prod and b"fa_fwd_w8" not in prod and b"fa_fwd_p8" not in prod
    dbg = _build.DEBUG_LIB.read_bytes()
    assert b"fa_fwd_w4" in dbg and b"fa_fwd_w8" in dbg and b"fa_fwd_p8" in dbg


def test_host_validation_under_asan_ubsan(tmp_path):
    """The C-ABI's host-side validation and dispatch (csrc/fa_fwd_gfx950.hip) built with
    AddressSanitizer + UBSan on the host code only (-Xarch_host -fsanitize=...; device code is never
    sanitized) and linked with host-only stub instantiations (tests/asan/stub_instances.hip): every
    entry point with valid and invalid parameters returns the right code with no sanitizer report
    (tests/asan/abi_validation_driver.cpp)."""
    import os
    import shutil

    hipcc = "/opt/rocm/bin/hipcc"
    if not shutil.which(hipcc):
        pytest.skip("hipcc not available")
    root = Path(__file__).resolve().parent.parent
    inc = [f"-I{root / 'include'}", f"-I{root / 'flash_attention_cute_amd' / 'csrc'}"]
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined"]
    base = [hipcc, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", *san, *inc, "-c"]
    objs = []
    for src in (root / "flash_attention_cute_amd" / "csrc" / "fa_fwd_gfx950.hip",
                root / "tests" / "asan" / "stub_instances.hip", root / "tests" / "asan" / "abi_validation_driver.cpp"):
        obj = tmp_path / (src.stem + ".o")
        subprocess.run([*base, str(src), "-o", str(obj)], check=True, capture_output=True)
        objs.append(str(obj))
    exe = tmp_path / "abi_asan"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-fsanitize=address", "-fsanitize=undefined", "-fno-gpu-sanitize",
                    *objs, "-o", str(exe)], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    res = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0 and "abi validation ok" in res.stdout, res.stdout + res.stderr
    assert "runtime error" not in res.stderr and "AddressSanitizer" not in res.stderr, res.stderr


def test_mfma_hazard_rules_on_synthetic_streams():
    """_asm_check.hazards (the build gate around fa_fwd_w4's inline-asm MFMAs): each rule fires on a
    minimal stream and stays quiet once the wait states the gfx950 compiler itself inserts for the
    same pair are there (R1 1, R2 2, R3 passes + 4 = 12 for 32x32x16)."""
    from flash_attention_cute_amd import _asm_check as A

    k = "_ZN2fa9fa_fwd_w4ITEST:\n"

    def run(body):
        return A.hazards(k + body + "\ts_endpgm\n")

    asm = lambda ins: f"\t;;#ASMSTART\n\t{ins}\n\t;;#ASMEND\n"  # noqa: E731
    mf = "v_mfma_f32_32x32x16_f16"
    r1 = "\tv_mov_b32_e32 v4, 0\n" + asm(f"{mf} a[0:15], v[4:7], v[8:11], 0")
    assert [h.split(": ")[1][:2] for h in run(r1)] == ["R1"]
    assert run("\tv_mov_b32_e32 v4, 0\n\ts_nop 0\n" + asm(f"{mf} a[0:15], v[4:7], v[8:11], 0")) == []
    zero16 = "".join(f"\tv_accvgpr_write_b32 a{i}, 0\n" for i in range(16))
    r2 = zero16 + "\ts_nop 0\n" + asm(f"{mf} a[0:15], v[4:7], v[8:11], a[0:15]")
    assert [h.split(": ")[1][:2] for h in run(r2)] == ["R2"]
    assert run(r2.replace("s_nop 0", "s_nop 1")) == []
    r3 = asm(f"{mf} v[0:15], v[20:23], v[24:27], 0") + "\ts_nop 3\n\tv_add_f32_e32 v30, v1, v2\n"
    assert {h.split(": ")[1][:2] for h in run(r3)} == {"R3"}
    assert run(asm(f"{mf} v[0:15], v[20:23], v[24:27], 0") + "\ts_nop 11\n\tv_add_f32_e32 v30, v1, v2\n") == []
    # back-to-back MFMAs issue 8 slots apart (the pipe): three of them cover the 12 wait states
    three = asm(f"{mf} v[0:15], v[20:23], v[24:27], 0\n\t{mf} v[40:55], v[20:23], v[24:27], 0\n\t"
                f"{mf} v[60:75], v[20:23], v[24:27], 0")
    assert run(three + "\tv_add_f32_e32 v30, v1, v2\n") == []
    # R5: an accumulator read out (epilogue) and accumulated into again without a re-zeroing write
    z = "".join(f"\tv_accvgpr_write_b32 a{i}, 0\n" for i in range(16)) + "\ts_nop 1\n"
    body = z + asm(f"{mf} a[0:15], v[4:7], v[8:11], a[0:15]") + "\ts_nop 15\n\tv_accvgpr_read_b32 v50, a0\n"
    loop = ".LBB0_1:\n" + body + "\ts_cbranch_scc1 .LBB0_1\n"
    assert any("R5" in h for h in run(loop.replace(z, "")))  # never zeroed: undefined, then stale
    assert run(loop) == []
    # code placed after an s_endpgm and reached by a long branch (s_getpc / s_add_u32 (.LBBn - .Lpost_getpc)
    # / s_setpc_b64, what hipcc emits when a kernel outgrows 16-bit branch offsets) is part of the CFG:
    # the violation in it is found, and the long branch is not a fall-through into the next block
    far = (z + "\ts_getpc_b64 s[0:1]\n.Lpost_getpc0:\n\ts_add_u32 s0, s0, (.LBB0_9-.Lpost_getpc0)&4294967295\n"
           "\ts_addc_u32 s1, s1, (.LBB0_9-.Lpost_getpc0)>>32\n\ts_setpc_b64 s[0:1]\n"
           ".LBB0_5:\n\tv_accvgpr_read_b32 v50, a0\n\ts_endpgm\n"
           ".LBB0_9:\n\tv_mov_b32_e32 v4, 0\n" + asm(f"{mf} a[0:15], v[4:7], v[8:11], a[0:15]") + "\ts_nop 15\n\ts_branch .LBB0_5\n")
    assert [h.split(": ")[1][:2] for h in A.hazards(k + far + ".Lfunc_end0:\n")] == ["R1"]
    # hipcc's structurised joins: a flag pair set to -1 / 0 on the incoming edges and tested after the join.
    # The accumulating MFMA is reached only on the edge that zeroed O (flag 0): no R5; with the flag
    # values swapped the stale path is feasible and R5 fires
    def joined(flag_zeroed, flag_skipped):
        return ("\ts_cbranch_scc1 .LBB0_2\n" + zero16 + f"\ts_mov_b64 s[68:69], {flag_zeroed}\n\ts_branch .LBB0_3\n"
                f".LBB0_2:\n\tv_accvgpr_read_b32 v50, a0\n\ts_mov_b64 s[68:69], {flag_skipped}\n"
                ".LBB0_3:\n\ts_and_b64 vcc, exec, s[68:69]\n\ts_cbranch_vccz .LBB0_4\n\ts_endpgm\n"
                ".LBB0_4:\n\ts_nop 1\n" + asm(f"{mf} a[0:15], v[4:7], v[8:11], a[0:15]"))
    assert run(joined(0, -1)) == []
    assert any("R5" in h for h in run(joined(-1, 0)))


def test_mfma_hazard_gate_passes_the_product_assembly():
    from flash_attention_cute_amd import _asm_check as A
    from flash_attention_cute_amd import _build

    files = sorted((_build.ROOT / "build" / "obj").glob("*/fa_inst-hip-amdgcn-amd-amdhsa-gfx950.s"))
    if not files:
        pytest.skip("no product assembly in build/obj (run __graft_entry__.build())")
    assert len(files) == 16
    for f in files:
        assert A.hazards(f.read_text()) == [], f
