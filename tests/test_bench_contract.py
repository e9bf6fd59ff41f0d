"""bench.py's measurement bookkeeping on CPU: the PMC traffic it reports is tied to the library that
ran ("roofline.traffic is a stored constant"), and the roofline arithmetic uses the
algorithmic FLOPs / bytes of DESIGN.md section 5. No GPU needed."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _fake_tree(tmp_path, lib_bytes: bytes, pmc: dict | None):
    (tmp_path / "flash_attention_cute_amd" / "lib").mkdir(parents=True)
    (tmp_path / "flash_attention_cute_amd" / "lib" / "libfa_gfx950.so").write_bytes(lib_bytes)
    (tmp_path / "profiles").mkdir()
    if pmc is not None:
        (tmp_path / "profiles" / "pmc_c2.json").write_text(json.dumps(pmc))


def test_traffic_is_used_only_for_the_profiled_library(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    _fake_tree(tmp_path, b"library A", None)
    sha = bench.lib_sha16()
    assert len(sha) == 16
    (tmp_path / "profiles" / "pmc_c2.json").write_text(json.dumps({"lib_sha16": sha, "hbm_bytes_per_launch": 123.0}))
    traffic, why = bench.load_traffic("c2")
    assert traffic == 123.0 and why["traffic_stale"] is False
    # the library changes, the committed PMC file does not: no stale number, and the reason says why
    (tmp_path / "flash_attention_cute_amd" / "lib" / "libfa_gfx950.so").write_bytes(b"library B")
    traffic, why = bench.load_traffic("c2")
    assert traffic is None and why["traffic_stale"] is True
    assert why["traffic_profiled_lib"] == sha and why["traffic_this_lib"] != sha
    assert why["traffic_of_profiled_lib"] == 123.0


def test_traffic_absent_without_a_pmc_file(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    _fake_tree(tmp_path, b"library", None)
    assert bench.load_traffic("c2") == (None, {"traffic_source": None})


def test_committed_pmc_files_carry_a_library_hash():
    for p in sorted((ROOT / "profiles").glob("pmc_*.json")):
        d = json.loads(p.read_text())
        assert len(d.get("lib_sha16", "")) == 16, p.name
        assert d["hbm_bytes_per_launch"] > 0, p.name


def test_algorithmic_counts_of_the_headline_config():
    c = bench.CONFIGS["c2"]
    assert bench.flops(c) == 4 * 4 * 32 * 4096 * 4096 * 128  # 4 Sq Sk D per (b, head), non-causal
    assert bench.algo_bytes(c) == 536870912  # q, k, v, o once each
