"""Build tagged stamps/experiment variants of the ABI library (only the instantiations that
scripts/stamps.py c2 / c4 run). usage: python scripts/experiments/build_exp.py tag[:DEF1,DEF2][:flag flag] ..."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from flash_attention_cute_amd import _build  # noqa: E402

ONLY = (("F16", 0, 128, 1), ("F16", 1, 128, 1), ("BF16", 1, 128, 1))


def one(spec):
    parts = spec.split(":")
    tag = parts[0]
    defs = tuple(x for x in parts[1].split(",") if x) if len(parts) > 1 else ()
    flags = tuple(parts[2].split()) if len(parts) > 2 else ()
    stamps = not tag.startswith("x")  # tags starting with "x": plain experiment builds (no stamps)
    # EXP_NOGATE=1: the _asm_check gate's findings become warnings (diagnostic builds such as
    # FA_EXP_CZERO, which the gate rejects by design)
    return _build.build_abi(stamps=stamps, tag=tag, defines=defs, flags=flags, only=ONLY, force=True,
                            gate=os.environ.get("EXP_NOGATE") != "1")


with ThreadPoolExecutor(max_workers=4) as ex:
    for r in ex.map(one, sys.argv[1:]):
        print(r)
