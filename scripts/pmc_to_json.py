"""Turn a scripts/profile.sh (or pmc.sh) output dir into profiles/pmc_<config>.json.

HBM traffic per launch of the attention kernel, corrected as MI355X_MICROARCH.md 'HBM' prescribes:
FETCH_SIZE and WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B / lane) streaming read, so it is doubled; WRITE_SIZE is exact for 16 B / lane stores.
usage: python scripts/pmc_to_json.py <prof dir> <config> <out json> [source note]
"""
import collections
import csv
import glob
import json
import os
import sys

# kernels whose dispatches are averaged (the dominant kernel of the config)
KERNELS = os.environ.get("PMC_KERNELS", "fa::fa_fwd,fa::fa_decode<").split(",")

src, cfg, out = sys.argv[1], sys.argv[2], sys.argv[3]
note = sys.argv[4] if len(sys.argv) > 4 else src
agg = collections.defaultdict(list)
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in KERNELS):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
if not agg:  # (a missing or empty profile directory must not overwrite a good pmc_<cfg>.json)
    sys.exit(f"pmc_to_json: no counter rows of {KERNELS} under {src}")
mean = {k: sum(v) / len(v) for k, v in agg.items()}
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import code_sha16, lib_sha16  # noqa: E402  (the library these passes profiled: bench.py uses
#                                   the traffic only while the loaded library's device code has this hash)

res = {"config": cfg, "source": note, "lib_sha16": lib_sha16(), "code_sha16": code_sha16(), "dispatches": {k: len(v) for k, v in agg.items()},
       "counters_mean_per_dispatch": mean}
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    fetch = mean["FETCH_SIZE"] * 1024 * 2
    write = mean["WRITE_SIZE"] * 1024
    res.update({"fetch_bytes_corrected": fetch, "write_bytes": write, "hbm_bytes_per_launch": fetch + write})
if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
    res["l2_hit_rate"] = mean["TCC_HIT_sum"] / max(1.0, mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
if "TCC_EA0_RDREQ_sum" in mean and "TCC_EA0_RDREQ_DRAM_sum" in mean:
    # the L2's memory-side read requests (FETCH_SIZE counts them all, Infinity-Cache hits included) and
    # the share of them the fabric sends on to DRAM
    res["rdreq_dram_frac"] = mean["TCC_EA0_RDREQ_DRAM_sum"] / max(1.0, mean["TCC_EA0_RDREQ_sum"])
    if "fetch_bytes_corrected" in res:
        res["fetch_bytes_dram"] = res["fetch_bytes_corrected"] * res["rdreq_dram_frac"]
        res["hbm_bytes_per_launch_dram"] = res["fetch_bytes_dram"] + res["write_bytes"]
if "GRBM_GUI_ACTIVE" in mean:
    res["xcd_active_cycles"] = mean["GRBM_GUI_ACTIVE"] / 8
if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
    res["mfma_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (mean["GRBM_GUI_ACTIVE"] / 8)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
