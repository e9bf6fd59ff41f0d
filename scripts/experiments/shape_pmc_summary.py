#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the attention kernels (run_counter_collection.csv): per body, the mean
per dispatch of each counter over the fa_fwd_* dispatches, the kernel time from the same rows, the effective
clock GRBM_GUI_ACTIVE / 8 / time (rocprofv3 sums the 8 XCDs, MI355X_MICROARCH "DVFS give-back") and the
VALU instructions per MFMA.  usage: shape_pmc_summary.py <dir> [<dir> ...]"""
import csv
import sys
from collections import defaultdict

csv.field_size_limit(1 << 30)
for d in sys.argv[1:]:
    acc = defaultdict(list)
    times = {}
    name = None
    with open(f"{d}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if "fa_fwd" not in row["Kernel_Name"]:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
            times[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    if not acc:
        print(d, "no fa_fwd dispatches")
        continue
    mean = {k: sum(v) / len(v) for k, v in acc.items()}
    t = sum(times.values()) / len(times)
    out = {"dispatches": len(times), "kernel_ms": round(t * 1e3, 4)}
    if "GRBM_GUI_ACTIVE" in mean:
        out["eff_clock_GHz"] = round(mean["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 3)
    if "SQ_INSTS_VALU" in mean and "SQ_INSTS_MFMA" in mean:
        out["valu_per_mfma"] = round(mean["SQ_INSTS_VALU"] / mean["SQ_INSTS_MFMA"], 3)
    out.update({k: f"{v:.4g}" for k, v in sorted(mean.items())})
    print(d.rstrip("/").split("/")[-1], name[:60], out)
