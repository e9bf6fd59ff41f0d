"""Average each PMC counter over the fa_fwd_kernel dispatches of a scripts/pmc.sh output dir."""
import collections
import csv
import glob
import os
import sys

# kernels whose dispatches are averaged (the dominant kernel of the config)
KERNELS = os.environ.get("PMC_KERNELS", "fa::fa_fwd,fa::fa_decode<").split(",")

agg = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in KERNELS):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:32s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
