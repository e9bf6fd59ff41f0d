#!/bin/bash
# fine in-kernel stamps (FA_STAMPS_FINE: phase 2 in quarters, phase 1 in halves) of C2 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4fine; mkdir -p $OUT
for c in c2 c4; do
  STAMPS_WIDTH=16 FA_STAMPS_LIB=ab/stamps_fine_r4.so timeout -k 10 120 python scripts/stamps.py $c > $OUT/stamps_fine_$c.log 2>&1 || { tail -5 $OUT/stamps_fine_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/stamps_fine_$c.log | head -20
done
