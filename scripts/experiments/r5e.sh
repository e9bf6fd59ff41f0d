#!/bin/bash
# round 5: A/B of the if-then tile-end rescale (xres) against r5c, whole configs and C4's 8-way share
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5e; mkdir -p $OUT
for c in c2 c4 c5 c3; do
  AB_REPS=9 timeout -k 10 240 python scripts/ab_libs.py $c ab/r5c.so ab/xres.so > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$c.log
done
AB_REPS=9 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 200 python scripts/ab_libs.py c4 ab/r5c.so ab/xres.so > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
