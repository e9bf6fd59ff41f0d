#!/bin/bash
# round 5: stamps of the final kernel body (stamps_lib/${STLIB:-stamps_r5z}.so, -DFA_STAMPS of the committed source) on
# C2, C4 and C4's 8-way share (key-split, with each wave's hand-off role)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/${STLIB:-stamps_r5z}; mkdir -p $OUT
for c in c2 c4; do
  FA_STAMPS_LIB=stamps_lib/${STLIB:-stamps_r5z}.so timeout -k 10 120 python scripts/stamps.py $c > $OUT/stamps_$c.log 2>&1 || { tail -5 $OUT/stamps_$c.log; exit 1; }
done
STAMPS_WS=1 STAMPS_SHAPE=1,16,4,4096,1,fp16 FA_STAMPS_LIB=stamps_lib/${STLIB:-stamps_r5z}.so timeout -k 10 120 python scripts/stamps.py c4 > $OUT/stamps_c4share.log 2>&1 || { tail -5 $OUT/stamps_c4share.log; exit 1; }
for f in $OUT/stamps_*.log; do echo "== $f"; grep -vE "amdgpu.ids|xcd [0-9]" $f; done
