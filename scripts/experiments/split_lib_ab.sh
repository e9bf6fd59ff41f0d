#!/bin/bash
# same-process A/B of key-split library builds (workspace passed) on one-round causal shapes
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/splitlib; mkdir -p $OUT
for sh in 1,16,4,4096,128,fp16,1 1,8,2,4096,128,bf16,1 1,8,8,8192,128,bf16,1 1,16,4,3072,128,bf16,1; do
  AB_WS=1 AB_SHAPE=$sh AB_REPS=7 timeout -k 10 200 python scripts/ab_libs.py c4 "$@" > $OUT/ab_$sh.log 2>&1 || { tail -5 $OUT/ab_$sh.log; exit 1; }
  echo "shape $sh"; grep -v amdgpu.ids $OUT/ab_$sh.log
done
