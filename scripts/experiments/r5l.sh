#!/bin/bash
# round 5: the key-split pairs' split-point shift FA_PAIR_SHIFT (0, 1, 3, 4 against the product's 2) on C4's
# 8-way share and a B1 H8 S8192 causal prefill
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5l; mkdir -p $OUT
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
for sh in 1,16,4,4096,128,fp16,1 1,8,8,8192,128,fp16,1; do
  AB_REPS=11 AB_WS=1 AB_SHAPE=$sh timeout -k 10 300 python scripts/ab_libs.py c4 $NEW abx/ps0.so abx/ps1.so abx/ps3.so abx/ps4.so > $OUT/ab_$sh.log 2>&1 || { tail -5 $OUT/ab_$sh.log; exit 1; }
  echo "== $sh"; grep -v amdgpu.ids $OUT/ab_$sh.log
done
