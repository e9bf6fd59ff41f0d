#!/bin/bash
# round 5, packed key-split combine (FA_SPLIT_PK): pytest -m gpu, A/B against r5f (the committed product)
# on C4's 8-way share (key-split) and on C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
AB_REPS=11 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 240 python scripts/ab_libs.py c4 ab/r5f.so $NEW > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
for c in c4 c5; do
  AB_REPS=7 timeout -k 10 200 python scripts/ab_libs.py $c ab/r5f.so $NEW > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$c.log
done
