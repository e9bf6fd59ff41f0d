#!/bin/bash
# round 5: the softmax scale-and-subtract two scores per v_pk_fma_f32, one pair ahead (FA_PK_FMA): pytest -m gpu,
# same-process A/B against abx/fold.so (one v_fma_f32 per score) on C2, C4, C5, C3 and C4's 8-way share
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
for c in c2 c4 c5 c3; do
  AB_REPS=9 timeout -k 10 240 python scripts/ab_libs.py $c abx/fold.so $NEW > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$c.log
done
AB_REPS=11 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 240 python scripts/ab_libs.py c4 abx/fold.so $NEW > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
