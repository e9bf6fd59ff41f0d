#!/bin/bash
# round 5, first GPU pass: pytest -m gpu on the first-tile build, same-process A/B against the round-4
# library (ab/base.so) on the whole configs and on C4's 8-way share (key-split), stamps of the new body
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
for c in c2 c4 c5 c3; do
  timeout -k 10 200 python scripts/ab_libs.py $c ab/base.so $NEW > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$c.log
done
AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 200 python scripts/ab_libs.py c4 ab/base.so $NEW > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
for c in c2 c4; do
  FA_STAMPS_LIB=ab/stamps_new.so timeout -k 10 120 python scripts/stamps.py $c > $OUT/stamps_$c.log 2>&1 || { tail -5 $OUT/stamps_$c.log; exit 1; }
done
grep -v amdgpu.ids $OUT/stamps_c4.log | head -40
