#!/bin/bash
# round 5, third GPU pass: pytest -m gpu on the product (deferred epilogue off, key-split combine from
# AGPRs), A/B against r5a / xa34, and stamps (prologue wait, next-block issue, first tile) of the product
# body (st3) and of the deferred-epilogue body (st4) on C2, C4 and C4's 8-way share (key-split)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5c; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
AB_REPS=9 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 200 python scripts/ab_libs.py c4 ab/r5a.so ab/xa34.so $NEW > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
for c in c4 c5; do
  AB_REPS=7 timeout -k 10 200 python scripts/ab_libs.py $c ab/r5a.so $NEW > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$c.log
done
for v in st3 st4; do
  for c in c2 c4; do
    FA_STAMPS_LIB=ab/stamps_$v.so timeout -k 10 120 python scripts/stamps.py $c > $OUT/stamps_${v}_$c.log 2>&1 || { tail -5 $OUT/stamps_${v}_$c.log; exit 1; }
  done
  STAMPS_WS=1 STAMPS_SHAPE=1,16,4,4096,1,fp16 FA_STAMPS_LIB=ab/stamps_$v.so timeout -k 10 120 python scripts/stamps.py c4 > $OUT/stamps_${v}_c4share.log 2>&1 || { tail -5 $OUT/stamps_${v}_c4share.log; exit 1; }
done
for f in $OUT/stamps_*.log; do echo "== $f"; grep -E "per tile|p50|clock|utilisation|total" $f; done
