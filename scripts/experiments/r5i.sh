#!/bin/bash
# round 5: key-split pieces finish one block each with a one-hop state word (FA_SPLIT_HALF): pytest -m gpu,
# A/B on C4's 8-way share against pk (packed combine, the second piece finishes both), stamps of both
# protocols with each wave's key-split role
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5i; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
AB_REPS=11 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 240 python scripts/ab_libs.py c4 ab/pk.so $NEW > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
for v in h0 h1; do
  STAMPS_WS=1 STAMPS_SHAPE=1,16,4,4096,1,fp16 FA_STAMPS_LIB=ab/stamps_$v.so timeout -k 10 120 python scripts/stamps.py c4 > $OUT/stamps_${v}_c4share.log 2>&1 || { tail -5 $OUT/stamps_${v}_c4share.log; exit 1; }
  echo "== $v"; grep -E "span|epilogue|block cycles" $OUT/stamps_${v}_c4share.log
done
