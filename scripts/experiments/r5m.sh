#!/bin/bash
# round 5: the key-split ready flag folded into the arrivals word (one round trip less for a combining piece
# whose partner is done): split GPU tests, A/B against abx/pairs.so (separate flag word) on C4's 8-way share
# (pairs), B1 H8 S8192 (pairs) and B1 H8 S4096 (halves)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5m; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "pairs or key_split or golden" --timeout 120 --timeout-method thread > $OUT/pytest_split.log 2>&1 || { tail -30 $OUT/pytest_split.log; exit 1; }
tail -2 $OUT/pytest_split.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
for sh in 1,16,4,4096,128,fp16,1 1,8,8,8192,128,fp16,1 1,8,8,4096,128,fp16,1; do
  AB_REPS=11 AB_WS=1 AB_SHAPE=$sh timeout -k 10 300 python scripts/ab_libs.py c4 abx/pairs.so $NEW > $OUT/ab_$sh.log 2>&1 || { tail -5 $OUT/ab_$sh.log; exit 1; }
  echo "== $sh"; grep -v amdgpu.ids $OUT/ab_$sh.log
done
