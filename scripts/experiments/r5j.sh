#!/bin/bash
# round 5: key-split split point n_end / 2 - s (FA_SPLIT_SHIFT s = -1, 1, 2) against the product (s = 0) on C4's
# 8-way share and a B1 H8 S8192 causal prefill (both one-round key-split grids)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5j; mkdir -p $OUT
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
AB_REPS=11 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 300 python scripts/ab_libs.py c4 $NEW abx/shm1.so abx/sh1.so abx/sh2.so > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
AB_REPS=9 AB_WS=1 AB_SHAPE=1,8,8,8192,128,fp16,1 timeout -k 10 300 python scripts/ab_libs.py c4 $NEW abx/shm1.so abx/sh1.so abx/sh2.so > $OUT/ab_s8192.log 2>&1 || { tail -5 $OUT/ab_s8192.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_s8192.log
