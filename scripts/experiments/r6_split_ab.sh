#!/bin/bash
# round 6: same-process A/B of the round-5 library (ab6/r5head.so, built from c04f5bf) against the current one
# on the key-split layouts the abandon-on-timeout hand-off touches (C4's 8-way share: pairs; a halves
# shape) and on C4 / C2 whole (no hand-off), AB_REPS interleaved repetitions.
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r6_split_ab; mkdir -p $OUT
export AB_WS=1 AB_REPS=${AB_REPS:-9}
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so OLD=ab6/r5head.so
AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 200 python scripts/ab_libs.py c4 $OLD $NEW > $OUT/c4_share8.log 2>&1 || exit 1
AB_SHAPE=1,8,8,4096,128,fp16,1 timeout -k 10 200 python scripts/ab_libs.py c4 $OLD $NEW > $OUT/halves_h8.log 2>&1 || exit 1
timeout -k 10 200 python scripts/ab_libs.py c4 $OLD $NEW > $OUT/c4.log 2>&1 || exit 1
timeout -k 10 200 python scripts/ab_libs.py c2 $OLD $NEW > $OUT/c2.log 2>&1 || exit 1
tail -n 2 $OUT/*.log
