#!/bin/bash
# row-sum microbench, then same-process A/B of the product library vs the dot2 row-sum build
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4dot; mkdir -p $OUT
timeout -k 10 60 ./scripts/microbench/rowsum_filler > $OUT/rowsum_filler.log 2>&1 || { cat $OUT/rowsum_filler.log; exit 1; }
grep -v amdgpu.ids $OUT/rowsum_filler.log
AB_REPS=7 bash scripts/experiments/ab_run.sh "c2 c4 c5 c3" flash_attention_cute_amd/lib/libfa_gfx950.so "$@" > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
cat $OUT/ab.log
