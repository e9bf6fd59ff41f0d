#!/bin/bash
# round 6: the MFMA-shape A/B body (csrc/fa_fwd_mb.hpp). Phase "tests": the parity sweep and every
# reference-produced fixture on both shapes (debug library); phase "ab": same-process interleaved A/B of
# the product kernel (fa_fwd_w4, 32x32x16) against fa_fwd_mb with 32x32x16 (m32) and 16x16x32 (m16) on
# C2 / C3 / C4 / C5 (AB_WS=1: the product takes its workspace layouts); phase "pmc": per body, one
# rocprofv3 PMC pass (GRBM_GUI_ACTIVE -> effective clock, SQ_INSTS_VALU / SQ_INSTS_MFMA, SQ_BUSY_CYCLES).
# usage: r6_shape.sh <tag> [tests|ab|pmc|all]
set -o pipefail
TAG=${1:-r6s}; PH=${2:-all}
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/$TAG; mkdir -p $OUT
DBG=flash_attention_cute_amd/lib/libfa_gfx950_debug.so PROD=flash_attention_cute_amd/lib/libfa_gfx950.so
if [ $PH = all ] || [ $PH = tests ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 200 \
    --timeout-method thread -k "m16 or m32 or shape_bodies" > $OUT/pytest_shape.log 2>&1; rc=$?
  tail -3 $OUT/pytest_shape.log; [ $rc -eq 0 ] || exit 1
fi
if [ $PH = all ] || [ $PH = ab ]; then
  export AB_WS=1 AB_REPS=${AB_REPS:-7}
  for c in c2 c3 c4; do
    timeout -k 10 300 python scripts/ab_libs.py $c $PROD $DBG@m32 $DBG@m16 > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
    cat $OUT/ab_$c.log
  done
  AB_SHAPE=8,32,8,4096,128,bf16,1 timeout -k 10 300 python scripts/ab_libs.py c5 $PROD $DBG@m32 $DBG@m16 > $OUT/ab_c5.log 2>&1 || { tail -5 $OUT/ab_c5.log; exit 1; }
  cat $OUT/ab_c5.log
fi
if [ $PH = all ] || [ $PH = pmc ]; then
  for v in m32 m16; do
    for c in c2 c4; do
      FA_GFX950_VARIANT=$v AB_REPS=2 AB_ITERS=10 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        --kernel-trace -d $OUT/pmc_${v}_$c -o run --output-format csv -- python3 scripts/ab_libs.py $c $DBG@$v > $OUT/pmc_${v}_$c.log 2>&1 || { tail -5 $OUT/pmc_${v}_$c.log; exit 1; }
    done
  done
  FA_GFX950_VARIANT= AB_REPS=2 AB_ITERS=10 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --kernel-trace -d $OUT/pmc_w4_c2 -o run --output-format csv -- python3 scripts/ab_libs.py c2 $PROD > $OUT/pmc_w4_c2.log 2>&1 || exit 1
  ls $OUT
fi
