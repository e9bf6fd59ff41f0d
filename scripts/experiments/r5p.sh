#!/bin/bash
# round 5: same-process A/B of the decode kernels, the library before the fused decode merge (abd/prev.so) against
# the final one, on decode (B32, unsplit), decode_padded-like B32 and decode_long (split-KV, workspace)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5p; mkdir -p $OUT
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
AB_REPS=11 timeout -k 10 200 python scripts/ab_libs.py decode abd/prev.so $NEW > $OUT/ab_decode.log 2>&1 || { tail -5 $OUT/ab_decode.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_decode.log
AB_REPS=11 AB_WS=1 timeout -k 10 200 python scripts/ab_libs.py decode_long abd/prev.so $NEW > $OUT/ab_decode_long.log 2>&1 || { tail -5 $OUT/ab_decode_long.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_decode_long.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
