#!/bin/bash
# round 5, second GPU pass: pytest -m gpu on the product build (first tile + MFMA zeroing + overlapped drain
# + deferred epilogue + key-split combine from AGPRs), A/B of r5a (committed) / xa34 (zeroing + drain) /
# xa345 (+ deferred epilogue) / the product build
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in c2 c4 c5 c3; do
  AB_REPS=7 timeout -k 10 240 python scripts/ab_libs.py $c ab/r5a.so ab/xa34.so ab/xa345.so flash_attention_cute_amd/lib/libfa_gfx950.so > $OUT/ab_$c.log 2>&1 || { tail -5 $OUT/ab_$c.log; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$c.log
done
AB_REPS=7 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 200 python scripts/ab_libs.py c4 ab/r5a.so ab/xa34.so ab/xa345.so flash_attention_cute_amd/lib/libfa_gfx950.so > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
timeout -k 10 60 rocprofv3 --list-avail > $OUT/rocprof_avail.txt 2>&1 || true
grep -ciE "TCC_EA0_RDREQ|MALL|DRAM" $OUT/rocprof_avail.txt || true
