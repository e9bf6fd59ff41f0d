#!/bin/bash
# round 5: key-split pieces that meet store one block each (FA_SPLIT_HALF): pytest -m gpu, A/B on C4's
# 8-way share against r5f (committed before the packed combine) and pk (packed combine, HALF=0)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
AB_REPS=11 AB_WS=1 AB_SHAPE=1,16,4,4096,128,fp16,1 timeout -k 10 240 python scripts/ab_libs.py c4 ab/r5f.so ab/pk.so $NEW > $OUT/ab_c4share.log 2>&1 || { tail -5 $OUT/ab_c4share.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_c4share.log
python -c "import flash_attention_cute_amd as m; print('split errors', m.split_errors())"
for c in c2 c4 c5; do
  for w in 8; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --world $w --rank 0 --steps 100 > $OUT/bench_${c}_w${w}r0.json 2> $OUT/bench_${c}_w${w}r0.err || { tail -5 $OUT/bench_${c}_w${w}r0.err; exit 1; }
    cut -c1-200 $OUT/bench_${c}_w${w}r0.json
  done
done
