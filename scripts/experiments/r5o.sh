#!/bin/bash
# round 5: split-KV decode with the merge fused into fa_decode (the last split of a unit merges; FA_DEC_FUSE):
# decode GPU tests, the whole GPU suite, and decode_long / decode bench lines with the fused and the separate
# merge (FA_DEC_FUSE=0), alternating, in separate processes on one box
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_decode.log 2>&1 || { tail -30 $OUT/pytest_decode.log; exit 1; }
tail -2 $OUT/pytest_decode.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for rep in 1 2; do
  for f in 1 0; do
    FA_DEC_FUSE=$f timeout -k 10 200 python bench.py --config decode_long --no-cpu-baseline --steps 200 > $OUT/bench_decode_long_f${f}_$rep.json 2> $OUT/bench_decode_long_f${f}_$rep.err || { tail -5 $OUT/bench_decode_long_f${f}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_decode_long_f${f}_$rep.json').read()); print('decode_long fuse=$f', d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel_ms_median'))"
  done
done
