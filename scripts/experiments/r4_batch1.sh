#!/bin/bash
# round-4 GPU batch: pytest -m gpu of the product tree, the C=0 reproduction, A/B of experiment libs
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-r4b}; mkdir -p $OUT; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -4 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python scripts/experiments/czero_repro.py ab/czero_libfa_gfx950.so > $OUT/czero_repro.log 2>&1; rc=$?
cat $OUT/czero_repro.log
[ $rc -le 1 ] || exit $rc
shift
if [ $# -gt 0 ]; then
  AB_REPS=7 bash scripts/experiments/ab_run.sh "c2 c4 c5" "$@" > $OUT/ab.log 2>&1 || exit 1
  cat $OUT/ab.log
fi
# one-rank shares of the 8-way strong split (zigzag layout for the small causal grids)
for c in c2 c4 c5; do
  timeout -k 10 200 python bench.py --config $c --world 8 --rank 0 --steps 200 > $OUT/bench_${c}_w8r0.json 2> $OUT/bench_${c}_w8r0.err || exit 1
  cut -c1-220 $OUT/bench_${c}_w8r0.json
done
