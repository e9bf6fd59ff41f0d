#!/bin/bash
# pytest -m gpu, the default bench line, and one-rank shares of the 8-way strong split (C2, C4, C5)
# next to their whole-workload lines. usage: r4_shares.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r4a}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
cut -c1-400 $OUT/bench_default.json
for c in c2 c4 c5; do
  if [ $c != c2 ]; then
    timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  fi
  for r in 0 7; do
    timeout -k 10 200 python bench.py --config $c --world 8 --rank $r --steps 200 > $OUT/bench_${c}_w8r$r.json 2> $OUT/bench_${c}_w8r$r.err || { tail -5 $OUT/bench_${c}_w8r$r.err; exit 1; }
    cut -c1-300 $OUT/bench_${c}_w8r$r.json
  done
done
