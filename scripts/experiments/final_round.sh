#!/bin/bash
# bench lines of every config + rocprofv3 kernel-trace stats of C2 / C4 (one GPU call)
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r2f}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
for c in c2 c3 c4 c5 window decode; do
  timeout -k 10 200 python bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
export TMPDIR=/tmp; cd /tmp
for c in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$c -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --config $c > $OUT/trace_$c.log 2>&1 || { echo "trace $c failed"; exit 1; }
  find $OUT/trace_$c -name "*kernel_stats.csv" -exec cp {} $OUT/${c}_kernel_stats.csv \;
done
