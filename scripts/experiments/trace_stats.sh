#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py per config -> gpurun_out/trace_<cfg>/kernel_stats.csv + bench line
set -o pipefail
export TMPDIR=/tmp
for c in $1; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_$c; mkdir -p $OUT
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline > $OUT/trace.log 2>&1) || { tail -20 $OUT/trace.log; exit 1; }
  find $OUT/t -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
  grep '^{"metric"' $OUT/trace.log > $OUT/bench_line.json
done
