#!/bin/bash
# decode kernel: GPU tests, benches, rocprofv3 kernel stats + HBM PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_decode.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_decode.log; [ $rc -le 1 ] || exit $rc
for c in decode decode_long; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_$c.log || exit 1
done
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_decode; mkdir -p $OUT
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --config decode"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
for CTR in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc_$CTR -o run -- python3 $B > $OUT/pmc_$CTR.log 2>&1 || { echo "pmc $CTR failed"; tail -5 $OUT/pmc_$CTR.log; exit 1; }
done
find $OUT -name "*stats.csv"
