#!/bin/bash
# rocprofv3 passes for one bench config: kernel trace + stats, then separate PMC passes.
# usage: bash scripts/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline $*"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
# (round 5: the L2 hit split and the memory-side read requests that go to DRAM, one pass of 4 TCC counters)
for CTR in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" ; do
  N=$(echo $CTR | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc_$N -o run -- python3 $BENCH --warmup-seconds 0.5 > $OUT/pmc_$N.log 2>&1 || { echo "pmc $CTR failed"; tail -5 $OUT/pmc_$N.log; }
done
cp $OUT/trace/*/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null || find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
grep "^{\"metric\"" $OUT/trace.log > $OUT/bench_line.json
find $OUT -name "*.csv" | head -50
