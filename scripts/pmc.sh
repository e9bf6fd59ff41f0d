#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over bench.py; usage: scripts/pmc.sh <tag> <config> "<grp1>" "<grp2>" ...
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --config $CFG"
for CTR in "$@"; do
  N=$(echo $CTR | tr ' ' '_' | cut -c1-60)
  timeout -k 10 240 rocprofv3 --pmc $CTR --output-format csv -d $OUT/$N -o run -- python3 $BENCH > $OUT/$N.log 2>&1 || { echo "pmc $CTR failed"; tail -5 $OUT/$N.log; }
done
python3 $GRAFT_REPO_ROOT/scripts/pmc_summary.py $OUT | tee $OUT/summary.txt
