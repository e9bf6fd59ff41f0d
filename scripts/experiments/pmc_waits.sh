#!/bin/bash
# Where the waves of one bench config wait: the SQ wait / active-instruction counters this gfx950
# exposes (rocprofv3 --list-avail), at most 6 SQ counters per pass, each pass its own run.
# usage: bash scripts/experiments/pmc_waits.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r4}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcw_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || { echo "list-avail failed"; tail -5 $OUT/list_avail.txt; exit 1; }
CANDS="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_INSTS_BRANCH SQ_WAIT_INST_VMEM"
HAVE=""
for c in $CANDS; do grep -qw "$c" $OUT/list_avail.txt && HAVE="$HAVE $c"; done
echo "available: $HAVE"
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --warmup-seconds 0.5 $*"
cd /tmp
set -- $HAVE
i=0
while [ $# -gt 0 ]; do
  PASS="$1 ${2:-} ${3:-} ${4:-} ${5:-} ${6:-}"; PASS=$(echo $PASS)
  shift 6 2>/dev/null || shift $#
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $PASS --output-format csv -d $OUT/pass$i -o run -- python3 $BENCH > $OUT/pass$i.log 2>&1 || { echo "pass $i ($PASS) failed"; tail -3 $OUT/pass$i.log; exit 1; }
  echo "pass $i: $PASS"
done
