#!/bin/bash
# key-split with 2 / 4 pieces: the split tests, then the sweep with both piece counts
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4p; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 120 --timeout-method thread \
  -k "key_split or zigzag or sharded or graph_capture or persistent_grid or deterministic" > $OUT/pytest_split.log 2>&1; rc=$?
tail -8 $OUT/pytest_split.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python scripts/experiments/split_ab.py --sweep --pieces > $OUT/sweep.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/sweep.log
