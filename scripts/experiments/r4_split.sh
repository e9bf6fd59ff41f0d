#!/bin/bash
# key-split causal blocks: their GPU tests (and the tests they touch), then the same-process layout A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4split; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 120 --timeout-method thread \
  -k "key_split or zigzag or sharded or graph_capture or persistent_grid or deterministic" > $OUT/pytest_split.log 2>&1; rc=$?
tail -15 $OUT/pytest_split.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/experiments/split_ab.py > $OUT/split_ab.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/split_ab.log
exit $rc
