#!/bin/bash
# final library (key-split, both blocks' records per round trip): GPU suite, smoke, profiles of every config
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash scripts/experiments/profile_all.sh r4w "c2 c3 c4 c5 window decode decode_long decode_padded" 2>&1 | cut -c1-160
