#!/bin/bash
# key-split on by default: the whole GPU suite, smoke, and the layout A/B (default rule)
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4s2; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -12 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python scripts/experiments/split_ab.py > $OUT/split_ab.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/split_ab.log
exit $rc
