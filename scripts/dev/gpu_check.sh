#!/bin/bash
# One GPU round: diag -> smoke -> pytest -m gpu -> bench (C2 + other configs). Stops at the first
# GPU fault / timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== diag"
timeout -k 10 300 python scripts/dev/diag.py 2>&1 | tee gpurun_out/diag.log || exit 1
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log || exit 1
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | tee gpurun_out/bench_c2.log || exit 1
for c in ${EXTRA_CONFIGS:-c3 c4 decode}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config $c --no-cpu-baseline 2>&1 | tee gpurun_out/bench_$c.log || exit 1
done
