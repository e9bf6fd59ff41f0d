#!/bin/bash
# A/B of the persistent fa_fwd_w4 grid: default cap vs FA_W4_GRID values, per config.
# usage: bash scripts/dev/ab_grid.sh "c2 c4 c5" "100000 512"
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in ${1:-c2}; do
  for g in default ${2:-100000}; do
    if [ $g = default ]; then unset FA_W4_GRID; else export FA_W4_GRID=$g; fi
    v=$(timeout -k 10 120 python bench.py --steps 30 --warmup 10 --config $c --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*') || exit 1
    echo "$c grid=$g $v"
  done
done
