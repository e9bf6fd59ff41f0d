#!/bin/bash
# Quick perf loop on the GPU box: stamps diagnostic + SQ PMC pass + bench for the given configs.
# usage: bash scripts/experiments/gpu_perf.sh "c2 c4" [pmc-tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${1:-c2}; do
  timeout -k 10 120 python scripts/stamps.py $c 2>&1 | grep -v amdgpu.ids | tee gpurun_out/stamps_$c.log || exit 1
done
for c in ${1:-c2}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config $c --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_$c.log || exit 1
done
