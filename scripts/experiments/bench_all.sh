#!/bin/bash
# Every bench config once (C2 with the CPU baseline), one JSON line each -> gpurun_out/bench_<cfg>.log
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_c2.log || exit 1
for c in ${1:-c3 c4 c5 decode decode_long}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_$c.log || exit 1
done
