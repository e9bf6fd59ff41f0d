#!/bin/bash
# usage: bash scripts/experiments/ab_run.sh "c2 c4 c5" lib1.so lib2.so ...   (interleaved A/B of library builds)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
CFGS=$1; shift
for c in $CFGS; do
  timeout -k 10 180 python scripts/ab_libs.py $c "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
