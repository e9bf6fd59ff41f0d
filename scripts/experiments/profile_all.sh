#!/bin/bash
# End-of-round profiling of the in-tree library on the GPU box: per config a kernel trace + stats
# and the PMC passes of scripts/profile.sh, then a plain bench line. usage: profile_all.sh <tag> "<cfgs>"
set -o pipefail
TAG=$1; CFGS=${2:-"c2 c3 c4 c5 window decode decode_long decode_padded"}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in $CFGS; do
  echo "== $c $(date +%T)"
  bash scripts/profile.sh ${TAG}_$c --config $c > gpurun_out/prof_${TAG}_$c.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_$c.out; exit 1; }
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$c.json | cut -c1-300
done
