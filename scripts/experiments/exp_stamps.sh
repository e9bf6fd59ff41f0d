#!/bin/bash
# run scripts/stamps.py on each tagged experiment build: usage exp_stamps.sh "tag1 tag2" [cfg]
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for t in $1; do
  echo "=== $t"
  FA_STAMPS_LIB=build/stamps_$t/libfa_gfx950.so timeout -k 10 60 python scripts/stamps.py ${2:-c2} 2>&1 | grep -E "per tile|clock|total |p50" || exit 1
done
