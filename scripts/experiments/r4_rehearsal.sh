#!/bin/bash
# multi-rank rehearsal of the strong split on ONE GPU (BENCH_SHARE_GPU=1: every rank on cuda:0; the
# numbers are not scaling numbers): bench.py --gpus N self-launches torch.distributed.run, ranks meet on
# a gloo group, each runs its (batch, kv-head) share; N = 2 and 4, C2 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4r; mkdir -p $OUT
for n in 2 4; do
  for c in c2 c5; do
    BENCH_SHARE_GPU=1 timeout -k 10 240 python bench.py --gpus $n --config $c --steps 20 --warmup 3 --no-cpu-baseline > $OUT/rehearsal_${c}_n$n.json 2> $OUT/rehearsal_${c}_n$n.err || { tail -8 $OUT/rehearsal_${c}_n$n.err; exit 1; }
    cut -c1-260 $OUT/rehearsal_${c}_n$n.json
  done
done
