#!/bin/bash
# plain bench lines of every config on the committed library, after its PMC passes (profiles/pmc_<cfg>.json
# carries this library's hash, so each line's roofline.traffic is live). usage: r5_benches.sh <tag>
set -o pipefail
TAG=${1:-r5z}; cd $GRAFT_REPO_ROOT; OUT=gpurun_out/${TAG}_benches; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/default_bench.json 2> $OUT/default_bench.err || { tail -5 $OUT/default_bench.err; exit 1; }
cut -c1-200 $OUT/default_bench.json
for c in c2 c3 c4 c5 c5_layer window decode decode_long decode_padded; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  cut -c1-160 $OUT/bench_$c.json
done
