#!/bin/bash
# round-4 final lines of the final library (wide key-split epilogue): the driver's default bench, every config's bench line
# (PMC traffic live: profiles/pmc_<cfg>.json carries this library's hash), one GPU's share of the
# 8-way strong split of the causal configs, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r4wf; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/default_bench.json 2> $OUT/default_bench.err || { tail -5 $OUT/default_bench.err; exit 1; }
cut -c1-300 $OUT/default_bench.json
for c in c2 c3 c4 c5 window decode decode_long decode_padded; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  cut -c1-200 $OUT/bench_$c.json
done
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --world 8 --rank 0 > $OUT/bench_${c}_w8r0.json 2> $OUT/bench_${c}_w8r0.err || { tail -5 $OUT/bench_${c}_w8r0.err; exit 1; }
  cut -c1-250 $OUT/bench_${c}_w8r0.json
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
