#!/bin/bash
# round 5, final library: GPU suite, smoke, the driver's default bench line, one GPU's share of the 2-, 4- and
# 8-way strong split of C2 / C4 / C5 (the predicted 1 -> 8 curve), then every config's rocprofv3 kernel
# trace + stats and PMC passes (scripts/profile.sh, incl. the L2 hit / DRAM split) and a plain bench line.
# usage: [CFGS="<configs to profile>"] r5_final.sh <tag> [phase: all | tests | shares | profiles]
set -o pipefail
TAG=${1:-r5f}; PH=${2:-all}
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ $PH = all ] || [ $PH = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  timeout -k 10 300 python bench.py > $OUT/default_bench.json 2> $OUT/default_bench.err || { tail -5 $OUT/default_bench.err; exit 1; }
  cut -c1-300 $OUT/default_bench.json
fi
if [ $PH = all ] || [ $PH = shares ]; then
  for c in c2 c4 c5; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_${c}_w1.json 2> $OUT/bench_${c}_w1.err || { tail -5 $OUT/bench_${c}_w1.err; exit 1; }
    for w in 2 4 8; do
      timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --world $w --rank 0 --steps 100 > $OUT/bench_${c}_w${w}r0.json 2> $OUT/bench_${c}_w${w}r0.err || { tail -5 $OUT/bench_${c}_w${w}r0.err; exit 1; }
    done
    python - $OUT $c <<'PY'
import json, sys
out, c = sys.argv[1], sys.argv[2]
w1 = json.loads(open(f"{out}/bench_{c}_w1.json").read())["value"]
for w in (2, 4, 8):
    v = json.loads(open(f"{out}/bench_{c}_w{w}r0.json").read())["value"]
    print(f"{c} share 1/{w}: {v:.1f} TFLOPS vs whole {w1:.1f}: {v / w1:.3f}")
PY
  done
fi
if [ $PH = all ] || [ $PH = profiles ]; then
  bash scripts/experiments/profile_all.sh $TAG "${CFGS:-c2 c3 c4 c5 window decode decode_long decode_padded}" 2>&1 | cut -c1-200
fi
