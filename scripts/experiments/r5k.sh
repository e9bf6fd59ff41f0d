#!/bin/bash
# round 5: key-split pairs (a heavy and a light q-tile on two workgroups, one pass): pytest -m gpu (the new
# pair tests first), A/B against the halves layout (abx/nopairs.so, FA_SPLIT_PAIRS=0) on C4's 8-way share,
# B1 H8 S8192 and B1 H32 S2048 causal prefills, and the C4 share's line through bench.py
set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out/r5k; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pairs or key_split" --timeout 120 --timeout-method thread > $OUT/pytest_pairs.log 2>&1 || { tail -30 $OUT/pytest_pairs.log; exit 1; }
tail -2 $OUT/pytest_pairs.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
NEW=flash_attention_cute_amd/lib/libfa_gfx950.so
for sh in 1,16,4,4096,128,fp16,1 1,8,8,8192,128,fp16,1 1,32,32,2048,128,fp16,1; do
  AB_REPS=11 AB_WS=1 AB_SHAPE=$sh timeout -k 10 300 python scripts/ab_libs.py c4 abx/nopairs.so $NEW > $OUT/ab_$sh.log 2>&1 || { tail -5 $OUT/ab_$sh.log; exit 1; }
  echo "== $sh"; grep -v amdgpu.ids $OUT/ab_$sh.log
done
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --world 8 --rank 0 --steps 100 > $OUT/bench_c4_w8r0.json 2> $OUT/bench_c4_w8r0.err || { tail -5 $OUT/bench_c4_w8r0.err; exit 1; }
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $OUT/bench_c4_w1.json 2> $OUT/bench_c4_w1.err || { tail -5 $OUT/bench_c4_w1.err; exit 1; }
python -c "
import json; a=json.loads(open('$OUT/bench_c4_w8r0.json').read())['value']; b=json.loads(open('$OUT/bench_c4_w1.json').read())['value']
print(f'c4 share 1/8 {a:.1f} vs whole {b:.1f}: {a/b:.3f}')"
