#!/bin/bash
# scripts/benchmark_kernel.py over the reference's default config and the BASELINE configs
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { timeout -k 10 300 python scripts/benchmark_kernel.py "$@" 2>&1 | grep -v amdgpu.ids; }
{ run --iter 100 &&
  run --batch-size 4 --num-heads-q 32 --num-heads-kv 32 --seqlen-q 4096 --seqlen-kv 4096 --iter 50 &&
  run --batch-size 4 --num-heads-q 32 --num-heads-kv 32 --seqlen-q 8192 --seqlen-kv 8192 --dtype bfloat16 --causal --iter 20 &&
  run --batch-size 4 --num-heads-q 32 --num-heads-kv 8 --seqlen-q 4096 --seqlen-kv 4096 --causal --iter 50 &&
  run --batch-size 1 --num-heads-q 32 --num-heads-kv 8 --seqlen-q 4096 --seqlen-kv 4096 --dtype bfloat16 --causal --iter 50
} | tee gpurun_out/kernel_bench.log
