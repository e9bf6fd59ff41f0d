#!/bin/bash
# LLM harness on the GPU box: Llama-3-8B / Qwen2-7B shapes, random weights, patched vs HF sdpa.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for m in llama3-8b qwen2-7b; do
  for a in custom sdpa; do
    timeout -k 10 300 python scripts/benchmark_llm.py --model $m --attn $a --prompt-len ${PLEN:-4096} --max-new-tokens 32 --num-trials 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/llm_${m}_${a}.log || exit 1
  done
done
