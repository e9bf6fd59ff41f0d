#!/bin/bash
# Dump the main-loop instruction mix of one kernel instantiation (host-side, no GPU).
# usage: scripts/dev/asm_loop.sh [DT] [CAUSAL] [D] [EXACT] [kernel-name-regex] [top-N]
DT=${1:-F16}; C=${2:-0}; DD=${3:-128}; E=${4:-1}
K=${5:-_ZN2fa9fa_fwd_w4}
D=/root/repo/build/asm; mkdir -p $D; cd $D
CS=/root/repo/flash_attention_cute_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I/root/repo/include -I$CS \
  -DFA_INST_DT=$DT -DFA_INST_CAUSAL=$C -DFA_INST_D=$DD -DFA_INST_EXACT=$E \
  ${FLAGS:--ffinite-math-only -fno-signed-zeros -mcode-object-version=5} $CS/fa_inst.hip -o $D/x.o -save-temps 2>&1 | grep -iE "error" | head
S=$D/fa_inst-hip-amdgcn-amd-amdhsa-gfx950.s
awk -v k="$K" '$0 ~ "^"k"[^ ]*: " {p=1} p {print} p && /s_endpgm/ {exit}' $S > $D/kernel.s
awk '/Inner Loop Header/{p=1} p' $D/kernel.s | awk 'NR>1 && /Inner Loop Header|^\.LBB[0-9_]+:.*crit_edge/{exit} {print}' > $D/loop.s
echo "kernel lines: $(wc -l < $D/kernel.s)  loop lines: $(wc -l < $D/loop.s)"
grep -v "^\s*;" $D/loop.s | awk '{print $1}' | grep -v "^\.LBB" | sort | uniq -c | sort -rn | head -${6:-40}
