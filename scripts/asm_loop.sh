#!/bin/bash
# Dump the main-loop instruction mix of one kernel instantiation (host-side, no GPU).
# usage: scripts/asm_loop.sh [mangled-kernel-regex] [source]
K=${1:-_ZN2fa9fa_fwd_w4INS_3F16ELb0ELi128ELb1EEEv13fa_fwd_paramsii}
SRC=${2:-/root/repo/flash_attention_cute_amd/csrc/fa_fwd_gfx950.hip}
D=/root/repo/build/asm; mkdir -p $D; cd $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -include stdarg.h -I/root/repo/include \
  ${FLAGS:--ffinite-math-only -fno-signed-zeros -mcode-object-version=5} $SRC -o $D/x.so -save-temps 2>&1 | grep -iE "error|warning: (?!.*clobber)" | head
S=$D/$(basename $SRC .hip)-hip-amdgcn-amd-amdhsa-gfx950.s
awk -v k="$K" '$0 ~ "^"k":" {p=1} p {print} p && /s_endpgm/ {exit}' $S > $D/kernel.s
awk '/Inner Loop Header/{p=1} p' $D/kernel.s | awk 'NR>1 && /Inner Loop Header|^\.LBB[0-9_]+:.*crit_edge/{exit} {print}' > $D/loop.s
echo "kernel lines: $(wc -l < $D/kernel.s)  loop lines: $(wc -l < $D/loop.s)"
grep -v "^\s*;" $D/loop.s | awk '{print $1}' | grep -v "^\.LBB" | sort | uniq -c | sort -rn | head -${3:-40}
