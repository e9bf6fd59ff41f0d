#!/bin/bash
# Build libfa_gfx950.so from a source tree (e.g. a git archive of an older commit) for A/B runs.
# usage: scripts/experiments/build_lib_from.sh <src-root-with-include-and-csrc> <out.so>
set -e
SRC=$1; OUT=$2; T=$(mktemp -d)
CS=$SRC/flash_attention_cute_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -ffinite-math-only -fno-signed-zeros -Wno-inline-asm ${EXTRA_DEFS:-}"
for dt in F16 BF16; do for c in 0 1; do for d in 64 128; do for e in 0 1; do
  /opt/rocm/bin/hipcc $F -I$SRC/include -I$CS -DFA_INST_DT=$dt -DFA_INST_CAUSAL=$c -DFA_INST_D=$d -DFA_INST_EXACT=$e \
    -c $CS/fa_inst.hip -o $T/i_${dt}_${c}_${d}_${e}.o &
done; done; done; done
/opt/rocm/bin/hipcc $F -I$SRC/include -I$CS -c $CS/fa_fwd_gfx950.hip -o $T/disp.o &
[ -f $CS/fa_rope.hip ] && /opt/rocm/bin/hipcc $F -I$SRC/include -I$CS -c $CS/fa_rope.hip -o $T/rope.o &
wait
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/*.o -o $OUT
rm -rf $T
