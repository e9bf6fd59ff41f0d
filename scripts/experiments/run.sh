#!/bin/bash
# One parametrised GPU runner for the measurement and A/B sequences of a round. It replaces the
# round-specific r4*/r5*/r6* scripts (each was one fixed mix of the phases below; they are in git
# history: the r4 / r5 ones at c04f5bf, the r6 ones at ea750dc). Every GPU step runs under its own time limit and the first failure
# ends the run (no retries).
#
# usage: bash scripts/experiments/run.sh <tag> <phase> [<phase> ...]      (outputs: gpurun_out/<tag>/)
#   tests                  the whole `pytest -m gpu` suite
#   tests=<expr>           the GPU tests matching `-k <expr>`
#   smoke                  __graft_entry__.smoke()
#   bench                  the driver's default `python bench.py` line (with the CPU baseline)
#   bench=<c1,c2,..>       `bench.py --config <c>` lines (no CPU baseline)
#   shares=<c1,c2,..>      one GPU's share of the 2-, 4- and 8-way strong split next to the whole problem
#   ab=<cfg>[@<B,Hq,Hkv,S,D,dtype,causal>]
#                          same-process interleaved A/B (scripts/ab_libs.py) of $AB_LIBS, a space-separated
#                          list of lib.so[@variant] (default: the product library), on cfg or the given
#                          shape; AB_WS, AB_REPS, AB_ITERS pass through
#   profile=<c1,c2,..>     rocprofv3 kernel trace + stats and the PMC passes of scripts/profile.sh
#   shapepmc=<c1,c2,..>    per MFMA-shape body (debug library m32 / m16) and the product: one PMC pass
#                          (clock, VALU / MFMA; scripts/experiments/shape_pmc_summary.py)
# e.g. the round-6 records:
#   run.sh r6_split_ab ab=c4@1,16,4,4096,128,fp16,1 ab=c4@1,8,8,4096,128,fp16,1 ab=c4 ab=c2
#        (AB_WS=1 AB_LIBS="ab6/r5head.so flash_attention_cute_amd/lib/libfa_gfx950.so")
#   run.sh r6s2 tests=m16\ or\ m32\ or\ shape_bodies ab=c2 ab=c3 ab=c4 ab=c5@8,32,8,4096,128,bf16,1 shapepmc=c2,c4
#        (AB_WS=1 AB_LIBS="<product> <debug>@m32 <debug>@m16")
set -o pipefail
TAG=${1:?tag}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
PROD=flash_attention_cute_amd/lib/libfa_gfx950.so DBG=flash_attention_cute_amd/lib/libfa_gfx950_debug.so
fail() { echo "run.sh: $1 failed"; tail -20 "$2"; exit 1; }
for ph in "$@"; do
  arg=${ph#*=}; [ "$arg" = "$ph" ] && arg=""
  name=${ph%%=*}
  echo "== $ph $(date +%T)"
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread "${k[@]}" \
        > "$OUT/pytest_gpu.log" 2>&1 || fail tests "$OUT/pytest_gpu.log"
      tail -1 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail smoke "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      if [ -z "$arg" ]; then
        timeout -k 10 300 python bench.py > "$OUT/default_bench.json" 2> "$OUT/default_bench.err" || fail bench "$OUT/default_bench.err"
        cut -c1-300 "$OUT/default_bench.json"
      else
        for c in ${arg//,/ }; do
          timeout -k 10 300 python bench.py --config "$c" --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" \
            || fail "bench $c" "$OUT/bench_$c.err"
          cut -c1-300 "$OUT/bench_$c.json"
        done
      fi ;;
    shares)
      for c in ${arg//,/ }; do
        timeout -k 10 300 python bench.py --config "$c" --no-cpu-baseline > "$OUT/bench_${c}_w1.json" 2> "$OUT/bench_${c}_w1.err" \
          || fail "share $c" "$OUT/bench_${c}_w1.err"
        for w in 2 4 8; do
          timeout -k 10 300 python bench.py --config "$c" --no-cpu-baseline --world $w --rank 0 --steps 100 \
            > "$OUT/bench_${c}_w${w}r0.json" 2> "$OUT/bench_${c}_w${w}r0.err" || fail "share $c/$w" "$OUT/bench_${c}_w${w}r0.err"
        done
        python - "$OUT" "$c" <<'PY'
import json, sys
out, c = sys.argv[1], sys.argv[2]
w1 = json.loads(open(f"{out}/bench_{c}_w1.json").read())["value"]
for w in (2, 4, 8):
    v = json.loads(open(f"{out}/bench_{c}_w{w}r0.json").read())["value"]
    print(f"{c} share 1/{w}: {v:.1f} TFLOPS vs whole {w1:.1f}: {v / w1:.3f}")
PY
      done ;;
    ab)
      cfg=${arg%%@*}; shape=""; [ "$cfg" != "$arg" ] && shape=${arg#*@}
      log="$OUT/ab_${cfg}${shape:+_${shape//,/_}}.log"
      AB_SHAPE=$shape timeout -k 10 300 python scripts/ab_libs.py "$cfg" ${AB_LIBS:-$PROD} > "$log" 2>&1 || fail "ab $arg" "$log"
      grep -v amdgpu.ids "$log" ;;
    profile)
      bash scripts/experiments/profile_all.sh "$TAG" "${arg//,/ }" 2>&1 | cut -c1-200 || exit 1 ;;
    shapepmc)
      for c in ${arg//,/ }; do
        for v in m32 m16 w4; do
          lib=$DBG@$v; [ $v = w4 ] && lib=$PROD
          FA_GFX950_VARIANT=$([ $v = w4 ] || echo $v) AB_REPS=2 AB_ITERS=10 timeout -s KILL 120 rocprofv3 \
            --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
            -d "$OUT/pmc_${v}_$c" -o run --output-format csv -- python3 scripts/ab_libs.py "$c" "$lib" \
            > "$OUT/pmc_${v}_$c.log" 2>&1 || fail "shapepmc $v $c" "$OUT/pmc_${v}_$c.log"
        done
      done
      python3 scripts/experiments/shape_pmc_summary.py $(ls -d "$OUT"/pmc_*/) | cut -c1-220 ;;
    *) echo "run.sh: unknown phase $ph"; exit 2 ;;
  esac
done
