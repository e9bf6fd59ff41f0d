set -o pipefail
# GPU box only: it copies ab/<lib>.so over the box copy of the product library between passes (gpurun snapshots are discarded).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/icache; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
for lib in adead base; do
  cp $R/ab/$lib.so $R/flash_attention_cute_amd/lib/libfa_gfx950.so
  for cfg in c4 c2; do
    for CTR in SQC_ICACHE_MISSES SQC_ICACHE_HITS; do
      timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $OUT/${lib}_${cfg}_$CTR -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --config $cfg > $OUT/${lib}_${cfg}_$CTR.log 2>&1 || { echo "fail $lib $cfg $CTR"; exit 1; }
    done
  done
done
