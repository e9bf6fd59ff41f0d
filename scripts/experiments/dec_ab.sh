set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for f in 0 1; do for t in 256 512 1024; do
 echo "flags=$f target=$t"
 FA_DEC_FLAGS=$f FA_DEC_TARGET_WGS=$t timeout -k 10 120 python bench.py --config decode --no-cpu-baseline 2>&1 | grep -o '"roofline": {[^}]*}' || exit 1
done; done
for f in 0 1; do
 echo "long flags=$f"
 FA_DEC_FLAGS=$f timeout -k 10 120 python bench.py --config decode_long --no-cpu-baseline 2>&1 | grep -o '"roofline": {[^}]*}' || exit 1
done
