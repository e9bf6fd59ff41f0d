set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4c
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/r4c/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r4c/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/experiments/zigzag_ab.py > gpurun_out/r4c/zigzag_ab.log 2>&1; rc=$?
cat gpurun_out/r4c/zigzag_ab.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
# in-kernel stamps of C4's 8-way share, plain and zigzag blocks (per-block cycle spread, tiles)
for z in 0 1; do
  STAMPS_SHAPE=1,16,4,4096,1,fp16 STAMPS_ZIGZAG=$z FA_STAMPS_LIB=ab/stamps_r4.so timeout -k 10 120 python scripts/stamps.py c4 > gpurun_out/r4c/stamps_c4share_z$z.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/r4c/stamps_c4share_z$z.log | head -14
done
