set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abcfg
for c in c2 c3 c4 c5; do for sp in 0 1 2; do
  FA_SPLIT=$sp timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/abcfg/${c}_$sp.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/abcfg/${c}_$sp.json')); print('$c split=$sp', d['value'], d['unit'], d['config'].get('workload'))"
done; done
