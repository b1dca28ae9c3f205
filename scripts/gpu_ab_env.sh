# A/B of (library, TFG_BLOCKS) pairs: AB_CASES="lib:blocks lib:blocks ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in $AB_CASES; do
  lib=${c%%:*}; blk=${c##*:}
  TFG_LIB=$PWD/$lib TFG_BLOCKS=$blk timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie $BENCH_EXTRA > gpurun_out/ab.log 2>&1 || { echo "$c fail"; tail -3 gpurun_out/ab.log; continue; }
  python -c "import json; r=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$c', 'value=%.4e'%r['value'], 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
done
