set -o pipefail
cd $GRAFT_REPO_ROOT
for b in ${BLOCKS:-2048 4096 8192 16384 32768}; do
  TFG_BLOCKS=$b timeout -k 10 300 python bench.py --catchments ${CATCH:-43} --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/blk.log 2>&1 || { tail -3 gpurun_out/blk.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/blk.log').read().strip().splitlines()[-1]); print('catch ${CATCH:-43} blocks $b', '%.3e'%r['value'], 'ms/launch %.2f'%r['roofline']['kernel_ms_per_launch'])"
done
