# Throughput vs launch grid size (TFG_BLOCKS), same binary, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in ${BLOCKS:-1024 2048 4096 8192 16384 2048}; do
  TFG_BLOCKS=$b timeout -k 10 300 python bench.py --steps 288 --no-cpu-baseline --no-pcie > gpurun_out/blk.log 2>&1 || { tail -3 gpurun_out/blk.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/blk.log').read().strip().splitlines()[-1]); print('blocks $b', '%.3e'%r['value'], 'ms/launch %.2f'%r['roofline']['kernel_ms_per_launch'])"
done
