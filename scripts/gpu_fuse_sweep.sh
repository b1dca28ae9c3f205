# Throughput vs steps fused per launch (same binary, same box).
set -o pipefail
cd $GRAFT_REPO_ROOT
for f in ${FUSES:-24 48 96 24}; do
  timeout -k 10 300 python bench.py --fuse $f --steps $((f * 5)) --warmup $f --no-cpu-baseline --no-pcie > gpurun_out/fuse_$f.log 2>&1 || { echo "fuse $f failed"; tail -3 gpurun_out/fuse_$f.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/fuse_$f.log').read().strip().splitlines()[-1]); print('fuse $f', 'value=%.3e'%r['value'], 'GB/s=%.0f'%r['roofline']['achieved'], 'B/cu=%.2f'%r['roofline']['bytes_per_cell_update'], 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
done
