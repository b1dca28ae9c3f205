# The 1024 x 8192 slab (N = 8 shard) at 192- and 384-step launches with the
# plane skew, 2304 timed steps each (12 / 6 launches), alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slab_k
for rep in 1 2 3; do
  for k in 192 384; do
    timeout -k 10 300 python bench.py --ny 1024 --nx 8192 --fuse $k --steps 2304 --warmup 5 --no-cpu-baseline > gpurun_out/slab_k/run.log 2>&1 || { tail -5 gpurun_out/slab_k/run.log; exit 1; }
    python3 -c "import json; r=json.loads([l for l in open('gpurun_out/slab_k/run.log') if l.startswith('{')][-1]); L=r['launches']; print('K=$k', 'G=%.2f'%(r['value']/1e9), 'n', L['count'], 'ms each', L['ms_each'])"
  done
done
