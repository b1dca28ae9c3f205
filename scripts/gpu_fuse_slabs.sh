# Launch depth K (steps fused per launch) for the per-rank slabs of config 4's
# strong scaling (8192/N rows x 8192): each slab at several K on one GPU.
# Smaller slabs lose the launch's state-in / state-out phases to less step
# traffic; a deeper launch amortises them (footprint kept <= ~160 GB).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-fuse_slabs}; mkdir -p $OUT
for spec in "8192 96" "4096 96" "4096 192" "2048 96" "2048 192" "2048 384" "1024 96" "1024 192" "1024 384" "1024 768"; do
  set -- $spec
  rows=$1; k=$2
  timeout -k 10 300 python bench.py --ny $rows --nx 8192 --fuse $k --steps $((3*k)) --warmup $k --no-cpu-baseline > $OUT/r${rows}_k$k.log 2>&1 || { tail -5 $OUT/r${rows}_k$k.log; exit 1; }
  grep '^{' $OUT/r${rows}_k$k.log | tail -1 > $OUT/r${rows}_k$k.json
  python3 -c "import json; r=json.load(open('$OUT/r${rows}_k$k.json')); l=r['launches']; print('$rows rows K=$k', '%.2f G/s'%(r['value']/1e9), 'frac %.3f'%r['roofline']['frac'], 'launch ms %.2f..%.2f'%(l['ms_min'], l['ms_max']))"
done
