# The driver's bench command on the per-rank shard of each strong-scaling N
# (8192/N rows x 8192, the automatic launch depth), one process each, one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/strong_shapes; mkdir -p $OUT
for rows in 8192 4096 2048 1024; do
  timeout -k 10 300 python bench.py --ny $rows --nx 8192 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/r$rows.log 2>&1 || { tail -5 $OUT/r$rows.log; exit 1; }
  grep '^{' $OUT/r$rows.log | tail -1 > $OUT/r$rows.json
  python3 -c "import json; r=json.load(open('$OUT/r$rows.json')); L=r['launches']; print('$rows rows', 'K=%d'%L['steps_each'], 'n=%d'%L['count'], 'G=%.2f'%(r['value']/1e9), 'frac %.3f'%r['roofline']['frac'], 'first/min/mean ms %.2f/%.2f/%.2f'%(L['ms_each'][0], L['ms_min'], L['ms_mean']))"
done
