# BASELINE config 2 (1024^2, a year of hourly steps) at several launch depths K.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-config2}; mkdir -p $OUT
for k in 96 120 240 480 960 1920; do
  timeout -k 10 300 python bench.py --ny 1024 --nx 1024 --fuse $k --steps 8760 --warmup $k --no-cpu-baseline > $OUT/k$k.log 2>&1 || { tail -5 $OUT/k$k.log; exit 1; }
  grep '^{' $OUT/k$k.log | tail -1 > $OUT/k$k.json
  python3 -c "import json; r=json.load(open('$OUT/k$k.json')); l=r['launches']; print('1024^2 K=$k', r['steps'], 'steps', '%.2f G/s'%(r['value']/1e9), 'frac %.3f'%r['roofline']['frac'], 'launch ms %.3f..%.3f'%(l['ms_min'], l['ms_max']))"
done
