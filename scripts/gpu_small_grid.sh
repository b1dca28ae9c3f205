# Small grids (BASELINE config 2, 1024^2): workgroup-count sweep (TFG_BLOCKS) and
# the 2048^2 point between config 2 and config 3, K = 96.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-small}; mkdir -p $OUT
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  grep '^{' $OUT/$name.log | tail -1 > $OUT/$name.json
  python3 -c "import json; r=json.load(open('$OUT/$name.json')); l=r['launches']; print('$name', '%.2f G/s'%(r['value']/1e9), 'frac %.3f'%r['roofline']['frac'], 'launch ms %.3f..%.3f'%(l['ms_min'], l['ms_max']))"
}
for b in ${BLOCKS:-512 1024 2048 4096}; do
  run b$b TFG_BLOCKS=$b python bench.py --ny 1024 --nx 1024 --fuse 96 --steps 1920 --warmup 96 --no-cpu-baseline
done
run g2048 python bench.py --ny 2048 --nx 2048 --fuse 96 --steps 960 --warmup 96 --no-cpu-baseline
