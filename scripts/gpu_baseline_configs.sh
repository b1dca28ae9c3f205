# Every BASELINE.json GPU config in its per-GPU form, one box, one JSON line each
# (gpurun_out/configs/<name>.json).  Config 4/5 at N>1 are the driver's runs;
# here config 5 runs its per-rank slab (16384^2 / 8 GPUs = 2048 x 16384 rows).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/configs; mkdir -p $OUT
run() { name=$1; shift
  timeout -k 10 600 python bench.py "$@" > $OUT/$name.log 2>&1 || { echo "$name FAILED"; tail -5 $OUT/$name.log; return 1; }
  grep '^{' $OUT/$name.log | tail -1 > $OUT/$name.json
  python3 -c "import json; r=json.load(open('$OUT/$name.json')); print('$name', '%.2f G cell-updates/s'%(r['value']/1e9), '%.0f GB/s'%r['roofline']['achieved'], 'frac %.3f'%r['roofline']['frac'], 'ms/launch %.2f'%r['roofline']['kernel_ms_per_launch'])"; }
run cfg2_1024sq_year      --ny 1024 --nx 1024 --steps 8760 --warmup 120 --fuse 120 --no-pcie &&
run cfg3_4096sq           --ny 4096 --nx 4096 --steps 480 --no-pcie &&
run cfg4_8192sq_per_gpu   --ny 8192 --nx 8192 --steps 480 --no-pcie --no-cpu-baseline &&
run cfg5_slab_2048x16384_dt025_43catch --ny 2048 --nx 16384 --dt 0.25 --catchments 43 --steps 480 --no-pcie --no-cpu-baseline
