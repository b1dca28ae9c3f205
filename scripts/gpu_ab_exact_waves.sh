cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for v in base exact3; do
    if [ $v = base ]; then unset TFG_LIB; else export TFG_LIB=$PWD/tools/abvar/exact3.so; fi
    timeout -k 10 200 python bench.py --engine float64 --ny 4096 --nx 4096 --steps 48 --warmup 24 --fuse 24 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]); print('$v', round(d['value']/1e9,2), round(d['launches']['ms_mean'],2))"
  done
done
