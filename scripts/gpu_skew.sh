# Plane-stride skew A/B: bare streaming mix (tools/hbm_mix) and k_fused (bench) with
# plane strides of n + skew cells (n = 8192^2 = 2^26: power-of-two strides at skew 0).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/skew; mkdir -p $OUT
for sk in 0 256 4096; do
  timeout -k 10 120 tools/hbm_mix 67108864 24 32768 $sk > $OUT/mix_$sk.json 2>&1 || exit $?
  echo "mix skew=$sk"; head -2 $OUT/mix_$sk.json
done
for sk in 0 256 4096 0 256 4096; do
  TFG_PLANE_SKEW=$sk timeout -k 10 300 python bench.py --steps 288 --warmup 96 --no-cpu-baseline --no-pcie > $OUT/bench_$sk.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$sk.log').read().strip().splitlines()[-1]); print('bench skew=$sk', round(d['value']/1e9,2), 'G/s', round(d['roofline']['achieved']), 'GB/s')"
done
