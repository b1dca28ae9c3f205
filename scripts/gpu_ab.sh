set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in ${AB_LIBS:-build_variants/*.so}; do
  TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --ny 8192 --nx 8192 --steps 120 --no-cpu-baseline $BENCH_EXTRA > gpurun_out/ab.log 2>&1 || { echo "$lib bench fail"; tail -3 gpurun_out/ab.log; continue; }
  python -c "import json; r=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$lib', 'value=%.3e'%r['value'], 'frac=%.3f'%r['roofline']['frac'], 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
done
