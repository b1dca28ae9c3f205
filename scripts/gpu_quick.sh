set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/gpu_tests.log
for cfg in "--ny 8192 --nx 8192 --steps 120"; do
  timeout -k 10 300 python bench.py $cfg --no-cpu-baseline $BENCH_EXTRA > gpurun_out/q.log 2>&1 || { echo "bench fail"; tail -5 gpurun_out/q.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('gpurun_out/q.log').read().strip().splitlines()[-1]); print('$cfg', 'value=%.3e'%r['value'], 'frac=%.3f'%r['roofline']['frac'], 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
done
