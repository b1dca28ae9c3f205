# fp64-engine A/B over library variants: bulk throughput (4096^2, K=96) and single-catchment BMI latency.
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in ${AB_LIBS:-build_variants/*.so}; do
  TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --engine float64 --ny 4096 --nx 4096 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/abx.log 2>&1 || { echo "$lib bench fail"; tail -3 gpurun_out/abx.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/abx.log').read().strip().splitlines()[-1]); print('$lib', 'value=%.3e'%r['value'], 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
  TFG_LIB=$PWD/$lib timeout -k 10 120 python tests/diagnostics/bmi_latency.py 2>&1 | tail -2 || exit 1
done
