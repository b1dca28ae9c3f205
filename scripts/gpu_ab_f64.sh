# Same-box A/B of the fp64 engine over library variants (abvar/*.so),
# alternating A B A B: bulk throughput at 4096^2 (192-step launches) and the
# single-catchment BMI latency.  Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_f64
for rep in 1 2; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --engine float64 --ny 4096 --nx 4096 --steps 192 --no-cpu-baseline > gpurun_out/ab_f64/run.log 2>&1 || { echo "$lib bench fail"; tail -3 gpurun_out/ab_f64/run.log; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/ab_f64/run.log').read().strip().splitlines()[-1]); print('$lib', 'G cell-updates/s=%.2f'%(r['value']/1e9), 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
    TFG_LIB=$PWD/$lib timeout -k 10 120 python tests/diagnostics/bmi_latency.py 2>&1 | tail -1 || exit 1
  done
done
