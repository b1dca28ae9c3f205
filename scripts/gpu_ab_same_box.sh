# Same-box A/B of library variants (abvar/*.so), alternating A B A B:
# default bench workload without the CPU legs; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > gpurun_out/ab/run.log 2>&1 || { echo "$lib bench fail"; tail -3 gpurun_out/ab/run.log; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/ab/run.log').read().strip().splitlines()[-1]); print('$lib', 'value=%.4e'%r['value'], 'ms/launch=%.2f'%r['roofline']['kernel_ms_per_launch'])"
  done
done
