# Round 5: the fp64 engine's bench line at 4096^2 twice (full line: parity sample and drop-in legs), then a
# same-box A/B against the previous build, to separate box-to-box spread from the build's own speed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5l}
mkdir -p gpurun_out/$TAG
for i in 1 2; do
  timeout -k 10 300 python bench.py --engine float64 --ny 4096 --nx 4096 --no-cpu-baseline > gpurun_out/$TAG/bench_f64_$i.log 2>&1
  rc=$?; echo "bench f64 $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/$TAG/bench_f64_$i.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('G=%.3f' % (r['value']/1e9), 'ms/launch=%.3f' % r['roofline']['kernel_ms_per_launch'])"
done
LIBS="diag_libs/_tfg_q.so topoflow-glacier_amd/topoflow_glacier/_tfg.so" TAG=${TAG}_ab REPS=2 \
  BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" bash scripts/gpu_r5_ab.sh
