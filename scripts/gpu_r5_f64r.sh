# Round 5, fp64 engine: one reciprocal of T_K for the pressure exponent and em_air's argument, the
# stability correction with one quotient, the Halley correction by a one-Newton reciprocal.  Same-box A/B
# against the previous build (diag_libs/_tfg_q.so) at 4096^2, then the fp64 parity tests on the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5r}
LIBS="diag_libs/_tfg_q.so topoflow-glacier_amd/topoflow_glacier/_tfg.so" TAG=${TAG}_ab REPS=${REPS:-3} \
  BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" bash scripts/gpu_r5_ab.sh || exit $?
TFG_REPORT_DIR=gpurun_out/$TAG/reports timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_power_rewrites.py tests/test_fastmath.py -m gpu \
  -k "fp64 or one_cell or satterlund or power_rewrites or fastmath or bmi or nan or checkpoint" \
  > gpurun_out/${TAG}_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/${TAG}_parity.log; exit $rc
