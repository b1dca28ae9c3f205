# Round 5: an fp64-engine variant (LIB, a diag_libs build of the working tree): same-box A/B against the
# in-tree library at 4096^2, then the GPU tests that exercise the fp64 engine, run on the variant (TFG_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5f64v}_ab REPS=${REPS:-2} BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" \
  LIBS="topoflow-glacier_amd/topoflow_glacier/_tfg.so $LIB" bash scripts/gpu_r5_ab.sh || exit $?
export TFG_LIB=$PWD/$LIB TFG_REPORT_DIR=gpurun_out/${TAG:-r5f64v}_reports
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fp64 or float64 or fastmath or one_cell or power or workflow or bmi or update or checkpoint or catchment or quarter or satterlund or dark" \
  > gpurun_out/${TAG:-r5f64v}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG:-r5f64v}_tests.log
exit $rc
