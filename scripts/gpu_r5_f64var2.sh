# Round 5: two fp64-engine variants (LIB_A, LIB_B; diag_libs builds), same-box A/B at 4096^2, then the fp64
# engine's fixture tests on LIB_B (TFG_LIB), test measurements under gpurun_out/$TAG_reports.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5f64w}_ab REPS=${REPS:-2} BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" \
  LIBS="$LIB_A $LIB_B" bash scripts/gpu_r5_ab.sh || exit $?
export TFG_LIB=$PWD/$LIB_B TFG_REPORT_DIR=gpurun_out/${TAG:-r5f64w}_reports
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fp64_engine_vs_reference_fixtures or one_cell or fp64_synthetic or float64" > gpurun_out/${TAG:-r5f64w}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG:-r5f64w}_tests.log
exit $rc
