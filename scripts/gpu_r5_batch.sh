# Round 5 batch A: fp32 variant A/B, fp64 A/B and the fp64 GPU tests on the newest fp64 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r5ab3 LIBS="diag_libs/_tfg_p0.so diag_libs/_tfg_p35b.so diag_libs/_tfg_p39.so diag_libs/_tfg_p55.so diag_libs/_tfg_p295.so diag_libs/_tfg_p423.so diag_libs/_tfg_p311.so" REPS=2 bash scripts/gpu_r5_ab.sh || exit $?
TAG=r5ab64c LIBS="diag_libs/_tfg_p0.so diag_libs/_tfg_f64d.so diag_libs/_tfg_f64e.so" REPS=2 BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" bash scripts/gpu_r5_ab.sh || exit $?
TFG_LIB=$PWD/diag_libs/_tfg_f64e.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fastmath.py tests/test_power_rewrites.py "tests/test_gpu_parity.py::test_fp64_engine_vs_reference_fixtures" \
  tests/test_gpu_parity.py::test_one_cell_kernels_equal_the_grid_kernel tests/test_gpu_parity.py::test_fp64_synthetic_vs_oracle \
  "tests/test_gpu_parity.py::test_engine_propagates_nan_forcing_like_the_reference" \
  "tests/test_gpu_parity.py::test_fp64_dark_test_on_every_slope_through_whole_days" tests/test_gpu_parity.py::test_full_model_workflow \
  > gpurun_out/r5_f64_tests.log 2>&1; rc=$?; tail -25 gpurun_out/r5_f64_tests.log; exit $rc
