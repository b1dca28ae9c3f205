# Round 5: the shortwave skipped at flat-dark steps (exact): same-box A/B of the in-tree library against the
# previous build (PREV) for both engines, the GPU suite, and the rank-0 N = 4 tail (must equal the earlier one).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
main=topoflow-glacier_amd/topoflow_glacier/_tfg.so
TAG=r5night_ab32 REPS=2 LIBS="$PREV $main" bash scripts/gpu_r5_ab.sh || exit $?
TAG=r5night_ab64 REPS=2 BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" LIBS="$PREV $main" bash scripts/gpu_r5_ab.sh || exit $?
TAG=r5night SAMPLES="n4" bash scripts/gpu_r5_tail.sh || exit $?
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5night_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5night_tests.log
exit $rc
