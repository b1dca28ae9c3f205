set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2p
for rep in 1 2; do AB_LIBS="abvar/b256.so abvar/pow4.so" bash scripts/gpu_ab_exact.sh || exit 1; done 2>&1 | tee gpurun_out/r2p/ab_exact.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2p/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r2p/gpu_tests.log; exit $rc
