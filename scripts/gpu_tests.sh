set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/gpu_tests.log
exit $rc
