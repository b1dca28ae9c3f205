set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"
tail -60 gpurun_out/gpu_tests.log
