# The GPU suite (as the driver runs it), then the command given as arguments
# (e.g. an A/B or a study script), stopping at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-tests}
export TFG_REPORT_DIR=gpurun_out/${TAG:-tests}/reports
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG:-tests}/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG:-tests}/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG:-tests}/gpu_tests.log | head -20; exit $rc; }
[ $# -gt 0 ] || exit 0
"$@"
