# Round 5, final fp64 code: the GPU suite (measurements under gpurun_out/$TAG/reports), the fp64 PMC profile,
# bench line and the issue counters of both engines (gpu_r5_final_b.sh without the rank samples), smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r5fc}
mkdir -p gpurun_out/$TAG
TFG_REPORT_DIR=gpurun_out/$TAG/reports timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
NO_RANKS=1 TAG=$TAG bash scripts/gpu_r5_final_b.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
exit $rc
