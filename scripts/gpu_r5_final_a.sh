# Round 5, final code, call A: the GPU suite (test measurements under gpurun_out/$TAG/reports), then the
# fp32 profile set without PMC (rocprofv3 kernel-trace stats of the driver's bench command, the driver and
# default bench lines: gpu_prof.sh with SKIP_PMC; the PMC profile's kernel hash is unchanged) and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r5fa}
mkdir -p gpurun_out/$TAG
export TFG_REPORT_DIR=gpurun_out/$TAG/reports
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
unset TFG_REPORT_DIR
SKIP_PMC=1 TAG=$TAG bash scripts/gpu_prof.sh || exit $?
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
exit $rc
