# Round verification on one MI355X: GPU parity suite, smoke, the bench as the
# driver runs it (--steps 20 --warmup 5) and with its defaults.  Outputs under
# gpurun_out/$TAG/ (TAG defaults to verify); test measurements (TFG_REPORT_DIR)
# under gpurun_out/$TAG/reports/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-verify}
mkdir -p gpurun_out/$TAG
export TFG_REPORT_DIR=gpurun_out/$TAG/reports
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$TAG/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
[ $rc -eq 0 ] || exit $rc
echo "== bench as the driver runs it"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/$TAG/bench_driver.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
echo "== bench default"
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/$TAG/bench_default.log | cut -c1-400
exit $rc
