# Round verification on one MI355X: GPU parity suite, smoke, default bench,
# rocprofv3 kernel-trace stats of the bench workload.  Outputs under
# gpurun_out/$TAG/ (TAG defaults to verify).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-verify}
mkdir -p gpurun_out/$TAG
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$TAG/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
[ $rc -eq 0 ] || exit $rc
echo "== bench default"
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench_default.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
echo "== rocprof kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pcie > gpurun_out/$TAG/trace.log 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
