# Default bench (the driver's command) + rocprofv3 kernel-trace stats of the same workload.
# PROF_TAG names the output directories (gpurun_out/<tag>/...).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${PROF_TAG:-prof}
mkdir -p gpurun_out/$TAG
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/$TAG/smoke.log
[ $rc -eq 0 ] || exit $rc
echo "== bench default"
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench_default.log
[ $rc -eq 0 ] || exit $rc
echo "== rocprof kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pcie > gpurun_out/$TAG/trace.log 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
