# The round's profile set on one MI355X: PMC traffic + kernel-trace stats + the
# two bench lines (scripts/gpu_prof.sh), smoke, the fp64 engine bench line at
# 4096^2 and the instruction-issue counters of both engines.  TAG names the
# output directory under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-round}
bash scripts/gpu_prof.sh || exit $?
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
[ $rc -eq 0 ] || exit $rc
echo "== fp64 engine bench"
timeout -k 10 300 python bench.py --engine float64 --ny 4096 --nx 4096 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/$TAG/bench_f64.log 2>&1; rc=$?; echo "bench f64 rc=$rc"
grep '^{' gpurun_out/$TAG/bench_f64.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
echo "== issue counters"
TAG=$TAG/issue bash scripts/gpu_pmc_issue.sh
