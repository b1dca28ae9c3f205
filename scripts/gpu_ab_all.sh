# Same-box A/B of two library builds over every timed path: the fp32 bench,
# the fp64 engine (4096^2) with the single-catchment BMI latency, the one-cell
# multi-step kernel, the ice-flow sub-step and the conduction term.
# AB_LIBS="abvar/a.so abvar/b.so"; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== fp32 bench"; bash scripts/gpu_ab_same_box.sh || exit 1
echo "== fp64 engine + BMI latency"; AB_LIBS="$AB_LIBS $AB_LIBS" bash scripts/gpu_ab_exact.sh || exit 1
echo "== one-cell multi-step"; bash scripts/gpu_ab_cellrun.sh || exit 1
echo "== ice flow"; bash scripts/gpu_ab_flow.sh || exit 1
echo "== conduction"
for lib in $AB_LIBS; do
  TFG_LIB=$PWD/$lib timeout -k 10 120 python -u tests/diagnostics/conduction_timing.py 8192 8192 5 96 > gpurun_out/ab/cond.log 2>&1 || { echo "$lib cond fail"; tail -3 gpurun_out/ab/cond.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab/cond.log | cut -c1-300)"
done
