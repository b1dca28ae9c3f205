# Round 4, second session: the fp32 accuracy variants A/B (scripts/gpu_acc_ab.sh),
# the fp64 engine's PMC traffic at its bench shape (4096^2, 192-step launches),
# then the per-workgroup timelines of config 2 and the headline shape.
# Every GPU step has its own time limit; a crash, abort or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4b}
TAG=$tag bash scripts/gpu_acc_ab.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
if [ -z "$NO_PMC" ]; then
  PMC_TAG=${tag}_pmc_f64 PMC_ENGINE=float64 PMC_SHAPE="4096 4096 192" \
    PMC_ARGS="--ny 4096 --nx 4096 --engine float64 --fuse 192 --steps 1152 --warmup 192 --no-cpu-baseline --no-dropin --no-parity" \
    PMC_PROFILE=gpurun_out/${tag}_pmc_4096x4096_fuse192_f64.json bash scripts/gpu_pmc.sh
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --ny 4096 --nx 4096 --engine float64 --no-cpu-baseline --no-dropin \
      > gpurun_out/${tag}_bench_f64.json 2> gpurun_out/${tag}_bench_f64.err
  rc=$?; echo "bench f64 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NO_TIMELINE" ]; then
  TFG_LIB=diag_libs/_tfg_wgt.so timeout -k 10 300 python -u tests/diagnostics/wg_timeline.py gpurun_out/${tag}_wg_timeline.json > gpurun_out/${tag}_wg_timeline.log 2>&1
  echo "timeline rc=$?"; tail -12 gpurun_out/${tag}_wg_timeline.log
fi
