# Round 6, final code: PART=a -- the GPU suite (test measurements under gpurun_out/$TAG/reports) and
# smoke().  PART=p -- the fp32 PMC traffic profile (installed as profiles/pmc_8192x8192_fuse128.json for
# the bench to quote), rocprofv3 kernel-trace stats of the driver's bench command and the driver / no-flag
# bench lines (scripts/gpu_prof.sh).  PART=b -- the fp64 engine's PMC profile and bench line, the issue counters of
# both engines and the fp64-flux form, the fp64-flux bench line (with its parity check).  PART=c -- every
# BASELINE configuration's line (scripts/gpu_baseline_configs.sh) and the N > 1 rehearsal on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r6f${PART}}
mkdir -p gpurun_out/$TAG
if [ "$PART" = a ]; then
  export TFG_REPORT_DIR=gpurun_out/$TAG/reports
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$TAG/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  unset TFG_REPORT_DIR
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
  exit $rc
fi
if [ "$PART" = p ]; then
  TAG=$TAG bash scripts/gpu_prof.sh
  exit $?
fi
if [ "$PART" = c ]; then
  echo "== configurations"
  bash scripts/gpu_baseline_configs.sh
  rc=$?; [ $rc -eq 0 ] || exit $rc
  echo "== N > 1 rehearsal (gloo, every rank on cuda:0)"
  TAG=$TAG/reh bash scripts/gpu_rehearse.sh
  exit $?
fi
# the fp64-flux form's PMC traffic (round 6: its bench line quotes it)
PMC_TAG=$TAG/pmcflux PMC_ENGINE=float32_flux64 \
  PMC_ARGS="--flux fp64 --ny 8192 --nx 8192 --fuse 128 --steps 768 --warmup 128 --no-cpu-baseline --no-dropin --no-parity" \
  PMC_PROFILE=gpurun_out/$TAG/pmc_8192x8192_fuse128_fluxf64.json bash scripts/gpu_pmc.sh || exit $?
cp gpurun_out/$TAG/pmc_8192x8192_fuse128_fluxf64.json profiles/pmc_8192x8192_fuse128_fluxf64.json
[ -n "$SKIP_F64PMC" ] || PMC_TAG=$TAG/pmc64 PMC_ENGINE=float64 PMC_SHAPE="4096 4096 192" \
  PMC_ARGS="--engine float64 --ny 4096 --nx 4096 --fuse 192 --steps 768 --warmup 192 --no-cpu-baseline --no-dropin --no-parity" \
  PMC_PROFILE=gpurun_out/$TAG/pmc_4096x4096_fuse192_f64.json bash scripts/gpu_pmc.sh || exit $?
[ -n "$SKIP_F64PMC" ] || cp gpurun_out/$TAG/pmc_4096x4096_fuse192_f64.json profiles/pmc_4096x4096_fuse192_f64.json
echo "== fp64 bench"
timeout -k 10 300 python bench.py --engine float64 --ny 4096 --nx 4096 --no-cpu-baseline > gpurun_out/$TAG/bench_f64.log 2>&1
rc=$?; echo "bench f64 rc=$rc"; grep '^{' gpurun_out/$TAG/bench_f64.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
echo "== fp64-flux bench (with its parity check)"
timeout -k 10 300 python bench.py --flux fp64 --no-cpu-baseline --no-dropin > gpurun_out/$TAG/bench_flux_f64.log 2>&1
rc=$?; echo "bench flux f64 rc=$rc"; grep '^{' gpurun_out/$TAG/bench_flux_f64.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
echo "== issue counters"
TAG=$TAG/issue bash scripts/gpu_pmc_issue.sh > gpurun_out/$TAG/issue.log 2>&1 || { tail -5 gpurun_out/$TAG/issue.log; exit 1; }
grep -c pass gpurun_out/$TAG/issue.log
exit 0
