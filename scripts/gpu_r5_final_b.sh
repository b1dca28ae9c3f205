# Round 5, final code, call B: the fp64 engine's PMC traffic profile at 4096^2 (192-step launches, 4 / 8 /
# 16 B lane calibrations), its bench line, the issue counters of both engines at the bench shapes, then the
# other ranks' parity samples of the strong-scaling lines (gpu_r5_ranks.sh) unless NO_RANKS is set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r5fb}
mkdir -p gpurun_out/$TAG
PMC_TAG=$TAG/pmc64 PMC_ENGINE=float64 PMC_SHAPE="4096 4096 192" \
  PMC_ARGS="--engine float64 --ny 4096 --nx 4096 --fuse 192 --steps 768 --warmup 192 --no-cpu-baseline --no-dropin --no-parity" \
  PMC_PROFILE=gpurun_out/$TAG/pmc_4096x4096_fuse192_f64.json bash scripts/gpu_pmc.sh || exit $?
cp gpurun_out/$TAG/pmc_4096x4096_fuse192_f64.json profiles/pmc_4096x4096_fuse192_f64.json
echo "== fp64 bench"
timeout -k 10 300 python bench.py --engine float64 --ny 4096 --nx 4096 --no-cpu-baseline > gpurun_out/$TAG/bench_f64.log 2>&1
rc=$?; echo "bench f64 rc=$rc"; grep '^{' gpurun_out/$TAG/bench_f64.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
echo "== issue counters"
TAG=$TAG/issue bash scripts/gpu_pmc_issue.sh > gpurun_out/$TAG/issue.log 2>&1 || { tail -5 gpurun_out/$TAG/issue.log; exit 1; }
grep -c pass gpurun_out/$TAG/issue.log
[ -n "$NO_RANKS" ] || TAG=$TAG/rank bash scripts/gpu_r5_ranks.sh
