# Profiles of HEAD on one MI355X: PMC traffic with the 4-byte-lane calibration
# (scripts/gpu_pmc.sh -> gpurun_out/$TAG/pmc_8192x8192_fuse128.json, also
# installed as profiles/pmc_8192x8192_fuse128.json on the box so the next bench
# quotes it; SKIP_PMC=1 skips it), rocprofv3 kernel-trace stats of the driver's
# bench command with its summary (scripts/trace_summary.py), and that bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_PMC" ]; then
  PMC_TAG=$TAG/pmc PMC_PROFILE=gpurun_out/$TAG/pmc_8192x8192_fuse128.json bash scripts/gpu_pmc.sh || exit $?
  cp gpurun_out/$TAG/pmc_8192x8192_fuse128.json profiles/pmc_8192x8192_fuse128.json
fi
echo "== rocprof kernel trace of the driver's bench"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_traced.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/trace_summary.py gpurun_out/$TAG/trace gpurun_out/$TAG/bench_traced.log gpurun_out/$TAG/trace_summary.json
echo "== bench (driver command)"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver.log 2>&1; rc=$?; echo "bench rc=$rc"
grep '^{' gpurun_out/$TAG/bench_driver.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
echo "== bench (no flags)"
timeout -k 10 600 python3 bench.py > gpurun_out/$TAG/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"
grep '^{' gpurun_out/$TAG/bench_default.log | cut -c1-300
exit $rc
