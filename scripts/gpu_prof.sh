# Profiles of HEAD on one MI355X: PMC traffic with the 4-byte-lane calibration
# (scripts/gpu_pmc.sh -> gpurun_out/$TAG/pmc/profile.json, also installed as
# profiles/pmc_8192x8192_fuse96.json on the box so the next bench quotes it),
# rocprofv3 kernel-trace stats of the driver's bench command, and that bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out/$TAG
PMC_TAG=$TAG/pmc PMC_PROFILE=gpurun_out/$TAG/pmc_8192x8192_fuse96.json bash scripts/gpu_pmc.sh || exit $?
cp gpurun_out/$TAG/pmc_8192x8192_fuse96.json profiles/pmc_8192x8192_fuse96.json
echo "== rocprof kernel trace of the driver's bench"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_traced.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/$TAG/bench_traced.log | cut -c1-300
echo "== bench (driver command) with the fresh PMC profile"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver.log 2>&1; rc=$?; echo "bench rc=$rc"
grep -o '"roofline": {[^}]*}[^}]*}' gpurun_out/$TAG/bench_driver.log
exit $rc
