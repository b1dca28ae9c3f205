# Round 5: the fp32 profile set of the in-tree library (gpu_prof.sh: PMC traffic with calibration,
# rocprofv3 kernel-trace stats of the driver's bench command, the driver and default bench lines),
# smoke(), then the ablation A/Bs (gpu_r5_ablate.sh: F64LIBS, F32LIBS) when given.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r5prof}
mkdir -p gpurun_out/$TAG
TAG=$TAG bash scripts/gpu_prof.sh || exit $?
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
[ $rc -eq 0 ] || exit $rc
[ -z "$F64LIBS$F32LIBS" ] || TAG=${TAG}_abl bash scripts/gpu_r5_ablate.sh
