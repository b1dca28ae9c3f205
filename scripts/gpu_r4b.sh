# Round 4, second session: the fp32 accuracy variants A/B (scripts/gpu_acc_ab.sh),
# then the per-workgroup timelines of config 2 and the headline shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4b} bash scripts/gpu_acc_ab.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
TFG_LIB=diag_libs/_tfg_wgt.so timeout -k 10 300 python -u tests/diagnostics/wg_timeline.py gpurun_out/${TAG:-r4b}_wg_timeline.json > gpurun_out/${TAG:-r4b}_wg_timeline.log 2>&1
echo "timeline rc=$?"; tail -12 gpurun_out/${TAG:-r4b}_wg_timeline.log
