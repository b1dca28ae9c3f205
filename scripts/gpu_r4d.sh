# Round 4, fourth session: the plane-skew A/B (scripts/gpu_ab_skew.sh), config 2
# at its automatic 384-step depth (parity of a 384-step launch, progress on
# stderr), and the per-workgroup timelines with the skew no longer stepped.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4d}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
TAG=${tag}_skew bash scripts/gpu_ab_skew.sh; rc=$?; stop $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --ny 1024 --nx 1024 --steps 2304 --no-cpu-baseline --no-dropin \
    > gpurun_out/${tag}_cfg2_auto.json 2> gpurun_out/${tag}_cfg2_auto.err
rc=$?; echo "cfg2 auto rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_cfg2_auto.err; exit $rc; }
timeout -k 10 400 python -u bench.py --ny 4096 --nx 4096 --steps 2304 --no-cpu-baseline --no-dropin \
    > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
rc=$?; echo "cfg3 rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_cfg3.err; exit $rc; }
TFG_LIB=diag_libs/_tfg_wgt.so timeout -k 10 300 python -u tests/diagnostics/wg_timeline.py gpurun_out/${tag}_wg_timeline.json 1024,1024,120 2048,2048,384 > gpurun_out/${tag}_wg_timeline.log 2>&1
rc=$?; echo "timeline rc=$rc"; grep -v Warn gpurun_out/${tag}_wg_timeline.log | cut -c1-300 | tail -6
