# Round 4, third session: the GPU suite, the driver's bench command (parity now
# read from the bench handle's own first launches), configs 2 and 3 (k_fused
# no longer steps the plane skew), and the per-workgroup timelines again.
# Every GPU step has its own time limit; a crash, abort or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4c}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_gpu_tests.log; stop $rc; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.json 2> gpurun_out/${tag}_bench_driver.err
rc=$?; echo "bench rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -c 1500 gpurun_out/${tag}_bench_driver.err; exit $rc; }
OUT=gpurun_out/${tag}_configs; mkdir -p $OUT
run() { name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $OUT/$name.log 2>&1; rc=$?; stop $rc
  [ $rc -eq 0 ] || { echo "$name FAILED"; tail -5 $OUT/$name.log; return 1; }
  grep '^{' $OUT/$name.log | tail -1 > $OUT/$name.json
  python3 -c "import json; r=json.load(open('$OUT/$name.json')); print('$name', '%.2f G cell-updates/s'%(r['value']/1e9), '%.0f GB/s'%r['roofline']['achieved'], 'frac %.3f'%r['roofline']['frac'], 'ms/launch %.2f'%r['roofline']['kernel_ms_per_launch'], 'parity', (r.get('sample_parity') or {}).get('ok'))"; }
run cfg2_1024sq_year --ny 1024 --nx 1024 --steps 8760 --warmup 120 --fuse 120 --no-cpu-baseline --no-dropin &&
run cfg2_1024sq_auto --ny 1024 --nx 1024 --steps 2304 --no-cpu-baseline --no-dropin &&
run cfg3_4096sq --ny 4096 --nx 4096 --steps 480 --no-cpu-baseline --no-dropin || exit 1
if [ -z "$NO_TIMELINE" ]; then
  TFG_LIB=diag_libs/_tfg_wgt.so timeout -k 10 300 python -u tests/diagnostics/wg_timeline.py gpurun_out/${tag}_wg_timeline.json 1024,1024,120 2048,2048,384 > gpurun_out/${tag}_wg_timeline.log 2>&1
  rc=$?; echo "timeline rc=$rc"; stop $rc; grep -v Warn gpurun_out/${tag}_wg_timeline.log | cut -c1-400 | tail -6
fi
