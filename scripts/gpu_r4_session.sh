# Round-4 verification session: the driver's bench command, the GPU suite,
# then the fp32 term attribution (tests/diagnostics/term_attribution.py).
# Each GPU step has its own time limit; a crash, abort or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4a}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.json 2> gpurun_out/${tag}_bench_driver.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${tag}_bench_driver.err; stop $rc; [ $rc -eq 0 ] || exit $rc
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${tag}_gpu_tests.log; stop $rc
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$TERMS" ]; then
  timeout -k 10 120 python -u tests/diagnostics/term_attribution.py dump diag_libs/_tfg_terms.so /tmp/terms.npz 8 129 &&
  timeout -k 10 120 python -u tests/diagnostics/term_attribution.py dump topoflow-glacier_amd/topoflow_glacier/_tfg.so /tmp/outs.npz 8 129
  rc=$?; stop $rc; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 900 python -u tests/diagnostics/term_attribution.py analyse /tmp/terms.npz /tmp/outs.npz gpurun_out/${tag}_term_attribution.json > gpurun_out/${tag}_term_attribution.log 2>&1
  echo "attribution rc=$?"
fi
