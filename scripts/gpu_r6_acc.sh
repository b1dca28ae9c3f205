# Round 6: fp64 turbulent-flux variants of the fp32 engine (TFG_FLUX64): same-box speed A/B against the
# baseline build (LIBS), then the accuracy tests (ACC_LIBS) -- the year-long free run (TFG_REPORT_DIR
# year_divergence) and the N = 4 deep-launch samples -- through TFG_LIB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r6acc}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS}; do
    v=$(basename $lib .so)
    TFG_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --no-parity $BENCH_ARGS \
      > gpurun_out/${tag}_${v}_$rep.json 2> gpurun_out/${tag}_${v}_$rep.err
    rc=$?; stop $rc; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/${tag}_${v}_$rep.err; exit $rc; }
    python3 -c "import json; r=json.loads(open('gpurun_out/${tag}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', 'G=%.3f' % (r['value']/1e9), 'ms/launch=%.3f' % r['roofline']['kernel_ms_per_launch'], 'frac=%.4f' % r['roofline']['frac'], flush=True)"
  done
done
for lib in ${ACC_LIBS}; do
  v=$(basename $lib .so)
  TFG_LIB=$PWD/$lib TFG_REPORT_DIR=gpurun_out/${tag}_reports_$v timeout -k 10 600 python -u -m pytest -x -v -s \
    --timeout 500 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py::test_fp32_free_run_over_a_year tests/test_gpu_deep_sample.py} \
    > gpurun_out/${tag}_tests_$v.log 2>&1
  rc=$?; echo "== $v tests rc=$rc"; grep -E "passed|failed|max_floored|Error|assert" gpurun_out/${tag}_tests_$v.log | tail -12; stop $rc
  cat gpurun_out/${tag}_reports_$v/year_divergence.json 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps(d['per_variable_diverged_cells'])); print(json.dumps(d['annual_runoff_rel_error']['gpu_fp32_other_cells']))"
done
