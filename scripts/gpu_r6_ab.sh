# Round 6: same-box A/B of bench variants, alternating, REPS rounds; each entry of RUNS is
# "<library path>|<extra bench args>" (the default bench workload without parity and CPU legs),
# then optional GPU tests (TESTS, with TFG_REPORT_DIR=gpurun_out/<tag>_reports).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r6ab}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
i=0
for rep in $(seq 1 ${REPS:-2}); do
  for run in ${RUNS}; do
    lib=${run%%|*}; extra=${run#*|}; extra=${extra//,/ }
    v=$(basename $lib .so)_$(echo "$extra" | tr -d ' -' | tr -c 'a-zA-Z0-9_\n' '_')
    TFG_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --no-parity $extra \
      > gpurun_out/${tag}_${v}_$rep.json 2> gpurun_out/${tag}_${v}_$rep.err
    rc=$?; stop $rc; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/${tag}_${v}_$rep.err; exit $rc; }
    python3 -c "import json; r=json.loads(open('gpurun_out/${tag}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', 'G=%.3f' % (r['value']/1e9), 'ms/launch=%.3f' % r['roofline']['kernel_ms_per_launch'], 'frac=%.4f' % r['roofline']['frac'], flush=True)"
  done
done
if [ -n "$TESTS" ]; then
  TFG_REPORT_DIR=gpurun_out/${tag}_reports timeout -k 10 900 python -u -m pytest -x -v -s --timeout 500 \
    --timeout-method thread $TESTS > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; echo "== tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|max_floored|passed|failed" gpurun_out/${tag}_tests.log | tail -30; exit $rc
fi
