# Round 5: same-box A/B of library variants (LIBS="diag_libs/_tfg_<v>.so ..."), alternating, REPS rounds,
# the default bench workload (8192^2, 128-step launches) without parity and CPU legs (BENCH_ARGS adds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${TAG:-r5ab}
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS}; do
    v=$(basename $lib .so)
    TFG_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --no-parity $BENCH_ARGS \
      > gpurun_out/${tag}_${v}_$rep.json 2> gpurun_out/${tag}_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/${tag}_${v}_$rep.err; exit $rc; }
    python3 -c "import json; r=json.loads(open('gpurun_out/${tag}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', 'G=%.3f' % (r['value']/1e9), 'ms/launch=%.3f' % r['roofline']['kernel_ms_per_launch'], 'frac=%.4f' % r['roofline']['frac'], flush=True)"
  done
done
